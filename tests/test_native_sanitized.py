"""C++ host mirror under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5
"race detection / sanitizers"; host code only -- GPU ASan/XNACK are not
available on this pool).  Builds tests/native/host_selftest.cpp together with
csrc/host.cpp as a standalone executable and runs it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "analyzer_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_mirror_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-I" + CSRC, os.path.join(ROOT, "tests", "native", "host_selftest.cpp"),
           os.path.join(CSRC, "host.cpp"), "-o", exe]
    res = subprocess.run(cmd, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert run.returncode == 0, (run.stdout + run.stderr)[-4000:]
    assert "host selftest ok" in run.stdout
