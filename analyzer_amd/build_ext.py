"""In-tree build of the native extension ``analyzer_amd._C`` for gfx950.

Device code (``*.hip``) is compiled by ``hipcc --offload-arch=gfx950``; the
torch binding and the C++ host mirror by ``g++``; everything is linked into
``analyzer_amd/_C*.so`` next to this file, so the built library travels with
the repository snapshot to the GPU box and is what the tests load.

    python -m analyzer_amd.build_ext [--force] [--jobs N]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import sysconfig
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "analyzer_amd"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

HIP_SOURCES = ["kernels.hip", "radix_sort.hip", "dataflow.hip", "sweep.hip", "telemetry.hip", "levels.hip",
               "digest.hip"]
# per-file device flags.  The executor's divisions/sqrt take the 1-ulp hardware
# paths (v_rcp_f32 instead of the ~10-instruction IEEE division expansion: -9%
# static instructions); NaN/Inf semantics are untouched (no -ffinite-math-only),
# which the NULL = NaN convention relies on.
HIP_FLAGS = {n: ["-fapprox-func", "-freciprocal-math", "-fno-signed-zeros"]
             for n in ("dataflow.hip",)}
CPP_SOURCES = ["host.cpp", "ingest.cpp", "batch_host.cpp", "telemetry_file.cpp", "bindings.cpp"]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path(diag: bool = False, variant: str = "") -> Path:
    """The in-tree library: ``_C`` (production) or ``_C_diag`` (``--diag``: also
    the telemetry kernel's diagnostic / tuning variants, ANA_TELE_DEBUG and
    ANA_TELE_SPAN; load it with ANA_NATIVE_LIB)."""
    if variant:  # experiment builds (--variant): ab/<name>_C.so, loaded with ANA_NATIVE_LIB
        return PKG.parent / "ab" / (variant + "_C.so")
    return PKG / (("_C_diag" if diag else "_C") + _ext_suffix())


def _torch_paths():
    import torch.utils.cpp_extension as ce

    return ce.include_paths(), ce.library_paths()


def _deps_mtime(src: Path) -> float:
    headers = [p.stat().st_mtime for p in CSRC.glob("*.h")]
    return max([src.stat().st_mtime] + headers)


def _compile(cmd, src: Path, obj: Path, force: bool) -> str:
    if not force and obj.exists() and obj.stat().st_mtime >= _deps_mtime(src):
        return "up-to-date %s" % src.name
    obj.parent.mkdir(parents=True, exist_ok=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s\n%s" % (" ".join(cmd), res.stdout, res.stderr))
    return "built %s" % src.name


def _host_id() -> str:
    """This machine: host name + kernel boot id (the image -- and with it
    /etc/machine-id and often the host name -- is the same here and on a GPU box)."""
    try:
        boot = Path("/proc/sys/kernel/random/boot_id").read_text().strip()[:8]
    except OSError:  # pragma: no cover
        boot = "?"
    return "%s/%s" % (socket.gethostname(), boot)


def _hipcc_version() -> str:
    try:
        res = subprocess.run(["hipcc", "--version"], capture_output=True, text=True, timeout=120)
        return " | ".join(ln.strip() for ln in res.stdout.splitlines() if "version" in ln.lower())
    except Exception as e:  # pragma: no cover - no toolchain
        return "unavailable: %s" % e


def source_digest(dflags=(), hip_flags=()) -> str:
    """sha256 over every source and header of the extension, the device flags and
    this file (which holds the compile commands)."""
    h = hashlib.sha256()
    files = sorted(set(CSRC.glob("*.h")) | {CSRC / n for n in HIP_SOURCES + CPP_SOURCES} | {Path(__file__)})
    for f in files:
        if f.exists():
            h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    h.update(repr((ARCH, sorted(HIP_FLAGS.items()), list(dflags), list(hip_flags))).encode())
    return h.hexdigest()


def stamp_path(out: Path) -> Path:
    """``<library>.build.json``: what the library next to it was built from, where."""
    return out.with_name(out.name.split(".")[0] + ".build.json")


def read_stamp(out: Path) -> dict:
    try:
        return json.loads(stamp_path(out).read_text())
    except (OSError, ValueError):
        return {}


def build(force: bool = False, jobs: int = 4, verbose: bool = False, diag: bool = False,
          variant: str = "", defines=(), hip_flags=()) -> Path:
    out = target_path(diag, variant)
    out.parent.mkdir(parents=True, exist_ok=True)
    objdir = BUILD / ("variant_" + variant) if variant else BUILD / "diag" if diag else BUILD
    dflags = (["-DANA_DIAG_BUILD=1"] if diag else []) + ["-D" + d for d in defines]
    sources = [CSRC / n for n in HIP_SOURCES + CPP_SOURCES if (CSRC / n).exists()]
    digest = source_digest(dflags, hip_flags)
    hipcc = _hipcc_version()
    stamp = read_stamp(out)
    # provenance: the library is current only if its stamp names these exact sources,
    # this compiler and THIS host -- a library that travelled from another machine (the
    # container build on a GPU box) is rebuilt from source, so a box build proves the
    # sources compile there
    current = (out.exists() and stamp.get("sources_sha256") == digest and stamp.get("hipcc") == hipcc
               and stamp.get("host") == _host_id())
    if not force and current:
        if verbose:
            print("up-to-date", out, "(stamp %s, built on %s)" % (digest[:12], stamp.get("host")), flush=True)
        return out
    if not force and (not stamp or stamp.get("host") != _host_id() or stamp.get("hipcc") != hipcc):
        force = True  # objects here may belong to another build: compile every source
        if verbose:
            print("stamp %s: rebuilding every source" % (
                "missing" if not stamp else "from host %s" % stamp.get("host")
                if stamp.get("host") != _host_id() else "of another hipcc"), flush=True)
    elif not force and verbose:
        print("sources changed since stamp %s: rebuilding what changed" % str(stamp.get("sources_sha256"))[:12],
              flush=True)
    incs, libs = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    objs = []
    tasks = []
    for name in HIP_SOURCES:
        src = CSRC / name
        if not src.exists():
            continue
        obj = objdir / (name + ".o")
        cmd = ["hipcc", "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
               "-I" + str(CSRC)] + HIP_FLAGS.get(name, []) + dflags + list(hip_flags) + ["-c", str(src), "-o", str(obj)]
        tasks.append((cmd, src, obj))
        objs.append(obj)
    for name in CPP_SOURCES:
        src = CSRC / name
        obj = objdir / (name + ".o")
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-pthread", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
               "-D_GLIBCXX_USE_CXX11_ABI=1", "-I" + str(CSRC), "-I" + ROCM + "/include",
               "-I" + py_inc] + ["-I" + p for p in incs] + ["-c", str(src), "-o", str(obj)]
        tasks.append((cmd, src, obj))
        objs.append(obj)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for msg in ex.map(lambda t: _compile(t[0], t[1], t[2], force), tasks):
            if verbose:
                print(msg, flush=True)
    newest = max(o.stat().st_mtime for o in objs)
    if force or not out.exists() or out.stat().st_mtime < newest:
        cmd = ["g++", "-shared", "-o", str(out)] + [str(o) for o in objs]
        for p in libs:
            cmd += ["-L" + p, "-Wl,-rpath," + p]
        cmd += ["-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip", "-ltorch_hip", "-ltorch_python",
                "-L" + ROCM + "/lib", "-Wl,-rpath," + ROCM + "/lib", "-lamdhip64"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (res.stdout, res.stderr))
        if verbose:
            print("linked", out, flush=True)
    stamp_path(out).write_text(json.dumps({
        "library": out.name, "sources_sha256": digest, "hipcc": hipcc, "host": _host_id(),
        "arch": ARCH, "sources": [s_.name for s_ in sources], "defines": dflags,
        "built_at": time.strftime("%Y-%m-%dT%H:%M:%S%z")}, indent=1) + "\n")
    return out


def _abi_flag() -> str:  # pragma: no cover - informational
    import torch

    return "-D_GLIBCXX_USE_CXX11_ABI=%d" % int(torch._C._GLIBCXX_USE_CXX11_ABI)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--diag", action="store_true",
                    help="build _C_diag with the diagnostic kernel variants (scripts/tune_tele.py)")
    ap.add_argument("--variant", default="",
                    help="experiment build: ab/<VARIANT>_C.so with --define flags (in-call A/B, gpu.sh ab)")
    ap.add_argument("--define", action="append", default=[], help="extra -D for the device code")
    ap.add_argument("--hip-flag", action="append", default=[],
                    help="extra hipcc flag for the HIP sources (experiment builds)")
    args = ap.parse_args(argv)
    path = build(force=args.force, jobs=args.jobs, verbose=True, diag=args.diag, variant=args.variant, hip_flags=args.hip_flag,
                 defines=args.define)
    print(path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
