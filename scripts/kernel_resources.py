"""Per-kernel VGPRs / spills / LDS / occupancy of a HIP source (hipcc
-Rpass-analysis=kernel-resource-usage): python scripts/kernel_resources.py <src.hip> [name-substring]
[extra hipcc flags...].  Compiles to /tmp; prints one line per kernel."""
import re
import subprocess
import sys

src = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3:]
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Ianalyzer_amd/csrc", "-fapprox-func",
       "-freciprocal-math", "-fno-signed-zeros", "-Rpass-analysis=kernel-resource-usage", "-c", src,
       "-o", "/tmp/kernel_resources.o"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark: ([A-Za-z /\[\]]+?): (\S+) \[-Rpass", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    if sub in r["name"]:
        print("%-70s VGPRs %4s  AGPRs %3s  VGPR spill %3s  SGPR spill %3s  LDS %6s  occupancy %s" % (
            r["name"][:70], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
            r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))
