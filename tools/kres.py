"""Per-kernel VGPRs / occupancy of one HIP source for gfx950 (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                      "-Wno-unused-function", "-I", "build/gen", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
name = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()
        rows[name] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and name:
        rows[name][m.group(1).split()[0]] = m.group(2)
for n, r in rows.items():
    if pat in n:
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('Occupancy','?'):>2} occ {r.get('ScratchSize','?'):>3} scr  {n[:150]}")
