"""VGPRs / scratch / occupancy per kernel of krr_kernels.hip (hipcc -Rpass-analysis), for
checking that a change left the hot kernels' register allocation alone.
    python scripts/regs.py [extra hipcc flags...]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-Iinclude",
       "-Ikrr_amd/csrc", "--cuda-device-only", "-c", "krr_amd/csrc/krr_kernels.hip", "-o", "/tmp/_regs.o",
       "-Rpass-analysis=kernel-resource-usage", *sys.argv[1:]]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
name = None
rows = {}
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        name = m.group(1)
        rows[name] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", ln)
    if m and name:
        rows[name][m.group(1).split()[0]] = int(m.group(2))
    if "error" in ln:
        print(ln)
for n, r in rows.items():
    if n.startswith("_ZN3krr"):
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('ScratchSize', '?'):>4} scratch {r.get('Occupancy', '?')} waves  {n}")
