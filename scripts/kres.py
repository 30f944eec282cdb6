"""Per-kernel VGPR / scratch / occupancy summary of one HIP source (gfx950):
  python scripts/kres.py csrc/kernels/<file>.hip [extra hipcc flags]"""
import os
import re
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", os.path.join(root, "csrc"),
       "-c", os.path.abspath(sys.argv[1]), "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage", *sys.argv[2:]]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur = {}
for line in out.splitlines():
    if "error" in line:
        print(line)
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        continue
    for key, pat in (("v", r"VGPRs: (\d+)"), ("a", r"AGPRs: (\d+)"), ("scr", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            cur[key] = m.group(1)
    if cur and "occ" in cur:
        print(f"v{cur.get('v')} a{cur.get('a')} scr{cur.get('scr')} occ{cur['occ']}  {cur['name'][:120]}")
        cur = {}
