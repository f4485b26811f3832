#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy of one HIP source, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (CPU only; no GPU needed).
  python tools/kres.py csrc/k_resize_direct.hip [name-filter]"""
import re
import subprocess
import sys
from pathlib import Path

src = Path(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=off",
       "-fno-fast-math", "-x", "hip", "-c", str(src), "-o", "/tmp/_kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            rows[cur][key] = int(m.group(1))
for name, r in rows.items():
    if flt in name:
        print(f"{r.get('vgpr', '?'):>4} vgpr {r.get('sgpr', '?'):>4} sgpr {r.get('scratch', 0):>4} scratch "
              f"{r.get('occ', '?'):>2} occ {r.get('lds', 0):>6} lds  {name}")
