#!/usr/bin/env python3
"""Per-phase clock totals of warp_exp_kernel from a VACV_RING_DBG=16 build
(printf from a few waves): python tools/warp_prof.py <lib dir> [rot]"""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "arm-neon-opencv_amd"))
import vacv_amd._lib as L  # noqa: E402
L.HIP_LIB = Path(sys.argv[1]).resolve() / "libvacv_hip.so"
import torch  # noqa: E402
from vacv_amd import ops  # noqa: E402
rot = float(sys.argv[2]) if len(sys.argv) > 2 else 15.0
dev = torch.device("cuda:0")
src = torch.randint(0, 256, (128, 720, 1280, 3), dtype=torch.uint8, device=dev)
o = torch.empty_like(src)
m = ops.rotation_matrix(0.9, rot, (640, 360, 640, 360))
for _ in range(3):
    ops.warp_affine(src, m, 1280, 720, out=o)
torch.cuda.synchronize()
print("---- last launch above", flush=True)
