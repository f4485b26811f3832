#!/usr/bin/env python3
"""Per-phase clock totals of warp_exp_kernel from a VACV_RING_DBG=16 build
(printf from a few waves): python tools/warp_prof.py <lib dir> [rot] [linear|nearest|normalize]"""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "arm-neon-opencv_amd"))
import vacv_amd._lib as L  # noqa: E402
L.HIP_LIB = Path(sys.argv[1]).resolve() / "libvacv_hip.so"
import torch  # noqa: E402
from vacv_amd import ops  # noqa: E402
rot = float(sys.argv[2]) if len(sys.argv) > 2 else 15.0
kind = sys.argv[3] if len(sys.argv) > 3 else "linear"
dev = torch.device("cuda:0")
src = torch.randint(0, 256, (128, 720, 1280, 3), dtype=torch.uint8, device=dev)
o = torch.empty_like(src)
m = ops.rotation_matrix(0.9, rot, (640, 360, 640, 360))
import vacv_amd  # noqa: E402
of = torch.empty((128, 720, 1280, 3), dtype=torch.float32, device=dev) if kind == "normalize" else None
for _ in range(3):
    if kind == "nearest":
        ops.warp_affine(src, m, 1280, 720, flags=vacv_amd.INTER_NEAREST, out=o)
    elif kind == "normalize":
        ops.warp_affine_normalize(src, m, 1280, 720, [103.94, 116.78, 123.68], [57.375, 57.12, 58.395], out=of)
    else:
        ops.warp_affine(src, m, 1280, 720, out=o)
torch.cuda.synchronize()
print("---- last launch above", flush=True)
