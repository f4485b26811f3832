"""vacv_amd -- MI355X-native vacv pixel operators (host side of the C ABI).

``ops`` mirrors the reference's ``va_cv::`` operator API on batched device
tensors; ``dist`` adds the multi-GPU (RCCL) statistics reduction.  All
compute happens in lib/libvacv_hip.so (hand-written gfx950 kernels).
"""
from . import _lib
from ._lib import (BORDER_CONSTANT, BORDER_REFLECT, BORDER_REFLECT_101, BORDER_REPLICATE, BORDER_TRANSPARENT,
                   BORDER_WRAP, COLOR_GRAY2BGR, COLOR_YUV2BGR_NV12, COLOR_YUV2BGR_NV21, COLOR_YUV2BGR_YV12,
                   COLOR_YUV2BGRA_NV12, COLOR_YUV2BGRA_NV21, COLOR_YUV2RGB_NV12, COLOR_YUV2RGB_NV21,
                   COLOR_YUV2RGBA_NV12, COLOR_YUV2RGBA_NV21,
                   FP16, FP32, FP64, INT8, INTER_AREA, INTER_CUBIC, INTER_LANCZOS4, INTER_LINEAR, INTER_NEAREST, LINEAR_NEON, LINEAR_OPENCV,
                   LINEAR_REFERENCE, NCHW, NHWC, WARP_INVERSE_MAP, VacvError, build)

__all__ = ["ops", "dist", "build", "VacvError"]


def __getattr__(name):
    # ops/dist import torch; keep `import vacv_amd` cheap for build-only users
    if name in ("ops", "dist"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
