"""ctypes binding of the C ABI in include/vacv_hip.h (lib/libvacv_hip.so).

This is the same binding any FFI consumer would write (INTEGRATION.md shows
the cgo/JNI equivalents).  The library is loaded from the package's own
``lib/`` directory; if it is missing the import fails loudly -- there is no
CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # arm-neon-opencv_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_DIR = PKG_ROOT / "lib"
# VACV_LIB_DIR: another in-tree build of the same library (A/B variant
# builds, tools/variants.sh); the default is lib/
HIP_LIB = (Path(os.environ["VACV_LIB_DIR"]).resolve() if os.environ.get("VACV_LIB_DIR") else LIB_DIR) / "libvacv_hip.so"
API_LIB = LIB_DIR / "libvacv.so"
HEADER = REPO_ROOT / "include" / "vacv_hip.h"

# status codes / enums (include/vacv_hip.h)
OK, ERR_INVALID_ARG, ERR_UNSUPPORTED, ERR_HIP, ERR_NO_MEMORY = 0, -1, -2, -3, -4
FP32, FP16, INT8, FP64 = 0, 1, 2, 3
NCHW, NHWC = 0, 1
INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA, INTER_LANCZOS4 = 0, 1, 2, 3, 4
BORDER_CONSTANT, BORDER_REPLICATE, BORDER_REFLECT, BORDER_WRAP, BORDER_REFLECT_101, BORDER_TRANSPARENT = 0, 1, 2, 3, 4, 5
WARP_INVERSE_MAP = 16  # warp flag: m is the dst -> src map
COLOR_YUV2RGB_NV12, COLOR_YUV2BGR_NV12, COLOR_YUV2RGB_NV21, COLOR_YUV2BGR_NV21 = 90, 91, 92, 93
# the codes the reference hands to cv::cvtColor (OpenCV 2.4 arithmetic)
COLOR_GRAY2BGR = 8
COLOR_YUV2RGBA_NV12, COLOR_YUV2BGRA_NV12, COLOR_YUV2RGBA_NV21, COLOR_YUV2BGRA_NV21 = 94, 95, 96, 97
COLOR_YUV2BGR_YV12 = 99
LINEAR_REFERENCE, LINEAR_NEON, LINEAR_OPENCV = 0, 1, 2
TM_SQDIFF, TM_SQDIFF_NORMED, TM_CCORR, TM_CCORR_NORMED, TM_CCOEFF, TM_CCOEFF_NORMED = 0, 1, 2, 3, 4, 5


class VacvError(RuntimeError):
    def __init__(self, fn: str, status: int):
        self.status = status
        super().__init__(f"{fn} failed: {status_string(status)} ({status})")


class VacvImage(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("n", ctypes.c_int32),
        ("w", ctypes.c_int32),
        ("h", ctypes.c_int32),
        ("c", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("layout", ctypes.c_int32),
        ("row_pitch", ctypes.c_int64),
        ("plane_pitch", ctypes.c_int64),
        ("batch_pitch", ctypes.c_int64),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_IMG = ctypes.POINTER(VacvImage)
_FP = ctypes.POINTER(ctypes.c_float)
_DP = ctypes.POINTER(ctypes.c_double)

# name -> (argtypes, restype); the single source of truth for the exported
# surface (tests check it against include/vacv_hip.h and the .so).
SIGNATURES = {
    "vacv_abi_version": ([], _I),
    "vacv_status_string": ([_I], ctypes.c_char_p),
    "vacv_image_bytes": ([_IMG], ctypes.c_int64),
    "vacv_crop": ([_IMG, _IMG, _I, _I, _P], _I),
    "vacv_change_layout": ([_IMG, _IMG, _P], _I),
    "vacv_change_dtype": ([_IMG, _IMG, _P], _I),
    "vacv_resize": ([_IMG, _IMG, _I, _I, _P], _I),
    "vacv_resize_scaled": ([_IMG, _IMG, _I, _I, _D, _D, _P], _I),
    "vacv_warp_affine": ([_IMG, _IMG, _FP, _I, _I, _DP, _P], _I),
    "vacv_rotation_matrix": ([ctypes.c_float, ctypes.c_float, _DP, _FP], _I),
    "vacv_invert_affine": ([_FP, _FP], _I),
    "vacv_cvt_color": ([_IMG, _IMG, _I, _P], _I),
    "vacv_normalize": ([_IMG, _IMG, _FP, _FP, _P], _I),
    "vacv_channel_sums": ([_IMG, _P, _I, _P], _I),
    "vacv_stats_from_sums": ([_P, _I, _I, _D, _P, _P, _P], _I),
    "vacv_resize_channel_sums": ([_IMG, _IMG, _I, _I, _P, _I, _P], _I),
    "vacv_resize_mean_stddev": ([_IMG, _IMG, _I, _I, _P, _P, _P, _I, _P], _I),
    "vacv_mean_stddev": ([_IMG, _P, _P, _P], _I),
    "vacv_resize_normalize": ([_IMG, _IMG, _I, _I, _FP, _FP, _P], _I),
    "vacv_warp_affine_normalize": ([_IMG, _IMG, _FP, _I, _I, _DP, _FP, _FP, _P], _I),
    "vacv_cvt_color_normalize": ([_IMG, _IMG, _I, _FP, _FP, _P], _I),
    "vacv_cvt_color_resize": ([_IMG, _IMG, _I, _I, _I, _P], _I),
    "vacv_cvt_color_resize_normalize": ([_IMG, _IMG, _I, _I, _I, _FP, _FP, _P], _I),
    "vacv_stream_synchronize": ([_P], _I),
    "vacv_release_workspace": ([], _I),
    "vacv_match_template": ([_IMG, _IMG, _IMG, _I, _P], _I),
    "vacv_min_max_idx": ([_IMG, _IMG, _P, _P, _P], _I),
    "vacv_set_tuning": ([_I, _I], _I),
    "vacv_get_tuning": ([_I], _I),
}

# kernel-variant knobs (VACV_TUNE_*, include/vacv_hip.h)
TUNE = {"RESIZE_DIRECT": 0, "CUBIC_DIRECT": 1, "RESIZE_INTERLEAVE": 2, "DIRECT_XCD": 3, "WARP_PX": 4,
        "NEAREST_KERNEL": 5, "AREA_KERNEL": 6, "AREA_ROWS": 7, "RESIZE_WGS": 8, "RESIZE_TILE_H": 9,
        "RESIZE_TILE_W": 10, "RESIZE_WORK": 11, "WARP_KERNEL": 12, "RESIZE_STRIP": 13, "MATCH_KERNEL": 14,
        "WARP_FRAMES": 15, "WARP_TILE_H": 16, "WARP_SLOTS": 17,
        "LANCZOS_KERNEL": 18}

# include/vacv_hip.h VACV_ABI_VERSION: the tuning enum above and every
# signature here are laid out for it (tests/test_abi.py checks the header).
# Bumped with every change to a signature or to the tuning enum (3: round 6,
# after round 5 added LANCZOS_KERNEL under version 2)
ABI_VERSION = 3

_lib = None


def build(quiet: bool = True) -> None:
    """Compile lib/libvacv_hip.so and lib/libvacv.so for gfx950 (hipcc)."""
    jobs = str(min(16, os.cpu_count() or 4))
    cmd = ["make", "-C", str(PKG_ROOT), "-j", jobs]
    if quiet:
        cmd.insert(1, "-s")
    subprocess.run(cmd, check=True)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    path = HIP_LIB
    if not path.exists():
        raise ImportError(
            f"{path} is missing: the vacv HIP library has not been built "
            f"(run `make -C {PKG_ROOT}` or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(str(path))
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    got = lib.vacv_abi_version()
    if got != ABI_VERSION:
        # e.g. a stale variant build under VACV_LIB_DIR: its tuning knobs and
        # entry points would not mean what this binding passes
        raise ImportError(f"{path} implements C ABI version {got}, this binding expects {ABI_VERSION}: rebuild it")
    # and the tuning enum has exactly this binding's keys (VACV_TUNE_COUNT):
    # the last key is accepted (set to the value it holds: an environment
    # override survives), the one after it is not.  vacv_get_tuning alone
    # cannot tell: its "built-in choice" -1 is INVALID_ARG's code
    n = len(TUNE)
    if lib.vacv_set_tuning(n - 1, lib.vacv_get_tuning(n - 1)) != OK or lib.vacv_set_tuning(n, -1) != ERR_INVALID_ARG:
        raise ImportError(f"{path}: its tuning enum does not have the {n} keys this binding knows: rebuild it")
    _lib = lib
    return lib


def status_string(status: int) -> str:
    try:
        return load().vacv_status_string(status).decode()
    except Exception:  # pragma: no cover - only when the library itself is broken
        return "unknown"


def check(fn: str, status: int) -> None:
    if status != OK:
        raise VacvError(fn, status)
