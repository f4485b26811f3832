"""numpy front-end for the CPU oracle (TEST INFRASTRUCTURE ONLY).

``Oracle`` wraps oracle/liboracle.so (the C restatement in vacv_oracle.c);
``Reference`` wraps oracle/_ref/libvacv_ref.so (the reference's own pixel
loops compiled from /root/reference by oracle/Makefile).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product package (arm-neon-opencv_amd/vacv_amd) never does.

Images are numpy arrays: HWC (h, w, c) or a single plane (h, w).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ORACLE_SO = HERE / "liboracle.so"
REF_SO = HERE / "_ref" / "libvacv_ref.so"

LINEAR_NAIVE, LINEAR_NEON, LINEAR_OPENCV = 0, 1, 2

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE), "oracle"], check=True)


def build_reference() -> bool:
    """Build oracle/_ref when the reference sources are present."""
    if not Path("/root/reference/src/cv/resize_naive.cpp").exists():
        return REF_SO.exists()
    subprocess.run(["make", "-s", "-C", str(HERE), "ref"], check=True)
    return True


def _shape(img: np.ndarray):
    if img.ndim == 2:
        return img.shape[1], img.shape[0], 1
    return img.shape[1], img.shape[0], img.shape[2]


def _out(h, w, c, dtype):
    return np.zeros((h, w, c) if c > 1 else (h, w), dtype=dtype)


class Oracle:
    """C restatement of the reference (vacv_oracle.c)."""

    def __init__(self, path: Path = ORACLE_SO):
        if not path.exists():
            build_oracle()
        self.lib = ctypes.CDLL(str(path))
        L = self.lib
        for name, args, res in [
            ("oracle_sat_short", [_F], _I),
            ("oracle_linear_table", [_I, _I, _I, _P, _P, _P], None),
            ("oracle_cubic_table", [_I, _I, _P, _P], None),
            ("oracle_invert_affine", [_P, _P], None),
            ("oracle_rotation_matrix", [_F, _F, _P, _P], None),
            ("oracle_resize_linear_u8", [_P, _I, _I, _I, _P, _I, _I, _I], None),
            ("oracle_resize_linear_f32", [_P, _I, _I, _I, _P, _I, _I], None),
            ("oracle_resize_cubic_f32", [_P, _I, _I, _I, _P, _I, _I], None),
            ("oracle_resize_nearest", [_P, _I, _I, _I, _I, _P, _I, _I], None),
            ("oracle_resize_area", [_P, _I, _I, _I, _I, _P, _I, _I], None),
            ("oracle_warp_affine_u8", [_P, _I, _I, _I, _P, _I, _I, _P], None),
            ("oracle_warp_affine_f32", [_P, _I, _I, _I, _P, _I, _I, _P], None),
            ("oracle_resize_area_any", [_P, _I, _I, _I, _I, _P, _I, _I, ctypes.c_double, ctypes.c_double], None),
            ("oracle_resize_lanczos4", [_P, _I, _I, _I, _I, _P, _I, _I, ctypes.c_double, ctypes.c_double], None),
            ("oracle_match_template", [_P, _I, _I, _P, _I, _I, _I, _I, _I, _P], None),
            ("oracle_min_max_idx", [_P, _I, _I, _I, _P, _P, _P], None),
            ("oracle_warp_affine_border", [_P, _I, _I, _I, _I, _P, _I, _I, _P, _I], None),
            ("oracle_yuv420sp_to_bgr", [_P, _P, _I, _I, _I, _I], None),
            ("oracle_bgr2nv21", [_P, _P, _I, _I], None),
            ("oracle_yuv420_cv", [_P, _P, _I, _I, _I, _I, _I], None),
            ("oracle_warp_affine_nn", [_P, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P], None),
            ("oracle_gray_to_bgr", [_P, _P, _L, _I, _I], None),
            ("oracle_hwc_to_chw", [_P, _P, _I, _I, _I, _I], None),
            ("oracle_chw_to_hwc", [_P, _P, _I, _I, _I, _I], None),
            ("oracle_u8_to_f32", [_P, _P, _L], None),
            ("oracle_f32_to_u8", [_P, _P, _L], None),
            ("oracle_crop", [_P, _I, _I, _I, _I, _I, _P, _I, _I, _I, _I], None),
            ("oracle_normalize_f32", [_P, _P, _L, _I, _P, _P], None),
            ("oracle_mean_stddev_ref_f32", [_P, _L, _I, _P, _P], None),
            ("oracle_channel_sums_f64", [_P, _L, _I, _P], None),
            ("oracle_channel_sums_u8", [_P, _L, _I, _P], None),
            ("oracle_stats_from_sums", [_P, ctypes.c_double, _I, _P, _P], None),
            ("oracle_cosine_f32acc_u8", [_P, _P, _L], _F),
            ("oracle_cosine_f64_f32", [_P, _P, _L], ctypes.c_double),
        ]:
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res

    # -- tables / host math -------------------------------------------------
    def linear_table(self, n_in, n_out, mode=LINEAR_NAIVE):
        ofs = np.zeros(n_out, np.int32)
        w0 = np.zeros(n_out, np.int16)
        w1 = np.zeros(n_out, np.int16)
        self.lib.oracle_linear_table(n_in, n_out, mode, _ptr(ofs), _ptr(w0), _ptr(w1))
        return ofs, w0, w1

    def cubic_table(self, n_in, n_out):
        ofs = np.zeros(n_out, np.int32)
        coef = np.zeros((n_out, 4), np.float32)
        self.lib.oracle_cubic_table(n_in, n_out, _ptr(ofs), _ptr(coef))
        return ofs, coef

    def invert_affine(self, m):
        m = np.ascontiguousarray(m, np.float32).reshape(6)
        inv = np.zeros(6, np.float32)
        self.lib.oracle_invert_affine(_ptr(m), _ptr(inv))
        return inv

    def rotation_matrix(self, scale, rot, aux):
        aux = np.ascontiguousarray(aux, np.float64).reshape(4)
        m = np.zeros(6, np.float32)
        self.lib.oracle_rotation_matrix(scale, rot, _ptr(aux), _ptr(m))
        return m

    # -- samplers ------------------------------------------------------------
    def resize_linear(self, img, w_out, h_out, mode=LINEAR_NAIVE):
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        out = _out(h_out, w_out, c, img.dtype)
        if img.dtype == np.uint8:
            self.lib.oracle_resize_linear_u8(_ptr(img), w, h, c, _ptr(out), w_out, h_out, mode)
        else:
            assert img.dtype == np.float32
            self.lib.oracle_resize_linear_f32(_ptr(img), w, h, c, _ptr(out), w_out, h_out)
        return out

    def resize_nearest(self, img, w_out, h_out):
        """OpenCV 2.4 resizeNN restated (parity unpinned, vacv_oracle.c)."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        out = _out(h_out, w_out, c, img.dtype)
        self.lib.oracle_resize_nearest(_ptr(img), w, h, c, img.dtype.itemsize, _ptr(out), w_out, h_out)
        return out

    def resize_area(self, img, w_out, h_out):
        """OpenCV 2.4 resizeAreaFast_ restated (integer downscales only;
        parity unpinned, vacv_oracle.c)."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        assert w % w_out == 0 and h % h_out == 0, "integer downscales only"
        out = _out(h_out, w_out, c, img.dtype)
        self.lib.oracle_resize_area(_ptr(img), w, h, c, img.dtype.itemsize, _ptr(out), w_out, h_out)
        return out

    def resize_area_any(self, img, w_out, h_out, inv_x=0.0, inv_y=0.0):
        """INTER_AREA at any scale (OpenCV 2.4 cv::resize restated; parity
        unpinned, vacv_oracle.c).  inv_x / inv_y: cv::resize's fx / fy when
        dsize is derived from them (0: dsize / ssize)."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        out = _out(h_out, w_out, c, img.dtype)
        self.lib.oracle_resize_area_any(_ptr(img), w, h, c, img.dtype.itemsize, _ptr(out), w_out, h_out,
                                        float(inv_x), float(inv_y))
        return out

    def resize_lanczos4(self, img, w_out, h_out, inv_x=0.0, inv_y=0.0):
        """INTER_LANCZOS4 (OpenCV 2.4 cv::resize restated; parity unpinned,
        vacv_oracle.c).  inv_x / inv_y: fx / fy when dsize derives from them."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        out = _out(h_out, w_out, c, img.dtype)
        self.lib.oracle_resize_lanczos4(_ptr(img), w, h, c, img.dtype.itemsize, _ptr(out), w_out, h_out,
                                        float(inv_x), float(inv_y))
        return out

    def match_template(self, img, tpl, method):
        """cv::matchTemplate restated (OpenCV 2.4 templmatch.cpp; exact
        correlation, parity unpinned): (H - h + 1, W - w + 1) fp32."""
        img = np.ascontiguousarray(img)
        tpl = np.ascontiguousarray(tpl, img.dtype)
        W, H, c = _shape(img)
        w, h, c2 = _shape(tpl)
        assert c == c2
        out = np.zeros((H - h + 1, W - w + 1), np.float32)
        self.lib.oracle_match_template(_ptr(img), W, H, _ptr(tpl), w, h, c, img.dtype.itemsize, int(method), _ptr(out))
        return out

    def min_max_idx(self, a, mask=None):
        """cv::minMaxIdx of a 2-D array: (min, max, (row, col) of min, of max)."""
        a = np.ascontiguousarray(a)
        h, w = a.shape
        mm = np.zeros(2, np.float64)
        idx = np.zeros(4, np.int32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self.lib.oracle_min_max_idx(_ptr(a), w, h, a.dtype.itemsize, None if m is None else _ptr(m), _ptr(mm), _ptr(idx))
        return float(mm[0]), float(mm[1]), (int(idx[0]), int(idx[1])), (int(idx[2]), int(idx[3]))

    def resize_cubic(self, img, w_out, h_out):
        img = np.ascontiguousarray(img, np.float32)
        w, h, c = _shape(img)
        out = _out(h_out, w_out, c, np.float32)
        self.lib.oracle_resize_cubic_f32(_ptr(img), w, h, c, _ptr(out), w_out, h_out)
        return out

    def warp_affine(self, img, m_forward, w_out, h_out, border=0, border_mode=0, dst=None):
        """warp_affine_naive (the inverse computed as warp_affine.cpp does).
        border_mode 0 CONSTANT: skipped pixels = `border`; 1 REPLICATE, 2
        REFLECT, 3 WRAP, 4 REFLECT_101: the build's extension (parity
        unpinned, vacv_oracle.c); 5 TRANSPARENT: skipped pixels keep `dst`."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        inv = self.invert_affine(m_forward)
        if border_mode == 5:
            out = np.ascontiguousarray(dst).copy()
        else:
            out = _out(h_out, w_out, c, img.dtype)
            out[...] = border
        if img.dtype == np.uint8:
            self.lib.oracle_warp_affine_u8(_ptr(img), w, h, c, _ptr(out), w_out, h_out, _ptr(inv))
        else:
            self.lib.oracle_warp_affine_f32(_ptr(img), w, h, c, _ptr(out), w_out, h_out, _ptr(inv))
        if border_mode in (1, 2, 3, 4):
            self.lib.oracle_warp_affine_border(_ptr(img), w, h, c, img.dtype.itemsize, _ptr(out), w_out, h_out,
                                               _ptr(inv), border_mode)
        return out

    # -- colour ----------------------------------------------------------------
    def warp_affine_nn(self, img, m, w_out, h_out, inverse_map=False, border_mode=0, border=(0, 0, 0, 0), dst=None):
        """cv::warpAffine INTER_NEAREST (OpenCV 2.4), m forward (or inverse
        with inverse_map); border_mode 5 keeps `dst` where unmapped."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        out = np.ascontiguousarray(dst).copy() if dst is not None else _out(h_out, w_out, c, img.dtype)
        mm = np.ascontiguousarray(m, np.float32)
        bv = np.ascontiguousarray(border, np.float64)
        self.lib.oracle_warp_affine_nn(_ptr(img), w, h, c, img.itemsize, _ptr(out), w_out, h_out, _ptr(mm),
                                       int(inverse_map), int(border_mode), _ptr(bv))
        return out

    def yuv420sp_to_bgr(self, yuv, v_first=True, rgb=False):
        yuv = np.ascontiguousarray(yuv, np.uint8)
        h = yuv.shape[0] // 3 * 2
        w = yuv.shape[1]
        out = np.zeros((h, w, 3), np.uint8)
        self.lib.oracle_yuv420sp_to_bgr(_ptr(yuv), _ptr(out), w, h, int(v_first), int(rgb))
        return out

    def bgr2nv21(self, bgr):
        bgr = np.ascontiguousarray(bgr, np.uint8)
        h, w = bgr.shape[:2]
        out = np.zeros((h * 3 // 2, w), np.uint8)
        self.lib.oracle_bgr2nv21(_ptr(bgr), _ptr(out), w, h)
        return out

    # cv::cvtColor codes the reference delegates to OpenCV (cvt_color.cpp:139-141)
    CV_YUV_CODES = {94: (0, 4, 2), 95: (0, 4, 0), 96: (1, 4, 2), 97: (1, 4, 0), 99: (2, 3, 0)}

    def yuv420_cv(self, yuv, code):
        """OpenCV 2.4's YUV420 -> BGR(A)/RGB(A) for COLOR_YUV2RGBA/BGRA_NV12/NV21
        (94-97) and COLOR_YUV2BGR_YV12 (99); yuv = (h*3/2, w) u8."""
        layout, dcn, bidx = self.CV_YUV_CODES[code]
        yuv = np.ascontiguousarray(yuv, np.uint8)
        h = yuv.shape[0] // 3 * 2
        w = yuv.shape[1]
        out = np.zeros((h, w, dcn), np.uint8)
        self.lib.oracle_yuv420_cv(_ptr(yuv), _ptr(out), w, h, layout, dcn, bidx)
        return out

    def gray_to_bgr(self, gray, dcn=3):
        """cv::cvtColor COLOR_GRAY2BGR (dcn 3) / GRAY2BGRA (4), u8 or fp32."""
        g = np.ascontiguousarray(gray)
        out = np.zeros(g.shape[:2] + (dcn,), g.dtype)
        self.lib.oracle_gray_to_bgr(_ptr(g), _ptr(out), g.shape[0] * g.shape[1], dcn, g.itemsize)
        return out

    # -- layout / dtype / crop -------------------------------------------------
    def hwc_to_chw(self, img):
        img = np.ascontiguousarray(img)
        h, w, c = img.shape
        out = np.zeros((c, h, w), img.dtype)
        self.lib.oracle_hwc_to_chw(_ptr(img), _ptr(out), w, h, c, img.itemsize)
        return out

    def chw_to_hwc(self, img):
        img = np.ascontiguousarray(img)
        c, h, w = img.shape
        out = np.zeros((h, w, c), img.dtype)
        self.lib.oracle_chw_to_hwc(_ptr(img), _ptr(out), w, h, c, img.itemsize)
        return out

    def u8_to_f32(self, a):
        a = np.ascontiguousarray(a, np.uint8)
        out = np.zeros(a.shape, np.float32)
        self.lib.oracle_u8_to_f32(_ptr(a), _ptr(out), a.size)
        return out

    def f32_to_u8(self, a):
        a = np.ascontiguousarray(a, np.float32)
        out = np.zeros(a.shape, np.uint8)
        self.lib.oracle_f32_to_u8(_ptr(a), _ptr(out), a.size)
        return out

    def crop(self, img, left, top, cw, ch, chw=False):
        img = np.ascontiguousarray(img)
        if chw:
            c, h, w = img.shape
            out = np.zeros((c, ch, cw), img.dtype)
            self.lib.oracle_crop(_ptr(img), w, h, 1, c, img.itemsize, _ptr(out), left, top, cw, ch)
        else:
            w, h, c = _shape(img)
            out = _out(ch, cw, c, img.dtype)
            self.lib.oracle_crop(_ptr(img), w, h, c, 1, img.itemsize, _ptr(out), left, top, cw, ch)
        return out

    # -- normalize / stats ---------------------------------------------------
    def normalize(self, img, mean, std):
        img = np.ascontiguousarray(img, np.float32)
        w, h, c = _shape(img)
        mean = np.ascontiguousarray(mean, np.float32)
        std = np.ascontiguousarray(std, np.float32)
        out = np.zeros(img.shape, np.float32)
        self.lib.oracle_normalize_f32(_ptr(img), _ptr(out), w * h, c, _ptr(mean), _ptr(std))
        return out

    def mean_stddev_ref(self, img):
        img = np.ascontiguousarray(img, np.float32)
        w, h, c = _shape(img)
        mean = np.zeros(c, np.float32)
        std = np.zeros(c, np.float32)
        self.lib.oracle_mean_stddev_ref_f32(_ptr(img), w * h, c, _ptr(mean), _ptr(std))
        return mean, std

    def channel_sums(self, img):
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        sums = np.zeros(2 * c, np.float64)
        if img.dtype == np.uint8:
            self.lib.oracle_channel_sums_u8(_ptr(img), w * h, c, _ptr(sums))
        else:
            img = np.ascontiguousarray(img, np.float32)
            self.lib.oracle_channel_sums_f64(_ptr(img), w * h, c, _ptr(sums))
        return sums

    def stats_from_sums(self, sums, count):
        sums = np.ascontiguousarray(sums, np.float64)
        c = sums.size // 2
        mean = np.zeros(c, np.float32)
        std = np.zeros(c, np.float32)
        self.lib.oracle_stats_from_sums(_ptr(sums), float(count), c, _ptr(mean), _ptr(std))
        return mean, std

    def mean_stddev_exact(self, img):
        w, h, _ = _shape(img)
        return self.stats_from_sums(self.channel_sums(img), w * h)

    def cosine_u8(self, a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return self.lib.oracle_cosine_f32acc_u8(_ptr(a), _ptr(b), a.size)

    def cosine_f64(self, a, b):
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        return self.lib.oracle_cosine_f64_f32(_ptr(a), _ptr(b), a.size)


class Reference:
    """The reference's own pixel loops (oracle/_ref/libvacv_ref.so)."""

    def __init__(self, path: Path = REF_SO):
        self.lib = ctypes.CDLL(str(path), mode=os.RTLD_LAZY)
        L = self.lib
        for name, args, res in [
            ("ref_resize_linear_u8", [_P, _I, _I, _I, _P, _I, _I], None),
            ("ref_resize_linear_f32", [_P, _I, _I, _I, _P, _I, _I], None),
            ("ref_cubic_coeffs", [_I, _I, _P, _P], None),
            ("ref_resize_cubic_f32", [_P, _I, _I, _I, _P, _I, _I], None),
            ("ref_resize_cubic_f32_hwc_wrapper", [_P, _I, _I, _P, _I, _I], None),
            ("ref_warp_affine_u8", [_P, _I, _I, _I, _P, _I, _I, _P], None),
            ("ref_warp_affine_f32", [_P, _I, _I, _I, _P, _I, _I, _P], None),
            ("ref_mean_stddev_hwc3", [_P, _I, _P, _P], None),
            ("ref_mean_stddev_chw", [_P, _I, _I, _P, _P], None),
            ("ref_normalize_hwc3", [_P, _P, _I, _P, _P], None),
            ("ref_normalize_chw", [_P, _P, _I, _I, _P, _P], None),
            ("ref_nv_to_bgr", [_P, _P, _I, _I, _I, _I], None),
            ("ref_bgr2nv21", [_P, _P, _I, _I], None),
            ("ref_compare_image_data_u8", [_P, _P, _I], _F),
            ("ref_compare_image_data_f32", [_P, _P, _I], _F),
        ]:
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res

    @staticmethod
    def available() -> bool:
        return REF_SO.exists()

    def resize_linear(self, img, w_out, h_out):
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        out = _out(h_out, w_out, c, img.dtype)
        fn = self.lib.ref_resize_linear_u8 if img.dtype == np.uint8 else self.lib.ref_resize_linear_f32
        fn(_ptr(img), w, h, c, _ptr(out), w_out, h_out)
        return out

    def cubic_table(self, n_in, n_out):
        ofs = np.zeros(n_out, np.int32)
        coef = np.zeros((n_out, 4), np.float32)
        self.lib.ref_cubic_coeffs(n_in, n_out, _ptr(ofs), _ptr(coef))
        return ofs, coef

    def resize_cubic(self, img, w_out, h_out, wrapper=False):
        img = np.ascontiguousarray(img, np.float32)
        w, h, c = _shape(img)
        assert c in (1, 3)
        out = _out(h_out, w_out, c, np.float32)
        if wrapper:
            assert c == 3 and w_out == h_out
            self.lib.ref_resize_cubic_f32_hwc_wrapper(_ptr(img), w, h, _ptr(out), w_out, h_out)
        else:
            self.lib.ref_resize_cubic_f32(_ptr(img), w, h, c, _ptr(out), w_out, h_out)
        return out

    def warp_affine_inv(self, img, inv, w_out, h_out, border=0):
        """warp with an already-inverted map (the naive kernel's contract)."""
        img = np.ascontiguousarray(img)
        w, h, c = _shape(img)
        inv = np.ascontiguousarray(inv, np.float32)
        out = _out(h_out, w_out, c, img.dtype)
        out[...] = border
        fn = self.lib.ref_warp_affine_u8 if img.dtype == np.uint8 else self.lib.ref_warp_affine_f32
        fn(_ptr(img), w, h, c, _ptr(out), w_out, h_out, _ptr(inv))
        return out

    def mean_stddev(self, img):
        img = np.ascontiguousarray(img, np.float32)
        w, h, c = _shape(img)
        mean = np.zeros(c, np.float32)
        std = np.zeros(c, np.float32)
        if c == 3:
            self.lib.ref_mean_stddev_hwc3(_ptr(img), w * h, _ptr(mean), _ptr(std))
        else:
            assert c == 1
            self.lib.ref_mean_stddev_chw(_ptr(img), w * h, 1, _ptr(mean), _ptr(std))
        return mean, std

    def mean_stddev_chw(self, planes):
        planes = np.ascontiguousarray(planes, np.float32)
        c, h, w = planes.shape
        mean = np.zeros(c, np.float32)
        std = np.zeros(c, np.float32)
        self.lib.ref_mean_stddev_chw(_ptr(planes), w * h, c, _ptr(mean), _ptr(std))
        return mean, std

    def normalize(self, img, mean, std):
        img = np.ascontiguousarray(img, np.float32)
        w, h, c = _shape(img)
        mean = np.ascontiguousarray(mean, np.float32)
        std = np.ascontiguousarray(std, np.float32)
        out = np.zeros(img.shape, np.float32)
        if c == 3:
            self.lib.ref_normalize_hwc3(_ptr(img), _ptr(out), w * h, _ptr(mean), _ptr(std))
        else:
            assert c == 1
            self.lib.ref_normalize_chw(_ptr(img), _ptr(out), w * h, 1, _ptr(mean), _ptr(std))
        return out

    def normalize_chw(self, planes, mean, std):
        planes = np.ascontiguousarray(planes, np.float32)
        c, h, w = planes.shape
        out = np.zeros(planes.shape, np.float32)
        self.lib.ref_normalize_chw(_ptr(planes), _ptr(out), w * h, c,
                                   _ptr(np.ascontiguousarray(mean, np.float32)),
                                   _ptr(np.ascontiguousarray(std, np.float32)))
        return out

    def nv21_to_bgr(self, yuv):
        yuv = np.ascontiguousarray(yuv, np.uint8)
        h = yuv.shape[0] // 3 * 2
        w = yuv.shape[1]
        out = np.zeros((h, w, 3), np.uint8)
        self.lib.ref_nv_to_bgr(_ptr(yuv), _ptr(out), w, h, 0, 1)
        return out

    def bgr2nv21(self, bgr):
        bgr = np.ascontiguousarray(bgr, np.uint8)
        h, w = bgr.shape[:2]
        out = np.zeros((h * 3 // 2, w), np.uint8)
        self.lib.ref_bgr2nv21(_ptr(bgr), _ptr(out), w, h)
        return out

    def compare_u8(self, a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return self.lib.ref_compare_image_data_u8(_ptr(a), _ptr(b), a.size)


def synthetic_image(seed: int, h: int, w: int, c: int = 3) -> np.ndarray:
    """Deterministic u8 test image: smooth gradients plus splitmix64 noise.

    Restated in tests/golden/make_golden.py's header so fixtures can be
    regenerated anywhere."""
    yy, xx = np.meshgrid(np.arange(h, dtype=np.int64), np.arange(w, dtype=np.int64), indexing="ij")
    base = []
    for k in range(c):
        g = (xx * (37 + 11 * k) // max(w, 1) + yy * (53 + 7 * k) // max(h, 1) + 29 * k) % 256
        base.append(g)
    base = np.stack(base, axis=-1)
    gamma = 0x9E3779B97F4A7C15
    offset = np.array([(seed * gamma) & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64)
    idx = np.arange(h * w * c, dtype=np.uint64) + offset
    z = idx * np.uint64(gamma)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    noise = (z & np.uint64(0x7F)).astype(np.int64).reshape(h, w, c) - 64
    img = np.clip(base + noise, 0, 255).astype(np.uint8)
    return img if c > 1 else img[..., 0]
