"""Batched vacv operators on device tensors, through the C ABI.

The names and argument meanings follow the reference's ``va_cv::`` API
(/root/reference/src/cv/cv.h:85-209); every call goes straight to a HIP
kernel in lib/libvacv_hip.so.  PyTorch is only the allocator and the stream
provider here: tensors must live on a HIP device, and nothing is computed on
the CPU.

Image tensors
  NHWC: (n, h, w, c), (h, w, c) or (h, w)          -- the reference's default
  NCHW: (n, c, h, w) or (c, h, w)                   -- pass layout=NCHW
Rows may be pitched (e.g. a slice of a larger image) as long as each row's
pixels are contiguous; the descriptor carries the byte pitches.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L
from ._lib import (BORDER_CONSTANT, FP16, FP32, FP64, INT8, INTER_CUBIC, INTER_LINEAR, LINEAR_REFERENCE, NCHW,
                   NHWC, VacvImage, check)

_DTYPES = {torch.uint8: INT8, torch.float32: FP32, torch.float16: FP16, torch.float64: FP64}
_TORCH = {v: k for k, v in _DTYPES.items()}


def _stream(stream=None) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


def _as4d(t: torch.Tensor, layout: int) -> torch.Tensor:
    if t.dim() == 4:
        return t
    if t.dim() == 3:
        return t.unsqueeze(0)
    if t.dim() == 2:
        return t.unsqueeze(0).unsqueeze(-1 if layout == NHWC else 1)
    raise ValueError(f"expected a 2-4 dimensional image tensor, got shape {tuple(t.shape)}")


def describe(t: torch.Tensor, layout: int = NHWC) -> VacvImage:
    """vacv_image descriptor of a device tensor (no copy)."""
    if not t.is_cuda:
        raise ValueError("vacv operators take device tensors (the C++ API stages host images)")
    if t.dtype not in _DTYPES:
        raise TypeError(f"unsupported dtype {t.dtype}")
    t4 = _as4d(t, layout)
    es = t4.element_size()
    st = t4.stride()
    # strides of size-1 dimensions are meaningless (numpy/torch may report 0):
    # pass 0 there and let the C side use the dense pitch
    if layout == NHWC:
        n, h, w, c = t4.shape
        if (c > 1 and st[3] != 1) or (w > 1 and st[2] != c):
            raise ValueError("NHWC rows must be contiguous (pixel stride == c)")
        row, plane, batch = (st[1] * es if h > 1 else 0), 0, (st[0] * es if n > 1 else 0)
    else:
        n, c, h, w = t4.shape
        if w > 1 and st[3] != 1:
            raise ValueError("NCHW rows must be contiguous")
        row, plane, batch = (st[2] * es if h > 1 else 0), (st[1] * es if c > 1 else 0), (st[0] * es if n > 1 else 0)
    return VacvImage(t4.data_ptr(), n, w, h, c, _DTYPES[t.dtype], layout, row, plane, batch)


def _empty_like_shape(src4: torch.Tensor, layout: int, w: int, h: int, dtype, squeeze: bool, src_dim: int,
                      c: Optional[int] = None):
    n = src4.shape[0]
    c = c if c is not None else (src4.shape[3] if layout == NHWC else src4.shape[1])
    shape = (n, h, w, c) if layout == NHWC else (n, c, h, w)
    out = torch.empty(shape, dtype=dtype, device=src4.device)
    return out


def _shape_back(out4: torch.Tensor, src: torch.Tensor, layout: int) -> torch.Tensor:
    if src.dim() == 4:
        return out4
    if src.dim() == 3:
        return out4[0]
    return out4[0, ..., 0] if layout == NHWC else out4[0, 0]


def _fptr(a) -> Tuple[object, ctypes.POINTER(ctypes.c_float)]:
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
    return arr, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _dptr(a) -> Tuple[object, ctypes.POINTER(ctypes.c_double)]:
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
    return arr, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _meanstd(mean, std, c):
    if mean is None and std is None:
        return (None, None), (None, None)
    if mean is None or std is None:
        raise ValueError("give both mean and stddev, or neither (per-image statistics)")
    m, s = _fptr(mean), _fptr(std)
    if m[0].size != c or s[0].size != c:
        raise ValueError(f"mean/stddev need {c} values")
    return m, s


# ---------------------------------------------------------------------------
# geometry / dtype

def crop(src: torch.Tensor, rect: Sequence[float], layout: int = NHWC, out=None, stream=None) -> torch.Tensor:
    """va_cv::crop (cv.h:209): rect = (left, top, right, bottom), truncated
    to int exactly as crop_naive does (crop.cpp:128-131)."""
    left, top = int(rect[0]), int(rect[1])
    cw, ch = int(np.float32(rect[2]) - np.float32(rect[0])), int(np.float32(rect[3]) - np.float32(rect[1]))
    s4 = _as4d(src, layout)
    if out is None:
        out = _empty_like_shape(s4, layout, cw, ch, src.dtype, True, src.dim())
    o4 = _as4d(out, layout)
    check("vacv_crop", L.load().vacv_crop(ctypes.byref(describe(s4, layout)), ctypes.byref(describe(o4, layout)),
                                          left, top, _stream(stream)))
    return _shape_back(o4, src, layout)


def change_layout(src: torch.Tensor, to_layout: int, layout: int = NHWC, stream=None) -> torch.Tensor:
    """Tensor::change_layout (tensor.cpp:393-457)."""
    s4 = _as4d(src, layout)
    if layout == NHWC:
        n, h, w, c = s4.shape
    else:
        n, c, h, w = s4.shape
    out = torch.empty((n, h, w, c) if to_layout == NHWC else (n, c, h, w), dtype=src.dtype, device=src.device)
    check("vacv_change_layout", L.load().vacv_change_layout(ctypes.byref(describe(s4, layout)),
                                                            ctypes.byref(describe(out, to_layout)), _stream(stream)))
    return out


def change_dtype(src: torch.Tensor, dtype: torch.dtype, layout: int = NHWC, stream=None) -> torch.Tensor:
    """Tensor::change_dtype (tensor.cpp:459-502): u8<->fp32."""
    s4 = _as4d(src, layout)
    out = torch.empty(s4.shape, dtype=dtype, device=src.device)
    check("vacv_change_dtype", L.load().vacv_change_dtype(ctypes.byref(describe(s4, layout)),
                                                          ctypes.byref(describe(out, layout)), _stream(stream)))
    return _shape_back(out, src, layout)


def resize(src: torch.Tensor, w: int, h: int, interpolation: int = INTER_LINEAR, mode: int = LINEAR_REFERENCE,
           layout: int = NHWC, out=None, stream=None, fx: float = 0.0, fy: float = 0.0) -> torch.Tensor:
    """va_cv::resize (cv.h:85-87).  INTER_CUBIC on u8 input returns fp32.
    w = h = 0 with fx, fy > 0 (INTER_NEAREST / INTER_AREA / INTER_LANCZOS4): cv::resize's
    dsize = (round(w_in * fx), round(h_in * fy)) and inv_scale = (fx, fy)."""
    s4 = _as4d(src, layout)
    dt = torch.float32 if (interpolation == INTER_CUBIC) else src.dtype
    scaled = w == 0 and h == 0 and fx > 0 and fy > 0
    if scaled:  # saturate_cast<int>(double): round half to even, as Python's round
        w_in, h_in = (s4.shape[2], s4.shape[1]) if layout == NHWC else (s4.shape[3], s4.shape[2])
        w, h = int(round(w_in * fx)), int(round(h_in * fy))
    if out is None:
        out = _empty_like_shape(s4, layout, w, h, dt, True, src.dim())
    if scaled:
        check("vacv_resize_scaled", L.load().vacv_resize_scaled(
            ctypes.byref(describe(s4, layout)), ctypes.byref(describe(out, layout)), interpolation, mode,
            float(fx), float(fy), _stream(stream)))
    else:
        check("vacv_resize", L.load().vacv_resize(ctypes.byref(describe(s4, layout)),
                                                  ctypes.byref(describe(out, layout)), interpolation, mode,
                                                  _stream(stream)))
    return _shape_back(out, src, layout)


def resize_normalize(src: torch.Tensor, w: int, h: int, mean=None, std=None, interpolation: int = INTER_LINEAR,
                     mode: int = LINEAR_REFERENCE, layout: int = NHWC, out=None, stream=None) -> torch.Tensor:
    """va_cv::resize_normalize (cv.h:154-158): resize, fp32, normalize."""
    s4 = _as4d(src, layout)
    c = s4.shape[3] if layout == NHWC else s4.shape[1]
    if out is None:
        out = _empty_like_shape(s4, layout, w, h, torch.float32, True, src.dim())
    (ma, mp), (sa, sp) = _meanstd(mean, std, c)
    check("vacv_resize_normalize",
          L.load().vacv_resize_normalize(ctypes.byref(describe(s4, layout)), ctypes.byref(describe(out, layout)),
                                         interpolation, mode, mp, sp, _stream(stream)))
    return _shape_back(out, src, layout)


def rotation_matrix(scale: float, rot: float, aux: Sequence[float] = (0, 0, 0, 0)) -> np.ndarray:
    """get_rotation_matrix_2D + aux fix (warp_affine.cpp:76-109), host."""
    m = np.zeros(6, np.float32)
    a, ap = _dptr(aux)
    check("vacv_rotation_matrix", L.load().vacv_rotation_matrix(scale, rot, ap,
                                                                m.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return m


def invert_affine(m) -> np.ndarray:
    mm, mp = _fptr(m)
    inv = np.zeros(6, np.float32)
    check("vacv_invert_affine", L.load().vacv_invert_affine(mp, inv.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return inv


def warp_affine(src: torch.Tensor, m, w: int, h: int, flags: int = INTER_LINEAR, border_mode: int = BORDER_CONSTANT,
                border_value=(0, 0, 0, 0), layout: int = NHWC, out=None, stream=None) -> torch.Tensor:
    """va_cv::warp_affine (cv.h:118-122); m is the forward 2x3 map, or the
    inverse one with flags | WARP_INVERSE_MAP; flags INTER_LINEAR (the
    reference's naive sampler) or INTER_NEAREST (OpenCV 2.4's)."""
    s4 = _as4d(src, layout)
    if out is None:
        out = _empty_like_shape(s4, layout, w, h, src.dtype, True, src.dim())
    mm, mp = _fptr(m)
    bv, bp = _dptr(border_value)
    check("vacv_warp_affine", L.load().vacv_warp_affine(ctypes.byref(describe(s4, layout)),
                                                        ctypes.byref(describe(out, layout)), mp, flags, border_mode,
                                                        bp, _stream(stream)))
    return _shape_back(out, src, layout)


def warp_affine_rot(src: torch.Tensor, scale: float, rot: float, w: int, h: int, aux=(0, 0, 0, 0), **kw):
    """va_cv::warp_affine(src, dst, scale, rot, dsize, aux, ...) (cv.h:136-141)."""
    return warp_affine(src, rotation_matrix(scale, rot, aux), w, h, **kw)


def warp_affine_normalize(src: torch.Tensor, m, w: int, h: int, mean=None, std=None, flags: int = INTER_LINEAR,
                          border_mode: int = BORDER_CONSTANT, border_value=(0, 0, 0, 0), layout: int = NHWC,
                          out=None, stream=None) -> torch.Tensor:
    """va_cv::warp_affine_normalize (cv.h:172-201)."""
    s4 = _as4d(src, layout)
    c = s4.shape[3] if layout == NHWC else s4.shape[1]
    if out is None:
        out = _empty_like_shape(s4, layout, w, h, torch.float32, True, src.dim())
    mm, mp = _fptr(m)
    bv, bp = _dptr(border_value)
    (ma, meanp), (sa, stdp) = _meanstd(mean, std, c)
    check("vacv_warp_affine_normalize",
          L.load().vacv_warp_affine_normalize(ctypes.byref(describe(s4, layout)), ctypes.byref(describe(out, layout)),
                                              mp, flags, border_mode, bp, meanp, stdp, _stream(stream)))
    return _shape_back(out, src, layout)


# ---------------------------------------------------------------------------
# colour

def _yuv_desc(yuv: torch.Tensor) -> VacvImage:
    y4 = yuv if yuv.dim() == 3 else yuv.unsqueeze(0)
    return describe(y4.unsqueeze(-1), NHWC)


_DCN4 = (L.COLOR_YUV2RGBA_NV12, L.COLOR_YUV2BGRA_NV12, L.COLOR_YUV2RGBA_NV21, L.COLOR_YUV2BGRA_NV21)


def cvt_color(yuv: torch.Tensor, code: int = L.COLOR_YUV2BGR_NV21, out=None, stream=None) -> torch.Tensor:
    """va_cv::cvt_color (cv.h:95): (n, h*3/2, w) u8 -> (n, h, w, 3) u8 (4
    channels for the RGBA/BGRA codes; YV12 is Y then the V and U planes).
    COLOR_GRAY2BGR: (n, h, w) u8/fp32 -> (n, h, w, 3) of the same dtype.
    `out` (optional): a preallocated output of that shape."""
    if code == L.COLOR_GRAY2BGR:
        g4 = yuv if yuv.dim() == 3 else yuv.unsqueeze(0)
        if out is None:
            out = torch.empty(tuple(g4.shape) + (3,), dtype=g4.dtype, device=yuv.device)
        out = out if out.dim() == 4 else out.unsqueeze(0)
        check("vacv_cvt_color", L.load().vacv_cvt_color(ctypes.byref(describe(g4.unsqueeze(-1), NHWC)),
                                                        ctypes.byref(describe(out, NHWC)), code, _stream(stream)))
        return out if yuv.dim() == 3 else out[0]
    y4 = yuv if yuv.dim() == 3 else yuv.unsqueeze(0)
    n, hh, w = y4.shape
    if out is None:
        out = torch.empty((n, hh // 3 * 2, w, 4 if code in _DCN4 else 3), dtype=torch.uint8, device=yuv.device)
    out = out if out.dim() == 4 else out.unsqueeze(0)
    check("vacv_cvt_color", L.load().vacv_cvt_color(ctypes.byref(_yuv_desc(y4)), ctypes.byref(describe(out, NHWC)),
                                                    code, _stream(stream)))
    return out if yuv.dim() == 3 else out[0]


def cvt_color_normalize(yuv: torch.Tensor, code: int = L.COLOR_YUV2BGR_NV21, mean=None, std=None, out=None,
                        stream=None) -> torch.Tensor:
    y4 = yuv if yuv.dim() == 3 else yuv.unsqueeze(0)
    n, hh, w = y4.shape
    if out is None:
        out = torch.empty((n, hh // 3 * 2, w, 3), dtype=torch.float32, device=yuv.device)
    (ma, mp), (sa, sp) = _meanstd(mean, std, 3)
    check("vacv_cvt_color_normalize",
          L.load().vacv_cvt_color_normalize(ctypes.byref(_yuv_desc(y4)), ctypes.byref(describe(out, NHWC)), code, mp,
                                            sp, _stream(stream)))
    return out if yuv.dim() == 3 else out[0]


def cvt_color_resize(yuv: torch.Tensor, w: int, h: int, code: int = L.COLOR_YUV2BGR_NV21, layout: int = NHWC,
                     dtype: torch.dtype = torch.uint8, mode: int = LINEAR_REFERENCE, out=None,
                     stream=None) -> torch.Tensor:
    """cvt_color -> resize(INTER_LINEAR) [-> change_dtype(FP32)] [-> change_layout]
    (cvt_color.cpp:39-157, resize_naive.cpp:10-68) in one kernel:
    (n, h_in*3/2, w_in) u8 -> (n, h, w, 3) NHWC or (n, 3, h, w) NCHW."""
    y4 = yuv if yuv.dim() == 3 else yuv.unsqueeze(0)
    n = y4.shape[0]
    if out is None:
        shape = (n, h, w, 3) if layout == NHWC else (n, 3, h, w)
        out = torch.empty(shape, dtype=dtype, device=yuv.device)
    check("vacv_cvt_color_resize",
          L.load().vacv_cvt_color_resize(ctypes.byref(_yuv_desc(y4)), ctypes.byref(describe(out, layout)), code,
                                         INTER_LINEAR, mode, _stream(stream)))
    return out if yuv.dim() == 3 else out[0]


def cvt_color_resize_normalize(yuv: torch.Tensor, w: int, h: int, mean=None, std=None,
                               code: int = L.COLOR_YUV2BGR_NV21, layout: int = NCHW, mode: int = LINEAR_REFERENCE,
                               out=None, stream=None) -> torch.Tensor:
    """The camera-frame -> model-input step: cvt_color, resize, convert to
    fp32, normalize((x - mean) / (std + 1e-6)), change_layout -- one kernel.
    Default layout NCHW (planar fp32).  mean/std None = per-image stats of
    the resized image (two passes)."""
    y4 = yuv if yuv.dim() == 3 else yuv.unsqueeze(0)
    n = y4.shape[0]
    if out is None:
        shape = (n, h, w, 3) if layout == NHWC else (n, 3, h, w)
        out = torch.empty(shape, dtype=torch.float32, device=yuv.device)
    (ma, mp), (sa, sp) = _meanstd(mean, std, 3)
    check("vacv_cvt_color_resize_normalize",
          L.load().vacv_cvt_color_resize_normalize(ctypes.byref(_yuv_desc(y4)), ctypes.byref(describe(out, layout)),
                                                   code, INTER_LINEAR, mode, mp, sp, _stream(stream)))
    return out if yuv.dim() == 3 else out[0]


# ---------------------------------------------------------------------------
# normalize / statistics

def normalize(src: torch.Tensor, mean=None, std=None, layout: int = NHWC, out=None, stream=None) -> torch.Tensor:
    """va_cv::normalize (cv.h:104-106)."""
    s4 = _as4d(src, layout)
    c = s4.shape[3] if layout == NHWC else s4.shape[1]
    if out is None:
        out = torch.empty(s4.shape, dtype=torch.float32, device=src.device)
    (ma, mp), (sa, sp) = _meanstd(mean, std, c)
    check("vacv_normalize", L.load().vacv_normalize(ctypes.byref(describe(s4, layout)), ctypes.byref(describe(out, layout)),
                                                    mp, sp, _stream(stream)))
    return _shape_back(out, src, layout)


def channel_sums(src: torch.Tensor, per_image: bool = True, layout: int = NHWC, stream=None) -> torch.Tensor:
    """(groups, c, 2) fp64 device tensor of (Sum x, Sum x^2)."""
    s4 = _as4d(src, layout)
    n = s4.shape[0]
    c = s4.shape[3] if layout == NHWC else s4.shape[1]
    out = torch.empty((n if per_image else 1, c, 2), dtype=torch.float64, device=src.device)
    check("vacv_channel_sums", L.load().vacv_channel_sums(ctypes.byref(describe(s4, layout)), out.data_ptr(),
                                                          int(per_image), _stream(stream)))
    return out


def resize_channel_sums(src: torch.Tensor, w: int, h: int, interpolation: int = INTER_LINEAR,
                        mode: int = LINEAR_REFERENCE, per_image: bool = True, layout: int = NHWC, out=None,
                        stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """resize() and channel_sums() of its output in one pass where the kernel
    fuses them (u8 -> fp32 INTER_CUBIC).  Returns (resized, sums)."""
    s4 = _as4d(src, layout)
    if out is None:
        dt = torch.float32 if (interpolation == INTER_CUBIC or src.dtype == torch.float32) else src.dtype
        out = _empty_like_shape(s4, layout, w, h, dt, False, src.dim())
    o4 = _as4d(out, layout)
    c = o4.shape[3] if layout == NHWC else o4.shape[1]
    sums = torch.empty((o4.shape[0] if per_image else 1, c, 2), dtype=torch.float64, device=src.device)
    check("vacv_resize_channel_sums",
          L.load().vacv_resize_channel_sums(ctypes.byref(describe(s4, layout)), ctypes.byref(describe(o4, layout)),
                                            interpolation, mode, sums.data_ptr(), int(per_image), _stream(stream)))
    return out, sums


def resize_mean_stddev(src: torch.Tensor, w: int, h: int, interpolation: int = INTER_LINEAR,
                       mode: int = LINEAR_REFERENCE, per_image: bool = True, layout: int = NHWC, out=None,
                       stream=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """resize() and the population mean / stddev of its output (per image, or
    over the whole batch) in one call: the one-GPU form of cfg5 (resize, then
    normalize_naive.cpp:7-48's mean_stddev).  Returns (resized, sums, mean,
    stddev); sums is (groups, c, 2) fp64, mean / stddev (groups, c) fp32."""
    s4 = _as4d(src, layout)
    if out is None:
        dt = torch.float32 if (interpolation == INTER_CUBIC or src.dtype == torch.float32) else src.dtype
        out = _empty_like_shape(s4, layout, w, h, dt, False, src.dim())
    o4 = _as4d(out, layout)
    c = o4.shape[3] if layout == NHWC else o4.shape[1]
    groups = o4.shape[0] if per_image else 1
    sums = torch.empty((groups, c, 2), dtype=torch.float64, device=src.device)
    mean = torch.empty((groups, c), dtype=torch.float32, device=src.device)
    std = torch.empty((groups, c), dtype=torch.float32, device=src.device)
    check("vacv_resize_mean_stddev",
          L.load().vacv_resize_mean_stddev(ctypes.byref(describe(s4, layout)), ctypes.byref(describe(o4, layout)),
                                           interpolation, mode, sums.data_ptr(), mean.data_ptr(), std.data_ptr(),
                                           int(per_image), _stream(stream)))
    return out, sums, mean, std


def stats_from_sums(sums: torch.Tensor, count: float, stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    sums = sums.contiguous()
    groups, c = sums.shape[0], sums.shape[1]
    mean = torch.empty((groups, c), dtype=torch.float32, device=sums.device)
    std = torch.empty((groups, c), dtype=torch.float32, device=sums.device)
    check("vacv_stats_from_sums", L.load().vacv_stats_from_sums(sums.data_ptr(), groups, c, float(count),
                                                                mean.data_ptr(), std.data_ptr(), _stream(stream)))
    return mean, std


def mean_stddev(src: torch.Tensor, layout: int = NHWC, stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-image (n, c) population mean / stddev (normalize_naive.cpp:7-72)."""
    s4 = _as4d(src, layout)
    n = s4.shape[0]
    c = s4.shape[3] if layout == NHWC else s4.shape[1]
    mean = torch.empty((n, c), dtype=torch.float32, device=src.device)
    std = torch.empty((n, c), dtype=torch.float32, device=src.device)
    check("vacv_mean_stddev", L.load().vacv_mean_stddev(ctypes.byref(describe(s4, layout)), mean.data_ptr(),
                                                        std.data_ptr(), _stream(stream)))
    return mean, std


def match_template(img: torch.Tensor, templ: torch.Tensor, method: int, out=None, stream=None) -> torch.Tensor:
    """va_cv::match_template (cv.h:211-219): cv::matchTemplate of every image
    (NHWC, u8 or fp32) against one template -> (n,) H-h+1 x W-w+1 fp32."""
    i4 = _as4d(img, NHWC)
    t4 = _as4d(templ, NHWC)
    n, H, W, _ = i4.shape
    _, h, w, _ = t4.shape
    if w > W and h > H and n == 1:
        W, H, w, h = w, h, W, H
    if out is None:
        out = torch.empty((n, H - h + 1, W - w + 1), dtype=torch.float32, device=img.device)
    o4 = out.reshape(n, H - h + 1, W - w + 1, 1)  # one channel, NHWC
    check("vacv_match_template", L.load().vacv_match_template(
        ctypes.byref(describe(i4, NHWC)), ctypes.byref(describe(t4, NHWC)), ctypes.byref(describe(o4, NHWC)),
        int(method), _stream(stream)))
    return out if img.dim() == 4 else out[0]


def min_max_idx(src: torch.Tensor, mask: Optional[torch.Tensor] = None, stream=None):
    """va_cv::minMaxIdx (cv.h:221-231) of a 2-D single-channel tensor:
    (min, max, (row, col) of the min, (row, col) of the max)."""
    if src.dim() != 2:
        raise ValueError("minMaxIdx takes a 2-D single-channel tensor")
    vals = torch.empty(2, dtype=torch.float64, device=src.device)
    idx = torch.empty(4, dtype=torch.int32, device=src.device)
    md = ctypes.byref(describe(mask)) if mask is not None else None
    check("vacv_min_max_idx", L.load().vacv_min_max_idx(ctypes.byref(describe(src)), md, vals.data_ptr(),
                                                        idx.data_ptr(), _stream(stream)))
    v = vals.cpu().tolist()
    i = idx.cpu().tolist()
    return v[0], v[1], (i[0], i[1]), (i[2], i[3])


def set_tuning(name: str, value: int) -> int:
    """Select a kernel variant (VACV_TUNE_<name>, include/vacv_hip.h); value
    < 0 restores the built-in choice.  Returns the previous value."""
    key = L.TUNE[name]
    lib = L.load()
    old = lib.vacv_get_tuning(key)
    check("vacv_set_tuning", lib.vacv_set_tuning(key, int(value)))
    return old


class tuning:
    """Context manager: `with ops.tuning(WARP_KERNEL=0): ...` runs the block
    with those kernel variants and restores the previous choices after."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.old = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.old[k] = set_tuning(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_tuning(k, v)
        return False
