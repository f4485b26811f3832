// vacv_abi.cpp -- the extern "C" entry points of include/vacv_hip.h.
//
// Host side of every operator: validate the descriptors (the reference
// silently does nothing or recurses forever on unsupported input, SURVEY.md
// App. C; here that is a status code), derive the geometry, plan the tiles,
// and queue kernels on the caller's stream.  No call synchronises the device
// and no C++ exception escapes.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <mutex>
#include <tuple>
#include <utility>

#include "vacv_internal.hpp"
#include "vacv_semantics.hpp"

namespace vacv {
namespace {

int esize_of(int dtype) {
    switch (dtype) {
        case VACV_FP32: return 4;
        case VACV_FP16: return 2;
        case VACV_INT8: return 1;
        case VACV_FP64: return 8;
        default: return 0;
    }
}

// A validated descriptor with every pitch filled in.
struct Img {
    unsigned char* data;
    int n, w, h, c, dtype, layout, es;
    int64_t row, plane, batch;
};

int load(const vacv_image* d, Img& m) {
    if (!d || !d->data) return VACV_ERR_INVALID_ARG;
    if (d->n < 1 || d->w < 1 || d->h < 1 || d->c < 1) return VACV_ERR_INVALID_ARG;
    m.es = esize_of(d->dtype);
    if (!m.es) return VACV_ERR_UNSUPPORTED;
    if (d->layout != VACV_NHWC && d->layout != VACV_NCHW) return VACV_ERR_UNSUPPORTED;
    m.data = static_cast<unsigned char*>(d->data);
    m.n = d->n; m.w = d->w; m.h = d->h; m.c = d->c;
    m.dtype = d->dtype; m.layout = d->layout;
    const int64_t min_row = (int64_t)m.w * (m.layout == VACV_NHWC ? m.c : 1) * m.es;
    m.row = d->row_pitch ? d->row_pitch : min_row;
    if (m.row < min_row) return VACV_ERR_INVALID_ARG;
    if (m.layout == VACV_NCHW) {
        const int64_t min_plane = m.row * (m.h - 1) + min_row;
        m.plane = d->plane_pitch ? d->plane_pitch : m.row * m.h;
        if (m.plane < min_plane) return VACV_ERR_INVALID_ARG;
        const int64_t min_batch = m.plane * (m.c - 1) + min_plane;
        m.batch = d->batch_pitch ? d->batch_pitch : m.plane * m.c;
        if (m.n > 1 && m.batch < min_batch) return VACV_ERR_INVALID_ARG;
    } else {
        m.plane = 0;
        const int64_t min_batch = m.row * (m.h - 1) + min_row;
        m.batch = d->batch_pitch ? d->batch_pitch : m.row * m.h;
        if (m.n > 1 && m.batch < min_batch) return VACV_ERR_INVALID_ARG;
    }
    return VACV_OK;
}

bool dense(const Img& m) {
    const int64_t row = (int64_t)m.w * (m.layout == VACV_NHWC ? m.c : 1) * m.es;
    if (m.row != row) return false;
    if (m.layout == VACV_NCHW && m.plane != row * m.h) return false;
    const int64_t img = row * m.h * (m.layout == VACV_NCHW ? m.c : 1);
    return m.n == 1 || m.batch == img;
}

PlaneGeom geom(const Img& m) {
    PlaneGeom g;
    g.base = m.data;
    g.img_pitch = m.batch;
    g.row_pitch = m.row;
    g.w = m.w;
    g.h = m.h;
    g.esize = m.es;
    if (m.layout == VACV_NHWC) {
        g.planes = 1;
        g.cc = m.c;
        g.plane_pitch = 0;
    } else {
        g.planes = m.c;
        g.cc = 1;
        g.plane_pitch = m.plane;
    }
    g.plane_bytes = m.row * (m.h - 1) + (int64_t)m.w * g.cc * m.es;
    return g;
}

int hip_status(hipError_t e) { return e == hipSuccess ? VACV_OK : VACV_ERR_HIP; }

bool same_shape(const Img& a, const Img& b) {
    return a.n == b.n && a.w == b.w && a.h == b.h && a.c == b.c && a.layout == b.layout;
}

// ---- per-(device, stream) workspace for the statistics paths ---------------
struct Workspace {
    void* buf = nullptr;
    size_t cap = 0;
};
std::mutex g_ws_mu;
std::map<std::tuple<int, void*, int>, Workspace> g_ws;

// zero_new: a new allocation is zeroed (queued on s, so before any use)
int workspace(hipStream_t s, size_t bytes, void** out, int slot = 0, bool zero_new = false) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VACV_ERR_HIP;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    Workspace& w = g_ws[std::make_tuple(dev, (void*)s, slot)];
    if (w.cap < bytes) {
        if (w.buf) {
            // the previous buffer may still be read by queued work
            if (hipStreamSynchronize(s) != hipSuccess) return VACV_ERR_HIP;
            (void)hipFree(w.buf);
            w.buf = nullptr;
            w.cap = 0;
        }
        size_t cap = std::max<size_t>(bytes, 1 << 20);
        if (hipMalloc(&w.buf, cap) != hipSuccess) return VACV_ERR_NO_MEMORY;
        w.cap = cap;
        if (zero_new && hipMemsetAsync(w.buf, 0, cap, s) != hipSuccess) return VACV_ERR_HIP;
    }
    *out = w.buf;
    return VACV_OK;
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---- statistics -------------------------------------------------------------
// Sum / Sum^2 per channel of `m` into `sums` ([groups][c][2] doubles, device).
int channel_sums_into(const Img& m, double* sums, int per_image, double* partials, int blocks, hipStream_t s) {
    SumsLaunch L{};
    L.src = geom(m);
    L.n = m.n;
    L.c = m.c;
    L.src_u8 = m.dtype == VACV_INT8;
    L.blocks_per_image = blocks;
    L.partials = partials;
    L.sums = sums;
    L.per_image = per_image;
    L.scalar_only = 0;
    for (int i = 0; i < m.n && !L.scalar_only; ++i)
        for (int p = 0; p < L.src.planes; ++p) {
            uintptr_t a = reinterpret_cast<uintptr_t>(m.data + (int64_t)i * m.batch + (int64_t)p * L.src.plane_pitch);
            if (a & 15) { L.scalar_only = 1; break; }
        }
    return hip_status(launch_channel_sums(L, s));
}

int sums_blocks(const Img& m) {
    const int64_t elems = (int64_t)m.w * m.h * (m.layout == VACV_NHWC ? m.c : 1);
    const int64_t planes = (int64_t)m.n * (m.layout == VACV_NHWC ? 1 : m.c);
    // ~1-4K workgroups over the whole batch, >= 4K elements each
    int64_t b = std::max<int64_t>(1, 2048 / std::max<int64_t>(planes, 1));
    b = std::min<int64_t>(b, std::max<int64_t>(1, elems / 4096));
    return (int)std::min<int64_t>(b, 1024);
}

// Per-image mean/std of `m` into workspace arrays; returns device pointers.
int per_image_stats(const Img& m, hipStream_t s, float** mean, float** stdv) {
    if (m.layout == VACV_NHWC && m.c > 4) return VACV_ERR_UNSUPPORTED;
    if (!dense(m)) return VACV_ERR_UNSUPPORTED;
    const int blocks = sums_blocks(m);
    const int planes = m.layout == VACV_NHWC ? 1 : m.c;
    const int cc = m.layout == VACV_NHWC ? m.c : 1;
    const size_t part_b = align_up((size_t)m.n * planes * blocks * 2 * cc * sizeof(double), 256);
    const size_t sums_b = align_up((size_t)m.n * m.c * 2 * sizeof(double), 256);
    const size_t stat_b = align_up((size_t)m.n * m.c * sizeof(float), 256);
    void* ws = nullptr;
    int st = workspace(s, part_b + sums_b + 2 * stat_b, &ws);
    if (st) return st;
    char* p = static_cast<char*>(ws);
    double* partials = reinterpret_cast<double*>(p);
    double* sums = reinterpret_cast<double*>(p + part_b);
    *mean = reinterpret_cast<float*>(p + part_b + sums_b);
    *stdv = reinterpret_cast<float*>(p + part_b + sums_b + stat_b);
    st = channel_sums_into(m, sums, 1, partials, blocks, s);
    if (st) return st;
    return hip_status(launch_stats(sums, m.n, m.c, (double)m.w * m.h, *mean, *stdv, s));
}

int norm_spec(const Img& shape, const float* mean, const float* stdv, NormSpec& ns) {
    std::memset(&ns, 0, sizeof(ns));
    ns.c_total = shape.c;
    if (!mean && !stdv) return VACV_OK;  // caller fills mode 2
    if (!mean || !stdv) return VACV_ERR_INVALID_ARG;
    if (shape.c > kMaxC) return VACV_ERR_UNSUPPORTED;
    ns.mode = 1;
    ns.mul_ok = 0;
    ns.f32_ok = 0;
    for (int k = 0; k < shape.c; ++k) {
        ns.mean[k] = mean[k];
        ns.stdv[k] = stdv[k];
        ns.inv[k] = 1.0 / ((double)stdv[k] + 1e-6);
        ns.inv_hi[k] = (float)ns.inv[k];
        ns.inv_lo[k] = (float)(ns.inv[k] - (double)ns.inv_hi[k]);
        bool ok = true, ok32 = true;
        for (int v = 0; v < 256; ++v) {
            const float d = (float)v - mean[k];
            const float want = normalize_value((float)v, mean[k], stdv[k]);
            ok = ok && (float)((double)d * ns.inv[k]) == want;
            const float lo = d * ns.inv_lo[k];  // -ffp-contract=off: rounded, then the fma
            const float got = std::fma(d, ns.inv_hi[k], lo);
            ok32 = ok32 && std::memcmp(&got, &want, sizeof(float)) == 0;
        }
        if (ok) ns.mul_ok |= 1u << k;
        if (ok32) ns.f32_ok |= 1u << k;
    }
    return VACV_OK;
}

// In-place normalize of an fp32 image with per-image device statistics.
int normalize_with(const Img& src, const Img& dst, const NormSpec& ns, hipStream_t s) {
    NormLaunch L{};
    L.src = geom(src);
    L.dst = geom(dst);
    L.n = src.n;
    L.src_u8 = src.dtype == VACV_INT8;
    L.norm = ns;
    return hip_status(launch_normalize(L, s));
}

// fx / fy > 0: cv::resize's inv_scale (the reference passes them through to
// OpenCV for NEAREST / AREA, resize.cpp:35); 0: dsize / ssize
// FusedSums: the cubic gather kernel's per-workgroup statistics epilogue
// (vacv_resize_channel_sums / vacv_resize_mean_stddev); `used` tells whether
// that kernel ran with it.
struct FusedSums {
    double* partials;            // [cc][2][n][workgroups], sized by the caller
    double* sums;                // [n][cc][2] (per_image) or [cc][2]
    int per_image;
    float* mean;                 // [n][cc] or [cc], or null
    float* stddev;
    int groups;                  // out: workgroups per plane
    bool used;                   // out
    int64_t* acc;                // [n][cc][2], zero between calls (the column kernel's fixed-point sums)
};

int resize_impl(const vacv_image* src_d, const vacv_image* dst_d, int interpolation, int mode, int out_kind,
                const NormSpec* ns, hipStream_t s, double fx = 0.0, double fy = 0.0, FusedSums* fs = nullptr) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (src.n != dst.n || src.c != dst.c || src.layout != dst.layout) return VACV_ERR_INVALID_ARG;
    if (src.layout == VACV_NHWC && src.c > 4) return VACV_ERR_UNSUPPORTED;
    if (mode < VACV_LINEAR_REFERENCE || mode > VACV_LINEAR_OPENCV) return VACV_ERR_INVALID_ARG;

    ResizeLaunch L{};
    L.src = geom(src);
    L.dst = geom(dst);
    // the kernel addresses one plane through a 32-bit buffer resource
    if (L.src.plane_bytes > kMaxPlaneBytes || L.dst.plane_bytes > kMaxPlaneBytes) return VACV_ERR_UNSUPPORTED;
    L.n = src.n;
    L.mode = mode;
    L.out = out_kind;
    if (ns) L.norm = *ns;
    if (interpolation == VACV_INTER_LINEAR) {
        if (src.w < 2 || src.h < 2) return VACV_ERR_INVALID_ARG;  // resize_naive.cpp:28-31 needs 2 taps
        if (src.dtype == VACV_INT8) {
            L.kind = kLinearFixed;
            const int want = out_kind == kOutSame ? VACV_INT8 : VACV_FP32;
            if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
        } else if (src.dtype == VACV_FP32) {
            L.kind = kLinearFloat;
            if (dst.dtype != VACV_FP32) return VACV_ERR_INVALID_ARG;
            if (out_kind == kOutF32) L.out = kOutSame;
        } else {
            return VACV_ERR_UNSUPPORTED;
        }
    } else if (interpolation == VACV_INTER_CUBIC) {
        if (src.w < 4 || src.h < 4) return VACV_ERR_INVALID_ARG;  // resize_naive.cpp:154-181 folds need 4
        if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
        if (dst.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;  // u8 cubic = fused widen to fp32
        L.kind = kCubic;
        if (L.out == kOutSame && src.dtype == VACV_INT8) L.out = kOutF32;
        if (L.out == kOutF32 && src.dtype == VACV_FP32) L.out = kOutSame;
    } else if (interpolation == VACV_INTER_NEAREST) {
        // resize.cpp:44-49 hands it to cv::resize (recursing forever without
        // OpenCV); OpenCV 2.4's resizeNN semantics
        if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
        L.out = out_kind;
        if (src.dtype == VACV_FP32 && L.out == kOutF32) L.out = kOutSame;
        const int want = L.out == kOutSame ? src.dtype : VACV_FP32;
        if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
        L.scale_xd = 1. / (fx > 0 ? fx : (double)dst.w / src.w);  // ifx, as cv::resize computes it
        L.scale_yd = 1. / (fy > 0 ? fy : (double)dst.h / src.h);
        return hip_status(launch_resize_nearest(L, s));
    } else if (interpolation == VACV_INTER_AREA) {
        // resize.cpp:44-49 hands it to cv::resize; OpenCV 2.4 (imgwarp.cpp)
        // takes resizeAreaFast_ when both scales are integers to within
        // DBL_EPSILON, resizeArea_'s weight tables for other down-scales and
        // its bilinear resize with area-mode taps for up-scales (k_area.hip)
        if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
        L.out = out_kind;
        if (src.dtype == VACV_FP32 && L.out == kOutF32) L.out = kOutSame;
        const int want = L.out == kOutSame ? src.dtype : VACV_FP32;
        if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
        const double ifx = fx > 0 ? fx : (double)dst.w / src.w, ify = fy > 0 ? fy : (double)dst.h / src.h;
        const double sx = 1. / ifx, sy = 1. / ify;
        const double ix = std::nearbyint(sx), iy = std::nearbyint(sy);
        if (sx >= 1 && sy >= 1 && std::fabs(sx - ix) < DBL_EPSILON && std::fabs(sy - iy) < DBL_EPSILON) {
            L.area_x = (int)ix;
            L.area_y = (int)iy;
            // an fx-derived size with partial blocks (OpenCV averages those by
            // count) is not built
            if ((int64_t)dst.w * L.area_x != src.w || (int64_t)dst.h * L.area_y != src.h) return VACV_ERR_UNSUPPORTED;
            L.area_scale = 1.f / (float)(L.area_x * L.area_y);
            // OpenCV's ResizeAreaFastVec<uchar>::fast_mode: 2x2 blocks with 1, 3 or
            // 4 interleaved channels (an NCHW plane is one) take (a+b+c+d+2)>>2
            L.area_half_up = src.dtype == VACV_INT8 && L.area_x == 2 && L.area_y == 2 &&
                             (L.src.cc == 1 || L.src.cc == 3 || L.src.cc == 4);
            return hip_status(launch_resize_area(L, s));
        }
        return launch_resize_area_general(L, ifx, ify, s);
    } else if (interpolation == VACV_INTER_LANCZOS4) {
        // resize.cpp:46-48 hands it to cv::resize; OpenCV 2.4's 8x8 Lanczos
        // (k_lanczos.hip), u8 in fixed point, fp32 in float
        if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
        L.out = out_kind;
        if (src.dtype == VACV_FP32 && L.out == kOutF32) L.out = kOutSame;
        const int want = L.out == kOutSame ? src.dtype : VACV_FP32;
        if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
        const double ifx = fx > 0 ? fx : (double)dst.w / src.w, ify = fy > 0 ? fy : (double)dst.h / src.h;
        return launch_resize_lanczos(L, ifx, ify, s);
    } else {
        return VACV_ERR_UNSUPPORTED;  // resize.cpp:46-49 recurses forever for other modes
    }
    L.scale_xf = (float)src.w / (float)dst.w;
    L.scale_yf = (float)src.h / (float)dst.h;
    L.scale_xd = (double)src.w / (double)dst.w;
    L.scale_yd = (double)src.h / (double)dst.h;
    // u8 bilinear whose output rows each weight ONE source row (downscales by
    // an integer factor >= 2, e.g. the 1080p -> 640x360 headline): the
    // per-pixel gather kernel (k_resize_direct.hip).  Elsewhere the staged
    // kernel measured faster (1280x720: 0.63 vs 0.69 ms).  VACV_TUNE_RESIZE_DIRECT
    // = 0 never / 2 always uses the gather kernel, for A/B tests (3: as 1; the
    // NV21 resize then also leaves out its point-sampling instance, A/B).
    // Otherwise resize_kernel with interleaved (address-ordered) tasks;
    // VACV_TUNE_RESIZE_INTERLEAVE = 0 selects its strip order.
    const int direct = tune_or(VACV_TUNE_RESIZE_DIRECT, 1);
    if (L.kind == kLinearFixed && L.src.cc <= 4 && dst.w < (1 << 23) && dst.h < (1 << 23) &&
        (direct == 2 || ((direct == 1 || direct == 3) && resize_one_tap_rows(L))))
        return hip_status(launch_resize_direct(L, s));
    // the other u8 bilinear geometries (two weighted rows per output row):
    // column strips with an LDS ring of source rows (k_resize_strip.hip;
    // 1080p -> 1280x720: 0.565 vs 0.62 ms staged); VACV_TUNE_RESIZE_STRIP = 0
    // selects the staged kernel below, 2 the strip kernel's 128-column strips
    if (L.kind == kLinearFixed && tune_or(VACV_TUNE_RESIZE_STRIP, 1) >= 1 && resize_strip_applies(L))
        return hip_status(launch_resize_strip(L, s));
    // u8 cubic (fused widen to fp32), c <= 3 interleaved: per-pixel gathers
    // (k_cubic_direct.hip); VACV_CUBIC_DIRECT=0 selects the staged kernel
    if (cubic_direct_applies(L)) {
        if (fs && L.out == kOutF32 && fs->partials && L.src.planes == 1) {
            L.sum_partials = fs->partials;
            L.sum_out = fs->sums;
            L.sum_per_image = fs->per_image;
            L.sum_mean = fs->mean;
            L.sum_std = fs->stddev;
            L.sum_acc = fs->acc;
            fs->groups = cubic_direct_groups(L);
            fs->used = true;
        }
        return hip_status(launch_cubic_direct(L, s));
    }
    L.interleave = tune(VACV_TUNE_RESIZE_INTERLEAVE) != 0;
    if ((st = plan_resize(L, s))) return st;
    return hip_status(launch_resize(L, s));
}

int copy_rows(const Img& src, const Img& dst, int64_t src_off, int rows_h, int64_t row_bytes, hipStream_t s) {
    CopyLaunch L{};
    L.src = geom(src);
    L.dst = geom(dst);
    L.src.base += src_off;
    L.src.h = rows_h;
    L.n = src.n;
    L.row_bytes = row_bytes;
    return hip_status(launch_row_copy(L, s));
}

int dtype_convert(const Img& src, const Img& dst, hipStream_t s) {
    if (!dense(src) || !dense(dst)) return VACV_ERR_UNSUPPORTED;
    DtypeLaunch L{};
    L.src = src.data;
    L.dst = dst.data;
    L.count = (int64_t)src.n * src.w * src.h * src.c;
    L.to_f32 = src.dtype == VACV_INT8;
    return hip_status(launch_dtype(L, s));
}

int border_values(const Img& src, const double* bv, float out[4]) {
    for (int k = 0; k < 4; ++k) {
        const double v = bv ? bv[k] : 0.0;
        if (src.dtype == VACV_INT8) {
            double r = std::nearbyint(v);
            out[k] = (float)std::min(255.0, std::max(0.0, r));
        } else {
            out[k] = (float)v;
        }
    }
    return VACV_OK;
}

int warp_impl(const vacv_image* src_d, const vacv_image* dst_d, const float m[6], int flags, int border_mode,
              const double bv[4], int out_kind, const NormSpec* ns, hipStream_t s) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (!m) return VACV_ERR_INVALID_ARG;
    if (src.n != dst.n || src.c != dst.c || src.layout != dst.layout) return VACV_ERR_INVALID_ARG;
    if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
    // warp_affine.cpp:114-118: anything but LINEAR + CONSTANT recurses into the
    // OpenCV stub; the other border modes are built here (vacv_semantics.hpp
    // border_index: the naive sampler with OpenCV's borderInterpolate taps)
    // flags as cv::warpAffine reads them (the reference hands every flag but
    // INTER_LINEAR to OpenCV): the interpolation in bits 0-2, WARP_INVERSE_MAP
    // (m is already the dst -> src map: no inversion).  INTER_LINEAR keeps the
    // naive sampler; INTER_NEAREST is OpenCV 2.4's fixed-point nearest.
    const int interp = flags & 7;
    const bool inverse_map = (flags & VACV_WARP_INVERSE_MAP) != 0;
    if (flags & ~(7 | VACV_WARP_INVERSE_MAP)) return VACV_ERR_UNSUPPORTED;
    if (interp != VACV_INTER_LINEAR && interp != VACV_INTER_NEAREST) return VACV_ERR_UNSUPPORTED;
    if (border_mode < VACV_BORDER_CONSTANT || border_mode > VACV_BORDER_TRANSPARENT) return VACV_ERR_UNSUPPORTED;
    if (src.layout == VACV_NHWC && src.c > 4) return VACV_ERR_UNSUPPORTED;
    if (interp == VACV_INTER_LINEAR && (src.w < 2 || src.h < 2)) return VACV_ERR_INVALID_ARG;
    WarpLaunch L{};
    L.src = geom(src);
    L.dst = geom(dst);
    L.n = src.n;
    L.out = out_kind;
    if (src.dtype == VACV_FP32 && out_kind == kOutF32) L.out = kOutSame;
    const int want = (L.out == kOutSame) ? src.dtype : VACV_FP32;
    if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
    if (inverse_map) std::memcpy(L.inv, m, sizeof(L.inv));
    else vacv_invert_affine(m, L.inv);
    border_values(src, bv, L.border);
    L.border_mode = border_mode;
    if (border_mode == VACV_BORDER_TRANSPARENT && dst.data == src.data) return VACV_ERR_INVALID_ARG;  // in place
    if (ns) L.norm = *ns;
    if (interp == VACV_INTER_NEAREST) {
        // cv::warpAffine: the float map widened to double and, unless
        // WARP_INVERSE_MAP, inverted in double (imgwarp.cpp)
        double* M = L.invd;
        for (int i = 0; i < 6; ++i) M[i] = (double)m[i];
        if (!inverse_map) {
            double D = M[0] * M[4] - M[1] * M[3];
            D = D != 0 ? 1. / D : 0;
            const double A11 = M[4] * D, A22 = M[0] * D;
            M[0] = A11;
            M[1] *= -D;
            M[3] *= -D;
            M[4] = A22;
            const double b1 = -M[0] * M[2] - M[1] * M[5];
            const double b2 = -M[3] * M[2] - M[4] * M[5];
            M[2] = b1;
            M[5] = b2;
        }
        return hip_status(launch_warp_nearest(L, s));
    }
    return hip_status(launch_warp(L, s));
}

int color_code(int code, int& v_first, int& rgb) {
    switch (code) {
        case VACV_COLOR_YUV2BGR_NV21: v_first = 1; rgb = 0; return VACV_OK;
        case VACV_COLOR_YUV2RGB_NV21: v_first = 1; rgb = 1; return VACV_OK;
        case VACV_COLOR_YUV2BGR_NV12: v_first = 0; rgb = 0; return VACV_OK;
        case VACV_COLOR_YUV2RGB_NV12: v_first = 0; rgb = 1; return VACV_OK;
        default: return VACV_ERR_UNSUPPORTED;
    }
}

int color_impl(const vacv_image* src_d, const vacv_image* dst_d, int code, int out_kind, const NormSpec* ns,
               hipStream_t s) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    int v_first, rgb;
    if ((st = color_code(code, v_first, rgb))) return st;
    if (src.dtype != VACV_INT8 || src.c != 1) return VACV_ERR_INVALID_ARG;
    const int h = src.h / 3 * 2;  // cvt_color.cpp:152
    if (src.w % 2 || h % 2 || h < 2 || src.h != h / 2 * 3) return VACV_ERR_INVALID_ARG;
    if (dst.w != src.w || dst.h != h || dst.c != 3 || dst.layout != VACV_NHWC || dst.n != src.n)
        return VACV_ERR_INVALID_ARG;
    const int want = out_kind == kOutSame ? VACV_INT8 : VACV_FP32;
    if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
    ColorLaunch L{};
    L.src = src.data;
    L.src_img = src.batch;
    L.src_row = src.row;
    L.dst = dst.data;
    L.dst_img = dst.batch;
    L.dst_row = dst.row;
    L.n = src.n;
    L.w = src.w;
    L.h = h;
    L.v_first = v_first;
    L.rgb = rgb;
    L.out = out_kind;
    if (ns) L.norm = *ns;
    return hip_status(launch_color(L, s));
}

// The cvt_color codes the reference hands to cv::cvtColor (cvt_color.cpp:
// 139-141), OpenCV 2.4's arithmetic (k_color_cv.hip).
int color_cv_impl(const vacv_image* src_d, const vacv_image* dst_d, int code, hipStream_t s) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (src.layout != VACV_NHWC || dst.layout != VACV_NHWC || src.c != 1 || dst.n != src.n) return VACV_ERR_INVALID_ARG;
    CvColorLaunch L{};
    L.src = src.data;
    L.src_img = src.batch;
    L.src_row = src.row;
    L.dst = dst.data;
    L.dst_img = dst.batch;
    L.dst_row = dst.row;
    L.n = src.n;
    L.w = src.w;
    if (code == VACV_COLOR_GRAY2BGR) {
        if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
        if (dst.dtype != src.dtype || dst.w != src.w || dst.h != src.h || dst.c != 3) return VACV_ERR_INVALID_ARG;
        if (src.es == 4 && ((src.row | dst.row | src.batch | dst.batch) % 4 ||
                            reinterpret_cast<uintptr_t>(src.data) % 4 || reinterpret_cast<uintptr_t>(dst.data) % 4))
            return VACV_ERR_INVALID_ARG;
        L.gray = 1;
        L.h = src.h;
        L.dcn = 3;
        L.esize = src.es;
        return hip_status(launch_color_cv(L, s));
    }
    if (src.dtype != VACV_INT8 || dst.dtype != VACV_INT8) return VACV_ERR_INVALID_ARG;
    const int h = src.h / 3 * 2;  // cvt_color.cpp:152, as cv::cvtColor's YUV420 sizes
    if (src.w % 2 || h % 2 || h < 2 || src.h != h / 2 * 3) return VACV_ERR_INVALID_ARG;
    L.h = h;
    switch (code) {
        case VACV_COLOR_YUV2RGBA_NV12: L.layout = 0; L.dcn = 4; L.bidx = 2; break;
        case VACV_COLOR_YUV2BGRA_NV12: L.layout = 0; L.dcn = 4; L.bidx = 0; break;
        case VACV_COLOR_YUV2RGBA_NV21: L.layout = 1; L.dcn = 4; L.bidx = 2; break;
        case VACV_COLOR_YUV2BGRA_NV21: L.layout = 1; L.dcn = 4; L.bidx = 0; break;
        default: L.layout = 2; L.dcn = 3; L.bidx = 0; break;  // YV12
    }
    if (L.layout == 2 && src.row != src.w) return VACV_ERR_INVALID_ARG;  // planar chroma: dense rows
    if (dst.w != src.w || dst.h != h || dst.c != L.dcn) return VACV_ERR_INVALID_ARG;
    const int al = L.dcn == 4 ? 8 : 2;
    L.aligned = !((dst.row | dst.batch) % al) && !(reinterpret_cast<uintptr_t>(dst.data) % al);
    return hip_status(launch_color_cv(L, s));
}

// YUV420sp -> BGR -> bilinear resize (-> fp32 / normalize) in one kernel
// (k_yuv_resize.hip).  dst = (wo, ho, 3) NHWC or NCHW, INT8 (out_kind
// kOutSame) or FP32.
int yuv_resize_impl(const vacv_image* src_d, const vacv_image* dst_d, int code, int interpolation, int mode,
                    int out_kind, const NormSpec* ns, hipStream_t s) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    int v_first, rgb;
    if ((st = color_code(code, v_first, rgb))) return st;
    if (interpolation != VACV_INTER_LINEAR) return VACV_ERR_UNSUPPORTED;
    if (mode < VACV_LINEAR_REFERENCE || mode > VACV_LINEAR_OPENCV) return VACV_ERR_INVALID_ARG;
    if (src.dtype != VACV_INT8 || src.c != 1 || src.layout != VACV_NHWC) return VACV_ERR_INVALID_ARG;
    const int h = src.h / 3 * 2;  // cvt_color.cpp:152
    // w >= 4: the chroma gather reads 4 bytes within the row
    if (src.w % 2 || h % 2 || h < 2 || src.w < 4 || src.h != h / 2 * 3) return VACV_ERR_INVALID_ARG;
    if (dst.c != 3 || dst.n != src.n) return VACV_ERR_INVALID_ARG;
    const int want = out_kind == kOutSame ? VACV_INT8 : VACV_FP32;
    if (dst.dtype != want) return VACV_ERR_INVALID_ARG;
    const int64_t src_bytes = src.row * (src.h - 1) + src.w;
    const int64_t P = (int64_t)dst.w * dst.h;
    if (src_bytes > kMaxPlaneBytes || P > 0x7FFFFFFFLL - 1024 || src.n > 65535) return VACV_ERR_UNSUPPORTED;
    YuvResizeLaunch L{};
    L.src = src.data;
    L.src_img = src.batch;
    L.src_row = src.row;
    L.src_bytes = src_bytes;
    L.dst = dst.data;
    L.dst_img = dst.batch;
    L.dst_row = dst.row;
    L.dst_plane = dst.plane;
    L.n = src.n;
    L.w = src.w;
    L.h = h;
    L.wo = dst.w;
    L.ho = dst.h;
    L.v_first = v_first;
    L.rgb = rgb;
    L.chw = dst.layout == VACV_NCHW;
    L.mode = mode;
    L.out = out_kind;
    L.scale_xf = (float)L.w / (float)L.wo;
    L.scale_yf = (float)L.h / (float)L.ho;
    L.scale_xd = (double)L.w / (double)L.wo;
    L.scale_yd = (double)L.h / (double)L.ho;
    if (ns) L.norm = *ns;
    return hip_status(launch_yuv_resize(L, s));
}

// Shape of the fp32 output viewed as its own image (for the auto-stats passes).
int fused_normalize(const vacv_image* dst_d, const float* mean, const float* stddev, hipStream_t s,
                    int (*pass)(const void*, int, const NormSpec*, hipStream_t), const void* ctx) {
    Img dst;
    int st = load(dst_d, dst);
    if (st) return st;
    if (dst.dtype != VACV_FP32) return VACV_ERR_INVALID_ARG;
    NormSpec ns;
    if ((st = norm_spec(dst, mean, stddev, ns))) return st;
    if (ns.mode == 1) return pass(ctx, kOutNorm, &ns, s);
    // auto statistics: raw fp32 result, per-image stats of it, normalize in place
    if ((st = pass(ctx, kOutF32, nullptr, s))) return st;
    float *dm = nullptr, *ds = nullptr;
    if ((st = per_image_stats(dst, s, &dm, &ds))) return st;
    ns.mode = 2;
    ns.dev_mean = dm;
    ns.dev_std = ds;
    return normalize_with(dst, dst, ns, s);
}

struct ResizeCtx {
    const vacv_image* src;
    const vacv_image* dst;
    int interpolation, mode;
};
int resize_pass(const void* c, int out, const NormSpec* ns, hipStream_t s) {
    const ResizeCtx* r = static_cast<const ResizeCtx*>(c);
    return resize_impl(r->src, r->dst, r->interpolation, r->mode, out, ns, s);
}

struct WarpCtx {
    const vacv_image* src;
    const vacv_image* dst;
    const float* m;
    int flags, border;
    const double* bv;
};
int warp_pass(const void* c, int out, const NormSpec* ns, hipStream_t s) {
    const WarpCtx* w = static_cast<const WarpCtx*>(c);
    return warp_impl(w->src, w->dst, w->m, w->flags, w->border, w->bv, out, ns, s);
}

struct ColorCtx {
    const vacv_image* src;
    const vacv_image* dst;
    int code;
};
int color_pass(const void* c, int out, const NormSpec* ns, hipStream_t s) {
    const ColorCtx* k = static_cast<const ColorCtx*>(c);
    return color_impl(k->src, k->dst, k->code, out, ns, s);
}

struct YuvResizeCtx {
    const vacv_image* src;
    const vacv_image* dst;
    int code, interpolation, mode;
};
int yuv_resize_pass(const void* c, int out, const NormSpec* ns, hipStream_t s) {
    const YuvResizeCtx* k = static_cast<const YuvResizeCtx*>(c);
    return yuv_resize_impl(k->src, k->dst, k->code, k->interpolation, k->mode, out, ns, s);
}

}  // namespace
}  // namespace vacv

using namespace vacv;

extern "C" {

int vacv_abi_version(void) { return VACV_ABI_VERSION; }

const char* vacv_status_string(int status) {
    switch (status) {
        case VACV_OK: return "ok";
        case VACV_ERR_INVALID_ARG: return "invalid argument";
        case VACV_ERR_UNSUPPORTED: return "unsupported";
        case VACV_ERR_HIP: return "HIP runtime error";
        case VACV_ERR_NO_MEMORY: return "out of device memory";
        default: return "unknown status";
    }
}

int64_t vacv_image_bytes(const vacv_image* d) {
    Img m;
    if (load(d, m)) return -1;
    return m.layout == VACV_NCHW ? m.plane * (m.c - 1) + m.row * (m.h - 1) + (int64_t)m.w * m.es
                                 : m.row * (m.h - 1) + (int64_t)m.w * m.c * m.es;
}

int vacv_crop(const vacv_image* src_d, const vacv_image* dst_d, int left, int top, void* stream) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (src.n != dst.n || src.c != dst.c || src.layout != dst.layout || src.dtype != dst.dtype)
        return VACV_ERR_INVALID_ARG;
    if (left < 0 || top < 0 || left + dst.w > src.w || top + dst.h > src.h) return VACV_ERR_INVALID_ARG;
    const int cc = src.layout == VACV_NHWC ? src.c : 1;
    const int64_t off = (int64_t)top * src.row + (int64_t)left * cc * src.es;
    return copy_rows(src, dst, off, dst.h, (int64_t)dst.w * cc * src.es, (hipStream_t)stream);
}

int vacv_change_layout(const vacv_image* src_d, const vacv_image* dst_d, void* stream) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (src.n != dst.n || src.w != dst.w || src.h != dst.h || src.c != dst.c || src.dtype != dst.dtype)
        return VACV_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (src.layout == dst.layout || src.c == 1) {
        // clone() (tensor.cpp:398-400); a 1-channel image is the same bytes in both layouts
        if (src.layout != dst.layout) {
            if (!dense(src) || !dense(dst)) return VACV_ERR_UNSUPPORTED;
            Img a = src, b = dst;
            a.layout = b.layout = VACV_NHWC;
            return copy_rows(a, b, 0, a.h, (int64_t)a.w * a.es, s);
        }
        const int cc = src.layout == VACV_NHWC ? src.c : 1;
        return copy_rows(src, dst, 0, src.h, (int64_t)src.w * cc * src.es, s);
    }
    if (!dense(src) || !dense(dst)) return VACV_ERR_UNSUPPORTED;
    LayoutLaunch L{};
    L.src = src.data;
    L.dst = dst.data;
    L.n = src.n;
    L.w = src.w;
    L.h = src.h;
    L.c = src.c;
    L.esize = src.es;
    L.to_chw = dst.layout == VACV_NCHW;
    L.src_img = src.batch;
    L.dst_img = dst.batch;
    return hip_status(launch_layout(L, s));
}

int vacv_change_dtype(const vacv_image* src_d, const vacv_image* dst_d, void* stream) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (!same_shape(src, dst)) return VACV_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (src.dtype == dst.dtype) {
        const int cc = src.layout == VACV_NHWC ? src.c : 1;
        return copy_rows(src, dst, 0, src.h, (int64_t)src.w * cc * src.es, s);
    }
    const bool ok = (src.dtype == VACV_INT8 && dst.dtype == VACV_FP32) ||
                    (src.dtype == VACV_FP32 && dst.dtype == VACV_INT8);
    if (!ok) return VACV_ERR_UNSUPPORTED;  // tensor.cpp:494-499 returns garbage
    return dtype_convert(src, dst, s);
}

int vacv_resize(const vacv_image* src_d, const vacv_image* dst_d, int interpolation, int mode, void* stream) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    hipStream_t s = (hipStream_t)stream;
    if (src.w == dst.w && src.h == dst.h && (interpolation == VACV_INTER_LINEAR || interpolation == VACV_INTER_CUBIC) &&
        same_shape(src, dst)) {
        // resize.cpp:58-61 short-circuits equal sizes with a copy (the
        // reference copies w*h*c BYTES, a quarter of an fp32 image; this
        // copies the whole image)
        if (src.dtype == dst.dtype) {
            const int cc = src.layout == VACV_NHWC ? src.c : 1;
            return copy_rows(src, dst, 0, src.h, (int64_t)src.w * cc * src.es, s);
        }
        if (src.dtype == VACV_INT8 && dst.dtype == VACV_FP32 && interpolation == VACV_INTER_CUBIC)
            return dtype_convert(src, dst, s);
    }
    return resize_impl(src_d, dst_d, interpolation, mode, kOutSame, nullptr, s);
}

int vacv_resize_scaled(const vacv_image* src, const vacv_image* dst, int interpolation, int mode, double fx,
                       double fy, void* stream) {
    if (!(fx > 0) || !(fy > 0)) return VACV_ERR_INVALID_ARG;
    if (interpolation != VACV_INTER_NEAREST && interpolation != VACV_INTER_AREA && interpolation != VACV_INTER_LANCZOS4)
        return VACV_ERR_UNSUPPORTED;
    return resize_impl(src, dst, interpolation, mode, kOutSame, nullptr, (hipStream_t)stream, fx, fy);
}

int vacv_rotation_matrix(float scale, float rot_deg, const double aux[4], float m[6]) {
    if (!m) return VACV_ERR_INVALID_ARG;
    const double a[4] = {aux ? aux[0] : 0.0, aux ? aux[1] : 0.0, aux ? aux[2] : 0.0, aux ? aux[3] : 0.0};
    // warp_affine.cpp:76-94 with point (0,0): angle in float radians,
    // alpha/beta = scale * cosf/sinf (float products widened to double)
    const float angle = (float)((double)rot_deg * (M_PI / 180));
    const double alpha = (double)(scale * cosf(angle));
    const double beta = (double)(scale * sinf(angle));
    m[0] = (float)alpha;
    m[1] = (float)beta;
    m[3] = (float)-beta;
    m[4] = (float)alpha;
    // warp_affine.cpp:105-106 (aux translation fix, double arithmetic)
    m[2] = (float)(a[2] - (double)m[0] * a[0] - (double)m[1] * a[1]);
    m[5] = (float)(a[3] - (double)m[3] * a[0] - (double)m[4] * a[1]);
    return VACV_OK;
}

int vacv_invert_affine(const float m[6], float inv[6]) {
    if (!m || !inv) return VACV_ERR_INVALID_ARG;
    // warp_affine.cpp:121-133: float products, double D, stored as float
    float a[6];
    std::memcpy(a, m, sizeof(a));
    double D = (double)(a[0] * a[4] - a[1] * a[3]);
    D = D != 0 ? 1. / D : 0;
    const double A11 = (double)a[4] * D;
    const double A22 = (double)a[0] * D;
    a[0] = (float)A11;
    a[1] = (float)((double)a[1] * -D);
    a[3] = (float)((double)a[3] * -D);
    a[4] = (float)A22;
    const float b1 = -a[0] * a[2] - a[1] * a[5];
    const float b2 = -a[3] * a[2] - a[4] * a[5];
    a[2] = b1;
    a[5] = b2;
    std::memcpy(inv, a, sizeof(a));
    return VACV_OK;
}

int vacv_warp_affine(const vacv_image* src, const vacv_image* dst, const float m[6], int flags, int border_mode,
                     const double border_value[4], void* stream) {
    return warp_impl(src, dst, m, flags, border_mode, border_value, kOutSame, nullptr, (hipStream_t)stream);
}

int vacv_cvt_color(const vacv_image* src, const vacv_image* dst, int code, void* stream) {
    switch (code) {
        case VACV_COLOR_GRAY2BGR:
        case VACV_COLOR_YUV2RGBA_NV12:
        case VACV_COLOR_YUV2BGRA_NV12:
        case VACV_COLOR_YUV2RGBA_NV21:
        case VACV_COLOR_YUV2BGRA_NV21:
        case VACV_COLOR_YUV2BGR_YV12:
            return color_cv_impl(src, dst, code, (hipStream_t)stream);
        default:
            return color_impl(src, dst, code, kOutSame, nullptr, (hipStream_t)stream);
    }
}

int vacv_normalize(const vacv_image* src_d, const vacv_image* dst_d, const float* mean, const float* stddev,
                   void* stream) {
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (!same_shape(src, dst) || dst.dtype != VACV_FP32) return VACV_ERR_INVALID_ARG;
    if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    NormSpec ns;
    if ((st = norm_spec(src, mean, stddev, ns))) return st;
    if (ns.mode == 0) {
        float *dm = nullptr, *ds = nullptr;
        if ((st = per_image_stats(src, s, &dm, &ds))) return st;
        ns.mode = 2;
        ns.dev_mean = dm;
        ns.dev_std = ds;
    }
    return normalize_with(src, dst, ns, s);
}

int vacv_channel_sums(const vacv_image* src_d, double* sums, int per_image, void* stream) {
    Img src;
    int st = load(src_d, src);
    if (st) return st;
    if (!sums) return VACV_ERR_INVALID_ARG;
    if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
    if (src.layout == VACV_NHWC && src.c > 4) return VACV_ERR_UNSUPPORTED;
    if (!dense(src)) return VACV_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const int blocks = sums_blocks(src);
    const int planes = src.layout == VACV_NHWC ? 1 : src.c;
    const int cc = src.layout == VACV_NHWC ? src.c : 1;
    void* ws = nullptr;
    if ((st = workspace(s, (size_t)src.n * planes * blocks * 2 * cc * sizeof(double), &ws))) return st;
    return channel_sums_into(src, sums, per_image ? 1 : 0, static_cast<double*>(ws), blocks, s);
}

namespace {
// vacv_resize_channel_sums with optional statistics: u8 -> fp32 cubic into a
// dense NHWC output (cfg5) takes the cubic kernel's sums epilogue (the column
// kernel: per-image fixed-point integer accumulators, then one tiny launch
// for the sums and mean / stddev; the gather kernel: per-workgroup partials
// and a fixed-order reduction launch) -- the output is not read back (a
// separate vacv_channel_sums pass re-read 77 MB per cfg5 batch).  Everything
// else: resize, then vacv_channel_sums (and vacv_stats_from_sums).
int resize_sums(const vacv_image* src_d, const vacv_image* dst_d, int interpolation, int mode, double* sums,
                int per_image, float* mean, float* stddev, void* stream) {
    if (!sums) return VACV_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)stream;
    Img src, dst;
    int st = load(src_d, src);
    if (st) return st;
    if ((st = load(dst_d, dst))) return st;
    if (interpolation == VACV_INTER_CUBIC && src.dtype == VACV_INT8 && dst.dtype == VACV_FP32 &&
        dst.layout == VACV_NHWC && dst.c <= 3 && dense(dst) && src.n == dst.n) {
        const int64_t groups = cubic_sums_groups_bound(dst.w, dst.h);  // the workspace's bound
        void* ws = nullptr;
        void* acc = nullptr;
        if ((st = workspace(s, (size_t)(dst.n * groups * 2 * dst.c) * sizeof(double), &ws))) return st;
        // fixed-point accumulators: zeroed when allocated, and every call leaves them zero
        if ((st = workspace(s, (size_t)dst.n * 2 * dst.c * sizeof(int64_t), &acc, 4, true))) return st;
        FusedSums fs{static_cast<double*>(ws), sums, per_image ? 1 : 0, mean, stddev, 0, false,
                     static_cast<int64_t*>(acc)};
        if ((st = resize_impl(src_d, dst_d, interpolation, mode, kOutSame, nullptr, s, 0.0, 0.0, &fs))) return st;
        if (fs.used) return fs.groups <= groups ? VACV_OK : VACV_ERR_HIP;  // (a layout mismatch cannot happen)
    } else if ((st = resize_impl(src_d, dst_d, interpolation, mode, kOutSame, nullptr, s))) {
        return st;
    }
    if ((st = vacv_channel_sums(dst_d, sums, per_image, stream))) return st;
    if (!mean) return VACV_OK;
    const double count = (double)dst.w * dst.h * (per_image ? 1 : dst.n);
    return hip_status(launch_stats(sums, per_image ? dst.n : 1, dst.c, count, mean, stddev, s));
}
}  // namespace

int vacv_resize_channel_sums(const vacv_image* src_d, const vacv_image* dst_d, int interpolation, int mode,
                             double* sums, int per_image, void* stream) {
    return resize_sums(src_d, dst_d, interpolation, mode, sums, per_image, nullptr, nullptr, stream);
}

int vacv_resize_mean_stddev(const vacv_image* src_d, const vacv_image* dst_d, int interpolation, int mode,
                            double* sums, float* mean, float* stddev, int per_image, void* stream) {
    if (!mean || !stddev) return VACV_ERR_INVALID_ARG;
    return resize_sums(src_d, dst_d, interpolation, mode, sums, per_image, mean, stddev, stream);
}

int vacv_stats_from_sums(const double* sums, int groups, int c, double count, float* mean, float* stddev,
                         void* stream) {
    if (!sums || !mean || !stddev || groups < 1 || c < 1 || !(count > 0)) return VACV_ERR_INVALID_ARG;
    return hip_status(launch_stats(sums, groups, c, count, mean, stddev, (hipStream_t)stream));
}

int vacv_mean_stddev(const vacv_image* src_d, float* mean, float* stddev, void* stream) {
    Img src;
    int st = load(src_d, src);
    if (st) return st;
    if (!mean || !stddev) return VACV_ERR_INVALID_ARG;
    if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    float *dm = nullptr, *ds = nullptr;
    if ((st = per_image_stats(src, s, &dm, &ds))) return st;
    const size_t b = (size_t)src.n * src.c * sizeof(float);
    if (hipMemcpyAsync(mean, dm, b, hipMemcpyDeviceToDevice, s) != hipSuccess) return VACV_ERR_HIP;
    if (hipMemcpyAsync(stddev, ds, b, hipMemcpyDeviceToDevice, s) != hipSuccess) return VACV_ERR_HIP;
    return VACV_OK;
}

int vacv_resize_normalize(const vacv_image* src, const vacv_image* dst, int interpolation, int mode,
                          const float* mean, const float* stddev, void* stream) {
    ResizeCtx c{src, dst, interpolation, mode};
    return fused_normalize(dst, mean, stddev, (hipStream_t)stream, resize_pass, &c);
}

int vacv_warp_affine_normalize(const vacv_image* src, const vacv_image* dst, const float m[6], int flags,
                               int border_mode, const double border_value[4], const float* mean, const float* stddev,
                               void* stream) {
    WarpCtx c{src, dst, m, flags, border_mode, border_value};
    return fused_normalize(dst, mean, stddev, (hipStream_t)stream, warp_pass, &c);
}

int vacv_cvt_color_normalize(const vacv_image* src, const vacv_image* dst, int code, const float* mean,
                             const float* stddev, void* stream) {
    ColorCtx c{src, dst, code};
    return fused_normalize(dst, mean, stddev, (hipStream_t)stream, color_pass, &c);
}

int vacv_cvt_color_resize(const vacv_image* src, const vacv_image* dst, int code, int interpolation, int mode,
                          void* stream) {
    if (!dst) return VACV_ERR_INVALID_ARG;
    const int out = dst->dtype == VACV_FP32 ? kOutF32 : kOutSame;
    return yuv_resize_impl(src, dst, code, interpolation, mode, out, nullptr, (hipStream_t)stream);
}

int vacv_cvt_color_resize_normalize(const vacv_image* src, const vacv_image* dst, int code, int interpolation,
                                    int mode, const float* mean, const float* stddev, void* stream) {
    YuvResizeCtx c{src, dst, code, interpolation, mode};
    return fused_normalize(dst, mean, stddev, (hipStream_t)stream, yuv_resize_pass, &c);
}

int vacv_match_template(const vacv_image* img_d, const vacv_image* tpl_d, const vacv_image* res_d, int method,
                        void* stream) {
    Img img, tpl, res;
    int st = load(img_d, img);
    if (st) return st;
    if ((st = load(tpl_d, tpl))) return st;
    if ((st = load(res_d, res))) return st;
    if (method < VACV_TM_SQDIFF || method > VACV_TM_CCOEFF_NORMED) return VACV_ERR_UNSUPPORTED;
    if (img.dtype != VACV_INT8 && img.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
    if (tpl.dtype != img.dtype || tpl.c != img.c || tpl.n != 1) return VACV_ERR_INVALID_ARG;
    if (img.layout != VACV_NHWC || tpl.layout != VACV_NHWC || img.c > 4) return VACV_ERR_UNSUPPORTED;
    // cv::matchTemplate swaps a template larger than the image (n = 1 only)
    if (tpl.w >= img.w && tpl.h >= img.h && (tpl.w > img.w || tpl.h > img.h)) {
        if (img.n != 1) return VACV_ERR_INVALID_ARG;
        std::swap(img, tpl);
    }
    if (tpl.w > img.w || tpl.h > img.h) return VACV_ERR_INVALID_ARG;
    const int rw = img.w - tpl.w + 1, rh = img.h - tpl.h + 1;
    if (res.dtype != VACV_FP32 || res.c != 1 || res.w != rw || res.h != rh || res.n != img.n)
        return VACV_ERR_INVALID_ARG;
    if (match_lds_bytes(tpl.w, tpl.h, img.c, img.es) > 64 * 1024 || rh > 65535 * 4 || img.n > 65535)
        return VACV_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    MatchLaunch M{};
    M.img = img.data;
    M.img_pitch = img.batch;
    M.img_row = img.row;
    M.iw = img.w;
    M.ih = img.h;
    M.cn = img.c;
    M.esize = img.es;
    M.n = img.n;
    M.tpl = tpl.data;
    M.tpl_row = tpl.row;
    M.tw = tpl.w;
    M.th = tpl.h;
    M.res = res.data;
    M.res_pitch = res.batch;
    M.res_row = res.row;
    M.rw = rw;
    M.rh = rh;
    M.method = method;
    M.inv_area = 1. / ((double)tpl.h * tpl.w);
    if (img.dtype == VACV_INT8) {  // the matrix-core correlation's B fragments
        const size_t bytes = match_bfrag_bytes(tpl.w, tpl.h, img.c);
        if (bytes) {
            void* ws = nullptr;
            if ((st = workspace(s, bytes, &ws, 3))) return st;
            M.bfrag = ws;
        }
    }
    if (method != VACV_TM_CCORR) {
        const size_t box = align_up((size_t)img.n * 2 * (img.h + 1) * (img.w + 1) * img.c * sizeof(double), 256);
        void* ws = nullptr;
        if ((st = workspace(s, box + 256, &ws))) return st;
        M.box = static_cast<double*>(ws);
        M.tstats = reinterpret_cast<double*>(static_cast<char*>(ws) + box);
    }
    return hip_status(launch_match_template(M, s));
}

int vacv_min_max_idx(const vacv_image* src_d, const vacv_image* mask_d, double* vals, int* idx, void* stream) {
    Img src, mask;
    int st = load(src_d, src);
    if (st) return st;
    if (!vals || !idx) return VACV_ERR_INVALID_ARG;
    if (src.n != 1 || src.c != 1) return VACV_ERR_INVALID_ARG;  // cv::minMaxIdx: one channel
    if (src.dtype != VACV_INT8 && src.dtype != VACV_FP32) return VACV_ERR_UNSUPPORTED;
    MinMaxLaunch L{};
    L.src = src.data;
    L.row = src.row;
    L.w = src.w;
    L.h = src.h;
    L.esize = src.es;
    if (mask_d) {
        if ((st = load(mask_d, mask))) return st;
        if (mask.dtype != VACV_INT8 || mask.c != 1 || mask.w != src.w || mask.h != src.h) return VACV_ERR_INVALID_ARG;
        L.mask = mask.data;
        L.mask_row = mask.row;
    }
    L.out_val = vals;
    L.out_idx = idx;
    hipStream_t s = (hipStream_t)stream;
    void* ws = nullptr;
    // its own workspace key: a match_template result on the same stream may
    // still be using the stream's main workspace
    if ((st = workspace(s, min_max_workspace_bytes(), &ws, 1))) return st;
    return hip_status(launch_min_max(L, ws, s));
}

int vacv_stream_synchronize(void* stream) {
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? VACV_OK : VACV_ERR_HIP;
}

int vacv_release_workspace(void) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    int st = VACV_OK;
    for (auto& kv : g_ws) {
        if (kv.second.buf) {
            if (hipStreamSynchronize((hipStream_t)std::get<1>(kv.first)) != hipSuccess) st = VACV_ERR_HIP;
            if (hipFree(kv.second.buf) != hipSuccess) st = VACV_ERR_HIP;
        }
    }
    g_ws.clear();
    const int pst = release_plans();
    const int ast = release_area_tables();
    const int lst = release_lanczos_tables();
    return st ? st : (pst ? pst : (ast ? ast : lst));
}

}  // extern "C"
