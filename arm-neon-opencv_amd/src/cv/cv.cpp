// va_cv:: over the C ABI (include/vacv_hip.h).  Each function reproduces the
// reference operator's output-tensor contract (shape, dtype, layout via
// dst.create) and hands the pixel work to the HIP kernels; detail::Staging
// moves host operands across PCIe and leaves device operands in HBM.
#include "cv.h"

#include <cmath>
#include <cstring>
#include <vector>

#include "../common/hip_context.h"

namespace va_cv {

using namespace vision;
using detail::fail;
using detail::Staging;

namespace {

// Small host-side parameter vectors (mean / stddev / M) read from a Tensor of
// FP32 values, wherever it lives.
std::vector<float> host_floats(const char* fn, const Tensor& t, size_t want) {
    if (t.dtype != FP32) fail(fn, "parameter tensors must be FP32");
    if (t.size() != want) fail(fn, "parameter tensor has the wrong number of values");
    const Tensor h = t.to_host();
    std::vector<float> v(want);
    std::memcpy(v.data(), h.data, want * sizeof(float));
    return v;
}

// mean / stddev: (nullptr, nullptr) = per-image statistics.  `either_empty`
// picks the rule of resize_normalize_opencv (resize_normalize.cpp:58: either
// empty -> computed); otherwise both must be empty (normalize.cpp:98).
struct Stats {
    std::vector<float> mean, stdv;
    const float* m() const { return mean.empty() ? nullptr : mean.data(); }
    const float* s() const { return stdv.empty() ? nullptr : stdv.data(); }
};

Stats read_stats(const char* fn, const Tensor& mean, const Tensor& stddev, int c, bool either_empty) {
    Stats st;
    const bool me = mean.empty(), se = stddev.empty();
    if (me && se) return st;
    if (me || se) {
        if (either_empty) return st;
        fail(fn, "mean and stddev must both be given or both be empty");
    }
    // resize_normalize.cpp:82-84 / normalize.cpp: one value per channel
    if ((int)mean.size() != c || (int)stddev.size() != c)
        fail(fn, "The input mean or stddev channels is not matched with tensor dims");
    st.mean = host_floats(fn, mean, c);
    st.stdv = host_floats(fn, stddev, c);
    return st;
}

DType resize_out_dtype(const char* fn, const Tensor& src, int interpolation) {
    if (interpolation == INTER_LINEAR) {
        if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "INTER_LINEAR takes INT8 or FP32");
        return src.dtype;
    }
    if (interpolation == INTER_CUBIC) {
        if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "INTER_CUBIC takes INT8 or FP32");
        return FP32;  // INT8 cubic = fused widen to FP32 (reference: infinite recursion)
    }
    if (interpolation == INTER_NEAREST) {
        // resize.cpp:46-49 hands it to cv::resize; OpenCV 2.4's resizeNN here
        if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "INTER_NEAREST takes INT8 or FP32");
        return src.dtype;
    }
    if (interpolation == INTER_AREA) {
        // resize.cpp:46-49 hands it to cv::resize; OpenCV 2.4's area resize
        // at every scale (resizeAreaFast_, resizeArea_, area-mode bilinear)
        if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "INTER_AREA takes INT8 or FP32");
        return src.dtype;
    }
    if (interpolation == INTER_LANCZOS4) {
        // resize.cpp:46-49 hands it to cv::resize; OpenCV 2.4's 8x8 Lanczos here
        if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "INTER_LANCZOS4 takes INT8 or FP32");
        return src.dtype;
    }
    // every other mode goes to OpenCV in the reference, which this build
    // does not ship (the reference without OpenCV recurses forever)
    fail(fn, "only INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA and INTER_LANCZOS4 are supported");
}

std::vector<float> affine_of(const char* fn, const Tensor& M) { return host_floats(fn, M, 6); }

void check_warp_modes(const char* fn, const Tensor& src, int flags, int borderMode) {
    // warp_affine.cpp:114-118
    if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "warp_affine takes INT8 or FP32");
    // INTER_LINEAR / INTER_NEAREST, optionally | WARP_INVERSE_MAP (the
    // reference hands all but INTER_LINEAR to cv::warpAffine; OpenCV 2.4's
    // semantics here, vacv_hip.h)
    const int interp = flags & INTER_MAX;
    if ((flags & ~(INTER_MAX | WARP_INVERSE_MAP)) || (interp != INTER_LINEAR && interp != INTER_NEAREST))
        fail(fn, "only INTER_LINEAR and INTER_NEAREST (optionally | WARP_INVERSE_MAP) are supported");
    // BORDER_CONSTANT is the reference's naive path; REPLICATE, REFLECT, WRAP,
    // REFLECT_101 and TRANSPARENT extend it (the reference hands them to
    // OpenCV: warp_affine.cpp:114-118); BORDER_ISOLATED has no meaning here
    if (borderMode < BORDER_CONSTANT || borderMode > BORDER_TRANSPARENT)
        fail(fn, "unsupported border mode");
}

std::vector<float> rotation(float scale, float rot, const VScalar& aux) {
    const double a[4] = {aux.v0, aux.v1, aux.v2, aux.v3};
    std::vector<float> m(6);
    detail::check("va_cv::warp_affine", vacv_rotation_matrix(scale, rot, a, m.data()));
    return m;
}

void warp_into(const char* fn, const Tensor& src, Tensor& dst, const float* m, VSize dsize, int flags,
               int borderMode, const VScalar& bv, bool normalize, const Stats* stats) {
    check_warp_modes(fn, src, flags, borderMode);
    if (dsize.w < 1 || dsize.h < 1) fail(fn, "dsize must be positive");
    const double border[4] = {bv.v0, bv.v1, bv.v2, bv.v3};
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    // BORDER_TRANSPARENT keeps dst's bytes where the sampler has no taps
    const vacv_image d = st.out(dst, dsize.w, dsize.h, src.c, normalize ? FP32 : src.dtype, src.layout, 1,
                                borderMode == BORDER_TRANSPARENT);
    if (normalize) {
        st.run(vacv_warp_affine_normalize(&s, &d, m, flags, borderMode, border, stats->m(), stats->s(),
                                          st.stream()));
    } else {
        st.run(vacv_warp_affine(&s, &d, m, flags, borderMode, border, st.stream()));
    }
    st.finish();
}

int yuv_rows(const char* fn, const Tensor& src) {
    if (src.dtype != INT8 || src.c != 1) fail(fn, "YUV420sp input must be a (w, h*3/2, 1) INT8 tensor");
    return src.h / 3 * 2;  // cvt_color.cpp:152
}

void check_yuv_code(const char* fn, int code) {
    if (code != COLOR_YUV2BGR_NV21 && code != COLOR_YUV2RGB_NV21 && code != COLOR_YUV2BGR_NV12 &&
        code != COLOR_YUV2RGB_NV12)
        fail(fn, "unsupported colour conversion code");
}

}  // namespace

void resize(const Tensor& src, Tensor& dst, VSize dsize, double fx, double fy, int interpolation) {
    static const char* fn = "va_cv::resize";
    const DType out = resize_out_dtype(fn, src, interpolation);
    // INTER_NEAREST / INTER_AREA go to cv::resize in the reference, which also
    // takes dsize = 0 with fx, fy: dsize = saturate_cast<int>(w * fx) (round
    // half to even) and inv_scale = fx, fy.  The naive LINEAR / CUBIC paths
    // use dsize alone (resize.cpp:77-135).
    const bool scaled = dsize.w == 0 && dsize.h == 0 && fx > 0 && fy > 0 &&
                        (interpolation == INTER_NEAREST || interpolation == INTER_AREA || interpolation == INTER_LANCZOS4);
    if (scaled) {
        dsize.w = static_cast<int>(std::nearbyint(src.w * fx));
        dsize.h = static_cast<int>(std::nearbyint(src.h * fy));
    }
    if (dsize.w < 1 || dsize.h < 1) fail(fn, "dsize must be positive");
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image d = st.out(dst, dsize.w, dsize.h, src.c, out, src.layout, 1);
    if (scaled) st.run(vacv_resize_scaled(&s, &d, interpolation, VACV_LINEAR_REFERENCE, fx, fy, st.stream()));
    else st.run(vacv_resize(&s, &d, interpolation, VACV_LINEAR_REFERENCE, st.stream()));
    st.finish();
}

void cvt_color(const Tensor& src, Tensor& dst, int code) {
    static const char* fn = "va_cv::cvt_color";
    // the codes the reference hands to cv::cvtColor (cvt_color.cpp:139-141),
    // with OpenCV 2.4's arithmetic: GRAY2BGR, YUV420 -> RGBA/BGRA, YV12
    if (code == COLOR_GRAY2BGR) {
        if ((src.dtype != INT8 && src.dtype != FP32) || src.c != 1 || src.layout != NHWC)
            fail(fn, "COLOR_GRAY2BGR takes a (w, h, 1) INT8 or FP32 NHWC tensor");
        Staging st(fn, src);
        const vacv_image s = st.in(src, 0);
        const vacv_image d = st.out(dst, src.w, src.h, 3, src.dtype, NHWC, 1);
        st.run(vacv_cvt_color(&s, &d, code, st.stream()));
        st.finish();
        return;
    }
    const bool cv4 = code == COLOR_YUV2RGBA_NV12 || code == COLOR_YUV2BGRA_NV12 || code == COLOR_YUV2RGBA_NV21 ||
                     code == COLOR_YUV2BGRA_NV21;
    if (!cv4 && code != COLOR_YUV2BGR_YV12) check_yuv_code(fn, code);
    const int h = yuv_rows(fn, src);
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image d = st.out(dst, src.w, h, cv4 ? 4 : 3, INT8, NHWC, 1);
    st.run(vacv_cvt_color(&s, &d, code, st.stream()));
    st.finish();
}

void cvt_color_normalize(const Tensor& src, Tensor& dst, int code, const Tensor& mean, const Tensor& stddev) {
    static const char* fn = "va_cv::cvt_color_normalize";
    check_yuv_code(fn, code);
    const int h = yuv_rows(fn, src);
    const Stats stats = read_stats(fn, mean, stddev, 3, false);
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image d = st.out(dst, src.w, h, 3, FP32, NHWC, 1);
    st.run(vacv_cvt_color_normalize(&s, &d, code, stats.m(), stats.s(), st.stream()));
    st.finish();
}

void normalize(const Tensor& src, Tensor& dst, const Tensor& mean, const Tensor& stddev) {
    static const char* fn = "va_cv::normalize";
    if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "normalize takes INT8 or FP32");
    const Stats stats = read_stats(fn, mean, stddev, src.c, false);
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image d = st.out(dst, src.w, src.h, src.c, FP32, src.layout, 1);
    st.run(vacv_normalize(&s, &d, stats.m(), stats.s(), st.stream()));
    st.finish();
}

void mean_stddev(const Tensor& src, Tensor& mean, Tensor& stddev) {
    static const char* fn = "va_cv::mean_stddev";
    if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "mean_stddev takes INT8 or FP32");
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image m = st.out(mean, src.c, 1, 1, FP32, NCHW, 1);
    const vacv_image d = st.out(stddev, src.c, 1, 1, FP32, NCHW, 2);
    st.run(vacv_mean_stddev(&s, static_cast<float*>(m.data), static_cast<float*>(d.data), st.stream()));
    st.finish();
}

void warp_affine(const Tensor& src, Tensor& dst, const Tensor& M, VSize dsize, int flags, int borderMode,
                 const VScalar& borderValue) {
    static const char* fn = "va_cv::warp_affine";
    const std::vector<float> m = affine_of(fn, M);
    warp_into(fn, src, dst, m.data(), dsize, flags, borderMode, borderValue, false, nullptr);
}

void warp_affine(const Tensor& src, Tensor& dst, float scale, float rot, VSize dsize, const VScalar& aux_param,
                 int flags, int borderMode, const VScalar& borderValue) {
    static const char* fn = "va_cv::warp_affine";
    const std::vector<float> m = rotation(scale, rot, aux_param);
    warp_into(fn, src, dst, m.data(), dsize, flags, borderMode, borderValue, false, nullptr);
}

void resize_normalize(const Tensor& src, Tensor& dst, VSize dsize, double /*fx*/, double /*fy*/, int interpolation,
                      const Tensor& mean, const Tensor& stddev) {
    static const char* fn = "va_cv::resize_normalize";
    (void)resize_out_dtype(fn, src, interpolation);
    if (dsize.w < 1 || dsize.h < 1) fail(fn, "dsize must be positive");
    const Stats stats = read_stats(fn, mean, stddev, src.c, true);
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image d = st.out(dst, dsize.w, dsize.h, src.c, FP32, src.layout, 1);
    st.run(vacv_resize_normalize(&s, &d, interpolation, VACV_LINEAR_REFERENCE, stats.m(), stats.s(), st.stream()));
    st.finish();
}

void warp_affine_normalize(const Tensor& src, Tensor& dst, const Tensor& M, VSize dsize, int flags, int borderMode,
                           const VScalar& borderValue, const Tensor& mean, const Tensor& stddev) {
    static const char* fn = "va_cv::warp_affine_normalize";
    const std::vector<float> m = affine_of(fn, M);
    const Stats stats = read_stats(fn, mean, stddev, src.c, false);
    warp_into(fn, src, dst, m.data(), dsize, flags, borderMode, borderValue, true, &stats);
}

void warp_affine_normalize(const Tensor& src, Tensor& dst, float scale, float rot, VSize dsize,
                           const VScalar& aux_param, int flags, int borderMode, const VScalar& borderValue,
                           const Tensor& mean, const Tensor& stddev) {
    static const char* fn = "va_cv::warp_affine_normalize";
    const std::vector<float> m = rotation(scale, rot, aux_param);
    const Stats stats = read_stats(fn, mean, stddev, src.c, false);
    warp_into(fn, src, dst, m.data(), dsize, flags, borderMode, borderValue, true, &stats);
}

void crop(const Tensor& src, Tensor& dst, const VRect& rect) {
    static const char* fn = "va_cv::crop";
    // crop.cpp:128-131
    const int left = static_cast<int>(rect.left);
    const int top = static_cast<int>(rect.top);
    const int cw = static_cast<int>(rect.width());
    const int ch = static_cast<int>(rect.height());
    if (cw < 1 || ch < 1 || left < 0 || top < 0 || left + cw > src.w || top + ch > src.h)
        fail(fn, "rect must lie inside the image");  // the reference reads out of bounds
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    const vacv_image d = st.out(dst, cw, ch, src.c, src.dtype, src.layout, 1);
    st.run(vacv_crop(&s, &d, left, top, st.stream()));
    st.finish();
}

// ---- batched frames (FramePipeline: overlapped PCIe staging) ---------------

namespace {

using detail::FramePipeline;

void check_batch(const char* fn, const std::vector<Tensor>& src, std::vector<Tensor>& dst) {
    if (src.empty()) fail(fn, "empty frame list");
    for (const Tensor& t : src)
        if (t.device() != src[0].device()) fail(fn, "frames live on different devices");
    dst.resize(src.size());
}

}  // namespace

void resize(const std::vector<Tensor>& src, std::vector<Tensor>& dst, VSize dsize, double fx, double fy,
            int interpolation) {
    static const char* fn = "va_cv::resize";
    check_batch(fn, src, dst);
    const DType out = resize_out_dtype(fn, src[0], interpolation);
    // dsize = 0 with fx, fy: cv::resize's form, per frame (see the single-frame overload)
    const bool scaled = dsize.w == 0 && dsize.h == 0 && fx > 0 && fy > 0 &&
                        (interpolation == INTER_NEAREST || interpolation == INTER_AREA || interpolation == INTER_LANCZOS4);
    std::vector<VSize> sizes(src.size(), dsize);
    if (scaled)
        for (size_t i = 0; i < src.size(); ++i)
            sizes[i] = VSize(static_cast<int>(std::nearbyint(src[i].w * fx)), static_cast<int>(std::nearbyint(src[i].h * fy)));
    for (const VSize& z : sizes)
        if (z.w < 1 || z.h < 1) fail(fn, "dsize must be positive");
    FramePipeline p(fn, detail::compute_device(src[0]));
    for (size_t i = 0; i < src.size(); ++i)
        p.frame(src[i], dst[i], sizes[i].w, sizes[i].h, src[i].c, out, src[i].layout,
                [&](const vacv_image& s, const vacv_image& d, hipStream_t st) {
                    if (scaled) return vacv_resize_scaled(&s, &d, interpolation, VACV_LINEAR_REFERENCE, fx, fy, st);
                    return vacv_resize(&s, &d, interpolation, VACV_LINEAR_REFERENCE, st);
                });
    p.finish();
}

void resize_normalize(const std::vector<Tensor>& src, std::vector<Tensor>& dst, VSize dsize, double /*fx*/,
                      double /*fy*/, int interpolation, const Tensor& mean, const Tensor& stddev) {
    static const char* fn = "va_cv::resize_normalize";
    check_batch(fn, src, dst);
    (void)resize_out_dtype(fn, src[0], interpolation);
    if (dsize.w < 1 || dsize.h < 1) fail(fn, "dsize must be positive");
    const Stats stats = read_stats(fn, mean, stddev, src[0].c, true);
    FramePipeline p(fn, detail::compute_device(src[0]));
    for (size_t i = 0; i < src.size(); ++i)
        p.frame(src[i], dst[i], dsize.w, dsize.h, src[i].c, FP32, src[i].layout,
                [&](const vacv_image& s, const vacv_image& d, hipStream_t st) {
                    return vacv_resize_normalize(&s, &d, interpolation, VACV_LINEAR_REFERENCE, stats.m(), stats.s(),
                                                 st);
                });
    p.finish();
}

void warp_affine(const std::vector<Tensor>& src, std::vector<Tensor>& dst, const Tensor& M, VSize dsize, int flags,
                 int borderMode, const VScalar& bv) {
    static const char* fn = "va_cv::warp_affine";
    check_batch(fn, src, dst);
    check_warp_modes(fn, src[0], flags, borderMode);
    if (borderMode == BORDER_TRANSPARENT) fail(fn, "BORDER_TRANSPARENT needs the per-frame call");
    if (dsize.w < 1 || dsize.h < 1) fail(fn, "dsize must be positive");
    const std::vector<float> m = affine_of(fn, M);
    const double border[4] = {bv.v0, bv.v1, bv.v2, bv.v3};
    FramePipeline p(fn, detail::compute_device(src[0]));
    for (size_t i = 0; i < src.size(); ++i)
        p.frame(src[i], dst[i], dsize.w, dsize.h, src[i].c, src[i].dtype, src[i].layout,
                [&](const vacv_image& s, const vacv_image& d, hipStream_t st) {
                    return vacv_warp_affine(&s, &d, m.data(), flags, borderMode, border, st);
                });
    p.finish();
}

void cvt_color(const std::vector<Tensor>& src, std::vector<Tensor>& dst, int code) {
    static const char* fn = "va_cv::cvt_color";
    check_batch(fn, src, dst);
    check_yuv_code(fn, code);
    FramePipeline p(fn, detail::compute_device(src[0]));
    for (size_t i = 0; i < src.size(); ++i) {
        const int h = yuv_rows(fn, src[i]);
        p.frame(src[i], dst[i], src[i].w, h, 3, INT8, NHWC,
                [&](const vacv_image& s, const vacv_image& d, hipStream_t st) {
                    return vacv_cvt_color(&s, &d, code, st);
                });
    }
    p.finish();
}

void cvt_color_normalize(const std::vector<Tensor>& src, std::vector<Tensor>& dst, int code, const Tensor& mean,
                         const Tensor& stddev) {
    static const char* fn = "va_cv::cvt_color_normalize";
    check_batch(fn, src, dst);
    check_yuv_code(fn, code);
    const Stats stats = read_stats(fn, mean, stddev, 3, false);
    FramePipeline p(fn, detail::compute_device(src[0]));
    for (size_t i = 0; i < src.size(); ++i) {
        const int h = yuv_rows(fn, src[i]);
        p.frame(src[i], dst[i], src[i].w, h, 3, FP32, NHWC,
                [&](const vacv_image& s, const vacv_image& d, hipStream_t st) {
                    return vacv_cvt_color_normalize(&s, &d, code, stats.m(), stats.s(), st);
                });
    }
    p.finish();
}

void match_template(const Tensor& src, const Tensor& target, Tensor& result, int method) {
    static const char* fn = "va_cv::match_template";
    // match_template.cpp:13-41 -> cv::matchTemplate (OpenCV 2.4 semantics,
    // exact correlation; the C ABI swaps a larger template as OpenCV does)
    if (src.dtype != INT8 && src.dtype != FP32) fail(fn, "match_template takes INT8 or FP32");
    if (target.dtype != src.dtype || target.c != src.c) fail(fn, "the template must match the image's dtype and channels");
    if (src.layout != NHWC || target.layout != NHWC) fail(fn, "match_template takes NHWC tensors");
    const bool swap = target.w >= src.w && target.h >= src.h && (target.w > src.w || target.h > src.h);
    const Tensor& a = swap ? target : src;
    const Tensor& b = swap ? src : target;
    if (b.w > a.w || b.h > a.h) fail(fn, "the template does not fit the image");
    Staging st(fn, src);
    const vacv_image s = st.in(a, 0);
    const vacv_image t = st.in(b, 1);
    const vacv_image d = st.out(result, a.w - b.w + 1, a.h - b.h + 1, 1, FP32, NHWC, 2);
    st.run(vacv_match_template(&s, &t, &d, method, st.stream()));
    st.finish();
}

void minMaxIdx(const Tensor& src, double* minVal, double* maxVal, int* minIdx, int* maxIdx, const Tensor& mask) {
    static const char* fn = "va_cv::minMaxIdx";
    // match_template.cpp:43-46 -> cv::minMaxIdx of a single-channel array;
    // minIdx / maxIdx receive (row, col)
    if (src.c != 1) fail(fn, "minMaxIdx takes a single-channel tensor");
    Staging st(fn, src);
    const vacv_image s = st.in(src, 0);
    vacv_image m{};
    const bool has_mask = !mask.empty();
    if (has_mask) m = st.in(mask, 1);
    Tensor out;
    const vacv_image o = st.out(out, 48, 1, 1, INT8, NHWC, 2);  // 2 doubles + 4 ints, device scratch
    double* vals = static_cast<double*>(o.data);
    int* idx = reinterpret_cast<int*>(static_cast<char*>(o.data) + 16);
    st.run(vacv_min_max_idx(&s, has_mask ? &m : nullptr, vals, idx, st.stream()));
    double hv[2];
    int hi[4];
    detail::check_hip(fn, hipMemcpyAsync(hv, vals, sizeof(hv), hipMemcpyDeviceToHost, st.stream()));
    detail::check_hip(fn, hipMemcpyAsync(hi, idx, sizeof(hi), hipMemcpyDeviceToHost, st.stream()));
    st.finish();
    if (minVal) *minVal = hv[0];
    if (maxVal) *maxVal = hv[1];
    if (minIdx) { minIdx[0] = hi[0]; minIdx[1] = hi[1]; }
    if (maxIdx) { maxIdx[0] = hi[2]; maxIdx[1] = hi[3]; }
}

void imencode(const Tensor&, std::vector<unsigned char>&, const char*) {
    fail("va_cv::imencode", "not provided by the MI355X build (OpenCV-only in the reference)");
}

}  // namespace va_cv
