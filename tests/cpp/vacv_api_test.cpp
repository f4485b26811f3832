// C++ harness for the source-compatible va_cv:: / vision::Tensor layer
// (libvacv.so), shaped like the reference's src/test harness
// (src/test/src/test_main.cpp, impl/test_*.cpp, profile/cv_profile.cpp):
// each case runs one va_cv:: call the way the reference's test does, times it
// with TIME_PERF beside the comparator, and scores the output with
// ImageUtil::compare_image_data against the MAX_DIFF 5e-4 bar of
// cv_profile.cpp:10.  The reference compares against OpenCV 2.4, which cannot
// ship here; the comparator is the CPU oracle (oracle/liboracle.so, test
// infrastructure), and on top of the cosine bar every case also states the
// exact bar the build is held to (bit-exact, or a max |diff|).
//
// Images: `--res DIR` reads raw BGR frames DIR/<W>x<H>.bgr (and
// <W>x<H>_grey.gray) that tests/test_cpp_api.py decodes from the reference's
// test JPEGs; without it, deterministic synthetic frames are used.
//
//   vacv_api_test [--res DIR] [--filter SUBSTR] [--times N]
// Exit status 0 iff every case passes.  The last line is a JSON summary.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../arm-neon-opencv_amd/src/common/tensor_converter.h"
#include "../../arm-neon-opencv_amd/src/common/va_allocator.h"
#include "../../arm-neon-opencv_amd/src/cv/cv.h"
#include "../../arm-neon-opencv_amd/src/util/image_util.h"
#include "../../arm-neon-opencv_amd/src/util/perf_util.h"
#include "../../oracle/vacv_oracle.h"

using namespace vision;
using namespace va_cv;

namespace {

constexpr double kMaxDiff = 5e-4;  // cv_profile.cpp:10

std::string g_res;
int g_times = 3;

struct Result {
    double oracle_ms = 0, vacv_ms = 0;
    double cosine = 0;     // ImageUtil::compare_image_data
    double max_abs = 0;    // max |vacv - oracle|
    double tol = 0;        // allowed max |diff| (0 = bit-exact)
    std::string note;
};

using Case = std::function<Result()>;

// ---- inputs ----------------------------------------------------------------
std::vector<unsigned char> synthetic(int w, int h, int c, unsigned seed) {
    std::vector<unsigned char> v((size_t)w * h * c);
    unsigned long long z = 0x9E3779B97F4A7C15ull * (seed + 1);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            for (int k = 0; k < c; ++k) {
                z += 0x9E3779B97F4A7C15ull;
                unsigned long long r = z;
                r = (r ^ (r >> 30)) * 0xBF58476D1CE4E5B9ull;
                r = (r ^ (r >> 27)) * 0x94D049BB133111EBull;
                r ^= r >> 31;
                const int g = (x * (37 + 11 * k) / w + y * (53 + 7 * k) / h + 29 * k) % 256;
                const int val = g + (int)(r & 0x7F) - 64;
                v[((size_t)y * w + x) * c + k] = (unsigned char)(val < 0 ? 0 : (val > 255 ? 255 : val));
            }
    return v;
}

// the reference's test image <W>x<H><suffix> as BGR (c = 3, cv::imread's
// default) or one grey channel (c = 1, imread(..., 0)), else synthetic
Tensor load_image(int w, int h, int c = 3, const char* suffix = "") {
    Tensor t(w, h, c, INT8, NHWC);
    if (!g_res.empty()) {
        const std::string p = g_res + "/" + std::to_string(w) + "x" + std::to_string(h) + suffix +
                              (c == 1 ? ".gray" : ".bgr");
        std::ifstream f(p, std::ios::binary);
        if (f && f.read(static_cast<char*>(t.data), (std::streamsize)t.len())) return t;
    }
    const auto v = synthetic(w, h, c, (unsigned)(w * 7 + h + c));
    std::memcpy(t.data, v.data(), v.size());
    return t;
}

Tensor floats_of(const std::vector<float>& v) {
    Tensor t((int)v.size(), 1, 1, FP32, NCHW);
    std::memcpy(t.data, v.data(), v.size() * sizeof(float));
    return t;
}

// ---- scoring ---------------------------------------------------------------
template <typename T>
void score(Result& r, const T* want, const Tensor& got_any) {
    const Tensor got = got_any.to_host();
    const T* g = static_cast<const T*>(got.data);
    const int n = (int)got.size();
    r.cosine = ImageUtil::compare_image_data(want, g, n);
    double m = 0;
    for (int i = 0; i < n; ++i) {
        const double d = std::fabs((double)want[i] - (double)g[i]);
        if (!(d <= m)) m = d;  // NaN-propagating max
    }
    r.max_abs = m;
}

bool passed(const Result& r) {
    return std::fabs(r.cosine - 1.0) <= kMaxDiff && r.max_abs <= r.tol;
}

// oracle helpers over whole images ------------------------------------------
void oracle_resize_u8(const Tensor& s, std::vector<unsigned char>& out, int wo, int ho) {
    const int planes = s.layout == NCHW ? s.c : 1, cc = s.layout == NCHW ? 1 : s.c;
    out.assign((size_t)wo * ho * s.c, 0);
    for (int p = 0; p < planes; ++p)
        oracle_resize_linear_u8((const uint8_t*)s.data + (size_t)p * s.w * s.h, s.w, s.h, cc,
                                out.data() + (size_t)p * wo * ho, wo, ho, ORACLE_LINEAR_NAIVE);
}

void oracle_resize_f32(const Tensor& s, std::vector<float>& out, int wo, int ho, bool cubic) {
    const int planes = s.layout == NCHW ? s.c : 1, cc = s.layout == NCHW ? 1 : s.c;
    out.assign((size_t)wo * ho * s.c, 0);
    for (int p = 0; p < planes; ++p) {
        const float* src = (const float*)s.data + (size_t)p * s.w * s.h;
        float* dst = out.data() + (size_t)p * wo * ho;
        if (cubic) {
            oracle_resize_cubic_f32(src, s.w, s.h, cc, dst, wo, ho);
        } else {
            oracle_resize_linear_f32(src, s.w, s.h, cc, dst, wo, ho);
        }
    }
}

template <typename T>
void oracle_warp(const Tensor& s, std::vector<T>& out, int wo, int ho, const float m[6]) {
    float inv[6];
    oracle_invert_affine(m, inv);
    const int planes = s.layout == NCHW ? s.c : 1, cc = s.layout == NCHW ? 1 : s.c;
    out.assign((size_t)wo * ho * s.c, T(0));  // border value 0 where the reference leaves dst untouched
    for (int p = 0; p < planes; ++p) {
        if (sizeof(T) == 1) {
            oracle_warp_affine_u8((const uint8_t*)s.data + (size_t)p * s.w * s.h, s.w, s.h, cc,
                                  (uint8_t*)out.data() + (size_t)p * wo * ho, wo, ho, inv);
        } else {
            oracle_warp_affine_f32((const float*)s.data + (size_t)p * s.w * s.h, s.w, s.h, cc,
                                   (float*)out.data() + (size_t)p * wo * ho, wo, ho, inv);
        }
    }
}

// exact per-channel statistics, then the reference's normalize arithmetic
void oracle_normalize_auto(const float* src, int w, int h, int c, DLayout layout, std::vector<float>& out) {
    out.assign((size_t)w * h * c, 0.f);
    const int64_t px = (int64_t)w * h;
    if (layout == NHWC) {
        std::vector<double> sums(2 * c);
        std::vector<float> m(c), s(c);
        oracle_channel_sums_f64(src, px, c, sums.data());
        oracle_stats_from_sums(sums.data(), (double)px, c, m.data(), s.data());
        oracle_normalize_f32(src, out.data(), px, c, m.data(), s.data());
    } else {
        for (int k = 0; k < c; ++k) {
            double sums[2];
            float m, s;
            oracle_channel_sums_f64(src + k * px, px, 1, sums);
            oracle_stats_from_sums(sums, (double)px, 1, &m, &s);
            oracle_normalize_f32(src + k * px, out.data() + k * px, px, 1, &m, &s);
        }
    }
}

// ---- cases (mirroring src/test/src/impl/test_*.cpp) -------------------------
const float kM[6] = {0.849158f, 0.012257f, -474.827f, -0.01225f, 0.849158f, -379.18f};  // test_warp_affine.cpp:31-32
const float kRotScale = 1.073914f, kRotAngle = -3.314525f;                              // :199-205
VScalar rot_aux() {
    VScalar a;
    a.v0 = 738.518372f;
    a.v1 = 537.672852f;
    a.v2 = 204.766998f;
    a.v3 = 73.329681f;
    return a;
}

Result crop_case(VRect rect, DLayout layout, DType dtype) {  // test_crop.cpp:44-90
    Result r;
    Tensor src = load_image(2560, 1440).change_layout(layout).change_dtype(dtype);
    const Tensor host = src.to_host();
    const int cw = (int)rect.width(), ch = (int)rect.height();
    std::vector<unsigned char> want((size_t)cw * ch * 3 * dtype_size(dtype));
    {
        TIME_PERF(r.oracle_ms);
        oracle_crop(host.data, src.w, src.h, layout == NHWC ? 3 : 1, layout == NHWC ? 1 : 3, (int)dtype_size(dtype),
                    want.data(), (int)rect.left, (int)rect.top, cw, ch);
    }
    Tensor out;
    {
        TIME_PERF(r.vacv_ms);
        va_cv::crop(src, out, rect);
    }
    if (out.w != cw || out.h != ch || out.layout != layout || out.dtype != dtype) r.note = "bad output shape";
    if (dtype == FP32) {
        score(r, (const float*)want.data(), out);
    } else {
        score(r, want.data(), out);
    }
    return r;
}

Result resize_case(DLayout layout, DType dtype, int interp, int wo, int ho) {  // test_resize.cpp
    Result r;
    Tensor src = load_image(2560, 1440).change_layout(layout);
    if (dtype == FP32) src = src.change_dtype(FP32);
    Tensor out;
    if (dtype == INT8 && interp == INTER_LINEAR) {
        std::vector<unsigned char> want;
        {
            TIME_PERF(r.oracle_ms);
            oracle_resize_u8(src, want, wo, ho);
        }
        {
            TIME_PERF(r.vacv_ms);
            va_cv::resize(src, out, VSize(wo, ho), 0, 0, interp);
        }
        score(r, want.data(), out);
    } else {
        const Tensor srcf = dtype == FP32 ? src : src.change_dtype(FP32);
        std::vector<float> want;
        {
            TIME_PERF(r.oracle_ms);
            oracle_resize_f32(srcf, want, wo, ho, interp == INTER_CUBIC);
        }
        {
            TIME_PERF(r.vacv_ms);
            va_cv::resize(src, out, VSize(wo, ho), 0, 0, interp);
        }
        score(r, want.data(), out);
        if (interp == INTER_CUBIC) r.tol = 1e-3;  // cubic bar
    }
    if (out.w != wo || out.h != ho || out.layout != layout) r.note = "bad output shape";
    return r;
}

// grey_c: 0 = 1280x720.jpg; 3 / 1 = 1280x720_grey.jpg read as BGR / one channel
Result warp_case(DLayout layout, DType dtype, bool by_rotation, int grey_c) {  // test_warp_affine.cpp
    Result r;
    Tensor src = (grey_c ? load_image(1280, 720, grey_c, "_grey") : load_image(1280, 720)).change_layout(layout);
    if (dtype == FP32) src = src.change_dtype(FP32);
    float m[6];
    VSize dsize(240, 240);
    if (by_rotation) {
        const VScalar a = rot_aux();
        const double aux[4] = {a.v0, a.v1, a.v2, a.v3};
        oracle_rotation_matrix(kRotScale, kRotAngle, aux, m);
        dsize = VSize(140, 210);
    } else {
        std::memcpy(m, kM, sizeof(m));
    }
    Tensor M(3, 2, 1, NCHW, FP32);
    std::memcpy(M.data, kM, sizeof(kM));
    Tensor out;
    if (dtype == INT8) {
        std::vector<unsigned char> want;
        {
            TIME_PERF(r.oracle_ms);
            oracle_warp(src, want, dsize.w, dsize.h, m);
        }
        {
            TIME_PERF(r.vacv_ms);
            if (by_rotation) {
                va_cv::warp_affine(src, out, kRotScale, kRotAngle, dsize, rot_aux());
            } else {
                va_cv::warp_affine(src, out, M, dsize);
            }
        }
        score(r, want.data(), out);
    } else {
        std::vector<float> want;
        {
            TIME_PERF(r.oracle_ms);
            oracle_warp(src, want, dsize.w, dsize.h, m);
        }
        {
            TIME_PERF(r.vacv_ms);
            if (by_rotation) {
                va_cv::warp_affine(src, out, kRotScale, kRotAngle, dsize, rot_aux());
            } else {
                va_cv::warp_affine(src, out, M, dsize);
            }
        }
        score(r, want.data(), out);
    }
    if (std::memcmp(M.data, kM, sizeof(kM)) != 0) r.note = "M was modified";
    return r;
}

Result normalize_case(int w, int h, DLayout layout) {  // test_normalize.cpp:22-127
    Result r;
    Tensor src = load_image(w, h).change_layout(layout);
    const Tensor srcf = src.change_dtype(FP32);
    std::vector<float> want;
    {
        TIME_PERF(r.oracle_ms);
        oracle_normalize_auto((const float*)srcf.data, w, h, 3, layout, want);
    }
    Tensor f, out;
    {
        TIME_PERF(r.vacv_ms);
        f = src.change_dtype(FP32);
        va_cv::normalize(f, out);
    }
    score(r, want.data(), out);
    return r;
}

Result cvt_case(int w, int h) {  // test_cvt_color.cpp:23-57
    Result r;
    const Tensor bgr = load_image(w, h);
    Tensor yuv(w, h * 3 / 2, 1, INT8, NHWC);
    ImageUtil::bgr2nv21((unsigned char*)bgr.data, (unsigned char*)yuv.data, w, h);
    std::vector<unsigned char> want((size_t)w * h * 3);
    {
        TIME_PERF(r.oracle_ms);
        oracle_yuv420sp_to_bgr((const uint8_t*)yuv.data, want.data(), w, h, 1, 0);
    }
    Tensor out;
    {
        TIME_PERF(r.vacv_ms);
        va_cv::cvt_color(yuv, out, COLOR_YUV2BGR_NV21);
    }
    score(r, want.data(), out);
    // the reference scores against the original BGR frame (lossy NV21 round
    // trip); report that cosine too
    const float rt = ImageUtil::compare_image_data((const unsigned char*)bgr.data,
                                                   (const unsigned char*)out.data, (int)out.size());
    char buf[64];
    std::snprintf(buf, sizeof(buf), "bgr round-trip cosine %.5f", rt);
    r.note = std::fabs(rt - 1.0) <= 1e-2 ? std::string(buf) : std::string("LOW ") + buf;
    if (r.note.compare(0, 4, "LOW ") == 0) r.tol = -1;  // fail
    return r;
}

Result layout_case(DType dtype) {  // test_change_layout.cpp
    Result r;
    Tensor src = load_image(176, 144);
    if (dtype == FP32) src = src.change_dtype(FP32);
    std::vector<unsigned char> want(src.len());
    {
        TIME_PERF(r.oracle_ms);
        oracle_hwc_to_chw(src.data, want.data(), src.w, src.h, 3, (int)dtype_size(dtype));
    }
    Tensor out;
    {
        TIME_PERF(r.vacv_ms);
        out = src.change_layout(NCHW);
    }
    if (out.layout != NCHW) r.note = "layout not NCHW";
    if (dtype == FP32) {
        score(r, (const float*)want.data(), out);
    } else {
        score(r, want.data(), out);
    }
    return r;
}

Result dtype_case(bool to_f32) {  // test_change_dtype.cpp
    Result r;
    Tensor u8 = load_image(176, 144);
    if (to_f32) {
        std::vector<float> want(u8.size());
        {
            TIME_PERF(r.oracle_ms);
            oracle_u8_to_f32((const uint8_t*)u8.data, want.data(), (int64_t)u8.size());
        }
        Tensor out;
        {
            TIME_PERF(r.vacv_ms);
            out = u8.change_dtype(FP32);
        }
        score(r, want.data(), out);
    } else {
        // values with fractions, negatives and > 255: the truncating, wrapping cast
        Tensor f(176, 144, 3, FP32, NHWC);
        float* p = (float*)f.data;
        for (size_t i = 0; i < f.size(); ++i) p[i] = ((const unsigned char*)u8.data)[i] * 1.37f - 40.25f;
        std::vector<unsigned char> want(f.size());
        {
            TIME_PERF(r.oracle_ms);
            oracle_f32_to_u8(p, want.data(), (int64_t)f.size());
        }
        Tensor out;
        {
            TIME_PERF(r.vacv_ms);
            out = f.change_dtype(INT8);
        }
        score(r, want.data(), out);
        r.cosine = 1.0;  // wrapped values make the cosine meaningless; bit-exact is the bar
    }
    return r;
}

Result resize_normalize_case(int wi, int hi, int wo, int ho) {  // the headline op (cv.h:154)
    Result r;
    const Tensor src = load_image(wi, hi);
    const std::vector<float> mean = {103.94f, 116.78f, 123.68f}, stdv = {57.375f, 57.12f, 58.395f};
    std::vector<unsigned char> rs;
    std::vector<float> want;
    {
        TIME_PERF(r.oracle_ms);
        oracle_resize_u8(src, rs, wo, ho);
        std::vector<float> f(rs.size());
        oracle_u8_to_f32(rs.data(), f.data(), (int64_t)rs.size());
        want.resize(f.size());
        oracle_normalize_f32(f.data(), want.data(), (int64_t)wo * ho, 3, mean.data(), stdv.data());
    }
    Tensor out;
    {
        TIME_PERF(r.vacv_ms);
        va_cv::resize_normalize(src, out, VSize(wo, ho), 0, 0, INTER_LINEAR, floats_of(mean), floats_of(stdv));
    }
    score(r, want.data(), out);
    return r;
}

// batched frames (FramePipeline: H2D / kernel / D2H overlapped on three
// streams) give the same bytes as one call per frame, for host and device
// frames and every batched operator
Result batch_frames_case() {
    Result r;
    r.cosine = 1.0;
    std::string err;
    const Tensor base = load_image(1920, 1080);
    const int n = 7;  // more frames than the ring has slots
    std::vector<Tensor> src(n);
    for (int i = 0; i < n; ++i) {
        src[i] = base.clone();
        unsigned char* p = static_cast<unsigned char*>(src[i].data);
        for (size_t b = 0; b < src[i].len(); b += 97) p[b] = (unsigned char)(p[b] + 13 * i);
    }
    const std::vector<float> mean = {103.94f, 116.78f, 123.68f}, stdv = {57.375f, 57.12f, 58.395f};
    const Tensor tm = floats_of(mean), ts = floats_of(stdv);
    std::vector<Tensor> out;
    {
        TIME_PERF(r.vacv_ms);
        va_cv::resize_normalize(src, out, VSize(640, 360), 0, 0, INTER_LINEAR, tm, ts);
    }
    {
        TIME_PERF(r.oracle_ms);  // here: the per-frame calls
        for (int i = 0; i < n; ++i) {
            Tensor one;
            va_cv::resize_normalize(src[i], one, VSize(640, 360), 0, 0, INTER_LINEAR, tm, ts);
            if ((int)out.size() != n || out[i].len() != one.len() || std::memcmp(out[i].data, one.data, one.len()))
                err += "batched resize_normalize differs; ";
        }
    }
    std::vector<Tensor> o2;
    va_cv::resize(src, o2, VSize(1280, 720));
    Tensor m(3, 2, 1, FP32, NHWC);
    const float mv[6] = {0.9f, 0.1f, -20.f, -0.1f, 0.9f, 40.f};
    std::memcpy(m.data, mv, sizeof(mv));
    std::vector<Tensor> o3;
    va_cv::warp_affine(src, o3, m, VSize(1000, 600));
    for (int i = 0; i < n; ++i) {
        Tensor a, b;
        va_cv::resize(src[i], a, VSize(1280, 720));
        va_cv::warp_affine(src[i], b, m, VSize(1000, 600));
        if (std::memcmp(o2[i].data, a.data, a.len())) err += "batched resize differs; ";
        if (std::memcmp(o3[i].data, b.data, b.len())) err += "batched warp differs; ";
    }
    // dsize = 0 with fx / fy (cv::resize's form) through the batched overload
    std::vector<Tensor> o4;
    va_cv::resize(src, o4, VSize(0, 0), 0.5, 0.25, INTER_AREA);
    for (int i = 0; i < n; ++i) {
        Tensor a;
        va_cv::resize(src[i], a, VSize(0, 0), 0.5, 0.25, INTER_AREA);
        if (o4[i].w != 960 || o4[i].h != 270 || a.len() != o4[i].len() || std::memcmp(o4[i].data, a.data, a.len()))
            err += "batched fx/fy resize differs; ";
    }
    std::vector<Tensor> dev(n), od;
    for (int i = 0; i < n; ++i) dev[i] = src[i].to_device(0);
    va_cv::resize_normalize(dev, od, VSize(640, 360), 0, 0, INTER_LINEAR, tm, ts);
    for (int i = 0; i < n; ++i) {
        const Tensor h = od[i].to_host();
        if (!od[i].on_device() || std::memcmp(h.data, out[i].data, h.len())) err += "device frames differ; ";
    }
    if (!err.empty()) {
        r.note = err;
        r.tol = -1;
    }
    return r;
}

// device placement: the same pipeline on a device-resident tensor gives the
// same bytes as on a host tensor, and nothing leaves HBM in between
Result device_chain_case() {
    Result r;
    const Tensor host = load_image(1920, 1080);
    Tensor a, b;
    {
        TIME_PERF(r.oracle_ms);
        va_cv::resize(host, a, VSize(640, 360));
        a = a.change_layout(NCHW);
    }
    const Tensor dev = host.to_device(0);
    Tensor d;
    {
        TIME_PERF(r.vacv_ms);
        va_cv::resize(dev, d, VSize(640, 360));
        d = d.change_layout(NCHW);
    }
    if (!d.on_device() || a.on_device()) r.note = "wrong placement";
    score(r, (const unsigned char*)a.data, d);
    return r;
}

// Host-only Tensor semantics of tensor.cpp (no GPU needed): refcounted
// sharing, create() reuse, clone() independence, non-owning views; and
// without a HIP device every operator fails loudly (no CPU fallback).
Result tensor_host_case() {
    Result r;
    r.cosine = 1.0;
    std::string err;
    Tensor a(64, 32, 3, INT8, NHWC);
    std::memset(a.data, 7, a.len());
    {
        Tensor b = a;
        if (a.get_ref_count() != 2 || b.data != a.data) err += "copy does not share; ";
        Tensor e;
        e = b;
        if (a.get_ref_count() != 3) err += "assignment does not share; ";
    }
    if (a.get_ref_count() != 1) err += "refcount not restored; ";
    if (a.size() != 64u * 32 * 3 || a.len() != a.size() || a.stride != 64 * 32 || a.dims != 3) err += "bad size; ";
    void* before = a.data;
    a.create(64, 32, 3, INT8, NHWC);
    if (a.data != before) err += "create() did not reuse a matching buffer; ";
    Tensor c = a.clone();
    ((unsigned char*)c.data)[0] = 9;
    if (((unsigned char*)a.data)[0] != 7) err += "clone() shares memory; ";
    Tensor v(64, 32, 3, a.data, INT8, NHWC);
    if (v.get_ref_count() != 0 || v.data != a.data) err += "view owns memory; ";
    Tensor f(10, 4, FP32, NCHW);
    if (f.len() != 160 || f.dims != 2) err += "2-D FP32 tensor has the wrong size; ";
    f.release();
    if (!f.empty() || f.w != 0 || f.data) err += "release() left state; ";
    if (!err.empty()) {
        r.note = err;
        r.tol = -1;
    }
    return r;
}

// va_cv:: without a HIP device must throw, never compute on the host
Result no_device_case() {
    Result r;
    r.cosine = 1.0;
    Tensor a(64, 32, 3, INT8, NHWC), o;
    std::memset(a.data, 1, a.len());
    try {
        va_cv::resize(a, o, VSize(32, 16));
        r.note = "resize returned without a device";
        r.tol = -1;
    } catch (const std::runtime_error&) {
    }
    return r;
}

// Tensor semantics with the GPU: aliasing dst == src, loud failures
Result tensor_semantics_case() {
    Result r;
    r.cosine = 1.0;
    std::string err;
    Tensor a(64, 32, 3, INT8, NHWC);
    std::memset(a.data, 7, a.len());
    {
        Tensor b = a;
        if (a.get_ref_count() != 2 || b.data != a.data) err += "copy does not share; ";
    }
    if (a.get_ref_count() != 1) err += "refcount not restored; ";
    void* before = a.data;
    a.create(64, 32, 3, INT8, NHWC);
    if (a.data != before) err += "create() did not reuse a matching buffer; ";
    Tensor c = a.clone();
    ((unsigned char*)c.data)[0] = 9;
    if (((unsigned char*)a.data)[0] != 7) err += "clone() shares memory; ";
    Tensor v(64, 32, 3, a.data, INT8, NHWC);
    if (v.get_ref_count() != 0) err += "view owns memory; ";
    // dst aliases src, with a shape change
    Tensor img = load_image(640, 360);
    Tensor want;
    va_cv::resize(img, want, VSize(320, 180));
    va_cv::resize(img, img, VSize(320, 180));
    if (std::memcmp(img.data, want.data, want.len()) != 0) err += "aliased resize differs; ";
    // unsupported combinations fail loudly
    {
        // fractional INTER_AREA (OpenCV 2.4 resizeArea_) and dsize = 0 with
        // fx / fy (cv::resize derives the size): shapes only here, values in
        // the Python parity tests
        Tensor o;
        va_cv::resize(img, o, VSize(7, 7), 0, 0, INTER_AREA);
        if (o.w != 7 || o.h != 7 || o.c != 3) err += "fractional INTER_AREA shape; ";
        Tensor p;
        va_cv::resize(img, p, VSize(0, 0), 0.25, 0.5, INTER_NEAREST);
        if (p.w != 80 || p.h != 90) err += "fx/fy INTER_NEAREST shape; ";
    }
    {
        // integer INTER_AREA (OpenCV 2.4 resizeAreaFast_): 2x2 block means of a
        // 3-channel image take ResizeAreaFastVec's fast_mode, rounded half up
        Tensor o;
        va_cv::resize(img, o, VSize(160, 90), 0, 0, INTER_AREA);
        const uint8_t* s = static_cast<const uint8_t*>(img.data);
        const uint8_t* d = static_cast<const uint8_t*>(o.data);
        for (int y = 0; y < 90; y += 7)
            for (int x = 0; x < 160; x += 5)
                for (int k = 0; k < 3; ++k) {
                    const int sum = s[((2 * y) * 320 + 2 * x) * 3 + k] + s[((2 * y) * 320 + 2 * x + 1) * 3 + k] +
                                    s[((2 * y + 1) * 320 + 2 * x) * 3 + k] + s[((2 * y + 1) * 320 + 2 * x + 1) * 3 + k];
                    const int want_v = (sum + 2) >> 2;  // ResizeAreaFastVec fast_mode: half up
                    if (d[(y * 160 + x) * 3 + k] != want_v) { err += "INTER_AREA value; "; y = 90; x = 160; break; }
                }
    }
    {
        // BORDER_TRANSPARENT on a host dst: pixels without taps keep dst's
        // bytes, not whatever an earlier call left in the device scratch slot
        const float mv[6] = {0.6f, 0.1f, -60.f, -0.1f, 0.6f, 30.f};  // much of the output maps outside
        Tensor M(3, 2, 1, FP32, NHWC);
        std::memcpy(M.data, mv, sizeof(mv));
        Tensor stale;
        va_cv::warp_affine(img, stale, M, VSize(320, 180));  // fills the scratch slot with other bytes
        Tensor keep(320, 180, 3, INT8, NHWC);
        std::memset(keep.data, 77, keep.len());
        std::vector<unsigned char> want(keep.len(), 77);
        float inv[6];
        oracle_invert_affine(mv, inv);
        oracle_warp_affine_u8((const uint8_t*)img.data, img.w, img.h, 3, want.data(), 320, 180, inv);
        va_cv::warp_affine(img, keep, M, VSize(320, 180), INTER_LINEAR, BORDER_TRANSPARENT);
        if (keep.on_device() || std::memcmp(keep.data, want.data(), want.size()) != 0)
            err += "BORDER_TRANSPARENT on a host dst lost dst's bytes; ";
    }
    try {
        Tensor o;
        va_cv::crop(img, o, VRect(300, 0, 400, 10));
        err += "out-of-range crop did not throw; ";
    } catch (const std::runtime_error&) {
    }
    if (!VaAllocator::host_pinned()) err += "host tensors are not pinned; ";
    if (!err.empty()) {
        r.note = err;
        r.tol = -1;
    }
    return r;
}

}  // namespace

int main(int argc, char** argv) {
    std::string filter;
    bool host_only = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--res") && i + 1 < argc) g_res = argv[++i];
        else if (!std::strcmp(argv[i], "--filter") && i + 1 < argc) filter = argv[++i];
        else if (!std::strcmp(argv[i], "--times") && i + 1 < argc) g_times = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--host-only")) host_only = true;
    }
    const std::vector<std::pair<std::string, Case>> host_cases = {
        {"test_tensor_host_semantics", [] { return tensor_host_case(); }},
        {"test_no_device_fails_loudly", [] { return no_device_case(); }},
    };
    const std::vector<std::pair<std::string, Case>> gpu_cases = {
        // test_main.cpp:20-62 (the reference's case names)
        {"test_crop_hwc_5x5", [] { return crop_case(VRect(0, 0, 5, 5), NHWC, INT8); }},
        {"test_crop_hwc_5x5_FP32", [] { return crop_case(VRect(0, 0, 5, 5), NHWC, FP32); }},
        {"test_crop_hwc_320x180", [] { return crop_case(VRect(0, 0, 320, 180), NHWC, INT8); }},
        {"test_crop_hwc_640x360", [] { return crop_case(VRect(0, 0, 640, 360), NHWC, INT8); }},
        {"test_crop_hwc_1280x720", [] { return crop_case(VRect(0, 0, 1280, 720), NHWC, INT8); }},
        {"test_crop_hwc_1920x1080", [] { return crop_case(VRect(0, 0, 1920, 1080), NHWC, INT8); }},
        {"test_crop_chw_320x180", [] { return crop_case(VRect(0, 0, 320, 180), NCHW, INT8); }},
        {"test_crop_chw_320x180_FP32", [] { return crop_case(VRect(0, 0, 320, 180), NCHW, FP32); }},
        {"test_crop_chw_640x360", [] { return crop_case(VRect(0, 0, 640, 360), NCHW, INT8); }},
        {"test_crop_chw_5x5", [] { return crop_case(VRect(0, 0, 5, 5), NCHW, INT8); }},
        {"test_crop_chw_offset_FP32", [] { return crop_case(VRect(10.7f, 20.2f, 330.9f, 200.5f), NCHW, FP32); }},
        {"test_resize_bilinear_hwc_u8_320x180", [] { return resize_case(NHWC, INT8, INTER_LINEAR, 320, 180); }},
        {"test_resize_bilinear_chw_u8_320x180", [] { return resize_case(NCHW, INT8, INTER_LINEAR, 320, 180); }},
        {"test_resize_bilinear_hwc_fp32_320x180", [] { return resize_case(NHWC, FP32, INTER_LINEAR, 320, 180); }},
        {"test_resize_bilinear_chw_fp32_320x180", [] { return resize_case(NCHW, FP32, INTER_LINEAR, 320, 180); }},
        {"test_resize_cubic_hwc_fp32_320x180", [] { return resize_case(NHWC, FP32, INTER_CUBIC, 320, 180); }},
        {"test_resize_cubic_chw_fp32_320x180", [] { return resize_case(NCHW, FP32, INTER_CUBIC, 320, 180); }},
        {"test_resize_cubic_hwc_u8_224x224", [] { return resize_case(NHWC, INT8, INTER_CUBIC, 224, 224); }},
        {"test_change_dtype_u8_to_fp32_176x144", [] { return dtype_case(true); }},
        {"test_change_dtype_fp32_to_u8_176x144", [] { return dtype_case(false); }},
        {"test_change_layout_hwc_to_chw_u8_176x144", [] { return layout_case(INT8); }},
        {"test_change_layout_hwc_to_chw_fp32_176x144", [] { return layout_case(FP32); }},
        {"test_normalize_hwc_176x144", [] { return normalize_case(176, 144, NHWC); }},
        {"test_normalize_chw_176x144", [] { return normalize_case(176, 144, NCHW); }},
        {"test_normalize_hwc_284x214", [] { return normalize_case(284, 214, NHWC); }},
        {"test_normalize_chw_284x214", [] { return normalize_case(284, 214, NCHW); }},
        {"test_warp_affine_hwc_u8", [] { return warp_case(NHWC, INT8, false, 0); }},
        {"test_warp_affine_hwc_fp32", [] { return warp_case(NHWC, FP32, false, 0); }},
        {"test_warp_affine_chw_u8", [] { return warp_case(NCHW, INT8, false, 0); }},
        {"test_warp_affine_chw_fp32", [] { return warp_case(NCHW, FP32, false, 0); }},
        {"test_get_rotation_matrix_hwc_u8", [] { return warp_case(NHWC, INT8, true, 3); }},
        {"test_get_rotation_matrix_hwc_fp32", [] { return warp_case(NHWC, FP32, true, 1); }},
        {"test_get_rotation_matrix_chw_u8", [] { return warp_case(NCHW, INT8, true, 1); }},
        {"test_nv21_to_bgr_176x144", [] { return cvt_case(176, 144); }},
        {"test_nv21_to_bgr_640x360", [] { return cvt_case(640, 360); }},
        {"test_nv21_to_bgr_1280x720", [] { return cvt_case(1280, 720); }},
        {"test_nv21_to_bgr_1920x1080", [] { return cvt_case(1920, 1080); }},
        {"test_nv21_to_bgr_2560x1440", [] { return cvt_case(2560, 1440); }},
        // additions: the headline fused op, device placement, Tensor semantics
        {"test_resize_normalize_hwc_1920x1080_640x360", [] { return resize_normalize_case(1920, 1080, 640, 360); }},
        {"test_device_chain_1920x1080", [] { return device_chain_case(); }},
        {"test_batch_frames_1920x1080", [] { return batch_frames_case(); }},
        {"test_tensor_semantics", [] { return tensor_semantics_case(); }},
        {"test_tensor_host_semantics", [] { return tensor_host_case(); }},
    };
    const auto& cases = host_only ? host_cases : gpu_cases;

    int run = 0, failed = 0;
    std::string failures;
    std::printf("%-48s %12s %12s %10s %12s  %s\n", "case", "oracle ms", "vacv ms", "cosine", "max|diff|", "bar");
    for (const auto& c : cases) {
        if (!filter.empty() && c.first.find(filter) == std::string::npos) continue;
        Result acc;
        bool ok = true;
        std::string note;
        try {
            for (int t = 0; t < g_times; ++t) {  // cv_profile.cpp:42-72 averages repeated runs
                const Result r = c.second();
                acc.oracle_ms += r.oracle_ms / g_times;
                acc.vacv_ms += r.vacv_ms / g_times;
                acc.cosine = r.cosine;
                acc.max_abs = std::max(acc.max_abs, r.max_abs);
                acc.tol = r.tol;
                note = r.note;
                ok = ok && passed(r) && (r.note.empty() || r.note.find("cosine") != std::string::npos);
            }
        } catch (const std::exception& e) {
            ok = false;
            note = std::string("exception: ") + e.what();
        }
        ++run;
        if (!ok) {
            ++failed;
            failures += (failures.empty() ? "\"" : ", \"") + c.first + "\"";
        }
        char bar[32];
        if (acc.tol == 0) {
            std::snprintf(bar, sizeof(bar), "bit-exact");
        } else {
            std::snprintf(bar, sizeof(bar), "<= %g", acc.tol);
        }
        std::printf("%-48s %12.3f %12.3f %10.6f %12.3g  %-10s %s %s\n", c.first.c_str(), acc.oracle_ms, acc.vacv_ms,
                    acc.cosine, acc.max_abs, bar, ok ? "[TEST SUCCESS]" : "[TEST FAILED!]", note.c_str());
    }
    std::printf("{\"cases\": %d, \"failed\": %d, \"failures\": [%s]}\n", run, failed, failures.c_str());
    return failed ? 1 : 0;
}
