// k_area.hip -- INTER_AREA at scales the integer fast path does not cover.
//
// The reference hands INTER_AREA to cv::resize (resize.cpp:44-49); the
// pinned OpenCV 2.4.13.4 (CMakeLists.txt:23) then takes, for a non-integer
// scale (imgwarp.cpp, cv::resize):
//  * both scales >= 1 (a down-scale): resizeArea_ over computeResizeAreaTab's
//    weight tables.  Output (x, y, c) = saturate(sum_j beta_j * buf_j), where
//    buf_j = sum_k S(si_k, sy_j) * alpha_k over the x table entries of x, all
//    fp32 in table order (buf from 0, sum from its first term) -- the order of
//    its row loop, made per output element here; u8 rounds half to even;
//  * otherwise (an up-scale on either axis): its bilinear resize with the
//    area-mode taps (sx = floor(dx * scale), fx = (float)((dx + 1) - (sx + 1) *
//    inv_scale), ...), u8 in OpenCV's fixed point ((h >> 4) * b >> 16 rows,
//    + 2 >> 2; the arithmetic of this build's OPENCV bilinear mode), fp32 as
//    h = S0 * a0 + S1 * a1 per row, out = h0 * b0 + h1 * b1.
// Both tables are built on the host with OpenCV's double arithmetic
// (area_tables, below) and cached on the device per geometry, as the resize
// plans are (resize_plan.cpp).  The test oracle restates the same algorithm
// independently (parity unpinned: no reference entry runs these modes here).
//
// Kernels: one thread per output element, a workgroup row = one output row.
// Neighbouring threads read neighbouring source bytes, so the table walks
// coalesce; these modes are delegated to OpenCV by the reference and are not
// on the metric path.
#pragma clang fp contract(off)

#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "vacv_device.hpp"

namespace vacv {
namespace {

struct AreaTabsDev {
    // fractional down-scale (CSR per output column / row)
    const int* xoff;     // [w_out + 1]
    const int* xsi;      // [nx] source element offset (column * cc)
    const float* xal;    // [nx]
    const int* yoff;     // [h_out + 1]
    const int* ysi;      // [ny] source row
    const float* yal;    // [ny]
    // up-scale (bilinear, area-mode taps)
    const int* ux;       // [w_out] {x0, x1} source columns
    const float* uxa;    // [w_out] {a0, a1} fp32 coefficients
    const int* uxi;      // [w_out] packed {a0, a1} u16 fixed-point coefficients (saturate_cast<short>)
    const int* uy;       // [h_out] {y0, y1}
    const float* uya;    // [h_out] {b0, b1}
    const int* uyi;      // [h_out] {b0, b1} int
};

struct AreaLaunch {
    PlaneGeom src, dst;
    int n;
    int out;
    NormSpec norm;
    AreaTabsDev t;
};

template <typename TIn, int OUT, int CC>
__device__ __forceinline__ void area_store(const AreaLaunch& L, unsigned char* drow, int e, int img, int plane, int k,
                                           float f, int vi) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    TOut* d = reinterpret_cast<TOut*>(drow) + e;
    constexpr bool U8 = std::is_same<TIn, uint8_t>::value;
    if (OUT == kOutSame) {
        if (U8) *d = (TOut)vi;
        else *d = (TOut)f;
    } else if (OUT == kOutF32) {
        *d = (TOut)(U8 ? (float)vi : f);
    } else {
        const ChanNorm cn = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
        *d = (TOut)(U8 ? normalize_u8v(cn, vi) : normalize_f(cn, f));
    }
}

template <typename TIn, int OUT, int CC>
__global__ void __launch_bounds__(kBlock) area_frac_kernel(AreaLaunch L) {
    const int e = (int)(blockIdx.x * kBlock + threadIdx.x);
    const int y = blockIdx.y;
    const int pidx = blockIdx.z;
    if (e >= L.dst.w * CC) return;
    const int x = e / CC, k = e - x * CC;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const int x0 = L.t.xoff[x], x1 = L.t.xoff[x + 1];
    const int y0 = L.t.yoff[y], y1 = L.t.yoff[y + 1];
    float sum = 0.f;
    for (int j = y0; j < y1; ++j) {
        const TIn* row = reinterpret_cast<const TIn*>(sp + (int64_t)L.t.ysi[j] * L.src.row_pitch) + k;
        float buf = 0.f;
        for (int i = x0; i < x1; ++i) buf = buf + (float)row[L.t.xsi[i]] * L.t.xal[i];
        const float b = L.t.yal[j] * buf;
        sum = j == y0 ? b : sum + b;
    }
    int vi = 0;
    if (std::is_same<TIn, uint8_t>::value) vi = clamp_u8((int)rintf(sum));  // saturate_cast<uchar>: cvRound
    unsigned char* drow = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                          (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch;
    area_store<TIn, OUT, CC>(L, drow, e, img, plane, k, sum, vi);
}

template <typename TIn, int OUT, int CC>
__global__ void __launch_bounds__(kBlock) area_up_kernel(AreaLaunch L) {
    const int e = (int)(blockIdx.x * kBlock + threadIdx.x);
    const int y = blockIdx.y;
    const int pidx = blockIdx.z;
    if (e >= L.dst.w * CC) return;
    const int x = e / CC, k = e - x * CC;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const int sx0 = L.t.ux[2 * x] * CC + k, sx1 = L.t.ux[2 * x + 1] * CC + k;
    const TIn* r0 = reinterpret_cast<const TIn*>(sp + (int64_t)L.t.uy[2 * y] * L.src.row_pitch);
    const TIn* r1 = reinterpret_cast<const TIn*>(sp + (int64_t)L.t.uy[2 * y + 1] * L.src.row_pitch);
    float f = 0.f;
    int vi = 0;
    if constexpr (std::is_same<TIn, uint8_t>::value) {
        const int pa = L.t.uxi[x];
        const int a0 = pa & 0xFFFF, a1 = pa >> 16;
        const int h0 = (int)r0[sx0] * a0 + (int)r0[sx1] * a1;
        const int h1 = (int)r1[sx0] * a0 + (int)r1[sx1] * a1;
        const int b0 = L.t.uyi[2 * y], b1 = L.t.uyi[2 * y + 1];
        const int v = ((((int)(short)(h0 >> 4)) * b0) >> 16) + ((((int)(short)(h1 >> 4)) * b1) >> 16) + 2;
        vi = clamp_u8(v >> 2);
    } else {
        const float a0 = L.t.uxa[2 * x], a1 = L.t.uxa[2 * x + 1];
        const bool edge = sx0 == sx1;  // dx >= xmax: D = S[sx] (HResizeLinear's tail)
        const float h0 = edge ? (float)r0[sx0] : (float)r0[sx0] * a0 + (float)r0[sx1] * a1;
        const float h1 = edge ? (float)r1[sx0] : (float)r1[sx0] * a0 + (float)r1[sx1] * a1;
        f = h0 * L.t.uya[2 * y] + h1 * L.t.uya[2 * y + 1];
    }
    unsigned char* drow = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                          (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch;
    area_store<TIn, OUT, CC>(L, drow, e, img, plane, k, f, vi);
}

// ---- host: OpenCV's tables ------------------------------------------------

// computeResizeAreaTab (imgwarp.cpp), per output index: entries (si, alpha)
void area_tab(int ssize, int dsize, double scale, std::vector<int>& off, std::vector<int>& si,
              std::vector<float>& al) {
    off.assign(dsize + 1, 0);
    si.clear();
    al.clear();
    for (int dx = 0; dx < dsize; ++dx) {
        off[dx] = (int)si.size();
        const double fsx1 = dx * scale;
        const double fsx2 = fsx1 + scale;
        const double cell = std::min(scale, ssize - fsx1);
        int sx1 = (int)std::ceil(fsx1), sx2 = (int)std::floor(fsx2);
        sx2 = std::min(sx2, ssize - 1);
        sx1 = std::min(sx1, sx2);
        if (sx1 - fsx1 > 1e-3) {
            si.push_back(sx1 - 1);
            al.push_back((float)((sx1 - fsx1) / cell));
        }
        for (int sx = sx1; sx < sx2; ++sx) {
            si.push_back(sx);
            al.push_back((float)(1.0 / cell));
        }
        if (fsx2 - sx2 > 1e-3) {
            si.push_back(sx2);
            al.push_back((float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell));
        }
    }
    off[dsize] = (int)si.size();
}

// cv::resize's area-mode bilinear tap of one axis: source index pair and the
// fp32 / fixed-point coefficients (saturate_cast<short>(c * 2048): half even)
void area_up_tab(int n_in, int n_out, double scale, double inv, std::vector<int>& idx, std::vector<float>& cf,
                 std::vector<int>& ci) {
    idx.resize(2 * n_out);
    cf.resize(2 * n_out);
    ci.resize(2 * n_out);
    for (int d = 0; d < n_out; ++d) {
        int sx = (int)std::floor(d * scale);
        float fx = (float)((d + 1) - (sx + 1) * inv);
        fx = fx <= 0 ? 0.f : fx - (float)std::floor(fx);
        if (sx >= n_in - 1) {
            fx = 0.f;
            sx = n_in - 1;
        }
        idx[2 * d] = sx;
        idx[2 * d + 1] = std::min(sx + 1, n_in - 1);
        cf[2 * d] = 1.f - fx;
        cf[2 * d + 1] = fx;
        ci[2 * d] = (int)std::nearbyint(cf[2 * d] * 2048.f);
        ci[2 * d + 1] = (int)std::nearbyint(cf[2 * d + 1] * 2048.f);
    }
}

struct CachedTabs {
    int device = 0;  // owner of dev
    void* dev = nullptr;
    AreaTabsDev t{};
};
std::mutex g_area_mu;
// keyed by device first: the C++ layer leases any device, and a table lives on one
std::map<std::tuple<int, int, int, int, int, int, double, double, int>, CachedTabs> g_area_tabs;
bool free_tabs(CachedTabs& c) { return hipFree(c.dev) == hipSuccess; }

int area_tables(const ResizeLaunch& R, double inv_x, double inv_y, bool up, int cc, hipStream_t s,
                AreaTabsDev& out) {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return VACV_ERR_HIP;
    const auto key = std::make_tuple(device, R.src.w, R.src.h, R.dst.w, R.dst.h, cc, inv_x, inv_y, (int)up);
    std::lock_guard<std::mutex> lk(g_area_mu);
    auto it = g_area_tabs.find(key);
    if (it == g_area_tabs.end()) {
        const double sx = 1. / inv_x, sy = 1. / inv_y;
        std::vector<unsigned char> img;
        auto put = [&img](const void* p, size_t b) {
            const size_t o = (img.size() + 15) & ~size_t(15);
            img.resize(o + b);
            if (b) std::memcpy(img.data() + o, p, b);
            return o;
        };
        size_t o[12] = {};
        if (!up) {
            std::vector<int> xoff, xsi, yoff, ysi;
            std::vector<float> xal, yal;
            area_tab(R.src.w, R.dst.w, sx, xoff, xsi, xal);
            area_tab(R.src.h, R.dst.h, sy, yoff, ysi, yal);
            for (int& v : xsi) v *= cc;  // element offsets, as OpenCV's si
            o[0] = put(xoff.data(), xoff.size() * 4);
            o[1] = put(xsi.data(), xsi.size() * 4);
            o[2] = put(xal.data(), xal.size() * 4);
            o[3] = put(yoff.data(), yoff.size() * 4);
            o[4] = put(ysi.data(), ysi.size() * 4);
            o[5] = put(yal.data(), yal.size() * 4);
        } else {
            std::vector<int> ux, uxi, uy, uyi;
            std::vector<float> uxa, uya;
            area_up_tab(R.src.w, R.dst.w, sx, inv_x, ux, uxa, uxi);
            area_up_tab(R.src.h, R.dst.h, sy, inv_y, uy, uya, uyi);
            std::vector<int> packed(R.dst.w);
            for (int d = 0; d < R.dst.w; ++d) packed[d] = uxi[2 * d] | (uxi[2 * d + 1] << 16);
            o[6] = put(ux.data(), ux.size() * 4);
            o[7] = put(uxa.data(), uxa.size() * 4);
            o[8] = put(packed.data(), packed.size() * 4);
            o[9] = put(uy.data(), uy.size() * 4);
            o[10] = put(uya.data(), uya.size() * 4);
            o[11] = put(uyi.data(), uyi.size() * 4);
        }
        if (g_area_tabs.size() > 64)  // bounded cache
            (void)evict_device_cache(g_area_tabs, free_tabs);
        CachedTabs c;
        c.device = device;
        if (hipMalloc(&c.dev, img.size() + 16) != hipSuccess) return VACV_ERR_NO_MEMORY;
        // one upload per geometry; synchronised so any stream may use it next
        if (hipMemcpyAsync(c.dev, img.data(), img.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            (void)hipFree(c.dev);
            return VACV_ERR_HIP;
        }
        const unsigned char* b = static_cast<const unsigned char*>(c.dev);
        if (!up) {
            c.t.xoff = reinterpret_cast<const int*>(b + o[0]);
            c.t.xsi = reinterpret_cast<const int*>(b + o[1]);
            c.t.xal = reinterpret_cast<const float*>(b + o[2]);
            c.t.yoff = reinterpret_cast<const int*>(b + o[3]);
            c.t.ysi = reinterpret_cast<const int*>(b + o[4]);
            c.t.yal = reinterpret_cast<const float*>(b + o[5]);
        } else {
            c.t.ux = reinterpret_cast<const int*>(b + o[6]);
            c.t.uxa = reinterpret_cast<const float*>(b + o[7]);
            c.t.uxi = reinterpret_cast<const int*>(b + o[8]);
            c.t.uy = reinterpret_cast<const int*>(b + o[9]);
            c.t.uya = reinterpret_cast<const float*>(b + o[10]);
            c.t.uyi = reinterpret_cast<const int*>(b + o[11]);
        }
        it = g_area_tabs.emplace(key, c).first;
    }
    out = it->second.t;
    return VACV_OK;
}

template <typename TIn, int OUT, int CC>
hipError_t launch_cc(const AreaLaunch& A, bool up, dim3 grid, hipStream_t s) {
    if (up) hipLaunchKernelGGL((area_up_kernel<TIn, OUT, CC>), grid, dim3(kBlock), 0, s, A);
    else hipLaunchKernelGGL((area_frac_kernel<TIn, OUT, CC>), grid, dim3(kBlock), 0, s, A);
    return hipGetLastError();
}

template <typename TIn, int OUT>
hipError_t launch_out(const AreaLaunch& A, bool up, dim3 grid, hipStream_t s) {
    switch (A.src.cc) {
        case 1: return launch_cc<TIn, OUT, 1>(A, up, grid, s);
        case 2: return launch_cc<TIn, OUT, 2>(A, up, grid, s);
        case 3: return launch_cc<TIn, OUT, 3>(A, up, grid, s);
        case 4: return launch_cc<TIn, OUT, 4>(A, up, grid, s);
        default: return hipErrorInvalidValue;
    }
}

template <typename TIn>
hipError_t launch_t(const AreaLaunch& A, bool up, dim3 grid, hipStream_t s) {
    if (A.out == kOutSame) return launch_out<TIn, kOutSame>(A, up, grid, s);
    if (A.out == kOutF32) return launch_out<TIn, kOutF32>(A, up, grid, s);
    return launch_out<TIn, kOutNorm>(A, up, grid, s);
}

}  // namespace

int launch_resize_area_general(const ResizeLaunch& R, double inv_x, double inv_y, hipStream_t s) {
    if (R.src.cc > 4) return VACV_ERR_UNSUPPORTED;  // OpenCV asserts cn <= 4 here
    if (R.dst.h > 65535 || (int64_t)R.n * R.src.planes > 65535) return VACV_ERR_UNSUPPORTED;
    const bool up = !(1. / inv_x >= 1. && 1. / inv_y >= 1.);
    AreaLaunch A{};
    A.src = R.src;
    A.dst = R.dst;
    A.n = R.n;
    A.out = R.out;
    A.norm = R.norm;
    const int st = area_tables(R, inv_x, inv_y, up, R.src.cc, s, A.t);
    if (st) return st;
    const dim3 grid((R.dst.w * R.src.cc + kBlock - 1) / kBlock, R.dst.h, R.n * R.src.planes);
    const hipError_t e = R.src.esize == 1 ? launch_t<uint8_t>(A, up, grid, s) : launch_t<float>(A, up, grid, s);
    return e == hipSuccess ? VACV_OK : VACV_ERR_HIP;
}

int release_area_tables() {
    std::lock_guard<std::mutex> lk(g_area_mu);
    return evict_device_cache(g_area_tabs, free_tabs);
}

}  // namespace vacv
