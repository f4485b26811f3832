// k_match.hip -- match_template and minMaxIdx.
//
// The reference's MatchTemplate::match_template / minMaxIdx call
// cv::matchTemplate / cv::minMaxIdx (match_template.cpp:13-46; the
// naive/NEON bodies are empty todo stubs, :48-61).  OpenCV 2.4.13.4's
// algorithm (templmatch.cpp): R = crossCorr(image, templ) as float, then a
// per-method normalisation in double from window sums (integral images) and
// the template's mean / stddev.  Here:
//  * match_corr_u8_kernel: the correlation EXACTLY (u8: v_dot4_u32_u8 over
//    4 bytes at a time, per-template-row u32 sums into u64), one image row per
//    wave staged in LDS, the whole template in LDS, 4 adjacent outputs per
//    lane sharing a sliding window of source dwords (v_alignbyte picks each
//    output's 4 bytes); fp32 input: match_corr_f32_kernel, fp64 sums;
//  * match_integral_rows_kernel / _cols_kernel: OpenCV's double integral
//    images (sum, sqsum) in its summation order;
//  * match_finish_kernel: the window's per-channel S_c and Q as their 4-term
//    differences, then OpenCV's normalisation formula, in double, in OpenCV's
//    operation order;
//  * match_tstats_kernel: the template's per-channel mean / stddev (one
//    workgroup, fixed-order tree: deterministic).
// For u8 every sum is exact, so the result is the exact correlation rounded
// to float followed by OpenCV's double formula (OpenCV's own DFT crossCorr
// rounds differently: parity unpinned).
//  * min_max_kernel + min_max_final_kernel: cv::minMaxIdx of one channel --
//    the first (row-major) min / max of the unmasked, non-NaN elements.
#pragma clang fp contract(off)

#include <algorithm>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kOutPerLane = 4;
constexpr int kTileX = 64 * kOutPerLane;  // result columns per wave

// ---- correlation ------------------------------------------------------------

// wave w of the workgroup: result row r = blockIdx.y * 4 + w, columns
// [blockIdx.x * kTileX, +kTileX); lane l: columns x0 + 4l .. 4l + 3
template <int CN>
__global__ void __launch_bounds__(kBlock) match_corr_u8_kernel(MatchLaunch M) {
    extern __shared__ uint32_t lds[];
    const int w = M.tw, h = M.th;
    const int K = w * CN, K4 = (K + 3) >> 2;          // template row bytes, dwords (zero padded)
    constexpr int NW = (3 * CN) / 4 + 2;          // window dwords per k4 step
    const int span4 = 64 * CN + K4 + NW + 1;      // staged image dwords per row: every lane's window
    uint32_t* tpl = lds;                               // [h][K4]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* row = lds + h * K4 + wave * span4;
    const int img = blockIdx.z;
    const unsigned char* ib = M.img + (int64_t)img * M.img_pitch;
    // the template, zero padded per row, once per workgroup
    for (int i = threadIdx.x; i < h * K4; i += kBlock) {
        const int yy = i / K4, k4 = i - yy * K4;
        const unsigned char* tr = M.tpl + (int64_t)yy * M.tpl_row;
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (4 * k4 + b < K) v |= (uint32_t)tr[4 * k4 + b] << (8 * b);
        tpl[i] = v;
    }
    __syncthreads();

    const int r = blockIdx.y * 4 + wave;
    const int x0 = blockIdx.x * kTileX;
    if (r >= M.rh) return;  // whole wave (no barrier below)
    const int ebase = x0 * CN;                    // first staged byte of each image row
    const int row_bytes = M.iw * CN;
    uint64_t acc[kOutPerLane] = {0, 0, 0, 0};
    for (int yy = 0; yy < h; ++yy) {
        // stage image row r + yy, bytes [ebase, ebase + 4*span4), zero past the row
        const unsigned char* ir = ib + (int64_t)(r + yy) * M.img_row;
        for (int d = lane; d < span4; d += 64) {
            const int e = ebase + 4 * d;
            uint32_t v = 0;
            if (e + 4 <= row_bytes && ((reinterpret_cast<uintptr_t>(ir + e) & 3) == 0)) {
                v = *reinterpret_cast<const uint32_t*>(ir + e);
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (e + b < row_bytes) v |= (uint32_t)ir[e + b] << (8 * b);
            }
            row[d] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // lane's outputs start at byte 4*lane*CN = dword lane*CN
        const uint32_t* rp = row + lane * CN;
        const uint32_t* tp = tpl + yy * K4;
        uint32_t win[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) win[j] = rp[j];
        uint32_t a32[kOutPerLane] = {0, 0, 0, 0};
        for (int k4 = 0; k4 < K4; ++k4) {
            const uint32_t t = tp[k4];  // LDS broadcast
#pragma unroll
            for (int o = 0; o < kOutPerLane; ++o) {
                const int off = o * CN;  // byte offset of output o's window
                const uint32_t v = (off & 3) ? __builtin_amdgcn_alignbyte(win[(off >> 2) + 1], win[off >> 2], off & 3)
                                             : win[off >> 2];
                a32[o] = __builtin_amdgcn_udot4(v, t, a32[o], false);
            }
#pragma unroll
            for (int j = 0; j < NW - 1; ++j) win[j] = win[j + 1];
            win[NW - 1] = rp[k4 + NW];
        }
#pragma unroll
        for (int o = 0; o < kOutPerLane; ++o) acc[o] += a32[o];  // a row: <= 255^2 * K < 2^32
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    float* out = reinterpret_cast<float*>(M.res + (int64_t)img * M.res_pitch + (int64_t)r * M.res_row);
#pragma unroll
    for (int o = 0; o < kOutPerLane; ++o) {
        const int x = x0 + 4 * lane + o;
        if (x < M.rw) out[x] = (float)(double)acc[o];  // crossCorr's float result
    }
}

template <int CN>
__global__ void __launch_bounds__(kBlock) match_corr_f32_kernel(MatchLaunch M) {
    extern __shared__ uint32_t lds[];
    float* tpl = reinterpret_cast<float*>(lds);
    const int w = M.tw, h = M.th, K = w * CN;
    const int span = (kTileX + w - 1) * CN;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* row = tpl + h * K + wave * span;
    const int img = blockIdx.z;
    const unsigned char* ib = M.img + (int64_t)img * M.img_pitch;
    for (int i = threadIdx.x; i < h * K; i += kBlock) {
        const int yy = i / K, k = i - yy * K;
        tpl[i] = reinterpret_cast<const float*>(M.tpl + (int64_t)yy * M.tpl_row)[k];
    }
    __syncthreads();
    const int r = blockIdx.y * 4 + wave;
    const int x0 = blockIdx.x * kTileX;
    if (r >= M.rh) return;
    const int ebase = x0 * CN, row_el = M.iw * CN;
    double acc[kOutPerLane] = {0, 0, 0, 0};
    for (int yy = 0; yy < h; ++yy) {
        const float* ir = reinterpret_cast<const float*>(ib + (int64_t)(r + yy) * M.img_row);
        for (int e = lane; e < span; e += 64) row[e] = ebase + e < row_el ? ir[ebase + e] : 0.f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float* rp = row + 4 * lane * CN;
        const float* tp = tpl + yy * K;
        for (int k = 0; k < K; ++k) {
            const double t = tp[k];
#pragma unroll
            for (int o = 0; o < kOutPerLane; ++o) acc[o] += t * (double)rp[o * CN + k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    float* out = reinterpret_cast<float*>(M.res + (int64_t)img * M.res_pitch + (int64_t)r * M.res_row);
#pragma unroll
    for (int o = 0; o < kOutPerLane; ++o) {
        const int x = x0 + 4 * lane + o;
        if (x < M.rw) out[x] = (float)acc[o];
    }
}

// ---- window statistics: OpenCV's integral images -----------------------------
// cv::integral(img, sum, sqsum, CV_64F) as templmatch.cpp builds them, in its
// order: per channel a running row sum s (s += v left to right), then
// sum[y+1][x+1] = sum[y][x+1] + s (sqsum likewise with (double)v * v).  The
// window sums are then its 4-term differences, so S_c and Q are OpenCV's own
// double values (exact for u8).  Layout per image: [H+1][(W+1)*cn] for sum,
// then the same for sqsum; row 0 and column 0 are zero.

// pass 1: the running row sums of row y, channel c, into integral row y+1
template <typename T>
__global__ void __launch_bounds__(kBlock) match_integral_rows_kernel(MatchLaunch M) {
    const int cn = M.cn;
    const int t = blockIdx.x * kBlock + threadIdx.x;  // y * cn + c
    const int img = blockIdx.y;
    if (t >= M.ih * cn) return;
    const int y = t / cn, c = t - y * cn;
    const int64_t step = (int64_t)(M.iw + 1) * cn;
    double* sum = M.box + (int64_t)img * 2 * (M.ih + 1) * step;
    double* sq = sum + (int64_t)(M.ih + 1) * step;
    const T* src = reinterpret_cast<const T*>(M.img + (int64_t)img * M.img_pitch + (int64_t)y * M.img_row);
    double s = 0, q = 0;
    sum[(int64_t)(y + 1) * step + c] = 0;
    sq[(int64_t)(y + 1) * step + c] = 0;
    for (int x = 0; x < M.iw; ++x) {
        const double v = (double)src[x * cn + c];
        s += v;
        q += v * v;
        sum[(int64_t)(y + 1) * step + (x + 1) * cn + c] = s;
        sq[(int64_t)(y + 1) * step + (x + 1) * cn + c] = q;
    }
    if (y == 0) {  // row 0 is zero
        for (int x = 0; x <= M.iw; ++x) {
            sum[x * cn + c] = 0;
            sq[x * cn + c] = 0;
        }
    }
}

// pass 1 for u8 (round 5): every running sum is an integer (< 2^31 for rows
// up to 33,000 pixels: host-checked), exact in int32 and in double, so the
// order of the additions cannot change a value -- a WAVE per row: 64
// consecutive row elements per step, an inclusive scan across the lanes of
// each channel (lanes cn apart), plus the channel's carry from the steps
// before; its stores are 64 consecutive doubles (the per-thread kernel above
// wrote one double per lane 30 KiB apart).
__global__ void __launch_bounds__(kBlock) match_integral_rows_u8_kernel(MatchLaunch M) {
    const int cn = M.cn;
    const int lane = threadIdx.x & 63;
    const int y = (int)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int img = blockIdx.y;
    if (y >= M.ih) return;  // whole wave
    const int64_t step = (int64_t)(M.iw + 1) * cn;
    double* sum = M.box + (int64_t)img * 2 * (M.ih + 1) * step;
    double* sq = sum + (int64_t)(M.ih + 1) * step;
    const unsigned char* src = M.img + (int64_t)img * M.img_pitch + (int64_t)y * M.img_row;
    double* os = sum + (int64_t)(y + 1) * step;
    double* oq = sq + (int64_t)(y + 1) * step;
    if (lane < cn) {
        os[lane] = 0;
        oq[lane] = 0;
    }
    if (y == 0) {  // row 0 is zero
        for (int64_t e = lane; e < step; e += 64) {
            sum[e] = 0;
            sq[e] = 0;
        }
    }
    const int n = M.iw * cn;
    int cs[4] = {0, 0, 0, 0}, cq[4] = {0, 0, 0, 0};  // per-channel carries (uniform)
    int c0 = 0;                                        // the channel of the step's first element
    for (int base = 0; base < n; base += 64) {
        const int e = base + lane;
        const int v = e < n ? (int)src[e] : 0;
        const int c = (c0 + lane) % cn;
        int s = v, q = v * v;
        for (int d = cn; d < 64; d <<= 1) {
            const int ts = __shfl_up(s, d, 64), tq = __shfl_up(q, d, 64);
            if (lane >= d) {
                s += ts;
                q += tq;
            }
        }
        s += c == 0 ? cs[0] : c == 1 ? cs[1] : c == 2 ? cs[2] : cs[3];
        q += c == 0 ? cq[0] : c == 1 ? cq[1] : c == 2 ? cq[2] : cq[3];
        if (e < n) {
            os[cn + e] = (double)s;
            oq[cn + e] = (double)q;
        }
        // each channel's carry: its last lane in this step
        const int m = min(64, n - base);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < cn) {
                const int last = m - 1 - (((c0 + m - 1 - k) % cn) + cn) % cn;
                if (last >= 0) {
                    cs[k] = __shfl(s, last, 64);
                    cq[k] = __shfl(q, last, 64);
                }
            }
        }
        c0 = (c0 + 64) % cn;
    }
}

// pass 2: sum[y+1][e] = sum[y][e] + rowsum, down each column, in place; a
// thread per column of ONE of the two images (sum, sqsum: twice the threads
// of one per column pair)
__global__ void __launch_bounds__(kBlock) match_integral_cols_kernel(MatchLaunch M) {
    const int64_t step = (int64_t)(M.iw + 1) * M.cn;
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int img = blockIdx.y;
    if (g >= 2 * step) return;
    const int arr = g >= step ? 1 : 0;
    const int64_t e = g - arr * step;
    double* col = M.box + (int64_t)img * 2 * (M.ih + 1) * step + (int64_t)arr * (M.ih + 1) * step + e;
    // the same additions in the same order, kIntU rows at a time: their loads
    // are issued together before the dependent adds (one row per step waited
    // out a memory round trip per row of every column)
    constexpr int kIntU = 32;
    double a = 0;
    for (int y = 1; y <= M.ih; y += kIntU) {
        double va[kIntU];
#pragma unroll
        for (int u = 0; u < kIntU; ++u)
            if (y + u <= M.ih) va[u] = col[(int64_t)(y + u) * step];
#pragma unroll
        for (int u = 0; u < kIntU; ++u) {
            if (y + u <= M.ih) {
                a = a + va[u];
                col[(int64_t)(y + u) * step] = a;
            }
        }
    }
}

// one output: S_c / Q from the integral images (templmatch.cpp's p0 - p1 -
// p2 + p3), then its normalisation formula, in its operation order
__global__ void __launch_bounds__(kBlock) match_finish_kernel(MatchLaunch M) {
    const int x = blockIdx.x * kBlock + threadIdx.x;
    const int r = blockIdx.y, img = blockIdx.z;
    if (x >= M.rw) return;
    const int cn = M.cn;
    const int64_t step = (int64_t)(M.iw + 1) * cn;
    const double* sum = M.box + (int64_t)img * 2 * (M.ih + 1) * step;
    const double* sq = sum + (int64_t)(M.ih + 1) * step;
    const double* ts = M.tstats;  // tmean[4], templNorm, templSum2, all-ones flag
    float* out = reinterpret_cast<float*>(M.res + (int64_t)img * M.res_pitch + (int64_t)r * M.res_row) + x;
    const int method = M.method;
    if (ts[6] != 0.0) {  // CCOEFF_NORMED of a flat template
        *out = 1.f;
        return;
    }
    const int64_t i0 = (int64_t)r * step + (int64_t)x * cn;
    const int64_t dw = (int64_t)M.tw * cn, dh = (int64_t)M.th * step;
    const int numType = (method == VACV_TM_CCORR || method == VACV_TM_CCORR_NORMED)     ? 0
                        : (method == VACV_TM_CCOEFF || method == VACV_TM_CCOEFF_NORMED) ? 1
                                                                                        : 2;
    const bool isNormed = method == VACV_TM_CCORR_NORMED || method == VACV_TM_SQDIFF_NORMED ||
                          method == VACV_TM_CCOEFF_NORMED;
    const double invArea = M.inv_area;
    double num = (double)*out, t;
    double wndMean2 = 0, wndSum2 = 0;
    if (numType == 1) {
        for (int c = 0; c < cn; ++c) {
            t = sum[i0 + c] - sum[i0 + dw + c] - sum[i0 + dh + c] + sum[i0 + dh + dw + c];
            wndMean2 += t * t;
            num -= t * ts[c];
        }
        wndMean2 *= invArea;
    }
    if (isNormed || numType == 2) {
        for (int c = 0; c < cn; ++c) {
            t = sq[i0 + c] - sq[i0 + dw + c] - sq[i0 + dh + c] + sq[i0 + dh + dw + c];
            wndSum2 += t;
        }
        if (numType == 2) {
            num = wndSum2 - 2 * num + ts[5];
            num = num > 0. ? num : 0.;
        }
    }
    if (isNormed) {
        t = sqrt(wndSum2 - wndMean2 > 0. ? wndSum2 - wndMean2 : 0.) * ts[4];
        if (fabs(num) < t) num /= t;
        else if (fabs(num) < t * 1.125) num = num > 0 ? 1 : -1;
        else num = method != VACV_TM_SQDIFF_NORMED ? 0 : 1;
    }
    *out = (float)num;
}

// ---- u8 window statistics: exact integer box sums (round 6) -----------------
// For u8 every window sum is an integer: per channel S_c <= 255 tw th and Q_c
// <= 255^2 tw th, both < 2^32 for tw th <= 66,000 (host-checked), so they are
// kept in uint32 -- with wrap-around: the difference of two wrapped prefix
// sums is the exact window sum whenever that sum is < 2^32 -- and they equal
// the 4-term differences of the double integrals above exactly (every double
// there is an integer < 2^53).  Two passes of 4-byte sums instead of three
// over 8-byte integral images:
//  * match_vsum_u8_kernel: the vertical window sums V[r][e] = the sum of rows
//    r .. r + th - 1 of row element e (= x cn + c), and the same of squares;
//    a thread per element and chunk of kVsRows result rows, sliding down;
//  * match_finish_u8_kernel: a workgroup per result row stages V's row (both
//    arrays) in LDS, turns each channel into exclusive prefix sums, and each
//    result element takes S_c and Q_c as 2-term differences, then applies
//    match_finish_kernel's normalisation in the same operation order.
// Layout per image: [2][rh][iw * cn] uint32 (sums, then squares).
constexpr int kVsRows = 64;  // result rows per thread of the vertical pass
constexpr int kVsU = 8;      // rows whose loads are issued together

__global__ void __launch_bounds__(kBlock) match_vsum_u8_kernel(MatchLaunch M) {
    const int E = M.iw * M.cn;
    const int e = (int)blockIdx.x * kBlock + (int)threadIdx.x;
    const int img = blockIdx.z;
    if (e >= E) return;
    const int r0 = (int)blockIdx.y * kVsRows, r1 = min(r0 + kVsRows, M.rh);
    const unsigned char* col = M.img + (int64_t)img * M.img_pitch + e;
    const int64_t row = M.img_row;
    uint32_t s = 0, q = 0;
    for (int y = 0; y < M.th; y += kVsU) {  // the first window: rows r0 .. r0 + th - 1
        uint32_t v[kVsU];
#pragma unroll
        for (int u = 0; u < kVsU; ++u) v[u] = y + u < M.th ? (uint32_t)col[(int64_t)(r0 + y + u) * row] : 0u;
#pragma unroll
        for (int u = 0; u < kVsU; ++u) {
            s += v[u];
            q += v[u] * v[u];
        }
    }
    uint32_t* vs = reinterpret_cast<uint32_t*>(M.box) + (int64_t)img * 2 * M.rh * E + e;
    uint32_t* vq = vs + (int64_t)M.rh * E;
    for (int r = r0; r < r1; r += kVsU) {  // then slide: + row r + th, - row r
        uint32_t a[kVsU], b[kVsU];
#pragma unroll
        for (int u = 0; u < kVsU; ++u) {
            const bool in = r + u + 1 < r1;
            a[u] = in ? (uint32_t)col[(int64_t)(r + u + M.th) * row] : 0u;
            b[u] = in ? (uint32_t)col[(int64_t)(r + u) * row] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kVsU; ++u) {
            if (r + u < r1) {
                vs[(int64_t)(r + u) * E] = s;
                vq[(int64_t)(r + u) * E] = q;
            }
            s += a[u] - b[u];  // wraps when negative: the sum stays exact modulo 2^32
            q += a[u] * a[u] - b[u] * b[u];
        }
    }
}

// grid (rh, n); dynamic LDS 2 (iw + 1) cn uint32
__global__ void __launch_bounds__(kBlock) match_finish_u8_kernel(MatchLaunch M) {
    extern __shared__ __attribute__((aligned(16))) uint32_t pre[];
    const int cn = M.cn, E = M.iw * cn, PE = E + cn;  // prefix row: cn leading zeros
    const int r = blockIdx.x, img = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t* vs = reinterpret_cast<const uint32_t*>(M.box) + (int64_t)img * 2 * M.rh * E + (int64_t)r * E;
    const uint32_t* vq = vs + (int64_t)M.rh * E;
    uint32_t* ps = pre;
    uint32_t* pq = pre + PE;
    for (int i = tid; i < E; i += kBlock) {
        ps[cn + i] = vs[i];
        pq[cn + i] = vq[i];
    }
    if (tid < cn) ps[tid] = pq[tid] = 0u;
    __syncthreads();
    // thread t: pixels [t L, min((t + 1) L, iw)) -- a running sum per channel
    // (its elements are 15 dwords apart for L = 5, cn = 3: no bank conflicts)
    const int L = (M.iw + kBlock - 1) / kBlock;
    const int p0 = min(tid * L, M.iw), p1 = min(p0 + L, M.iw);
    uint32_t ts[4] = {0u, 0u, 0u, 0u}, tq[4] = {0u, 0u, 0u, 0u};
    for (int x = p0; x < p1; ++x) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < cn) {
                const int i = cn + x * cn + c;
                ts[c] += ps[i];
                tq[c] += pq[i];
                ps[i] = ts[c];
                pq[i] = tq[c];
            }
        }
    }
    // exclusive scan of the thread totals over the workgroup, per channel
    __shared__ uint32_t wtot[2][4][kBlock / 64];
    uint32_t xs[4], xq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t a = ts[c], b = tq[c];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t ua = (uint32_t)__shfl_up((int)a, o, 64), ub = (uint32_t)__shfl_up((int)b, o, 64);
            if (lane >= o) {
                a += ua;
                b += ub;
            }
        }
        xs[c] = a - ts[c];
        xq[c] = b - tq[c];
        if (lane == 63) {
            wtot[0][c][wave] = a;
            wtot[1][c][wave] = b;
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        for (int w = 0; w < wave; ++w) {
            xs[c] += wtot[0][c][w];
            xq[c] += wtot[1][c][w];
        }
    }
    for (int x = p0; x < p1; ++x) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < cn) {
                const int i = cn + x * cn + c;
                ps[i] += xs[c];
                pq[i] += xq[c];
            }
        }
    }
    __syncthreads();
    // the result row: match_finish_kernel's formula with the window sums
    const double* tsd = M.tstats;  // tmean[4], templNorm, templSum2, all-ones flag
    const int method = M.method;
    const int numType = (method == VACV_TM_CCORR || method == VACV_TM_CCORR_NORMED)     ? 0
                        : (method == VACV_TM_CCOEFF || method == VACV_TM_CCOEFF_NORMED) ? 1
                                                                                        : 2;
    const bool isNormed = method == VACV_TM_CCORR_NORMED || method == VACV_TM_SQDIFF_NORMED ||
                          method == VACV_TM_CCOEFF_NORMED;
    const double invArea = M.inv_area;
    const int dw = M.tw * cn;
    float* orow = reinterpret_cast<float*>(M.res + (int64_t)img * M.res_pitch + (int64_t)r * M.res_row);
    for (int x = tid; x < M.rw; x += kBlock) {
        float* out = orow + x;
        if (tsd[6] != 0.0) {  // CCOEFF_NORMED of a flat template
            *out = 1.f;
            continue;
        }
        const int i0 = x * cn;
        double num = (double)*out, t;
        double wndMean2 = 0, wndSum2 = 0;
        if (numType == 1) {
            for (int c = 0; c < cn; ++c) {
                t = (double)(ps[i0 + dw + c] - ps[i0 + c]);
                wndMean2 += t * t;
                num -= t * tsd[c];
            }
            wndMean2 *= invArea;
        }
        if (isNormed || numType == 2) {
            for (int c = 0; c < cn; ++c) {
                t = (double)(pq[i0 + dw + c] - pq[i0 + c]);
                wndSum2 += t;
            }
            if (numType == 2) {
                num = wndSum2 - 2 * num + tsd[5];
                num = num > 0. ? num : 0.;
            }
        }
        if (isNormed) {
            t = sqrt(wndSum2 - wndMean2 > 0. ? wndSum2 - wndMean2 : 0.) * tsd[4];
            if (fabs(num) < t) num /= t;
            else if (fabs(num) < t * 1.125) num = num > 0 ? 1 : -1;
            else num = method != VACV_TM_SQDIFF_NORMED ? 0 : 1;
        }
        *out = (float)num;
    }
}

// the template's mean / population stddev per channel (one workgroup per
// image's template -- templates are shared: blockIdx.x = 0 only), then the
// method's constants as templmatch.cpp derives them
template <typename T>
__global__ void __launch_bounds__(kBlock) match_tstats_kernel(MatchLaunch M) {
    __shared__ double red[2][4][kBlock];
    const int cn = M.cn, n = M.tw * M.th;
    double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += kBlock) {
        const int yy = i / M.tw, xx = i - yy * M.tw;
        const T* tr = reinterpret_cast<const T*>(M.tpl + (int64_t)yy * M.tpl_row) + xx * cn;
        for (int c = 0; c < cn; ++c) {
            const double v = (double)tr[c];
            s[c] += v;
            q[c] += v * v;
        }
    }
    for (int c = 0; c < 4; ++c) {
        red[0][c][threadIdx.x] = s[c];
        red[1][c][threadIdx.x] = q[c];
    }
    __syncthreads();
    for (int st = kBlock / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st)
            for (int c = 0; c < 4; ++c) {
                red[0][c][threadIdx.x] += red[0][c][threadIdx.x + st];
                red[1][c][threadIdx.x] += red[1][c][threadIdx.x + st];
            }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    double tm[4] = {0, 0, 0, 0}, td[4] = {0, 0, 0, 0};
    for (int c = 0; c < cn; ++c) {  // meanStdDev: population
        tm[c] = red[0][c][0] / n;
        const double var = red[1][c][0] / n - tm[c] * tm[c];
        td[c] = sqrt(var > 0 ? var : 0);
    }
    const int method = M.method;
    const double invArea = M.inv_area;
    double templNorm = 0, templSum2 = 0, ones = 0;
    double tmean[4] = {tm[0], tm[1], tm[2], tm[3]};
    if (method != VACV_TM_CCOEFF) {
        templNorm = td[0] * td[0] + td[1] * td[1] + td[2] * td[2] + td[3] * td[3];
        if (templNorm < 2.220446049250313e-16 && method == VACV_TM_CCOEFF_NORMED) ones = 1;
        templSum2 = templNorm + tm[0] * tm[0] + tm[1] * tm[1] + tm[2] * tm[2] + tm[3] * tm[3];
        const bool ccoeff = method == VACV_TM_CCOEFF || method == VACV_TM_CCOEFF_NORMED;
        if (!ccoeff) {
            tmean[0] = tmean[1] = tmean[2] = tmean[3] = 0;
            templNorm = templSum2;
        }
        templSum2 /= invArea;
        templNorm = sqrt(templNorm);
        templNorm /= sqrt(invArea);
    }
    double* o = M.tstats;
    for (int c = 0; c < 4; ++c) o[c] = tmean[c];
    o[4] = templNorm;
    o[5] = templSum2;
    o[6] = ones;
}

// ---- minMaxIdx ---------------------------------------------------------------

struct MinMax {
    double mn, mx;
    long long imn, imx;  // linear indices, -1 = none
};

__device__ __forceinline__ void mm_merge(MinMax& a, const MinMax& b) {
    // first occurrence wins ties: the smaller index
    if (b.imn >= 0 && (a.imn < 0 || b.mn < a.mn || (b.mn == a.mn && b.imn < a.imn))) {
        a.mn = b.mn;
        a.imn = b.imn;
    }
    if (b.imx >= 0 && (a.imx < 0 || b.mx > a.mx || (b.mx == a.mx && b.imx < a.imx))) {
        a.mx = b.mx;
        a.imx = b.imx;
    }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) min_max_kernel(MinMaxLaunch L, MinMax* part) {
    __shared__ MinMax red[kBlock];
    const long long n = (long long)L.w * L.h;
    MinMax m = {0, 0, -1, -1};
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock) {
        const int y = (int)(i / L.w), x = (int)(i - (long long)y * L.w);
        if (L.mask && !L.mask[(int64_t)y * L.mask_row + x]) continue;
        const double v = (double)reinterpret_cast<const T*>(L.src + (int64_t)y * L.row)[x];
        if (v != v) continue;
        const MinMax b = {v, v, i, i};
        mm_merge(m, b);
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int st = kBlock / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) mm_merge(red[threadIdx.x], red[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(kBlock) min_max_final_kernel(MinMaxLaunch L, const MinMax* part, int parts) {
    __shared__ MinMax red[kBlock];
    MinMax m = {0, 0, -1, -1};
    for (int i = threadIdx.x; i < parts; i += kBlock) mm_merge(m, part[i]);
    red[threadIdx.x] = m;
    __syncthreads();
    for (int st = kBlock / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) mm_merge(red[threadIdx.x], red[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const MinMax r = red[0];
    L.out_val[0] = r.imn >= 0 ? r.mn : 0.0;
    L.out_val[1] = r.imx >= 0 ? r.mx : 0.0;
    L.out_idx[0] = r.imn >= 0 ? (int)(r.imn / L.w) : -1;
    L.out_idx[1] = r.imn >= 0 ? (int)(r.imn % L.w) : -1;
    L.out_idx[2] = r.imx >= 0 ? (int)(r.imx / L.w) : -1;
    L.out_idx[3] = r.imx >= 0 ? (int)(r.imx % L.w) : -1;
}

}  // namespace
size_t match_lds_bytes(int tw, int th, int cn, int esize);
namespace {

// ---- u8 correlation on the matrix cores ------------------------------------
// For template row yy the correlation of an output tile is a GEMM: with
// a' = image - 128 (i8) and the template split into nibbles b = 16*b_hi +
// b_lo (both in [0, 15], i8), D[r][x] = sum_k a'(r + yy, cn*x + k) * b(yy, k)
// = sum_kappa A[r][kappa] * B[kappa][x] where A is the image block (rows r,
// columns cn*x0 + kappa) and B the Toeplitz matrix B[kappa][x] = b(yy,
// kappa - cn*x) (0 outside [0, K)).  Then sum a*b = 16*D_hi + D_lo + 128*T, T
// = the template's byte sum.  Each accumulator is exact in int32: |D_hi|,
// |D_lo| <= 128 * 15 * K*h < 2^31 for K*h <= 2^19 (match_mfma_plan's guard);
// the recombination, up to 255^2 * K*h, is done in int64.
// v_mfma_i32_32x32x32_i8, a wave owns 32 x 32 outputs; B
// depends only on (yy, kappa - cn*x), so its fragments are built once per
// launch (match_bfrag_kernel) and read from L2 by every wave.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// bf[((part * th + yy) * KB + kb) * 64 + lane]: lane (j = lane & 31, h =
// lane >> 5) element e is B[kappa = 32 kb + 16 h + e][j] of nibble part
__global__ void match_bfrag_kernel(MatchLaunch M, int KB, uint4* bf, int* tsum) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int K = M.tw * M.cn;
    if (blockIdx.x == 0) {  // the template's byte sum (one workgroup, fixed order)
        __shared__ int part_sum[256];
        int acc = 0;
        for (int i = threadIdx.x; i < K * M.th; i += blockDim.x) {
            const int yy = i / K, k = i - yy * K;
            acc += M.tpl[(int64_t)yy * M.tpl_row + k];
        }
        part_sum[threadIdx.x] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            int sum = 0;
            for (int i = 0; i < (int)blockDim.x; ++i) sum += part_sum[i];
            *tsum = sum;
        }
    }
    if (t >= 2 * M.th * KB * 64) return;
    const int lane = t & 63;
    int rest = t >> 6;
    const int kb = rest % KB;
    rest /= KB;
    const int yy = rest % M.th, part = rest / M.th;
    const int j = lane & 31, h = lane >> 5;
    const unsigned char* trow = M.tpl + (int64_t)yy * M.tpl_row;
    uint32_t d[4] = {0u, 0u, 0u, 0u};
    for (int e = 0; e < 16; ++e) {
        const int tt = kb * 32 + 16 * h + e - M.cn * j;
        uint32_t v = 0u;
        if (tt >= 0 && tt < K) {
            const uint32_t b = trow[tt];
            v = part == 0 ? (b >> 4) : (b & 15u);
        }
        d[e >> 2] |= v << (8 * (e & 3));
    }
    bf[t] = make_uint4(d[0], d[1], d[2], d[3]);
}

constexpr int kMatchPF = 4;  // match_corr_mfma_kernel: (yy, kb) steps whose operands are in flight

// workgroup: 64 output rows x 64 output columns of one image; wave w: rows
// 32 (w & 1) .., columns 32 (w >> 1) ..; the image block (rows r0 .. r0 + 63
// + th - 1, bytes cn*x0 .. + stride) staged in LDS as i8 (XOR 0x80)
template <int CN>
__global__ void __launch_bounds__(kBlock) match_corr_mfma_kernel(MatchLaunch M, int KB, int stride,
                                                                 const uint4* __restrict__ bf, const int* tsum) {
    extern __shared__ __attribute__((aligned(16))) unsigned char blk[];
    const int x0 = blockIdx.x * 64, r0 = blockIdx.y * 64, img = blockIdx.z;
    const int rows = 63 + M.th;
    const int chunks = stride >> 4;
    {
        const unsigned char* base = M.img + (int64_t)img * M.img_pitch;
        // the image's readable bytes from row r0 on: loads past them read 0
        const int64_t avail = (int64_t)(M.ih - r0) * M.img_row;
        const Rsrc rs = make_rsrc(base + (int64_t)r0 * M.img_row, avail - (M.img_row - (int64_t)M.iw * CN));
        const uint32_t magic = (uint32_t)((0x100000000ull + (uint64_t)chunks - 1) / (uint64_t)chunks);
        for (int i = threadIdx.x; i < rows * chunks; i += kBlock) {
            const uint32_t rr = chunks == 1 ? (uint32_t)i : __umulhi((uint32_t)i, magic);
            const uint32_t c = (uint32_t)i - rr * (uint32_t)chunks;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if ((int)rr + r0 < M.ih) {
                const uint32_t o = rr * (uint32_t)M.img_row + (uint32_t)(CN * x0) + 16u * c + rs.delta;
                const uint32_t lim = (uint32_t)(avail - (M.img_row - (int64_t)M.iw * CN)) + rs.delta;
                if (o + 16u <= lim) {
                    v = load16(rs, o);
                } else {  // straddles the image's end: a 16-byte load would read as zeros
                    uint32_t d[4] = {0u, 0u, 0u, 0u};
#pragma unroll 1
                    for (uint32_t e = 0; e < 16u; ++e)
                        if (o + e < lim)
                            d[e >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs.r, (int)(o + e), 0, 0) << (8 * (e & 3));
                    v = make_uint4(d[0], d[1], d[2], d[3]);
                }
            }
            v.x ^= 0x80808080u; v.y ^= 0x80808080u; v.z ^= 0x80808080u; v.w ^= 0x80808080u;
            *reinterpret_cast<uint4*>(blk + (int)rr * stride + 16 * (int)c) = v;
        }
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int mi = wave & 1, ni = wave >> 1;
    const int i = lane & 31, h = lane >> 5;
    const unsigned char* abase = blk + (mi * 32 + i) * stride + ni * CN * 32 + 16 * h;
    const int per_part = M.th * KB * 64;
    v16i acc_hi = {}, acc_lo = {};
    // The (yy, kb) steps flattened and software-pipelined (round 5): the B
    // fragments come from L2 (shared by every workgroup), so each step's
    // loads are issued kMatchPF steps ahead -- the loop that loaded them just
    // before its two MFMAs waited out an L2 round trip per step
    // (s_waitcnt vmcnt(0) between the loads and the MFMAs).
    constexpr int PF = kMatchPF;
    const int nit = M.th * KB;
    v4i pa[2][PF];
    uint4 ph[2][PF], pl[2][PF];
    int fy = 0, fk = 0;  // the next step to fetch: (yy, kb), held at the last step once past it
    auto fetch = [&](v4i& a, uint4& h, uint4& l) {
        a = *reinterpret_cast<const v4i*>(abase + fy * stride + 32 * fk);
        const uint4* bh = bf + ((int64_t)fy * KB + fk) * 64 + lane;
        h = bh[0];
        l = bh[per_part];
        if (++fk == KB) {
            if (fy + 1 < M.th) { fk = 0; ++fy; }
            else fk = KB - 1;
        }
    };
    auto step = [&](const v4i& a, const uint4& h, const uint4& l) {
        const v4i b_hi = {(int)h.x, (int)h.y, (int)h.z, (int)h.w};
        const v4i b_lo = {(int)l.x, (int)l.y, (int)l.z, (int)l.w};
        acc_hi = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b_hi, acc_hi, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b_lo, acc_lo, 0, 0, 0);
    };
    // two register sets of PF steps: the next set's operands are fetched
    // before this set's MFMAs, so they are in flight during them (a single
    // set was refetched only after its own MFMAs).  Past the last step a
    // fetch reads the last step again, so every group issues all its loads
    // and the compiler's waits count them exactly.
#pragma unroll
    for (int u = 0; u < PF; ++u) fetch(pa[0][u], ph[0][u], pl[0][u]);
    int it = 0;
    for (; it + 2 * PF <= nit; it += 2 * PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) fetch(pa[1][u], ph[1][u], pl[1][u]);
#pragma unroll
        for (int u = 0; u < PF; ++u) step(pa[0][u], ph[0][u], pl[0][u]);
#pragma unroll
        for (int u = 0; u < PF; ++u) fetch(pa[0][u], ph[0][u], pl[0][u]);
#pragma unroll
        for (int u = 0; u < PF; ++u) step(pa[1][u], ph[1][u], pl[1][u]);
    }
    // the remainder (< 2 PF steps, uniform): set 0 holds steps it .. it + PF - 1
#pragma unroll
    for (int u = 0; u < PF; ++u) fetch(pa[1][u], ph[1][u], pl[1][u]);
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (it + u < nit) step(pa[0][u], ph[0][u], pl[0][u]);
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (it + PF + u < nit) step(pa[1][u], ph[1][u], pl[1][u]);
    const int64_t t128 = 128 * (int64_t)*tsum;  // T <= 255 * K*h: past int32 once multiplied
    const int x = x0 + ni * 32 + i;
    if (x >= M.rw) return;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int r = r0 + mi * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (r >= M.rh) continue;
        // the recombined sum is up to 255^2 * K * th: int64 (each accumulator stays in int32, see above)
        const int64_t d = 16 * (int64_t)acc_hi[reg] + (int64_t)acc_lo[reg] + t128;
        reinterpret_cast<float*>(M.res + (int64_t)img * M.res_pitch + (int64_t)r * M.res_row)[x] = (float)(double)d;
    }
}

template <int CN>
hipError_t launch_corr_cn(const MatchLaunch& M, hipStream_t s) {
    const dim3 grid((M.rw + kTileX - 1) / kTileX, (M.rh + 3) / 4, M.n);
    int KB = 0, stride = 0;
    if (M.esize == 1 && M.bfrag && match_mfma_plan(M.tw, M.th, CN, KB, stride)) {
        uint4* bf = static_cast<uint4*>(M.bfrag);
        int* tsum = reinterpret_cast<int*>(bf + 2 * (size_t)M.th * KB * 64);
        const int nfrag = 2 * M.th * KB * 64;
        hipLaunchKernelGGL(match_bfrag_kernel, dim3((nfrag + kBlock - 1) / kBlock), dim3(kBlock), 0, s, M, KB, bf, tsum);
        const dim3 g((M.rw + 63) / 64, (M.rh + 63) / 64, M.n);
        const size_t lds = (size_t)(63 + M.th) * stride;
        hipLaunchKernelGGL((match_corr_mfma_kernel<CN>), g, dim3(kBlock), lds, s, M, KB, stride, bf, tsum);
        return hipGetLastError();
    }
    if (M.esize == 1) {
        const size_t lds = match_lds_bytes(M.tw, M.th, CN, 1);
        hipLaunchKernelGGL((match_corr_u8_kernel<CN>), grid, dim3(kBlock), lds, s, M);
    } else {
        const size_t lds = match_lds_bytes(M.tw, M.th, CN, 4);
        hipLaunchKernelGGL((match_corr_f32_kernel<CN>), grid, dim3(kBlock), lds, s, M);
    }
    return hipGetLastError();
}

}  // namespace

// The MFMA path's K blocks per template row and LDS row stride, or false when
// its image block does not fit 64 KiB or the int32 sums could overflow.
bool match_mfma_plan(int tw, int th, int cn, int& KB, int& stride) {
    if (tune(VACV_TUNE_MATCH_KERNEL) == 0) return false;
    const int K = tw * cn;
    KB = (cn * 31 + K + 31) / 32;
    stride = (cn * 32 + KB * 32 + 15) / 16 * 16;
    return (size_t)(63 + th) * stride <= 64 * 1024 && (int64_t)K * th <= (1 << 19);
}

size_t match_bfrag_bytes(int tw, int th, int cn) {
    int KB = 0, stride = 0;
    if (!match_mfma_plan(tw, th, cn, KB, stride)) return 0;
    return 2 * (size_t)th * KB * 64 * 16 + 256;
}

size_t match_lds_bytes(int tw, int th, int cn, int esize) {
    if (esize == 1) {
        const size_t K4 = ((size_t)tw * cn + 3) / 4, span4 = 64 * (size_t)cn + K4 + (3 * cn) / 4 + 2 + 1;
        return ((size_t)th * K4 + 4 * span4) * 4;
    }
    return ((size_t)th * tw * cn + 4 * (size_t)(kTileX + tw - 1) * cn) * 4;
}

hipError_t launch_match_template(const MatchLaunch& M, hipStream_t s) {
    hipError_t e;
    switch (M.cn) {
        case 1: e = launch_corr_cn<1>(M, s); break;
        case 2: e = launch_corr_cn<2>(M, s); break;
        case 3: e = launch_corr_cn<3>(M, s); break;
        case 4: e = launch_corr_cn<4>(M, s); break;
        default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess || M.method == VACV_TM_CCORR) return e;
    if (M.esize == 1) hipLaunchKernelGGL(match_tstats_kernel<uint8_t>, dim3(1), dim3(kBlock), 0, s, M);
    else hipLaunchKernelGGL(match_tstats_kernel<float>, dim3(1), dim3(kBlock), 0, s, M);
    if (M.esize == 1 && (int64_t)M.tw * M.th <= 66000 && 2 * (int64_t)(M.iw + 1) * M.cn * 4 <= 64 * 1024) {
        // u8: exact integer box sums (the same values as the integrals)
        const int E = M.iw * M.cn;
        const dim3 gv((E + kBlock - 1) / kBlock, (M.rh + kVsRows - 1) / kVsRows, M.n);
        hipLaunchKernelGGL(match_vsum_u8_kernel, gv, dim3(kBlock), 0, s, M);
        hipLaunchKernelGGL(match_finish_u8_kernel, dim3(M.rh, M.n), dim3(kBlock), (size_t)(2 * (E + M.cn) * 4), s, M);
        return hipGetLastError();
    }
    const dim3 gr((M.ih * M.cn + kBlock - 1) / kBlock, M.n);
    if (M.esize == 1 && M.iw <= 33000) {
        const dim3 gw((M.ih + kBlock / 64 - 1) / (kBlock / 64), M.n);
        hipLaunchKernelGGL(match_integral_rows_u8_kernel, gw, dim3(kBlock), 0, s, M);
    } else if (M.esize == 1) {
        hipLaunchKernelGGL(match_integral_rows_kernel<uint8_t>, gr, dim3(kBlock), 0, s, M);
    } else {
        hipLaunchKernelGGL(match_integral_rows_kernel<float>, gr, dim3(kBlock), 0, s, M);
    }
    const dim3 gc((2 * (M.iw + 1) * M.cn + kBlock - 1) / kBlock, M.n);
    hipLaunchKernelGGL(match_integral_cols_kernel, gc, dim3(kBlock), 0, s, M);
    const dim3 gf((M.rw + kBlock - 1) / kBlock, M.rh, M.n);
    hipLaunchKernelGGL(match_finish_kernel, gf, dim3(kBlock), 0, s, M);
    return hipGetLastError();
}

size_t min_max_workspace_bytes() { return 1024 * sizeof(MinMax); }

hipError_t launch_min_max(const MinMaxLaunch& L, void* ws, hipStream_t s) {
    const long long n = (long long)L.w * L.h;
    const int parts = (int)std::min<long long>(1024, std::max<long long>(1, (n + kBlock * 16 - 1) / (kBlock * 16)));
    MinMax* part = static_cast<MinMax*>(ws);
    if (L.esize == 1) hipLaunchKernelGGL(min_max_kernel<uint8_t>, dim3(parts), dim3(kBlock), 0, s, L, part);
    else hipLaunchKernelGGL(min_max_kernel<float>, dim3(parts), dim3(kBlock), 0, s, L, part);
    hipLaunchKernelGGL(min_max_final_kernel, dim3(1), dim3(kBlock), 0, s, L, part, parts);
    return hipGetLastError();
}

}  // namespace vacv
