// k_cubic_direct.hip -- Keys cubic resize (A = -0.75) of u8 images to fp32
// (optionally normalised) as per-pixel gathers: no LDS staging of source
// rows, no planner tables, no barriers.  The u8 -> fp32 conversion the
// reference requires before its cubic (resize.cpp:89-98, App. C) is fused.
//
// Reference arithmetic (as resize_kernel<kCubic>, k_resize.hip):
//   taps   cubic_tap() = resize_naive.cpp:130-185 (coefficients, replicate
//          folding), shared host/device code
//   rows   h_r = S[-1]*a0 + S[0]*a1 + S[1]*a2 + S[2]*a3  (resize_naive.cpp:325-328)
//   value  h_0*b0 + h_1*b1 + h_2*b2 + h_3*b3             (resize_naive.cpp:349-351)
//   all fp32, left to right, no contraction (-ffp-contract=off).
//
// Shape.  Output pixels of one plane are numbered row-major; a wave owns 128
// consecutive ones and lane l samples pixels p0 + 64j + l (j < 2), so one
// gather instruction reads the taps of 64 consecutive output pixels.  Per
// pixel and tap row ONE dword-aligned 16-byte buffer load brings the four
// horizontal taps of all CC <= 3 channels (4*CC + 3 <= 16 bytes).  The
// vertical taps of the (at most two) output rows a wave touches are computed
// once per wave.  Results are re-assembled in LDS and leave as 16-byte
// non-temporal stores.
#pragma clang fp contract(off)

#include <cstdlib>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kPxl = 2;               // pixels per lane
constexpr int kWavePx = 64 * kPxl;    // 128 output pixels per wave

// 32 tap dwords per lane plus coefficients: ~70-90 VGPRs for CC >= 2 (64
// spills; 80 still spills the normalised 3-channel kernel)
constexpr int cubic_waves(int cc, int out) { return cc == 1 ? 8 : (cc == 3 && out == kOutNorm ? 5 : 6); }

// SUMS: the statistics half of cfg5 fused (normalize_naive.cpp:7-72 on the
// resized image, here as fixed-order sums for the global mean_stddev): each
// lane adds its (at most 2) pixels' values and squares per channel in fp32
// (fp32 only over <= 2 pixels), the wave reduces those in fp64 in
// a fixed shuffle order, the workgroup adds its 4 waves in order (one LDS
// exchange, one barrier), and thread v stores value v of the workgroup's
// (Sum x, Sum x^2) as an fp64 partial; group_sums_kernel sums those in a fixed
// order (deterministic, run to run).  (Reducing across workgroups inside the
// launch -- the last wave of each image, found by an agent-scope
// release/acquire counter -- took 2.2 ms: an agent-scope release per wave
// writes back the L2.)
template <int CC, int OUT, bool SUMS>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(cubic_waves(CC, OUT))))
cubic_direct_kernel(ResizeLaunch L, int blocks_per_plane) {
    __shared__ __attribute__((aligned(16))) float xch[4][kWavePx * CC];

    __shared__ double wsum[SUMS ? 4 : 1][2 * CC];
    const int pidx = blockIdx.x / blocks_per_plane;  // image * planes + plane
    const int blk = blockIdx.x - pidx * blocks_per_plane;
    const int W = L.dst.w;
    const int P = W * L.dst.h;
    const int p0 = (blk * 4 + (int)threadIdx.y) * kWavePx;
    if (p0 >= P) {  // whole wave
        if (SUMS) {
            // no pixels: zero sums, then the workgroup's barrier below
            if (threadIdx.x < 2 * CC) wsum[threadIdx.y][threadIdx.x] = 0.0;
            __syncthreads();
            if (threadIdx.y == 0 && threadIdx.x < 2 * CC) {
                const int64_t groups = (int64_t)L.n * blocks_per_plane;
                double a = 0.0;
#pragma unroll
                for (int w = 0; w < 4; ++w) a += wsum[w][threadIdx.x];
                L.sum_partials[threadIdx.x * groups + blockIdx.x] = a;
            }
        }
        return;
    }
    const int npx = min(kWavePx, P - p0);
    const int lane = threadIdx.x;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp = (uint32_t)L.src.row_pitch;  // plane < 2^31 bytes (kMaxPlaneBytes)

    const int y_first = p0 / W;  // wave-uniform
    const int x_first = p0 - y_first * W;
    const bool wide = W >= kWavePx;
    const CubicTap ty0 = cubic_tap(y_first, L.src.h, L.scale_yd);
    const CubicTap ty1 = cubic_tap(min(y_first + 1, L.dst.h - 1), L.src.h, L.scale_yd);

    // ---- gathers: the 16 bytes at (row ty.i - 1 + r, column tx.i - 1) ------
    uint32_t ch[kPxl][4][4];
#pragma unroll
    for (int j = 0; j < kPxl; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ch[j][r][0] = ch[j][r][1] = ch[j][r][2] = ch[j][r][3] = 0u;
        if (j * 64 + lane >= npx) continue;
        const int d = x_first + j * 64 + lane;
        const int dy = wide ? (d >= W ? 1 : 0) : d / W;
        const int x = wide ? (dy ? d - W : d) : d - dy * W;
        const CubicTap tyn = wide ? (dy ? ty1 : ty0) : cubic_tap(y_first + dy, L.src.h, L.scale_yd);
        const int txi = cubic_tap(x, L.src.w, L.scale_xd).i;
        const uint32_t o0 = (uint32_t)(tyn.i - 1) * rp + (uint32_t)((txi - 1) * CC) + srs.delta;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t a4 = (o0 + (uint32_t)r * rp) & ~3u;
            // a tap row of weight 0 (every 7th output row of 1440 -> 224 has
            // three: f = 0 exactly) is not read.  Its term is h * 0 in the
            // reference and 0 * 0 here: both zeros, and a zero addend leaves
            // the sum's bits alone (x + 0 = x; an all-zero sum is +0 either
            // way, since the row of weight 1 contributes +0).
            if (tyn.c[r] == 0.f) continue;
            if (a4 + 16u <= slimit) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)a4, 0, VACV_LOAD_AUX);
                ch[j][r][0] = v[0];
                ch[j][r][1] = v[1];
                ch[j][r][2] = v[2];
                ch[j][r][3] = v[3];
            } else {  // the plane's last bytes: an overhanging load would read zeros
                const unsigned char* b = sp + ((int64_t)a4 - (int64_t)srs.delta);
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (a4 + (uint32_t)e < slimit) ch[j][r][e >> 2] |= (uint32_t)b[e] << (8 * (e & 3));
            }
        }
    }

    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }

    // ---- blend into the wave's LDS buffer (coefficients recomputed here so
    // they do not hold registers across the loads) ------------------------------
    float* xo = xch[threadIdx.y];
#pragma unroll
    for (int j = 0; j < kPxl; ++j) {
        if (j * 64 + lane >= npx) continue;
        const int d = x_first + j * 64 + lane;
        const int dy = wide ? (d >= W ? 1 : 0) : d / W;
        const int x = wide ? (dy ? d - W : d) : d - dy * W;
        CubicTap ty;
        if (wide) {
            ty.i = dy ? ty1.i : ty0.i;
#pragma unroll
            for (int q = 0; q < 4; ++q) ty.c[q] = dy ? ty1.c[q] : ty0.c[q];
        } else {
            ty = cubic_tap(y_first + dy, L.src.h, L.scale_yd);
        }
        const CubicTap tx = cubic_tap(x, L.src.w, L.scale_xd);
        const uint32_t o0 = (uint32_t)(ty.i - 1) * rp + (uint32_t)((tx.i - 1) * CC) + srs.delta;
        float h[4][CC];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t sh = (o0 + (uint32_t)r * rp) & 3u;
            const uint32_t w0 = __builtin_amdgcn_alignbyte(ch[j][r][1], ch[j][r][0], sh);
            const uint32_t w1 = __builtin_amdgcn_alignbyte(ch[j][r][2], ch[j][r][1], sh);
            const uint32_t w2 = __builtin_amdgcn_alignbyte(ch[j][r][3], ch[j][r][2], sh);
            const uint32_t wv[3] = {w0, w1, w2};
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                float s[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int e = m * CC + k;  // byte of the 4*CC tap bytes
                    s[m] = (float)((wv[e >> 2] >> (8 * (e & 3))) & 0xFFu);
                }
                // resize_naive.cpp:325-328
                h[r][k] = s[0] * tx.c[0] + s[1] * tx.c[1] + s[2] * tx.c[2] + s[3] * tx.c[3];
            }
        }
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            // resize_naive.cpp:349-351
            float v = h[0][k] * ty.c[0] + h[1][k] * ty.c[1] + h[2][k] * ty.c[2] + h[3][k] * ty.c[3];
            if (OUT == kOutNorm) v = normalize_f(cn[k], v);
            xo[(j * 64 + lane) * CC + k] = v;
        }
    }
    if (SUMS) {
        // this lane's own values back from LDS (summed in the blend loop they
        // held 6 registers across it: a spill at the 80-VGPR cap)
        float s1[CC], s2[CC];
#pragma unroll
        for (int k = 0; k < CC; ++k) s1[k] = s2[k] = 0.f;
#pragma unroll
        for (int j = 0; j < kPxl; ++j) {
            if (j * 64 + lane >= npx) continue;
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                const float v = xo[(j * 64 + lane) * CC + k];
                s1[k] += v;
                s2[k] += v * v;
            }
        }
        double d[2 * CC];
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            d[2 * k] = (double)s1[k];
            d[2 * k + 1] = (double)s2[k];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int v = 0; v < 2 * CC; ++v) d[v] += __shfl_xor(d[v], o, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int v = 0; v < 2 * CC; ++v) wsum[threadIdx.y][v] = d[v];
        }
        __syncthreads();
        if (threadIdx.y == 0 && lane < 2 * CC) {
            // value-major [CC][2][image][workgroup]: a value's partials are one
            // contiguous run for group_sums_kernel
            const int64_t groups = (int64_t)L.n * blocks_per_plane;
            double a = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) a += wsum[w][lane];
            L.sum_partials[lane * groups + blockIdx.x] = a;
        }
    }
    // ---- LDS -> HBM: dense byte b of the plane's output lives at row
    // b / out_row, column byte b % out_row --------------------------------------
    // Lanes read bytes other lanes of the wave wrote to xch: order those
    // writes before the reads (the SUMS instance's __syncthreads already did).
    if (!SUMS) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const uint32_t out_row = (uint32_t)W * CC * 4u;
    const uint32_t rowp = (uint32_t)L.dst.row_pitch;
    const bool dense = L.dst.row_pitch == (int64_t)out_row;
    const bool chunked = (reinterpret_cast<uintptr_t>(dp) & 15) == 0 && (L.dst.row_pitch & 15) == 0 &&
                         (dense || (out_row & 15) == 0);  // 16-byte chunks never straddle rows
    const uint32_t vbytes = (uint32_t)npx * CC * 4u;
    const uint32_t b0 = (uint32_t)p0 * CC * 4u;
    const unsigned char* xs = reinterpret_cast<const unsigned char*>(xch[threadIdx.y]);
    if (chunked) {
        for (uint32_t c = lane; c * 16 < vbytes; c += 64) {
            const uint32_t b = b0 + 16 * c;
            uint32_t off = b;
            if (!dense) {
                const uint32_t r = b / out_row;
                off = r * rowp + (b - r * out_row);
            }
            if (c * 16 + 16 <= vbytes) {
                __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(xs + 16 * c),
                                            reinterpret_cast<u32x4*>(dp + off));
            } else {
                for (uint32_t e = c * 16; e < vbytes; ++e) dp[off + (e - c * 16)] = xs[e];
            }
        }
    } else {
        for (uint32_t e = lane; e < vbytes; e += 64) {
            const uint32_t b = b0 + e;
            const uint32_t r = b / out_row;
            dp[(int64_t)r * rowp + (b - r * out_row)] = xs[e];
        }
    }
}

// ---- the column kernel's statistics: fixed-point integer sums -----------------
// Each workgroup rounds its fp64 (Sum x, Sum x^2) to integers in units of
// 2^-q1 / 2^-q2 and adds them to its image's int64 accumulators with
// fire-and-forget agent-scope atomics: integer addition is associative, so
// the totals are the same bits whatever the order the workgroups finish in
// (deterministic without a fixed reduction order, no partials buffer, no
// waiting).  q1 / q2 leave 2 bits of headroom over the largest possible total
// (|v| < 2^10: a u8 source through Keys cubic weights, fixed_shifts()), so the
// integers never overflow; each workgroup's rounding is <= 2^-(q + 1), e.g.
// cfg5: q1 = 29, q2 = 19, i.e. <= 7e-6 and <= 7e-3 absolute over the batch's
// 7,168 workgroups on totals of ~1e9 and ~1e11.  fixed_sums_kernel (one
// workgroup) then converts, derives mean / stddev and zeroes the accumulators.
// (Finishing inside the cubic launch instead -- write-through partials, an
// arrival counter, the last workgroup reducing -- measured +10 us of kernel
// time: every workgroup's wave 0 waited out a store drain and an atomic's
// round trip.)
__device__ __forceinline__ void acc_add(int64_t* p, double v, int q) {
    const long long x = __double2ll_rn(ldexp(v, q));
    __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned long long*)p, (unsigned long long)x,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// cubic_cols_kernel: the same arithmetic with COLUMN-stationary lanes (as
// resize_cols_kernel, k_resize_direct.hip).  A wave owns 64 output columns x
// kCcRows output rows of one plane; lane l keeps column x0 + l, so its
// horizontal tap (index and 4 coefficients) is computed once instead of per
// pixel, and lanes 0..kCcRows-1 compute the rows' vertical taps in parallel
// (broadcast by readlane: scalar weights, a scalar skip of zero-weight rows).
// Per pixel and tap row one dword-aligned 16-byte load, as above; a load
// instruction reads one contiguous run of a source row.  The 4 waves of a
// workgroup are the column blocks of the same rows, in order (224 columns: one
// workgroup = 4 full output rows); workgroups never straddle planes, so the
// SUMS partials stay per workgroup and per image.  SUMS adds each value and
// its square in fp64 per lane (exact squares), then as the kernel above.
constexpr int kCcRows = 4;  // output rows per wave task
constexpr int cubic_cols_waves(int cc) { return cc == 1 ? 8 : 5; }
template <int CC, int OUT, bool SUMS>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(cubic_cols_waves(CC))))
cubic_cols_kernel(ResizeLaunch L, int col_blocks, int plane_tasks, int blocks_per_plane) {
    constexpr int kRowB = 64 * CC * 4;  // LDS bytes of one block row
    __shared__ __attribute__((aligned(16))) float xch[4][kCcRows * 64 * CC];
    __shared__ double wsum[SUMS ? 4 : 1][2 * CC];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int pidx = (int)blockIdx.x / blocks_per_plane;  // image * planes + plane
    const int t = ((int)blockIdx.x - pidx * blocks_per_plane) * 4 + wave;
    double d[2 * CC];
#pragma unroll
    for (int v = 0; v < 2 * CC; ++v) d[v] = 0.0;
    if (t < plane_tasks) {  // uniform
        const int rg = t / col_blocks, cb = t - rg * col_blocks;
        const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
        const int W = L.dst.w, H = L.dst.h;
        const int x0 = cb * 64, y0 = rg * kCcRows;
        const int ncol = min(64, W - x0), nrow = min(kCcRows, H - y0);  // uniform
        const bool col_ok = lane < ncol;
        const int x = col_ok ? x0 + lane : W - 1;  // idle lanes repeat the last column

        const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
        const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
        const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
        const uint32_t rp = (uint32_t)L.src.row_pitch;  // plane < 2^31 bytes (kMaxPlaneBytes)
        const uint32_t xoff = (uint32_t)((cubic_tap(x, L.src.w, L.scale_xd).i - 1) * CC) + srs.delta;
        int my_i = 0;
        float my_c[4] = {0.f, 0.f, 0.f, 0.f};
        if (lane < kCcRows) {
            const CubicTap ty = cubic_tap(min(y0 + lane, H - 1), L.src.h, L.scale_yd);
            my_i = ty.i;
#pragma unroll
            for (int q = 0; q < 4; ++q) my_c[q] = ty.c[q];
        }

        // ---- gathers: the 16 bytes at (row ty.i - 1 + q, column tx.i - 1) ----
        uint32_t ch[kCcRows][4][4];
        // uniform: can any gather of the task reach past the plane's last
        // byte?  If not, no per-lane range check (no exec-mask branch per load)
        const uint32_t last_a = (uint32_t)(__builtin_amdgcn_readlane(my_i, nrow - 1) + 2) * rp + xoff;
        const bool safe = __builtin_amdgcn_ballot_w64(last_a + 16u > slimit) == 0;
        auto gather = [&](auto safe_c) {
        constexpr bool SAFE = decltype(safe_c)::value;
#pragma unroll
        for (int r = 0; r < kCcRows; ++r) {
            const uint32_t ro = (uint32_t)(__builtin_amdgcn_readlane(my_i, r) - 1) * rp + xoff;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                ch[r][q][0] = ch[r][q][1] = ch[r][q][2] = ch[r][q][3] = 0u;
                // a tap row of weight 0 is not read (as above: its term is 0)
                const float cq = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(my_c[q]), r));
                if (r >= nrow || cq == 0.f) continue;  // uniform
                const uint32_t a4 = (ro + (uint32_t)q * rp) & ~3u;
                if (SAFE || a4 + 16u <= slimit) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)a4, 0, VACV_LOAD_AUX);
                    ch[r][q][0] = v[0];
                    ch[r][q][1] = v[1];
                    ch[r][q][2] = v[2];
                    ch[r][q][3] = v[3];
                } else {  // the plane's last bytes: an overhanging load would read zeros
                    const unsigned char* b = sp + ((int64_t)a4 - (int64_t)srs.delta);
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        if (a4 + (uint32_t)e < slimit) ch[r][q][e >> 2] |= (uint32_t)b[e] << (8 * (e & 3));
                }
            }
        }
        };
        if (safe) gather(std::true_type());
        else gather(std::false_type());

        ChanNorm cn[CC] = {};
        if (OUT == kOutNorm) {
#pragma unroll
            for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
        }
        // the column's coefficients, recomputed after the loads (registers)
        const CubicTap tx = cubic_tap(x, L.src.w, L.scale_xd);
        float* xo = xch[wave];
#pragma unroll
        for (int r = 0; r < kCcRows; ++r) {
            float cy[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                cy[q] = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(my_c[q]), r));
            const uint32_t ro = (uint32_t)(__builtin_amdgcn_readlane(my_i, r) - 1) * rp + xoff;
            float h[4][CC];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t sh = (ro + (uint32_t)q * rp) & 3u;
                const uint32_t wv[3] = {__builtin_amdgcn_alignbyte(ch[r][q][1], ch[r][q][0], sh),
                                        __builtin_amdgcn_alignbyte(ch[r][q][2], ch[r][q][1], sh),
                                        __builtin_amdgcn_alignbyte(ch[r][q][3], ch[r][q][2], sh)};
#pragma unroll
                for (int k = 0; k < CC; ++k) {
                    float sv[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const int e = m * CC + k;
                        sv[m] = (float)((wv[e >> 2] >> (8 * (e & 3))) & 0xFFu);
                    }
                    // resize_naive.cpp:325-328
                    h[q][k] = sv[0] * tx.c[0] + sv[1] * tx.c[1] + sv[2] * tx.c[2] + sv[3] * tx.c[3];
                }
            }
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                // resize_naive.cpp:349-351
                float v = h[0][k] * cy[0] + h[1][k] * cy[1] + h[2][k] * cy[2] + h[3][k] * cy[3];
                if (OUT == kOutNorm) v = normalize_f(cn[k], v);
                xo[(r * 64 + lane) * CC + k] = v;
                if (SUMS && col_ok && r < nrow) {
                    const double dv = (double)v;
                    d[2 * k] += dv;
                    d[2 * k + 1] += dv * dv;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- LDS -> HBM: nrow rows of ncol * CC floats (the host checked the
        // destination's 16-byte alignment) ----------------------------------------
        unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                            (int64_t)plane * L.dst.plane_pitch;
        const Rsrc rd = make_rsrc(dp, L.dst.plane_bytes);
        const uint32_t rowp = (uint32_t)L.dst.row_pitch;
        const uint32_t base = (uint32_t)y0 * rowp + (uint32_t)(x0 * CC * 4) + rd.delta;
        const unsigned char* xs = reinterpret_cast<const unsigned char*>(xch[wave]);
        const int rb = ncol * CC * 4;  // bytes of one block row
        if ((rb & 15) == 0) {
            const int cpr = rb >> 4;
            for (int c = lane; c < nrow * cpr; c += 64) {
                const int rr = c / cpr, cc = c - rr * cpr;
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(xs + rr * kRowB + 16 * cc), rd.r,
                                                       (int)(base + (uint32_t)rr * rowp + 16u * (uint32_t)cc), 0,
                                                       VACV_STORE_AUX);
            }
        } else {
            for (int e = lane; e < nrow * rb; e += 64) {
                const int rr = e / rb, cc = e - rr * rb;
                __builtin_amdgcn_raw_buffer_store_b8(xs[rr * kRowB + cc], rd.r, (int)(base + (uint32_t)rr * rowp + cc), 0,
                                                     VACV_STORE_AUX);
            }
        }
    }
    if (SUMS) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int v = 0; v < 2 * CC; ++v) d[v] += __shfl_xor(d[v], o, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int v = 0; v < 2 * CC; ++v) wsum[wave][v] = d[v];
        }
        __syncthreads();
        if (wave == 0) {
            double a = 0.0;
            if (lane < 2 * CC) {
#pragma unroll
                for (int w = 0; w < 4; ++w) a += wsum[w][lane];
            }
            if (L.sum_acc) {
                if (lane < 2 * CC) acc_add(L.sum_acc + (int64_t)pidx * 2 * CC + lane, a, (lane & 1) ? L.sum_q2 : L.sum_q1);
            } else if (lane < 2 * CC) {
                // value-major [CC][2][image][workgroup], as above (group_sums_kernel)
                L.sum_partials[lane * (int64_t)L.n * blocks_per_plane + blockIdx.x] = a;
            }
        }
    }
}

// The column kernel's grid, or false where it does not apply (16-byte aligned
// destination rows, the tuning knob).
bool cubic_cols_plan(const ResizeLaunch& L, int& col_blocks, int& plane_tasks, int& blocks_per_plane) {
    if (tune(VACV_TUNE_CUBIC_DIRECT) == 2) return false;  // 2: the gather kernel (A/B)
    const uintptr_t dbits = reinterpret_cast<uintptr_t>(L.dst.base) | (uintptr_t)L.dst.row_pitch |
                            (uintptr_t)L.dst.img_pitch | (uintptr_t)L.dst.plane_pitch;
    if (dbits & 15) return false;
    const int64_t cbk = (L.dst.w + 63) / 64;
    const int64_t tasks = cbk * ((L.dst.h + kCcRows - 1) / kCcRows);
    const int64_t bpp = (tasks + 3) / 4;
    if (tasks > 0x7FFFFFF0LL || bpp * L.n * L.src.planes > 0x7FFFFFF0LL) return false;
    col_blocks = (int)cbk;
    plane_tasks = (int)tasks;
    blocks_per_plane = (int)bpp;
    return true;
}

// The fixed-order sum of the per-workgroup partials and, optionally, the
// population mean / stddev (stats_kernel's formula, k_pixel.hip): one
// 1024-thread workgroup per (group, channel) sums both of the channel's
// values.  Thread t adds terms t, t + 1024, ... in order, issuing a batch of
// kSumDepth loads (clamped to the run, zeroed past it) before any add, so a
// batch costs one memory latency (cfg5: 12,544 terms per value = one batch);
// then each wave reduces in a fixed xor-shuffle order and thread 0 adds the
// 16 wave sums in order: deterministic run to run, no communication between
// workgroups (round 3's per-wave partials took 16 split workgroups per value,
// an agent-scope counter and a separate stats launch).
constexpr int kSumThreads = 1024;
constexpr int kSumDepth = 16;
__global__ void __launch_bounds__(kSumThreads) group_sums_kernel(const double* partials, int groups, int n, int cc,
                                                                int per_image, double count, double* sums,
                                                                float* mean, float* stddev) {
    __shared__ double red[2][kSumThreads / 64];
    const int g = blockIdx.x / cc;  // output group (image, or 0)
    const int k = blockIdx.x - g * cc;
    const int64_t run = per_image ? groups : (int64_t)n * groups;  // terms of this (group, value), >= 1
    const int64_t vstride = (int64_t)n * groups;
    const double* p1 = partials + (int64_t)(2 * k) * vstride + (per_image ? (int64_t)g * groups : 0);
    const double* p2 = p1 + vstride;
    double a1 = 0.0, a2 = 0.0;
    for (int64_t b = threadIdx.x; b < run; b += (int64_t)kSumDepth * kSumThreads) {
        double x[kSumDepth], y[kSumDepth];
#pragma unroll
        for (int q = 0; q < kSumDepth; ++q) {
            const int64_t t = min(b + (int64_t)q * kSumThreads, run - 1);
            x[q] = p1[t];
            y[q] = p2[t];
        }
#pragma unroll
        for (int q = 0; q < kSumDepth; ++q) {
            const bool ok = b + (int64_t)q * kSumThreads < run;
            a1 += ok ? x[q] : 0.0;
            a2 += ok ? y[q] : 0.0;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a1 += __shfl_xor(a1, o, 64);
        a2 += __shfl_xor(a2, o, 64);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wave] = a1;
        red[1][wave] = a2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s1 = 0.0, s2 = 0.0;
        for (int w = 0; w < kSumThreads / 64; ++w) {
            s1 += red[0][w];
            s2 += red[1][w];
        }
        const int idx = g * cc + k;
        sums[2 * idx] = s1;
        sums[2 * idx + 1] = s2;
        if (mean) {
            const double m = s1 / count;
            double var = s2 / count - m * m;
            if (var < 0) var = 0;
            mean[idx] = (float)m;
            stddev[idx] = (float)sqrt(var);
        }
    }
}

// The accumulators -> sums (fp64), optionally mean / stddev (stats_kernel's
// formula); zeroes the accumulators for the next call.  One workgroup: wave w
// takes values w, w + 4, ... of the n x 2cc; per_image: one value per lane.
// Batch totals: a wave sums one value's n images (integers: any order).
__global__ void __launch_bounds__(kBlock) fixed_sums_kernel(int64_t* acc, int n, int cc, int per_image, int q1,
                                                            int q2, double count, double* sums, float* mean,
                                                            float* stddev) {
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int nv = 2 * cc;
    if (per_image) {
        for (int i = (int)threadIdx.x; i < n * nv; i += kBlock) {
            const int64_t x = acc[i];
            acc[i] = 0;
            sums[i] = ldexp((double)x, -((i & 1) ? q2 : q1));
        }
        __syncthreads();
        if (mean) {
            for (int i = (int)threadIdx.x; i < n * cc; i += kBlock) {
                const double m = sums[2 * i] / count;
                double var = sums[2 * i + 1] / count - m * m;
                if (var < 0) var = 0;
                mean[i] = (float)m;
                stddev[i] = (float)sqrt(var);
            }
        }
        return;
    }
    __shared__ double tot[2 * kMaxC];
    for (int v = wave; v < nv; v += kBlock / 64) {
        int64_t a = 0;
        for (int g = lane; g < n; g += 64) {
            a += acc[(int64_t)g * nv + v];
            acc[(int64_t)g * nv + v] = 0;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) {
            tot[v] = ldexp((double)a, -((v & 1) ? q2 : q1));
            sums[v] = tot[v];
        }
    }
    __syncthreads();
    if (mean && (int)threadIdx.x < cc) {
        const int k = (int)threadIdx.x;
        const double m = tot[2 * k] / count;
        double var = tot[2 * k + 1] / count - m * m;
        if (var < 0) var = 0;
        mean[k] = (float)m;
        stddev[k] = (float)sqrt(var);
    }
}

// The fixed-point units (fixed_sums_kernel): the batch's total of |v| < 2^10
// (Sum x) or v^2 < 2^20 (Sum x^2) over n * P values stays below 2^61.
void fixed_shifts(int64_t values, int& q1, int& q2) {
    int lg = 0;
    while (lg < 62 && (int64_t(1) << lg) < values) ++lg;
    q1 = 61 - 10 - lg;
    q2 = 61 - 20 - lg;
}

template <int CC>
hipError_t launch_cc(const ResizeLaunch& L, hipStream_t s) {
    const bool sums = L.out == kOutF32 && L.sum_partials;
    int groups = 0;  // workgroups per plane
    int col_blocks = 0, plane_tasks = 0;
    const bool cols = cubic_cols_plan(L, col_blocks, plane_tasks, groups);
    ResizeLaunch La = L;
    if (!cols || !sums) La.sum_acc = nullptr;
    if (La.sum_acc) {
        fixed_shifts((int64_t)L.n * L.dst.w * L.dst.h, La.sum_q1, La.sum_q2);
        if (La.sum_q2 < 0) La.sum_acc = nullptr;  // enormous batches: partials and group_sums
    }
    if (cols) {
        const dim3 grid((unsigned)((int64_t)groups * L.n * L.src.planes));
        if (L.out == kOutNorm)
            hipLaunchKernelGGL((cubic_cols_kernel<CC, kOutNorm, false>), grid, dim3(kBlock), 0, s, La, col_blocks,
                               plane_tasks, groups);
        else if (sums)
            hipLaunchKernelGGL((cubic_cols_kernel<CC, kOutF32, true>), grid, dim3(kBlock), 0, s, La, col_blocks,
                               plane_tasks, groups);
        else
            hipLaunchKernelGGL((cubic_cols_kernel<CC, kOutF32, false>), grid, dim3(kBlock), 0, s, La, col_blocks,
                               plane_tasks, groups);
    } else {
        constexpr int kBlockPx = 4 * kWavePx;
        const int64_t P = (int64_t)L.dst.w * L.dst.h;
        const int64_t per_plane = (P + kBlockPx - 1) / kBlockPx;
        const int64_t total = per_plane * L.n * L.src.planes;
        if (P >= 0x7FFFFFFF - kBlockPx || total > 0x7FFFFFF0LL) return hipErrorInvalidValue;
        groups = (int)per_plane;
        if (L.out == kOutNorm)
            hipLaunchKernelGGL((cubic_direct_kernel<CC, kOutNorm, false>), dim3((unsigned)total), dim3(64, 4), 0, s, L,
                               groups);
        else if (sums)
            hipLaunchKernelGGL((cubic_direct_kernel<CC, kOutF32, true>), dim3((unsigned)total), dim3(64, 4), 0, s, L,
                               groups);
        else
            hipLaunchKernelGGL((cubic_direct_kernel<CC, kOutF32, false>), dim3((unsigned)total), dim3(64, 4), 0, s, L,
                               groups);
    }
    if (!sums) return hipGetLastError();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (La.sum_acc) {
        const double cnt = (double)L.dst.w * L.dst.h * (L.sum_per_image ? 1 : L.n);
        hipLaunchKernelGGL(fixed_sums_kernel, dim3(1), dim3(kBlock), 0, s, La.sum_acc, L.n, CC, L.sum_per_image,
                           La.sum_q1, La.sum_q2, cnt, L.sum_out, L.sum_mean, L.sum_std);
        const hipError_t e2 = hipGetLastError();
        // the accumulators must be zero for the next call: if the finishing
        // launch did not go in, clear them here (the error is still returned)
        if (e2 != hipSuccess) (void)hipMemsetAsync(La.sum_acc, 0, (size_t)L.n * 2 * CC * sizeof(int64_t), s);
        return e2;
    }
    const int blocks = (L.sum_per_image ? L.n : 1) * CC;
    const double count = (double)L.dst.w * L.dst.h * (L.sum_per_image ? 1 : L.n);
    hipLaunchKernelGGL(group_sums_kernel, dim3((unsigned)blocks), dim3(kSumThreads), 0, s,
                       (const double*)L.sum_partials, groups, L.n, CC, L.sum_per_image, count, L.sum_out, L.sum_mean,
                       L.sum_std);
    return hipGetLastError();
}

}  // namespace

bool cubic_direct_applies(const ResizeLaunch& L) {
    if (tune(VACV_TUNE_CUBIC_DIRECT) == 0) return false;  // A/B: the staged kernel
    return L.kind == kCubic && L.src.esize == 1 && L.src.cc <= 3 && (L.out == kOutF32 || L.out == kOutNorm);
}

int cubic_direct_groups(const ResizeLaunch& L) {
    int col_blocks = 0, plane_tasks = 0, groups = 0;
    if (cubic_cols_plan(L, col_blocks, plane_tasks, groups)) return groups;
    constexpr int kBlockPx = 4 * kWavePx;
    const int64_t P = (int64_t)L.dst.w * L.dst.h;
    return (int)((P + kBlockPx - 1) / kBlockPx);
}

int64_t cubic_sums_groups_bound(int w, int h) {
    const int64_t gather = ((int64_t)w * h + 4 * kWavePx - 1) / (4 * kWavePx);
    const int64_t cols = (((int64_t)(w + 63) / 64) * ((h + kCcRows - 1) / kCcRows) + 3) / 4;
    return gather > cols ? gather : cols;
}

hipError_t launch_cubic_direct(const ResizeLaunch& L, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_cc<1>(L, s);
        case 2: return launch_cc<2>(L, s);
        case 3: return launch_cc<3>(L, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace vacv
