// k_resize.hip -- separable resamplers (bilinear u8 / fp32, Keys cubic) with
// optional fused u8->fp32 widening and normalisation epilogues.
//
// Reference loops restated: ResizeNaive::resize_naive_inter_linear_u8/_fp32
// (resize_naive.cpp:10-128), ResizeNeon (resize_neon.cpp:12-188), the cubic
// pair (resize_naive.cpp:130-569), and the fused ResizeNormalize semantics
// (resize_normalize.cpp:33-107 = resize, convertTo fp32, per-channel
// (x-mean)/(std+1e-6)).  The tap tables come from the host planner
// (resize_plan.cpp), computed with the same arithmetic.
//
// Structure (HBM-bound gather; no MFMA):
//   * a workgroup owns a strip: one plane, one tile column, a run of
//     consecutive row tiles ("tasks");
//   * per task the source rows with a non-zero vertical weight are staged
//     into LDS as the column span the tile needs, by 16-byte buffer loads
//     (bounds-safe past the end of the batch).  Task i+1's loads are issued
//     into registers before task i is computed, so HBM latency hides under
//     the compute of the previous tile (register-staged software pipeline);
//   * compute: a wave takes one segment of one output row at a time (64
//     lanes x PX pixels), so the vertical taps are wave-uniform scalars; a
//     lane reads its pixel's column taps from LDS, gathers the source bytes
//     from the staged rows, and stores its PX*CC outputs contiguously
//     (a wave store covers 64 consecutive lanes' bytes).
// Rows whose vertical weight is zero are never read: at an exact 3x
// downscale only every third source row moves (B_alg).
#pragma clang fp contract(off)

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kMaxChunks = 8;  // 16-byte prefetch registers per thread (planner bound)

// 16 bytes at byte offset o (from the 16-aligned base) with a clean tail: a
// raw-buffer load that straddles num_records returns all zeros, so the
// chunk that crosses the end of a plane is assembled byte by byte.
__device__ __forceinline__ uint4 load16_safe(const Rsrc& rs, uint32_t o, uint32_t limit) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        if (o + b < limit) {
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b8(rs.r, (int)(o + b), 0, 0);
            w[b >> 2] |= (v & 0xFFu) << (8 * (b & 3));
        }
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

template <typename T>
__device__ __forceinline__ T lds_ld(const unsigned char* p) {
    return *reinterpret_cast<const T*>(p);
}

template <typename T>
__device__ __forceinline__ float as_f(T v) {
    return (float)v;
}

// Vertical taps of one output row, as staged in rowinfo: LDS offsets of the
// tap rows and the weights (int bits for fixed point, float bits otherwise).
struct RowTaps {
    int rb[4];
    int w[4];
};

__device__ __forceinline__ RowTaps row_taps(const int* ri) {
    const int4 a = *reinterpret_cast<const int4*>(ri);
    const int4 b = *reinterpret_cast<const int4*>(ri + 4);
    return RowTaps{{a.x, a.y, a.z, a.w}, {b.x, b.y, b.z, b.w}};
}

// Channel k of one output pixel, from the staged rows.  TWO: the second
// vertical tap may be non-zero (a zero-weight tap adds exactly 0 and is not
// read).  XW = the column-tap record of the kind.
template <int KIND, int CC, typename TIn, int MODE>
struct Sampler;

// u8 bilinear, 11-bit fixed point
template <int CC, int MODE>
struct Sampler<kLinearFixed, CC, uint8_t, MODE> {
    using XW = uint32_t;  // short2 {a0, a1}
    static constexpr int ES = 1;
    template <bool TWO>
    __device__ __forceinline__ static int at(const unsigned char* rows, int off, XW xw, const RowTaps& r) {
        // The column weights a0, a1 and row weights wA, wB are SATURATE_CAST
        // values of (1-f)*2048 and f*2048 with f in [0, 1], i.e. in
        // [0, 2048]: xw = {a0, a1} is a u16 pair, the row sums tl*a0 + tr*a1
        // (< 2^24) are one packed dot product (v_dot2_u32_u16), and every
        // further product is an exact full-rate 24-bit multiply.
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        const us2 wx = __builtin_bit_cast(us2, xw);
        const unsigned char* pa = rows + r.rb[0] + off;
        const unsigned char* pb = rows + r.rb[1] + off;
        const uint32_t top = (uint32_t)pa[0] | ((uint32_t)pa[CC] << 16);
        uint32_t bot = 0;
        if (TWO) bot = (uint32_t)pb[0] | ((uint32_t)pb[CC] << 16);
        const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
        const uint32_t hb = TWO ? __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false) : 0u;
        const uint32_t wA = (uint32_t)r.w[0], wB = (uint32_t)r.w[1];
        if (MODE == VACV_LINEAR_REFERENCE) {
            // resize_naive.cpp:61-64: (Sum S*wx*wy) >> 22, stored as a byte;
            // (tl*a0 + tr*a1)*wA + (bl*a0 + br*a1)*wB is the same int32 value
            // (all terms >= 0, total <= 255*2049^2 < 2^31)
            if (TWO) return (int)(((__umul24(ht, wA) + __umul24(hb, wB)) >> 22) & 0xFF);
            return (int)((__umul24(ht, wA) >> 22) & 0xFF);
        }
        // resize_neon.cpp:103,122-123 (int16 rows), :150-167 (vertical)
        const int h0 = (int)(short)(ht >> 4);
        const int h1 = (int)(short)(hb >> 4);
        return clamp_u8((((h0 * (int)wA) >> 16) + ((h1 * (int)wB) >> 16) + 2) >> 2);
    }
};

// fp32 bilinear
template <int CC, int MODE>
struct Sampler<kLinearFloat, CC, float, MODE> {
    using XW = float2;
    static constexpr int ES = 4;
    template <bool TWO>
    __device__ __forceinline__ static float at(const unsigned char* rows, int off, XW wx, const RowTaps& r) {
        const unsigned char* pa = rows + r.rb[0] + off;
        const unsigned char* pb = rows + r.rb[1] + off;
        const float wy0 = __int_as_float(r.w[0]), wy1 = __int_as_float(r.w[1]);
        const float tl = lds_ld<float>(pa), tr = lds_ld<float>(pa + 4 * CC);
        float bl = 0.f, br = 0.f;
        if (TWO) { bl = lds_ld<float>(pb); br = lds_ld<float>(pb + 4 * CC); }
        // resize_naive.cpp:121-124, summed left to right
        float val = tl * wx.x * wy0;
        val += bl * wx.x * wy1;
        val += tr * wx.y * wy0;
        val += br * wx.y * wy1;
        return val;
    }
};

// Keys cubic (A = -0.75), u8 or fp32 source
template <int CC, typename TIn, int MODE>
struct Sampler<kCubic, CC, TIn, MODE> {
    using XW = float4;
    static constexpr int ES = sizeof(TIn);
    template <bool TWO>
    __device__ __forceinline__ static float at(const unsigned char* rows, int off, XW a, const RowTaps& r) {
        float h[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // zero-weight taps read a valid staged row (slot 0); the reference
            // multiplies them by 0 as well
            const unsigned char* sp = rows + r.rb[q] + off;
            const float s0 = as_f(lds_ld<TIn>(sp)), s1 = as_f(lds_ld<TIn>(sp + ES * CC));
            const float s2 = as_f(lds_ld<TIn>(sp + 2 * ES * CC)), s3 = as_f(lds_ld<TIn>(sp + 3 * ES * CC));
            // resize_naive.cpp:325-328
            h[q] = s0 * a.x + s1 * a.y + s2 * a.z + s3 * a.w;
        }
        // resize_naive.cpp:349-351
        return h[0] * __int_as_float(r.w[0]) + h[1] * __int_as_float(r.w[1]) + h[2] * __int_as_float(r.w[2]) +
               h[3] * __int_as_float(r.w[3]);
    }
};

// v[i] for a small runtime i, without a scratch-indexed array
template <int N, typename T>
__device__ __forceinline__ T pick(const T (&v)[N], int i) {
    T r = v[0];
#pragma unroll
    for (int q = 1; q < N; ++q)
        if (i == q) r = v[q];
    return r;
}

template <int N>
__device__ __forceinline__ ChanNorm pick(const ChanNorm (&v)[N], int i) {
    ChanNorm r = v[0];
#pragma unroll
    for (int q = 1; q < N; ++q) {
        const bool s = i == q;
        r.mean = s ? v[q].mean : r.mean;
        r.stdv = s ? v[q].stdv : r.stdv;
        r.inv = s ? v[q].inv : r.inv;
        r.mul = s ? v[q].mul : r.mul;
    }
    return r;
}

}  // namespace

template <int KIND, int CC, typename TIn, int OUT, int MODE>
__global__ void __launch_bounds__(kBlock)
resize_kernel(ResizeLaunch L) {
    constexpr int TAPS = (KIND == kCubic) ? 4 : 2;
    constexpr int ES = sizeof(TIn);
    constexpr int XW = (KIND == kLinearFixed) ? 4 : (KIND == kLinearFloat ? 8 : 16);
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    constexpr int PX = 4;  // byte output: consecutive pixels per lane
    using Smp = Sampler<KIND, CC, TIn, MODE>;

    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- which tasks -----------------------------------------------------------
    // Strips: a run of consecutive row tiles of one (plane, column).
    // Interleaved (L.interleave): tasks t = blockIdx.x + k*gridDim.x of the
    // address-ordered list (plane, row tile, column), so all workgroups advance
    // through HBM together and the chip's in-flight window stays compact
    // (tools/membench2.hip: that traffic shape streams ~20 % faster).  The
    // host makes gridDim.x a multiple of tiles_x, so in both modes a
    // workgroup keeps one column and its lane-stationary constants.
    int tx, task0 = 0, ntask, col_pidx = 0;
    if (L.interleave) {
        tx = blockIdx.x % L.tiles_x;
        const int T = L.n * L.src.planes * L.tiles_y * L.tiles_x;
        ntask = (int)blockIdx.x < T ? (T - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    } else {
        const int strip = blockIdx.x % L.strips;
        const int col = blockIdx.x / L.strips;
        tx = col % L.tiles_x;
        col_pidx = col / L.tiles_x;
        task0 = strip * L.tasks_per_strip;
        ntask = min(L.tiles_y, task0 + L.tasks_per_strip) - task0;
    }
    if (ntask <= 0) return;
    // k-th task of this workgroup -> (image * planes + plane, row tile)
    auto task_of = [&](int k, int& pidx, int& ty) {
        if (L.interleave) {
            const int r = ((int)blockIdx.x + k * (int)gridDim.x) / L.tiles_x;
            ty = r % L.tiles_y;
            pidx = r / L.tiles_y;
        } else {
            pidx = col_pidx;
            ty = task0 + k;
        }
    };

    const int x0 = tx * L.tile_w;
    const int nx = min(L.tile_w, L.dst.w - x0);
    const int cpr = L.plan.cpr[tx];

    // ---- LDS carve-up: xoff | xw | rowinfo[32][8] | head[max_slots] | rows -----
    int* xoff_l = reinterpret_cast<int*>(lds);
    unsigned char* p = lds + ((L.tile_w * 4 + 15) & ~15);
    unsigned char* xw_l = p;
    p += (L.tile_w * XW + 15) & ~15;
    int* rowinfo_l = reinterpret_cast<int*>(p);   // [tile_h][8]
    p += 32 * 8 * 4;
    int* head_l = reinterpret_cast<int*>(p);
    p += (L.max_slots * 4 + 15) & ~15;
    unsigned char* rows_l = p;

    const int64_t rp = L.src.row_pitch;
    const uint32_t col_off = (uint32_t)(L.plan.col_first[tx] * CC * ES);
    auto src_rsrc = [&](int pidx) {
        const int im = pidx / L.src.planes, pl = pidx - im * L.src.planes;
        return make_rsrc(L.src.base + (int64_t)im * L.src.img_pitch + (int64_t)pl * L.src.plane_pitch,
                         L.src.plane_bytes);
    };

    // ---- prefetch a task's rows into registers ------------------------------
    // (slot, chunk) of this thread's m-th chunk is fixed per strip
    // (recomputed where used rather than held in registers across the compute)
    const uint32_t cpr_magic = (uint32_t)(((1ull << 32) + cpr - 1) / cpr);  // k / cpr for k < kMaxChunks*kBlock
    auto chunk_slot = [&](int m, int& sl, int& c) {
        const int k = tid + m * kBlock;
        sl = cpr == 1 ? k : (int)__umulhi((uint32_t)k, cpr_magic);
        c = k - sl * cpr;
    };
    uint4 R[kMaxChunks];
    auto prefetch = [&](int k) {
        int pidx, task;
        task_of(k, pidx, task);
        const Rsrc rs = src_rsrc(pidx);
        const uint32_t limit = (uint32_t)L.src.plane_bytes + rs.delta;
        const uint32_t span_off = col_off + rs.delta;
        const int ns = L.plan.task_nslots[task];
        const int* trow = L.plan.task_rows + (int64_t)task * L.max_slots;
        uint32_t off[kMaxChunks];
        bool live[kMaxChunks];
#pragma unroll
        for (int m = 0; m < kMaxChunks; ++m) {
            int sl, c;
            chunk_slot(m, sl, c);
            live[m] = sl < ns;
            off[m] = live[m] ? (((uint32_t)((int64_t)trow[sl] * rp) + span_off) & ~15u) + 16u * c : 0u;
        }
        bool tail = false;
#pragma unroll
        for (int m = 0; m < kMaxChunks; ++m) {
            if (live[m]) {
                if (off[m] + 16u <= limit) R[m] = load16(rs, off[m]);
                else tail = true;
            }
        }
        if (tail) {  // only the chunk that crosses the end of the plane
#pragma unroll
            for (int m = 0; m < kMaxChunks; ++m)
                if (live[m] && off[m] + 16u > limit) R[m] = load16_safe(rs, off[m], limit);
        }
    };
    prefetch(0);

    // ---- per-strip column taps (overlap the first task's loads) -------------
    for (int i = tid; i < nx; i += kBlock) {
        const int e = tx * L.tile_w + i;
        xoff_l[i] = L.plan.xoff[e];
        if (XW == 4) reinterpret_cast<uint32_t*>(xw_l)[i] = reinterpret_cast<const uint32_t*>(L.plan.xw)[e];
        else if (XW == 8) reinterpret_cast<uint2*>(xw_l)[i] = reinterpret_cast<const uint2*>(L.plan.xw)[e];
        else reinterpret_cast<uint4*>(xw_l)[i] = reinterpret_cast<const uint4*>(L.plan.xw)[e];
    }
    ChanNorm cn[CC] = {};
    bool all_mul = false;
    int cur_img = -1;
    const int gpr = (nx + PX - 1) / PX;  // pixel groups per output row

    // fp32-output chunk state (see the compute section)
    constexpr int E = 4;
    constexpr int MAXM = kResizeMaxChunksPerLane;
    const int rl = nx * CC;  // elements per tile row
    int c_e0[MAXM];
    // per element: LDS byte offset of its first tap | pixel << 16, its column
    // weights (cubic: re-read from LDS, 16 B each), and its channel's
    // normalisation (x - mean) op a, op = * (verified inverse) or / (divisor)
    constexpr bool kHoldXW = sizeof(typename Smp::XW) <= 8;
    int c_off[MAXM][E];
    typename Smp::XW c_xw[MAXM][kHoldXW ? E : 1];
    float c_mean[MAXM][E];
    double c_a[MAXM][E];

    for (int k = 0; k < ntask; ++k) {
        int pidx, task;
        task_of(k, pidx, task);
        const int img = pidx / L.src.planes;
        const int plane = pidx - img * L.src.planes;
        const bool img_changed = img != cur_img;  // uniform
        if (OUT == kOutNorm && img_changed) {
#pragma unroll
            for (int q = 0; q < CC; ++q) cn[q] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : q);
            // u8 normalisation as one multiply per element when the host
            // verified it exact for every channel (NormSpec.mul_ok)
            all_mul = true;
#pragma unroll
            for (int q = 0; q < CC; ++q) all_mul = all_mul && cn[q].mul;
        }
        cur_img = img;
        unsigned char* dst_plane = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                                   (int64_t)plane * L.dst.plane_pitch;
        const Rsrc rd = make_rsrc(dst_plane, L.dst.plane_bytes);
        const uint32_t span_off = col_off + src_rsrc(pidx).delta;
        if (k) __syncthreads();  // everyone is done reading the previous tile
        // ---- registers -> LDS ----------------------------------------------
        const int ns = L.plan.task_nslots[task];
#pragma unroll
        for (int m = 0; m < kMaxChunks; ++m)
        {
            int sl, c;
            chunk_slot(m, sl, c);
            if (sl < ns) *reinterpret_cast<uint4*>(rows_l + sl * L.slot_stride + 16 * c) = R[m];
        }
        if (tid < ns) {
            const int row = L.plan.task_rows[(int64_t)task * L.max_slots + tid];
            head_l[tid] = (int)(((uint32_t)((int64_t)row * rp) + span_off) & 15u);
        }
        __syncthreads();
        // rowinfo[t]: LDS offset of each vertical tap's row (weight 0: a
        // harmless valid row, slot 0), then the TAPS weights and a flag mask
        const int y0 = task * L.tile_h;
        const int ny = min(L.tile_h, L.dst.h - y0);
        if (tid < ny) {
            const int nc = L.tile_h * TAPS;
            int* ri = rowinfo_l + tid * 8;
            int nzmask = 0;
#pragma unroll
            for (int q = 0; q < TAPS; ++q) {
                const int sl = L.plan.task_cand[(int64_t)task * nc + tid * TAPS + q];
                ri[q] = sl >= 0 ? sl * L.slot_stride + head_l[sl] : head_l[0];
                nzmask |= (sl >= 0) << q;
            }
            if (KIND == kLinearFixed) {
                const int2 w = reinterpret_cast<const int2*>(L.plan.yw)[y0 + tid];
                ri[4] = w.x; ri[5] = w.y; ri[6] = nzmask;
            } else if (KIND == kLinearFloat) {
                const float2 w = reinterpret_cast<const float2*>(L.plan.yw)[y0 + tid];
                ri[4] = __float_as_int(w.x); ri[5] = __float_as_int(w.y); ri[6] = nzmask;
            } else {
                const float4 w = reinterpret_cast<const float4*>(L.plan.yw)[y0 + tid];
                ri[4] = __float_as_int(w.x); ri[5] = __float_as_int(w.y);
                ri[6] = __float_as_int(w.z); ri[7] = __float_as_int(w.w);
            }
        }
        __syncthreads();
        if (k + 1 < ntask) prefetch(k + 1);  // in flight during this tile's compute

        // ---- compute -----------------------------------------------------------
        const bool two = (L.plan.task_flags[task] & 2) != 0;  // uniform: some row uses tap 1
        auto run = [&](auto two_tag, auto mul_tag) {
            constexpr bool TWO = decltype(two_tag)::value;
            constexpr bool MUL = decltype(mul_tag)::value;  // every channel normalises by the verified multiply
            if constexpr (sizeof(TOut) == 1) {
                // byte output: a lane takes PX consecutive pixels of a row
                // (PX*CC bytes, dword stores)
                const int ngroups = ny * gpr;
                for (int g = tid; g < ngroups; g += kBlock) {
                    const int t = g / gpr;
                    const int pbase = (g - t * gpr) * PX;  // tile-relative first pixel
                    const RowTaps rt = row_taps(rowinfo_l + t * 8);
                    unsigned char* drow = dst_plane + (int64_t)(y0 + t) * L.dst.row_pitch;
                    TOut out[PX * CC];
#pragma unroll
                    for (int q = 0; q < PX; ++q) {
                        const int pxl = min(pbase + q, nx - 1);  // clamp; the store masks it
                        const typename Smp::XW xw = reinterpret_cast<const typename Smp::XW*>(xw_l)[pxl];
#pragma unroll
                        for (int k = 0; k < CC; ++k)
                            out[q * CC + k] = (TOut)Smp::template at<TWO>(rows_l, xoff_l[pxl] + Smp::ES * k, xw, rt);
                    }
                    const int valid = min(PX, nx - pbase);
                    unsigned char* dp = drow + (int64_t)(x0 + pbase) * CC;
                    constexpr int kBytes = PX * CC;
                    if (valid == PX && kBytes % 4 == 0 && (reinterpret_cast<uintptr_t>(dp) & 3) == 0) {
#pragma unroll
                        for (int b = 0; b < kBytes / 4; ++b)
                            reinterpret_cast<uint32_t*>(dp)[b] = reinterpret_cast<const uint32_t*>(out)[b];
                    } else {
#pragma unroll
                        for (int e = 0; e < kBytes; ++e)
                            if (e < valid * CC) dp[e] = out[e];
                    }
                }
            }
        };
        if constexpr (sizeof(TOut) == 1) {
            if (two) run(std::true_type{}, std::false_type{});
            else run(std::false_type{}, std::false_type{});
        } else {
            // fp32 output: lane-stationary chunks.  Lane tid owns 4-element
            // output chunks j = tid + m*kBlock of every row of the tile (the
            // planner keeps a row within MAXM*kBlock chunks), so its column
            // taps, channel constants and store offsets are computed once per
            // strip; the vertical taps of a row are wave-uniform scalars.  One
            // wave store instruction writes 1 KiB of contiguous output.
            if (k == 0 || (OUT == kOutNorm && img_changed)) {
#pragma unroll
                for (int m = 0; m < MAXM; ++m) {
                    const int e0 = (tid + m * kBlock) * E;
                    const int p0 = e0 / CC;
                    const int k0 = e0 - p0 * CC;
                    c_e0[m] = e0;
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        const int kk = k0 + i;
                        const int dp = kk / CC;
                        const int k = kk - dp * CC;
                        const int px = min(p0 + dp, nx - 1);  // clamp; the store masks it
                        c_off[m][i] = (xoff_l[px] + Smp::ES * k) | (px << 16);
                        if constexpr (kHoldXW) c_xw[m][i] = reinterpret_cast<const typename Smp::XW*>(xw_l)[px];
                        const ChanNorm c = pick(cn, k);
                        c_mean[m][i] = c.mean;
                        c_a[m][i] = (KIND == kLinearFixed && all_mul) ? c.inv : (double)c.stdv + 1e-6;  // normalize_naive.cpp:84-87
                    }
                }
            }
            for (int t = 0; t < ny; ++t) {
                RowTaps rt;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    rt.rb[q] = __builtin_amdgcn_readfirstlane(rowinfo_l[t * 8 + q]);
                    rt.w[q] = __builtin_amdgcn_readfirstlane(rowinfo_l[t * 8 + 4 + q]);
                }
                const int64_t orow = (int64_t)(y0 + t) * L.dst.row_pitch + (int64_t)x0 * CC * 4;
                auto row_pass = [&](auto two_tag, auto mul_tag) {
                    constexpr bool TWO = decltype(two_tag)::value;
                    constexpr bool MUL = decltype(mul_tag)::value;
#pragma unroll
                    for (int m = 0; m < MAXM; ++m) {
                        if (c_e0[m] >= rl) break;
                        float out[E];
#pragma unroll
                        for (int i = 0; i < E; ++i) {
                            typename Smp::XW xw;
                            if constexpr (kHoldXW) xw = c_xw[m][i];
                            else xw = reinterpret_cast<const typename Smp::XW*>(xw_l)[c_off[m][i] >> 16];
                            const auto v = Smp::template at<TWO>(rows_l, c_off[m][i] & 0xFFFF, xw, rt);
                            if constexpr (OUT == kOutNorm) {
                                // normalize_naive.cpp:74-90: float subtract, fp64 divide
                                const double d = (double)((float)v - c_mean[m][i]);
                                if constexpr (MUL) out[i] = (float)(d * c_a[m][i]);
                                else out[i] = (float)(d / c_a[m][i]);
                            } else {
                                out[i] = (float)v;
                            }
                        }
                        const int64_t ob = orow + (int64_t)c_e0[m] * 4;
                        const int valid = min(E, rl - c_e0[m]);
                        const uint32_t boff = (uint32_t)ob + rd.delta;
                        if (valid == E && (boff & 15u) == 0) {
                            store16(rd, boff, make_uint4(__float_as_uint(out[0]), __float_as_uint(out[1]),
                                                         __float_as_uint(out[2]), __float_as_uint(out[3])));
                        } else {
                            float* dp = reinterpret_cast<float*>(dst_plane + ob);
#pragma unroll
                            for (int i = 0; i < E; ++i)
                                if (i < valid) dp[i] = out[i];
                        }
                    }
                };
                const bool row_two = KIND == kCubic || (rt.w[2] & 2) != 0;  // linear: w[2] = tap mask
                if (KIND == kLinearFixed && OUT == kOutNorm && all_mul) {
                    if (row_two) row_pass(std::true_type{}, std::true_type{});
                    else row_pass(std::false_type{}, std::true_type{});
                } else {
                    if (row_two) row_pass(std::true_type{}, std::false_type{});
                    else row_pass(std::false_type{}, std::false_type{});
                }
            }
        }
    }
}

namespace {

template <typename K>
int64_t resident_workgroups(K kernel, int lds_bytes) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, int64_t> cache;  // (device, lds) -> workgroups
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({dev, lds_bytes});
    if (it != cache.end()) return it->second;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds_bytes) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const int64_t r = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
    cache.emplace(std::make_pair(dev, lds_bytes), r);
    return r;
}

template <int KIND, int CC, typename TIn, int OUT, int MODE>
hipError_t launch_one(ResizeLaunch L, hipStream_t s) {
    auto kernel = resize_kernel<KIND, CC, TIn, OUT, MODE>;
    const int64_t resident = resident_workgroups(kernel, L.lds_bytes);
    if (resident <= 0) return hipErrorInvalidValue;
    if (L.interleave) {
        // one wave of resident workgroups, a multiple of tiles_x (a workgroup
        // keeps its column); VACV_RESIZE_WGS overrides, for measurement
        const int64_t tasks = (int64_t)L.n * L.src.planes * L.tiles_y * L.tiles_x;
        if (tasks > 0x7FFFFFFF) return hipErrorInvalidValue;
        const int wgs = tune(VACV_TUNE_RESIZE_WGS);
        // 3 x residency measured best (0.2326 vs 0.2351 ms at 1x on the
        // headline): queued workgroups fill in as early ones drain
        int64_t want = wgs > 0 ? wgs : 3 * resident;
        want = std::max<int64_t>(L.tiles_x, want / L.tiles_x * L.tiles_x);
        const int64_t blocks = std::min<int64_t>(want, tasks);
        hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(kBlock), L.lds_bytes, s, L);
        return hipGetLastError();
    }
    set_strips(L, resident);
    const int64_t blocks = (int64_t)L.n * L.src.planes * L.tiles_x * L.strips;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(kBlock), L.lds_bytes, s, L);
    return hipGetLastError();
}

template <int KIND, typename TIn, int OUT, int MODE>
hipError_t launch_cc(const ResizeLaunch& L, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<KIND, 1, TIn, OUT, MODE>(L, s);
        case 2: return launch_one<KIND, 2, TIn, OUT, MODE>(L, s);
        case 3: return launch_one<KIND, 3, TIn, OUT, MODE>(L, s);
        case 4: return launch_one<KIND, 4, TIn, OUT, MODE>(L, s);
        default: return hipErrorInvalidValue;
    }
}

template <int OUT>
hipError_t launch_fixed(const ResizeLaunch& L, hipStream_t s) {
    switch (L.mode) {
        case VACV_LINEAR_REFERENCE: return launch_cc<kLinearFixed, uint8_t, OUT, VACV_LINEAR_REFERENCE>(L, s);
        case VACV_LINEAR_NEON: return launch_cc<kLinearFixed, uint8_t, OUT, VACV_LINEAR_NEON>(L, s);
        default: return launch_cc<kLinearFixed, uint8_t, OUT, VACV_LINEAR_OPENCV>(L, s);
    }
}

}  // namespace

hipError_t launch_resize(const ResizeLaunch& L, hipStream_t s) {
    if (L.kind == kLinearFixed) {
        if (L.out == kOutSame) return launch_fixed<kOutSame>(L, s);
        if (L.out == kOutF32) return launch_fixed<kOutF32>(L, s);
        return launch_fixed<kOutNorm>(L, s);
    }
    if (L.kind == kLinearFloat) {
        if (L.out == kOutNorm) return launch_cc<kLinearFloat, float, kOutNorm, 0>(L, s);
        return launch_cc<kLinearFloat, float, kOutSame, 0>(L, s);
    }
    if (L.src.esize == 1) {
        if (L.out == kOutNorm) return launch_cc<kCubic, uint8_t, kOutNorm, 0>(L, s);
        return launch_cc<kCubic, uint8_t, kOutF32, 0>(L, s);
    }
    if (L.out == kOutNorm) return launch_cc<kCubic, float, kOutNorm, 0>(L, s);
    return launch_cc<kCubic, float, kOutSame, 0>(L, s);
}

}  // namespace vacv
