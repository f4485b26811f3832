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

// One output pixel: CC channel values.  TW = weight type of the kind.
template <int KIND, int CC, typename TIn, int MODE>
struct Pixel;

// u8 bilinear, 11-bit fixed point
template <int CC, int MODE>
struct Pixel<kLinearFixed, CC, uint8_t, MODE> {
    __device__ __forceinline__ static void eval(const unsigned char* rows, int xo, uint32_t xw, int rbA, int rbB,
                                                int wA, int wB, bool two, int out[CC]) {
        const int a0 = (int)(short)(xw & 0xFFFFu), a1 = (int)(short)(xw >> 16);
        const unsigned char* pa = rows + rbA + xo;
        const unsigned char* pb = rows + rbB + xo;
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            const int tl = pa[k], tr = pa[CC + k];
            int bl = 0, br = 0;
            if (two) { bl = pb[k]; br = pb[CC + k]; }
            if (MODE == VACV_LINEAR_REFERENCE) {
                // resize_naive.cpp:61-64: (Sum S*wx*wy) >> 22, stored as a byte
                out[k] = ((tl * a0 * wA + bl * a0 * wB + tr * a1 * wA + br * a1 * wB) >> 22) & 0xFF;
            } else {
                // resize_neon.cpp:103,122-123 (int16 rows), :150-167 (vertical)
                const int h0 = (int)(short)((tl * a0 + tr * a1) >> 4);
                const int h1 = (int)(short)((bl * a0 + br * a1) >> 4);
                out[k] = clamp_u8((((h0 * wA) >> 16) + ((h1 * wB) >> 16) + 2) >> 2);
            }
        }
    }
};

}  // namespace

template <int KIND, int CC, typename TIn, int OUT, int MODE>
__global__ void __launch_bounds__(kBlock)
resize_kernel(ResizeLaunch L) {
    constexpr int TAPS = (KIND == kCubic) ? 4 : 2;
    constexpr int ES = sizeof(TIn);
    constexpr int XW = (KIND == kLinearFixed) ? 4 : (KIND == kLinearFloat ? 8 : 16);
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    // pixels per lane per segment: keep each lane's store >= 4 bytes
    constexpr int PX = (CC * (int)sizeof(TOut) < 4) ? 4 : ((CC * (int)sizeof(TOut) < 8) ? 2 : 1);
    constexpr int SEG = 64 * PX;

    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- which strip ---------------------------------------------------------
    const int strip = blockIdx.x % L.strips;
    const int col = blockIdx.x / L.strips;
    const int tx = col % L.tiles_x;
    const int pidx = col / L.tiles_x;                 // image * planes + plane
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int task0 = strip * L.tasks_per_strip;
    const int task1 = min(L.tiles_y, task0 + L.tasks_per_strip);
    if (task0 >= task1) return;

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

    const unsigned char* src_plane = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc rs = make_rsrc(src_plane, L.src.plane_bytes);
    const uint32_t limit = (uint32_t)L.src.plane_bytes + rs.delta;
    const uint32_t span_off = (uint32_t)(L.plan.col_first[tx] * CC * ES) + rs.delta;
    const int64_t rp = L.src.row_pitch;

    // ---- prefetch a task's rows into registers ------------------------------
    // (slot, chunk) of this thread's m-th chunk is fixed per strip
    int ch_s[kMaxChunks], ch_c[kMaxChunks];
#pragma unroll
    for (int m = 0; m < kMaxChunks; ++m) {
        const int k = tid + m * kBlock;
        ch_s[m] = k / cpr;
        ch_c[m] = k - ch_s[m] * cpr;
    }
    uint4 R[kMaxChunks];
    auto prefetch = [&](int task) {
        const int ns = L.plan.task_nslots[task];
        const int* trow = L.plan.task_rows + (int64_t)task * L.max_slots;
        uint32_t off[kMaxChunks];
#pragma unroll
        for (int m = 0; m < kMaxChunks; ++m)
            off[m] = ch_s[m] < ns ? (((uint32_t)((int64_t)trow[ch_s[m]] * rp) + span_off) & ~15u) + 16u * ch_c[m] : 0u;
        bool tail = false;
#pragma unroll
        for (int m = 0; m < kMaxChunks; ++m) {
            if (ch_s[m] < ns) {
                if (off[m] + 16u <= limit) R[m] = load16(rs, off[m]);
                else tail = true;
            }
        }
        if (tail) {  // only the chunk that crosses the end of the plane
#pragma unroll
            for (int m = 0; m < kMaxChunks; ++m)
                if (ch_s[m] < ns && off[m] + 16u > limit) R[m] = load16_safe(rs, off[m], limit);
        }
    };
    prefetch(task0);

    // ---- per-strip column taps (overlap the first task's loads) -------------
    for (int i = tid; i < nx; i += kBlock) {
        const int e = tx * L.tile_w + i;
        xoff_l[i] = L.plan.xoff[e];
        if (XW == 4) reinterpret_cast<uint32_t*>(xw_l)[i] = reinterpret_cast<const uint32_t*>(L.plan.xw)[e];
        else if (XW == 8) reinterpret_cast<uint2*>(xw_l)[i] = reinterpret_cast<const uint2*>(L.plan.xw)[e];
        else reinterpret_cast<uint4*>(xw_l)[i] = reinterpret_cast<const uint4*>(L.plan.xw)[e];
    }
    ChanNorm cn[CC];
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }

    unsigned char* dst_plane = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                               (int64_t)plane * L.dst.plane_pitch;
    const int segs_per_row = (nx + SEG - 1) / SEG;

    for (int task = task0; task < task1; ++task) {
        if (task != task0) __syncthreads();  // everyone is done reading the previous tile
        // ---- registers -> LDS ----------------------------------------------
        const int ns = L.plan.task_nslots[task];
#pragma unroll
        for (int m = 0; m < kMaxChunks; ++m)
            if (ch_s[m] < ns) *reinterpret_cast<uint4*>(rows_l + ch_s[m] * L.slot_stride + 16 * ch_c[m]) = R[m];
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
        if (task + 1 < task1) prefetch(task + 1);  // in flight during this tile's compute

        // ---- compute: one wave = one segment of one row at a time ----------
        const int nseg = ny * segs_per_row;
        for (int sg = wave; sg < nseg; sg += kBlock / 64) {
            const int t = sg / segs_per_row;               // wave-uniform
            const int sidx = sg - t * segs_per_row;
            const int* ri = rowinfo_l + t * 8;
            int rb[4];
#pragma unroll
            for (int q = 0; q < TAPS; ++q) rb[q] = __builtin_amdgcn_readfirstlane(ri[q]);
            const int w4 = __builtin_amdgcn_readfirstlane(ri[4]);
            const int w5 = __builtin_amdgcn_readfirstlane(ri[5]);
            const int w6 = __builtin_amdgcn_readfirstlane(ri[6]);
            const int w7 = __builtin_amdgcn_readfirstlane(ri[7]);
            const int dy = y0 + t;
            unsigned char* drow = dst_plane + (int64_t)dy * L.dst.row_pitch;
            const int pbase = sidx * SEG + lane * PX;     // first pixel of this lane (tile-relative)

            TOut out[PX * CC];
#pragma unroll
            for (int q = 0; q < PX; ++q) {
                const int pxl = min(pbase + q, nx - 1);       // clamp; the store masks it
                const int xo = xoff_l[pxl];
                if (KIND == kLinearFixed) {
                    const uint32_t wx = reinterpret_cast<const uint32_t*>(xw_l)[pxl];
                    int v[CC];
                    const bool two = (w6 & 2) != 0;            // wave-uniform
                    Pixel<kLinearFixed, CC, uint8_t, MODE>::eval(rows_l, xo, wx, rb[0], rb[1], w4, w5, two, v);
#pragma unroll
                    for (int k = 0; k < CC; ++k) {
                        if (OUT == kOutSame) out[q * CC + k] = (TOut)v[k];
                        else if (OUT == kOutF32) out[q * CC + k] = (TOut)(float)v[k];
                        else out[q * CC + k] = (TOut)normalize_u8v(cn[k], v[k]);
                    }
                } else if (KIND == kLinearFloat) {
                    const float2 wx = reinterpret_cast<const float2*>(xw_l)[pxl];
                    const float wy0 = __int_as_float(w4), wy1 = __int_as_float(w5);
                    const bool two = (w6 & 2) != 0;
                    const unsigned char* pa = rows_l + rb[0] + xo;
                    const unsigned char* pb = rows_l + rb[1] + xo;
#pragma unroll
                    for (int k = 0; k < CC; ++k) {
                        const float tl = lds_ld<float>(pa + 4 * k), tr = lds_ld<float>(pa + 4 * (CC + k));
                        float bl = 0.f, br = 0.f;
                        if (two) { bl = lds_ld<float>(pb + 4 * k); br = lds_ld<float>(pb + 4 * (CC + k)); }
                        // resize_naive.cpp:121-124, summed left to right
                        float val = tl * wx.x * wy0;
                        val += bl * wx.x * wy1;
                        val += tr * wx.y * wy0;
                        val += br * wx.y * wy1;
                        if (OUT == kOutNorm) val = normalize_f(cn[k], val);
                        out[q * CC + k] = (TOut)val;
                    }
                } else {
                    const float4 a = reinterpret_cast<const float4*>(xw_l)[pxl];
                    const float wy[4] = {__int_as_float(w4), __int_as_float(w5), __int_as_float(w6), __int_as_float(w7)};
#pragma unroll
                    for (int k = 0; k < CC; ++k) {
                        float h[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            h[r] = 0.f;
                            if (wy[r] != 0.f) {  // wave-uniform
                                const unsigned char* sp = rows_l + rb[r] + xo + ES * k;
                                const float s0 = as_f(lds_ld<TIn>(sp)), s1 = as_f(lds_ld<TIn>(sp + ES * CC));
                                const float s2 = as_f(lds_ld<TIn>(sp + 2 * ES * CC)), s3 = as_f(lds_ld<TIn>(sp + 3 * ES * CC));
                                // resize_naive.cpp:325-328
                                h[r] = s0 * a.x + s1 * a.y + s2 * a.z + s3 * a.w;
                            }
                        }
                        // resize_naive.cpp:349-351
                        float val = h[0] * wy[0] + h[1] * wy[1] + h[2] * wy[2] + h[3] * wy[3];
                        if (OUT == kOutNorm) val = normalize_f(cn[k], val);
                        out[q * CC + k] = (TOut)val;
                    }
                }
            }

            // ---- store PX*CC contiguous outputs -------------------------------
            const int valid = min(PX, nx - pbase);
            if (valid > 0) {
                unsigned char* dp = drow + ((int64_t)(x0 + pbase) * CC) * (int64_t)sizeof(TOut);
                constexpr int kBytes = PX * CC * (int)sizeof(TOut);
                const uintptr_t a = reinterpret_cast<uintptr_t>(dp);
                if (valid == PX && kBytes % 16 == 0 && (a & 15) == 0) {
#pragma unroll
                    for (int b = 0; b < kBytes / 16; ++b) reinterpret_cast<uint4*>(dp)[b] = reinterpret_cast<const uint4*>(out)[b];
                } else if (valid == PX && kBytes == 12 && (a & 3) == 0) {
                    const uint32_t* o32 = reinterpret_cast<const uint32_t*>(out);
                    reinterpret_cast<uint32_t*>(dp)[0] = o32[0];
                    reinterpret_cast<uint32_t*>(dp)[1] = o32[1];
                    reinterpret_cast<uint32_t*>(dp)[2] = o32[2];
                } else if (valid == PX && kBytes % 8 == 0 && (a & 7) == 0) {
#pragma unroll
                    for (int b = 0; b < kBytes / 8; ++b) reinterpret_cast<uint2*>(dp)[b] = reinterpret_cast<const uint2*>(out)[b];
                } else if (valid == PX && kBytes % 4 == 0 && (a & 3) == 0) {
#pragma unroll
                    for (int b = 0; b < kBytes / 4; ++b) reinterpret_cast<uint32_t*>(dp)[b] = reinterpret_cast<const uint32_t*>(out)[b];
                } else {
#pragma unroll
                    for (int e = 0; e < PX * CC; ++e)
                        if (e < valid * CC) reinterpret_cast<TOut*>(dp)[e] = out[e];
                }
            }
        }
    }
}

namespace {

template <int KIND, int CC, typename TIn, int OUT, int MODE>
hipError_t launch_one(const ResizeLaunch& L, hipStream_t s) {
    const int64_t blocks = (int64_t)L.n * L.src.planes * L.tiles_x * L.strips;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL((resize_kernel<KIND, CC, TIn, OUT, MODE>), dim3((unsigned)blocks), dim3(kBlock), L.lds_bytes, s, L);
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
