// k_resize.hip -- separable resamplers (bilinear u8 / fp32, Keys cubic) with
// optional fused u8->fp32 widening and normalisation epilogues.
//
// Reference loops restated: ResizeNaive::resize_naive_inter_linear_u8/_fp32
// (resize_naive.cpp:10-128), ResizeNeon (resize_neon.cpp:12-188), the cubic
// pair (resize_naive.cpp:130-569), and the fused ResizeNormalize semantics
// (resize_normalize.cpp:33-107 = resize, convertTo fp32, per-channel
// (x-mean)/(std+1e-6)).
//
// One workgroup = one output tile (tile_w x tile_h pixels) of one plane.
//   1. tap tables for the tile's columns go to LDS (the arithmetic is the
//      reference's; see vacv_semantics.hpp), one entry per output column;
//   2. every source row with a non-zero vertical weight is staged into LDS
//      once, as the column span the tile needs, by 16-byte buffer loads
//      (coalesced, bounds-safe past the end of the batch);
//   3. each work item produces 4 consecutive output pixels x CC channels from
//      LDS and writes them with 16-byte (fp32) / 4-byte (u8) stores.
// Rows whose vertical weight is zero are never read from HBM: at an exact
// 3x downscale only every third source row moves (B_alg).
#pragma clang fp contract(off)

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kPx = 4;  // output pixels per work item

struct TileCtx {
    int x0, nx, y0, ny;
    int col_first;      // first staged source column
    int span_bytes;     // staged bytes per row
    int cpr;            // 16-byte chunks per staged row
    int lo;             // dense mode: first staged row
    int nslots;
};

template <int KIND>
__device__ __forceinline__ int tap_origin(const ResizeLaunch& L, int d, bool vertical) {
    const int n_in = vertical ? L.src.h : L.src.w;
    if (KIND == kLinearFixed) {
        const int n_out = vertical ? L.dst.h : L.dst.w;
        return fixed_tap(d, n_in, n_out, vertical ? L.scale_yf : L.scale_xf,
                         vertical ? L.scale_yd : L.scale_xd, L.mode).i;
    } else if (KIND == kLinearFloat) {
        return float_tap(d, n_in, vertical ? L.scale_yf : L.scale_xf).i;
    } else {
        return cubic_tap(d, n_in, vertical ? L.scale_yd : L.scale_xd).i - 1;
    }
}

// Vertical taps of output row d: origin row, TAPS weights (as float for the
// float kinds, as int for the fixed kind).
template <int KIND>
struct VTaps {
    int row0;
    int wi[2];
    float wf[4];
};

template <int KIND>
__device__ __forceinline__ VTaps<KIND> vtaps(const ResizeLaunch& L, int d) {
    VTaps<KIND> v;
    if (KIND == kLinearFixed) {
        FixedTap t = fixed_tap(d, L.src.h, L.dst.h, L.scale_yf, L.scale_yd, L.mode);
        v.row0 = t.i;
        v.wi[0] = t.w0;
        v.wi[1] = t.w1;
    } else if (KIND == kLinearFloat) {
        FloatTap t = float_tap(d, L.src.h, L.scale_yf);
        v.row0 = t.i;
        v.wf[0] = t.w0;
        v.wf[1] = t.w1;
    } else {
        CubicTap t = cubic_tap(d, L.src.h, L.scale_yd);
        v.row0 = t.i - 1;
        v.wf[0] = t.c[0]; v.wf[1] = t.c[1]; v.wf[2] = t.c[2]; v.wf[3] = t.c[3];
    }
    return v;
}

// j may be a run-time value: select with constant indices so VTaps stays in
// registers (a dynamic index would spill the arrays to scratch).
template <int KIND>
__device__ __forceinline__ bool vweight_nonzero(const VTaps<KIND>& v, int j) {
    if (KIND == kLinearFixed) return (j == 0 ? v.wi[0] : v.wi[1]) != 0;
    const float w = j == 0 ? v.wf[0] : (j == 1 ? v.wf[1] : (j == 2 ? v.wf[2] : v.wf[3]));
    return w != 0.f;
}

template <int KIND, int CC, typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock)
resize_kernel(ResizeLaunch L) {
    constexpr int TAPS = (KIND == kCubic) ? 4 : 2;
    constexpr int ES = sizeof(TIn);
    constexpr bool kLut = (KIND == kLinearFixed) && (OUT == kOutNorm);
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;

    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x;
    const int tile = blockIdx.x;
    const int pidx = blockIdx.y;                  // image * planes + plane
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;

    TileCtx T;
    {
        const int tx = tile % L.tiles_x, ty = tile / L.tiles_x;
        T.x0 = tx * L.tile_w;
        T.nx = min(L.tile_w, L.dst.w - T.x0);
        T.y0 = ty * L.tile_h;
        T.ny = min(L.tile_h, L.dst.h - T.y0);
        T.col_first = tap_origin<KIND>(L, T.x0, false);
        const int col_last = tap_origin<KIND>(L, T.x0 + T.nx - 1, false) + TAPS - 1;
        T.span_bytes = (col_last - T.col_first + 1) * CC * ES;
        T.cpr = (T.span_bytes + 15 + 15) >> 4;
        if (L.sparse) {
            T.lo = 0;
            T.nslots = TAPS * T.ny;
        } else {
            T.lo = tap_origin<KIND>(L, T.y0, true);
            T.nslots = tap_origin<KIND>(L, T.y0 + T.ny - 1, true) + TAPS - 1 - T.lo + 1;
        }
    }

    // ---- LDS carve-up ----------------------------------------------------
    // xoff[tile_w] int | xw[tile_w][TAPS] (short pairs or floats) |
    // cand_slot[64] int | slot_row[max_slots] int | slot_head[max_slots] int |
    // lut[256*CC] float | rows[max_slots][slot_stride]
    int* xoff = reinterpret_cast<int*>(lds);
    unsigned char* p = lds + ((L.tile_w * 4 + 15) & ~15);
    unsigned char* xw = p;
    const int xw_bytes = (KIND == kLinearFixed) ? L.tile_w * 4 : L.tile_w * TAPS * 4;
    p += (xw_bytes + 15) & ~15;
    int* cand_slot = reinterpret_cast<int*>(p);   // [64] + slot count at [64]
    p += 80 * 4;
    int* slot_row = reinterpret_cast<int*>(p);
    p += ((L.max_slots * 4) + 15) & ~15;
    int* slot_head = reinterpret_cast<int*>(p);
    p += ((L.max_slots * 4) + 15) & ~15;
    float* lut = reinterpret_cast<float*>(p);
    if (kLut) p += 256 * CC * 4;
    unsigned char* rows = p;

    const unsigned char* src_plane = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc rs = make_rsrc(src_plane, L.src.plane_bytes);

    // ---- 1. column taps ----------------------------------------------------
    for (int i = tid; i < T.nx; i += kBlock) {
        const int d = T.x0 + i;
        if (KIND == kLinearFixed) {
            FixedTap t = fixed_tap(d, L.src.w, L.dst.w, L.scale_xf, L.scale_xd, L.mode);
            xoff[i] = (t.i - T.col_first) * CC * ES;
            reinterpret_cast<short2*>(xw)[i] = make_short2((short)t.w0, (short)t.w1);
        } else if (KIND == kLinearFloat) {
            FloatTap t = float_tap(d, L.src.w, L.scale_xf);
            xoff[i] = (t.i - T.col_first) * CC * ES;
            reinterpret_cast<float2*>(xw)[i] = make_float2(t.w0, t.w1);
        } else {
            CubicTap t = cubic_tap(d, L.src.w, L.scale_xd);
            xoff[i] = (t.i - 1 - T.col_first) * CC * ES;
            reinterpret_cast<float4*>(xw)[i] = make_float4(t.c[0], t.c[1], t.c[2], t.c[3]);
        }
    }
    // ---- 2a. which source row lives in which slot --------------------------
    // sparse: only (output row, tap) pairs with a non-zero vertical weight get
    // a slot, compacted by one wave (tile_h * TAPS <= 64); dense: the window
    // [lo, lo + nslots) of consecutive source rows.
    const uint32_t span_off = (uint32_t)(T.col_first * CC * ES) + rs.delta;
    if (L.sparse) {
        if (tid < 64) {
            const int t = tid / TAPS, j = tid - t * TAPS;
            int row = -1;
            if (t < T.ny) {
                VTaps<KIND> v = vtaps<KIND>(L, T.y0 + t);
                if (vweight_nonzero<KIND>(v, j)) row = v.row0 + j;
            }
            const uint64_t m = __ballot(row >= 0);
            const int slot = __popcll(m & ((1ull << tid) - 1ull));
            cand_slot[tid] = row >= 0 ? slot : -1;
            if (tid == 0) cand_slot[64] = __popcll(m);
            if (row >= 0) {
                slot_row[slot] = row;
                slot_head[slot] = (int)(((uint32_t)((int64_t)row * L.src.row_pitch) + span_off) & 15u);
            }
        }
    } else {
        for (int s = tid; s < T.nslots; s += kBlock) {
            const int row = T.lo + s;
            slot_row[s] = row;
            slot_head[s] = (int)(((uint32_t)((int64_t)row * L.src.row_pitch) + span_off) & 15u);
        }
    }
    if (kLut) {
        const int ch_base = (CC == 1) ? plane : 0;
        for (int i = tid; i < 256 * CC; i += kBlock) {
            const int k = i >> 8, v = i & 255;
            float m, sd;
            norm_params(L.norm, img, ch_base + k, m, sd);
            lut[i] = normalize_value((float)v, m, sd);
        }
    }
    __syncthreads();
    if (L.sparse) T.nslots = cand_slot[64];

    // ---- 2b. stage rows: 16-byte loads, all issued before the LDS writes ----
    {
        const int total = T.nslots * T.cpr;
        constexpr int kBatch = 4;
        for (int base = tid; base < total; base += kBlock * kBatch) {
            uint4 v[kBatch];
            int dsto[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const int k = base + b * kBlock;
                dsto[b] = -1;
                if (k < total) {
                    const int s = k / T.cpr, c = k - s * T.cpr;
                    const int row = slot_row[s];
                    if (row >= 0) {
                        const uint32_t off = (uint32_t)((int64_t)row * L.src.row_pitch) + span_off;
                        v[b] = load16(rs, (off & ~15u) + 16u * c);
                        dsto[b] = s * L.slot_stride + 16 * c;
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (dsto[b] >= 0) *reinterpret_cast<uint4*>(rows + dsto[b]) = v[b];
        }
    }
    __syncthreads();

    // ---- 3. compute ---------------------------------------------------------
    unsigned char* dst_plane = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                               (int64_t)plane * L.dst.plane_pitch;
    const int groups = (T.nx + kPx - 1) / kPx;
    const int items = groups * T.ny;

    float nmean[CC], nstd[CC];
    if (OUT == kOutNorm && !kLut) {
#pragma unroll
        for (int k = 0; k < CC; ++k) norm_params(L.norm, img, (CC == 1 ? plane : k), nmean[k], nstd[k]);
    }

    for (int it = tid; it < items; it += kBlock) {
        const int t = it / groups;
        const int g = it - t * groups;
        const VTaps<KIND> v = vtaps<KIND>(L, T.y0 + t);
        // LDS base of each vertical tap's row (or -1 when its weight is 0)
        int rb[TAPS];
#pragma unroll
        for (int j = 0; j < TAPS; ++j) {
            const int s = L.sparse ? cand_slot[t * TAPS + j] : v.row0 + j - T.lo;
            rb[j] = (s >= 0 && vweight_nonzero<KIND>(v, j)) ? s * L.slot_stride + slot_head[s] : -1;
        }

        TOut out[kPx * CC];
#pragma unroll
        for (int q = 0; q < kPx; ++q) {
            const int i = g * kPx + q;
            const int ii = i < T.nx ? i : T.nx - 1;  // clamp; the store masks it
            const int xo = xoff[ii];
            if (KIND == kLinearFixed) {
                const short2 w = reinterpret_cast<const short2*>(xw)[ii];
                const int a0 = w.x, a1 = w.y;
#pragma unroll
                for (int k = 0; k < CC; ++k) {
                    int t0l = 0, t0r = 0, t1l = 0, t1r = 0;
                    if (rb[0] >= 0) {
                        t0l = rows[rb[0] + xo + k];
                        t0r = rows[rb[0] + xo + CC + k];
                    }
                    if (rb[1] >= 0) {
                        t1l = rows[rb[1] + xo + k];
                        t1r = rows[rb[1] + xo + CC + k];
                    }
                    int val;
                    if (L.mode == VACV_LINEAR_REFERENCE) {
                        // resize_naive.cpp:61-64
                        val = (t0l * a0 * v.wi[0] + t1l * a0 * v.wi[1] + t0r * a1 * v.wi[0] + t1r * a1 * v.wi[1]) >> 22;
                        val &= 0xFF;
                    } else {
                        // resize_neon.cpp:103,122-123 then :150-167
                        const int h0 = (int)(short)((t0l * a0 + t0r * a1) >> 4);
                        const int h1 = (int)(short)((t1l * a0 + t1r * a1) >> 4);
                        val = (((h0 * v.wi[0]) >> 16) + ((h1 * v.wi[1]) >> 16) + 2) >> 2;
                        val = clamp_u8(val);
                    }
                    if (OUT == kOutSame) out[q * CC + k] = (TOut)val;
                    else if (OUT == kOutF32) out[q * CC + k] = (TOut)(float)val;
                    else out[q * CC + k] = (TOut)lut[k * 256 + val];
                }
            } else if (KIND == kLinearFloat) {
                const float2 w = reinterpret_cast<const float2*>(xw)[ii];
#pragma unroll
                for (int k = 0; k < CC; ++k) {
                    float t0l = 0.f, t0r = 0.f, t1l = 0.f, t1r = 0.f;
                    if (rb[0] >= 0) {
                        t0l = *reinterpret_cast<const float*>(rows + rb[0] + xo + 4 * k);
                        t0r = *reinterpret_cast<const float*>(rows + rb[0] + xo + 4 * (CC + k));
                    }
                    if (rb[1] >= 0) {
                        t1l = *reinterpret_cast<const float*>(rows + rb[1] + xo + 4 * k);
                        t1r = *reinterpret_cast<const float*>(rows + rb[1] + xo + 4 * (CC + k));
                    }
                    // resize_naive.cpp:121-124, summed left to right
                    float val = t0l * w.x * v.wf[0];
                    val += t1l * w.x * v.wf[1];
                    val += t0r * w.y * v.wf[0];
                    val += t1r * w.y * v.wf[1];
                    if (OUT == kOutNorm) val = normalize_value(val, nmean[k], nstd[k]);
                    out[q * CC + k] = (TOut)val;
                }
            } else {
                const float4 a = reinterpret_cast<const float4*>(xw)[ii];
#pragma unroll
                for (int k = 0; k < CC; ++k) {
                    float h[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        h[j] = 0.f;
                        if (rb[j] >= 0) {
                            const unsigned char* sp = rows + rb[j] + xo + ES * k;
                            float s0, s1, s2, s3;
                            if (ES == 1) {
                                s0 = (float)sp[0]; s1 = (float)sp[CC]; s2 = (float)sp[2 * CC]; s3 = (float)sp[3 * CC];
                            } else {
                                s0 = *reinterpret_cast<const float*>(sp);
                                s1 = *reinterpret_cast<const float*>(sp + 4 * CC);
                                s2 = *reinterpret_cast<const float*>(sp + 8 * CC);
                                s3 = *reinterpret_cast<const float*>(sp + 12 * CC);
                            }
                            // resize_naive.cpp:325-328
                            h[j] = s0 * a.x + s1 * a.y + s2 * a.z + s3 * a.w;
                        }
                    }
                    // resize_naive.cpp:349-351
                    float val = h[0] * v.wf[0] + h[1] * v.wf[1] + h[2] * v.wf[2] + h[3] * v.wf[3];
                    if (OUT == kOutNorm) val = normalize_value(val, nmean[k], nstd[k]);
                    out[q * CC + k] = (TOut)val;
                }
            }
        }

        // ---- store ---------------------------------------------------------
        const int x = T.x0 + g * kPx;
        unsigned char* dp = dst_plane + (int64_t)(T.y0 + t) * L.dst.row_pitch + (int64_t)x * CC * sizeof(TOut);
        const int valid = min(kPx, T.nx - g * kPx);
        constexpr int kBytes = kPx * CC * (int)sizeof(TOut);
        if (valid == kPx && (kBytes % 16 == 0) && ((reinterpret_cast<uintptr_t>(dp) & 15) == 0)) {
#pragma unroll
            for (int b = 0; b < kBytes / 16; ++b)
                reinterpret_cast<uint4*>(dp)[b] = reinterpret_cast<const uint4*>(out)[b];
        } else if (valid == kPx && (kBytes % 4 == 0) && ((reinterpret_cast<uintptr_t>(dp) & 3) == 0)) {
#pragma unroll
            for (int b = 0; b < kBytes / 4; ++b)
                reinterpret_cast<uint32_t*>(dp)[b] = reinterpret_cast<const uint32_t*>(out)[b];
        } else {
            TOut* o = reinterpret_cast<TOut*>(dp);
#pragma unroll
            for (int e = 0; e < kPx * CC; ++e)
                if (e < valid * CC) o[e] = out[e];
        }
    }
}

template <int KIND, int CC, typename TIn, int OUT>
hipError_t launch_one(const ResizeLaunch& L, hipStream_t s) {
    dim3 grid(L.tiles_x * L.tiles_y, L.n * L.src.planes);
    hipLaunchKernelGGL((resize_kernel<KIND, CC, TIn, OUT>), grid, dim3(kBlock), L.lds_bytes, s, L);
    return hipGetLastError();
}

template <int KIND, typename TIn, int OUT>
hipError_t launch_cc(const ResizeLaunch& L, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<KIND, 1, TIn, OUT>(L, s);
        case 2: return launch_one<KIND, 2, TIn, OUT>(L, s);
        case 3: return launch_one<KIND, 3, TIn, OUT>(L, s);
        case 4: return launch_one<KIND, 4, TIn, OUT>(L, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_resize(const ResizeLaunch& L, hipStream_t s) {
    if (L.kind == kLinearFixed) {
        if (L.out == kOutSame) return launch_cc<kLinearFixed, uint8_t, kOutSame>(L, s);
        if (L.out == kOutF32) return launch_cc<kLinearFixed, uint8_t, kOutF32>(L, s);
        return launch_cc<kLinearFixed, uint8_t, kOutNorm>(L, s);
    }
    if (L.kind == kLinearFloat) {
        if (L.out == kOutNorm) return launch_cc<kLinearFloat, float, kOutNorm>(L, s);
        return launch_cc<kLinearFloat, float, kOutSame>(L, s);
    }
    if (L.src.esize == 1) {
        if (L.out == kOutNorm) return launch_cc<kCubic, uint8_t, kOutNorm>(L, s);
        return launch_cc<kCubic, uint8_t, kOutF32>(L, s);
    }
    if (L.out == kOutNorm) return launch_cc<kCubic, float, kOutNorm>(L, s);
    return launch_cc<kCubic, float, kOutSame>(L, s);
}

}  // namespace vacv
