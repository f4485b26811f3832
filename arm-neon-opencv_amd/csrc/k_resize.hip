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
//   * every lane produces 4 consecutive output ELEMENTS, so each wave store
//     is 64 contiguous 16-byte (fp32) or 4-byte (u8) chunks.
// Rows whose vertical weight is zero are never read: at an exact 3x
// downscale only every third source row moves (B_alg).
#pragma clang fp contract(off)

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kElems = 4;      // output elements per work item
constexpr int kMaxChunks = 8;  // 16-byte prefetch registers per thread (planner bound)

// 16 bytes at byte offset o (from the 16-aligned base) with a clean tail: a
// raw-buffer load that straddles num_records returns all zeros, so the
// chunk that crosses the end of a plane is assembled byte by byte.
__device__ __forceinline__ uint4 load16_safe(const Rsrc& rs, uint32_t o, uint32_t limit) {
    if (o + 16u <= limit) return load16(rs, o);
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

template <int KIND, int CC, typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock)
resize_kernel(ResizeLaunch L) {
    constexpr int TAPS = (KIND == kCubic) ? 4 : 2;
    constexpr int ES = sizeof(TIn);
    constexpr bool kLut = (KIND == kLinearFixed) && (OUT == kOutNorm);
    constexpr int XW = (KIND == kLinearFixed) ? 4 : (KIND == kLinearFloat ? 8 : 16);
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;

    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;

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

    // ---- LDS carve-up: xoff | xw | rowinfo[32][8] | head[max_slots] | lut | rows ------
    int* xoff_l = reinterpret_cast<int*>(lds);
    unsigned char* p = lds + ((L.tile_w * 4 + 15) & ~15);
    unsigned char* xw_l = p;
    p += (L.tile_w * XW + 15) & ~15;
    int* rowinfo_l = reinterpret_cast<int*>(p);   // [tile_h][8]
    p += 32 * 8 * 4;
    int* head_l = reinterpret_cast<int*>(p);
    p += (L.max_slots * 4 + 15) & ~15;
    float* lut_l = reinterpret_cast<float*>(p);
    if (kLut) p += L.norm.c_total * 256 * 4;
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

    // ---- per-strip tables (overlap the first task's loads) ------------------
    for (int i = tid; i < nx; i += kBlock) {
        const int e = tx * L.tile_w + i;
        xoff_l[i] = L.plan.xoff[e];
        if (XW == 4) reinterpret_cast<uint32_t*>(xw_l)[i] = reinterpret_cast<const uint32_t*>(L.plan.xw)[e];
        else if (XW == 8) reinterpret_cast<uint2*>(xw_l)[i] = reinterpret_cast<const uint2*>(L.plan.xw)[e];
        else reinterpret_cast<uint4*>(xw_l)[i] = reinterpret_cast<const uint4*>(L.plan.xw)[e];
    }
    if (kLut) {
        for (int i = tid; i < L.norm.c_total * 256; i += kBlock) {
            if (L.plan.lut) {
                lut_l[i] = L.plan.lut[i];
            } else {
                float m, sd;
                norm_params(L.norm, img, i >> 8, m, sd);
                lut_l[i] = normalize_value((float)(i & 255), m, sd);
            }
        }
    }
    float nmean[CC], nstd[CC];
    if (OUT == kOutNorm && !kLut) {
#pragma unroll
        for (int k = 0; k < CC; ++k) norm_params(L.norm, img, (CC == 1 ? plane % L.norm.c_total : k), nmean[k], nstd[k]);
    }
    const int lut_base = (CC == 1) ? (plane % max(L.norm.c_total, 1)) * 256 : 0;

    unsigned char* dst_plane = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                               (int64_t)plane * L.dst.plane_pitch;
    const int row_elems = nx * CC;
    const int ipr = (row_elems + kElems - 1) / kElems;  // items per output row

    for (int task = task0; task < task1; ++task) {
        if (task != task0) __syncthreads();  // everyone is done reading the previous tile
        // ---- registers -> LDS, per-row tap info ----------------------------
        {
            const int ns = L.plan.task_nslots[task];
#pragma unroll
            for (int m = 0; m < kMaxChunks; ++m)
                if (ch_s[m] < ns) *reinterpret_cast<uint4*>(rows_l + ch_s[m] * L.slot_stride + 16 * ch_c[m]) = R[m];
            if (tid < ns) {
                const int row = L.plan.task_rows[(int64_t)task * L.max_slots + tid];
                head_l[tid] = (int)(((uint32_t)((int64_t)row * rp) + span_off) & 15u);
            }
        }
        __syncthreads();
        // rowinfo[t] = LDS byte offset of each vertical tap's row (-1: weight 0)
        // followed by the TAPS weights
        const int y0 = task * L.tile_h;
        const int ny = min(L.tile_h, L.dst.h - y0);
        if (tid < ny) {
            const int nc = L.tile_h * TAPS;
            int* ri = rowinfo_l + tid * 8;
#pragma unroll
            for (int q = 0; q < TAPS; ++q) {
                const int sl = L.plan.task_cand[(int64_t)task * nc + tid * TAPS + q];
                ri[q] = sl >= 0 ? sl * L.slot_stride + head_l[sl] : -1;
            }
            if (KIND == kLinearFixed) {
                const int2 w = reinterpret_cast<const int2*>(L.plan.yw)[y0 + tid];
                ri[4] = w.x; ri[5] = w.y;
            } else if (KIND == kLinearFloat) {
                const float2 w = reinterpret_cast<const float2*>(L.plan.yw)[y0 + tid];
                ri[4] = __float_as_int(w.x); ri[5] = __float_as_int(w.y);
            } else {
                const float4 w = reinterpret_cast<const float4*>(L.plan.yw)[y0 + tid];
                ri[4] = __float_as_int(w.x); ri[5] = __float_as_int(w.y);
                ri[6] = __float_as_int(w.z); ri[7] = __float_as_int(w.w);
            }
        }
        __syncthreads();
        if (task + 1 < task1) prefetch(task + 1);  // in flight during this tile's compute

        // ---- compute this tile ------------------------------------------------
        const int items = ny * ipr;
        int t = tid / ipr;
        int j = tid - t * ipr;
        for (int it = tid; it < items; it += kBlock) {
            const int dy = y0 + t;
            const int4 ra = *reinterpret_cast<const int4*>(rowinfo_l + t * 8);
            const int4 rw = *reinterpret_cast<const int4*>(rowinfo_l + t * 8 + 4);
            int rb[4] = {ra.x, ra.y, ra.z, ra.w};
            const int wyi[2] = {rw.x, rw.y};
            const float wyf[4] = {__int_as_float(rw.x), __int_as_float(rw.y), __int_as_float(rw.z), __int_as_float(rw.w)};

            TOut out[kElems];
#pragma unroll
            for (int q = 0; q < kElems; ++q) {
                int e = j * kElems + q;
                e = e < row_elems ? e : row_elems - 1;  // clamp; the store masks it
                const int px = e / CC;
                const int k = e - px * CC;
                const int xo = xoff_l[px] + k * ES;
                if (KIND == kLinearFixed) {
                    const uint32_t wx = reinterpret_cast<const uint32_t*>(xw_l)[px];
                    const int a0 = (int)(short)(wx & 0xFFFFu), a1 = (int)(short)(wx >> 16);
                    int t0l = 0, t0r = 0, t1l = 0, t1r = 0;
                    if (rb[0] >= 0) { t0l = rows_l[rb[0] + xo]; t0r = rows_l[rb[0] + xo + CC]; }
                    if (rb[1] >= 0) { t1l = rows_l[rb[1] + xo]; t1r = rows_l[rb[1] + xo + CC]; }
                    int val;
                    if (L.mode == VACV_LINEAR_REFERENCE) {
                        // resize_naive.cpp:61-64 (truncating >> 22, stored as a byte)
                        val = ((t0l * a0 * wyi[0] + t1l * a0 * wyi[1] + t0r * a1 * wyi[0] + t1r * a1 * wyi[1]) >> 22) & 0xFF;
                    } else {
                        // resize_neon.cpp:103,122-123 (int16 rows) then :150-167
                        const int h0 = (int)(short)((t0l * a0 + t0r * a1) >> 4);
                        const int h1 = (int)(short)((t1l * a0 + t1r * a1) >> 4);
                        val = clamp_u8((((h0 * wyi[0]) >> 16) + ((h1 * wyi[1]) >> 16) + 2) >> 2);
                    }
                    if (OUT == kOutSame) out[q] = (TOut)val;
                    else if (OUT == kOutF32) out[q] = (TOut)(float)val;
                    else out[q] = (TOut)lut_l[lut_base + (CC == 1 ? 0 : k * 256) + val];
                } else if (KIND == kLinearFloat) {
                    const float2 wx = reinterpret_cast<const float2*>(xw_l)[px];
                    float t0l = 0.f, t0r = 0.f, t1l = 0.f, t1r = 0.f;
                    if (rb[0] >= 0) {
                        t0l = *reinterpret_cast<const float*>(rows_l + rb[0] + xo);
                        t0r = *reinterpret_cast<const float*>(rows_l + rb[0] + xo + 4 * CC);
                    }
                    if (rb[1] >= 0) {
                        t1l = *reinterpret_cast<const float*>(rows_l + rb[1] + xo);
                        t1r = *reinterpret_cast<const float*>(rows_l + rb[1] + xo + 4 * CC);
                    }
                    // resize_naive.cpp:121-124, summed left to right
                    float val = t0l * wx.x * wyf[0];
                    val += t1l * wx.x * wyf[1];
                    val += t0r * wx.y * wyf[0];
                    val += t1r * wx.y * wyf[1];
                    if (OUT == kOutNorm) val = normalize_value(val, nmean[k], nstd[k]);
                    out[q] = (TOut)val;
                } else {
                    const float4 a = reinterpret_cast<const float4*>(xw_l)[px];
                    float h[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        h[r] = 0.f;
                        if (rb[r] >= 0) {
                            const unsigned char* sp = rows_l + rb[r] + xo;
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
                            h[r] = s0 * a.x + s1 * a.y + s2 * a.z + s3 * a.w;
                        }
                    }
                    // resize_naive.cpp:349-351
                    float val = h[0] * wyf[0] + h[1] * wyf[1] + h[2] * wyf[2] + h[3] * wyf[3];
                    if (OUT == kOutNorm) val = normalize_value(val, nmean[k], nstd[k]);
                    out[q] = (TOut)val;
                }
            }

            // ---- store 4 consecutive elements --------------------------------
            unsigned char* dp = dst_plane + (int64_t)dy * L.dst.row_pitch +
                                ((int64_t)x0 * CC + (int64_t)j * kElems) * (int64_t)sizeof(TOut);
            const int valid = min(kElems, row_elems - j * kElems);
            if (sizeof(TOut) == 4) {
                if (valid == kElems && (reinterpret_cast<uintptr_t>(dp) & 15) == 0) {
                    *reinterpret_cast<uint4*>(dp) = *reinterpret_cast<const uint4*>(out);
                } else {
#pragma unroll
                    for (int q = 0; q < kElems; ++q)
                        if (q < valid) reinterpret_cast<TOut*>(dp)[q] = out[q];
                }
            } else {
                if (valid == kElems && (reinterpret_cast<uintptr_t>(dp) & 3) == 0) {
                    const uint32_t v = (uint32_t)(uint8_t)out[0] | ((uint32_t)(uint8_t)out[1] << 8) |
                                       ((uint32_t)(uint8_t)out[2] << 16) | ((uint32_t)(uint8_t)out[3] << 24);
                    *reinterpret_cast<uint32_t*>(dp) = v;
                } else {
#pragma unroll
                    for (int q = 0; q < kElems; ++q)
                        if (q < valid) reinterpret_cast<TOut*>(dp)[q] = out[q];
                }
            }
            j += kBlock;
            while (j >= ipr) { j -= ipr; ++t; }
        }
    }
}

template <int KIND, int CC, typename TIn, int OUT>
hipError_t launch_one(const ResizeLaunch& L, hipStream_t s) {
    const int64_t blocks = (int64_t)L.n * L.src.planes * L.tiles_x * L.strips;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL((resize_kernel<KIND, CC, TIn, OUT>), dim3((unsigned)blocks), dim3(kBlock), L.lds_bytes, s, L);
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
