// k_lanczos.hip -- INTER_LANCZOS4 resize (u8 / fp32 in; same-type, fp32 or
// normalised fp32 out).
//
// The reference hands every interpolation but LINEAR / CUBIC to cv::resize
// (resize.cpp:46-48; cv.h:33 names INTER_LANCZOS4), which recurses forever
// without OpenCV.  Restated from OpenCV 2.4's cv::resize (imgwarp.cpp:
// interpolateLanczos4, the xofs / alpha / yofs / beta tables of resize(),
// resizeGeneric_ with HResizeLanczos4 and VResizeLanczos4); parity unpinned,
// no reference entry or fixture runs OpenCV here (the test-side restatement
// is independent of this file).
//  * Tables (host, once per geometry, cached on the device like the
//    INTER_AREA tables): per output column the tap origin sx = floor(fx)
//    (fx = (float)((dx + 0.5) * scale_x - 0.5)) and 8 coefficients, per
//    output row sy and 8 coefficients.  u8: coefficients
//    saturate_cast<short>(c * 2048); fp32: the float coefficients.
//  * Horizontal pass (HResizeLanczos4): per source row and output column the
//    8 taps sx - 3 .. sx + 4 of each channel (an out-of-range tap walks by cn
//    to the nearest pixel of its channel: a clamp), summed in tap order --
//    int for u8, fp32 for fp32 (columns outside [xmin, xmax) start from
//    0 +, as OpenCV's border loop does).
//  * Vertical pass (VResizeLanczos4): rows clip(sy - 3 + k, 0, h - 1); u8 in
//    int (order immaterial), rounded by FixedPtCast<int, uchar, 22>; fp32:
//    elements e < (dst.w * cn & ~3) as the 4-wide NEON loop of
//    VResizeLanczos4Vec_32f, (b0 h0 + .. + b3 h3) + (b4 h4 + .. + b7 h7),
//    the rest as the scalar tail, b0 h0 + b1 h1 + .. + b7 h7 left to right.
// Shape (as resizeGeneric_ itself): a wave owns a strip of 64 output columns
// (one per lane) and a band of output rows and walks down it.  Each source
// row the band needs is resized horizontally ONCE -- per lane one
// dword-aligned window load of its 8 CC tap bytes (u8) or 8 CC floats --
// into the lane's own slot of an 8-row LDS ring (row r -> slot r mod 8);
// an output row then reads its 8 rows' values from the ring.  Every lane
// reads and writes only its own ring entries: no barriers.  At a 3x
// downscale that is ~3 horizontal rows per output row instead of the 8 a
// per-output-element gather pays, and no table reads per tap.
#pragma clang fp contract(off)

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "vacv_device.hpp"

namespace vacv {
namespace {

struct LanczosTabsDev {
    const int* xofs;     // [dst.w]: floor(fx)
    const short* xai;    // [dst.w][8] u8 coefficients
    const float* xaf;    // [dst.w][8] fp32 coefficients
    const int* yofs;     // [dst.h]
    const short* yai;    // [dst.h][8]
    const int* yrot;     // [dst.h][4] u8: the 8 coefficients per ring SLOT (row mod 8) as short pairs
    const float* yaf;    // [dst.h][8]
    const int* yrec;     // [dst.h][16] u8, lanczos_u8_kernel: [0, 8) the coefficients by slot (row - rs) & 7, rs
                         // the first source row of the row's band; [8] its last tap row; [9] 1 if row y + 1's
                         // last tap row is the same
    int xmin, xmax;      // output columns [xmin, xmax) take the unrolled horizontal sum
    int run_ni;          // lanczos_u8_kernel: 16-byte loads per lane of a staged run (0: per-lane windows)
};

struct LanczosLaunch {
    PlaneGeom src, dst;
    int n;
    int out;
    NormSpec norm;
    LanczosTabsDev t;
};

// A lane's horizontal taps as an 8-pixel WINDOW of its source row, starting
// at column wstart = clamp(sx - 3, 0, w - 8): tap j is window pixel
// clamp(j + SH, 0, 7) with SH = (sx - 3) - wstart in [-4, 4] -- 0 for the
// interior columns (OpenCV's unrolled loop), else the border clamp (its
// `sxj += cn` walk).  Every lane's row data is then one window load, the
// same shape for all lanes, which is what lets the loads run ahead.
template <int SH>
__device__ __forceinline__ constexpr int lz_pos(int j) {
    return j + SH < 0 ? 0 : (j + SH > 7 ? 7 : j + SH);
}

// u8: the window's bytes (after the byte shift) in NW dwords; the 8 taps of a
// channel as 4 packed-u16 pairs (v_perm_b32) against the coefficient pairs
// (v_dot2_i32_i16): int sums, the order is immaterial
typedef short sh2 __attribute__((ext_vector_type(2)));
template <int CC, int SH, int NW>
__device__ __forceinline__ void lz_h_u8(const uint32_t* wv, const uint32_t (&cp)[4], int (&hv)[CC]) {
#pragma unroll
    for (int k = 0; k < CC; ++k) {
        int v = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            constexpr int dummy = 0;
            (void)dummy;
            const int e0 = lz_pos<SH>(2 * m) * CC + k, e1 = lz_pos<SH>(2 * m + 1) * CC + k;
            const int q0 = e0 >> 2;
            const uint32_t lo = wv[q0], hi = q0 + 1 < NW ? wv[q0 + 1] : 0u;
            const uint32_t sel = (uint32_t)(e0 - 4 * q0) | (0x0Cu << 8) | ((uint32_t)(e1 - 4 * q0) << 16) | (0x0Cu << 24);
            const uint32_t pr = __builtin_amdgcn_perm(hi, lo, sel);
            v = __builtin_amdgcn_sdot2(__builtin_bit_cast(sh2, pr), __builtin_bit_cast(sh2, cp[m]), v, false);
        }
        hv[k] = v;
    }
}

// fp32: the window's 8 CC floats; HResizeLanczos4's sum in tap order, from
// 0 + in the border loop (SH != 0)
template <int CC, int SH>
__device__ __forceinline__ void lz_h_f32(const float* wf, const float (&c)[8], float (&hv)[CC]) {
#pragma unroll
    for (int k = 0; k < CC; ++k) {
        float a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = wf[lz_pos<SH>(j) * CC + k] * c[j];
        float v = SH == 0 ? a[0] : 0.f + a[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) v = v + a[j];
        hv[k] = v;
    }
}

// The per-row tables are read through the constant address space: their
// indices are wave-uniform, so these are scalar loads -- as vector loads they
// would be counted behind the in-flight row windows and wait for all of them.
template <typename T>
__device__ __forceinline__ T lz_const(const T* p, int i) {
    return ((const __attribute__((address_space(4))) T*)(uintptr_t)p)[i];
}

constexpr int kLzWaves = 4;  // waves (strip tasks) per workgroup; each owns its own ring
constexpr int kLzD = 3;      // u8 source rows in flight per wave (1 / 2 / 3 / 4 / 6 / 8: 0.580 / 0.522 / 0.495 / 0.525 / 0.534 / 0.565 ms)
template <typename TIn, int OUT, int CC>
__global__ void __launch_bounds__(64 * kLzWaves) lanczos_kernel(LanczosLaunch L, int strips, int bands, int band_rows, int blocks, int xcd_per) {
    constexpr bool U8 = std::is_same<TIn, uint8_t>::value;
    using TW = typename std::conditional<U8, int, float>::type;
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    // the row window in registers: u8 8 CC bytes at any byte offset, fp32 8 CC floats
    constexpr int ND = U8 ? (8 * CC + 6) / 4 : 8 * CC;
    // source rows in flight per wave (the loads of rows r + 1 .. r + D - 1
    // run while row r is resized)
    constexpr int D = U8 ? kLzD : 2;
    // per wave: 8 source rows x 64 columns x RS (padding c = 3 to 4, for one
    // 16-byte LDS access per lane and row, cost a workgroup per CU of LDS:
    // 0.589 vs 0.530 ms)
    constexpr int RS = CC;
    __shared__ __attribute__((aligned(16))) TW ring[kLzWaves][8][64 * RS];

    // wave-uniform, and said so: the plane's buffer resource stays in SGPRs
    // (derived from a per-lane value it would be waterfalled at every load)
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = (int)(threadIdx.x & 63);
    // xcd_per > 0: XCD-contiguous order -- workgroup b runs on XCD b % 8, and
    // each XCD takes a run of xcd_per consecutive workgroups, so the strips
    // that share the 128-byte lines at their windows' edges (a window reaches
    // 7 pixels past the strip) are fetched into one L2, not two
    const int blk = xcd_per > 0 ? (int)(blockIdx.x % 8) * xcd_per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    if (blk >= blocks) return;  // whole workgroup: the grid's round-up to 8
    const int task = blk * kLzWaves + wave;  // (plane, band, strip), strip fastest
    const int strip = task % strips;
    const int rest = task / strips;
    const int band = rest % bands;
    const int pidx = rest / bands;
    if (pidx >= L.n * L.src.planes) return;  // whole wave
    const int y0 = band * band_rows, y1 = min(y0 + band_rows, L.dst.h);
    const int x = strip * 64 + lane;
    const bool live = x < L.dst.w;
    const int xc = live ? x : L.dst.w - 1;  // idle lanes resize a valid column and store nothing
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int w = L.src.w, h = L.src.h;
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp = (uint32_t)L.src.row_pitch;  // plane < 2^31 bytes (kMaxPlaneBytes)

    // this column's window and coefficients (the host guarantees w >= 8)
    const int sx = L.t.xofs[xc];
    const int wstart = min(max(sx - 3, 0), w - 8);
    const int shift = (sx - 3) - wstart;  // [-4, 4]; 0 <=> OpenCV's [xmin, xmax)
    TW c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if constexpr (U8) c[j] = (int)L.t.xai[8 * xc + j];
        else c[j] = L.t.xaf[8 * xc + j];
    }
    uint32_t cp[4];  // u8: the coefficients as (c[2m], c[2m + 1]) short pairs
#pragma unroll
    for (int m = 0; m < 4; ++m) cp[m] = ((uint32_t)c[2 * m] & 0xFFFFu) | ((uint32_t)c[2 * m + 1] << 16);
    const uint32_t wbyte = (uint32_t)(wstart * CC * (int)sizeof(TIn)) + srs.delta;
    const uint32_t wsh = wbyte & 3u;  // u8: the window's byte offset in its first dword
    // uniform: every lane of the strip takes the unrolled sum (shift 0) -- all
    // strips but the image's first and last.  The per-lane switch below would
    // otherwise run its 9-way exec-mask chain for every source row (PMC: the
    // kernel issued more scalar than vector instructions).
    const bool interior = __builtin_amdgcn_ballot_w64(shift != 0) == 0;

    // the window of source row r (issued; consumed by hrow).  SAFE: the
    // window may reach past the plane's last byte (only in the waves holding
    // the plane's last row and right-most columns), so those dwords are read
    // bytewise -- an overhanging 16-byte load reads as zeros.
    auto load = [&](auto safe_c, uint32_t (&d)[ND], int r) {
        constexpr bool SAFE = decltype(safe_c)::value;
        const uint32_t a = (uint32_t)r * rp + (wbyte & ~3u);
        if (!SAFE || a + 4u * ND <= slimit) {
            int q = 0;
#pragma unroll
            for (; q + 4 <= ND; q += 4) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)(a + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1]; d[q + 2] = v[2]; d[q + 3] = v[3];
            }
            if constexpr (ND % 4 == 3) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b96(srs.r, (int)(a + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1]; d[q + 2] = v[2];
            } else if constexpr (ND % 4 == 2) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(srs.r, (int)(a + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1];
            } else if constexpr (ND % 4 == 1) {
                d[q] = __builtin_amdgcn_raw_buffer_load_b32(srs.r, (int)(a + 4 * q), 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < ND; ++q) {
                uint32_t v = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (a + 4u * q + e < slimit)
                        v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(a + 4u * q + e), 0, 0) << (8 * e);
                d[q] = v;
            }
        }
    };
    // HResizeLanczos4 of the loaded window -> ring slot
    auto hrow = [&](const uint32_t (&d)[ND], int slot) {
        TW hv[CC];
        if constexpr (U8) {
            uint32_t wv[ND - 1];
#pragma unroll
            for (int q = 0; q < ND - 1; ++q) wv[q] = __builtin_amdgcn_alignbyte(d[q + 1], d[q], wsh);
            if (interior) lz_h_u8<CC, 0, ND - 1>(wv, cp, hv);
            else switch (shift) {  // divergent: the strips at the image's edges
                case -4: lz_h_u8<CC, -4, ND - 1>(wv, cp, hv); break;
                case -3: lz_h_u8<CC, -3, ND - 1>(wv, cp, hv); break;
                case -2: lz_h_u8<CC, -2, ND - 1>(wv, cp, hv); break;
                case -1: lz_h_u8<CC, -1, ND - 1>(wv, cp, hv); break;
                case 1: lz_h_u8<CC, 1, ND - 1>(wv, cp, hv); break;
                case 2: lz_h_u8<CC, 2, ND - 1>(wv, cp, hv); break;
                case 3: lz_h_u8<CC, 3, ND - 1>(wv, cp, hv); break;
                case 4: lz_h_u8<CC, 4, ND - 1>(wv, cp, hv); break;
                default: lz_h_u8<CC, 0, ND - 1>(wv, cp, hv); break;
            }
        } else {
            float wf[ND];
            // (__builtin_bit_cast(float, v[i]) of a vector element read element 0
            // for every i with this compiler, ROCm 7.2 clang: scalars only here)
#pragma unroll
            for (int q = 0; q < ND; ++q) wf[q] = __uint_as_float(d[q]);
            if (interior) lz_h_f32<CC, 0>(wf, c, hv);
            else switch (shift) {
                case -4: lz_h_f32<CC, -4>(wf, c, hv); break;
                case -3: lz_h_f32<CC, -3>(wf, c, hv); break;
                case -2: lz_h_f32<CC, -2>(wf, c, hv); break;
                case -1: lz_h_f32<CC, -1>(wf, c, hv); break;
                case 1: lz_h_f32<CC, 1>(wf, c, hv); break;
                case 2: lz_h_f32<CC, 2>(wf, c, hv); break;
                case 3: lz_h_f32<CC, 3>(wf, c, hv); break;
                case 4: lz_h_f32<CC, 4>(wf, c, hv); break;
                default: lz_h_f32<CC, 0>(wf, c, hv); break;
            }
        }
#pragma unroll
        for (int k = 0; k < CC; ++k) ring[wave][slot][lane * RS + k] = hv[k];
        if constexpr (RS > CC) ring[wave][slot][lane * RS + CC] = 0;
    };

    const int dw = L.dst.w * CC;
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const Rsrc drs = make_rsrc(dp, L.dst.plane_bytes);
    const bool dst_al = ((reinterpret_cast<uintptr_t>(dp) | (uintptr_t)L.dst.row_pitch) & 3) == 0;
    const bool full = strip * 64 + 64 <= L.dst.w;  // uniform: every lane of the strip is live
    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }

    constexpr uint32_t kOobStore = 0x80000000u;  // a store offset past every plane: dropped
    // VResizeLanczos4 of output row y from the ring, and its store
    auto emit = [&](int y) {
        TOut o[CC];
        if constexpr (U8) {
            // The u8 sum is int arithmetic (wrapping, order immaterial), so it
            // is taken per ring SLOT: all 8 slots in a fixed order, from one
            // base address with immediate offsets, against the row's
            // coefficients regrouped by slot on the host (yrot: a clamped
            // border tap adds its coefficient to its row's slot; a slot no tap
            // reads gets 0).  No per-row slot arithmetic on the scalar unit.
            int hs[8][CC];
            int bb[8];
            if constexpr (OUT != kOutNorm) {  // (normalising: 0.647 vs 0.599 ms, registers)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
#pragma unroll
                    for (int q = 0; q < CC; ++q) hs[j][q] = ring[wave][j][lane * RS + q];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int wd = lz_const(L.t.yrot, 4 * y + k);
                    bb[2 * k] = (int)(short)(wd & 0xFFFF);
                    bb[2 * k + 1] = wd >> 16;
                }
            } else {  // A/B: the taps in tap order, slots clamped per row
                const int sy = lz_const(L.t.yofs, y);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int slot = min(max(sy - 3 + k, 0), h - 1) & 7;
#pragma unroll
                    for (int q = 0; q < CC; ++q) hs[k][q] = ring[wave][slot][lane * RS + q];
                }
                const int* b32 = reinterpret_cast<const int*>(L.t.yai);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int wd = lz_const(b32, 4 * y + k);
                    bb[2 * k] = (int)(short)(wd & 0xFFFF);
                    bb[2 * k + 1] = wd >> 16;
                }
            }
#pragma unroll
            for (int q = 0; q < CC; ++q) {
                // |h| < 2^23 (255 x sum |coefficient| <= 255 x ~2,900) and |b| < 2^12
                // (a slot's summed coefficients too): 24-bit multiplies, whose low
                // 32 bits are the int product (wrapping as OpenCV's int arithmetic does)
                const int s0 = __mul24(hs[0][q], bb[0]) + __mul24(hs[1][q], bb[1]) + __mul24(hs[2][q], bb[2]) +
                               __mul24(hs[3][q], bb[3]);
                const int s1 = __mul24(hs[4][q], bb[4]) + __mul24(hs[5][q], bb[5]) + __mul24(hs[6][q], bb[6]) +
                               __mul24(hs[7][q], bb[7]);
                const int vi = min(max((s0 + s1 + (1 << 21)) >> 22, 0), 255);  // FixedPtCast<int, uchar, 22>
                if (OUT == kOutSame) o[q] = (TOut)vi;
                else if (OUT == kOutF32) o[q] = (TOut)(float)vi;
                else o[q] = (TOut)normalize_u8v(cn[q], vi);
            }
        } else {
            const int sy = lz_const(L.t.yofs, y);
            TW hs[8][CC];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int slot = min(max(sy - 3 + k, 0), h - 1) & 7;
#pragma unroll
                for (int q = 0; q < CC; ++q) hs[k][q] = ring[wave][slot][lane * RS + q];
            }
            float bb[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) bb[k] = lz_const(L.t.yaf, 8 * y + k);
#pragma unroll
            for (int q = 0; q < CC; ++q) {
                float v;
                if (x * CC + q < (dw & ~3)) {  // VResizeLanczos4Vec_32f's 4-wide loop
                    const float s0 = ((hs[0][q] * bb[0] + hs[1][q] * bb[1]) + hs[2][q] * bb[2]) + hs[3][q] * bb[3];
                    const float s1 = ((hs[4][q] * bb[4] + hs[5][q] * bb[5]) + hs[6][q] * bb[6]) + hs[7][q] * bb[7];
                    v = s0 + s1;
                } else {  // the scalar tail
                    v = hs[0][q] * bb[0];
#pragma unroll
                    for (int k = 1; k < 8; ++k) v = v + hs[k][q] * bb[k];
                }
                if (OUT == kOutNorm) v = normalize_f(cn[q], v);
                o[q] = (TOut)v;
            }
        }
        uint32_t orow = (uint32_t)y * (uint32_t)L.dst.row_pitch + drs.delta;
        if constexpr (sizeof(TOut) == 1) {
            // u8: the quad's 4 CC bytes as CC dword stores (quad_pack) where the
            // quad is whole and the destination dword-aligned, else bytes
            uint32_t own = 0;
#pragma unroll
            for (int q = 0; q < CC; ++q) own |= (uint32_t)(uint8_t)o[q] << (8 * q);
            const int xq = x & ~3;
            const bool quad = dst_al && (full || xq + 4 <= L.dst.w);  // uniform per quad; per wave where full
            const uint32_t word = quad_pack<CC>(own, lane & 3);
            if (dst_al && full) {
                if ((lane & 3) < CC)
                    __builtin_amdgcn_raw_buffer_store_b32(word, drs.r, (int)(orow + (uint32_t)(xq * CC + 4 * (lane & 3))),
                                                          0, 0);
            } else if (quad) {
                if ((lane & 3) < CC)
                    __builtin_amdgcn_raw_buffer_store_b32(word, drs.r, (int)(orow + (uint32_t)(xq * CC + 4 * (lane & 3))),
                                                          0, 0);
            } else if (live) {
#pragma unroll
                for (int q = 0; q < CC; ++q)
                    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(own >> (8 * q)), drs.r,
                                                         (int)(orow + (uint32_t)(x * CC + q)), 0, 0);
            }
        } else if (live) {
            const uint32_t off = orow + (uint32_t)(x * CC) * 4u;
            uint32_t ov[CC];
#pragma unroll
            for (int q = 0; q < CC; ++q) ov[q] = __float_as_uint(o[q]);
            if (dst_al) {
                if constexpr (CC == 1) {
                    __builtin_amdgcn_raw_buffer_store_b32(ov[0], drs.r, (int)off, 0, 0);
                } else if constexpr (CC == 2) {
                    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{ov[0], ov[1]}, drs.r, (int)off, 0, 0);
                } else if constexpr (CC == 3) {
                    typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                    __builtin_amdgcn_raw_buffer_store_b96(u32x3{ov[0], ov[1], ov[2]}, drs.r, (int)off, 0, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{ov[0], ov[1], ov[2], ov[3]}, drs.r, (int)off, 0, 0);
                }
            } else {
                TOut* dq = reinterpret_cast<TOut*>(dp + (off - drs.delta));
#pragma unroll
                for (int q = 0; q < CC; ++q) dq[q] = o[q];
            }
        }
    };

    // Walk the band's source rows in order, D windows in flight; after row rr
    // is in the ring, emit every output row whose last tap row is rr.  Row rr
    // overwrites slot rr mod 8, whose row rr - 8 no pending output reads (an
    // output's 8 rows are consecutive rows, clamped).  Every step issues its
    // load (past the band's last row: the last row again), so the compiler's
    // wait for window u leaves the D - 1 later windows in flight.
    const int rs = max(lz_const(L.t.yofs, y0) - 3, 0);
    const int re = min(lz_const(L.t.yofs, y1 - 1) + 4, h - 1);
    auto walk = [&](auto safe_c) {
        int y = __builtin_amdgcn_readfirstlane(y0);
        int need = min(lz_const(L.t.yofs, y) + 4, h - 1);  // the last row output y taps
        uint32_t buf[D][ND];
#pragma unroll
        for (int u = 0; u < D; ++u) load(safe_c, buf[u], min(rs + u, re));
        // D - 1 dropped stores after the prologue's windows: the path into
        // the loop then has the steady state's shape (a store per step after
        // each window), and the compiler's wait for a window is not the
        // vmcnt(0) the prologue path alone would need
#pragma unroll
        for (int u = 0; u + 1 < D; ++u) __builtin_amdgcn_raw_buffer_store_b32(0u, drs.r, (int)kOobStore, 0, 0);
        for (int r = rs; r <= re; r += D) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
                // Every step runs, also the up to D - 1 past the band's last row
                // (their windows are the last row again; they only write ring
                // slots no pending output reads), and every step issues at
                // least one store: a row's, or a dropped one (an offset past
                // the plane).  The compiler's wait for a window then counts the
                // stores issued after it and leaves them in flight; with steps
                // of no store (or skipped) on some path, its waits drained the
                // stores too (vmcnt(0) at every loop iteration's first window).
                const int rr = r + u;
                hrow(buf[u], rr & 7);
                if (y < y1 && need == rr) {  // uniform
                    do {
                        // y is wave-uniform; said so, its table reads are scalar
                        // loads (as vector loads they would wait behind the windows)
                        y = __builtin_amdgcn_readfirstlane(y);
                        emit(y);
                        ++y;
                        if (y < y1) need = min(lz_const(L.t.yofs, y) + 4, h - 1);
                    } while (y < y1 && need == rr);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b32(0u, drs.r, (int)kOobStore, 0, 0);
                }
                load(safe_c, buf[u], min(rr + D, re));
            }
        }
    };
    // uniform: can any lane's window of the band's last row overhang the plane?
    const bool over = (uint32_t)re * rp + (wbyte & ~3u) + 4u * ND > slimit;
    if (__builtin_amdgcn_ballot_w64(over) != 0) walk(std::integral_constant<bool, true>());
    else walk(std::integral_constant<bool, false>());
}

// u8 sources: lanczos_u8_kernel.  The same strip walk as lanczos_kernel, but
// the 8 most recent horizontal rows live in REGISTERS, not an LDS ring: the
// walk is unrolled by 8 source rows, so row rr's values land in register row
// (rr - rs) & 7 -- a compile-time index (rs = the band's first source row).
// The host regroups each output row's 8 vertical coefficients by that
// relative slot (yrec), so an output row is 8 multiply-adds per channel on
// registers: no ring stores and reads, no LDS waits.  Diagnosis builds of the
// LDS-ring kernel (round 4) ran 0.41 ms without any window load against
// 0.49 with them: the per-row instruction stream around the loads, not the
// loads, bounded it.  Also: the border clamp is folded into each lane's
// coefficients once (window pixel p weighs the sum of the taps that clamp to
// it -- exact, the u8 sums are int arithmetic), so every lane runs the same
// unrolled horizontal sum and the per-row 9-way shift switch is gone.
constexpr int kLzTasks = 65536;  // wave tasks a launch aims for (bands shrink until there are about this many)
constexpr int kLzMinRows = 16;  // output rows per band at least
constexpr int kLzrD = 4;  // windows in flight per wave (a divisor of 8, the unroll)
// NI > 0 (round 5): the wave's source run of a row (the 64 lanes' windows,
// <= NI KiB, host-checked) moves as NI lane-contiguous 16-byte loads and
// reaches the lanes' windows through the wave's own LDS slice: at a 3x
// downscale one 600-byte instruction instead of two per lane (28 bytes per
// lane for 9 new ones).  NI = 0: every lane loads its own window.
// u8 output at 6 waves per SIMD (79 VGPRs, no spills; the default 5 at 95:
// 1080p -> 640x360 0.3939 -> 0.3822 ms); the fp32 outputs spill there
template <int OUT, int CC, int NI>
__global__ void __launch_bounds__(64 * kLzWaves) __attribute__((amdgpu_waves_per_eu(OUT == kOutSame ? 6 : 1)))
lanczos_u8_kernel(LanczosLaunch L, int strips, int bands, int band_rows,
                                                                     int blocks, int xcd_per) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr int ND = (8 * CC + 6) / 4;
    constexpr int D = kLzrD;
    static_assert(8 % D == 0, "the window buffers rotate with the 8-row unroll");

    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = (int)(threadIdx.x & 63);
    const int blk = xcd_per > 0 ? (int)(blockIdx.x % 8) * xcd_per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    if (blk >= blocks) return;
    const int task = blk * kLzWaves + wave;  // (plane, band, strip), strip fastest
    const int strip = task % strips;
    const int rest = task / strips;
    const int band = rest % bands;
    const int pidx = rest / bands;
    if (pidx >= L.n * L.src.planes) return;  // whole wave
    const int y0 = band * band_rows, y1 = min(y0 + band_rows, L.dst.h);
    const int x = strip * 64 + lane;
    const bool live = x < L.dst.w;
    const int xc = live ? x : L.dst.w - 1;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int w = L.src.w, h = L.src.h;
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp = (uint32_t)L.src.row_pitch;

    const int sx = L.t.xofs[xc];
    const int wstart = min(max(sx - 3, 0), w - 8);
    const int shift = (sx - 3) - wstart;  // [-4, 4]
    int cw[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) cw[p] = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = (int)L.t.xai[8 * xc + j];
#pragma unroll
        for (int p = 0; p < 8; ++p) cw[p] += min(max(j + shift, 0), 7) == p ? c : 0;
    }
    uint32_t cp[4];  // (cw[2m], cw[2m + 1]) short pairs; a folded sum stays within +-2^15
#pragma unroll
    for (int m = 0; m < 4; ++m) cp[m] = ((uint32_t)cw[2 * m] & 0xFFFFu) | ((uint32_t)cw[2 * m + 1] << 16);
    const uint32_t wbyte = (uint32_t)(wstart * CC) + srs.delta;
    const uint32_t wsh = wbyte & 3u;
    // NI > 0: the run's first byte (lane 0 has the smallest window start) and
    // this lane's window within the wave's slice
    const uint32_t wrun = (uint32_t)__builtin_amdgcn_readfirstlane((int)(wbyte & ~15u));
    const uint32_t wofs = (wbyte & ~3u) - wrun;
    // the run's bytes: up to the last lane's window end (windows are monotone
    // in the lane); chunks past it are not loaded (they belong to the next
    // strip's run: loading them here fetched 1.11 x the source rows)
    const uint32_t run_end = (uint32_t)__builtin_amdgcn_readlane((int)(wofs + 4u * ND), 63);
    __shared__ __attribute__((aligned(16))) uint32_t xs[NI > 0 ? kLzWaves : 1][NI > 0 ? 256 * NI : 1];
    using RowBuf = typename std::conditional<(NI > 0), u32x4[NI > 0 ? NI : 1], uint32_t[ND]>::type;
    auto load_run = [&](auto safe_c, u32x4 (&t)[NI > 0 ? NI : 1], int r) {
        constexpr bool SAFE = decltype(safe_c)::value;
#pragma unroll
        for (int i = 0; i < (NI > 0 ? NI : 1); ++i) {
            const uint32_t c16 = 16u * (uint32_t)(64 * i + lane);
            const uint32_t a = (uint32_t)r * rp + wrun + c16;
            // past the run: an out-of-range offset, no memory access (its LDS
            // words are never read)
            if (!SAFE || (c16 >= run_end || a + 16u <= slimit)) {
                t[i] = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)(c16 < run_end ? a : 0x80000000u), 0, 0);
            } else {  // the chunk overhangs the plane's end: bytewise (past it: zeros)
                uint32_t v[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (a + (uint32_t)e < slimit)
                        v[e >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(a + (uint32_t)e), 0, 0) << (8 * (e & 3));
                t[i] = u32x4{v[0], v[1], v[2], v[3]};
            }
        }
    };

    auto load = [&](auto safe_c, uint32_t (&d)[ND], int r) {
        constexpr bool SAFE = decltype(safe_c)::value;
        const uint32_t a = (uint32_t)r * rp + (wbyte & ~3u);
        if (!SAFE || a + 4u * ND <= slimit) {
            int q = 0;
#pragma unroll
            for (; q + 4 <= ND; q += 4) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)(a + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1]; d[q + 2] = v[2]; d[q + 3] = v[3];
            }
            if constexpr (ND % 4 == 3) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b96(srs.r, (int)(a + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1]; d[q + 2] = v[2];
            } else if constexpr (ND % 4 == 2) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(srs.r, (int)(a + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1];
            } else if constexpr (ND % 4 == 1) {
                d[q] = __builtin_amdgcn_raw_buffer_load_b32(srs.r, (int)(a + 4 * q), 0, 0);
            }
        } else {  // the window overhangs the plane's end: bytewise
#pragma unroll
            for (int q = 0; q < ND; ++q) {
                uint32_t v = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (a + 4u * q + e < slimit)
                        v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(a + 4u * q + e), 0, 0) << (8 * e);
                d[q] = v;
            }
        }
    };
    auto hrow = [&](const uint32_t (&d)[ND], int (&hv)[CC]) {
        uint32_t wv[ND - 1];
#pragma unroll
        for (int q = 0; q < ND - 1; ++q) wv[q] = __builtin_amdgcn_alignbyte(d[q + 1], d[q], wsh);
        lz_h_u8<CC, 0, ND - 1>(wv, cp, hv);
    };
    // NI > 0: the run through the wave's slice, then this lane's window
    auto hrow_run = [&](const u32x4 (&t)[NI > 0 ? NI : 1], int (&hv)[CC]) {
        uint32_t* xw = xs[NI > 0 ? wave : 0];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the previous row's window reads are done
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int i = 0; i < (NI > 0 ? NI : 1); ++i) *reinterpret_cast<u32x4*>(xw + 4 * (64 * i + lane)) = t[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t d[ND];
        const uint32_t* wp = xw + (wofs >> 2);
#pragma unroll
        for (int q = 0; q < ND; ++q) d[q] = wp[q];
        hrow(d, hv);
    };

    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const Rsrc drs = make_rsrc(dp, L.dst.plane_bytes);
    const bool dst_al = ((reinterpret_cast<uintptr_t>(dp) | (uintptr_t)L.dst.row_pitch) & 3) == 0;
    const bool full = strip * 64 + 64 <= L.dst.w;
    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }
    constexpr uint32_t kOobStore = 0x80000000u;  // a store offset past every plane: dropped

    // VResizeLanczos4 of output row y from the register rows; bb = its
    // coefficients by relative slot (wave-uniform)
    auto emit = [&](int y, const int (&hs)[8][CC], const int (&bb)[8]) {
        TOut o[CC];
#pragma unroll
        for (int q = 0; q < CC; ++q) {
            // 24-bit multiplies: |h| < 2^23, |b| < 2^12 (as lanczos_kernel)
            const int s0 = __mul24(hs[0][q], bb[0]) + __mul24(hs[1][q], bb[1]) + __mul24(hs[2][q], bb[2]) +
                           __mul24(hs[3][q], bb[3]);
            const int s1 = __mul24(hs[4][q], bb[4]) + __mul24(hs[5][q], bb[5]) + __mul24(hs[6][q], bb[6]) +
                           __mul24(hs[7][q], bb[7]);
            const int vi = min(max((s0 + s1 + (1 << 21)) >> 22, 0), 255);  // FixedPtCast<int, uchar, 22>
            if (OUT == kOutSame) o[q] = (TOut)vi;
            else if (OUT == kOutF32) o[q] = (TOut)(float)vi;
            else o[q] = (TOut)normalize_u8v(cn[q], vi);
        }
        const uint32_t orow = (uint32_t)y * (uint32_t)L.dst.row_pitch + drs.delta;
        if constexpr (sizeof(TOut) == 1) {
            uint32_t own = 0;
#pragma unroll
            for (int q = 0; q < CC; ++q) own |= (uint32_t)(uint8_t)o[q] << (8 * q);
            const int xq = x & ~3;
            const bool quad = dst_al && (full || xq + 4 <= L.dst.w);
            const uint32_t word = quad_pack<CC>(own, lane & 3);
            if (quad) {
                if ((lane & 3) < CC)
                    __builtin_amdgcn_raw_buffer_store_b32(word, drs.r, (int)(orow + (uint32_t)(xq * CC + 4 * (lane & 3))),
                                                          0, 0);
            } else if (live) {
#pragma unroll
                for (int q = 0; q < CC; ++q)
                    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(own >> (8 * q)), drs.r,
                                                         (int)(orow + (uint32_t)(x * CC + q)), 0, 0);
            }
        } else if (live) {
            const uint32_t off = orow + (uint32_t)(x * CC) * 4u;
            uint32_t ov[CC];
#pragma unroll
            for (int q = 0; q < CC; ++q) ov[q] = __float_as_uint(o[q]);
            if (dst_al) {
                if constexpr (CC == 1) {
                    __builtin_amdgcn_raw_buffer_store_b32(ov[0], drs.r, (int)off, 0, 0);
                } else if constexpr (CC == 2) {
                    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{ov[0], ov[1]}, drs.r, (int)off, 0, 0);
                } else if constexpr (CC == 3) {
                    typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                    __builtin_amdgcn_raw_buffer_store_b96(u32x3{ov[0], ov[1], ov[2]}, drs.r, (int)off, 0, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{ov[0], ov[1], ov[2], ov[3]}, drs.r, (int)off, 0, 0);
                }
            } else {
                TOut* dq = reinterpret_cast<TOut*>(dp + (off - drs.delta));
#pragma unroll
                for (int q = 0; q < CC; ++q) dq[q] = o[q];
            }
        }
    };

    // The walk: every step resizes one source row into its register row,
    // emits the output rows whose last tap row it is, and issues the window
    // load D rows ahead; a step that emits nothing issues a dropped store, so
    // every step holds at least one store and the compiler's wait for a
    // window leaves the later stores in flight (lanczos_kernel's walk).  The
    // next output row's record (coefficients, last tap row) is fetched when
    // the previous one is emitted, a step or more before it is read.
    const int rs = max(lz_const(L.t.yofs, y0) - 3, 0);
    const int re = min(lz_const(L.t.yofs, y1 - 1) + 4, h - 1);
    auto walk = [&](auto safe_c) {
        int hs[8][CC];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int q = 0; q < CC; ++q) hs[j][q] = 0;
        }
        int y = __builtin_amdgcn_readfirstlane(y0);
        int bb[8], need, same;
        auto fetch = [&](int yy) {
#pragma unroll
            for (int k = 0; k < 8; ++k) bb[k] = lz_const(L.t.yrec, 16 * yy + k);
            need = lz_const(L.t.yrec, 16 * yy + 8);
            same = lz_const(L.t.yrec, 16 * yy + 9);
        };
        fetch(y);
        RowBuf buf[D];
        auto issue = [&](RowBuf& b, int r) {
            if constexpr (NI > 0) load_run(safe_c, b, r);
            else load(safe_c, b, r);
        };
#pragma unroll
        for (int u = 0; u < D; ++u) issue(buf[u], min(rs + u, re));
#pragma unroll
        for (int u = 0; u + 1 < D; ++u) __builtin_amdgcn_raw_buffer_store_b32(0u, drs.r, (int)kOobStore, 0, 0);
        for (int r = rs;; r += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int rr = r + u;
                if constexpr (NI > 0) hrow_run(buf[u % D], hs[u]);
                else hrow(buf[u % D], hs[u]);
                if (need == rr) {  // uniform; y < y1 while the walk runs
                    // the first output row of the step outside any loop: the
                    // multiplies then take the register rows as they are (in
                    // a loop LLVM hoists a sign extension of all 8 CC rows
                    // out of it, 8 CC extra VALU per output row); `same`
                    // (the record's flag: the next row ends on this source
                    // row too) decides the loop without waiting for the
                    // next record, which is read a step later
                    y = __builtin_amdgcn_readfirstlane(y);
                    emit(y, hs, bb);
                    bool more = same != 0;
                    ++y;
                    if (y < y1) fetch(y);
                    while (more && y < y1) {  // upscales: more output rows per source row
                        y = __builtin_amdgcn_readfirstlane(y);
                        emit(y, hs, bb);
                        more = same != 0;
                        ++y;
                        if (y < y1) fetch(y);
                    }
                } else {
                    __builtin_amdgcn_raw_buffer_store_b32(0u, drs.r, (int)kOobStore, 0, 0);
                }
                if (y >= y1) return;  // the band's last output row is out
                issue(buf[u % D], min(rr + D, re));
            }
        }
    };
    const bool over = NI > 0 ? (uint32_t)re * rp + wrun + 1024u * (uint32_t)NI > slimit
                             : (uint32_t)re * rp + (wbyte & ~3u) + 4u * ND > slimit;
    if (__builtin_amdgcn_ballot_w64(over) != 0) walk(std::integral_constant<bool, true>());
    else walk(std::integral_constant<bool, false>());
}

// Sources narrower than the 8-pixel window (w < 8): every column is a border
// column of HResizeLanczos4 (no output column has all 8 taps inside), so each
// tap is clamped to [0, w - 1] and the horizontal sum starts from 0 +.  One
// thread per output pixel, the same tables and the same vertical arithmetic
// as lanczos_kernel; these images are tiny, so no staging.
template <typename TIn, int OUT>
__global__ void __launch_bounds__(256) lanczos_small_kernel(LanczosLaunch L) {
    constexpr bool U8 = std::is_same<TIn, uint8_t>::value;
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    const int64_t per_plane = (int64_t)L.dst.w * L.dst.h;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= per_plane * L.n * L.src.planes) return;
    const int pidx = (int)(i / per_plane);
    const int rem = (int)(i - (int64_t)pidx * per_plane);
    const int y = rem / L.dst.w, x = rem - y * L.dst.w;
    const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
    const int CC = L.src.cc, w = L.src.w, h = L.src.h;
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch;
    const int sx = L.t.xofs[x], sy = L.t.yofs[y];
    const int dw = L.dst.w * CC;
    for (int q = 0; q < CC; ++q) {
        TOut o;
        if constexpr (U8) {
            uint32_t acc = 0;  // int arithmetic, wrapping as OpenCV's
            for (int k = 0; k < 8; ++k) {
                const unsigned char* row = sp + (int64_t)min(max(sy - 3 + k, 0), h - 1) * L.src.row_pitch;
                uint32_t hv = 0;
                for (int j = 0; j < 8; ++j)
                    hv += (uint32_t)row[min(max(sx - 3 + j, 0), w - 1) * CC + q] * (uint32_t)(int)L.t.xai[8 * x + j];
                acc += hv * (uint32_t)(int)L.t.yai[8 * y + k];
            }
            const int vi = min(max(((int)acc + (1 << 21)) >> 22, 0), 255);  // FixedPtCast<int, uchar, 22>
            if (OUT == kOutSame) o = (TOut)vi;
            else if (OUT == kOutF32) o = (TOut)(float)vi;
            else o = (TOut)normalize_u8v(chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : q), vi);
        } else {
            float hs[8];
            for (int k = 0; k < 8; ++k) {
                const float* row = reinterpret_cast<const float*>(sp + (int64_t)min(max(sy - 3 + k, 0), h - 1) *
                                                                         L.src.row_pitch);
                float v = 0.f + row[min(max(sx - 3, 0), w - 1) * CC + q] * L.t.xaf[8 * x];
                for (int j = 1; j < 8; ++j) v = v + row[min(max(sx - 3 + j, 0), w - 1) * CC + q] * L.t.xaf[8 * x + j];
                hs[k] = v;
            }
            const float* bb = L.t.yaf + 8 * y;
            float v;
            if (x * CC + q < (dw & ~3)) {  // VResizeLanczos4Vec_32f's 4-wide loop
                const float s0 = ((hs[0] * bb[0] + hs[1] * bb[1]) + hs[2] * bb[2]) + hs[3] * bb[3];
                const float s1 = ((hs[4] * bb[4] + hs[5] * bb[5]) + hs[6] * bb[6]) + hs[7] * bb[7];
                v = s0 + s1;
            } else {  // the scalar tail
                v = hs[0] * bb[0];
                for (int k = 1; k < 8; ++k) v = v + hs[k] * bb[k];
            }
            if (OUT == kOutNorm) v = normalize_f(chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : q), v);
            o = (TOut)v;
        }
        reinterpret_cast<TOut*>(dp)[x * CC + q] = o;
    }
}

// interpolateLanczos4 (imgwarp.cpp): float x, double sin / cos, float sums
void lanczos4_coeffs(float x, float* c) {
    static const double s45 = 0.70710678118654752440084436210485;
    static const double cs[8][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
    const double pi = 3.1415926535897932384626433832795;
    if (x < FLT_EPSILON) {
        for (int i = 0; i < 8; ++i) c[i] = 0.f;
        c[3] = 1.f;
        return;
    }
    float sum = 0.f;
    const double y0 = -(double)(x + 3) * pi * 0.25, s0 = std::sin(y0), c0 = std::cos(y0);
    for (int i = 0; i < 8; ++i) {
        const double yv = -(double)(x + 3 - i) * pi * 0.25;
        c[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (yv * yv));
        sum += c[i];
    }
    sum = 1.f / sum;
    for (int i = 0; i < 8; ++i) c[i] *= sum;
}

// saturate_cast<short>(float): cvRound (lrint, half to even), then clamp
short sat_short(float v) {
    const long r = std::lrint(v);
    return (short)std::min<long>(std::max<long>(r, -32768), 32767);
}

// resize()'s per-axis tables for LANCZOS4: origin floor(f), 8 coefficients
void lanczos_axis(int n_in, int n_out, double scale, std::vector<int>& ofs, std::vector<short>& ci,
                  std::vector<float>& cf, int* lo, int* hi) {
    ofs.resize(n_out);
    ci.resize(8 * (size_t)n_out);
    cf.resize(8 * (size_t)n_out);
    int xmin = 0, xmax = n_out;
    for (int d = 0; d < n_out; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        const int s = (int)std::floor(f);
        f -= (float)s;
        if (s < 3) xmin = d + 1;                  // ksize2 - 1
        if (s + 4 >= n_in) xmax = std::min(xmax, d);  // sx + ksize2 >= ssize
        ofs[d] = s;
        float c[8];
        lanczos4_coeffs(f, c);
        for (int k = 0; k < 8; ++k) {
            cf[8 * (size_t)d + k] = c[k];
            ci[8 * (size_t)d + k] = sat_short(c[k] * 2048.f);  // INTER_RESIZE_COEF_SCALE
        }
    }
    if (lo) *lo = xmin;
    if (hi) *hi = xmax;
}

struct CachedLanczos {
    int device = 0;
    void* dev = nullptr;
    LanczosTabsDev t{};
};
std::mutex g_lz_mu;
// run_ni depends on the channel count too, so cc is part of the key
std::map<std::tuple<int, int, int, int, int, int, double, double, int>, CachedLanczos> g_lz_tabs;
bool free_lz(CachedLanczos& c) { return hipFree(c.dev) == hipSuccess; }

// lanczos_u8_kernel's staged runs: the 16-byte loads per lane (1 or 2) that
// cover every strip's windows (the kernel's run starts at lane 0's window
// rounded down to 16 bytes; 16 more for a base that is not 16-byte aligned),
// or 0 where a strip's windows span more than 2 KiB
int lanczos_run_loads(const ResizeLaunch& R, const std::vector<int>& xofs) {
    const int cc = R.src.cc, w = R.src.w, nd = (8 * cc + 6) / 4;
    auto ws = [&](int x) { return std::min(std::max(xofs[x] - 3, 0), w - 8); };
    int need = 0;
    for (int s0 = 0; s0 < R.dst.w; s0 += 64) {
        const int xl = std::min(s0 + 63, R.dst.w - 1);
        const int start = (ws(s0) * cc) & ~15, end = ((ws(xl) * cc) & ~3) + 4 * nd;
        need = std::max(need, end - start + 16);
    }
    return need <= 1024 ? 1 : need <= 2048 ? 2 : 0;
}

int lanczos_tables(const ResizeLaunch& R, double inv_x, double inv_y, int band_rows, hipStream_t s, LanczosTabsDev& out) {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return VACV_ERR_HIP;
    const auto key = std::make_tuple(device, R.src.cc, R.src.w, R.src.h, R.dst.w, R.dst.h, inv_x, inv_y, band_rows);
    std::lock_guard<std::mutex> lk(g_lz_mu);
    auto it = g_lz_tabs.find(key);
    if (it == g_lz_tabs.end()) {
        std::vector<int> xo, yo;
        std::vector<short> xi, yi;
        std::vector<float> xf, yf;
        int xmin = 0, xmax = 0;
        lanczos_axis(R.src.w, R.dst.w, 1. / inv_x, xo, xi, xf, &xmin, &xmax);
        lanczos_axis(R.src.h, R.dst.h, 1. / inv_y, yo, yi, yf, nullptr, nullptr);
        std::vector<unsigned char> img;
        auto put = [&img](const void* p, size_t b) {
            const size_t o = (img.size() + 15) & ~size_t(15);
            img.resize(o + b);
            if (b) std::memcpy(img.data() + o, p, b);
            return o;
        };
        // u8 vertical coefficients regrouped by ring slot: tap k of row y reads
        // source row clip(sy - 3 + k, 0, h - 1), held in slot (row & 7)
        std::vector<int> yr(4 * (size_t)R.dst.h);
        for (int y = 0; y < R.dst.h; ++y) {
            int b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int k = 0; k < 8; ++k)
                b[std::min(std::max(yo[y] - 3 + k, 0), R.src.h - 1) & 7] += yi[8 * (size_t)y + k];
            for (int m = 0; m < 4; ++m)
                yr[4 * (size_t)y + m] = (int)(((uint32_t)b[2 * m] & 0xFFFFu) | ((uint32_t)b[2 * m + 1] << 16));
        }
        // lanczos_u8_kernel: the same regrouping by slot relative to the band's
        // first source row (the kernel's rs), and the row's last tap row
        std::vector<int> yc(16 * (size_t)R.dst.h, 0);
        for (int y = 0; y < R.dst.h; ++y) {
            const int y0 = band_rows > 0 ? y / band_rows * band_rows : 0;
            const int rs = std::max(yo[y0] - 3, 0);
            for (int k = 0; k < 8; ++k) {
                const int row = std::min(std::max(yo[y] - 3 + k, 0), R.src.h - 1);
                yc[16 * (size_t)y + ((row - rs) & 7)] += yi[8 * (size_t)y + k];
            }
            yc[16 * (size_t)y + 8] = std::min(yo[y] + 4, R.src.h - 1);
        }
        for (int y = 0; y + 1 < R.dst.h; ++y) yc[16 * (size_t)y + 9] = yc[16 * (size_t)y + 8] == yc[16 * (size_t)y + 24];
        const size_t o0 = put(xo.data(), xo.size() * 4), o1 = put(xi.data(), xi.size() * 2),
                     o2 = put(xf.data(), xf.size() * 4), o3 = put(yo.data(), yo.size() * 4),
                     o4 = put(yi.data(), yi.size() * 2), o5 = put(yf.data(), yf.size() * 4),
                     o6 = put(yr.data(), yr.size() * 4), o7 = put(yc.data(), yc.size() * 4);
        if (g_lz_tabs.size() > 64)  // bounded cache
            (void)evict_device_cache(g_lz_tabs, free_lz);
        CachedLanczos c;
        c.device = device;
        if (hipMalloc(&c.dev, img.size() + 16) != hipSuccess) return VACV_ERR_NO_MEMORY;
        // one upload per geometry; synchronised so any stream may use it next
        if (hipMemcpyAsync(c.dev, img.data(), img.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            (void)hipFree(c.dev);
            return VACV_ERR_HIP;
        }
        const unsigned char* b = static_cast<const unsigned char*>(c.dev);
        c.t.xofs = reinterpret_cast<const int*>(b + o0);
        c.t.xai = reinterpret_cast<const short*>(b + o1);
        c.t.xaf = reinterpret_cast<const float*>(b + o2);
        c.t.yofs = reinterpret_cast<const int*>(b + o3);
        c.t.yai = reinterpret_cast<const short*>(b + o4);
        c.t.yaf = reinterpret_cast<const float*>(b + o5);
        c.t.yrot = reinterpret_cast<const int*>(b + o6);
        c.t.yrec = reinterpret_cast<const int*>(b + o7);
        c.t.xmin = xmin;
        c.t.xmax = xmax;
        c.t.run_ni = R.src.w >= 8 ? lanczos_run_loads(R, xo) : 0;
        it = g_lz_tabs.emplace(key, c).first;
    }
    out = it->second.t;
    return VACV_OK;
}

struct LzGrid {
    int blocks, strips, bands, band_rows, xcd_per;
};

template <typename TIn, int OUT>
hipError_t launch_out(const LanczosLaunch& A, const LzGrid& g, hipStream_t s) {
    const dim3 grid((unsigned)(g.xcd_per > 0 ? 8 * g.xcd_per : g.blocks)), block(64 * kLzWaves);
    switch (A.src.cc) {
        case 1: hipLaunchKernelGGL((lanczos_kernel<TIn, OUT, 1>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        case 2: hipLaunchKernelGGL((lanczos_kernel<TIn, OUT, 2>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        case 3: hipLaunchKernelGGL((lanczos_kernel<TIn, OUT, 3>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        case 4: hipLaunchKernelGGL((lanczos_kernel<TIn, OUT, 4>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int OUT, int NI>
hipError_t launch_u8_ni(const LanczosLaunch& A, const LzGrid& g, hipStream_t s) {
    const dim3 grid((unsigned)(g.xcd_per > 0 ? 8 * g.xcd_per : g.blocks)), block(64 * kLzWaves);
    switch (A.src.cc) {
        case 1: hipLaunchKernelGGL((lanczos_u8_kernel<OUT, 1, NI>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        case 2: hipLaunchKernelGGL((lanczos_u8_kernel<OUT, 2, NI>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        case 3: hipLaunchKernelGGL((lanczos_u8_kernel<OUT, 3, NI>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        case 4: hipLaunchKernelGGL((lanczos_u8_kernel<OUT, 4, NI>), grid, block, 0, s, A, g.strips, g.bands, g.band_rows, g.blocks, g.xcd_per); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int OUT>
hipError_t launch_u8(const LanczosLaunch& A, const LzGrid& g, int ni, hipStream_t s) {
    if (ni == 1) return launch_u8_ni<OUT, 1>(A, g, s);
    if (ni == 2) return launch_u8_ni<OUT, 2>(A, g, s);
    return launch_u8_ni<OUT, 0>(A, g, s);
}



template <typename TIn>
hipError_t launch_t(const LanczosLaunch& A, const LzGrid& g, hipStream_t s) {
    if (A.out == kOutSame) return launch_out<TIn, kOutSame>(A, g, s);
    if (A.out == kOutF32) return launch_out<TIn, kOutF32>(A, g, s);
    return launch_out<TIn, kOutNorm>(A, g, s);
}

}  // namespace

int launch_resize_lanczos(const ResizeLaunch& R, double inv_x, double inv_y, hipStream_t s) {
    if (R.src.cc > 4) return VACV_ERR_UNSUPPORTED;
    LanczosLaunch A{};
    A.src = R.src;
    A.dst = R.dst;
    A.n = R.n;
    A.out = R.out;
    A.norm = R.norm;
    // wave tasks: 64-column strips x bands of output rows x planes; bands
    // shrink until there are ~kLzTasks tasks (a band's first row resizes all 8 of
    // its source rows, later rows only the new ones)
    LzGrid g{};
    const int64_t planes = (int64_t)R.n * R.src.planes;
    const bool narrow = R.src.w < 8;
    if (!narrow) {
        g.strips = (R.dst.w + 63) / 64;
        const int64_t want = (kLzTasks + g.strips * planes - 1) / (g.strips * planes);
        g.bands = (int)std::max<int64_t>(1, std::min<int64_t>(want, (R.dst.h + kLzMinRows - 1) / kLzMinRows));
        g.band_rows = (R.dst.h + g.bands - 1) / g.bands;
        g.bands = (R.dst.h + g.band_rows - 1) / g.band_rows;
    }
    const int st = lanczos_tables(R, inv_x, inv_y, g.band_rows, s, A.t);
    if (st) return st;
    if (narrow) {
        // narrower than lanczos_kernel's 8-pixel row window: per-pixel kernel
        const int64_t total = (int64_t)R.dst.w * R.dst.h * R.n * R.src.planes;
        const int64_t blocks = (total + 255) / 256;
        if (blocks > 0x7FFFFFF0LL) return VACV_ERR_UNSUPPORTED;
        const dim3 grid((unsigned)blocks), block(256);
        if (R.src.esize == 1) {
            if (A.out == kOutSame) hipLaunchKernelGGL((lanczos_small_kernel<uint8_t, kOutSame>), grid, block, 0, s, A);
            else if (A.out == kOutF32) hipLaunchKernelGGL((lanczos_small_kernel<uint8_t, kOutF32>), grid, block, 0, s, A);
            else hipLaunchKernelGGL((lanczos_small_kernel<uint8_t, kOutNorm>), grid, block, 0, s, A);
        } else {
            if (A.out == kOutSame) hipLaunchKernelGGL((lanczos_small_kernel<float, kOutSame>), grid, block, 0, s, A);
            else if (A.out == kOutF32) hipLaunchKernelGGL((lanczos_small_kernel<float, kOutF32>), grid, block, 0, s, A);
            else hipLaunchKernelGGL((lanczos_small_kernel<float, kOutNorm>), grid, block, 0, s, A);
        }
        return hipGetLastError() == hipSuccess ? VACV_OK : VACV_ERR_HIP;
    }
    const int64_t tasks = (int64_t)g.strips * g.bands * planes;
    if ((tasks + kLzWaves - 1) / kLzWaves > 0x7FFFFFF0LL) return VACV_ERR_UNSUPPORTED;
    g.blocks = (int)((tasks + kLzWaves - 1) / kLzWaves);
    g.xcd_per = tune_or(VACV_TUNE_DIRECT_XCD, 1) ? (g.blocks + 7) / 8 : 0;
    hipError_t e;
    const int knob = tune_or(VACV_TUNE_LANCZOS_KERNEL, 0);
    if (R.src.esize == 1 && (knob == 0 || knob == 2)) {
        // the staged runs where they fit (LANCZOS_KERNEL = 2: per-lane windows, A/B)
        const int ni = knob == 0 ? A.t.run_ni : 0;
        if (A.out == kOutSame) e = launch_u8<kOutSame>(A, g, ni, s);
        else if (A.out == kOutF32) e = launch_u8<kOutF32>(A, g, ni, s);
        else e = launch_u8<kOutNorm>(A, g, ni, s);
    } else {
        e = R.src.esize == 1 ? launch_t<uint8_t>(A, g, s) : launch_t<float>(A, g, s);
    }
    return e == hipSuccess ? VACV_OK : VACV_ERR_HIP;
}

int release_lanczos_tables() {
    std::lock_guard<std::mutex> lk(g_lz_mu);
    return evict_device_cache(g_lz_tabs, free_lz);
}

}  // namespace vacv
