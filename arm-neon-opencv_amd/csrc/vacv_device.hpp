// vacv_device.hpp -- small gfx950 device helpers shared by the kernels.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <cstdint>
#include <utility>

#include "vacv_internal.hpp"
#include "vacv_semantics.hpp"

namespace vacv {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Cache-policy aux bits of the streaming buffer loads / stores (gfx950:
// 1 = sc0, 2 = nt, 16 = sc1).  Source rows and outputs are touched once:
// non-temporal on both sides measured 2-7 % faster on the resize kernels
// (profiles/r01_kbench.jsonl vs the nt sweep in DESIGN.md §3.1).
#ifndef VACV_LOAD_AUX
#define VACV_LOAD_AUX 2
#endif
#ifndef VACV_STORE_AUX
#define VACV_STORE_AUX 2
#endif

// A raw buffer resource over [base16, base16 + bytes): loads past the end
// return zeros instead of faulting, so a 16-byte staging load may overhang
// the last row of a batch.  base16 is the 16-byte aligned-down plane base;
// `delta` is what has to be added to offsets relative to the true base.
struct Rsrc {
    __amdgpu_buffer_rsrc_t r;
    uint32_t delta;
};

__device__ __forceinline__ Rsrc make_rsrc(const unsigned char* base, int64_t bytes) {
    uintptr_t p = reinterpret_cast<uintptr_t>(base);
    uintptr_t a = p & ~uintptr_t(15);
    Rsrc s;
    s.delta = static_cast<uint32_t>(p - a);
    int64_t n = bytes + s.delta;
    if (n > kMaxPlaneBytes + 16) n = kMaxPlaneBytes + 16;  // callers check plane sizes (kMaxPlaneBytes)
    s.r = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(a), (short)0, (int)n, 0x00020000);
    return s;
}

__device__ __forceinline__ uint4 load16(const Rsrc& s, uint32_t off_from_base16) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(s.r, (int)off_from_base16, 0, VACV_LOAD_AUX);
    return *reinterpret_cast<uint4*>(&v);
}


// 16-byte store through a buffer resource.  Kept distinct from plain stores
// on purpose: the compiler cannot merge it with a masked fallback path into
// narrower stores, so a wave's 64 lanes write 1 KiB in one instruction.
__device__ __forceinline__ void store16(const Rsrc& s, uint32_t off_from_base16, uint4 v) {
    u32x4 d = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(d, s.r, (int)off_from_base16, 0, VACV_STORE_AUX);
}

// The 2*CC tap bytes of a bilinear pixel (left tap's CC bytes, right tap's
// CC bytes) starting at buffer byte offset `off`, as bytes 0.. of (lo, hi).
// Two forms, each the faster one for its access pattern (kbench, MI355X):
//  * dword-aligned (b64 for CC <= 2, b96 for CC 3-4) and byte-shifted in
//    registers: the warp's rotated gathers, 0.34 -> 0.31 ms;
//  * one unaligned b64: lane-consecutive resize gathers 9 bytes apart, where
//    the aligned form was 10-20 % slower (0.220 -> 0.241 ms headline).
// The caller guarantees off + 8 <= size (unaligned) or
// (off & ~3) + 4 * kTapDwords<CC, true> <= size (aligned).
template <int CC, bool ALIGNED>
constexpr uint32_t kTapDwords = (!ALIGNED || CC <= 2) ? 2u : 3u;

template <int CC, bool ALIGNED, int AUX>
__device__ __forceinline__ void load_taps(const Rsrc& rs, uint32_t off, uint32_t& lo, uint32_t& hi) {
    if constexpr (!ALIGNED) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs.r, (int)off, 0, AUX);
        lo = v[0];
        hi = v[1];
        return;
    }
    const int a = (int)(off & ~3u);
    const uint32_t sh = off & 3u;
    if constexpr (CC <= 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs.r, a, 0, AUX);
        lo = __builtin_amdgcn_alignbyte(v[1], v[0], sh);
        hi = 0u;  // 2*CC <= 4 bytes: lo holds them all
    } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs.r, a, 0, AUX);
        lo = __builtin_amdgcn_alignbyte(v[1], v[0], sh);
        hi = __builtin_amdgcn_alignbyte(v[2], v[1], sh);
    }
}

// Per-workgroup mean/stddev for channel ch of image img.
__device__ __forceinline__ void norm_params(const NormSpec& ns, int img, int ch, float& m, float& s) {
    if (ns.mode == 2) {
        m = ns.dev_mean[(int64_t)img * ns.c_total + ch];
        s = ns.dev_std[(int64_t)img * ns.c_total + ch];
    } else {
        m = ns.mean[ch];
        s = ns.stdv[ch];
    }
}

// Normalisation constants of one channel, resolved once per workgroup.
struct ChanNorm {
    float mean, stdv;
    double inv;
    float hi, lo;
    bool mul;  // host-verified fp64 multiply is exact for u8-valued inputs
    bool f32;  // host-verified fp32 two-term multiply is exact (NormSpec.f32_ok)
};

__device__ __forceinline__ ChanNorm chan_norm(const NormSpec& ns, int img, int ch) {
    ChanNorm c;
    norm_params(ns, img, ch, c.mean, c.stdv);
    c.mul = ns.mode == 1 && ((ns.mul_ok >> ch) & 1u);
    c.f32 = ns.mode == 1 && ((ns.f32_ok >> ch) & 1u);
    c.inv = c.mul ? ns.inv[ch] : 0.0;
    c.hi = c.f32 ? ns.inv_hi[ch] : 0.f;
    c.lo = c.f32 ? ns.inv_lo[ch] : 0.f;
    return c;
}

// normalize_naive.cpp:74-90 for a value known to be an integer in [0,255]:
// the host proved one of the two short forms equal to the reference's
// (float)((double)d / ((double)std + 1e-6)) for all 256 values (norm_spec)
__device__ __forceinline__ float normalize_u8v(const ChanNorm& c, int v) {
    const float d = (float)v - c.mean;
    if (c.f32) return __builtin_fmaf(d, c.hi, d * c.lo);
    if (c.mul) return (float)((double)d * c.inv);
    return (float)((double)d / ((double)c.stdv + 1e-6));
}

__device__ __forceinline__ float normalize_f(const ChanNorm& c, float x) {
    return normalize_value(x, c.mean, c.stdv);
}

// ---- u8 bilinear fixed point (k_resize_direct.hip, k_yuv_resize.hip) ----

// ---- LDS-DMA (buffer_load ... lds) bookkeeping (k_warp_frames.hip, k_resize_strip.hip) ----

typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt vmcnt(n) lgkmcnt(0), n a uniform runtime value (clamped to 63:
// waiting for fewer outstanding operations is always safe).  The compiler
// does not track LDS-DMA writes, so the kernels wait for them themselves:
// gfx9 retires vector memory operations in issue order, so "the last n
// operations may still be in flight" means everything before them landed.
template <int N>
__device__ __forceinline__ void waitcnt_vm() {
    // gfx9 encoding: vmcnt [3:0] and [15:14], expcnt [6:4] (7: none), lgkmcnt [11:8]
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}
template <int... Ns>
__device__ __forceinline__ void wait_vm_impl(int n, std::integer_sequence<int, Ns...>) {
    (void)((n == Ns ? (waitcnt_vm<Ns>(), true) : false) || ...);
}
__device__ __forceinline__ void wait_vm(int n) {
    n = n < 0 ? 0 : (n > 63 ? 63 : n);
    n = __builtin_amdgcn_readfirstlane(n);
    wait_vm_impl(n, std::make_integer_sequence<int, 64>());
}
// s_waitcnt lgkmcnt(0) alone
__device__ __forceinline__ void wait_lgkm() { __builtin_amdgcn_s_waitcnt(0xF | (3 << 14) | (7 << 4)); }

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// One channel of one output pixel from its packed tap pairs.  A zero weight
// contributes exactly 0 in both formulas, so a skipped row is bot = 0, wB = 0.
template <int MODE>
__device__ __forceinline__ int blend_fixed(uint32_t top, uint32_t bot, us2 wx, uint32_t wA, uint32_t wB) {
    const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
    const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false);
    if (MODE == VACV_LINEAR_REFERENCE) {
        // (tl*a0 + tr*a1)*wA + (bl*a0 + br*a1)*wB: the reference's int32 sum
        // (terms >= 0, total <= 255*2049^2 < 2^31), 24-bit multiplies exact
        return (int)(((__umul24(ht, wA) + __umul24(hb, wB)) >> 22) & 0xFFu);
    }
    const int h0 = (int)(short)(ht >> 4);
    const int h1 = (int)(short)(hb >> 4);
    return clamp_u8((((h0 * (int)wA) >> 16) + ((h1 * (int)wB) >> 16) + 2) >> 2);
}

// fixed_tap() of the kernel.  REFERENCE mode: the coordinate
// (float)(((double)d + 0.5) * (double)scale_f - 0.5) is computed as ONE fp32
// fma, which is bit-identical: d + 0.5 (d < 2^23) and scale_f have 24-bit
// significands, so the product is exact in double and so is the - 0.5; the
// double path therefore rounds the exact value once to float -- exactly what
// fmaf does.  The rest is fixed_tap's own float arithmetic.
template <int MODE>
__device__ __forceinline__ FixedTap tap_of(int d, int n_in, int n_out, float scale_f, double scale_d) {
    if (MODE != VACV_LINEAR_REFERENCE) return fixed_tap(d, n_in, n_out, scale_f, scale_d, MODE);
    const float c = __builtin_fmaf((float)d + 0.5f, scale_f, -0.5f);
    const LinearTap t = linear_tap(c, n_in);
    FixedTap r;
    r.i = t.i;
    // sat_short_away of a value in [0, 2048]: the clamp and the sign test
    // are no-ops (t.f is in [0, 1])
    r.w0 = (int)((1.f - t.f) * 2048.f + 0.5f);
    r.w1 = (int)(t.f * 2048.f + 0.5f);
    return r;
}

// A warp pixel outside the naive sampler's range under a non-CONSTANT border
// mode (vacv_semantics.hpp border_index / border_tap): the four taps mapped
// through the border rule, the naive sampler's weights.  u8 results in vi
// (the >> 22 value), fp32 in vf.  sp = plane base, rp = row pitch in bytes.
template <int CC, typename TIn>
__device__ __forceinline__ void warp_border_sample(const unsigned char* sp, int64_t rp, int w, int h, int mode,
                                                   float fx, float fy, int (&vi)[CC], float (&vf)[CC]) {
    int ix, iy;
    float ax, ay;
    border_tap(fx, ix, ax);
    border_tap(fy, iy, ay);
    const int x0 = border_index(ix, w, mode) * CC, x1 = border_index(ix + 1, w, mode) * CC;
    const TIn* r0 = reinterpret_cast<const TIn*>(sp + (int64_t)border_index(iy, h, mode) * rp);
    const TIn* r1 = reinterpret_cast<const TIn*>(sp + (int64_t)border_index(iy + 1, h, mode) * rp);
    if constexpr (std::is_same<TIn, uint8_t>::value) {
        const int wy0 = (int)((1.f - ay) * 2048.f + 0.5f), wy1 = 2048 - wy0;
        const int wx0 = (int)((1.f - ax) * 2048.f + 0.5f), wx1 = 2048 - wx0;
#pragma unroll
        for (int k = 0; k < CC; ++k)
            vi[k] = ((int)r0[x0 + k] * wx0 * wy0 + (int)r1[x0 + k] * wx0 * wy1 + (int)r0[x1 + k] * wx1 * wy0 +
                     (int)r1[x1 + k] * wx1 * wy1) >> 22;
    } else {
        const float ya = 1.f - ay, yb = ay, xa = 1.f - ax, xb = ax;
#pragma unroll
        for (int k = 0; k < CC; ++k) {  // warp_affine_naive.cpp:98-102's order: lt, lb, rt, rb
            float v = r0[x0 + k] * xa * ya;
            v += r1[x0 + k] * xa * yb;
            v += r0[x1 + k] * xb * ya;
            v += r1[x1 + k] * xb * yb;
            vf[k] = v;
        }
    }
}

// quad-pack a pixel's CC bytes (low bytes of `own`) with its quad neighbours'
// into the quad's 4*CC output bytes: lane k < CC of the quad returns dword k
template <int CC>
__device__ __forceinline__ uint32_t quad_pack(uint32_t own, int k) {
    if constexpr (CC == 4) {
        return own;
    } else if constexpr (CC == 3) {
        const uint32_t nxt = (uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0xF9, 0xF, 0xF, false);  // [1,2,3,3]
        const uint32_t sel = k == 0 ? 0x04020100u : k == 1 ? 0x05040201u : 0x06050402u;
        return __builtin_amdgcn_perm(nxt, own, sel);
    } else if constexpr (CC == 2) {
        const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0x08, 0xF, 0xF, false);  // [0,2,.,.]
        const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0x0D, 0xF, 0xF, false);  // [1,3,.,.]
        return (a & 0xFFFFu) | (b << 16);
    } else {
        const uint32_t t = own | ((uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0xF9, 0xF, 0xF, false) << 8);
        return (t & 0xFFFFu) | ((uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0xFE, 0xF, 0xF, false) << 16);
    }
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace vacv
