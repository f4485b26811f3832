// vacv_semantics.hpp -- the reference's scalar arithmetic, shared by the host
// (tile planning, affine matrices) and the gfx950 kernels.
//
// Everything here is specified as separately rounded IEEE operations; the
// whole library is compiled with -ffp-contract=off and the pragma below so
// no a*b+c is fused (the reference's x86 build has no FMA either).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <cstdint>

#define VACV_HD __host__ __device__ __forceinline__

namespace vacv {

// SATURATE_CAST_SHORT (macro.h:25-30): add +-0.5f in float, truncate to int,
// clamp to [SHRT_MIN, SHRT_MAX].
VACV_HD int sat_short_away(float x) {
    float r = x + (x >= 0.f ? 0.5f : -0.5f);
    r = r < -32768.f ? -32768.f : (r > 32767.f ? 32767.f : r);
    return (int)r;
}

// OpenCV's saturate_cast<short>(float): round half to even, clamp.
VACV_HD int sat_short_even(float x) {
    float r = rintf(x);
    r = r < -32768.f ? -32768.f : (r > 32767.f ? 32767.f : r);
    return (int)r;
}

// Half-pixel-centre source coordinate (resize_naive.cpp:21,38: float scale
// widened to double; resize_neon.cpp:17-18,36 and resize_naive.cpp:144-148:
// double scale).  The product and the -0.5 are double, the result float.
VACV_HD float src_coord_f(int d, float scale) {
    return (float)(((double)d + 0.5) * (double)scale - 0.5);
}
VACV_HD float src_coord_d(int d, double scale) {
    return (float)(((double)d + 0.5) * scale - 0.5);
}

// One output index -> (left tap, fractional part), clamped as
// resize_naive.cpp:22-31: below 0 -> (0, 0); at/after n-1 -> (n-2, 1).
struct LinearTap {
    int i;
    float f;
};
VACV_HD LinearTap linear_tap(float coord, int n_in) {
    int i = (int)floorf(coord);
    float f = coord - (float)i;
    if (i < 0) { i = 0; f = 0.f; }
    if (i >= n_in - 1) { i = n_in - 2; f = 1.f; }
    return {i, f};
}

// 11-bit fixed-point weights of a linear tap.
//   mode 0 (reference naive) and 1 (NEON): half away from zero
//   mode 2 (OpenCV): half to even
struct FixedTap {
    int i;
    int w0;
    int w1;
};
VACV_HD FixedTap fixed_tap(int d, int n_in, int n_out, float scale_f, double scale_d, int mode) {
    float c = (mode == 0) ? src_coord_f(d, scale_f) : src_coord_d(d, scale_d);
    LinearTap t = linear_tap(c, n_in);
    float a = (1.f - t.f) * 2048.f;
    float b = t.f * 2048.f;
    FixedTap r;
    r.i = t.i;
    if (mode == 2) {
        r.w0 = sat_short_even(a);
        r.w1 = sat_short_even(b);
    } else {
        r.w0 = sat_short_away(a);
        r.w1 = sat_short_away(b);
    }
    return r;
}

struct FloatTap {
    int i;
    float w0;
    float w1;
};
VACV_HD FloatTap float_tap(int d, int n_in, float scale_f) {
    LinearTap t = linear_tap(src_coord_f(d, scale_f), n_in);
    return {t.i, 1.f - t.f, t.f};
}

// Keys cubic, A = -0.75, with the reference's replicate folding
// (resize_naive.cpp:130-185).  i is the centre tap: taps i-1 .. i+2.
struct CubicTap {
    int i;
    float c[4];
};
VACV_HD CubicTap cubic_tap(int d, int n_in, double scale_d) {
    const float A = -0.75f;
    float f = src_coord_d(d, scale_d);
    int i = (int)floorf(f);
    f -= (float)i;
    const float t0 = f + 1.f, t1 = f, t2 = 1.f - f;
    float c0 = A * t0 * t0 * t0 - 5.f * A * t0 * t0 + 8.f * A * t0 - 4.f * A;
    float c1 = (A + 2.f) * t1 * t1 * t1 - (A + 3.f) * t1 * t1 + 1.f;
    float c2 = (A + 2.f) * t2 * t2 * t2 - (A + 3.f) * t2 * t2 + 1.f;
    float c3 = 1.f - c0 - c1 - c2;
    if (i <= -1) { i = 1; c0 = 1.f - c3; c1 = c3; c2 = 0.f; c3 = 0.f; }
    if (i == 0) { i = 1; c0 = c0 + c1; c1 = c2; c2 = c3; c3 = 0.f; }
    if (i == n_in - 2) { i = n_in - 3; c3 = c2 + c3; c2 = c1; c1 = c0; c0 = 0.f; }
    if (i >= n_in - 1) { i = n_in - 3; c3 = 1.f - c0; c2 = c0; c1 = 0.f; c0 = 0.f; }
    CubicTap r;
    r.i = i;
    r.c[0] = c0; r.c[1] = c1; r.c[2] = c2; r.c[3] = c3;
    return r;
}

// Affine tap (warp_affine_naive.cpp:26-38): valid iff floor(f) in [0, n-2].
// Written as a float range test so far-away (or NaN) points never reach an
// undefined int conversion; the accept/skip decision is the reference's.
VACV_HD bool affine_tap(float f, int n, int& i, float& frac) {
    if (!(f >= 0.f && f < (float)(n - 1))) return false;
    i = (int)floorf(f);
    frac = f - (float)i;
    return true;
}

// Border modes for warp_affine beyond BORDER_CONSTANT.  The reference hands
// every other mode to OpenCV (warp_affine.cpp:114-118 -> :48-50, recursing
// forever without it); here they extend the reference's own naive sampler:
// a pixel whose top-left tap is inside [0,w-2]x[0,h-2] is computed exactly as
// for BORDER_CONSTANT, any other pixel takes its four taps at
// floor(f) and floor(f)+1 mapped through OpenCV 2.4's borderInterpolate
// (core: REPLICATE clamps; REFLECT fedcba|abcd|dcba; REFLECT_101 dcb|abcd|cba;
// WRAP modulo; the reflect loops in closed form), with the same fixed-point
// weights.  TRANSPARENT leaves such pixels untouched.  f is clamped to
// +-1e9 first (NaN -> -1e9) so floor() stays an int.  Parity unpinned: no
// reference entry runs these modes.
enum : int { kBorderConstant = 0, kBorderReplicate = 1, kBorderReflect = 2, kBorderWrap = 3,
             kBorderReflect101 = 4, kBorderTransparent = 5 };

VACV_HD int border_index(int p, int len, int mode) {
    if ((unsigned)p < (unsigned)len) return p;
    if (mode == kBorderReplicate) return p < 0 ? 0 : len - 1;
    if (mode == kBorderWrap) {
        int q = p % len;
        return q < 0 ? q + len : q;
    }
    // REFLECT (d = 0) / REFLECT_101 (d = 1)
    if (len == 1) return 0;
    const int d = mode == kBorderReflect101 ? 1 : 0;
    const long long period = 2LL * len - 2 * d;
    long long q = (long long)p % period;
    if (q < 0) q += period;
    return (int)(q < len ? q : period - 1 + d - q);
}

// floor(f) and frac of a warp coordinate outside the naive sampler's range
VACV_HD void border_tap(float f, int& i, float& frac) {
    const float c = fminf(fmaxf(f, -1e9f), 1e9f);
    i = (int)floorf(c);
    frac = c - (float)i;
}

// normalize_naive.cpp:74-90: float subtraction, double division, float result.
VACV_HD float normalize_value(float x, float mean, float stddev) {
    float d = x - mean;
    return (float)((double)d / ((double)stddev + 1e-6));
}

// f32_2_u8_neon (tensor.cpp:349-390): vcvtq_u32_f32 then truncating narrows.
VACV_HD uint8_t f32_to_u8_neon(float f) {
    uint32_t u;
    if (!(f > 0.f)) u = 0u;
    else if (f >= 4294967296.f) u = 0xFFFFFFFFu;
    else u = (uint32_t)f;
    return (uint8_t)(u & 0xFFu);
}

// NV21/NV12 -> BGR chroma terms, cvt_color.cpp:76-78 (arithmetic shifts).
struct Chroma {
    int ra, ga, ba;
};
VACV_HD Chroma chroma_terms(int u, int v) {
    Chroma c;
    c.ra = (179 * (v - 128)) >> 7;
    c.ga = (44 * (u - 128) + 91 * (v - 128)) >> 7;
    c.ba = (227 * (u - 128)) >> 7;
    return c;
}
VACV_HD int clamp_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

}  // namespace vacv
