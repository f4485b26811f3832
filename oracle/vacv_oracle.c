/*
 * vacv_oracle.c -- CPU restatement of the vacv pixel operators.
 *
 * TEST INFRASTRUCTURE ONLY (see vacv_oracle.h).  It is the checker for the
 * HIP kernels and the "port" CPU baseline in bench.py; the product library
 * (arm-neon-opencv_amd/lib/libvacv_hip.so) never links or loads it.
 *
 * Build: gcc -O2 -ffp-contract=off (oracle/Makefile).  fp contraction must be
 * off: the reference is specified by separately rounded IEEE operations (its
 * x86 build has no FMA), and so are the GPU kernels.
 *
 * Pinning: tests/test_oracle.py checks every function that has a buildable
 * reference counterpart against tests/golden/*.npz, which
 * tests/golden/make_golden.py generates by running the reference's own
 * sources (oracle/_ref/libvacv_ref.so).  Functions whose reference lives in
 * unbuildable Tensor code (crop, layout, dtype, rotation matrix, affine
 * inverse) are pinned by their documented equivalence instead.
 */
#include "vacv_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* SATURATE_CAST_SHORT, macro.h:25-30: add +-0.5f in float, truncate, clamp. */
int oracle_sat_short(float x) {
    float r = x + (x >= 0.f ? 0.5f : -0.5f);
    long v = (long)r;
    if (v < -32768) v = -32768;
    if (v > 32767) v = 32767;
    return (int)v;
}

/* round-half-even + clamp: OpenCV's saturate_cast<short>(float) (cvRound) */
static int sat_short_even(float x) {
    long v = lrintf(x);
    if (v < -32768) v = -32768;
    if (v > 32767) v = 32767;
    return (int)v;
}

/* Source coordinate of output index d for a half-pixel-centre map.
 * resize_naive.cpp:17-21 (float scale) / resize_neon.cpp:17-18,36 (double). */
static float src_coord(int d, int n_in, int n_out, int double_scale) {
    if (double_scale) {
        double s = (double)n_in / (double)n_out;
        return (float)(((double)d + 0.5) * s - 0.5);
    }
    float s = (float)n_in / (float)n_out;
    return (float)(((double)d + 0.5) * (double)s - 0.5);
}

/* Bilinear tap table, 11-bit fixed point.
 * naive: resize_naive.cpp:20-35 / :37-53; neon: resize_neon.cpp:35-78. */
void oracle_linear_table(int n_in, int n_out, int mode, int32_t* ofs, int16_t* w0, int16_t* w1) {
    for (int d = 0; d < n_out; ++d) {
        float f = src_coord(d, n_in, n_out, mode != ORACLE_LINEAR_NAIVE);
        int i = (int)floorf(f);
        f -= (float)i;
        if (i < 0) { i = 0; f = 0.f; }
        if (i >= n_in - 1) { i = n_in - 2; f = 1.f; }
        float a = (1.f - f) * 2048.f;
        float b = f * 2048.f;
        ofs[d] = i;
        if (mode == ORACLE_LINEAR_OPENCV) {
            w0[d] = (int16_t)sat_short_even(a);
            w1[d] = (int16_t)sat_short_even(b);
        } else {
            w0[d] = (int16_t)oracle_sat_short(a);
            w1[d] = (int16_t)oracle_sat_short(b);
        }
    }
}

/* fp32 bilinear taps, resize_naive.cpp:80-112 */
void oracle_linear_table_f32(int n_in, int n_out, int32_t* ofs, float* w0, float* w1) {
    for (int d = 0; d < n_out; ++d) {
        float f = src_coord(d, n_in, n_out, 0);
        int i = (int)floorf(f);
        f -= (float)i;
        if (i < 0) { i = 0; f = 0.f; }
        if (i >= n_in - 1) { i = n_in - 2; f = 1.f; }
        ofs[d] = i;
        w0[d] = 1.f - f;
        w1[d] = f;
    }
}

/* Keys cubic (A=-0.75) with replicate folding: resize_naive.cpp:130-185.
 * The folds are applied in the reference's order; ofs is the centre tap
 * (taps at ofs-1 .. ofs+2). */
void oracle_cubic_table(int n_in, int n_out, int32_t* ofs, float* coef) {
    const float A = -0.75f;
    double s = (double)n_in / (double)n_out;
    for (int d = 0; d < n_out; ++d) {
        float f = (float)(((double)d + 0.5) * s - 0.5);
        int i = (int)floorf(f);
        f -= (float)i;
        float t0 = f + 1.f, t1 = f, t2 = 1.f - f;
        float c0 = A * t0 * t0 * t0 - 5.f * A * t0 * t0 + 8.f * A * t0 - 4.f * A;
        float c1 = (A + 2.f) * t1 * t1 * t1 - (A + 3.f) * t1 * t1 + 1.f;
        float c2 = (A + 2.f) * t2 * t2 * t2 - (A + 3.f) * t2 * t2 + 1.f;
        float c3 = 1.f - c0 - c1 - c2;
        if (i <= -1) { i = 1; c0 = 1.f - c3; c1 = c3; c2 = 0.f; c3 = 0.f; }
        if (i == 0) { i = 1; c0 = c0 + c1; c1 = c2; c2 = c3; c3 = 0.f; }
        if (i == n_in - 2) { i = n_in - 3; c3 = c2 + c3; c2 = c1; c1 = c0; c0 = 0.f; }
        if (i >= n_in - 1) { i = n_in - 3; c3 = 1.f - c0; c2 = c0; c1 = 0.f; c0 = 0.f; }
        ofs[d] = i;
        coef[4 * d + 0] = c0;
        coef[4 * d + 1] = c1;
        coef[4 * d + 2] = c2;
        coef[4 * d + 3] = c3;
    }
}

/* In-place inverse of a forward 2x3 map, warp_affine.cpp:121-133.
 * Note the mixed precision: products of two floats are float, anything
 * touching D is double, results are stored back as float. */
void oracle_invert_affine(const float m[6], float inv[6]) {
    float a[6];
    memcpy(a, m, sizeof(a));
    double D = (double)(a[0] * a[4] - a[1] * a[3]);
    D = D != 0 ? 1. / D : 0;
    double A11 = (double)a[4] * D;
    double A22 = (double)a[0] * D;
    a[0] = (float)A11;
    a[1] = (float)((double)a[1] * -D);
    a[3] = (float)((double)a[3] * -D);
    a[4] = (float)A22;
    double b1 = (double)(-a[0] * a[2] - a[1] * a[5]);
    double b2 = (double)(-a[3] * a[2] - a[4] * a[5]);
    a[2] = (float)b1;
    a[5] = (float)b2;
    memcpy(inv, a, sizeof(a));
}

/* get_rotation_matrix_2D(VPoint(0,0), rot, scale) + the aux translation fix,
 * warp_affine.cpp:76-109.  angle is a float; cos/sin of a float resolve to the
 * float overloads in the reference's C++ (cosf/sinf). */
void oracle_rotation_matrix(float scale, float rot_deg, const double aux[4], float m[6]) {
    float angle = (float)((double)rot_deg * (M_PI / 180));
    double alpha = (double)(scale * cosf(angle));
    double beta = (double)(scale * sinf(angle));
    m[0] = (float)alpha;
    m[1] = (float)beta;
    m[3] = (float)-beta;
    m[4] = (float)alpha;
    m[2] = (float)(aux[2] - (double)m[0] * aux[0] - (double)m[1] * aux[1]);
    m[5] = (float)(aux[3] - (double)m[3] * aux[0] - (double)m[4] * aux[1]);
}

/* ------------------------------------------------------------------------ */
/* u8 bilinear.  naive: resize_naive.cpp:10-68 (Sum S*wx*wy >> 22, truncating).
 * neon/opencv: resize_neon.cpp:79-181 (row = (S0*a0+S1*a1)>>4 as int16, then
 * ((r0*b0)>>16 + (r1*b1)>>16 + 2)>>2 saturated to u8). */
void oracle_resize_linear_u8(const uint8_t* src, int w_in, int h_in, int cc,
                             uint8_t* dst, int w_out, int h_out, int mode) {
    int32_t* xo = (int32_t*)malloc(sizeof(int32_t) * w_out);
    int16_t* xa = (int16_t*)malloc(sizeof(int16_t) * w_out);
    int16_t* xb = (int16_t*)malloc(sizeof(int16_t) * w_out);
    int32_t* yo = (int32_t*)malloc(sizeof(int32_t) * h_out);
    int16_t* ya = (int16_t*)malloc(sizeof(int16_t) * h_out);
    int16_t* yb = (int16_t*)malloc(sizeof(int16_t) * h_out);
    oracle_linear_table(w_in, w_out, mode, xo, xa, xb);
    oracle_linear_table(h_in, h_out, mode, yo, ya, yb);
    const int64_t rs = (int64_t)w_in * cc;
    for (int y = 0; y < h_out; ++y) {
        const uint8_t* r0 = src + yo[y] * rs;
        const uint8_t* r1 = r0 + rs;
        uint8_t* out = dst + (int64_t)y * w_out * cc;
        for (int x = 0; x < w_out; ++x) {
            const int64_t p = (int64_t)xo[x] * cc;
            for (int k = 0; k < cc; ++k) {
                int32_t tl = r0[p + k], tr = r0[p + cc + k];
                int32_t bl = r1[p + k], br = r1[p + cc + k];
                int32_t v;
                if (mode == ORACLE_LINEAR_NAIVE) {
                    v = (tl * xa[x] * ya[y] + bl * xa[x] * yb[y] +
                         tr * xb[x] * ya[y] + br * xb[x] * yb[y]) >> 22;
                    out[x * cc + k] = (uint8_t)v;
                } else {
                    int16_t h0 = (int16_t)((tl * xa[x] + tr * xb[x]) >> 4);
                    int16_t h1 = (int16_t)((bl * xa[x] + br * xb[x]) >> 4);
                    v = (((int32_t)h0 * ya[y]) >> 16) + (((int32_t)h1 * yb[y]) >> 16) + 2;
                    v = (int16_t)(v >> 2);
                    out[x * cc + k] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
                }
            }
        }
    }
    free(xo); free(xa); free(xb); free(yo); free(ya); free(yb);
}

/* INTER_NEAREST.  The reference has no nearest loop of its own: Resize::resize
 * hands every mode but LINEAR/CUBIC to resize_opencv (resize.cpp:44-49),
 * i.e. cv::resize of the pinned OpenCV 2.4.13.4 (CMakeLists.txt:23).  Its
 * published algorithm (imgwarp.cpp, cv::resize -> resizeNN), restated:
 * inv_scale = (double)dsize / ssize, ifx = 1. / inv_scale, and
 *   sx = min(cvFloor(x * ifx), w_in - 1),  sy = min(cvFloor(y * ify), h_in - 1);
 * a same-size resize is a copy (cv::resize's dsize == ssize shortcut, which
 * the formula reproduces).  PARITY UNPINNED: no reference entry runs this
 * path here (OpenCV's binaries are not loaded) and its tests hold no nearest
 * output (test_resize.cpp passes INTER_NEAREST as fx).
 * esize bytes per element, cc interleaved channels. */
void oracle_resize_nearest(const void* src, int w_in, int h_in, int cc, int esize,
                           void* dst, int w_out, int h_out) {
    const double ifx = 1. / ((double)w_out / w_in), ify = 1. / ((double)h_out / h_in);
    const size_t px = (size_t)cc * esize;
    for (int y = 0; y < h_out; ++y) {
        int sy = (int)floor(y * ify);
        if (sy > h_in - 1) sy = h_in - 1;
        for (int x = 0; x < w_out; ++x) {
            int sx = (int)floor(x * ifx);
            if (sx > w_in - 1) sx = w_in - 1;
            memcpy((char*)dst + ((size_t)y * w_out + x) * px, (const char*)src + ((size_t)sy * w_in + sx) * px, px);
        }
    }
}

/* INTER_AREA at an integer downscale.  Like nearest, the reference hands it
 * to cv::resize (resize.cpp:44-49); its own attempt,
 * src_deprecated/img_resize_inter_area.cpp:21-55, builds OpenCV's ofs/xofs
 * tables and stops.  OpenCV 2.4.13.4's published algorithm (imgwarp.cpp,
 * resizeAreaFast_Invoker), restated: with ax = w_in / w_out, ay = h_in / h_out
 * exact integers, output (x, y, k) is
 *  - u8, ax == ay == 2 and cn in {1, 3, 4}: (a + b + c + d + 2) >> 2, the
 *    ResizeAreaFastVec<uchar>::fast_mode path (scalar loop and its SSE2/NEON
 *    vector op alike), i.e. the 2x2 block mean rounded half UP;
 *  - otherwise: the sum over the block rows r, columns q (taps grouped 4 per
 *    add as its CV_ENABLE_UNROLLED loop) of src(x*ax + q, y*ay + r, k), times
 *    1.f/(ax*ay) in fp32; u8 rounds half to even (saturate_cast<uchar> =
 *    cvRound = lrint).  For fp32 2x2 blocks (cn 1/4) the ARM build's NEON
 *    ResizeAreaFastVec_SIMD_32f sums (a+b)+(c+d) and multiplies by 0.25f on
 *    its vector body; this restatement keeps the generic order there (PARITY
 *    UNPINNED for fp32 2x2, by at most one ulp).
 * PARITY UNPINNED: no reference entry runs this path here and its tests hold
 * no area output.  esize 1 (u8, int sum) or 4 (fp32, float sum). */
void oracle_resize_area(const void* src, int w_in, int h_in, int cc, int esize,
                        void* dst, int w_out, int h_out) {
    const int ax = w_in / w_out, ay = h_in / h_out, area = ax * ay;
    const float scale = 1.f / (float)area;
    /* ResizeAreaFastVec<uchar>::fast_mode (scale 2x2, cn 1/3/4) */
    const int fast22 = esize == 1 && ax == 2 && ay == 2 && (cc == 1 || cc == 3 || cc == 4);
    for (int y = 0; y < h_out; ++y)
        for (int x = 0; x < w_out; ++x)
            for (int k = 0; k < cc; ++k) {
                int isum = 0;
                float fsum = 0.f;
                int t = 0;
                for (; t <= area - 4; t += 4) {
                    int iv[4];
                    float fv[4];
                    for (int j = 0; j < 4; ++j) {
                        const int r = (t + j) / ax, q = (t + j) % ax;
                        const size_t i = ((size_t)(y * ay + r) * w_in + (size_t)x * ax + q) * cc + k;
                        if (esize == 1) iv[j] = ((const uint8_t*)src)[i];
                        else fv[j] = ((const float*)src)[i];
                    }
                    if (esize == 1) isum += iv[0] + iv[1] + iv[2] + iv[3];
                    else fsum += ((fv[0] + fv[1]) + fv[2]) + fv[3];
                }
                for (; t < area; ++t) {
                    const int r = t / ax, q = t % ax;
                    const size_t i = ((size_t)(y * ay + r) * w_in + (size_t)x * ax + q) * cc + k;
                    if (esize == 1) isum += ((const uint8_t*)src)[i];
                    else fsum += ((const float*)src)[i];
                }
                const size_t o = ((size_t)y * w_out + x) * cc + k;
                if (esize == 1 && fast22) {
                    ((uint8_t*)dst)[o] = (uint8_t)((isum + 2) >> 2);
                } else if (esize == 1) {
                    const float m = (float)isum * scale;
                    ((uint8_t*)dst)[o] = (uint8_t)lrintf(m);
                } else {
                    ((float*)dst)[o] = fsum * scale;
                }
            }
}

/* INTER_AREA at any other scale.  The reference hands it to cv::resize
 * (resize.cpp:44-49); OpenCV 2.4.13.4's published algorithm (imgwarp.cpp,
 * cv::resize), restated.  inv_scale = dsize / ssize (double), scale = 1 /
 * inv_scale:
 *  - both scales >= 1 (a down-scale, not integral): resizeArea_ over the
 *    computeResizeAreaTab weight tables; per output row the source rows'
 *    horizontally weighted sums buf = sum_k S[si_k] * alpha_k (fp32, in table
 *    order from 0) are accumulated as sum = beta_0 * buf_0, sum += beta_j *
 *    buf_j (fp32), then saturate_cast (u8: cvRound, half to even);
 *  - otherwise (an up-scale on either axis): the bilinear resize with the
 *    area-mode taps sx = floor(dx * scale), fx = (float)((dx + 1) - (sx + 1)
 *    * inv_scale), fx = fx <= 0 ? 0 : fx - floor(fx); at sx >= n - 1 the tap
 *    is (n - 1, fx = 0).  u8: coefficients saturate_cast<short>(c * 2048)
 *    (half even) and OpenCV's fixed-point rows, ((h0 >> 4) * b0 >> 16) +
 *    ((h1 >> 4) * b1 >> 16) + 2 >> 2 (the VResizeLinearVec_32s8u form, the
 *    arithmetic of this build's OPENCV bilinear mode); fp32: h = S0 * a0 +
 *    S1 * a1 per row, out = h0 * b0 + h1 * b1.
 * PARITY UNPINNED: no reference entry runs this path here and its tests hold
 * no area output.  cn <= 4 (OpenCV asserts it for resizeArea_). */
typedef struct { int di, si; float alpha; } oracle_area_tab;

/* computeResizeAreaTab (imgwarp.cpp): returns the entry count */
int oracle_area_table(int ssize, int dsize, int cn, double scale, int* di, int* si, float* alpha) {
    int k = 0;
    for (int dx = 0; dx < dsize; ++dx) {
        const double fsx1 = dx * scale;
        const double fsx2 = fsx1 + scale;
        const double cell = scale < ssize - fsx1 ? scale : ssize - fsx1;
        int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
        if (sx2 > ssize - 1) sx2 = ssize - 1;
        if (sx1 > sx2) sx1 = sx2;
        if (sx1 - fsx1 > 1e-3) {
            di[k] = dx * cn; si[k] = (sx1 - 1) * cn; alpha[k++] = (float)((sx1 - fsx1) / cell);
        }
        for (int sx = sx1; sx < sx2; ++sx) {
            di[k] = dx * cn; si[k] = sx * cn; alpha[k++] = (float)(1.0 / cell);
        }
        if (fsx2 - sx2 > 1e-3) {
            double t = fsx2 - sx2;
            if (t > 1.) t = 1.;
            if (t > cell) t = cell;
            di[k] = dx * cn; si[k] = sx2 * cn; alpha[k++] = (float)(t / cell);
        }
    }
    return k;
}

static void area_frac(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out, int h_out,
                      double sx, double sy) {
    int *xdi = malloc(sizeof(int) * 2 * (w_in + 2)), *xsi = malloc(sizeof(int) * 2 * (w_in + 2));
    int *ydi = malloc(sizeof(int) * 2 * (h_in + 2)), *ysi = malloc(sizeof(int) * 2 * (h_in + 2));
    float *xal = malloc(sizeof(float) * 2 * (w_in + 2)), *yal = malloc(sizeof(float) * 2 * (h_in + 2));
    const int nx = oracle_area_table(w_in, w_out, cc, sx, xdi, xsi, xal);
    const int ny = oracle_area_table(h_in, h_out, 1, sy, ydi, ysi, yal);
    const int W = w_out * cc;
    float* buf = malloc(sizeof(float) * W);
    float* sum = malloc(sizeof(float) * W);
    int prev = ydi[0];
    for (int x = 0; x < W; ++x) sum[x] = 0.f;
    for (int j = 0; j < ny; ++j) {
        const float beta = yal[j];
        const int dy = ydi[j];
        const size_t row = (size_t)ysi[j] * w_in * cc;
        for (int x = 0; x < W; ++x) buf[x] = 0.f;
        for (int k = 0; k < nx; ++k)
            for (int c = 0; c < cc; ++c) {
                const float v = esize == 1 ? (float)((const uint8_t*)src)[row + xsi[k] + c]
                                           : ((const float*)src)[row + xsi[k] + c];
                buf[xdi[k] + c] = buf[xdi[k] + c] + v * xal[k];
            }
        if (dy != prev) {
            for (int x = 0; x < W; ++x) {
                const size_t o = (size_t)prev * W + x;
                if (esize == 1) {
                    long r = lrintf(sum[x]);
                    ((uint8_t*)dst)[o] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
                } else {
                    ((float*)dst)[o] = sum[x];
                }
                sum[x] = beta * buf[x];
            }
            prev = dy;
        } else {
            for (int x = 0; x < W; ++x) sum[x] = sum[x] + beta * buf[x];
        }
    }
    for (int x = 0; x < W; ++x) {
        const size_t o = (size_t)prev * W + x;
        if (esize == 1) {
            long r = lrintf(sum[x]);
            ((uint8_t*)dst)[o] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        } else {
            ((float*)dst)[o] = sum[x];
        }
    }
    free(xdi); free(xsi); free(ydi); free(ysi); free(xal); free(yal); free(buf); free(sum);
}

/* the area-mode bilinear taps of one axis (cv::resize, area_mode branch) */
void oracle_area_linear_tap(int d, int n_in, double scale, double inv_scale, int* i, float* f) {
    int sx = (int)floor(d * scale);
    float fx = (float)((d + 1) - (sx + 1) * inv_scale);
    fx = fx <= 0 ? 0.f : fx - (float)floor(fx);
    if (sx >= n_in - 1) { fx = 0.f; sx = n_in - 1; }
    *i = sx;
    *f = fx;
}

static void area_up(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out, int h_out,
                    double sx, double sy, double ix, double iy) {
    for (int y = 0; y < h_out; ++y) {
        int ty; float fy;
        oracle_area_linear_tap(y, h_in, sy, iy, &ty, &fy);
        const int ty1 = ty + 1 < h_in ? ty + 1 : h_in - 1;
        const float b0f = 1.f - fy, b1f = fy;
        const int b0 = (int)lrintf(b0f * 2048.f), b1 = (int)lrintf(b1f * 2048.f);
        for (int x = 0; x < w_out; ++x) {
            int tx; float fx;
            oracle_area_linear_tap(x, w_in, sx, ix, &tx, &fx);
            const int tx1 = tx + 1 < w_in ? tx + 1 : w_in - 1;
            const float a0f = 1.f - fx, a1f = fx;
            const int a0 = (int)lrintf(a0f * 2048.f), a1 = (int)lrintf(a1f * 2048.f);
            for (int c = 0; c < cc; ++c) {
                const size_t p00 = ((size_t)ty * w_in + tx) * cc + c, p01 = ((size_t)ty * w_in + tx1) * cc + c;
                const size_t p10 = ((size_t)ty1 * w_in + tx) * cc + c, p11 = ((size_t)ty1 * w_in + tx1) * cc + c;
                const size_t o = ((size_t)y * w_out + x) * cc + c;
                if (esize == 1) {
                    const uint8_t* S = (const uint8_t*)src;
                    /* dx >= xmax (tx == w_in - 1): S[tx] * 2048, i.e. a1 = 0 */
                    const int h0 = S[p00] * a0 + S[p01] * a1, h1 = S[p10] * a0 + S[p11] * a1;
                    int v = ((((int16_t)(h0 >> 4)) * b0) >> 16) + ((((int16_t)(h1 >> 4)) * b1) >> 16) + 2;
                    v >>= 2;
                    ((uint8_t*)dst)[o] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
                } else {
                    const float* S = (const float*)src;
                    const float h0 = tx >= w_in - 1 ? S[p00] : S[p00] * a0f + S[p01] * a1f;
                    const float h1 = tx >= w_in - 1 ? S[p10] : S[p10] * a0f + S[p11] * a1f;
                    ((float*)dst)[o] = h0 * b0f + h1 * b1f;
                }
            }
        }
    }
}

/* INTER_AREA at any scale: the integer fast path (above), resizeArea_ or the
 * area-mode bilinear.  inv_x / inv_y = cv::resize's inv_scale (0: dsize /
 * ssize, the dsize given case). */
void oracle_resize_area_any(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out,
                            int h_out, double inv_x, double inv_y) {
    if (inv_x <= 0) inv_x = (double)w_out / w_in;
    if (inv_y <= 0) inv_y = (double)h_out / h_in;
    const double sx = 1. / inv_x, sy = 1. / inv_y;
    if (sx >= 1 && sy >= 1) {
        const double rx = nearbyint(sx), ry = nearbyint(sy);
        if (fabs(sx - rx) < DBL_EPSILON && fabs(sy - ry) < DBL_EPSILON && (int)rx * w_out == w_in &&
            (int)ry * h_out == h_in) {
            oracle_resize_area(src, w_in, h_in, cc, esize, dst, w_out, h_out);
            return;
        }
        area_frac(src, w_in, h_in, cc, esize, dst, w_out, h_out, sx, sy);
        return;
    }
    area_up(src, w_in, h_in, cc, esize, dst, w_out, h_out, sx, sy, inv_x, inv_y);
}

/* fp32 bilinear, resize_naive.cpp:70-128; value summed lt,lb,rt,rb. */
void oracle_resize_linear_f32(const float* src, int w_in, int h_in, int cc,
                              float* dst, int w_out, int h_out) {
    int32_t* xo = (int32_t*)malloc(sizeof(int32_t) * w_out);
    float* xa = (float*)malloc(sizeof(float) * w_out);
    float* xb = (float*)malloc(sizeof(float) * w_out);
    int32_t* yo = (int32_t*)malloc(sizeof(int32_t) * h_out);
    float* ya = (float*)malloc(sizeof(float) * h_out);
    float* yb = (float*)malloc(sizeof(float) * h_out);
    oracle_linear_table_f32(w_in, w_out, xo, xa, xb);
    oracle_linear_table_f32(h_in, h_out, yo, ya, yb);
    const int64_t rs = (int64_t)w_in * cc;
    for (int y = 0; y < h_out; ++y) {
        const float* r0 = src + yo[y] * rs;
        const float* r1 = r0 + rs;
        float* out = dst + (int64_t)y * w_out * cc;
        for (int x = 0; x < w_out; ++x) {
            const int64_t p = (int64_t)xo[x] * cc;
            for (int k = 0; k < cc; ++k) {
                float v = r0[p + k] * xa[x] * ya[y];
                v += r1[p + k] * xa[x] * yb[y];
                v += r0[p + cc + k] * xb[x] * ya[y];
                v += r1[p + cc + k] * xb[x] * yb[y];
                out[x * cc + k] = v;
            }
        }
    }
    free(xo); free(xa); free(xb); free(yo); free(ya); free(yb);
}

/* fp32 cubic, resize_naive.cpp:187-366 (3ch) / :368-529 (1ch): horizontal
 * 4-tap per source row (S[-1]a0+S[0]a1+S[1]a2+S[2]a3), then vertical 4-tap
 * (r0b0+r1b1+r2b2+r3b3).  The reference's ring of row buffers only caches
 * these per-row values, so evaluating them per output pixel is identical.
 * Tables are kept separate (the reference's hwc/chw wrappers overlap them
 * when w_out != h_out, resize_naive.cpp:537). */
void oracle_resize_cubic_f32(const float* src, int w_in, int h_in, int cc,
                             float* dst, int w_out, int h_out) {
    int32_t* xo = (int32_t*)malloc(sizeof(int32_t) * w_out);
    float* xc = (float*)malloc(sizeof(float) * 4 * w_out);
    int32_t* yo = (int32_t*)malloc(sizeof(int32_t) * h_out);
    float* yc = (float*)malloc(sizeof(float) * 4 * h_out);
    oracle_cubic_table(w_in, w_out, xo, xc);
    oracle_cubic_table(h_in, h_out, yo, yc);
    const int64_t rs = (int64_t)w_in * cc;
    for (int y = 0; y < h_out; ++y) {
        const float* rows[4];
        for (int j = 0; j < 4; ++j) rows[j] = src + (int64_t)(yo[y] - 1 + j) * rs;
        const float* b = yc + 4 * y;
        for (int x = 0; x < w_out; ++x) {
            const float* a = xc + 4 * x;
            const int64_t p = (int64_t)(xo[x] - 1) * cc;
            for (int k = 0; k < cc; ++k) {
                float h[4];
                for (int j = 0; j < 4; ++j) {
                    const float* s = rows[j] + p + k;
                    h[j] = s[0] * a[0] + s[cc] * a[1] + s[2 * cc] * a[2] + s[3 * cc] * a[3];
                }
                dst[((int64_t)y * w_out + x) * cc + k] = h[0] * b[0] + h[1] * b[1] + h[2] * b[2] + h[3] * b[3];
            }
        }
    }
    free(xo); free(xc); free(yo); free(yc);
}

/* ------------------------------------------------------------------------ */
/* Affine bilinear, warp_affine_naive.cpp:9-106.  inv = the already inverted
 * map.  Pixels whose top-left tap falls outside [0,w-2]x[0,h-2] are skipped
 * (left untouched); the caller pre-fills dst with the border value.  The
 * reference tests floor(f) < 0 || floor(f) >= n-1 on an int; the equivalent
 * float test below avoids the undefined int conversion of far-away points. */
static int warp_tap(float f, int n, int* i, float* frac) {
    if (!(f >= 0.f && f < (float)(n - 1))) return 0;
    int k = (int)floorf(f);
    if (k >= n - 1) return 0;
    *i = k;
    *frac = f - (float)k;
    return 1;
}

void oracle_warp_affine_u8(const uint8_t* src, int w_in, int h_in, int cc,
                           uint8_t* dst, int w_out, int h_out, const float m[6]) {
    for (int y = 0; y < h_out; ++y) {
        for (int x = 0; x < w_out; ++x) {
            float fx = m[0] * (float)x + m[1] * (float)y + m[2];
            float fy = m[3] * (float)x + m[4] * (float)y + m[5];
            int sx, sy;
            float ax, ay;
            if (!warp_tap(fy, h_in, &sy, &ay)) continue;
            if (!warp_tap(fx, w_in, &sx, &ax)) continue;
            int32_t wy0 = oracle_sat_short((1.f - ay) * 2048.f), wy1 = 2048 - wy0;
            int32_t wx0 = oracle_sat_short((1.f - ax) * 2048.f), wx1 = 2048 - wx0;
            const uint8_t* r0 = src + ((int64_t)sy * w_in + sx) * cc;
            const uint8_t* r1 = r0 + (int64_t)w_in * cc;
            uint8_t* out = dst + ((int64_t)y * w_out + x) * cc;
            for (int k = 0; k < cc; ++k) {
                int32_t v = r0[k] * wx0 * wy0 + r1[k] * wx0 * wy1 +
                            r0[cc + k] * wx1 * wy0 + r1[cc + k] * wx1 * wy1;
                out[k] = (uint8_t)(v >> 22);
            }
        }
    }
}

void oracle_warp_affine_f32(const float* src, int w_in, int h_in, int cc,
                            float* dst, int w_out, int h_out, const float m[6]) {
    for (int y = 0; y < h_out; ++y) {
        for (int x = 0; x < w_out; ++x) {
            float fx = m[0] * (float)x + m[1] * (float)y + m[2];
            float fy = m[3] * (float)x + m[4] * (float)y + m[5];
            int sx, sy;
            float ax, ay;
            if (!warp_tap(fy, h_in, &sy, &ay)) continue;
            if (!warp_tap(fx, w_in, &sx, &ax)) continue;
            float y0 = 1.f - ay, y1 = ay, x0 = 1.f - ax, x1 = ax;
            const float* r0 = src + ((int64_t)sy * w_in + sx) * cc;
            const float* r1 = r0 + (int64_t)w_in * cc;
            float* out = dst + ((int64_t)y * w_out + x) * cc;
            for (int k = 0; k < cc; ++k) {
                float v = r0[k] * x0 * y0;
                v += r1[k] * x0 * y1;
                v += r0[cc + k] * x1 * y0;
                v += r1[cc + k] * x1 * y1;
                out[k] = v;
            }
        }
    }
}

/* Border modes other than BORDER_CONSTANT (build extension, PARITY UNPINNED:
 * the reference hands them to OpenCV, warp_affine.cpp:114-118 -> :48-50, and
 * recurses forever without it).  Pixels whose top-left tap is inside
 * [0,w-2]x[0,h-2] are exactly the naive sampler's (above); every other pixel
 * takes its four taps at floor(f), floor(f)+1 mapped through OpenCV 2.4's
 * borderInterpolate (core/base.hpp: REPLICATE clamps, REFLECT and
 * REFLECT_101 mirror, WRAP is modulo; the reflect loop restated in closed
 * form), with the naive sampler's weights: w0 = SATURATE_CAST_SHORT((1 -
 * frac) * 2048), w1 = 2048 - w0 for u8; (1 - frac, frac) in the lt, lb, rt,
 * rb order for fp32.  f is clamped to +-1e9 first (NaN -> -1e9).
 * TRANSPARENT (5) and CONSTANT (0) leave those pixels to the caller.
 * mode: 1 REPLICATE, 2 REFLECT, 3 WRAP, 4 REFLECT_101. */
static int oracle_border_index(int p, int len, int mode) {
    if (p >= 0 && p < len) return p;
    if (mode == 1) return p < 0 ? 0 : len - 1;
    if (mode == 3) {
        int q = p % len;
        return q < 0 ? q + len : q;
    }
    if (len == 1) return 0;
    {
        const int delta = mode == 4;
        /* borderInterpolate's loop: p < 0 -> -p - 1 + delta; p >= len ->
         * len - 1 - (p - len) - delta; repeat until inside.  Closed form: */
        const long long period = 2LL * len - 2 * delta;
        long long q = (long long)p % period;
        if (q < 0) q += period;
        return (int)(q < len ? q : period - 1 + delta - q);
    }
}

static void oracle_border_tap(float f, int* i, float* frac) {
    float c = f;
    if (!(c >= -1e9f)) c = -1e9f; /* also NaN */
    if (c > 1e9f) c = 1e9f;
    *i = (int)floorf(c);
    *frac = c - (float)*i;
}

void oracle_warp_affine_border(const void* src, int w_in, int h_in, int cc, int esize,
                               void* dst, int w_out, int h_out, const float m[6], int mode) {
    for (int y = 0; y < h_out; ++y) {
        for (int x = 0; x < w_out; ++x) {
            float fx = m[0] * (float)x + m[1] * (float)y + m[2];
            float fy = m[3] * (float)x + m[4] * (float)y + m[5];
            int sx, sy, ix, iy;
            float ax, ay;
            if (warp_tap(fy, h_in, &sy, &ay) && warp_tap(fx, w_in, &sx, &ax)) continue; /* interior */
            if (mode < 1 || mode > 4) continue;
            oracle_border_tap(fx, &ix, &ax);
            oracle_border_tap(fy, &iy, &ay);
            const int x0 = oracle_border_index(ix, w_in, mode), x1 = oracle_border_index(ix + 1, w_in, mode);
            const int y0 = oracle_border_index(iy, h_in, mode), y1 = oracle_border_index(iy + 1, h_in, mode);
            const size_t lt = ((size_t)y0 * w_in + x0) * cc, rt = ((size_t)y0 * w_in + x1) * cc;
            const size_t lb = ((size_t)y1 * w_in + x0) * cc, rb = ((size_t)y1 * w_in + x1) * cc;
            const size_t o = ((size_t)y * w_out + x) * cc;
            if (esize == 1) {
                const uint8_t* s = (const uint8_t*)src;
                const int32_t wy0 = oracle_sat_short((1.f - ay) * 2048.f), wy1 = 2048 - wy0;
                const int32_t wx0 = oracle_sat_short((1.f - ax) * 2048.f), wx1 = 2048 - wx0;
                for (int k = 0; k < cc; ++k) {
                    const int32_t v = s[lt + k] * wx0 * wy0 + s[lb + k] * wx0 * wy1 +
                                      s[rt + k] * wx1 * wy0 + s[rb + k] * wx1 * wy1;
                    ((uint8_t*)dst)[o + k] = (uint8_t)(v >> 22);
                }
            } else {
                const float* s = (const float*)src;
                const float ya = 1.f - ay, yb = ay, xa = 1.f - ax, xb = ax;
                for (int k = 0; k < cc; ++k) {
                    float v = s[lt + k] * xa * ya;
                    v += s[lb + k] * xa * yb;
                    v += s[rt + k] * xb * ya;
                    v += s[rb + k] * xb * yb;
                    ((float*)dst)[o + k] = v;
                }
            }
        }
    }
}

/* cv::warpAffine with INTER_NEAREST (the reference hands every flag but
 * INTER_LINEAR to OpenCV, warp_affine.cpp:114-118), as OpenCV 2.4.13's
 * imgwarp.cpp computes it: the float map widened to double and, unless
 * inverse_map (WARP_INVERSE_MAP), inverted in double; AB_BITS = 10 fixed
 * point with cvRound (half to even)
 *   X0 = cvRound((M1 y + M2) 1024) + 512, X = (X0 + cvRound(M0 x 1024)) >> 10
 * (Y likewise with M3..M5), clamped to short as remap's map; then remap's
 * nearest sampler: inside -> the source pixel; outside -> border (mode 0),
 * dst untouched (5), else the pixel at borderInterpolate (modes 1-4).
 * esize 1 (u8) or 4 (fp32); border[] already in the element type's range.
 * Parity unpinned: no OpenCV runs here. */
void oracle_warp_affine_nn(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out, int h_out,
                           const float m[6], int inverse_map, int mode, const double border[4]) {
    double M[6];
    for (int i = 0; i < 6; ++i) M[i] = (double)m[i];
    if (!inverse_map) {
        double D = M[0] * M[4] - M[1] * M[3];
        D = D != 0 ? 1. / D : 0;
        const double A11 = M[4] * D, A22 = M[0] * D;
        M[0] = A11;
        M[1] *= -D;
        M[3] *= -D;
        M[4] = A22;
        const double b1 = -M[0] * M[2] - M[1] * M[5];
        const double b2 = -M[3] * M[2] - M[4] * M[5];
        M[2] = b1;
        M[5] = b2;
    }
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    for (int y = 0; y < h_out; ++y) {
        const int X0 = (int)nearbyint((M[1] * y + M[2]) * 1024.0) + 512;
        const int Y0 = (int)nearbyint((M[4] * y + M[5]) * 1024.0) + 512;
        for (int x = 0; x < w_out; ++x) {
            int X = (int)((uint32_t)X0 + (uint32_t)(int)nearbyint(M[0] * x * 1024.0)) >> 10;
            int Y = (int)((uint32_t)Y0 + (uint32_t)(int)nearbyint(M[3] * x * 1024.0)) >> 10;
            X = X < -32768 ? -32768 : (X > 32767 ? 32767 : X);
            Y = Y < -32768 ? -32768 : (Y > 32767 ? 32767 : Y);
            uint8_t* o = d + ((int64_t)y * w_out + x) * cc * esize;
            const int inside = X >= 0 && X < w_in && Y >= 0 && Y < h_in;
            if (!inside && mode == 5) continue;
            if (!inside && mode == 0) {
                for (int k = 0; k < cc; ++k) {
                    if (esize == 1) o[k] = (uint8_t)border[k];
                    else { const float f = (float)border[k]; memcpy(o + 4 * k, &f, 4); }
                }
                continue;
            }
            const int sx = inside ? X : oracle_border_index(X, w_in, mode);
            const int sy = inside ? Y : oracle_border_index(Y, h_in, mode);
            memcpy(o, s + ((int64_t)sy * w_in + sx) * cc * esize, (size_t)cc * esize);
        }
    }
}

/* ------------------------------------------------------------------------ */
/* YUV420 semi-planar -> BGR, cvt_color.cpp:39-135 (BT.601 full range, 7-bit
 * integer coefficients, arithmetic shifts).  v_first=1: NV21 (VU pairs);
 * v_first=0: NV12 (UV pairs; the reference decodes NV12 as NV21, see
 * DESIGN.md).  rgb_out swaps the output order.  w, h = BGR size, both even. */
void oracle_yuv420sp_to_bgr(const uint8_t* src, uint8_t* dst, int w, int h, int v_first, int rgb_out) {
    const uint8_t* yp = src;
    const uint8_t* uv = src + (int64_t)w * h;
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            const uint8_t* pair = uv + (int64_t)(y / 2) * w + (x & ~1);
            int v = v_first ? pair[0] : pair[1];
            int u = v_first ? pair[1] : pair[0];
            int ra = (179 * (v - 128)) >> 7;
            int ga = (44 * (u - 128) + 91 * (v - 128)) >> 7;
            int ba = (227 * (u - 128)) >> 7;
            int Y = yp[(int64_t)y * w + x];
            int r = Y + ra, g = Y - ga, b = Y + ba;
            r = r < 0 ? 0 : (r > 255 ? 255 : r);
            g = g < 0 ? 0 : (g > 255 ? 255 : g);
            b = b < 0 ? 0 : (b > 255 ? 255 : b);
            uint8_t* o = dst + ((int64_t)y * w + x) * 3;
            o[0] = (uint8_t)(rgb_out ? r : b);
            o[1] = (uint8_t)g;
            o[2] = (uint8_t)(rgb_out ? b : r);
        }
    }
}

/* The cvt_color codes the reference hands to cv::cvtColor (cvt_color.cpp:
 * 139-141; cv.h:62-74): OpenCV 2.4.13's YUV420 -> RGB(A) of YUV420sp2RGB8
 * / YUV420p2RGB8 (ITU-R BT.601, 20-bit fixed point; the constants and the
 * formula as OpenCV 2.4.13.4's own YUV2RGBA_NV12 kernel text states them,
 * thirdparty/opencv_2.4.13.4/.../libopencv_ocl.so):
 *   y' = max(0, Y - 16) * 1220542
 *   R = sat((y' + 2^19 + 1673527 v) >> 20)
 *   G = sat((y' + 2^19 - 852492 v - 409993 u) >> 20)
 *   B = sat((y' + 2^19 + 2116026 u) >> 20),  u = U - 128, v = V - 128.
 * layout 0: NV12 (UV pairs), 1: NV21 (VU pairs), 2: YV12 (planar: Y, then
 * the (w/2)x(h/2) V plane, then U), 3: IYUV/I420 (Y, U, V).  dcn = 3 or 4
 * (alpha 255); bidx = 0: BGR(A) order, 2: RGB(A).  Parity unpinned (no
 * OpenCV runs here); w, h even. */
void oracle_yuv420_cv(const uint8_t* src, uint8_t* dst, int w, int h, int layout, int dcn, int bidx) {
    const uint8_t* yp = src;
    const uint8_t* c0 = src + (int64_t)w * h;
    const uint8_t* c1 = c0 + (int64_t)(w / 2) * (h / 2);
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            int U, V;
            if (layout <= 1) {
                const uint8_t* pair = c0 + (int64_t)(y / 2) * w + (x & ~1);
                U = layout == 0 ? pair[0] : pair[1];
                V = layout == 0 ? pair[1] : pair[0];
            } else {
                const int64_t k = (int64_t)(y / 2) * (w / 2) + x / 2;
                U = layout == 2 ? c1[k] : c0[k];
                V = layout == 2 ? c0[k] : c1[k];
            }
            const int u = U - 128, v = V - 128;
            const int ruv = (1 << 19) + 1673527 * v;
            const int guv = (1 << 19) - 852492 * v - 409993 * u;
            const int buv = (1 << 19) + 2116026 * u;
            int yy = (int)yp[(int64_t)y * w + x] - 16;
            yy = (yy < 0 ? 0 : yy) * 1220542;
            int r = (yy + ruv) >> 20, g = (yy + guv) >> 20, b = (yy + buv) >> 20;
            r = r < 0 ? 0 : (r > 255 ? 255 : r);
            g = g < 0 ? 0 : (g > 255 ? 255 : g);
            b = b < 0 ? 0 : (b > 255 ? 255 : b);
            uint8_t* o = dst + ((int64_t)y * w + x) * dcn;
            o[bidx] = (uint8_t)b;
            o[1] = (uint8_t)g;
            o[2 - bidx] = (uint8_t)r;
            if (dcn == 4) o[3] = 255;
        }
    }
}

/* cv::cvtColor COLOR_GRAY2BGR / GRAY2BGRA (OpenCV 2.4 Gray2RGB: the value
 * in every colour channel, alpha = the type's maximum) for u8 (esize 1) and
 * fp32 (esize 4, alpha 1.0). */
void oracle_gray_to_bgr(const void* src, void* dst, int64_t pixels, int dcn, int esize) {
    for (int64_t i = 0; i < pixels; ++i) {
        const uint8_t* s = (const uint8_t*)src + i * esize;
        uint8_t* d = (uint8_t*)dst + i * dcn * esize;
        for (int k = 0; k < 3; ++k) memcpy(d + k * esize, s, esize);
        if (dcn == 4) {
            if (esize == 1) {
                d[3] = 255;
            } else {
                const float one = 1.0f;
                memcpy(d + 3 * esize, &one, 4);
            }
        }
    }
}

/* BGR -> NV21 test-input generator, image_util.cpp:9-41 (14-bit fixed point,
 * unsigned wrap-around, VU order). */
void oracle_bgr2nv21(const uint8_t* bgr, uint8_t* dst, int w, int h) {
    uint8_t* yp = dst;
    uint8_t* vu = dst + (int64_t)w * h;
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            const uint8_t* p = bgr + ((int64_t)y * w + x) * 3;
            uint32_t Y = ((uint32_t)p[0] * 1868u + (uint32_t)p[1] * 9617u + (uint32_t)p[2] * 4899u) >> 14;
            yp[(int64_t)y * w + x] = (uint8_t)Y;
            if (((y | x) & 1) == 0) {
                uint32_t U = ((uint32_t)((int)p[0] - (int)Y) * 9241u + (128u << 14)) >> 14;
                uint32_t V = ((uint32_t)((int)p[2] - (int)Y) * 11682u + (128u << 14)) >> 14;
                uint8_t* o = vu + (int64_t)(y / 2) * w + x;
                o[0] = (uint8_t)V;
                o[1] = (uint8_t)U;
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* tensor.cpp:160-182 */
void oracle_hwc_to_chw(const void* src, void* dst, int w, int h, int c, int esize) {
    const int64_t hw = (int64_t)w * h;
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    for (int k = 0; k < c; ++k)
        for (int64_t i = 0; i < hw; ++i)
            memcpy(d + (k * hw + i) * esize, s + (i * c + k) * esize, esize);
}

void oracle_chw_to_hwc(const void* src, void* dst, int w, int h, int c, int esize) {
    const int64_t hw = (int64_t)w * h;
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    for (int64_t i = 0; i < hw; ++i)
        for (int k = 0; k < c; ++k)
            memcpy(d + (i * c + k) * esize, s + (k * hw + i) * esize, esize);
}

/* tensor.cpp:473-482 (exact) */
void oracle_u8_to_f32(const uint8_t* src, float* dst, int64_t count) {
    for (int64_t i = 0; i < count; ++i) dst[i] = (float)src[i];
}

/* fp32 -> u8 with the NEON semantics of f32_2_u8_neon, tensor.cpp:349-390:
 * vcvtq_u32_f32 (truncate, NaN and negatives -> 0, saturate at 2^32-1) then
 * two truncating narrows (keep the low 8 bits).  The naive x86 path
 * (tensor.cpp:488-492) agrees on [0,256) and is undefined elsewhere. */
void oracle_f32_to_u8(const float* src, uint8_t* dst, int64_t count) {
    for (int64_t i = 0; i < count; ++i) {
        float f = src[i];
        uint32_t u;
        if (!(f > 0.f)) u = 0;
        else if (f >= 4294967296.f) u = 0xFFFFFFFFu;
        else u = (uint32_t)f;
        dst[i] = (uint8_t)(u & 0xFFu);
    }
}

/* crop.cpp:44-125: rectangle copy, per plane, rows of cw*ppx elements. */
void oracle_crop(const void* src, int w, int h, int ppx, int planes, int esize,
                 void* dst, int left, int top, int cw, int chh) {
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    const int64_t srow = (int64_t)w * ppx * esize, drow = (int64_t)cw * ppx * esize;
    for (int p = 0; p < planes; ++p)
        for (int y = 0; y < chh; ++y)
            memcpy(d + ((int64_t)p * chh + y) * drow,
                   s + ((int64_t)p * h + top + y) * srow + (int64_t)left * ppx * esize, drow);
}

/* ------------------------------------------------------------------------ */
/* normalize_naive.cpp:74-90: (x - mean) in float, divided by the double
 * (stddev + 1e-6), rounded to float. */
void oracle_normalize_f32(const float* src, float* dst, int64_t pixels, int cc,
                          const float* mean, const float* stddev) {
    for (int64_t i = 0; i < pixels; ++i)
        for (int k = 0; k < cc; ++k) {
            float diff = src[i * cc + k] - mean[k];
            dst[i * cc + k] = (float)((double)diff / ((double)stddev[k] + 1e-6));
        }
}

/* normalize_naive.cpp:7-72: sequential fp32 sums, population variance
 * accumulated as sum((x-mean)^2 / N), std = sqrtf. */
void oracle_mean_stddev_ref_f32(const float* src, int64_t pixels, int cc, float* mean, float* stddev) {
    const int n = (int)pixels;
    for (int k = 0; k < cc; ++k) {
        float s = 0.f;
        for (int64_t i = 0; i < pixels; ++i) s += src[i * cc + k];
        mean[k] = s / (float)n;
    }
    for (int k = 0; k < cc; ++k) {
        float acc = 0.f;
        for (int64_t i = 0; i < pixels; ++i) {
            float d = src[i * cc + k] - mean[k];
            d = d * d;
            acc += d / (float)n;
        }
        stddev[k] = sqrtf(acc);
    }
}

/* exact/fp64 statistics used by the build (mean_stddev) */
void oracle_channel_sums_f64(const float* src, int64_t pixels, int cc, double* sums) {
    for (int k = 0; k < 2 * cc; ++k) sums[k] = 0.0;
    for (int64_t i = 0; i < pixels; ++i)
        for (int k = 0; k < cc; ++k) {
            double v = src[i * cc + k];
            sums[2 * k] += v;
            sums[2 * k + 1] += v * v;
        }
}

void oracle_channel_sums_u8(const uint8_t* src, int64_t pixels, int cc, double* sums) {
    for (int k = 0; k < cc; ++k) {
        int64_t s1 = 0, s2 = 0;
        for (int64_t i = 0; i < pixels; ++i) {
            int64_t v = src[i * cc + k];
            s1 += v;
            s2 += v * v;
        }
        sums[2 * k] = (double)s1;
        sums[2 * k + 1] = (double)s2;
    }
}

void oracle_stats_from_sums(const double* sums, double count, int cc, float* mean, float* stddev) {
    for (int k = 0; k < cc; ++k) {
        double m = sums[2 * k] / count;
        double var = sums[2 * k + 1] / count - m * m;
        if (var < 0) var = 0;
        mean[k] = (float)m;
        stddev[k] = (float)sqrt(var);
    }
}

/* ------------------------------------------------------------------------ */
/* ImageUtil::compare_image_data, image_util.h:16-32 (fp32 accumulation). */
float oracle_cosine_f32acc_u8(const uint8_t* a, const uint8_t* b, int64_t len) {
    float n1 = 0.000001f, n2 = 0.000001f, dot = 0.f;
    for (int64_t i = 0; i < len; ++i) {
        float x = (float)a[i], y = (float)b[i];
        dot += x * y;
        n1 += x * x;
        n2 += y * y;
    }
    return dot / sqrtf(n1 * n2);
}

double oracle_cosine_f64_f32(const float* a, const float* b, int64_t len) {
    double n1 = 1e-12, n2 = 1e-12, dot = 0.0;
    for (int64_t i = 0; i < len; ++i) {
        dot += (double)a[i] * b[i];
        n1 += (double)a[i] * a[i];
        n2 += (double)b[i] * b[i];
    }
    return dot / sqrt(n1 * n2);
}

/* ------------------------------------------------------------------------ */
/* match_template / minMaxIdx.  The reference's MatchTemplate::match_template
 * calls cv::matchTemplate (match_template.cpp:13-41; its naive/NEON bodies
 * are empty todo stubs, :48-61), so the semantics are OpenCV 2.4.13.4's
 * (templmatch.cpp, cv::matchTemplate), restated:
 *   R = crossCorr(img, templ) stored as float (here: the exact correlation
 *       -- integer for u8, double in row-major order for fp32 -- rounded to
 *       float; OpenCV's DFT path rounds differently: parity unpinned);
 *   then, in double, with the window sums S_c = sum of channel c over the
 *   window and Q = sum of squares over the window (all channels) -- taken as
 *   OpenCV takes them, 4-term differences of cv::integral's double sum /
 *   sqsum images built in its order (templmatch.cpp's p0 - p1 - p2 + p3) --
 *   invArea =
 *   1 / (w*h), the template's per-channel mean m_c and population stddev d_c:
 *     CCOEFF*:  num -= sum_c S_c * m_c;  wndMean2 = invArea * sum_c S_c^2
 *     SQDIFF*:  num = max(Q - 2*num + templSum2, 0), templSum2 = (sum d^2 + m^2) / invArea
 *     *_NORMED: t = sqrt(max(Q - wndMean2, 0)) * templNorm, templNorm =
 *               sqrt(sum d^2 (+ m^2 unless CCOEFF)) / sqrt(invArea);
 *               num = |num| < t ? num / t : |num| < 1.125 t ? sign(num) :
 *               (SQDIFF_NORMED ? 1 : 0)
 *     CCOEFF_NORMED with sum d^2 < DBL_EPSILON: every R = 1.
 * result: (W - w + 1) x (H - h + 1) fp32, one channel.  esize 1 (u8) or 4. */
void oracle_match_template(const void* img, int W, int H, const void* tpl, int w, int h, int cn, int esize,
                           int method, float* result) {
    const int RW = W - w + 1, RH = H - h + 1;
    const int n = w * h;
    double tm[4] = {0, 0, 0, 0}, td[4] = {0, 0, 0, 0};
#define PIX(p, i) (esize == 1 ? (double)((const uint8_t*)(p))[i] : (double)((const float*)(p))[i])
    for (int c = 0; c < cn; ++c) {
        double s = 0, q = 0;
        for (int i = 0; i < n; ++i) {
            const double v = PIX(tpl, (size_t)i * cn + c);
            s += v;
            q += v * v;
        }
        tm[c] = s / n;
        const double var = q / n - tm[c] * tm[c];
        td[c] = sqrt(var > 0 ? var : 0);
    }
    const double invArea = 1. / ((double)h * w);
    const int numType = (method == 2 || method == 3) ? 0 : (method == 4 || method == 5) ? 1 : 2;
    const int isNormed = method == 1 || method == 3 || method == 5;
    double templNorm = 0, templSum2 = 0;
    double tmean[4] = {tm[0], tm[1], tm[2], tm[3]};
    if (method != 4) {
        templNorm = td[0] * td[0] + td[1] * td[1] + td[2] * td[2] + td[3] * td[3];
        if (templNorm < DBL_EPSILON && method == 5) {
            for (int i = 0; i < RW * RH; ++i) result[i] = 1.f;
            return;
        }
        templSum2 = templNorm + tm[0] * tm[0] + tm[1] * tm[1] + tm[2] * tm[2] + tm[3] * tm[3];
        if (numType != 1) {
            tmean[0] = tmean[1] = tmean[2] = tmean[3] = 0;
            templNorm = templSum2;
        }
        templSum2 /= invArea;
        templNorm = sqrt(templNorm);
        templNorm /= sqrt(invArea);
    }
    /* cv::integral(img, sum, sqsum, CV_64F) in its order: a running row sum
     * per channel, added to the integral row above (imgproc/sumpixels.cpp) */
    const size_t step = (size_t)(W + 1) * cn;
    double* isum = (double*)calloc((size_t)(H + 1) * step, sizeof(double));
    double* isq = (double*)calloc((size_t)(H + 1) * step, sizeof(double));
    for (int y = 0; y < H; ++y)
        for (int c = 0; c < cn; ++c) {
            double s = 0, q = 0;
            for (int x = 0; x < W; ++x) {
                const double v = PIX(img, ((size_t)y * W + x) * cn + c);
                s += v;
                q += v * v;
                isum[(y + 1) * step + (x + 1) * cn + c] = isum[y * step + (x + 1) * cn + c] + s;
                isq[(y + 1) * step + (x + 1) * cn + c] = isq[y * step + (x + 1) * cn + c] + q;
            }
        }
    for (int y = 0; y < RH; ++y)
        for (int x = 0; x < RW; ++x) {
            double corr = 0, S[4] = {0, 0, 0, 0}, Q = 0;
            for (int yy = 0; yy < h; ++yy)
                for (int xx = 0; xx < w; ++xx)
                    for (int c = 0; c < cn; ++c) {
                        const double v = PIX(img, ((size_t)(y + yy) * W + x + xx) * cn + c);
                        corr += PIX(tpl, ((size_t)yy * w + xx) * cn + c) * v;
                    }
            /* the window sums as templmatch.cpp takes them: p0 - p1 - p2 + p3 */
            const size_t i0 = y * step + (size_t)x * cn, dw = (size_t)w * cn, dh = (size_t)h * step;
            for (int c = 0; c < cn; ++c) {
                S[c] = isum[i0 + c] - isum[i0 + dw + c] - isum[i0 + dh + c] + isum[i0 + dh + dw + c];
                Q += isq[i0 + c] - isq[i0 + dw + c] - isq[i0 + dh + c] + isq[i0 + dh + dw + c];
            }
            double num = (double)(float)corr, t;
            double wndMean2 = 0, wndSum2 = 0;
            if (method == 2) {
                result[(size_t)y * RW + x] = (float)num;
                continue;
            }
            if (numType == 1) {
                for (int c = 0; c < cn; ++c) {
                    t = S[c];
                    wndMean2 += t * t;
                    num -= t * tmean[c];
                }
                wndMean2 *= invArea;
            }
            if (isNormed || numType == 2) {
                wndSum2 = Q;
                if (numType == 2) {
                    num = wndSum2 - 2 * num + templSum2;
                    num = num > 0 ? num : 0;
                }
            }
            if (isNormed) {
                t = sqrt(wndSum2 - wndMean2 > 0 ? wndSum2 - wndMean2 : 0) * templNorm;
                if (fabs(num) < t) num /= t;
                else if (fabs(num) < t * 1.125) num = num > 0 ? 1 : -1;
                else num = method != 1 ? 0 : 1;
            }
            result[(size_t)y * RW + x] = (float)num;
        }
    free(isum);
    free(isq);
#undef PIX
}

/* cv::minMaxIdx of a single-channel array (core/stat.cpp): the first
 * (row-major) minimum and maximum among the elements whose mask byte is
 * non-zero (mask NULL: all); idx = (row, col).  No element: 0, 0 and -1s.
 * NaN elements are never selected (the comparisons are false for them). */
void oracle_min_max_idx(const void* src, int w, int h, int esize, const uint8_t* mask, double* mm, int* idx) {
    int have = 0;
    double mn = 0, mx = 0;
    long imn = -1, imx = -1;
    for (long i = 0; i < (long)w * h; ++i) {
        if (mask && !mask[i]) continue;
        const double v = esize == 1 ? (double)((const uint8_t*)src)[i] : (double)((const float*)src)[i];
        if (v != v) continue;
        if (!have) {
            mn = mx = v;
            imn = imx = i;
            have = 1;
            continue;
        }
        if (v < mn) { mn = v; imn = i; }
        if (v > mx) { mx = v; imx = i; }
    }
    mm[0] = mn;
    mm[1] = mx;
    idx[0] = imn < 0 ? -1 : (int)(imn / w);
    idx[1] = imn < 0 ? -1 : (int)(imn % w);
    idx[2] = imx < 0 ? -1 : (int)(imx / w);
    idx[3] = imx < 0 ? -1 : (int)(imx % w);
}


/* ---- INTER_LANCZOS4 (OpenCV 2.4.13 imgwarp.cpp restated; parity unpinned) ----
 * The reference hands the mode to cv::resize (resize.cpp:46-48).  resize():
 * per output column fx = (float)((dx + 0.5) * scale_x - 0.5), sx = cvFloor(fx),
 * fx -= sx, interpolateLanczos4(fx) -> 8 coefficients (u8: saturate_cast<short>
 * (c * INTER_RESIZE_COEF_SCALE)); rows the same.  resizeGeneric_: every source
 * row is resized horizontally into a WT buffer (HResizeLanczos4: taps sx - 3
 * .. sx + 4, an out-of-range tap walks by cn to the nearest pixel of its
 * channel; columns outside [xmin, xmax) sum from 0, the others unrolled),
 * then output row dy combines rows clip(sy - 3 + k, 0, h) (VResizeLanczos4; u8
 * in int, where the order is immaterial, rounded by FixedPtCast<int, uchar,
 * 22>; fp32: elements x < (dst.w * cn & ~3) in the 4-wide NEON loop of
 * VResizeLanczos4Vec_32f, (b0 r0 + .. + b3 r3) + (b4 r4 + .. + b7 r7), the
 * rest in the scalar tail's left-to-right b0 r0 + b1 r1 + .. + b7 r7). */
static void lz_coeffs(float x, float* coeffs) {
    static const double s45 = 0.70710678118654752440084436210485;
    static const double cs[8][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
    const double pi = 3.1415926535897932384626433832795;
    int i;
    float sum = 0.f;
    double y0, s0, c0;
    if (x < FLT_EPSILON) {
        for (i = 0; i < 8; i++) coeffs[i] = 0.f;
        coeffs[3] = 1.f;
        return;
    }
    y0 = -(x + 3) * pi * 0.25;
    s0 = sin(y0);
    c0 = cos(y0);
    for (i = 0; i < 8; i++) {
        double y = -(x + 3 - i) * pi * 0.25;
        coeffs[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
        sum += coeffs[i];
    }
    sum = 1.f / sum;
    for (i = 0; i < 8; i++) coeffs[i] *= sum;
}

static short lz_sat_short(float v) {
    long r = lrintf(v);
    return (short)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
}

void oracle_resize_lanczos4(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out, int h_out,
                            double inv_x, double inv_y) {
    const double scale_x = 1. / (inv_x > 0 ? inv_x : (double)w_out / w_in);
    const double scale_y = 1. / (inv_y > 0 ? inv_y : (double)h_out / h_in);
    const int sw = w_in * cc, dw = w_out * cc;
    int* xofs = (int*)malloc(sizeof(int) * dw);
    float* xa = (float*)malloc(sizeof(float) * 8 * w_out);
    short* xai = (short*)malloc(sizeof(short) * 8 * w_out);
    int* yofs = (int*)malloc(sizeof(int) * h_out);
    float* ya = (float*)malloc(sizeof(float) * 8 * h_out);
    short* yai = (short*)malloc(sizeof(short) * 8 * h_out);
    /* the horizontal pass of every source row: int (u8) or float (fp32) */
    int* bi = esize == 1 ? (int*)malloc(sizeof(int) * (size_t)dw * h_in) : NULL;
    float* bf = esize == 1 ? NULL : (float*)malloc(sizeof(float) * (size_t)dw * h_in);
    int xmin = 0, xmax = w_out, dx, dy, k, r, j;
    for (dx = 0; dx < w_out; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 3) xmin = dx + 1;
        if (sx + 4 >= w_in && dx < xmax) xmax = dx;
        for (k = 0; k < cc; k++) xofs[dx * cc + k] = sx * cc + k;
        lz_coeffs(fx, xa + 8 * dx);
        for (k = 0; k < 8; k++) xai[8 * dx + k] = lz_sat_short(xa[8 * dx + k] * 2048.f);
    }
    for (dy = 0; dy < h_out; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        yofs[dy] = sy;
        lz_coeffs(fy, ya + 8 * dy);
        for (k = 0; k < 8; k++) yai[8 * dy + k] = lz_sat_short(ya[8 * dy + k] * 2048.f);
    }
    for (r = 0; r < h_in; r++) {
        for (dx = 0; dx < dw; dx++) {
            const int px = dx / cc, fast = px >= xmin && px < xmax;
            const int sx = xofs[dx] - cc * 3;
            if (esize == 1) {
                const uint8_t* S = (const uint8_t*)src + (size_t)r * sw;
                int v = 0;
                for (j = 0; j < 8; j++) {
                    int sxj = sx + j * cc;
                    while (sxj < 0) sxj += cc;
                    while (sxj >= sw) sxj -= cc;
                    v += S[sxj] * xai[8 * px + j];
                }
                bi[(size_t)r * dw + dx] = v;
            } else {
                const float* S = (const float*)src + (size_t)r * sw;
                float v = 0.f, t[8];
                for (j = 0; j < 8; j++) {
                    int sxj = sx + j * cc;
                    while (sxj < 0) sxj += cc;
                    while (sxj >= sw) sxj -= cc;
                    t[j] = S[sxj] * xa[8 * px + j];
                }
                if (fast) {
                    v = t[0];
                    for (j = 1; j < 8; j++) v = v + t[j];
                } else {
                    for (j = 0; j < 8; j++) v += t[j];
                }
                bf[(size_t)r * dw + dx] = v;
            }
        }
    }
    for (dy = 0; dy < h_out; dy++) {
        int rows[8];
        for (k = 0; k < 8; k++) {
            int sy = yofs[dy] - 3 + k;
            rows[k] = sy < 0 ? 0 : sy >= h_in ? h_in - 1 : sy;
        }
        for (dx = 0; dx < dw; dx++) {
            if (esize == 1) {
                const short* b = yai + 8 * dy;
                int s0 = bi[(size_t)rows[0] * dw + dx] * b[0] + bi[(size_t)rows[1] * dw + dx] * b[1] +
                         bi[(size_t)rows[2] * dw + dx] * b[2] + bi[(size_t)rows[3] * dw + dx] * b[3];
                int s1 = bi[(size_t)rows[4] * dw + dx] * b[4] + bi[(size_t)rows[5] * dw + dx] * b[5] +
                         bi[(size_t)rows[6] * dw + dx] * b[6] + bi[(size_t)rows[7] * dw + dx] * b[7];
                int v = (s0 + s1 + (1 << 21)) >> 22;
                ((uint8_t*)dst)[(size_t)dy * dw + dx] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            } else {
                const float* b = ya + 8 * dy;
                float v;
                if (dx < (dw & ~3)) {
                    float s0 = bf[(size_t)rows[0] * dw + dx] * b[0] + bf[(size_t)rows[1] * dw + dx] * b[1] +
                               bf[(size_t)rows[2] * dw + dx] * b[2] + bf[(size_t)rows[3] * dw + dx] * b[3];
                    float s1 = bf[(size_t)rows[4] * dw + dx] * b[4] + bf[(size_t)rows[5] * dw + dx] * b[5] +
                               bf[(size_t)rows[6] * dw + dx] * b[6] + bf[(size_t)rows[7] * dw + dx] * b[7];
                    v = s0 + s1;
                } else {
                    v = bf[(size_t)rows[0] * dw + dx] * b[0];
                    for (k = 1; k < 8; k++) v = v + bf[(size_t)rows[k] * dw + dx] * b[k];
                }
                ((float*)dst)[(size_t)dy * dw + dx] = v;
            }
        }
    }
    free(xofs); free(xa); free(xai); free(yofs); free(ya); free(yai); free(bi); free(bf);
}
