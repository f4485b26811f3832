/*
 * vacv_oracle.h -- CPU restatement of the vacv (b1xian/arm-neon-opencv) pixel
 * operators.  TEST INFRASTRUCTURE ONLY: nothing in the product path may link,
 * load or call this.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Every function restates one reference routine (file:line under
 * /root/reference/src) and is pinned against golden vectors produced by the
 * reference's own sources (oracle/_ref, built by oracle/Makefile) -- see
 * tests/golden/make_golden.py and tests/test_oracle.py.
 *
 * Conventions: single image, host memory, dense rows.  "cc" = channels that
 * are interleaved in one row (HWC: c; a CHW plane: 1).  u8 pixels are
 * unsigned (ARM `char` semantics; the reference's x86 build is the odd one).
 */
#ifndef VACV_ORACLE_H
#define VACV_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* resize mode for u8 bilinear */
enum { ORACLE_LINEAR_NAIVE = 0, ORACLE_LINEAR_NEON = 1, ORACLE_LINEAR_OPENCV = 2 };

/* --- geometry / tables ------------------------------------------------- */
int  oracle_sat_short(float x);
void oracle_linear_table(int n_in, int n_out, int mode, int32_t* ofs, int16_t* w0, int16_t* w1);
void oracle_linear_table_f32(int n_in, int n_out, int32_t* ofs, float* w0, float* w1);
void oracle_cubic_table(int n_in, int n_out, int32_t* ofs, float* coef /* 4*n_out */);
void oracle_invert_affine(const float m[6], float inv[6]);
void oracle_rotation_matrix(float scale, float rot_deg, const double aux[4], float m[6]);

/* --- samplers ---------------------------------------------------------- */
void oracle_resize_linear_u8(const uint8_t* src, int w_in, int h_in, int cc,
                             uint8_t* dst, int w_out, int h_out, int mode);
void oracle_resize_linear_f32(const float* src, int w_in, int h_in, int cc,
                              float* dst, int w_out, int h_out);
void oracle_resize_nearest(const void* src, int w_in, int h_in, int cc, int esize,
                           void* dst, int w_out, int h_out);
void oracle_resize_area(const void* src, int w_in, int h_in, int cc, int esize,
                        void* dst, int w_out, int h_out);
/* INTER_AREA at any scale (cv::resize of OpenCV 2.4.13.4: resizeAreaFast_,
 * resizeArea_ or the area-mode bilinear); inv_x/inv_y <= 0: dsize / ssize */
void oracle_resize_area_any(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out,
                            int h_out, double inv_x, double inv_y);
int oracle_area_table(int ssize, int dsize, int cn, double scale, int* di, int* si, float* alpha);
void oracle_area_linear_tap(int d, int n_in, double scale, double inv_scale, int* i, float* f);
/* INTER_LANCZOS4 (OpenCV 2.4 cv::resize, 8x8 taps, replicate borders);
 * esize 1 (fixed point) or 4; inv_x / inv_y <= 0: dsize / ssize */
void oracle_resize_lanczos4(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out, int h_out,
                            double inv_x, double inv_y);
void oracle_resize_cubic_f32(const float* src, int w_in, int h_in, int cc,
                             float* dst, int w_out, int h_out);
void oracle_warp_affine_u8(const uint8_t* src, int w_in, int h_in, int cc,
                           uint8_t* dst, int w_out, int h_out, const float inv[6]);
void oracle_warp_affine_f32(const float* src, int w_in, int h_in, int cc,
                            float* dst, int w_out, int h_out, const float inv[6]);
/* non-CONSTANT border modes (1 REPLICATE, 2 REFLECT, 3 WRAP, 4 REFLECT_101) for
 * the pixels the naive sampler skips; esize 1 (u8) or 4 (fp32) */
void oracle_warp_affine_border(const void* src, int w_in, int h_in, int cc, int esize,
                               void* dst, int w_out, int h_out, const float m[6], int mode);

/* cv::warpAffine INTER_NEAREST (OpenCV 2.4 fixed point + remap nearest);
 * inverse_map: m is the dst -> src map; modes 0-5; esize 1 or 4 */
void oracle_warp_affine_nn(const void* src, int w_in, int h_in, int cc, int esize, void* dst, int w_out, int h_out,
                           const float m[6], int inverse_map, int mode, const double border[4]);

/* --- colour ------------------------------------------------------------ */
void oracle_yuv420sp_to_bgr(const uint8_t* src, uint8_t* dst, int w, int h, int v_first, int rgb_out);
void oracle_bgr2nv21(const uint8_t* bgr, uint8_t* dst, int w, int h);
/* cv::cvtColor's YUV420 (OpenCV 2.4 BT.601 fixed point): layout 0 NV12,
 * 1 NV21, 2 YV12, 3 IYUV; dcn 3/4; bidx 0 BGR(A), 2 RGB(A) */
void oracle_yuv420_cv(const uint8_t* src, uint8_t* dst, int w, int h, int layout, int dcn, int bidx);
/* cv::cvtColor GRAY2BGR(A): esize 1 (u8) or 4 (fp32) */
void oracle_gray_to_bgr(const void* src, void* dst, int64_t pixels, int dcn, int esize);

/* --- layout / dtype / crop -------------------------------------------- */
void oracle_hwc_to_chw(const void* src, void* dst, int w, int h, int c, int esize);
void oracle_chw_to_hwc(const void* src, void* dst, int w, int h, int c, int esize);
void oracle_u8_to_f32(const uint8_t* src, float* dst, int64_t count);
void oracle_f32_to_u8(const float* src, uint8_t* dst, int64_t count);
void oracle_crop(const void* src, int w, int h, int row_elems_per_px, int planes, int esize,
                 void* dst, int left, int top, int cw, int chh);

/* --- normalize / statistics ------------------------------------------- */
void oracle_normalize_f32(const float* src, float* dst, int64_t pixels, int cc,
                          const float* mean, const float* stddev);
void oracle_mean_stddev_ref_f32(const float* src, int64_t pixels, int cc, float* mean, float* stddev);
void oracle_channel_sums_f64(const float* src, int64_t pixels, int cc, double* sums /* 2*cc */);
void oracle_channel_sums_u8(const uint8_t* src, int64_t pixels, int cc, double* sums /* 2*cc */);
void oracle_stats_from_sums(const double* sums, double count, int cc, float* mean, float* stddev);

/* --- harness helper (image_util.h:16-32) ------------------------------ */
float  oracle_cosine_f32acc_u8(const uint8_t* a, const uint8_t* b, int64_t len);
double oracle_cosine_f64_f32(const float* a, const float* b, int64_t len);

/* cv::matchTemplate (OpenCV 2.4 templmatch.cpp) restated; method = TM_* */
void oracle_match_template(const void* img, int W, int H, const void* tpl, int w, int h, int cn, int esize,
                           int method, float* result);
/* cv::minMaxIdx of a single-channel array: mm = {min, max}, idx = {min row,
 * min col, max row, max col} */
void oracle_min_max_idx(const void* src, int w, int h, int esize, const uint8_t* mask, double* mm, int* idx);

#ifdef __cplusplus
}
#endif
#endif
