/*
 * vacv_hip.h -- C ABI of the MI355X-native vacv pixel operators.
 *
 * This is the drop-in boundary for the reference's operator API
 * (/root/reference/src/cv/cv.h:85-209, vision::Tensor in
 * src/common/tensor.h:27-84).  The C++ surface in
 * arm-neon-opencv_amd/src/{common,cv,util} keeps the reference's names and
 * signatures and is a thin wrapper over these entry points; any FFI
 * (ctypes, cgo, JNI, N-API) binds this header directly.
 *
 * Conventions
 *  - Every image pointer is DEVICE-accessible memory (hipMalloc, or mapped
 *    hipHostMalloc).  Nothing here copies host<->device; the C++ wrapper
 *    stages host tensors.
 *  - Batched: an image descriptor covers `n` images, `batch_pitch` bytes
 *    apart.  One call = one launch sequence on `stream` (a hipStream_t, or
 *    NULL for the default stream).  Calls are asynchronous and never
 *    synchronise the device; host-side arrays passed in (mean, stddev, M,
 *    border values) are consumed before the call returns.
 *  - Return value: VACV_OK (0) or a negative vacv_status.  No C++ exception
 *    crosses this boundary.
 *  - dtype / layout codes are the reference's vision::DType / DLayout values
 *    (tensor.h:12-24); interpolation, border and colour codes are the
 *    reference's va_cv enums (cv.h:27-74).
 */
#ifndef VACV_HIP_H
#define VACV_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VACV_ABI_VERSION 3
#define VACV_MAX_CHANNELS 16

typedef enum vacv_status {
    VACV_OK = 0,
    VACV_ERR_INVALID_ARG = -1,  /* bad pointer / size / pitch / rect */
    VACV_ERR_UNSUPPORTED = -2,  /* dtype, layout, mode or code not implemented */
    VACV_ERR_HIP = -3,          /* a HIP runtime call failed */
    VACV_ERR_NO_MEMORY = -4     /* device workspace allocation failed */
} vacv_status;

/* vision::DType (tensor.h:12-18) */
enum { VACV_FP32 = 0, VACV_FP16 = 1, VACV_INT8 = 2 /* unsigned bytes */, VACV_FP64 = 3 };
/* vision::DLayout (tensor.h:21-24) */
enum { VACV_NCHW = 0, VACV_NHWC = 1 };
/* va_cv::VInterMode (cv.h:27-35) */
enum { VACV_INTER_NEAREST = 0, VACV_INTER_LINEAR = 1, VACV_INTER_CUBIC = 2, VACV_INTER_AREA = 3, VACV_INTER_LANCZOS4 = 4 };
/* warp flag (cv.h:35): m is already the inverse (dst -> src) map */
enum { VACV_WARP_INVERSE_MAP = 16 };
/* va_cv::VBorderMode (cv.h:38-48) */
enum {
    VACV_BORDER_CONSTANT = 0, VACV_BORDER_REPLICATE = 1, VACV_BORDER_REFLECT = 2, VACV_BORDER_WRAP = 3,
    VACV_BORDER_REFLECT_101 = 4, VACV_BORDER_TRANSPARENT = 5
};
/* va_cv::InputImageFormat (cv.h:62-74) */
enum {
    VACV_COLOR_YUV2RGB_NV12 = 90, VACV_COLOR_YUV2BGR_NV12 = 91,
    VACV_COLOR_YUV2RGB_NV21 = 92, VACV_COLOR_YUV2BGR_NV21 = 93,
    /* the codes the reference hands to cv::cvtColor (cvt_color.cpp:139-141) */
    VACV_COLOR_GRAY2BGR = 8,
    VACV_COLOR_YUV2RGBA_NV12 = 94, VACV_COLOR_YUV2BGRA_NV12 = 95,
    VACV_COLOR_YUV2RGBA_NV21 = 96, VACV_COLOR_YUV2BGRA_NV21 = 97,
    VACV_COLOR_YUV2BGR_YV12 = 99
};
/* Arithmetic of the u8 bilinear sampler.
 *  REFERENCE: the path the reference's public API actually dispatches to,
 *             ResizeNaive::resize_naive_inter_linear_u8 (resize_naive.cpp:10-68).
 *  NEON:      ResizeNeon (resize_neon.cpp:12-188), two-pass fixed point.
 *  OPENCV:    NEON arithmetic with round-half-even coefficients (OpenCV 2.4's
 *             saturate_cast<short>); SURVEY.md App. B. */
enum { VACV_LINEAR_REFERENCE = 0, VACV_LINEAR_NEON = 1, VACV_LINEAR_OPENCV = 2 };

/* A batch of images.  Pitches are in BYTES; 0 selects the dense value.
 *   NHWC: pixel (x,y) channel k of image i at
 *         data + i*batch_pitch + y*row_pitch + (x*c + k)*esize
 *   NCHW: data + i*batch_pitch + k*plane_pitch + y*row_pitch + x*esize
 * For the NV21/NV12 input of vacv_cvt_color the descriptor is the
 * reference's (w, h*3/2, c=1) single-plane tensor (cvt_color.cpp:151-152). */
typedef struct vacv_image {
    void* data;
    int32_t n;
    int32_t w;
    int32_t h;
    int32_t c;
    int32_t dtype;
    int32_t layout;
    int64_t row_pitch;
    int64_t plane_pitch;
    int64_t batch_pitch;
} vacv_image;

int vacv_abi_version(void);
const char* vacv_status_string(int status);
/* bytes of one image's valid data under the dense-pitch rules above */
int64_t vacv_image_bytes(const vacv_image* img);

/* ---- geometry / dtype ------------------------------------------------- */

/* Crop::crop (crop.cpp:22-142, cv.h:209).  The rect is already truncated to
 * int as crop_naive does (crop.cpp:128-131); dst->w/h are the crop size and
 * dst->layout/dtype must equal src's.  Rect must lie inside src. */
int vacv_crop(const vacv_image* src, const vacv_image* dst, int left, int top, void* stream);

/* Tensor::change_layout (tensor.cpp:393-457): NHWC <-> NCHW of 1,2,4 or 8
 * byte elements.  Same layout or c == 1 is a plain copy (clone()). */
int vacv_change_layout(const vacv_image* src, const vacv_image* dst, void* stream);

/* Tensor::change_dtype (tensor.cpp:459-502): INT8 -> FP32 exact; FP32 ->
 * INT8 with the NEON f32_2_u8_neon semantics (truncate; NaN/negative -> 0;
 * low 8 bits kept).  Same dtype is a copy; other pairs VACV_ERR_UNSUPPORTED
 * (the reference silently returns an uninitialised tensor). */
int vacv_change_dtype(const vacv_image* src, const vacv_image* dst, void* stream);

/* Resize::resize (resize.cpp:19-100, cv.h:85-87).  Only dst->w/h select the
 * output size (fx/fy are ignored, as in the reference).
 *  INTER_LINEAR: INT8->INT8 (mode = VACV_LINEAR_*), FP32->FP32.
 *  INTER_CUBIC:  FP32->FP32 and INT8->FP32 (the u8->fp32 conversion the
 *                reference requires before cubic, fused).
 *  INTER_NEAREST: INT8->INT8, FP32->FP32 with OpenCV 2.4's resizeNN
 *                semantics, which the reference delegates to cv::resize
 *                (resize.cpp:44-49): sx = min(floor(x / (w_out / w_in)), w_in - 1).
 *  INTER_AREA:   INT8->INT8, FP32->FP32 (OpenCV 2.4's cv::resize, also
 *                behind resize.cpp:44-49): integer down-scales = the mean of
 *                each block (resizeAreaFast_; u8 rounded half to even, 2x2
 *                blocks of 1/3/4 channels half up), other down-scales =
 *                resizeArea_'s weight tables, up-scales = its bilinear with
 *                area-mode taps (parity unpinned).
 * NHWC channels 1..4; NCHW any c (per plane, as resize.cpp:72-88). */
int vacv_resize(const vacv_image* src, const vacv_image* dst, int interpolation, int mode, void* stream);

/* vacv_resize with cv::resize's explicit scale factors (the reference passes
 * fx / fy through to OpenCV, resize.cpp:35, :47): INTER_NEAREST and
 * INTER_AREA only; dst->w/h must be the size cv::resize derives,
 * saturate_cast<int>(w * fx) (round half to even), and the sampling uses
 * inv_scale = fx, fy instead of dst/src. */
int vacv_resize_scaled(const vacv_image* src, const vacv_image* dst, int interpolation, int mode, double fx,
                       double fy, void* stream);

/* WarpAffine::warp_affine (warp_affine.cpp:16-36, :111-169, cv.h:118-122).
 * m = the FORWARD 2x3 map, row-major; it is inverted on the host with the
 * reference's arithmetic and is NOT modified (the reference inverts the
 * caller's M in place).  flags = INTER_LINEAR or INTER_NEAREST, optionally
 * | VACV_WARP_INVERSE_MAP (m is then the dst -> src map, used as is); the
 * reference hands every flag but INTER_LINEAR to cv::warpAffine
 * (warp_affine.cpp:114-118), so those are restated from OpenCV 2.4 (parity
 * unpinned):
 *   INTER_NEAREST  cv::warpAffine's fp64 fixed point (AB_BITS = 10, round
 *                  half to even), remap's nearest sampler; the border modes
 *                  below on the mapped pixel
 * INTER_LINEAR: a pixel whose top-left tap is
 * inside [0,w-2]x[0,h-2] is the reference's naive sampler bit for bit (with
 * VACV_WARP_INVERSE_MAP too: the reference would hand that flag to
 * cv::warpAffine, whose INTER_BITS = 5 remap tables round differently, so
 * LINEAR | WARP_INVERSE_MAP keeps the naive arithmetic and does NOT
 * reproduce OpenCV's); the others depend on border_mode:
 *   BORDER_CONSTANT     border_value (the reference leaves them untouched);
 *                       border_value may be NULL (zeros)
 *   BORDER_TRANSPARENT  left untouched (the reference's own behaviour); dst
 *                       must not alias src
 *   BORDER_REPLICATE, _REFLECT, _WRAP, _REFLECT_101
 *                       the four taps at floor(f), floor(f)+1 mapped through
 *                       OpenCV 2.4's borderInterpolate, the naive sampler's
 *                       weights (the reference hands these modes to OpenCV,
 *                       warp_affine.cpp:114-118; parity unpinned) */
int vacv_warp_affine(const vacv_image* src, const vacv_image* dst, const float m[6],
                     int flags, int border_mode, const double border_value[4], void* stream);

/* get_rotation_matrix_2D(VPoint(0,0), rot, scale) + the aux translation fix
 * of the (scale, rot) overload (warp_affine.cpp:76-109).  Host only. */
int vacv_rotation_matrix(float scale, float rot_deg, const double aux[4], float m_out[6]);
/* The in-place inverse of warp_affine.cpp:121-133, out of place.  Host only. */
int vacv_invert_affine(const float m[6], float inv_out[6]);

/* ---- colour ----------------------------------------------------------- */

/* CvtColor::cvt_color (cvt_color.cpp:20-157, cv.h:95): YUV420sp -> 3ch u8
 * NHWC.  src = (w, h*3/2, 1) INT8; dst = (w, h, 3) INT8 NHWC.  Codes:
 * COLOR_YUV2BGR_NV21 (bit-exact with nv_to_bgr_naive), COLOR_YUV2BGR_NV12
 * (correct UV order; the reference decodes it as NV21), and the two RGB
 * variants.  w and h must be even.
 * The codes the reference hands to cv::cvtColor (cvt_color.cpp:139-141),
 * with OpenCV 2.4's arithmetic (BT.601, 20-bit fixed point; parity
 * unpinned):
 *   COLOR_YUV2RGBA/BGRA_NV12/NV21  src as above, dst (w, h, 4) INT8 NHWC, alpha 255
 *   COLOR_YUV2BGR_YV12             src = (w, h*3/2, 1) INT8 with dense rows:
 *                                  Y, then the (w/2)x(h/2) V and U planes;
 *                                  dst (w, h, 3) INT8 NHWC
 *   COLOR_GRAY2BGR                 src (w, h, 1) INT8 or FP32, dst (w, h, 3) same dtype */
int vacv_cvt_color(const vacv_image* src, const vacv_image* dst, int code, void* stream);

/* ---- normalize / statistics ------------------------------------------- */

/* Normalize::normalize (normalize.cpp:84-121, cv.h:104-106):
 *   dst = (float)(((float)x - mean[k]) / ((double)stddev[k] + 1e-6))
 * src INT8 or FP32, dst FP32, same layout.  mean/stddev are HOST arrays of
 * c floats; both NULL = per-image statistics first (exact, see
 * vacv_mean_stddev).  Exactly one NULL is VACV_ERR_INVALID_ARG. */
int vacv_normalize(const vacv_image* src, const vacv_image* dst,
                   const float* mean, const float* stddev, void* stream);

/* Per-channel sums for mean_stddev: sums[g*2c + 2k] = Sum x,
 * sums[g*2c + 2k + 1] = Sum x^2 over channel k, g = image (per_image=1) or
 * the whole batch (per_image=0, one group).  DEVICE output, fp64; exact for
 * INT8 input (integer sums), deterministic order for FP32.  These are the
 * partials the multi-GPU path all-reduces over RCCL. */
int vacv_channel_sums(const vacv_image* src, double* sums, int per_image, void* stream);

/* vacv_resize followed by vacv_channel_sums of its output: the statistics
 * half of BASELINE cfg5 (resize + mean_stddev, normalize_naive.cpp:7-72 on
 * the resized image); on several GPUs the sums are what one all-reduce
 * merges.  dst must be dense. */
int vacv_resize_channel_sums(const vacv_image* src, const vacv_image* dst, int interpolation, int mode,
                             double* sums, int per_image, void* stream);

/* vacv_resize_channel_sums followed by vacv_stats_from_sums, for one GPU:
 * the resize (cfg5: u8 -> fp32 INTER_CUBIC), the sums[groups][c][2] of its
 * output and the population mean / stddev [groups][c] (groups = n per
 * image, else 1) -- resize_naive.cpp:130-569, then NormalizeNaive::
 * mean_stddev_naive_* (normalize_naive.cpp:7-48) over the image or the whole
 * batch.  On several GPUs use vacv_resize_channel_sums, all-reduce the sums,
 * then vacv_stats_from_sums.  dst must be dense. */
int vacv_resize_mean_stddev(const vacv_image* src, const vacv_image* dst, int interpolation, int mode,
                            double* sums, float* mean, float* stddev, int per_image, void* stream);

/* mean = S1/count, stddev = sqrt(max(S2/count - mean^2, 0)) per group and
 * channel, on the device: sums[groups][c][2] -> mean/stddev[groups][c]. */
int vacv_stats_from_sums(const double* sums, int groups, int c, double count,
                         float* mean, float* stddev, void* stream);

/* NormalizeNaive::mean_stddev_naive_* (normalize_naive.cpp:7-72): per-image
 * population mean/stddev, DEVICE outputs [n][c].  Computed exactly (the
 * reference accumulates sequentially in fp32; DESIGN.md quantifies it). */
int vacv_mean_stddev(const vacv_image* src, float* mean, float* stddev, void* stream);

/* ---- fused pipelines -------------------------------------------------- */

/* ResizeNormalize::resize_normalize (resize_normalize.cpp:15-107, cv.h:154):
 * resize, convert to fp32, normalize -- one pass, dst FP32.  Identical to
 * vacv_resize followed by vacv_normalize (u8 resize results are normalized
 * exactly as the reference normalizes a converted u8 tensor).  NULL mean and
 * stddev: per-image statistics of the resized image. */
int vacv_resize_normalize(const vacv_image* src, const vacv_image* dst, int interpolation, int mode,
                          const float* mean, const float* stddev, void* stream);

/* WarpAffineNormalize::warp_affine_normalize (warp_affine_normalize.cpp,
 * cv.h:172-201): warp then normalize, dst FP32. */
int vacv_warp_affine_normalize(const vacv_image* src, const vacv_image* dst, const float m[6],
                               int flags, int border_mode, const double border_value[4],
                               const float* mean, const float* stddev, void* stream);

/* cvt_color then normalize (the cfg3 pipeline), dst (w,h,3) FP32 NHWC. */
int vacv_cvt_color_normalize(const vacv_image* src, const vacv_image* dst, int code,
                             const float* mean, const float* stddev, void* stream);

/* Camera frame -> model input in ONE pass: YUV420sp
 * decode, u8 bilinear resize, and optionally convert + normalize, with NHWC
 * or NCHW (planar, the model-input layout) output.  Bit-identical to the
 * reference's chain
 *   CvtColor::cvt_color (cvt_color.cpp:39-157)
 *   -> Resize::resize INTER_LINEAR u8 (resize_naive.cpp:10-68; `mode` as in
 *      vacv_resize)
 *   -> Tensor::change_dtype FP32 + Normalize::normalize
 *      (tensor.cpp:459-502, normalize_naive.cpp:74-90)
 *   -> Tensor::change_layout(NCHW) (tensor.cpp:393-457)
 * without materialising the decoded frame.  src = (w, h*3/2, 1) INT8, w and
 * h even, w >= 4; dst = (wo, ho, 3), any wo/ho >= 1, NHWC or NCHW.
 * interpolation must be INTER_LINEAR.
 *  vacv_cvt_color_resize:           dst INT8 (u8 BGR/RGB) or FP32 (widened)
 *  vacv_cvt_color_resize_normalize: dst FP32; NULL mean and stddev = per-image
 *                                   statistics of the resized image. */
int vacv_cvt_color_resize(const vacv_image* src, const vacv_image* dst, int code, int interpolation,
                          int mode, void* stream);
int vacv_cvt_color_resize_normalize(const vacv_image* src, const vacv_image* dst, int code, int interpolation,
                                    int mode, const float* mean, const float* stddev, void* stream);

/* ---- template matching ------------------------------------------------ */

/* va_cv::VMatchMode (cv.h:52-59) */
enum {
    VACV_TM_SQDIFF = 0, VACV_TM_SQDIFF_NORMED = 1, VACV_TM_CCORR = 2, VACV_TM_CCORR_NORMED = 3,
    VACV_TM_CCOEFF = 4, VACV_TM_CCOEFF_NORMED = 5
};

/* MatchTemplate::match_template (match_template.cpp:13-41, cv.h:211-219),
 * which the reference hands to cv::matchTemplate: OpenCV 2.4's algorithm
 * with the correlation computed exactly (parity unpinned).
 * img: n images (W, H, c) NHWC INT8 or FP32, c <= 4; templ: (w, h, c), same
 * dtype, n = 1, shared by every image; result: n x (W-w+1, H-h+1, 1) FP32.
 * A template larger than the image in both dimensions swaps the two, as
 * cv::matchTemplate does.  VACV_ERR_UNSUPPORTED when the template does not
 * fit the kernel's LDS budget (about 64 KiB of template bytes). */
int vacv_match_template(const vacv_image* img, const vacv_image* templ, const vacv_image* result, int method,
                        void* stream);

/* MatchTemplate::minMaxIdx (match_template.cpp:43-46) = cv::minMaxIdx of a
 * single-channel 2-D array (n = 1, c = 1, INT8 or FP32): the first
 * (row-major) minimum and maximum among the elements whose mask byte is
 * non-zero (mask: NULL, or (w, h, 1) INT8).  DEVICE outputs: vals[2] = {min,
 * max}, idx[4] = {min row, min col, max row, max col}; with no element 0, 0
 * and -1s.  NaNs are never selected. */
int vacv_min_max_idx(const vacv_image* src, const vacv_image* mask, double* vals, int* idx, void* stream);

/* ---- runtime ---------------------------------------------------------- */

/* Kernel-variant knobs, for A/B measurement and the parity tests that check
 * every variant against the same oracle; normal callers never need them.
 * Each starts from the environment variable of the same name (read once,
 * when the library loads), else -1 = the built-in choice. */
enum {
    VACV_TUNE_RESIZE_DIRECT = 0,     /* u8 bilinear: 0 staged, 1 gather kernel for one-tap rows, 2 gather always, 3 as 1 without the NV21 resize's point-sampling instance (A/B) */
    VACV_TUNE_CUBIC_DIRECT = 1,      /* u8 cubic: 0 staged kernel, else the gather kernel */
    VACV_TUNE_RESIZE_INTERLEAVE = 2, /* staged kernel: 0 strip order, else address-ordered tasks */
    VACV_TUNE_DIRECT_XCD = 3,        /* gather kernel block order: 0 plain, 1 XCD-contiguous */
    VACV_TUNE_WARP_PX = 4,           /* warp gather kernel: lane blocks per wave (4, 5, 8, 10) */
    VACV_TUNE_NEAREST_KERNEL = 5,    /* INTER_NEAREST: 0 per-pixel kernel, 1 row per workgroup, else row per wave (when they apply) */
    VACV_TUNE_AREA_KERNEL = 6,       /* u8 INTER_AREA: 1 per-pixel kernel, 2 dword column sums */
    VACV_TUNE_AREA_ROWS = 7,         /* u8 INTER_AREA column sums: output rows per workgroup */
    VACV_TUNE_RESIZE_WGS = 8,        /* staged kernel: workgroups launched */
    VACV_TUNE_RESIZE_TILE_H = 9,     /* staged kernel planner: tile height */
    VACV_TUNE_RESIZE_TILE_W = 10,    /* staged kernel planner: tile width; column kernel (resize_cols_kernel): 64 / 128 output columns per wave */
    VACV_TUNE_RESIZE_WORK = 11,      /* staged kernel planner: work per thread */
    VACV_TUNE_WARP_KERNEL = 12,      /* u8 CONSTANT warp: 0 per-pixel gathers, 2 batched gathers, 4 LDS-staged frames: an LDS-DMA ring of source boxes (k_warp_frames.hip; 3 channels re-laid as 4-byte pixels, warp_exp_kernel), 6 the same without the re-lay (warp_ring_kernel, A/B); 5: INTER_NEAREST u8 on the per-pixel kernel (A/B) */
    VACV_TUNE_RESIZE_STRIP = 13,     /* two-tap u8 bilinear: column strips with an LDS row ring, 1: 64 columns x 16-row batches, 2 (default): 128 x 8; 0 staged kernel */
    VACV_TUNE_MATCH_KERNEL = 14,     /* u8 match_template correlation: 0 v_dot4 kernel, else i8 MFMA where it fits */
    VACV_TUNE_WARP_FRAMES = 15,      /* u8 CONSTANT warp, LDS-staged kernel: frames per workgroup */
    VACV_TUNE_WARP_TILE_H = 16,      /* u8 CONSTANT warp, LDS-staged kernel: tile rows (16 or 32) */
    VACV_TUNE_WARP_SLOTS = 17,       /* u8 CONSTANT warp, LDS-staged kernel: source boxes in the LDS ring (2-4) */
    VACV_TUNE_LANCZOS_KERNEL = 18,   /* u8 INTER_LANCZOS4: 0 register-ring kernel (staged runs where they fit), 1 the LDS-ring kernel, 2 the register ring with per-lane windows (A/B) */
    VACV_TUNE_COUNT = 19
};
/* value < 0 restores the built-in choice.  Returns VACV_OK or INVALID_ARG. */
int vacv_set_tuning(int key, int value);
/* the current value (-1 = built-in), or VACV_ERR_INVALID_ARG for a bad key */
int vacv_get_tuning(int key);

/* Block until all work this library queued on `stream` has finished. */
int vacv_stream_synchronize(void* stream);
/* Release the per-device workspace the statistics paths cache. */
int vacv_release_workspace(void);

#ifdef __cplusplus
}
#endif
#endif /* VACV_HIP_H */
