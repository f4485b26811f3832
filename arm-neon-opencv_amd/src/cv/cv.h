// va_cv:: -- the vacv image-operator API, MI355X build.
//
// Same names, signatures, defaults and enum values as the reference's
// src/cv/cv.h:9-241, so code written against it (including the reference's
// src/test harness) compiles unchanged.  Every operator is one or more HIP
// kernels for gfx950 behind the C ABI in include/vacv_hip.h; nothing here
// computes pixels on the host.
//
// Behaviour relative to the reference:
//   - outputs take the placement of `src` (host tensors are staged through
//     pinned buffers; device tensors stay in HBM), and calls are synchronous;
//   - combinations the reference silently skips or recurses on forever throw
//     std::runtime_error instead;
//   - warp_affine does not modify M and writes borderValue outside the source.
#ifndef VISION_CV_H
#define VISION_CV_H

#include <vector>

#include "../common/tensor.h"
#include "../common/vision_structs.h"

namespace va_cv {

struct VSize {
    int w;
    int h;
    VSize() : w(0), h(0) {}
    VSize(int _w, int _h) : w(_w), h(_h) {}
};

struct VScalar {
    double v0;
    double v1;
    double v2;
    double v3;
    VScalar() : v0(0), v1(0), v2(0), v3(0) {}
};

/// interpolation (cv.h:27-36)
enum VInterMode {
    INTER_NEAREST = 0,
    INTER_LINEAR = 1,
    INTER_CUBIC = 2,
    INTER_AREA = 3,
    INTER_LANCZOS4 = 4,
    INTER_MAX = 7,
    WARP_INVERSE_MAP = 16
};

/// border handling (cv.h:39-49)
enum VBorderMode {
    BORDER_REPLICATE = 1,
    BORDER_CONSTANT = 0,
    BORDER_REFLECT = 2,
    BORDER_WRAP = 3,
    BORDER_REFLECT_101 = 4,
    BORDER_REFLECT101 = 4,
    BORDER_TRANSPARENT = 5,
    BORDER_DEFAULT = 4,
    BORDER_ISOLATED = 16
};

/// template-matching methods (cv.h:52-59)
enum VMatchMode {
    TM_SQDIFF = 0,
    TM_SQDIFF_NORMED = 1,
    TM_CCORR = 2,
    TM_CCORR_NORMED = 3,
    TM_CCOEFF = 4,
    TM_CCOEFF_NORMED = 5
};

/// colour conversion codes (cv.h:62-74)
enum InputImageFormat {
    COLOR_GRAY2RGB = 8,
    COLOR_GRAY2BGR = COLOR_GRAY2RGB,
    COLOR_YUV2RGB_NV12 = 90,
    COLOR_YUV2BGR_NV12 = 91,
    COLOR_YUV2RGB_NV21 = 92,
    COLOR_YUV2BGR_NV21 = 93,
    COLOR_YUV2RGBA_NV12 = 94,
    COLOR_YUV2BGRA_NV12 = 95,
    COLOR_YUV2RGBA_NV21 = 96,
    COLOR_YUV2BGRA_NV21 = 97,
    COLOR_YUV2BGR_YV12 = 99
};

/// Resize to dsize (fx, fy ignored, as in resize.cpp:51-56, except for
/// INTER_NEAREST / INTER_AREA with dsize = 0, which the reference hands to
/// cv::resize: dsize = round(w * fx, h * fy), inv_scale = fx, fy).
/// INTER_LINEAR: INT8 -> INT8 (bit-exact with resize_naive_inter_linear_u8),
/// FP32 -> FP32.  INTER_CUBIC: FP32 -> FP32, and INT8 -> FP32 (a fused widen;
/// the reference recurses forever on INT8 cubic).  NHWC or NCHW.
void resize(const vision::Tensor& src, vision::Tensor& dst,
            VSize dsize, double fx = 0, double fy = 0,
            int interpolation = INTER_LINEAR);

/// YUV420sp (w, h*3/2, 1) INT8 -> (w, h, 3) INT8 NHWC (cvt_color.cpp:137-157).
/// COLOR_YUV2BGR_NV21 is bit-exact with nv_to_bgr_naive; NV12 and the RGB
/// orders are also decoded.  The codes the reference hands to cv::cvtColor
/// (cvt_color.cpp:139-141) follow OpenCV 2.4: COLOR_YUV2RGBA/BGRA_NV12/NV21
/// -> (w, h, 4), COLOR_YUV2BGR_YV12 (planar V, U) -> (w, h, 3), and
/// COLOR_GRAY2BGR (w, h, 1) INT8/FP32 -> (w, h, 3) of the same dtype.
void cvt_color(const vision::Tensor& src, vision::Tensor& dst, int code);

/// dst = (x - mean[k]) / (stddev[k] + 1e-6), FP32, same layout
/// (normalize.cpp:84-121).  mean/stddev: FP32 tensors of c values; both
/// empty = per-image statistics of src.
void normalize(const vision::Tensor& src, vision::Tensor& dst,
               const vision::Tensor& mean = vision::Tensor(),
               const vision::Tensor& stddev = vision::Tensor());

/// Affine warp by the FORWARD 2x3 map M (3x2x1 FP32 tensor), INTER_LINEAR
/// (warp_affine.cpp:111-169).  M is not modified.  BORDER_CONSTANT is the
/// reference's naive path; REPLICATE / REFLECT / WRAP / REFLECT_101 /
/// TRANSPARENT extend it (the reference hands them to OpenCV).
void warp_affine(const vision::Tensor& src, vision::Tensor& dst,
                 const vision::Tensor& M, VSize dsize,
                 int flags = INTER_LINEAR,
                 int borderMode = BORDER_CONSTANT,
                 const VScalar& borderValue = VScalar());

/// Warp by rotation `rot` (degrees) and `scale` about the origin, translated
/// by aux_param (warp_affine.cpp:76-109).
void warp_affine(const vision::Tensor& src, vision::Tensor& dst,
                 float scale, float rot, VSize dsize,
                 const VScalar& aux_param = VScalar(),
                 int flags = INTER_LINEAR,
                 int borderMode = BORDER_CONSTANT,
                 const VScalar& borderValue = VScalar());

/// resize + convert to FP32 + normalize in one kernel (resize_normalize.cpp:
/// 33-107).  Either statistic empty = per-image statistics of the resized
/// image.
void resize_normalize(const vision::Tensor& src, vision::Tensor& dst,
                      VSize dsize, double fx = 0, double fy = 0,
                      int interpolation = INTER_LINEAR,
                      const vision::Tensor& mean = vision::Tensor(),
                      const vision::Tensor& stddev = vision::Tensor());

/// warp_affine + convert to FP32 + normalize in one kernel
/// (warp_affine_normalize.cpp:13-210).
void warp_affine_normalize(const vision::Tensor& src, vision::Tensor& dst,
                           const vision::Tensor& M, VSize dsize,
                           int flags = INTER_LINEAR,
                           int borderMode = BORDER_CONSTANT,
                           const VScalar& borderValue = VScalar(),
                           const vision::Tensor& mean = vision::Tensor(),
                           const vision::Tensor& stddev = vision::Tensor());

void warp_affine_normalize(const vision::Tensor& src, vision::Tensor& dst,
                           float scale, float rot, VSize dsize,
                           const VScalar& aux_param = VScalar(),
                           int flags = INTER_LINEAR,
                           int borderMode = BORDER_CONSTANT,
                           const VScalar& borderValue = VScalar(),
                           const vision::Tensor& mean = vision::Tensor(),
                           const vision::Tensor& stddev = vision::Tensor());

/// ROI copy; the rect is truncated to int (crop.cpp:127-142).
void crop(const vision::Tensor& src, vision::Tensor& dst, const vision::VRect& rect);

/// Template matching (match_template.cpp:13-41 hands it to cv::matchTemplate):
/// OpenCV 2.4's six TM_* methods, INT8 / FP32 NHWC, c <= 4; result =
/// (W-w+1, H-h+1, 1) FP32.  The correlation is computed exactly on the GPU.
void match_template(const vision::Tensor& src, const vision::Tensor& target,
                    vision::Tensor& result, int method);
/// cv::minMaxIdx of a single-channel tensor (match_template.cpp:43-46):
/// first minimum / maximum in row-major order among mask != 0; indices are
/// (row, col).
void minMaxIdx(const vision::Tensor& src, double* minVal, double* maxVal,
               int* minIdx = nullptr, int* maxIdx = nullptr, const vision::Tensor& mask = vision::Tensor());
/// OpenCV-only in the reference (imencode.cpp, a codec): throws.
void imencode(const vision::Tensor& src, std::vector<unsigned char>& buf, const char* format);

// ---- additions (not in the reference) -----------------------------------

/// Per-channel population mean / stddev of one image (the statistics the
/// reference computes inside normalize, normalize_naive.cpp:7-72), exact
/// (integer / fp64 accumulation).  mean, stddev: host FP32 tensors (c).
void mean_stddev(const vision::Tensor& src, vision::Tensor& mean, vision::Tensor& stddev);

/// cvt_color then normalize, one kernel (the BASELINE cfg3 pipeline).
void cvt_color_normalize(const vision::Tensor& src, vision::Tensor& dst, int code,
                         const vision::Tensor& mean = vision::Tensor(),
                         const vision::Tensor& stddev = vision::Tensor());

/// Batched frames: the operator above applied to every
/// frame of `src` into the matching `dst` (resized to src.size()).  Host
/// frames are staged through a ring of HBM buffers on three HIP streams, so
/// the H2D copy of frame i+1, the kernel of frame i and the D2H copy of frame
/// i-1 overlap -- one call per frame serialises them on one stream.  Device
/// frames run back to back.  Returns when every dst is written.
void resize(const std::vector<vision::Tensor>& src, std::vector<vision::Tensor>& dst, VSize dsize,
            double fx = 0, double fy = 0, int interpolation = INTER_LINEAR);
void resize_normalize(const std::vector<vision::Tensor>& src, std::vector<vision::Tensor>& dst, VSize dsize,
                      double fx = 0, double fy = 0, int interpolation = INTER_LINEAR,
                      const vision::Tensor& mean = vision::Tensor(),
                      const vision::Tensor& stddev = vision::Tensor());
void warp_affine(const std::vector<vision::Tensor>& src, std::vector<vision::Tensor>& dst,
                 const vision::Tensor& M, VSize dsize, int flags = INTER_LINEAR,
                 int borderMode = BORDER_CONSTANT, const VScalar& borderValue = VScalar());
void cvt_color(const std::vector<vision::Tensor>& src, std::vector<vision::Tensor>& dst, int code);
void cvt_color_normalize(const std::vector<vision::Tensor>& src, std::vector<vision::Tensor>& dst, int code,
                         const vision::Tensor& mean = vision::Tensor(),
                         const vision::Tensor& stddev = vision::Tensor());

}  // namespace va_cv

#endif  // VISION_CV_H
