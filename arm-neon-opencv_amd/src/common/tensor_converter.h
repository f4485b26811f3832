// TensorConverter: cv::Mat <-> vision::Tensor, as the reference's harness
// uses it (src/common/tensor_converter.{h,cpp}).
//
// Header-only: the specialisations below exist when the including code has
// OpenCV on its include path, so a caller that links OpenCV keeps
// `TensorConverter::convert_from<cv::Mat>(mat)` unchanged and this library
// itself never depends on OpenCV.  Conversions are host-side views/copies
// (a device Tensor is brought to the host first by convert_to).
#ifndef VISION_TENSOR_CONVERTER_H
#define VISION_TENSOR_CONVERTER_H

#include <cstring>
#include <stdexcept>

#include "tensor.h"

namespace vision {

class TensorConverter {
public:
    template <typename T>
    static T convert_to(const Tensor& tensor, bool copy = false);

    template <typename T>
    static Tensor convert_from(const T& mat, bool copy = false);
};

}  // namespace vision

#if defined(__has_include)
#if __has_include(<opencv2/core/core.hpp>)
#include <opencv2/core/core.hpp>
#define VACV_HAVE_OPENCV_CONVERTER 1

namespace vision {

// tensor_converter.cpp:15-44: FP32/FP16/INT8/FP64 -> CV_32F/16U/8U/64F, HWC
template <>
inline cv::Mat TensorConverter::convert_to<cv::Mat>(const Tensor& tensor_in, bool copy) {
    if (tensor_in.empty()) return cv::Mat();
    const Tensor tensor = tensor_in.to_host();
    int depth;
    switch (tensor.dtype) {
        case FP32: depth = CV_32F; break;
        case FP16: depth = CV_16U; break;
        case INT8: depth = CV_8U; break;
        case FP64: depth = CV_64F; break;
        default: throw std::runtime_error("TensorConverter: dtype has no cv::Mat equivalent");
    }
    const int type = CV_MAKETYPE(depth, tensor.c);
    if (copy || tensor.data != tensor_in.data) {
        cv::Mat mat(tensor.h, tensor.w, type);
        std::memcpy(mat.data, tensor.data, tensor.len());
        return mat;
    }
    return cv::Mat(tensor.h, tensor.w, type, tensor.data);
}

// tensor_converter.cpp:46-83: depth -> dtype, always NHWC
template <>
inline Tensor TensorConverter::convert_from<cv::Mat>(const cv::Mat& mat, bool copy) {
    if (mat.empty()) return Tensor();
    DType dt;
    switch (mat.depth()) {
        case CV_8U: case CV_8S: dt = INT8; break;
        case CV_16U: case CV_16S: dt = FP16; break;
        case CV_32S: case CV_32F: dt = FP32; break;
        case CV_64F: dt = FP64; break;
        default: throw std::runtime_error("TensorConverter: cv::Mat depth not supported");
    }
    if (copy) {
        Tensor t(mat.cols, mat.rows, mat.channels(), dt, NHWC);
        std::memcpy(t.data, mat.data, t.len());
        return t;
    }
    return Tensor(mat.cols, mat.rows, mat.channels(), mat.data, dt, NHWC);
}

}  // namespace vision
#endif
#endif

#endif  // VISION_TENSOR_CONVERTER_H
