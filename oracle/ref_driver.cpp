// ref_driver.cpp -- C entry points into the REFERENCE's own pixel loops.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles this file together with
// the reference sources where they lie (/root/reference/src/...) into
// oracle/_ref/libvacv_ref.so.  Nothing from the reference is copied into this
// repository.  The library pins the C restatement (vacv_oracle.c) and is
// what tests/golden/make_golden.py runs to produce the committed fixtures.
//
// Only pointer-level kernels are reachable: everything that goes through
// vision::Tensor needs tensor.cpp, which does not compile as shipped
// (tensor.cpp:536 calls VaAllocator::allocate(int); va_allocator.h:8 declares
// allocate(void**, int)).  cvt_color.o still references Tensor::create from
// cvt_color_naive; that symbol stays undefined and is never called (the
// library is linked -z lazy and loaded with RTLD_LAZY).
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "/root/reference/src/cv/resize_naive.h"
#include "/root/reference/src/cv/warp_affine_naive.h"
#include "/root/reference/src/cv/normalize_naive.h"
#include "/root/reference/src/util/image_util.h"
// nv_to_bgr_naive is a private static member; expose it for this TU only.
#define private public
#include "/root/reference/src/cv/cvt_color.h"
#undef private

using va_cv::ResizeNaive;

extern "C" {

// resize_naive.cpp:10-68
void ref_resize_linear_u8(const uint8_t* src, int w_in, int h_in, int c,
                          uint8_t* dst, int w_out, int h_out) {
    ResizeNaive::resize_naive_inter_linear_u8((const char*)src, w_in, h_in, c,
                                              (char*)dst, w_out, h_out);
}

// resize_naive.cpp:70-128
void ref_resize_linear_f32(const float* src, int w_in, int h_in, int c,
                           float* dst, int w_out, int h_out) {
    ResizeNaive::resize_naive_inter_linear_fp32(src, w_in, h_in, c, dst, w_out, h_out);
}

// resize_naive.cpp:143-185
void ref_cubic_coeffs(int n_in, int n_out, int* ofs, float* coef) {
    ResizeNaive::cubic_coeffs_naive(n_in, n_out, ofs, coef);
}

// resize_naive.cpp:187-529 driven with separate (non-overlapping) tables;
// channels must be 1 or 3 (the reference has exactly those two loops).
void ref_resize_cubic_f32(const float* src, int w_in, int h_in, int c,
                          float* dst, int w_out, int h_out) {
    std::vector<int> xofs(w_out), yofs(h_out);
    std::vector<float> alpha(4 * (size_t)w_out), beta(4 * (size_t)h_out);
    ResizeNaive::cubic_coeffs_naive(w_in, w_out, xofs.data(), alpha.data());
    ResizeNaive::cubic_coeffs_naive(h_in, h_out, yofs.data(), beta.data());
    if (c == 3) {
        ResizeNaive::resize_naive_inter_cubic_fp32_three_channel(
            const_cast<float*>(src), w_in, h_in, dst, w_out, h_out,
            alpha.data(), xofs.data(), beta.data(), yofs.data());
    } else {
        ResizeNaive::resize_naive_inter_cubic_fp32_one_channel(
            const_cast<float*>(src), w_in, h_in, dst, w_out, h_out,
            alpha.data(), xofs.data(), beta.data(), yofs.data());
    }
}

// resize_naive.cpp:531-545 exactly as shipped (valid when w_out == h_out)
void ref_resize_cubic_f32_hwc_wrapper(const float* src, int w_in, int h_in,
                                      float* dst, int w_out, int h_out) {
    ResizeNaive::resize_naive_inter_cubic_fp32_hwc(const_cast<float*>(src), w_in, h_in,
                                                   dst, w_out, h_out);
}

// warp_affine_naive.cpp:9-58 / :60-106 (m = the inverted map)
void ref_warp_affine_u8(const uint8_t* src, int w_in, int h_in, int c,
                        uint8_t* dst, int w_out, int h_out, const float* m) {
    float mm[6];
    std::memcpy(mm, m, sizeof(mm));
    va_cv::WarpAffineNaive::warp_affine_naive_hwc_u8((char*)src, w_in, h_in, c,
                                                     (char*)dst, w_out, h_out, mm);
}

void ref_warp_affine_f32(const float* src, int w_in, int h_in, int c,
                         float* dst, int w_out, int h_out, const float* m) {
    float mm[6];
    std::memcpy(mm, m, sizeof(mm));
    va_cv::WarpAffineNaive::warp_affine_naive_hwc_fp32(const_cast<float*>(src), w_in, h_in, c,
                                                       dst, w_out, h_out, mm);
}

// normalize_naive.cpp:7-90
void ref_mean_stddev_hwc3(const float* src, int pixels, float* mean, float* stddev) {
    va_cv::NormalizeNaive::mean_stddev_naive_hwc_bgr(const_cast<float*>(src), pixels, mean, stddev);
}

void ref_mean_stddev_chw(const float* src, int pixels, int c, float* mean, float* stddev) {
    va_cv::NormalizeNaive::mean_stddev_naive_chw(const_cast<float*>(src), pixels, c, mean, stddev);
}

void ref_normalize_hwc3(const float* src, float* dst, int pixels, const float* mean, const float* stddev) {
    va_cv::NormalizeNaive::normalize_naive_hwc_bgr(const_cast<float*>(src), dst, pixels,
                                                   const_cast<float*>(mean), const_cast<float*>(stddev));
}

void ref_normalize_chw(const float* src, float* dst, int pixels, int c, const float* mean, const float* stddev) {
    va_cv::NormalizeNaive::normalize_naive_chw(const_cast<float*>(src), dst, pixels, c,
                                               const_cast<float*>(mean), const_cast<float*>(stddev));
}

// cvt_color.cpp:39-135; x_num/y_num as cvt_color_naive passes them
void ref_nv_to_bgr(const uint8_t* src, uint8_t* dst, int w, int h, int x_num, int y_num) {
    va_cv::CvtColor::nv_to_bgr_naive(src, dst, w, h, x_num, y_num);
}

// image_util.cpp:9-41
void ref_bgr2nv21(const uint8_t* bgr, uint8_t* dst, int w, int h) {
    ImageUtil::bgr2nv21(const_cast<uint8_t*>(bgr), dst, w, h);
}

// image_util.h:16-32
float ref_compare_image_data_u8(const uint8_t* a, const uint8_t* b, int len) {
    return ImageUtil::compare_image_data<unsigned char>(a, b, len);
}

float ref_compare_image_data_f32(const float* a, const float* b, int len) {
    return ImageUtil::compare_image_data<float>(a, b, len);
}

}  // extern "C"
