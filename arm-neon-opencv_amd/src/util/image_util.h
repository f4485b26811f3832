// ImageUtil -- the reference harness's helpers (src/util/image_util.h):
// cosine similarity of two buffers, and BGR -> NV21 for making YUV inputs.
// Host-side test utilities; no operator of va_cv:: calls them.
#ifndef IMAGE_UTIL_H
#define IMAGE_UTIL_H

#include <math.h>

class ImageUtil {
public:
    /// cosine similarity with float accumulation, norms seeded at 1e-6,
    /// exactly as the reference harness scores outputs (image_util.h:15-32)
    template <typename T>
    static float compare_image_data(const T* first, const T* second, int len) {
        if (first == nullptr || second == nullptr) return 0.0f;
        float dot = 0.0f, n1 = 0.000001f, n2 = 0.000001f;
        for (int i = 0; i < len; ++i) {
            const float a = static_cast<float>(first[i]);
            const float b = static_cast<float>(second[i]);
            dot += a * b;
            n1 += a * a;
            n2 += b * b;
        }
        return dot / sqrt(n1 * n2);
    }

    /// BGR (w*h*3) -> NV21 (w*h luma + interleaved V,U at 2x2), 14-bit fixed
    /// point (image_util.cpp:3-41); odd sizes or null pointers do nothing
    static void bgr2nv21(unsigned char* src, unsigned char* dst, int width, int height);
};

#endif  // IMAGE_UTIL_H
