#include "image_util.h"

// BT.601 weights scaled by 2^14 (image_util.cpp:3-7): Y = (B*b + G*g + R*r) >> 14,
// U/V from (B - Y) / (R - Y) with a +128 bias, sampled at even (row, col).
void ImageUtil::bgr2nv21(unsigned char* src, unsigned char* dst, int width, int height) {
    if (!src || !dst || (width & 1) || (height & 1)) return;
    const unsigned kB = 1868, kG = 9617, kR = 4899, kU = 9241, kV = 11682;
    const unsigned kBias = 128u << 14;
    unsigned char* luma = dst;
    unsigned char* chroma = dst + (long)width * height;
    for (int y = 0; y < height; ++y) {
        for (int x = 0; x < width; ++x, src += 3) {
            const int Y = (int)((unsigned)(src[0] * kB + src[1] * kG + src[2] * kR) >> 14);
            *luma++ = (unsigned char)Y;
            if (((x | y) & 1) == 0) {
                // unsigned wrap-around of negative differences is the reference's arithmetic
                *chroma++ = (unsigned char)((unsigned)((src[2] - Y) * kV + kBias) >> 14);
                *chroma++ = (unsigned char)((unsigned)((src[0] - Y) * kU + kBias) >> 14);
            }
        }
    }
}
