// vacv_internal.hpp -- kernel parameter blocks and launcher declarations
// shared between the C-ABI layer (vacv_abi.cpp) and the kernels (*.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <set>

#include "../../include/vacv_hip.h"

namespace vacv {

constexpr int kBlock = 256;         // threads per workgroup (4 waves)
constexpr int kMaxC = VACV_MAX_CHANNELS;
constexpr int kResizeMaxChunksPerLane = 1;        // fp32 resize: 4-element chunks per lane per row
constexpr int64_t kMaxPlaneBytes = 0x7FFFFFF0LL;  // buffer-resource addressing limit of one plane

// A kernel-variant knob (tuning.cpp, VACV_TUNE_*): -1 = the built-in choice.
int tune(int key);
inline int tune_or(int key, int def) {
    const int v = tune(key);
    return v < 0 ? def : v;
}

// How a batch is walked: a "plane" is what one sampler pass sees -- a whole
// NHWC image (cc = c interleaved channels) or one NCHW channel plane (cc = 1).
struct PlaneGeom {
    const unsigned char* base;   // image 0, plane 0, pixel (0,0)
    int64_t img_pitch;           // bytes between images
    int64_t plane_pitch;         // bytes between planes of one image (NCHW)
    int64_t row_pitch;           // bytes between rows
    int planes;                  // planes per image (NCHW: c, NHWC: 1)
    int w, h;
    int cc;                      // interleaved channels per pixel
    int esize;                   // bytes per element
    int64_t plane_bytes;         // readable bytes from one plane's base
};

// Normalisation applied by a fused epilogue.
struct NormSpec {
    int mode;                    // 0 none, 1 host constants, 2 per-image device arrays
    int c_total;                 // channels of the image (NCHW plane p -> channel p % c_total)
    const float* dev_mean;       // [n][c_total] (mode 2)
    const float* dev_std;
    float mean[kMaxC];
    float stdv[kMaxC];
    // mode 1: inv[k] = 1 / ((double)stdv[k] + 1e-6).  Bit k of mul_ok is set
    // when the host verified, for all 256 u8 values v, that
    //   (float)((double)((float)v - mean[k]) * inv[k])
    // equals the reference's (float)((double)((float)v - mean[k]) /
    // ((double)stdv[k] + 1e-6)); kernels then use the multiply for
    // u8-valued inputs (an fp64 divide is ~10x the issue cost).
    double inv[kMaxC];
    uint32_t mul_ok;
    // Bit k of f32_ok: the host verified, for all 256 u8 values v, that the
    // fp32 form fmaf(d, inv_hi[k], d * inv_lo[k]) (d = (float)v - mean[k];
    // inv_hi + inv_lo = inv[k] to ~48 bits) equals the reference's result;
    // kernels then take it instead of the fp64 multiply (2 fp32 VALU
    // instead of 3 fp64 ones).
    float inv_hi[kMaxC];
    float inv_lo[kMaxC];
    uint32_t f32_ok;
};

enum SampleKind : int {
    kLinearFixed = 0,   // u8 bilinear (modes REFERENCE / NEON / OPENCV)
    kLinearFloat = 1,   // fp32 bilinear
    kCubic = 2,         // fp32 (or u8 widened) Keys cubic
};

enum OutKind : int {
    kOutSame = 0,       // u8 -> u8 or f32 -> f32
    kOutF32 = 1,        // widened to f32, no normalisation
    kOutNorm = 2,       // f32, normalised
};

// Exact tap tables of one resize geometry, built on the host with the
// reference's arithmetic (vacv_semantics.hpp) and cached on the device (the
// counterpart of the reference's xofs/ialpha/yofs/ibeta tables,
// resize_neon.cpp:20-78).  All arrays live in one device allocation.
struct ResizePlanDev {
    const int* xoff;             // [tiles_x][tile_w] byte offset of the first tap in the staged span
    const void* xw;              // [tiles_x][tile_w] short2 (fixed) | float2 | float4 (cubic)
    const int* col_first;        // [tiles_x] first staged source column
    const int* cpr;              // [tiles_x] 16-byte chunks per staged row
    const int* yrow;             // [h_out] first vertical tap row
    const void* yw;              // [h_out] int2 (fixed) | float2 | float4
    const int* task_nslots;      // [tiles_y]
    const int* task_rows;        // [tiles_y][max_slots] source row of each LDS slot
    const int* task_cand;        // [tiles_y][tile_h*TAPS] slot of (row t, tap j) or -1 (zero weight)
    const int* task_flags;       // [tiles_y] bit j: some row of the tile has a non-zero weight on tap j
    const float* lut;            // [c_total][256] normalised u8 values (host-constant mean/std) or null
};

struct ResizeLaunch {
    PlaneGeom src;
    PlaneGeom dst;
    int n;
    int kind;                    // SampleKind
    int mode;                    // VACV_LINEAR_* for kLinearFixed
    int out;                     // OutKind
    float scale_xf, scale_yf;    // (float)w_in / w_out (naive)
    double scale_xd, scale_yd;   // (double)w_in / w_out (NEON, cubic)
    int tile_w, tile_h, tiles_x, tiles_y;
    int sparse;                  // 1: slots hold only non-zero-weight rows; 0: dense row window
    int max_slots;               // LDS row slots per workgroup
    int slot_stride;             // bytes per slot
    int lds_bytes;               // dynamic LDS per workgroup
    int strips;                  // workgroups per (plane, tile column)
    int tasks_per_strip;         // row tiles per workgroup (software-pipelined)
    int interleave;              // resize_kernel: 1 = tasks grid-stride in address order, 0 = strips
    int area_x, area_y;          // INTER_AREA integer block (launch_resize_area)
    float area_scale;            // INTER_AREA: 1.f / (area_x * area_y)
    int area_half_up;            // INTER_AREA u8 2x2, cn 1/3/4: (sum + 2) >> 2 (ResizeAreaFastVec fast_mode)
    ResizePlanDev plan;
    NormSpec norm;
    // cubic gather kernel only (or null): the output's per-channel
    // (Sum x, Sum x^2) -- per-workgroup partials [cc][2][image][workgroup]
    // (cubic_direct_groups() per image, a workspace), then sum_out =
    // [n][cc][2] (sum_per_image) or [cc][2] in a fixed order; with sum_mean /
    // sum_std (or null) also the population mean / stddev of each group
    double* sum_partials;
    double* sum_out;
    int sum_per_image;
    float* sum_mean;
    float* sum_std;
    // the column kernel's fixed-point accumulators (or null: per-workgroup
    // partials and group_sums_kernel): [n][cc][2] int64, zero on entry and
    // left zero; Sum x in units of 2^-sum_q1, Sum x^2 in units of 2^-sum_q2
    // (set by the launcher)
    int64_t* sum_acc;
    int sum_q1, sum_q2;
};

// Fills tiles, strips and the cached device plan of L (host).
int plan_resize(ResizeLaunch& L, hipStream_t s);
void set_strips(ResizeLaunch& L, int64_t resident_workgroups);
int release_plans();

// Frees every entry of a device-side cache whose entries record their owning
// device (`.device`): each owner is synchronised and its allocations freed
// with that device current; the caller's device is restored.  Returns
// VACV_OK or VACV_ERR_HIP; the map is cleared either way.
template <class Map, class FreeFn>
int evict_device_cache(Map& m, FreeFn free_entry) {
    int cur = 0, st = VACV_OK;
    if (hipGetDevice(&cur) != hipSuccess) st = VACV_ERR_HIP;
    std::set<int> owners;
    for (auto& kv : m) owners.insert(kv.second.device);
    for (int d : owners)
        if (hipSetDevice(d) != hipSuccess || hipDeviceSynchronize() != hipSuccess) st = VACV_ERR_HIP;
    for (auto& kv : m)
        if (hipSetDevice(kv.second.device) != hipSuccess || !free_entry(kv.second)) st = VACV_ERR_HIP;
    if (!m.empty() && hipSetDevice(cur) != hipSuccess) st = VACV_ERR_HIP;
    m.clear();
    return st;
}

hipError_t launch_resize(const ResizeLaunch& L, hipStream_t s);
// u8 bilinear as per-pixel gathers (k_resize_direct.hip); needs no plan.
// resize_one_tap_rows: no output row of L has two weighted source rows.
hipError_t launch_resize_direct(const ResizeLaunch& L, hipStream_t s);
bool resize_one_tap_rows(const ResizeLaunch& L);
// u8 bilinear as column strips walking down the image with an LDS ring of
// source rows (k_resize_strip.hip): two-tap geometries
bool resize_strip_applies(const ResizeLaunch& L);
hipError_t launch_resize_strip(const ResizeLaunch& L, hipStream_t s);
// INTER_NEAREST (OpenCV 2.4 resizeNN): scale_xd / scale_yd carry ifx / ify
hipError_t launch_resize_nearest(const ResizeLaunch& L, hipStream_t s);
// INTER_AREA at an integer scale (OpenCV 2.4 resizeAreaFast_): area_x/y, area_scale
hipError_t launch_resize_area(const ResizeLaunch& L, hipStream_t s);
// INTER_AREA at any other scale (k_area.hip): OpenCV 2.4's resizeArea_ tables
// (down-scales) or its area-mode bilinear (up-scales); inv_x / inv_y =
// cv::resize's inv_scale.  Returns a vacv_status.
int launch_resize_area_general(const ResizeLaunch& L, double inv_x, double inv_y, hipStream_t s);
int release_area_tables();
// INTER_LANCZOS4 (k_lanczos.hip): OpenCV 2.4 cv::resize restated; inv_x /
// inv_y = dsize / ssize (or fx / fy)
int launch_resize_lanczos(const ResizeLaunch& L, double inv_x, double inv_y, hipStream_t s);
int release_lanczos_tables();
// u8 -> fp32 cubic as per-pixel gathers (k_cubic_direct.hip); needs no plan
bool cubic_direct_applies(const ResizeLaunch& L);
hipError_t launch_cubic_direct(const ResizeLaunch& L, hipStream_t s);
int cubic_direct_groups(const ResizeLaunch& L);  // workgroups per output plane (the sum_partials layout)
int64_t cubic_sums_groups_bound(int w, int h);  // >= cubic_direct_groups() for any w x h output

struct WarpLaunch {
    PlaneGeom src;
    PlaneGeom dst;
    int n;
    float inv[6];
    double invd[6];              // INTER_NEAREST: OpenCV's fp64 inverse map (warpAffine)
    float border[4];
    int border_mode;             // kBorder* (vacv_semantics.hpp)
    int out;                     // OutKind
    NormSpec norm;
};
hipError_t launch_warp(const WarpLaunch& L, hipStream_t s);
// INTER_NEAREST (OpenCV 2.4 warpAffine + remapNearest; the reference hands
// every flag but INTER_LINEAR to OpenCV, warp_affine.cpp:114-118)
hipError_t launch_warp_nearest(const WarpLaunch& L, hipStream_t s);
// u8 CONSTANT warp (1-4 interleaved channels, or NCHW planes) with the source boxes
// copied into an LDS ring by LDS-DMA and the geometry shared by kf frames per
// workgroup (k_warp_frames.hip)
struct WarpFramesPlan {
    int th;                      // tile rows (16 or 32; 64 columns)
    int S;                       // LDS bytes per staged source row (raw pixel bytes, a multiple of 16)
    int rows_max;                // staged rows per LDS slot
    int ns;                      // LDS slots of the ring (boxes: one being sampled, ns - 1 in flight)
    int slot;                    // bytes per slot (a 16-byte border head, rows in whole 1 KiB DMA units)
    int lds;                     // dynamic LDS per workgroup
    int kf;                      // frames per workgroup (<= 0: chosen at launch)
    int dst_al;                  // destination dword-aligned (u8 quad stores)
    int se;                      // 1: warp_exp_kernel (3 channels, compact spans, a 4-byte-pixel image); 0: warp_ring_kernel
    int raw_bytes;               // warp_exp_kernel: bytes of each of its two raw DMA slots
    int exp_units;               // warp_exp_kernel: 16-pixel units of its image
    int tw;                      // warp_exp_kernel: tile columns (64)
};
bool warp_frames_plan(const WarpLaunch& L, WarpFramesPlan& P);
hipError_t launch_warp_frames(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s);
// INTER_NEAREST with the same staging (3-channel u8, BORDER_CONSTANT)
bool warp_exp_nn_plan(const WarpLaunch& L, WarpFramesPlan& P);
hipError_t launch_warp_exp_nn(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s);

struct CopyLaunch {                // crop / clone: row copies
    PlaneGeom src;                 // base already offset to the crop origin
    PlaneGeom dst;
    int n;
    int64_t row_bytes;
};
hipError_t launch_row_copy(const CopyLaunch& L, hipStream_t s);

struct LayoutLaunch {
    const unsigned char* src;
    unsigned char* dst;
    int n, w, h, c, esize;
    int to_chw;                    // 1: NHWC -> NCHW, 0: NCHW -> NHWC
    int64_t src_img, dst_img;      // dense per-image bytes
};
hipError_t launch_layout(const LayoutLaunch& L, hipStream_t s);

struct DtypeLaunch {
    const unsigned char* src;
    unsigned char* dst;
    int64_t count;                 // elements (dense)
    int to_f32;                    // 1: u8 -> f32, 0: f32 -> u8
};
hipError_t launch_dtype(const DtypeLaunch& L, hipStream_t s);

struct ColorLaunch {
    const unsigned char* src;      // Y plane of image 0
    int64_t src_img, src_row;      // bytes
    unsigned char* dst;
    int64_t dst_img, dst_row;
    int n, w, h;                   // BGR size
    int v_first;                   // NV21
    int rgb;                       // swap output order
    int out;                       // kOutSame (u8) / kOutF32 / kOutNorm
    NormSpec norm;
};
hipError_t launch_color(const ColorLaunch& L, hipStream_t s);

// cv::cvtColor codes the reference delegates to OpenCV (k_color_cv.hip):
// YUV420 -> BGR(A)/RGB(A) in OpenCV 2.4's BT.601 fixed point, GRAY -> BGR(A)
struct CvColorLaunch {
    const unsigned char* src;      // Y plane (or the gray image) of image 0
    int64_t src_img, src_row;      // bytes
    unsigned char* dst;
    int64_t dst_img, dst_row;
    int n, w, h;                   // output size
    int gray;                      // 1: GRAY2BGR(A), else YUV420
    int layout;                    // YUV: 0 NV12, 1 NV21, 2 YV12, 3 IYUV
    int dcn;                       // 3 or 4 output channels
    int bidx;                      // 0: BGR(A) order, 2: RGB(A)
    int esize;                     // gray: 1 (u8) or 4 (fp32)
    int aligned;                   // YUV: dst rows allow 8-byte (dcn 4) / 2-byte (dcn 3) stores
};
hipError_t launch_color_cv(const CvColorLaunch& L, hipStream_t s);

// YUV420sp -> BGR -> u8 bilinear resize (-> fp32 / normalised fp32), NHWC or
// NCHW output: the model-input pipeline of SURVEY.md §8(f)2 in one pass
// (k_yuv_resize.hip).
struct YuvResizeLaunch {
    const unsigned char* src;      // Y plane of image 0
    int64_t src_img, src_row;      // bytes
    int64_t src_bytes;             // readable bytes of one image (Y + chroma planes)
    unsigned char* dst;
    int64_t dst_img, dst_row, dst_plane;  // bytes; dst_plane used for NCHW
    int n, w, h;                   // decoded BGR size
    int wo, ho;                    // output size
    int v_first;                   // NV21
    int rgb;                       // swap output channel order
    int chw;                       // 1: NCHW planar output, 0: NHWC
    int mode;                      // VACV_LINEAR_*
    int out;                       // kOutSame (u8) / kOutF32 / kOutNorm
    float scale_xf, scale_yf;
    double scale_xd, scale_yd;
    NormSpec norm;
};
hipError_t launch_yuv_resize(const YuvResizeLaunch& L, hipStream_t s);

struct NormLaunch {                // elementwise normalize
    PlaneGeom src;
    PlaneGeom dst;
    int n;
    int src_u8;
    NormSpec norm;
};
hipError_t launch_normalize(const NormLaunch& L, hipStream_t s);

struct SumsLaunch {
    PlaneGeom src;                 // whole images (NHWC: cc = c; NCHW: planes = c, cc = 1)
    int n;
    int c;
    int src_u8;
    int blocks_per_image;
    double* partials;              // [n][blocks][c][2]
    double* sums;                  // [groups][c][2]
    int per_image;
    int scalar_only;               // plane base not 16-byte aligned
};
hipError_t launch_channel_sums(const SumsLaunch& L, hipStream_t s);
hipError_t launch_stats(const double* sums, int groups, int c, double count,
                        float* mean, float* stddev, hipStream_t s);

// match_template (k_match.hip): n images against one template
struct MatchLaunch {
    const unsigned char* img;     // image 0
    int64_t img_pitch, img_row;   // bytes
    int iw, ih, cn, esize, n;
    const unsigned char* tpl;
    int64_t tpl_row;
    int tw, th;
    unsigned char* res;           // FP32 result of image 0
    int64_t res_pitch, res_row;   // bytes
    int rw, rh;
    int method;                   // VACV_TM_*
    double inv_area;              // 1 / (tw * th)
    double* box;                  // workspace: [n][2][ih+1][(iw+1)*cn] integral images (sum, sqsum)
    double* tstats;               // workspace: template mean[4], norm, sum2, all-ones flag
    void* bfrag;                  // workspace of match_bfrag_bytes() (u8 MFMA correlation), or null
};
size_t match_lds_bytes(int tw, int th, int cn, int esize);
bool match_mfma_plan(int tw, int th, int cn, int& KB, int& stride);
size_t match_bfrag_bytes(int tw, int th, int cn);
hipError_t launch_match_template(const MatchLaunch& M, hipStream_t s);

struct MinMaxLaunch {             // minMaxIdx of one single-channel image
    const unsigned char* src;
    int64_t row;
    int w, h, esize;
    const unsigned char* mask;    // INT8 (w, h), non-zero = included; or null
    int64_t mask_row;
    double* out_val;              // device: min, max
    int* out_idx;                 // device: min row, min col, max row, max col
};
size_t min_max_workspace_bytes();
hipError_t launch_min_max(const MinMaxLaunch& L, void* ws, hipStream_t s);

}  // namespace vacv
