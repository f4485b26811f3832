// resize_plan.cpp -- host planner for the separable resamplers.
//
// For one resize geometry it computes, with the reference's arithmetic
// (vacv_semantics.hpp, the same functions the kernels would evaluate):
//   * the column taps of every output column (resize_naive.cpp:37-53,
//     resize_neon.cpp:35-56, resize_naive.cpp:143-185),
//   * the row taps of every output row,
//   * the workgroup tiling: tile_w x tile_h output tiles, the source rows each
//     tile stages into LDS (only rows with a non-zero weight), and how many
//     consecutive row tiles one workgroup streams through its software
//     pipeline,
//   * for u8 input with host-constant mean/stddev, the 256-entry normalisation
//     table per channel (normalize_naive.cpp:74-90 applied to every u8 value).
// The result is uploaded once into a device buffer and cached by geometry,
// so repeated calls (a video stream, a training input pipeline) launch the
// kernel with no per-call table work.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "vacv_internal.hpp"
#include "vacv_semantics.hpp"

namespace vacv {
namespace {

constexpr int kLdsBudget = 40 * 1024;   // per workgroup; 4 resident per CU
constexpr int kMaxChunksPerThread = 8;  // register prefetch depth (uint4 per thread)
constexpr int kWorkPerThread = 16;      // target output work items per thread per task (capped by LDS / prefetch registers)

struct Taps {
    int origin;   // first tap (row or column)
    int wi[2];
    float wf[4];
    int taps;
};

Taps tap_of(const ResizeLaunch& L, int d, bool vertical) {
    const int n_in = vertical ? L.src.h : L.src.w;
    const int n_out = vertical ? L.dst.h : L.dst.w;
    Taps t{};
    if (L.kind == kLinearFixed) {
        FixedTap q = fixed_tap(d, n_in, n_out, vertical ? L.scale_yf : L.scale_xf, vertical ? L.scale_yd : L.scale_xd,
                               L.mode);
        t.origin = q.i;
        t.wi[0] = q.w0;
        t.wi[1] = q.w1;
        t.taps = 2;
    } else if (L.kind == kLinearFloat) {
        FloatTap q = float_tap(d, n_in, vertical ? L.scale_yf : L.scale_xf);
        t.origin = q.i;
        t.wf[0] = q.w0;
        t.wf[1] = q.w1;
        t.taps = 2;
    } else {
        CubicTap q = cubic_tap(d, n_in, vertical ? L.scale_yd : L.scale_xd);
        t.origin = q.i - 1;
        for (int j = 0; j < 4; ++j) t.wf[j] = q.c[j];
        t.taps = 4;
    }
    return t;
}

bool weight_nonzero(const ResizeLaunch& L, const Taps& t, int j) {
    if (L.kind == kLinearFixed) return t.wi[j] != 0;
    return t.wf[j] != 0.f;
}

size_t a16(size_t v) { return (v + 15) & ~size_t(15); }

struct Geometry {
    int tile_w, tile_h, tiles_x, tiles_y, sparse, max_slots, slot_stride, lds;
    int max_cpr;
};

// Evaluate one candidate tiling; false when it does not fit.
bool evaluate(const ResizeLaunch& L, const std::vector<Taps>& xt, const std::vector<Taps>& yt, int tile_w, int tile_h,
              Geometry& g) {
    const int taps = L.kind == kCubic ? 4 : 2;
    const int bp = L.src.cc * L.src.esize;
    g.tile_w = tile_w;
    g.tile_h = tile_h;
    g.tiles_x = (L.dst.w + tile_w - 1) / tile_w;
    g.tiles_y = (L.dst.h + tile_h - 1) / tile_h;
    g.sparse = ((double)L.src.h / L.dst.h) >= taps ? 1 : 0;
    int max_span = 0;
    for (int tx = 0; tx < g.tiles_x; ++tx) {
        const int x0 = tx * tile_w, x1 = std::min(L.dst.w, x0 + tile_w) - 1;
        max_span = std::max(max_span, (xt[x1].origin + taps - 1 - xt[x0].origin + 1) * bp);
    }
    g.max_cpr = (max_span + 30) / 16;
    g.slot_stride = g.max_cpr * 16;
    int slots = 1;
    for (int ty = 0; ty < g.tiles_y; ++ty) {
        const int y0 = ty * tile_h, ny = std::min(tile_h, L.dst.h - y0);
        int cnt = 0;
        if (g.sparse) {
            for (int t = 0; t < ny; ++t)
                for (int j = 0; j < taps; ++j) cnt += weight_nonzero(L, yt[y0 + t], j);
        } else {
            cnt = yt[y0 + ny - 1].origin + taps - 1 - yt[y0].origin + 1;
        }
        slots = std::max(slots, cnt);
    }
    g.max_slots = slots;
    const int xw = L.kind == kLinearFixed ? 4 : (L.kind == kLinearFloat ? 8 : 16);
    g.lds = (int)(a16(tile_w * 4) + a16((size_t)tile_w * xw) + 32 * 8 * 4 + a16(slots * 4) +
                  (size_t)slots * g.slot_stride);
    if (tile_h * taps > 64) return false;
    if (L.dst.esize == 4 && (int64_t)tile_w * L.dst.cc > 4 * kResizeMaxChunksPerLane * kBlock) return false;
    if ((int64_t)slots * g.max_cpr > (int64_t)kMaxChunksPerThread * kBlock) return false;
    return g.lds <= kLdsBudget;
}

int knob(int key, int def) { return tune_or(key, def); }

struct CachedPlan {
    int device = 0;              // owner of dev
    void* dev = nullptr;
    void* host = nullptr;
    size_t bytes = 0;
    Geometry g{};
    ResizePlanDev offs{};   // offsets (as pointers) relative to dev
};

std::mutex g_mu;
std::map<std::string, CachedPlan> g_plans;

bool free_plan(CachedPlan& p) {
    const bool a = hipFree(p.dev) == hipSuccess;
    return (hipHostFree(p.host) == hipSuccess) && a;
}

template <typename T>
void put(std::string& k, const T& v) {
    k.append(reinterpret_cast<const char*>(&v), sizeof(v));
}

}  // namespace

int plan_resize(ResizeLaunch& L, hipStream_t stream) {
    const int taps = L.kind == kCubic ? 4 : 2;
    const bool lut = false;  // kernels normalise arithmetically (NormSpec.inv / mul_ok)

    std::string key;
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return VACV_ERR_HIP;
    put(key, device);
    put(key, L.kind); put(key, L.mode); put(key, L.out);
    put(key, L.src.w); put(key, L.src.h); put(key, L.src.cc); put(key, L.src.esize);
    put(key, L.dst.w); put(key, L.dst.h); put(key, L.norm.c_total);

    const int force_h = knob(VACV_TUNE_RESIZE_TILE_H, 0);
    const int force_w = knob(VACV_TUNE_RESIZE_TILE_W, 0);
    const int work = std::max(1, knob(VACV_TUNE_RESIZE_WORK, kWorkPerThread));
    put(key, force_h); put(key, force_w); put(key, work);

    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
        std::vector<Taps> xt(L.dst.w), yt(L.dst.h);
        for (int d = 0; d < L.dst.w; ++d) xt[d] = tap_of(L, d, false);
        for (int d = 0; d < L.dst.h; ++d) yt[d] = tap_of(L, d, true);

        // --- tiling: whole output rows when the staged row is small, row
        // tiles sized for ~8 output elements per thread per task
        const int bp = L.src.cc * L.src.esize;
        int tile_w = L.dst.w;
        Geometry g{};
        bool ok = false;
        if ((int64_t)(L.src.w + taps) * bp > 12288) {
            const double sx = (double)L.src.w / L.dst.w;
            tile_w = std::min(L.dst.w, std::max(64, (int)(8192.0 / (sx * bp)) / 64 * 64));
        }
        if (L.dst.esize == 4) {
            // fp32 output: a tile row is at most kResizeMaxChunksPerLane
            // 4-element chunks per lane (k_resize.hip); split evenly
            const int max_w = std::max(4, (4 * kResizeMaxChunksPerLane * kBlock / L.dst.cc) / 4 * 4);
            if (tile_w > max_w) {
                const int nt = (L.dst.w + max_w - 1) / max_w;
                tile_w = std::min(max_w, ((L.dst.w + nt - 1) / nt + 3) / 4 * 4);
            }
        }
        if (force_w > 0) tile_w = std::min(force_w, L.dst.w);
        for (;;) {
            // work items per output row: 4-pixel groups (byte output) or
            // 4-element chunks (fp32 output), see k_resize.hip
            const int per_row = L.dst.esize == 1 ? (tile_w + 3) / 4 : (tile_w * L.dst.cc + 3) / 4;
            int th = std::max(1, std::min((work * kBlock + per_row - 1) / per_row, 64 / taps));
            if (force_h > 0) th = std::min(force_h, 64 / taps);
            th = std::min(th, L.dst.h);
            for (; th >= 1; --th)
                if (evaluate(L, xt, yt, tile_w, th, g)) { ok = true; break; }
            if (ok || tile_w <= 64) break;
            tile_w = std::max(64, (tile_w / 2) / 64 * 64);
        }
        if (!ok) return VACV_ERR_UNSUPPORTED;

        // --- host image of the plan
        const int xw_sz = L.kind == kLinearFixed ? 4 : (L.kind == kLinearFloat ? 8 : 16);
        const int yw_sz = L.kind == kLinearFixed ? 8 : (L.kind == kLinearFloat ? 8 : 16);
        const int cand_n = g.tile_h * taps;
        size_t off = 0;
        auto take = [&](size_t b) { size_t o = off; off = a16(off + b); return o; };
        const size_t o_xoff = take((size_t)g.tiles_x * g.tile_w * 4);
        const size_t o_xw = take((size_t)g.tiles_x * g.tile_w * xw_sz);
        const size_t o_cf = take((size_t)g.tiles_x * 4);
        const size_t o_cpr = take((size_t)g.tiles_x * 4);
        const size_t o_yrow = take((size_t)L.dst.h * 4);
        const size_t o_yw = take((size_t)L.dst.h * yw_sz);
        const size_t o_tn = take((size_t)g.tiles_y * 4);
        const size_t o_tr = take((size_t)g.tiles_y * g.max_slots * 4);
        const size_t o_tc = take((size_t)g.tiles_y * cand_n * 4);
        const size_t o_tf = take((size_t)g.tiles_y * 4);
        const size_t o_lut = take(lut ? (size_t)L.norm.c_total * 256 * 4 : 16);
        const size_t bytes = off;
        std::vector<unsigned char> img(bytes, 0);
        auto I = [&](size_t o) { return reinterpret_cast<int*>(img.data() + o); };
        auto F = [&](size_t o) { return reinterpret_cast<float*>(img.data() + o); };
        for (int tx = 0; tx < g.tiles_x; ++tx) {
            const int x0 = tx * g.tile_w, nx = std::min(g.tile_w, L.dst.w - x0);
            const int cf = xt[x0].origin;
            I(o_cf)[tx] = cf;
            I(o_cpr)[tx] = ((xt[x0 + nx - 1].origin + taps - 1 - cf + 1) * bp + 30) / 16;
            for (int i = 0; i < nx; ++i) {
                const Taps& t = xt[x0 + i];
                const int e = tx * g.tile_w + i;
                I(o_xoff)[e] = (t.origin - cf) * bp;
                if (L.kind == kLinearFixed) {
                    short* w = reinterpret_cast<short*>(img.data() + o_xw) + 2 * e;
                    w[0] = (short)t.wi[0];
                    w[1] = (short)t.wi[1];
                } else {
                    for (int j = 0; j < taps; ++j) F(o_xw)[taps * e + j] = t.wf[j];
                }
            }
        }
        for (int d = 0; d < L.dst.h; ++d) {
            const Taps& t = yt[d];
            I(o_yrow)[d] = t.origin;
            if (L.kind == kLinearFixed) {
                I(o_yw)[2 * d] = t.wi[0];
                I(o_yw)[2 * d + 1] = t.wi[1];
            } else {
                for (int j = 0; j < taps; ++j) F(o_yw)[(yw_sz / 4) * d + j] = t.wf[j];
            }
        }
        for (int ty = 0; ty < g.tiles_y; ++ty) {
            const int y0 = ty * g.tile_h, ny = std::min(g.tile_h, L.dst.h - y0);
            int* rows = I(o_tr) + (size_t)ty * g.max_slots;
            int* cand = I(o_tc) + (size_t)ty * cand_n;
            for (int c = 0; c < cand_n; ++c) cand[c] = -1;
            int ns = 0;
            if (g.sparse) {
                for (int t = 0; t < ny; ++t)
                    for (int j = 0; j < taps; ++j)
                        if (weight_nonzero(L, yt[y0 + t], j)) {
                            rows[ns] = yt[y0 + t].origin + j;
                            cand[t * taps + j] = ns++;
                        }
            } else {
                const int lo = yt[y0].origin;
                ns = yt[y0 + ny - 1].origin + taps - 1 - lo + 1;
                for (int s = 0; s < ns; ++s) rows[s] = lo + s;
                for (int t = 0; t < ny; ++t)
                    for (int j = 0; j < taps; ++j)
                        if (weight_nonzero(L, yt[y0 + t], j)) cand[t * taps + j] = yt[y0 + t].origin + j - lo;
            }
            I(o_tn)[ty] = ns;
            int flags = 0;
            for (int t = 0; t < ny; ++t)
                for (int j = 0; j < taps; ++j)
                    if (weight_nonzero(L, yt[y0 + t], j)) flags |= 1 << j;
            I(o_tf)[ty] = flags;
        }
        if (lut)
            for (int k = 0; k < L.norm.c_total; ++k)
                for (int v = 0; v < 256; ++v) F(o_lut)[k * 256 + v] = normalize_value((float)v, L.norm.mean[k], L.norm.stdv[k]);

        if (g_plans.size() > 256)  // bounded cache
            (void)evict_device_cache(g_plans, free_plan);
        CachedPlan cp;
        cp.device = device;
        cp.bytes = bytes;
        cp.g = g;
        if (hipHostMalloc(&cp.host, bytes, hipHostMallocDefault) != hipSuccess) return VACV_ERR_NO_MEMORY;
        std::memcpy(cp.host, img.data(), bytes);
        if (hipMalloc(&cp.dev, bytes) != hipSuccess) {
            (void)hipHostFree(cp.host);
            return VACV_ERR_NO_MEMORY;
        }
        // one upload per geometry; synchronised so any stream may use it next
        if (hipMemcpyAsync(cp.dev, cp.host, bytes, hipMemcpyHostToDevice, stream) != hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess) {
            (void)hipFree(cp.dev);
            (void)hipHostFree(cp.host);
            return VACV_ERR_HIP;
        }
        auto P = [&](size_t o) { return reinterpret_cast<const unsigned char*>(cp.dev) + o; };
        cp.offs.xoff = reinterpret_cast<const int*>(P(o_xoff));
        cp.offs.xw = P(o_xw);
        cp.offs.col_first = reinterpret_cast<const int*>(P(o_cf));
        cp.offs.cpr = reinterpret_cast<const int*>(P(o_cpr));
        cp.offs.yrow = reinterpret_cast<const int*>(P(o_yrow));
        cp.offs.yw = P(o_yw);
        cp.offs.task_nslots = reinterpret_cast<const int*>(P(o_tn));
        cp.offs.task_rows = reinterpret_cast<const int*>(P(o_tr));
        cp.offs.task_cand = reinterpret_cast<const int*>(P(o_tc));
        cp.offs.task_flags = reinterpret_cast<const int*>(P(o_tf));
        cp.offs.lut = lut ? reinterpret_cast<const float*>(P(o_lut)) : nullptr;
        it = g_plans.emplace(key, cp).first;
    }
    const CachedPlan& cp = it->second;
    const Geometry& g = cp.g;
    L.tile_w = g.tile_w;
    L.tile_h = g.tile_h;
    L.tiles_x = g.tiles_x;
    L.tiles_y = g.tiles_y;
    L.sparse = g.sparse;
    L.max_slots = g.max_slots;
    L.slot_stride = g.slot_stride;
    L.lds_bytes = g.lds;
    L.plan = cp.offs;
    L.strips = 0;  // set_strips(), once the kernel's residency is known
    return VACV_OK;
}

// Strips: one wave of resident workgroups, each streaming a contiguous run
// of row tiles of one (plane, tile column).  `resident` = workgroups the
// chosen kernel instance fits on the whole device at once (its VGPR and LDS
// use, from the occupancy API): a grid larger than that by a fraction would
// run a mostly idle second round.
void set_strips(ResizeLaunch& L, int64_t resident) {
    const int64_t columns = (int64_t)L.n * L.src.planes * L.tiles_x;
    const int64_t target = knob(VACV_TUNE_RESIZE_WGS, (int)std::max<int64_t>(1, resident));
    const int strips = (int)std::max<int64_t>(1, std::min<int64_t>(L.tiles_y, target / std::max<int64_t>(columns, 1)));
    L.tasks_per_strip = (L.tiles_y + strips - 1) / strips;
    L.strips = (L.tiles_y + L.tasks_per_strip - 1) / L.tasks_per_strip;
}

int release_plans() {
    std::lock_guard<std::mutex> lk(g_mu);
    return evict_device_cache(g_plans, free_plan);
}

}  // namespace vacv
