// k_resize_strip.hip -- u8 bilinear resize (all three fixed-point modes, u8 /
// fp32 / normalised-fp32 out) for geometries whose output rows weight TWO
// source rows (e.g. 1080p -> 1280x720), as column strips walking down an image.
//
// Reference arithmetic: the same as resize_direct_kernel (k_resize_direct.hip):
// fixed_tap() taps (resize_naive.cpp:19-45 / resize_neon.cpp:17-78) and
// blend_fixed<MODE> (resize_naive.cpp:61-64 / resize_neon.cpp:103-167).
//
// Why.  A source row of a two-tap geometry feeds ~1.33 output rows; the staged
// and gather kernels compute those output rows in different workgroups, often
// on different XCDs, so the row is fetched into L2 more than once and every
// workgroup pays its own latency.  Here a workgroup owns an SW-column output
// strip of one plane and walks down its rows, keeping the source rows in an
// LDS ring: every source byte of the strip leaves HBM once.
//  * The ring holds the source rows of two batches (slot = row mod ring).
//  * Batches of BR output rows; the source rows a batch adds to the ring are
//    loaded with
//    coalesced 16-byte loads into registers while the previous batch is being
//    blended (one barrier per batch).
//  * Lane l takes output columns ox0 + l + 64q: its horizontal taps and its byte
//    offset in a ring row are computed once; a row's vertical taps are
//    wave-uniform.  Per pixel: two (CC <= 2) or three dword LDS reads per tap
//    row, v_alignbyte, the packed-u16 dot products of resize_direct_kernel.
//  * u8 output: the lane quads' bytes are packed (DPP) into 4*CC-byte stores;
//    fp32: CC floats per lane, lane-contiguous.
#pragma clang fp contract(off)

#include <algorithm>
#include <cmath>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kFetchIters = 3;    // 16-byte chunks per thread and batch
constexpr int kOobOff = (int)0x80000000;  // a buffer offset past every plane: loads read 0, stores drop
constexpr int kMaxLds = 64 * 1024;
// cache policy of the strip loads: the default (0), not non-temporal.  The
// 16-byte chunks at a strip's edges share 128-byte lines with the
// neighbouring strips, which run at the same time on the same XCD (the
// workgroup order below); kept in L2 they are fetched from HBM once.  1080p
// -> 1280x720 u8, 256 frames: 0.551 ms nt (aux 2 or 3) -> 0.491 ms (0 or sc0).
// EXTRA=-DVACV_STRIP_AUX=n for A/B builds.
#ifndef VACV_STRIP_AUX
#define VACV_STRIP_AUX 0
#endif
// cache policy of the output stores (A/B builds: EXTRA=-DVACV_STRIP_SAUX=n)
#ifndef VACV_STRIP_SAUX
#define VACV_STRIP_SAUX VACV_STORE_AUX
#endif

// one output pixel (lane-quad packed for u8) at row byte offset row_off.
// Every store is issued (an offset past the plane where a lane has nothing to
// write: the store is dropped), so each path through a batch issues a fixed
// number of stores and the compiler's wait for the next batch's loads (park)
// is a counted vmcnt that leaves them in flight.  u8: the lane quad's dword
// store always; the CC byte stores of partial quads only in strips that have
// them (a uniform branch: every path still holds the dword stores).
constexpr uint32_t kOobStore = 0x80000000u;  // a lane offset (voffset) past the plane: the store is dropped

// blend_fixed with the value in bits 24..31 of the result (the bits below are
// not zero).  In the reference mode the row weights come times 4 (kRowW4: the
// row table holds them so), so the sum (tl*a0 + tr*a1)*4wA + (bl*a0 + br*a1)*4wB
// is the reference's int32 sum << 2 (<= 255*2049^2*4 < 2^32; every 24-bit
// multiply exact) and its top byte is sum >> 22: a pixel's channels pack with
// two v_perm, fp32 converts from the top byte (no shift, no mask)
template <int MODE>
constexpr uint32_t kRowW4 = MODE == VACV_LINEAR_REFERENCE ? 4u : 1u;
template <int MODE>
__device__ __forceinline__ uint32_t blend_fixed_hi(uint32_t top, uint32_t bot, us2 wx, uint32_t wA, uint32_t wB) {
    if constexpr (MODE == VACV_LINEAR_REFERENCE) {
        const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
        const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false);
        return __umul24(ht, wA) + __umul24(hb, wB);
    } else {
        return (uint32_t)blend_fixed<MODE>(top, bot, wx, wA, wB) << 24;
    }
}

// the channels' values (bits 24..31 of vh[k]) as the pixel's CC bytes
template <int CC>
__device__ __forceinline__ uint32_t pack_hi(const uint32_t (&vh)[CC]) {
    if constexpr (CC == 1) return vh[0] >> 24;
    else if constexpr (CC == 2) return __builtin_amdgcn_perm(vh[1], vh[0], 0x0C0C0703u);
    else if constexpr (CC == 3)
        return __builtin_amdgcn_perm(vh[2], __builtin_amdgcn_perm(vh[1], vh[0], 0x0C0C0703u), 0x0C070100u);
    else
        return __builtin_amdgcn_perm(__builtin_amdgcn_perm(vh[3], vh[2], 0x0C0C0703u),
                                     __builtin_amdgcn_perm(vh[1], vh[0], 0x0C0C0703u), 0x05040100u);
}

template <int CC, int OUT>
__device__ __forceinline__ void store_pixel(const uint32_t (&vh)[CC], const ChanNorm (&cn)[CC], const Rsrc& drs,
                                            uint32_t row_off, int ox, int qx, int W, bool quad_full, bool strip_full,
                                            int lane) {
    if constexpr (OUT == kOutSame) {
        const uint32_t own = pack_hi<CC>(vh);
        const uint32_t word = quad_pack<CC>(own, lane & 3);
        const bool wq = quad_full && (lane & 3) < CC;
        // the row's offset (uniform) as soffset, the lane's (fixed per strip) as
        // voffset (never out of range as a soffset: it is not range-checked)
        __builtin_amdgcn_raw_buffer_store_b32(word, drs.r, (int)(wq ? (uint32_t)(qx * CC + 4 * (lane & 3)) : kOobStore),
                                              (int)row_off, VACV_STRIP_SAUX);
        if (!strip_full) {  // uniform: the partial quads' bytes
            const bool wb = !quad_full && ox < W;
#pragma unroll
            for (int k = 0; k < CC; ++k)
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(own >> (8 * k)), drs.r,
                                                     (int)(wb ? (uint32_t)(ox * CC + k) : kOobStore), (int)row_off,
                                                     VACV_STRIP_SAUX);
        }
    } else {
        uint32_t f[CC];
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            const int v = (int)(vh[k] >> 24);
            f[k] = __builtin_bit_cast(uint32_t, OUT == kOutF32 ? (float)v : normalize_u8v(cn[k], v));
        }
        // the row in voffset here, soffset 0: with a register soffset the
        // compiler leaves out the wait between a store of more than 8 bytes
        // and a VALU write of its data registers, and on gfx950 the next
        // instruction then overwrote the third dword before it was stored
        const int off = (int)(ox < W ? row_off + (uint32_t)(ox * CC * 4) : kOobStore);
        const int soff = 0;
        if constexpr (CC == 1) {
            __builtin_amdgcn_raw_buffer_store_b32(f[0], drs.r, off, soff, VACV_STRIP_SAUX);
        } else if constexpr (CC == 2) {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{f[0], f[1]}, drs.r, off, soff, VACV_STRIP_SAUX);
        } else if constexpr (CC == 3) {
            typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
            __builtin_amdgcn_raw_buffer_store_b96(u32x3{f[0], f[1], f[2]}, drs.r, off, soff, VACV_STRIP_SAUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{f[0], f[1], f[2], f[3]}, drs.r, off, soff, VACV_STRIP_SAUX);
        }
    }
}

// SW output columns per workgroup (SW / 64 per lane), BR output rows per batch
template <int CC, int OUT, int MODE, int SW, int BR>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OUT == kOutSame ? 8 : 6)))
resize_strip_kernel(ResizeLaunch L, int strips_x, int groups, int rows_per_group, int ring, int stride, int dst_al,
                    int total) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, and said so
    // XCD-contiguous order: neighbouring strips share the 128-byte lines at
    // their edges; on one XCD those come from one L2
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;  // uniform
    const int per_plane = strips_x * groups;
    const int pidx = id / per_plane;
    const int rem = id - pidx * per_plane;
    const int grp = rem / strips_x, sxi = rem - grp * strips_x;
    const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
    const int W = L.dst.w, H = L.dst.h;
    const int oy_begin = grp * rows_per_group, oy_end = min(oy_begin + rows_per_group, H);
    constexpr int PXL = SW / 64;
    const int ox0 = sxi * SW;

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t lim = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp = (uint32_t)L.src.row_pitch;  // % 16 == 0 (host)

    // ---- the strip's source columns and the lane's taps -----------------------
    const int xs0 = tap_of<MODE>(ox0, L.src.w, W, L.scale_xf, L.scale_xd).i;  // uniform
    const int xs1 = tap_of<MODE>(min(ox0 + SW, W) - 1, L.src.w, W, L.scale_xf, L.scale_xd).i + 1;
    const uint32_t col0 = (uint32_t)(xs0 * CC) + srs.delta;  // strip's first byte within a row (from base16)
    const uint32_t dxb = col0 & 15u;                          // ... within its chunk (every row: rp % 16 == 0)
    const int chunks = (int)((dxb + (uint32_t)(xs1 - xs0 + 1) * CC + 15u) >> 4);
    int oxv[PXL];
    uint32_t lo4[PXL], sh[PXL], wxv[PXL];  // the lane's taps in a ring row, its horizontal weights
#pragma unroll
    for (int q = 0; q < PXL; ++q) {
        oxv[q] = ox0 + 64 * q + lane;
        const FixedTap tx = tap_of<MODE>(min(oxv[q], W - 1), L.src.w, W, L.scale_xf, L.scale_xd);
        const uint32_t lo = (uint32_t)((tx.i - xs0) * CC) + dxb;
        lo4[q] = lo & ~3u;
        sh[q] = lo & 3u;
        wxv[q] = (uint32_t)tx.w0 | ((uint32_t)tx.w1 << 16);
    }

    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const Rsrc drs = make_rsrc(dp, L.dst.plane_bytes);  // 32-bit store offsets
    constexpr int kTD = (int)kTapDwords<CC, true>;

    // ---- ring fill: source rows (next_row .. hi] --------------------------------
    // ring slot of source row r: r mod ring (exact: r < 2^16, ring < 2^8)
    const uint32_t rmagic = (uint32_t)((0x100000000ull + (uint64_t)ring - 1) / (uint64_t)ring);
    auto slot = [&](uint32_t r) { return r - (uint32_t)ring * __umulhi(r, rmagic); };
    // chunk u*kBlock + tid of a fill is (row rcu[u] >> 16, chunk rcu[u] & 0xFFFF)
    // of the rows being added, whatever the fill: the division happens once
    uint32_t rcu[kFetchIters];
    {
        const uint32_t magic = (uint32_t)((0x100000000ull + (uint64_t)chunks - 1) / (uint64_t)chunks);
#pragma unroll
        for (int u = 0; u < kFetchIters; ++u) {
            const uint32_t i = (uint32_t)(u * kBlock + tid);
            const uint32_t rr = chunks == 1 ? i : __umulhi(i, magic);  // i / chunks, exact (i < 2^12)
            rcu[u] = (rr << 16) | (i - rr * (uint32_t)chunks);
        }
    }
    uint4 pre[kFetchIters];
    uint32_t dst_off[kFetchIters], tail_o[kFetchIters];
    uint32_t tailm = 0;
    // every fetch issues all kFetchIters loads (chunks beyond the rows being
    // added read out of range: zeros, no fault; a chunk straddling the plane's
    // end likewise, assembled bytewise in park()), so the loads are
    // unconditional and the compiler can count them: park() then waits for
    // the loads only, not for the blend's stores issued after them.
    // per thread and chunk u, what no fill changes: the chunk's byte offset
    // from its row's strip start (rp % 16 == 0: (r rp + col0) & ~15 =
    // r rp + (col0 & ~15)), its row within the fill, its column in a ring row
    uint32_t koff[kFetchIters];
#pragma unroll
    for (int u = 0; u < kFetchIters; ++u)
        koff[u] = (rcu[u] >> 16) * rp + (col0 & ~15u) + 16u * (rcu[u] & 0xFFFFu);
    auto fetch = [&](int r_first, int r_last) {
        const uint32_t nrows = (uint32_t)max(r_last - r_first + 1, 0);
        const uint32_t obase = (uint32_t)r_first * rp;  // uniform
        const uint32_t s0 = slot((uint32_t)r_first);    // uniform
        tailm = 0;
#pragma unroll
        for (int u = 0; u < kFetchIters; ++u) {
            const uint32_t rr = rcu[u] >> 16, c = rcu[u] & 0xFFFFu;
            const uint32_t o = obase + koff[u];
            const bool live = rr < nrows;
            const bool tail = live && o + 16u > lim;
            uint32_t sl = s0 + rr;  // (r_first + rr) mod ring: rr < ring
            sl = sl >= (uint32_t)ring ? sl - (uint32_t)ring : sl;
            dst_off[u] = live ? sl * (uint32_t)stride + 16u * c : 0xFFFFFFFFu;
            tail_o[u] = o;
            tailm |= tail ? 1u << u : 0u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)(live && !tail ? o : kOobOff), 0,
                                                                 VACV_STRIP_AUX);
            pre[u] = *reinterpret_cast<const uint4*>(&v);
        }
    };
    auto park = [&]() {
        if (tailm) {  // the plane's last chunk: a straddling 16-byte load reads as zeros
#pragma unroll
            for (int u = 0; u < kFetchIters; ++u) {
                if ((tailm >> u) & 1u) {
                    uint32_t d[4] = {0u, 0u, 0u, 0u};
#pragma unroll 1
                    for (uint32_t e = 0; e < 16u; ++e)
                        if (tail_o[u] + e < lim)
                            d[e >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(tail_o[u] + e), 0, 0)
                                         << (8 * (e & 3));
                    pre[u] = make_uint4(d[0], d[1], d[2], d[3]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kFetchIters; ++u)
            if (dst_off[u] != 0xFFFFFFFFu) *reinterpret_cast<uint4*>(lds + dst_off[u]) = pre[u];
    };
    auto rows_of = [&](int b, int& lo_row, int& hi_row) {  // source rows batch b reads
        const int y0 = oy_begin + b * BR, y1 = min(y0 + BR, oy_end) - 1;
        lo_row = tap_of<MODE>(y0, L.src.h, H, L.scale_yf, L.scale_yd).i;
        hi_row = tap_of<MODE>(y1, L.src.h, H, L.scale_yf, L.scale_yd).i + 1;  // <= h - 1 (linear_tap)
    };

    // a batch's vertical taps, computed once per workgroup (lanes 0 .. BR - 1
    // of wave 0) into a table after the ring, one per batch parity: per row
    // the ring offsets of its two source rows and its weight pair (16 bytes).
    // Each wave computing its own rows' taps cost ~25 VALU per output row.
    unsigned char* rtab = lds + ring * stride + 16;
    auto put_rows = [&](int b) {
        if (tid < BR) {
            const int oy = min(oy_begin + b * BR + tid, oy_end - 1);  // rows past the group: its last
            const FixedTap ty = tap_of<MODE>(oy, L.src.h, H, L.scale_yf, L.scale_yd);
            *reinterpret_cast<uint4*>(rtab + ((b & 1) * BR + tid) * 16) =
                make_uint4(slot((uint32_t)ty.i) * (uint32_t)stride, slot((uint32_t)ty.i + 1u) * (uint32_t)stride,
                           kRowW4<MODE> * ((uint32_t)ty.w0 | ((uint32_t)ty.w1 << 16)), 0u);
        }
    };

    // uniform: every lane quad of the strip whole, the destination dword-aligned
    const bool strip_full = ox0 + SW <= W && dst_al;
    const int batches = (oy_end - oy_begin + BR - 1) / BR;
    if (batches <= 0) return;  // uniform
    int lo_row, hi_row;
    rows_of(0, lo_row, hi_row);
    fetch(lo_row, hi_row);
    put_rows(0);
    park();
    int loaded = hi_row;
    // park() of batch b + 1 sits at the END of iteration b, after its blend:
    // on every path into it the blend's stores follow the loads, so its wait
    // leaves them in flight (at the top of the loop, the path from the
    // prologue -- no stores -- made it a vmcnt(0) for every batch)
    for (int b = 0; b < batches; ++b) {
        __syncthreads();  // batch b's rows and taps are in LDS; batch b - 1's reads are done
        const bool more = b + 1 < batches;  // uniform
        if (more) {  // the next batch's new rows, in flight while this one blends
            int l1, h1;
            rows_of(b + 1, l1, h1);
            fetch(max(l1, loaded + 1), h1);
            loaded = max(loaded, h1);
            put_rows(b + 1);
        }
        // ---- blend: wave w takes rows w, w + 4, ... of the batch, 2 at a time ---
#pragma unroll
        for (int g = 0; g < BR / 8; ++g) {
            uint32_t wyv[2], ra[2], rb[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint4 e = *reinterpret_cast<const uint4*>(rtab + ((b & 1) * BR + 8 * g + wave + 4 * j) * 16);
                ra[j] = __builtin_amdgcn_readfirstlane(e.x);  // wave-uniform
                rb[j] = __builtin_amdgcn_readfirstlane(e.y);
                wyv[j] = __builtin_amdgcn_readfirstlane(e.z);
            }
#pragma unroll
            for (int q = 0; q < PXL; ++q) {
                uint32_t t0[2][3], t1[2][3];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t* pa = reinterpret_cast<const uint32_t*>(lds + ra[j] + lo4[q]);
                    const uint32_t* pb = reinterpret_cast<const uint32_t*>(lds + rb[j] + lo4[q]);
#pragma unroll
                    for (int d = 0; d < kTD; ++d) { t0[j][d] = pa[d]; t1[j][d] = pb[d]; }
                }
                const int ox = oxv[q];
                const int qx = ox0 + 64 * q + (lane & ~3);
                const bool quad_full = qx + 4 <= W && dst_al;
                const us2 wx = __builtin_bit_cast(us2, wxv[q]);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int oy = oy_begin + b * BR + 8 * g + wave + 4 * j;
                    const uint32_t a0 = __builtin_amdgcn_alignbyte(t0[j][1], t0[j][0], sh[q]);
                    const uint32_t c0 = __builtin_amdgcn_alignbyte(t1[j][1], t1[j][0], sh[q]);
                    uint32_t a1 = 0u, c1 = 0u;
                    if constexpr (kTD == 3) {
                        a1 = __builtin_amdgcn_alignbyte(t0[j][2], t0[j][1], sh[q]);
                        c1 = __builtin_amdgcn_alignbyte(t1[j][2], t1[j][1], sh[q]);
                    }
                    const uint32_t wA = wyv[j] & 0xFFFFu, wB = wyv[j] >> 16;
                    uint32_t v[CC];
#pragma unroll
                    for (int k = 0; k < CC; ++k) {
                        const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24);
                        v[k] = blend_fixed_hi<MODE>(__builtin_amdgcn_perm(a1, a0, sel), __builtin_amdgcn_perm(c1, c0, sel),
                                                    wx, wA, wB);
                    }
                    // rows past the group (its last batch) repeat the group's last
                    // row (put_rows), value for value: the soffset of a buffer
                    // store is not range-checked, so it always names a real row
                    const uint32_t row_off = (uint32_t)min(oy, oy_end - 1) * (uint32_t)L.dst.row_pitch + drs.delta;
                    store_pixel<CC, OUT>(v, cn, drs, row_off, ox, qx, W, quad_full, strip_full, lane);
                }
            }
        }
        if (more) park();
    }
}

struct StripPlan {
    int strips_x, groups, rows_per_group, ring, stride, lds, sw, br;
};

// The ring (a power of two holding two batches' source rows) and the row
// stride (a strip's source bytes plus the worst chunk offset), or false when
// the strip kernel does not apply.
bool strip_plan_w(const ResizeLaunch& L, StripPlan& p, bool wide) {
    if (L.kind != kLinearFixed || L.src.esize != 1 || L.src.cc < 1 || L.src.cc > 4) return false;
    if (L.src.row_pitch % 16) return false;
    if (L.dst.w >= (1 << 23) || L.dst.h >= (1 << 23)) return false;
    const int cc = L.src.cc;
    const double sx = L.scale_xd, sy = L.scale_yd;
    p.sw = wide ? 128 : 64;
    p.br = wide ? 8 : 16;
    const int span = (int)std::ceil((p.sw - 1) * sx) + 3;  // source columns of a strip, + taps and slack
    const int chunks = (15 + span * cc + 15) / 16;
    const int batch_rows = (int)std::ceil(p.br * sy) + 3;  // source rows one batch can add
    if ((int64_t)batch_rows * chunks > (int64_t)kFetchIters * kBlock) return false;
    const int ring = 2 * batch_rows + 2;  // rows of two batches (any size: the slot is r mod ring)
    if (ring >= 256 || L.src.h >= (1 << 16)) return false;
    p.stride = chunks * 16;
    p.ring = ring;
    p.lds = ring * p.stride + 16 + 2 * p.br * 16;  // + the last tap dword's overhang, the row-tap tables
    if (p.lds > kMaxLds) return false;
    p.strips_x = (L.dst.w + p.sw - 1) / p.sw;
    // enough workgroups for the chip: split the rows until there are >= 8192
    // (~4 rounds of the 2,048 resident at 64-column strips), so the last round's
    // partial occupancy is a small part of the run (256 x 1080p -> 1280x720:
    // 5,120 whole-height strips are 2.5 rounds, the last half-empty)
    const int64_t strips = (int64_t)p.strips_x * L.n * L.src.planes;
    p.groups = 1;
    while (strips * p.groups < 8192 && L.dst.h / (p.groups * 2) >= 4 * p.br) p.groups *= 2;
    p.rows_per_group = (L.dst.h + p.groups - 1) / p.groups;
    return strips * p.groups < 0x7FFFFFF0LL;
}

// 1: 64-column strips, 16-row batches; 2: 128 columns, 8 rows.  By default
// 128 where their fetch fits, else 64 (round 6: with >= 8,192 workgroups the
// 128-column strips' 600-byte row segments beat the 64-column ones' 300:
// 1080p -> 1280x720 u8 0.4687 -> 0.4635 ms, normalised 0.8758 -> 0.8723)
bool strip_plan(const ResizeLaunch& L, StripPlan& p) {
    const int v = tune(VACV_TUNE_RESIZE_STRIP);
    if (v == 1 || v == 2) return strip_plan_w(L, p, v == 2);
    return strip_plan_w(L, p, true) || strip_plan_w(L, p, false);
}

template <int CC, int OUT, int MODE>
hipError_t launch_one(const ResizeLaunch& L, const StripPlan& p, hipStream_t s) {
    const int64_t total = (int64_t)p.strips_x * p.groups * L.n * L.src.planes;
    const int64_t blocks = (total + 7) / 8 * 8;
    const int64_t out_align = OUT == kOutSame ? 4 : 4;
    const int dst_al = !(L.dst.row_pitch % out_align || L.dst.img_pitch % out_align || L.dst.plane_pitch % out_align ||
                         reinterpret_cast<uintptr_t>(L.dst.base) % out_align);
    if (p.sw == 128)
        hipLaunchKernelGGL((resize_strip_kernel<CC, OUT, MODE, 128, 8>), dim3((unsigned)blocks), dim3(kBlock), p.lds, s, L,
                           p.strips_x, p.groups, p.rows_per_group, p.ring, p.stride, dst_al, (int)total);
    else
        hipLaunchKernelGGL((resize_strip_kernel<CC, OUT, MODE, 64, 16>), dim3((unsigned)blocks), dim3(kBlock), p.lds, s, L,
                           p.strips_x, p.groups, p.rows_per_group, p.ring, p.stride, dst_al, (int)total);
    return hipGetLastError();
}

template <int OUT, int MODE>
hipError_t launch_cc(const ResizeLaunch& L, const StripPlan& p, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<1, OUT, MODE>(L, p, s);
        case 2: return launch_one<2, OUT, MODE>(L, p, s);
        case 3: return launch_one<3, OUT, MODE>(L, p, s);
        case 4: return launch_one<4, OUT, MODE>(L, p, s);
        default: return hipErrorInvalidValue;
    }
}

template <int OUT>
hipError_t launch_mode(const ResizeLaunch& L, const StripPlan& p, hipStream_t s) {
    switch (L.mode) {
        case VACV_LINEAR_REFERENCE: return launch_cc<OUT, VACV_LINEAR_REFERENCE>(L, p, s);
        case VACV_LINEAR_NEON: return launch_cc<OUT, VACV_LINEAR_NEON>(L, p, s);
        case VACV_LINEAR_OPENCV: return launch_cc<OUT, VACV_LINEAR_OPENCV>(L, p, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool resize_strip_applies(const ResizeLaunch& L) {
    StripPlan p;
    return strip_plan(L, p);
}

hipError_t launch_resize_strip(const ResizeLaunch& L, hipStream_t s) {
    StripPlan p;
    if (!strip_plan(L, p)) return hipErrorInvalidValue;
    if (L.out == kOutSame) return launch_mode<kOutSame>(L, p, s);
    if (L.out == kOutF32) return launch_mode<kOutF32>(L, p, s);
    return launch_mode<kOutNorm>(L, p, s);
}

}  // namespace vacv
