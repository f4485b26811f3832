// tuning.cpp -- kernel-variant selection knobs (vacv_set_tuning /
// vacv_get_tuning, include/vacv_hip.h).
//
// The launchers read these through vacv::tune(): one array load, no getenv
// on the launch path.  Each knob's initial value comes ONCE, when the library
// is loaded, from an environment variable of the same name (VACV_RESIZE_DIRECT,
// ...) so tools/kbench.py can sweep variants per process; vacv_set_tuning
// changes them at run time (the A/B parity tests).  A value < 0 means "the
// built-in choice" everywhere.
#include <atomic>
#include <cstdlib>

#include "vacv_internal.hpp"

namespace vacv {
namespace {

const char* const kNames[VACV_TUNE_COUNT] = {
    "VACV_RESIZE_DIRECT",      // VACV_TUNE_RESIZE_DIRECT
    "VACV_CUBIC_DIRECT",       // VACV_TUNE_CUBIC_DIRECT
    "VACV_RESIZE_INTERLEAVE",  // VACV_TUNE_RESIZE_INTERLEAVE
    "VACV_DIRECT_XCD",         // VACV_TUNE_DIRECT_XCD
    "VACV_WARP_PX",            // VACV_TUNE_WARP_PX
    "VACV_NEAREST_KERNEL",     // VACV_TUNE_NEAREST_KERNEL
    "VACV_AREA_KERNEL",        // VACV_TUNE_AREA_KERNEL
    "VACV_AREA_ROWS",          // VACV_TUNE_AREA_ROWS
    "VACV_RESIZE_WGS",         // VACV_TUNE_RESIZE_WGS
    "VACV_RESIZE_TILE_H",      // VACV_TUNE_RESIZE_TILE_H
    "VACV_RESIZE_TILE_W",      // VACV_TUNE_RESIZE_TILE_W
    "VACV_RESIZE_WORK",        // VACV_TUNE_RESIZE_WORK
    "VACV_WARP_KERNEL",        // VACV_TUNE_WARP_KERNEL
    "VACV_RESIZE_STRIP",       // VACV_TUNE_RESIZE_STRIP
    "VACV_MATCH_KERNEL",       // VACV_TUNE_MATCH_KERNEL
    "VACV_WARP_FRAMES",        // VACV_TUNE_WARP_FRAMES
    "VACV_WARP_TILE_H",        // VACV_TUNE_WARP_TILE_H
    "VACV_WARP_SLOTS",         // VACV_TUNE_WARP_SLOTS
    "VACV_LANCZOS_KERNEL",     // VACV_TUNE_LANCZOS_KERNEL
};

struct Table {
    std::atomic<int> v[VACV_TUNE_COUNT];
    Table() {
        for (int k = 0; k < VACV_TUNE_COUNT; ++k) {
            const char* e = std::getenv(kNames[k]);
            v[k].store(e && *e ? std::atoi(e) : -1, std::memory_order_relaxed);
        }
    }
};

Table& table() {
    static Table t;  // the environment is read once, at first use
    return t;
}

const int g_init = (table(), 0);  // ... which is library load

}  // namespace

int tune(int key) { return table().v[key].load(std::memory_order_relaxed); }

}  // namespace vacv

extern "C" int vacv_set_tuning(int key, int value) {
    if (key < 0 || key >= VACV_TUNE_COUNT) return VACV_ERR_INVALID_ARG;
    vacv::table().v[key].store(value < 0 ? -1 : value, std::memory_order_relaxed);
    return VACV_OK;
}

extern "C" int vacv_get_tuning(int key) {
    if (key < 0 || key >= VACV_TUNE_COUNT) return VACV_ERR_INVALID_ARG;
    return vacv::tune(key);
}
