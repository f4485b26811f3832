#include "perf_util.h"

AutoPerf::AutoPerf(double& duration) : _duration(&duration), _start(std::chrono::steady_clock::now()) {}

AutoPerf::~AutoPerf() {
    if (_duration)
        *_duration = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - _start).count();
}
