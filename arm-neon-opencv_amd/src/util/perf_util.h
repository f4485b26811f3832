// AutoPerf / TIME_PERF -- scoped timer of the reference harness
// (src/util/perf_util.h).  The reference reads clock() (process CPU time);
// a GPU operator mostly waits, so this measures wall time (steady_clock)
// instead.  Result in milliseconds, written when the scope ends.
#ifndef PERF_UTIL_H
#define PERF_UTIL_H

#include <chrono>

#define TIME_PERF(duration) AutoPerf perf(duration)

class AutoPerf {
public:
    explicit AutoPerf(double& duration);
    ~AutoPerf();

private:
    double* _duration;
    std::chrono::steady_clock::time_point _start;
};

#endif  // PERF_UTIL_H
