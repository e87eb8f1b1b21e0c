// devattr.hpp -- one-time, thread-safe hipFuncSetAttribute(MaxDynamicSharedMemorySize) per
// (device, kernel).  The attribute belongs to the kernel on the device that is current when it is
// set, so a process-wide "already set" flag is wrong twice over: two host threads race on it, and
// a solver on a second device never gets the attribute (its launches with more than 64 KiB of
// dynamic LDS then fail).  include/odesat.h allows one solver per GPU driven from its own thread.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <tuple>

namespace odesat {

inline hipError_t ensure_max_lds(const void *fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    static std::mutex mu;
    static std::set<std::tuple<int, const void *, int>> done;
    const auto key = std::make_tuple(dev, fn, bytes);
    std::lock_guard<std::mutex> lk(mu);
    if (done.count(key)) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.insert(key);
    return e;
}

}  // namespace odesat
