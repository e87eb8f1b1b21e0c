// callio.hpp -- per-call bookkeeping handed to the persistent kernels (k_onchip, k_resident, k_wave,
// k_solo, k_solo_fast) so that a simulate call needs no separate launch before its first kernel and
// no copy after its last one (odesat_hip.hip simulate_impl):
//   begin   the launch starts the call: every replica r < B starts active with sat_step -1,
//           steps_done 0 (and dt 0.01 for adaptive steps, system.rs:205) -- what k_begin_call does,
//           except the unsat flags: only the FUSED / TWOPASS step kernels set them and k_status clears
//           them after every step, so they are zero between calls whichever path ran -- without
//           reading the bookkeeping; one thread per replica stores those values first, so a workgroup
//           that returns early (padding replicas) leaves them too (test_call_sequences_fold_and_mirror_match_fused
//           continues a folded call on FUSED);
//   h_sat / h_done / h_dt   host-mapped pinned mirrors of sat_step, steps_done and dt: every replica's
//           epilogue also stores its final values there (used on STOP_NONE calls, where every real
//           replica runs every launch to its epilogue; finish_simulate then reads them directly).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

struct CallIO {
    int64_t *h_sat = nullptr, *h_done = nullptr;
    void *h_dt = nullptr;
    int32_t begin = 0, B = 0;
};

__device__ __forceinline__ bool io_active(const CallIO &io, const uint8_t *act, int g) {
    return io.begin ? g < io.B : act[g] != 0;
}
__device__ __forceinline__ int64_t io_sat(const CallIO &io, const int64_t *sat, int g) { return io.begin ? -1 : sat[g]; }
__device__ __forceinline__ int64_t io_done(const CallIO &io, const int64_t *done, int g) { return io.begin ? 0 : done[g]; }
template <typename T> __device__ __forceinline__ T io_dt(const CallIO &io, const T *dtr, int g) {
    return io.begin ? (T)0.01 : dtr[g];
}
// by ONE thread per replica g, before any early return
template <typename T>
__device__ __forceinline__ void io_begin_store(const CallIO &io, int g, uint8_t *act, int64_t *sat, int64_t *done,
                                               T *dtr, bool adaptive, int32_t *stop) {
    if (!io.begin) return;
    act[g] = g < io.B ? 1 : 0;
    sat[g] = -1;
    done[g] = 0;
    if (adaptive) dtr[g] = (T)0.01;
    if (g == 0) *stop = INT_MAX;
}
template <typename T>
__device__ __forceinline__ void io_mirror(const CallIO &io, int g, int64_t sat, int64_t done, T dtr, bool adaptive) {
    if (!io.h_sat) return;
    io.h_sat[g] = sat;
    io.h_done[g] = done;
    if (adaptive) reinterpret_cast<T *>(io.h_dt)[g] = dtr;
}
