// wave_k.hip -- the k_wave / k_solo / k_solo_fast kernels (wave.hpp) in a translation unit of their
// own, so they can be built with the max-ILP machine scheduler (Makefile WAVE_FLAGS) while the rest of
// odesat_hip.hip keeps the default one (the scheduler helps these kernels and slows
// k_resident and k_step).  odesat_hip.hip's launch_wave_k / launch_solo_k call the two functions
// below; every shape they dispatch is instantiated at the end.
#include <hip/hip_runtime.h>

#define ODK_NO_COMMON_KERNELS  // kernels.hpp's non-template kernels live in odesat_hip.hip
#include "devattr.hpp"
#include "wave.hpp"

namespace odk {

template <typename T, bool ADA, int WPW, int TW, bool FAST>
hipError_t wave_launch(bool prep, const WArgs<T> &a, unsigned grid, unsigned block, size_t lds, int lds_max,
                       hipStream_t st) {
    if (prep) return odesat::ensure_max_lds(reinterpret_cast<const void *>(&k_wave<T, ADA, WPW, TW, FAST>), lds_max);
    hipLaunchKernelGGL((k_wave<T, ADA, WPW, TW, FAST>), dim3(grid), dim3(block), lds, st, a);
    return hipGetLastError();
}

template <typename T, bool ADA, int CPL, int VPL, bool FAST>
hipError_t solo_launch(bool prep, const WArgs<T> &a, unsigned grid, unsigned block, size_t lds, int lds_max,
                       hipStream_t st) {
    if constexpr (FAST) {
        if (prep) return odesat::ensure_max_lds(reinterpret_cast<const void *>(&k_solo_fast<T, ADA, CPL, VPL>), lds_max);
        hipLaunchKernelGGL((k_solo_fast<T, ADA, CPL, VPL>), dim3(grid), dim3(block), lds, st, a);
    } else {
        if (prep) return odesat::ensure_max_lds(reinterpret_cast<const void *>(&k_solo<T, ADA, CPL, VPL>), lds_max);
        hipLaunchKernelGGL((k_solo<T, ADA, CPL, VPL>), dim3(grid), dim3(block), lds, st, a);
    }
    return hipGetLastError();
}

template <typename T, bool ADA, int CPL, int VPL>
hipError_t solo_cv_launch(bool prep, const WArgs<T> &a, unsigned grid, unsigned block, size_t lds, int lds_max,
                          hipStream_t st) {
    if (prep) return odesat::ensure_max_lds(reinterpret_cast<const void *>(&k_solo_cv<T, ADA, CPL, VPL>), lds_max);
    hipLaunchKernelGGL((k_solo_cv<T, ADA, CPL, VPL>), dim3(grid), dim3(block), lds, st, a);
    return hipGetLastError();
}

// the shapes odesat_hip.hip's launch_wave / launch_resident dispatch: (replicas per workgroup, waves per
// replica) for k_wave, (clause slots, variable slots per lane) for k_solo, each in f32 / f64, fixed /
// adaptive, general / short forms
#define WAVE_ONE(T, A, W, TW, F)                                                                          \
    template hipError_t wave_launch<T, A, W, TW, F>(bool, const WArgs<T> &, unsigned, unsigned, size_t, int, \
                                                    hipStream_t);
#define WAVE_TF(T, W, TW) WAVE_ONE(T, false, W, TW, false) WAVE_ONE(T, false, W, TW, true) \
    WAVE_ONE(T, true, W, TW, false) WAVE_ONE(T, true, W, TW, true)
#define WAVE_SHAPES(T) WAVE_TF(T, 4, 1) WAVE_TF(T, 4, 2) WAVE_TF(T, 4, 4) WAVE_TF(T, 2, 1) WAVE_TF(T, 2, 2) \
    WAVE_TF(T, 2, 4) WAVE_TF(T, 2, 8) WAVE_TF(T, 1, 1) WAVE_TF(T, 1, 2) WAVE_TF(T, 1, 4) WAVE_TF(T, 1, 8)  \
    WAVE_TF(T, 1, 16)
WAVE_SHAPES(float)
WAVE_SHAPES(double)

#define SOLO_ONE(T, A, C, V, F)                                                                           \
    template hipError_t solo_launch<T, A, C, V, F>(bool, const WArgs<T> &, unsigned, unsigned, size_t, int,   \
                                                   hipStream_t);
#define SOLO_TF(T, C, V) SOLO_ONE(T, false, C, V, false) SOLO_ONE(T, false, C, V, true) \
    SOLO_ONE(T, true, C, V, false) SOLO_ONE(T, true, C, V, true)
#define SOLO_SHAPES(T) SOLO_TF(T, 1, 1) SOLO_TF(T, 1, 2) SOLO_TF(T, 2, 1) SOLO_TF(T, 2, 2) SOLO_TF(T, 4, 1) \
    SOLO_TF(T, 4, 2)
SOLO_SHAPES(float)
SOLO_SHAPES(double)

#define SOLO_CV_ONE(T, A, C, V)                                                                          \
    template hipError_t solo_cv_launch<T, A, C, V>(bool, const WArgs<T> &, unsigned, unsigned, size_t, int, \
                                                   hipStream_t);
#define SOLO_CV_FA(T, C, V) SOLO_CV_ONE(T, false, C, V) SOLO_CV_ONE(T, true, C, V)
#define SOLO_CV_SHAPES(T) SOLO_CV_FA(T, 1, 0) SOLO_CV_FA(T, 1, 1) SOLO_CV_FA(T, 1, 2) SOLO_CV_FA(T, 2, 0) \
    SOLO_CV_FA(T, 2, 1) SOLO_CV_FA(T, 2, 2)
SOLO_CV_SHAPES(float)
SOLO_CV_SHAPES(double)

}  // namespace odk
