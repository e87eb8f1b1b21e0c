// odesat_hip.hip -- MI355X (gfx950) integrator for the Bearden-Pei-Di Ventra memcomputing ODE:
// the replacement of /root/reference/src/system.rs:25-359 behind the C ABI of include/odesat.h.
//
// Device layout.  Every per-item array (item = variable or clause) is
// replica-innermost in groups of W replicas:  X[g][item][W],  replica r = g*W + j.
// A wave covers one "row": LW lanes per item, VEC contiguous replicas per lane, W = LW*VEC.
//   * batches >= 256 (f32) / >= 128 (f64):  LW = 64, VEC = 16 B / sizeof(T): one wave = the
//     W replicas of ONE clause / variable, every state access is a 1 KiB dwordx4 wave-load, literal
//     indices are wave-uniform scalar loads;
//   * 128 <= B < 256 (f32): LW = 64, VEC = 2; 64 <= B < 128: LW = 64, VEC = 1;
//   * B < 64: LW = next pow2 >= B, VEC = 1: a wave spans 64/LW items.
// One Euler step = two kernels per replica chunk + one status kernel:
//   k_clause   (system.rs:35-90)   per clause: gather the literal voltages, strict-< min/second-min,
//              C, G, R, the per-literal dv contribution, dxs/dxl, the fused update_state of xs/xl
//              (system.rs:94-95) and the per-replica "some clause unsat" flag.  The contribution of
//              slot s is stored at w[g][wpos[s]][W]: slots are laid out variable-major (each
//              variable's slots sorted by clause, then literal position).
//   k_variable (system.rs:80,96)   per variable: dv = 0 + w[..] summed over its slots in that
//              order -- exactly the reference's sequential scatter order, so f32 and f64 results are
//              bit-identical to the CPU oracle -- then the clamped v update.  No atomics.
//   k_status   (system.rs:149-153, 122-136, 190-235, 291) per replica: sat bookkeeping, stop
//              policy, adaptive dt.
// FP contraction is OFF: every + and * rounds exactly as written in system.rs, in the solver dtype.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"

using odesat::fail;

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(ODESAT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

namespace {

// ------------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------------
template <typename T> struct Bits;
template <> struct Bits<float> { using U = uint32_t; };
template <> struct Bits<double> { using U = unsigned long long; };

__device__ __forceinline__ float dmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ double dmax(double a, double b) { return fmax(a, b); }
__device__ __forceinline__ float dmin(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ double dmin(double a, double b) { return fmin(a, b); }
__device__ __forceinline__ float dabs(float a) { return fabsf(a); }
__device__ __forceinline__ double dabs(double a) { return fabs(a); }
__device__ __forceinline__ float dsqrt(float a) { return sqrtf(a); }
__device__ __forceinline__ double dsqrt(double a) { return sqrt(a); }
__device__ __forceinline__ uint32_t tobits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ unsigned long long tobits(double x) {
    return (unsigned long long)__double_as_longlong(x);
}
__device__ __forceinline__ float frombits(uint32_t x) { return __uint_as_float(x); }
__device__ __forceinline__ double frombits(unsigned long long x) {
    return __longlong_as_double((long long)x);
}
template <typename T> __device__ __forceinline__ T inf_v() { return (T)__builtin_huge_val(); }

// VEC contiguous elements, loaded / stored as one 4-, 8- or 16-byte access per lane
template <typename T, int N> struct alignas(sizeof(T) * N) Vec {
    T e[N];
};
template <typename T, int N> __device__ __forceinline__ Vec<T, N> ldv(const T *p) {
    return *reinterpret_cast<const Vec<T, N> *>(p);
}
template <typename T, int N> __device__ __forceinline__ void stv(T *p, const Vec<T, N> &x) {
    *reinterpret_cast<Vec<T, N> *>(p) = x;
}
// store only the active elements (a partially frozen lane must not overwrite frozen replicas)
template <typename T, int N>
__device__ __forceinline__ void stv_masked(T *p, const Vec<T, N> &x, const bool (&on)[N], bool all_on) {
    if (all_on) {
        stv<T, N>(p, x);
    } else {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (on[k]) p[k] = x.e[k];
    }
}

// splitmix64 counter RNG -- same function as oracle/odesat_oracle.c (oc_hash3).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ double init_voltage(uint64_t seed, uint64_t replica, uint64_t var) {
    uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ULL);
    h = mix64(h ^ (replica * 0xD1B54A32D192ED03ULL + 0x632BE59BD9B4E019ULL));
    h = mix64(h ^ (var * 0x8CB92BA72F3D8DD7ULL + 0x9E3779B97F4A7C15ULL));
    const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
    return u * 2.0 - 1.0;
}

enum Mode : int { M_DERIV = 0, M_FIXED = 1, M_ADA = 2, M_ADB = 3 };

// The topology arrays are never written by a kernel: reading them through the constant address
// space lets wave-uniform indices become scalar (s_load) loads on the scalar cache.
typedef const __attribute__((address_space(4))) int32_t cint32;
__device__ __forceinline__ int32_t ldc(const int32_t *p, size_t i) { return ((cint32 *)p)[i]; }

template <typename T> struct KArgs {
    const int32_t *__restrict__ cptr;  // [m+1]
    const int32_t *__restrict__ lits;  // [L] var<<1 | neg, file order
    const int32_t *__restrict__ wpos;  // [L] slot -> variable-major position
    const int32_t *__restrict__ vptr;  // [n+1] variable -> first variable-major position
    T *v, *xs, *xl;                    // state        [G][n|m][W]
    T *w;                              // contributions [chunk groups][L][W]
    T *vh, *vf, *xsh, *xlh, *xsf, *xlf;  // half / full candidates (adaptive), derivatives (DERIV)
    T *dtr;                            // [Bp] per-replica adaptive dt
    typename Bits<T>::U *err;          // [Bp] max_error bits (non-negative floats order as ints)
    uint32_t *unsat;                   // [Bp] 1 = some clause had C >= gamma this step
    uint8_t *act;                      // [Bp] replica still stepping
    const int32_t *stop;               // first stop step (INT_MAX = none)
    int32_t n, m, L;
    int32_t g0, ng;                    // group range of this chunk
    int32_t rows;                      // rows (of 64/LW items) per wave
    int32_t tiles;                     // waves per group
    int32_t step;
    T dt, zeta, xl_max;
};

constexpr int WAVES_PER_BLOCK = 4;

// Per-wave geometry shared by the kernels.
template <int LW, int VEC> struct Geo {
    static constexpr int W = LW * VEC;  // replicas per group
    static constexpr int IPR = 64 / LW; // items per wave row
    int gl, g, tile, isub, lin;
    size_t off;  // element offset of this lane's first replica inside an item row
    int r0;      // this lane's first replica
    __device__ __forceinline__ bool init(int tiles, int g0, int ng) {
        const int lane = threadIdx.x & 63;
        const int wave = blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
        gl = wave / tiles;
        tile = wave - gl * tiles;
        if (gl >= ng) return false;
        g = g0 + gl;
        lin = lane % LW;
        isub = lane / LW;
        off = (size_t)lin * VEC;
        r0 = g * W + lin * VEC;
        return true;
    }
};

// :84-85 memory derivatives, then (by mode) the fused update_state of xs / xl (:94-95), the
// adaptive half / full candidates (:124-130) or the second half step and its max_error (:132),
// for the VEC replicas of one lane.
template <typename T, int VEC, int MODE>
__device__ __forceinline__ void clause_update(const KArgs<T> &a, size_t ci, const T (&C)[VEC],
                                              const Vec<T, VEC> &xs_m, const Vec<T, VEC> &xl_m,
                                              const T (&h)[VEC], const bool (&on)[VEC], bool all_on,
                                              T (&e)[VEC]) {
    const T one = (T)1.0, eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001;
    Vec<T, VEC> o1, o2, o3, o4;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const T dxs = (T)20.0 * (xs_m.e[k] + eps) * (C[k] - (T)0.25);  // :84
        const T dxl = (T)5.0 * (C[k] - (T)0.05);                       // :85
        const T half = (T)0.5 * h[k];
        if (MODE == M_DERIV) {
            o1.e[k] = dxs;
            o2.e[k] = dxl;
        } else if (MODE == M_FIXED) {
            o1.e[k] = dmin(dmax(xs_m.e[k] + h[k] * dxs, eps), xs_hi);
            o2.e[k] = dmin(dmax(xl_m.e[k] + h[k] * dxl, one), a.xl_max);
        } else if (MODE == M_ADA) {
            o1.e[k] = dmin(dmax(xs_m.e[k] + h[k] * dxs, eps), xs_hi);     // full-step clone
            o2.e[k] = dmin(dmax(xl_m.e[k] + h[k] * dxl, one), a.xl_max);
            o3.e[k] = dmin(dmax(xs_m.e[k] + half * dxs, eps), xs_hi);     // first half step
            o4.e[k] = dmin(dmax(xl_m.e[k] + half * dxl, one), a.xl_max);
        } else {
            o1.e[k] = dmin(dmax(xs_m.e[k] + half * dxs, eps), xs_hi);     // second half step
            o2.e[k] = dmin(dmax(xl_m.e[k] + half * dxl, one), a.xl_max);
        }
    }
    if (MODE == M_DERIV) {
        stv<T, VEC>(a.xsh + ci, o1);
        stv<T, VEC>(a.xlh + ci, o2);
    } else if (MODE == M_FIXED) {
        stv_masked<T, VEC>(a.xs + ci, o1, on, all_on);
        stv_masked<T, VEC>(a.xl + ci, o2, on, all_on);
    } else if (MODE == M_ADA) {
        stv<T, VEC>(a.xsf + ci, o1);
        stv<T, VEC>(a.xlf + ci, o2);
        stv<T, VEC>(a.xsh + ci, o3);
        stv<T, VEC>(a.xlh + ci, o4);
    } else {
        const Vec<T, VEC> fs = ldv<T, VEC>(a.xsf + ci), fl = ldv<T, VEC>(a.xlf + ci);
        stv_masked<T, VEC>(a.xs + ci, o1, on, all_on);
        stv_masked<T, VEC>(a.xl + ci, o2, on, all_on);
#pragma unroll
        for (int k = 0; k < VEC; ++k)  // :101-108 max_error terms
            e[k] = dmax(e[k], dmax(dabs(fs.e[k] - o1.e[k]), dabs(fl.e[k] - o2.e[k])));
    }
}

// The per-replica prologue shared by both clause kernels and the variable kernel.
template <typename T, int VEC, int MODE, bool CLAUSE>
__device__ __forceinline__ bool lane_state(const KArgs<T> &a, int r0, bool (&on)[VEC], bool &all_on,
                                           T (&h)[VEC]) {
    bool any = false;
    all_on = true;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        bool o = a.act[r0 + k] != 0;
        // adaptive: a replica allsat at the first RHS takes no step (system.rs:122)
        if (MODE == M_ADB || (!CLAUSE && MODE == M_ADA)) o = o && a.unsat[r0 + k] != 0;
        on[k] = o;
        any = any || o;
        all_on = all_on && o;
        h[k] = (MODE == M_ADA || MODE == M_ADB) ? a.dtr[r0 + k] : a.dt;
    }
    return __any(any);
}

// ------------------------------------------------------------------------------------------------
// k_clause_u: system.rs:35-90 (+ :94-95) for formulas whose clauses all have K literals (random
// k-SAT).  RB clauses per batch: their K*RB literal indices (scalar loads for LW = 64), K*RB voltage
// rows and 2*RB memory rows are all issued before the first use.  Out-of-range clauses of the last
// batch load clause m-1 and store nothing.
// ------------------------------------------------------------------------------------------------
template <typename T, int LW, int VEC, int MODE, int K>
__global__ __launch_bounds__(256) void k_clause_u(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    constexpr int RB = VEC >= 4 ? 2 : 4;
    G_ geo;
    if (!geo.init(a.tiles, a.g0, a.ng)) return;
    if (*a.stop < a.step) return;  // ODESAT_STOP_ANY already triggered
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, true>(a, geo.r0, on, all_on, h)) return;

    const T *__restrict__ V = (MODE == M_ADB) ? a.vh : a.v;
    const T *XS = (MODE == M_ADB) ? a.xsh : a.xs;
    const T *XL = (MODE == M_ADB) ? a.xlh : a.xl;
    const T one = (T)1.0, halfc = (T)0.5;
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const size_t cbase = (size_t)geo.g * a.m * W + geo.off;
    const size_t wbase = (size_t)geo.gl * a.L * W + geo.off;
    bool uns[VEC];
    T e[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        uns[k] = false;
        e[k] = (T)0.0;
    }

    for (int row0 = 0; row0 < a.rows; row0 += RB) {
        int cc[RB];
        bool ok[RB];
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            int c = (geo.tile * a.rows + row0 + b) * IPR + geo.isub;
            ok[b] = (row0 + b < a.rows) && (c < a.m);
            c = ok[b] ? c : a.m - 1;
            if (LW == 64) c = __builtin_amdgcn_readfirstlane(c);
            cc[b] = c;
        }
        int lit[RB][K], pos[RB][K];
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                lit[b][j] = ldc(a.lits, (size_t)cc[b] * K + j);
                pos[b][j] = ldc(a.wpos, (size_t)cc[b] * K + j);
            }
        Vec<T, VEC> vv[RB][K], xs_m[RB], xl_m[RB];
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int j = 0; j < K; ++j) vv[b][j] = ldv<T, VEC>(V + vbase + (size_t)(lit[b][j] >> 1) * W);
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            xs_m[b] = ldv<T, VEC>(XS + cbase + (size_t)cc[b] * W);
            xl_m[b] = ldv<T, VEC>(XL + cbase + (size_t)cc[b] * W);
        }
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            if (!ok[b]) continue;
            T C[VEC], mn[VEC], sec[VEC], t[VEC], tr[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                mn[k] = inf_v<T>();
                sec[k] = inf_v<T>();
#pragma unroll
                for (int j = 0; j < K; ++j) {  // :43-57 strict-< min / second-min, literal order
                    const T q = (lit[b][j] & 1) ? (T)-1.0 : (T)1.0;
                    const T val = one - q * vv[b][j].e[k];
                    const bool lt = val < mn[k];
                    sec[k] = lt ? mn[k] : (val < sec[k] ? val : sec[k]);
                    mn[k] = lt ? val : mn[k];
                }
                C[k] = halfc * mn[k];                                       // :60
                t[k] = xl_m[b].e[k] * xs_m[b].e[k];                         // :80 xl_m * xs_m
                tr[k] = (one + a.zeta * xl_m[b].e[k]) * (one - xs_m[b].e[k]);
                if (MODE != M_ADB) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));  // :88
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const T q = (lit[b][j] & 1) ? (T)-1.0 : (T)1.0;
                Vec<T, VEC> out;
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const T vi = vv[b][j].e[k];
                    const T val = one - q * vi;
                    const T g_ = halfc * q * (val != mn[k] ? mn[k] : sec[k]);        // :64-70
                    const T r_ = (C[k] == one - q * vi) ? halfc * (q - vi) : (T)0.0;  // :73-77
                    out.e[k] = t[k] * g_ + tr[k] * r_;                                // :80
                }
                stv<T, VEC>(a.w + wbase + (size_t)pos[b][j] * W, out);
            }
            clause_update<T, VEC, MODE>(a, cbase + (size_t)cc[b] * W, C, xs_m[b], xl_m[b], h, on, all_on, e);
        }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        if (MODE != M_ADB) {
            if (uns[k]) a.unsat[geo.r0 + k] = 1u;
        } else if (on[k]) {
            atomicMax(&a.err[geo.r0 + k], tobits(e[k]));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_clause: the same for mixed clause widths (literal values re-gathered for the second pass)
// ------------------------------------------------------------------------------------------------
template <typename T, int LW, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_clause(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    G_ geo;
    if (!geo.init(a.tiles, a.g0, a.ng)) return;
    if (*a.stop < a.step) return;
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, true>(a, geo.r0, on, all_on, h)) return;

    const T *__restrict__ V = (MODE == M_ADB) ? a.vh : a.v;
    const T *XS = (MODE == M_ADB) ? a.xsh : a.xs;
    const T *XL = (MODE == M_ADB) ? a.xlh : a.xl;
    const T one = (T)1.0, halfc = (T)0.5;
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const size_t cbase = (size_t)geo.g * a.m * W + geo.off;
    const size_t wbase = (size_t)geo.gl * a.L * W + geo.off;
    bool uns[VEC];
    T e[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        uns[k] = false;
        e[k] = (T)0.0;
    }
    for (int row = 0; row < a.rows; ++row) {
        int c = (geo.tile * a.rows + row) * IPR + geo.isub;
        if (LW == 64) c = __builtin_amdgcn_readfirstlane(c);
        if (c >= a.m) break;
        const int s0 = ldc(a.cptr, c), s1 = ldc(a.cptr, c + 1);
        const size_t ci = cbase + (size_t)c * W;
        const Vec<T, VEC> xs_m = ldv<T, VEC>(XS + ci), xl_m = ldv<T, VEC>(XL + ci);
        T mn[VEC], sec[VEC], C[VEC], t[VEC], tr[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            mn[k] = inf_v<T>();
            sec[k] = inf_v<T>();
        }
        for (int s = s0; s < s1; ++s) {  // :43-57
            const int lit = ldc(a.lits, s);
            const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
            const Vec<T, VEC> vv = ldv<T, VEC>(V + vbase + (size_t)(lit >> 1) * W);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T val = one - q * vv.e[k];
                const bool lt = val < mn[k];
                sec[k] = lt ? mn[k] : (val < sec[k] ? val : sec[k]);
                mn[k] = lt ? val : mn[k];
            }
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            C[k] = halfc * mn[k];
            t[k] = xl_m.e[k] * xs_m.e[k];
            tr[k] = (one + a.zeta * xl_m.e[k]) * (one - xs_m.e[k]);
            if (MODE != M_ADB) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));
        }
        for (int s = s0; s < s1; ++s) {  // :62-81
            const int lit = ldc(a.lits, s);
            const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
            const Vec<T, VEC> vv = ldv<T, VEC>(V + vbase + (size_t)(lit >> 1) * W);
            Vec<T, VEC> out;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T vi = vv.e[k];
                const T val = one - q * vi;
                const T g_ = halfc * q * (val != mn[k] ? mn[k] : sec[k]);
                const T r_ = (C[k] == one - q * vi) ? halfc * (q - vi) : (T)0.0;
                out.e[k] = t[k] * g_ + tr[k] * r_;
            }
            stv<T, VEC>(a.w + wbase + (size_t)ldc(a.wpos, s) * W, out);
        }
        clause_update<T, VEC, MODE>(a, ci, C, xs_m, xl_m, h, on, all_on, e);
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        if (MODE != M_ADB) {
            if (uns[k]) a.unsat[geo.r0 + k] = 1u;
        } else if (on[k]) {
            atomicMax(&a.err[geo.r0 + k], tobits(e[k]));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_variable: system.rs:33,80 (dv in the reference's accumulation order) + :96
// ------------------------------------------------------------------------------------------------
template <typename T, int LW, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_variable(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    G_ geo;
    if (!geo.init(a.tiles, a.g0, a.ng)) return;
    if (*a.stop < a.step) return;
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, false>(a, geo.r0, on, all_on, h)) return;
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const T *__restrict__ wsrc = a.w + (size_t)geo.gl * a.L * W + geo.off;
    T e[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) e[k] = (T)0.0;
    for (int row = 0; row < a.rows; ++row) {
        int i = (geo.tile * a.rows + row) * IPR + geo.isub;
        if (LW == 64) i = __builtin_amdgcn_readfirstlane(i);
        if (i >= a.n) break;
        const int p0 = ldc(a.vptr, i), p1 = ldc(a.vptr, i + 1);
        const size_t vi = vbase + (size_t)i * W;
        const Vec<T, VEC> v0 = ldv<T, VEC>(((MODE == M_ADB) ? a.vh : a.v) + vi);  // issued early
        T dv[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) dv[k] = (T)0.0;  // :33
        int p = p0;
        for (; p + 4 <= p1; p += 4) {  // four rows in flight, sequential adds (order kept)
            const Vec<T, VEC> w0 = ldv<T, VEC>(wsrc + (size_t)p * W);
            const Vec<T, VEC> w1 = ldv<T, VEC>(wsrc + (size_t)(p + 1) * W);
            const Vec<T, VEC> w2 = ldv<T, VEC>(wsrc + (size_t)(p + 2) * W);
            const Vec<T, VEC> w3 = ldv<T, VEC>(wsrc + (size_t)(p + 3) * W);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                dv[k] += w0.e[k];
                dv[k] += w1.e[k];
                dv[k] += w2.e[k];
                dv[k] += w3.e[k];
            }
        }
        for (; p < p1; ++p) {
            const Vec<T, VEC> w0 = ldv<T, VEC>(wsrc + (size_t)p * W);
#pragma unroll
            for (int k = 0; k < VEC; ++k) dv[k] += w0.e[k];
        }
        Vec<T, VEC> o1, o2;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            if (MODE == M_DERIV) {
                o1.e[k] = dv[k];
            } else if (MODE == M_FIXED) {
                o1.e[k] = dmin(dmax(v0.e[k] + h[k] * dv[k], (T)-1.0), (T)1.0);
            } else if (MODE == M_ADA) {
                const T half = (T)0.5 * h[k];
                o1.e[k] = dmin(dmax(v0.e[k] + h[k] * dv[k], (T)-1.0), (T)1.0);   // full-step clone
                o2.e[k] = dmin(dmax(v0.e[k] + half * dv[k], (T)-1.0), (T)1.0);  // first half step
            } else {
                const T half = (T)0.5 * h[k];
                o1.e[k] = dmin(dmax(v0.e[k] + half * dv[k], (T)-1.0), (T)1.0);  // second half step
            }
        }
        if (MODE == M_DERIV) {
            stv<T, VEC>(a.vh + vi, o1);
        } else if (MODE == M_FIXED) {
            stv_masked<T, VEC>(a.v + vi, o1, on, all_on);
        } else if (MODE == M_ADA) {
            stv<T, VEC>(a.vf + vi, o1);
            stv<T, VEC>(a.vh + vi, o2);
        } else {
            const Vec<T, VEC> f = ldv<T, VEC>(a.vf + vi);
            stv_masked<T, VEC>(a.v + vi, o1, on, all_on);
#pragma unroll
            for (int k = 0; k < VEC; ++k) e[k] = dmax(e[k], dabs(f.e[k] - o1.e[k]));
        }
    }
    if (MODE == M_ADB) {
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            if (on[k]) atomicMax(&a.err[geo.r0 + k], tobits(e[k]));
    }
}

// ------------------------------------------------------------------------------------------------
// k_status: per-replica bookkeeping after all kernels of one step of a replica range
// ------------------------------------------------------------------------------------------------
struct StatusArgs {
    uint8_t *act;
    uint32_t *unsat;
    void *err;
    void *dtr;
    int64_t *sat_step;
    int64_t *steps_done;
    int32_t *stop;
    int32_t r0, r1, step, stop_mode, adaptive;
    double tol;
};

template <typename T> __global__ void k_status(StatusArgs s) {
    const int r = s.r0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= s.r1) return;
    if (*s.stop < s.step) return;  // this step did not run
    auto *err = (typename Bits<T>::U *)s.err;
    T *dtr = (T *)s.dtr;
    if (s.act[r]) {
        const bool allsat = s.unsat[r] == 0u;
        s.steps_done[r] += 1;
        if (allsat) {
            if (s.sat_step[r] < 0) s.sat_step[r] = s.step;
            if (s.stop_mode == ODESAT_STOP_EACH) s.act[r] = 0;             // simulate() breaks (:193)
            if (s.stop_mode == ODESAT_STOP_ANY) atomicMin(s.stop, s.step);  // simulate_inter (:291)
        } else if (s.adaptive) {  // :133-135 dt <- clamp(dt * sqrt(tol / err), 2^-7, 1e3)
            const T error = frombits(err[r]);
            const T h = dtr[r];
            dtr[r] = dmax(dmin(h * dsqrt((T)s.tol / error), (T)1e3), (T)0.0078125);
        }
    }
    s.unsat[r] = 0u;
    if (s.adaptive) err[r] = 0;
}

// ------------------------------------------------------------------------------------------------
// init / layout kernels (not on the hot path: group width W is a runtime argument)
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void k_init(T *v, T *xs, T *xl, const int32_t *cptr, const int32_t *lits, int n, int m, int G,
                       int W, int B, uint64_t seed, int64_t replica0) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nv = (size_t)G * n * W, nc = (size_t)G * m * W;
    if (tid < nv) {
        const int lane = (int)(tid % W);
        const size_t gi = tid / W;
        const int i = (int)(gi % n);
        const int g = (int)(gi / n);
        const int r = g * W + lane;
        v[tid] = r < B ? (T)init_voltage(seed, (uint64_t)(replica0 + r), (uint64_t)i) : (T)0.0;
    }
    if (tid < nc) {
        const size_t gi = tid / W;
        const int c = (int)(gi % m);
        bool anyneg = false;  // system.rs:361-372
        for (int s = cptr[c]; s < cptr[c + 1]; ++s) anyneg |= (lits[s] & 1) != 0;
        xs[tid] = anyneg ? (T)1.0 : (T)-1.0;
        xl[tid] = (T)1.0;
    }
}

// compact [count][items] f64 <-> layout [G][items][W] in dtype T
template <typename T>
__global__ void k_scatter(T *dst, const double *src, int items, int W, int64_t r0, int64_t count) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)count * items) return;
    const int64_t b = (int64_t)(tid / items);
    const int i = (int)(tid % items);
    const int64_t r = r0 + b;
    dst[((size_t)(r / W) * items + i) * W + (r % W)] = (T)src[tid];
}

template <typename T>
__global__ void k_gather(double *dst, const T *src, int items, int W, int64_t r0, int64_t count) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)count * items) return;
    const int64_t b = (int64_t)(tid / items);
    const int i = (int)(tid % items);
    const int64_t r = r0 + b;
    dst[tid] = (double)src[((size_t)(r / W) * items + i) * W + (r % W)];
}

__global__ void k_reset_replicas(uint8_t *act, uint32_t *unsat, int64_t *sat_step, int64_t *steps_done,
                                 void *dtr, int dtype, int64_t r0, int64_t count, int64_t B, int64_t Bp) {
    const int64_t r = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= r0 + count || r >= Bp) return;
    act[r] = r < B ? 1 : 0;
    unsat[r] = 0;
    sat_step[r] = -1;
    steps_done[r] = 0;
    if (dtype == ODESAT_F64) ((double *)dtr)[r] = 0.01;
    else ((float *)dtr)[r] = 0.01f;
}

}  // namespace

// ================================================================================================
// host side
// ================================================================================================
struct odesat_solver {
    int device = 0, dtype = ODESAT_F32;
    int64_t n = 0, m = 0, L = 0, B = 0, Bp = 0;
    int LW = 64, VEC = 1, W = 64, G = 1;
    int chunk_groups = 1;
    int uniform_k = 0;  // every clause has this many literals (0 = mixed widths)
    int schedule = ODESAT_SCHED_AUTO;
    size_t tsize = 4;
    hipStream_t stream = nullptr;
    int32_t *cptr = nullptr, *lits = nullptr, *wpos = nullptr, *vptr = nullptr;
    void *v = nullptr, *xs = nullptr, *xl = nullptr, *w = nullptr;
    void *vh = nullptr, *vf = nullptr, *xsh = nullptr, *xlh = nullptr, *xsf = nullptr, *xlf = nullptr;
    void *dtr = nullptr, *err = nullptr;
    uint32_t *unsat = nullptr;
    uint8_t *act = nullptr;
    int64_t *sat_step = nullptr, *steps_done = nullptr;
    int32_t *stop = nullptr;
    int64_t bytes = 0;
    // profiling
    bool profile = false;
    struct Pending { int cls; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    double prof_ms[3] = {0, 0, 0};
    int64_t prof_n[3] = {0, 0, 0};
};

namespace {

template <int V> using IC = std::integral_constant<int, V>;

// Call f(IC<LW>, IC<VEC>) with the solver's compile-time layout.
template <typename T, typename F> int with_layout(const odesat_solver *s, F &&f) {
    if (s->VEC == 4) {
        if constexpr (sizeof(T) == 4) return f(IC<64>{}, IC<4>{});
        else return fail(ODESAT_EINVAL, "VEC=4 is f32-only");
    }
    if (s->VEC == 2) return f(IC<64>{}, IC<2>{});
    switch (s->LW) {
        case 1: return f(IC<1>{}, IC<1>{});
        case 2: return f(IC<2>{}, IC<1>{});
        case 4: return f(IC<4>{}, IC<1>{});
        case 8: return f(IC<8>{}, IC<1>{});
        case 16: return f(IC<16>{}, IC<1>{});
        case 32: return f(IC<32>{}, IC<1>{});
        default: return f(IC<64>{}, IC<1>{});
    }
}

int dmalloc(odesat_solver *s, void **p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(e == hipErrorOutOfMemory ? ODESAT_ENOMEM : ODESAT_EDEVICE,
                    "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    }
    s->bytes += (int64_t)bytes;
    return ODESAT_OK;
}

void dfree(void *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

size_t state_elems(const odesat_solver *s, int64_t items) { return (size_t)s->G * items * s->W; }

int ensure_scratch(odesat_solver *s) {
    if (s->vh) return ODESAT_OK;
    int rc;
    if ((rc = dmalloc(s, &s->vh, state_elems(s, s->n) * s->tsize))) return rc;
    if ((rc = dmalloc(s, &s->vf, state_elems(s, s->n) * s->tsize))) return rc;
    if ((rc = dmalloc(s, &s->xsh, state_elems(s, s->m) * s->tsize))) return rc;
    if ((rc = dmalloc(s, &s->xlh, state_elems(s, s->m) * s->tsize))) return rc;
    if ((rc = dmalloc(s, &s->xsf, state_elems(s, s->m) * s->tsize))) return rc;
    if ((rc = dmalloc(s, &s->xlf, state_elems(s, s->m) * s->tsize))) return rc;
    return ODESAT_OK;
}

int ensure_w(odesat_solver *s) {
    if (s->w) return ODESAT_OK;
    return dmalloc(s, &s->w, (size_t)s->chunk_groups * s->L * s->W * s->tsize);
}

hipEvent_t take_event(odesat_solver *s) {
    if (!s->pool.empty()) {
        hipEvent_t e = s->pool.back();
        s->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

int drain_profile(odesat_solver *s) {
    if (s->pending.empty()) return ODESAT_OK;
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (auto &p : s->pending) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
        s->prof_ms[p.cls] += ms;
        s->prof_n[p.cls] += 1;
        s->pool.push_back(p.a);
        s->pool.push_back(p.b);
    }
    s->pending.clear();
    return ODESAT_OK;
}

// rows per wave: enough waves to fill 256 CUs many times over, rows >= 1
int pick_rows(int64_t items_per_group, int ng, int LW) {
    const int64_t ipr = 64 / LW;
    const int64_t row_total = (items_per_group + ipr - 1) / ipr * ng;
    const int64_t rows = row_total / 16384;
    return (int)std::max<int64_t>(1, std::min<int64_t>(rows, 16));
}

template <typename T> KArgs<T> make_args(odesat_solver *s) {
    KArgs<T> a{};
    a.cptr = s->cptr;
    a.lits = s->lits;
    a.wpos = s->wpos;
    a.vptr = s->vptr;
    a.v = (T *)s->v;
    a.xs = (T *)s->xs;
    a.xl = (T *)s->xl;
    a.w = (T *)s->w;
    a.vh = (T *)s->vh;
    a.vf = (T *)s->vf;
    a.xsh = (T *)s->xsh;
    a.xlh = (T *)s->xlh;
    a.xsf = (T *)s->xsf;
    a.xlf = (T *)s->xlf;
    a.dtr = (T *)s->dtr;
    a.err = (typename Bits<T>::U *)s->err;
    a.unsat = s->unsat;
    a.act = s->act;
    a.stop = s->stop;
    a.n = (int32_t)s->n;
    a.m = (int32_t)s->m;
    a.L = (int32_t)s->L;
    a.xl_max = (T)1e4 * (T)s->m;  // system.rs:95 `1e4 * clause_nums`, in the solver's dtype
    return a;
}

struct Timed {  // brackets one launch with profiling events
    odesat_solver *s;
    int cls;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    Timed(odesat_solver *s_, int c) : s(s_), cls(c) {
        if (s->profile) {
            e0 = take_event(s);
            e1 = take_event(s);
            (void)hipEventRecord(e0, s->stream);
        }
    }
    ~Timed() {
        if (s->profile) {
            (void)hipEventRecord(e1, s->stream);
            s->pending.push_back({cls, e0, e1});
        }
    }
};

template <typename T, int LW, int VEC, int MODE>
int launch_kernel(odesat_solver *s, KArgs<T> a, bool clause) {
    const int64_t items = clause ? s->m : s->n;
    a.rows = pick_rows(items, a.ng, LW);
    const int64_t ipr = 64 / LW;
    a.tiles = (int)((items + ipr * a.rows - 1) / (ipr * a.rows));
    if (a.tiles == 0) return ODESAT_OK;
    const int64_t waves = (int64_t)a.tiles * a.ng;
    const int64_t blocks = (waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks > INT_MAX) return fail(ODESAT_EINVAL, "grid too large");
    const dim3 grid((unsigned)blocks), block(64 * WAVES_PER_BLOCK);
    {
        Timed tm(s, clause ? 0 : 1);
        if (clause && s->uniform_k == 3)
            hipLaunchKernelGGL((k_clause_u<T, LW, VEC, MODE, 3>), grid, block, 0, s->stream, a);
        else if (clause)
            hipLaunchKernelGGL((k_clause<T, LW, VEC, MODE>), grid, block, 0, s->stream, a);
        else
            hipLaunchKernelGGL((k_variable<T, LW, VEC, MODE>), grid, block, 0, s->stream, a);
    }
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

// One RHS(+update) of `MODE` for the groups [gA, gB): k_clause then k_variable per chunk.
template <typename T, int LW, int VEC, int MODE>
int step_chunks(odesat_solver *s, int step, T dt, T zeta, int gA, int gB) {
    KArgs<T> a = make_args<T>(s);
    a.step = step;
    a.dt = dt;
    a.zeta = zeta;
    int rc;
    for (int g0 = gA; g0 < gB; g0 += s->chunk_groups) {
        a.g0 = g0;
        a.ng = std::min(s->chunk_groups, gB - g0);
        if ((rc = launch_kernel<T, LW, VEC, MODE>(s, a, true))) return rc;
        if ((rc = launch_kernel<T, LW, VEC, MODE>(s, a, false))) return rc;
    }
    return ODESAT_OK;
}

template <typename T>
int launch_status(odesat_solver *s, int step, int stop_mode, bool adaptive, double tol, int64_t r0, int64_t r1) {
    r1 = std::min<int64_t>(r1, s->B);
    if (r1 <= r0) return ODESAT_OK;
    StatusArgs sa{};
    sa.act = s->act;
    sa.unsat = s->unsat;
    sa.err = s->err;
    sa.dtr = s->dtr;
    sa.sat_step = s->sat_step;
    sa.steps_done = s->steps_done;
    sa.stop = s->stop;
    sa.r0 = (int32_t)r0;
    sa.r1 = (int32_t)r1;
    sa.step = step;
    sa.stop_mode = stop_mode;
    sa.adaptive = adaptive ? 1 : 0;
    sa.tol = tol;
    const int threads = 256;
    const int blocks = (int)((r1 - r0 + threads - 1) / threads);
    {
        Timed tm(s, 2);
        hipLaunchKernelGGL((k_status<T>), dim3(blocks), dim3(threads), 0, s->stream, sa);
    }
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

// One full euler step (fixed or adaptive) for the replica groups [gA, gB), enqueued on the stream.
template <typename T>
int enqueue_step(odesat_solver *s, int step, bool adaptive, double dt, double zeta, double tol, int stop_mode,
                 int gA, int gB) {
    int rc = with_layout<T>(s, [&](auto lw, auto vec) -> int {
        constexpr int LW = decltype(lw)::value, VEC = decltype(vec)::value;
        int r;
        if (!adaptive) return step_chunks<T, LW, VEC, M_FIXED>(s, step, (T)dt, (T)zeta, gA, gB);
        // the two half steps of one chunk run back to back (one contribution buffer per chunk)
        for (int g0 = gA; g0 < gB; g0 += s->chunk_groups) {
            const int g1 = std::min(gB, g0 + s->chunk_groups);
            if ((r = step_chunks<T, LW, VEC, M_ADA>(s, step, (T)dt, (T)zeta, g0, g1))) return r;
            if ((r = step_chunks<T, LW, VEC, M_ADB>(s, step, (T)dt, (T)zeta, g0, g1))) return r;
        }
        return ODESAT_OK;
    });
    if (rc) return rc;
    return launch_status<T>(s, step, stop_mode, adaptive, tol, (int64_t)gA * s->W, (int64_t)gB * s->W);
}

int dispatch_step(odesat_solver *s, int step, bool adaptive, double dt, double zeta, double tol, int stop_mode,
                  int gA, int gB) {
    return s->dtype == ODESAT_F64 ? enqueue_step<double>(s, step, adaptive, dt, zeta, tol, stop_mode, gA, gB)
                                  : enqueue_step<float>(s, step, adaptive, dt, zeta, tol, stop_mode, gA, gB);
}

template <typename T> int deriv_t(odesat_solver *s, double zeta) {
    return with_layout<T>(s, [&](auto lw, auto vec) -> int {
        constexpr int LW = decltype(lw)::value, VEC = decltype(vec)::value;
        return step_chunks<T, LW, VEC, M_DERIV>(s, 0, (T)0, (T)zeta, 0, s->G);
    });
}

template <typename T>
int layout_t(odesat_solver *s, void *dev, const double *dsrc, double *ddst, int64_t items, int64_t r0,
             int64_t count, bool scatter) {
    const size_t total = (size_t)count * items;
    if (!total) return ODESAT_OK;
    const int threads = 256;
    const size_t blocks = (total + threads - 1) / threads;
    if (scatter)
        hipLaunchKernelGGL((k_scatter<T>), dim3((unsigned)blocks), dim3(threads), 0, s->stream, (T *)dev, dsrc,
                           (int)items, s->W, r0, count);
    else
        hipLaunchKernelGGL((k_gather<T>), dim3((unsigned)blocks), dim3(threads), 0, s->stream, ddst,
                           (const T *)dev, (int)items, s->W, r0, count);
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

int layout(odesat_solver *s, void *dev, const double *dsrc, double *ddst, int64_t items, int64_t r0,
           int64_t count, bool scatter) {
    return s->dtype == ODESAT_F64 ? layout_t<double>(s, dev, dsrc, ddst, items, r0, count, scatter)
                                  : layout_t<float>(s, dev, dsrc, ddst, items, r0, count, scatter);
}

// host f64 [count][items] <-> device layout, through a device staging buffer
int upload_items(odesat_solver *s, void *dev, const double *host, int64_t items, int64_t r0, int64_t count) {
    if (!host || !items || !count) return ODESAT_OK;
    void *stage = nullptr;
    const size_t bytes = (size_t)count * items * sizeof(double);
    HIP_TRY(hipMalloc(&stage, bytes));
    hipError_t e = hipMemcpyAsync(stage, host, bytes, hipMemcpyHostToDevice, s->stream);
    int rc = e == hipSuccess ? layout(s, dev, (const double *)stage, nullptr, items, r0, count, true)
                             : fail(ODESAT_EDEVICE, hipGetErrorString(e));
    hipError_t e2 = hipStreamSynchronize(s->stream);
    (void)hipFree(stage);
    if (rc) return rc;
    HIP_TRY(e2);
    return ODESAT_OK;
}

int download_items(odesat_solver *s, const void *dev, double *host, int64_t items, int64_t r0, int64_t count) {
    if (!host || !items || !count) return ODESAT_OK;
    void *stage = nullptr;
    const size_t bytes = (size_t)count * items * sizeof(double);
    HIP_TRY(hipMalloc(&stage, bytes));
    int rc = layout(s, const_cast<void *>(dev), nullptr, (double *)stage, items, r0, count, false);
    hipError_t e = rc ? hipSuccess : hipMemcpyAsync(host, stage, bytes, hipMemcpyDeviceToHost, s->stream);
    hipError_t e2 = hipStreamSynchronize(s->stream);
    (void)hipFree(stage);
    if (rc) return rc;
    HIP_TRY(e);
    HIP_TRY(e2);
    return ODESAT_OK;
}

int reset_replicas(odesat_solver *s, int64_t r0, int64_t count) {
    if (count <= 0) return ODESAT_OK;
    const int threads = 256;
    const int blocks = (int)((count + threads - 1) / threads);
    hipLaunchKernelGGL(k_reset_replicas, dim3(blocks), dim3(threads), 0, s->stream, s->act, s->unsat,
                       s->sat_step, s->steps_done, s->dtr, s->dtype, r0, count, s->B, s->Bp);
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

int set_stop(odesat_solver *s, int32_t value) {
    HIP_TRY(hipMemcpyAsync(s->stop, &value, sizeof(value), hipMemcpyHostToDevice, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

int check_solver(odesat_solver *s) {
    if (!s) return fail(ODESAT_EINVAL, "null solver");
    HIP_TRY(hipSetDevice(s->device));
    return ODESAT_OK;
}

template <typename T> int init_t(odesat_solver *s, uint64_t seed, int64_t replica0) {
    const size_t total = std::max(state_elems(s, s->n), state_elems(s, s->m));
    if (!total) return ODESAT_OK;
    const int threads = 256;
    const size_t blocks = (total + threads - 1) / threads;
    hipLaunchKernelGGL((k_init<T>), dim3((unsigned)blocks), dim3(threads), 0, s->stream, (T *)s->v, (T *)s->xs,
                       (T *)s->xl, s->cptr, s->lits, (int)s->n, (int)s->m, s->G, s->W, (int)s->B, seed, replica0);
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

int init_dispatch(odesat_solver *s, uint64_t seed, int64_t replica0) {
    return s->dtype == ODESAT_F64 ? init_t<double>(s, seed, replica0) : init_t<float>(s, seed, replica0);
}

double default_zeta(const odesat_solver *s) {  // system.rs:164-173
    const double d = (double)s->m / (double)s->n;
    return d >= 6.0 ? 0.1 : (d >= 4.9 ? 0.01 : 0.001);
}

void pick_chunk(odesat_solver *s, int64_t replicas) {
    // one chunk = state + contribution buffer of chunk_groups groups
    const int64_t per_group = (s->n + 2 * s->m + s->L) * s->W * (int64_t)s->tsize;
    int64_t groups;
    if (replicas > 0) {
        groups = std::max<int64_t>(1, replicas / s->W);
    } else {
        // keep one chunk's working set well inside the 256 MiB Infinity Cache
        const int64_t budget = 120ll << 20;
        groups = std::max<int64_t>(1, budget / std::max<int64_t>(per_group, 1));
    }
    s->chunk_groups = (int)std::min<int64_t>(groups, s->G);
}

std::vector<int64_t> host_i64(int64_t n, int64_t v) { return std::vector<int64_t>((size_t)n, v); }

int put_dt(odesat_solver *s, const double *vals, double fill) {
    if (s->dtype == ODESAT_F64) {
        std::vector<double> h(s->Bp, fill);
        if (vals) for (int64_t r = 0; r < s->B; ++r) h[r] = vals[r];
        HIP_TRY(hipMemcpy(s->dtr, h.data(), s->Bp * 8, hipMemcpyHostToDevice));
    } else {
        std::vector<float> h(s->Bp, (float)fill);
        if (vals) for (int64_t r = 0; r < s->B; ++r) h[r] = (float)vals[r];
        HIP_TRY(hipMemcpy(s->dtr, h.data(), s->Bp * 4, hipMemcpyHostToDevice));
    }
    return ODESAT_OK;
}

int get_dt(odesat_solver *s, double *out) {
    if (s->dtype == ODESAT_F64) {
        HIP_TRY(hipMemcpy(out, s->dtr, s->B * 8, hipMemcpyDeviceToHost));
    } else {
        std::vector<float> h(s->B);
        HIP_TRY(hipMemcpy(h.data(), s->dtr, s->B * 4, hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < s->B; ++r) out[r] = h[r];
    }
    return ODESAT_OK;
}

int set_all_active(odesat_solver *s) {
    std::vector<uint8_t> on(s->Bp, 0);
    for (int64_t r = 0; r < s->B; ++r) on[r] = 1;
    HIP_TRY(hipMemcpy(s->act, on.data(), s->Bp, hipMemcpyHostToDevice));
    return ODESAT_OK;
}

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" const char *odesat_version(void) { return "odesat_amd 0.2 (gfx950)"; }

extern "C" int odesat_device_count(int *count) {
    if (!count) return fail(ODESAT_EINVAL, "null count");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = e == hipSuccess ? c : 0;
    return ODESAT_OK;
}

extern "C" void odesat_solver_destroy(odesat_solver *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (auto &p : s->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : s->pool) (void)hipEventDestroy(e);
    void *ptrs[] = {s->cptr, s->lits, s->wpos, s->vptr, s->v, s->xs, s->xl, s->w, s->vh, s->vf,
                    s->xsh, s->xlh, s->xsf, s->xlf, s->dtr, s->err, s->unsat, s->act, s->sat_step,
                    s->steps_done, s->stop};
    for (void *p : ptrs) dfree(p);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

extern "C" int odesat_solver_create(int device, const odesat_cnf *f, int64_t batch, int dtype,
                                    odesat_solver **out) {
    if (!out) return fail(ODESAT_EINVAL, "null out");
    *out = nullptr;
    if (!f) return fail(ODESAT_EINVAL, "null formula");
    if (batch <= 0) return fail(ODESAT_EINVAL, "batch must be > 0");
    if (dtype != ODESAT_F32 && dtype != ODESAT_F64) return fail(ODESAT_EINVAL, "dtype must be ODESAT_F32 or ODESAT_F64");
    const int64_t n = f->varnum, m = f->nclauses(), L = f->nliterals();
    if (n <= 0) return fail(ODESAT_EINVAL, "varnum must be > 0");
    if (n >= (1ll << 30) || m >= INT_MAX / 4 || L >= INT_MAX || batch >= INT_MAX / 2)
        return fail(ODESAT_EINVAL, "formula or batch too large");
    for (int64_t s = 0; s < L; ++s)
        if (f->var[s] < 0 || f->var[s] >= n)
            return fail(ODESAT_EINVAL, "variable " + std::to_string(f->var[s]) + " out of range [0, " +
                                           std::to_string(n) + "): normalise the formula first "
                                           "(the reference would index out of bounds, system.rs:48)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(ODESAT_EDEVICE, "no HIP device available (odesat_amd has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(ODESAT_EINVAL, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
        return fail(ODESAT_EDEVICE, std::string("odesat_amd is built for gfx950, device is ") + prop.gcnArchName);

    auto *s = new (std::nothrow) odesat_solver();
    if (!s) return fail(ODESAT_ENOMEM, "out of memory");
    s->device = device;
    s->dtype = dtype;
    s->tsize = dtype == ODESAT_F64 ? 8 : 4;
    s->n = n;
    s->m = m;
    s->L = L;
    s->B = batch;
    // layout: 16-byte lanes once a batch fills 64 lanes of 16 B
    const int vmax = 16 / (int)s->tsize;
    if (batch >= 64 * vmax) {
        s->LW = 64;
        s->VEC = vmax;
    } else if (batch >= 128 && vmax >= 2) {
        s->LW = 64;
        s->VEC = 2;
    } else {
        int lw = 1;
        while (lw < batch && lw < 64) lw <<= 1;
        s->LW = lw;
        s->VEC = 1;
    }
    s->W = s->LW * s->VEC;
    s->Bp = (batch + s->W - 1) / s->W * s->W;
    s->G = (int)(s->Bp / s->W);
    pick_chunk(s, 0);
    s->uniform_k = m > 0 ? (int)(f->clause_ptr[1] - f->clause_ptr[0]) : 0;
    for (int64_t c = 0; c < m && s->uniform_k; ++c)
        if (f->clause_ptr[c + 1] - f->clause_ptr[c] != s->uniform_k) s->uniform_k = 0;
    if (s->uniform_k != 3) s->uniform_k = 0;  // the specialised kernel is instantiated for 3-SAT
    int rc = ODESAT_OK;
    auto bail = [&](int code) {
        odesat_solver_destroy(s);
        return code;
    };
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "hipStreamCreate failed"));

    // topology: clause CSR, packed literals, variable-major slot positions
    std::vector<int32_t> cptr(m + 1), lits(L), wpos(L), vptr(n + 1, 0);
    for (int64_t c = 0; c <= m; ++c) cptr[c] = (int32_t)f->clause_ptr[c];
    for (int64_t s2 = 0; s2 < L; ++s2) {
        lits[s2] = (int32_t)((f->var[s2] << 1) | (f->neg[s2] ? 1 : 0));
        vptr[f->var[s2] + 1] += 1;
    }
    for (int64_t i = 0; i < n; ++i) vptr[i + 1] += vptr[i];
    {
        std::vector<int32_t> fill(vptr.begin(), vptr.end() - 1);
        for (int64_t s2 = 0; s2 < L; ++s2) wpos[s2] = fill[f->var[s2]]++;  // slot order = clause order
    }
    if ((rc = dmalloc(s, (void **)&s->cptr, (m + 1) * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->lits, L * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->wpos, L * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->vptr, (n + 1) * 4))) return bail(rc);
    if (hipMemcpy(s->cptr, cptr.data(), (m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (L && hipMemcpy(s->lits, lits.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (L && hipMemcpy(s->wpos, wpos.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(s->vptr, vptr.data(), (n + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
    // state
    if ((rc = dmalloc(s, &s->v, state_elems(s, n) * s->tsize))) return bail(rc);
    if ((rc = dmalloc(s, &s->xs, state_elems(s, m) * s->tsize))) return bail(rc);
    if ((rc = dmalloc(s, &s->xl, state_elems(s, m) * s->tsize))) return bail(rc);
    if ((rc = dmalloc(s, &s->dtr, s->Bp * s->tsize))) return bail(rc);
    if ((rc = dmalloc(s, &s->err, s->Bp * 8))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->unsat, s->Bp * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->act, s->Bp))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->sat_step, s->Bp * 8))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->steps_done, s->Bp * 8))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->stop, 16))) return bail(rc);
    if (hipMemsetAsync(s->err, 0, s->Bp * 8, s->stream) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "memset failed"));
    // default state: v = 0, xs = init_short_term_memory, xl = 1
    if ((rc = init_dispatch(s, 0, 0))) return bail(rc);
    if (hipMemsetAsync(s->v, 0, state_elems(s, n) * s->tsize, s->stream) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "memset failed"));
    if ((rc = reset_replicas(s, 0, s->Bp))) return bail(rc);
    if ((rc = set_stop(s, INT_MAX))) return bail(rc);
    *out = s;
    return ODESAT_OK;
}

extern "C" int64_t odesat_solver_batch(const odesat_solver *s) { return s ? s->B : -1; }
extern "C" int64_t odesat_solver_varnum(const odesat_solver *s) { return s ? s->n : -1; }
extern "C" int64_t odesat_solver_nclauses(const odesat_solver *s) { return s ? s->m : -1; }
extern "C" int64_t odesat_solver_device_bytes(const odesat_solver *s) { return s ? s->bytes : -1; }

extern "C" int odesat_set_chunk_replicas(odesat_solver *s, int64_t replicas) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (replicas < 0) return fail(ODESAT_EINVAL, "replicas must be >= 0");
    const int old = s->chunk_groups;
    pick_chunk(s, replicas);
    if (s->chunk_groups != old && s->w) {
        HIP_TRY(hipStreamSynchronize(s->stream));
        s->bytes -= (int64_t)old * s->L * s->W * s->tsize;
        dfree(s->w);
    }
    return ODESAT_OK;
}

extern "C" int odesat_set_schedule(odesat_solver *s, int schedule) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (schedule < ODESAT_SCHED_AUTO || schedule > ODESAT_SCHED_CHUNK_MAJOR) return fail(ODESAT_EINVAL, "bad schedule");
    s->schedule = schedule;
    return ODESAT_OK;
}

extern "C" int odesat_set_state(odesat_solver *s, int64_t r0, int64_t count, const double *v, const double *xs,
                                const double *xl) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    if ((rc = upload_items(s, s->v, v, s->n, r0, count))) return rc;
    if ((rc = upload_items(s, s->xs, xs, s->m, r0, count))) return rc;
    if ((rc = upload_items(s, s->xl, xl, s->m, r0, count))) return rc;
    if ((rc = reset_replicas(s, r0, count))) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

extern "C" int odesat_init_state(odesat_solver *s, uint64_t seed, int64_t replica0) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if ((rc = init_dispatch(s, seed, replica0))) return rc;
    if ((rc = reset_replicas(s, 0, s->Bp))) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

extern "C" int odesat_get_state(odesat_solver *s, int64_t r0, int64_t count, double *v, double *xs, double *xl) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    if ((rc = download_items(s, s->v, v, s->n, r0, count))) return rc;
    if ((rc = download_items(s, s->xs, xs, s->m, r0, count))) return rc;
    if ((rc = download_items(s, s->xl, xl, s->m, r0, count))) return rc;
    return ODESAT_OK;
}

extern "C" int odesat_get_assignment(odesat_solver *s, int64_t r, uint8_t *assignment) {
    if (!assignment) return fail(ODESAT_EINVAL, "null assignment");
    int rc;
    if ((rc = check_solver(s))) return rc;
    std::vector<double> v(s->n);
    if ((rc = odesat_get_state(s, r, 1, v.data(), nullptr, nullptr))) return rc;
    for (int64_t i = 0; i < s->n; ++i) assignment[i] = v[i] > 0.0 ? 1 : 0;  // system.rs:238
    return ODESAT_OK;
}

extern "C" int odesat_compute_derivatives(odesat_solver *s, double zeta, double *dv, double *dxs, double *dxl,
                                          uint8_t *allsat) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if ((rc = ensure_scratch(s)) || (rc = ensure_w(s))) return rc;
    if ((rc = set_stop(s, INT_MAX))) return rc;
    // every real replica evaluates (act = 1) without touching the stored sat bookkeeping
    std::vector<uint8_t> act_save(s->Bp);
    HIP_TRY(hipMemcpy(act_save.data(), s->act, s->Bp, hipMemcpyDeviceToHost));
    if ((rc = set_all_active(s))) return rc;
    HIP_TRY(hipMemset(s->unsat, 0, s->Bp * 4));
    rc = s->dtype == ODESAT_F64 ? deriv_t<double>(s, zeta) : deriv_t<float>(s, zeta);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    if ((rc = download_items(s, s->vh, dv, s->n, 0, s->B))) return rc;
    if ((rc = download_items(s, s->xsh, dxs, s->m, 0, s->B))) return rc;
    if ((rc = download_items(s, s->xlh, dxl, s->m, 0, s->B))) return rc;
    if (allsat) {
        std::vector<uint32_t> u(s->Bp);
        HIP_TRY(hipMemcpy(u.data(), s->unsat, s->Bp * 4, hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < s->B; ++r) allsat[r] = u[r] == 0u;
    }
    HIP_TRY(hipMemset(s->unsat, 0, s->Bp * 4));
    HIP_TRY(hipMemcpy(s->act, act_save.data(), s->Bp, hipMemcpyHostToDevice));
    return drain_profile(s);
}

// one step of every replica, with STOP_NONE bookkeeping that is restored afterwards
static int single_step(odesat_solver *s, bool adaptive, double tol, double dt, double zeta, double *dt_io,
                       uint8_t *allsat) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (adaptive && std::isnan(tol)) return fail(ODESAT_EINVAL, "tol is NaN");
    if ((rc = ensure_w(s))) return rc;
    if (adaptive && (rc = ensure_scratch(s))) return rc;
    if ((rc = set_stop(s, INT_MAX))) return rc;
    std::vector<uint8_t> act_save(s->Bp);
    HIP_TRY(hipMemcpy(act_save.data(), s->act, s->Bp, hipMemcpyDeviceToHost));
    if ((rc = set_all_active(s))) return rc;
    if (adaptive && dt_io && (rc = put_dt(s, dt_io, 0.01))) return rc;
    std::vector<int64_t> sat_save(s->Bp), done_save(s->Bp), minus = host_i64(s->Bp, -1);
    HIP_TRY(hipMemcpy(sat_save.data(), s->sat_step, s->Bp * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(done_save.data(), s->steps_done, s->Bp * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(s->sat_step, minus.data(), s->Bp * 8, hipMemcpyHostToDevice));
    if ((rc = dispatch_step(s, 0, adaptive, dt, zeta, tol, ODESAT_STOP_NONE, 0, s->G))) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    std::vector<int64_t> sat(s->Bp);
    HIP_TRY(hipMemcpy(sat.data(), s->sat_step, s->Bp * 8, hipMemcpyDeviceToHost));
    if (allsat)
        for (int64_t r = 0; r < s->B; ++r) allsat[r] = sat[r] == 0;
    if (adaptive && dt_io && (rc = get_dt(s, dt_io))) return rc;
    HIP_TRY(hipMemcpy(s->act, act_save.data(), s->Bp, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->sat_step, sat_save.data(), s->Bp * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->steps_done, done_save.data(), s->Bp * 8, hipMemcpyHostToDevice));
    return drain_profile(s);
}

extern "C" int odesat_euler_step_fixed(odesat_solver *s, double dt, double zeta, uint8_t *allsat) {
    return single_step(s, false, 0.0, dt, zeta, nullptr, allsat);
}

extern "C" int odesat_euler_step(odesat_solver *s, double tol, double *dt, double zeta, uint8_t *allsat) {
    return single_step(s, true, tol, 0.0, zeta, dt, allsat);
}

extern "C" int odesat_simulate(odesat_solver *s, const odesat_params *p, int64_t *first_sat_step,
                               int64_t *steps_done, double *dt_out, int64_t *steps_run) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (!p) return fail(ODESAT_EINVAL, "null params");
    if (p->max_steps <= 0 || p->max_steps > INT_MAX - 1)
        return fail(ODESAT_EINVAL, "max_steps must be in [1, 2^31-2] (unbounded runs are refused)");
    if (p->stop != ODESAT_STOP_EACH && p->stop != ODESAT_STOP_ANY && p->stop != ODESAT_STOP_NONE)
        return fail(ODESAT_EINVAL, "bad stop policy");
    const bool adaptive = p->adaptive != 0;
    const double tol = p->tol;
    const double zeta = p->zeta < 0 ? default_zeta(s) : p->zeta;
    if ((rc = ensure_w(s))) return rc;
    if (adaptive && (rc = ensure_scratch(s))) return rc;
    if ((rc = set_stop(s, INT_MAX))) return rc;
    {   // per-call bookkeeping: sat step / steps done restart; adaptive dt restarts at 0.01 (:205)
        std::vector<int64_t> minus = host_i64(s->Bp, -1), zero = host_i64(s->Bp, 0);
        HIP_TRY(hipMemcpy(s->sat_step, minus.data(), s->Bp * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(s->steps_done, zero.data(), s->Bp * 8, hipMemcpyHostToDevice));
        if ((rc = set_all_active(s))) return rc;
        if (adaptive && (rc = put_dt(s, nullptr, 0.01))) return rc;
    }
    const int poll = p->poll_interval > 0 ? p->poll_interval : 32;
    int32_t *h_stop = nullptr;
    uint8_t *h_act = nullptr;
    HIP_TRY(hipHostMalloc((void **)&h_stop, sizeof(int32_t)));
    if (hipHostMalloc((void **)&h_act, s->Bp) != hipSuccess) {
        (void)hipHostFree(h_stop);
        return fail(ODESAT_ENOMEM, "hipHostMalloc failed");
    }
    // Schedule: replicas are independent, so with STOP_EACH / STOP_NONE the batch may be stepped
    // chunk by chunk (all steps of one chunk, then the next): one chunk's state + contribution buffer
    // stays resident in the Infinity Cache across steps.  STOP_ANY needs lock-step (step-major).
    const bool chunk_major = p->stop != ODESAT_STOP_ANY &&
                             (s->schedule == ODESAT_SCHED_CHUNK_MAJOR ||
                              (s->schedule == ODESAT_SCHED_AUTO && s->G > s->chunk_groups));
    const int span = chunk_major ? s->chunk_groups : s->G;
    int64_t t_run = 0;
    rc = ODESAT_OK;
    for (int gA = 0; gA < s->G && rc == ODESAT_OK; gA += span) {
        const int gB = std::min(s->G, gA + span);
        const int64_t r0 = (int64_t)gA * s->W, r1 = std::min<int64_t>((int64_t)gB * s->W, s->B);
        int64_t t = 0;
        for (; t < p->max_steps; ++t) {
            if ((rc = dispatch_step(s, (int)t, adaptive, p->dt, zeta, tol, p->stop, gA, gB))) break;
            if (p->stop != ODESAT_STOP_NONE && (t + 1) % poll == 0 && t + 1 < p->max_steps) {
                // poll the stop condition (results are exact regardless: later launches are no-ops)
                if (hipMemcpyAsync(h_stop, s->stop, 4, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
                    hipMemcpyAsync(h_act + r0, s->act + r0, r1 - r0, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
                    hipStreamSynchronize(s->stream) != hipSuccess) {
                    rc = fail(ODESAT_EDEVICE, "poll failed");
                    break;
                }
                if (p->stop == ODESAT_STOP_ANY && *h_stop != INT_MAX) { ++t; break; }
                if (p->stop == ODESAT_STOP_EACH) {
                    bool any = false;
                    for (int64_t r = r0; r < r1 && !any; ++r) any = h_act[r] != 0;
                    if (!any) { ++t; break; }
                }
            }
        }
        t_run = std::max(t_run, t);
    }
    (void)hipHostFree(h_stop);
    (void)hipHostFree(h_act);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (steps_run) *steps_run = t_run;
    if (first_sat_step) HIP_TRY(hipMemcpy(first_sat_step, s->sat_step, s->B * 8, hipMemcpyDeviceToHost));
    if (steps_done) HIP_TRY(hipMemcpy(steps_done, s->steps_done, s->B * 8, hipMemcpyDeviceToHost));
    if (dt_out) {
        if (!adaptive) {
            for (int64_t r = 0; r < s->B; ++r) dt_out[r] = p->dt;
        } else if ((rc = get_dt(s, dt_out))) {
            return rc;
        }
    }
    return s->profile ? ODESAT_OK : drain_profile(s);
}

extern "C" int odesat_synchronize(odesat_solver *s) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

extern "C" int odesat_profile_enable(odesat_solver *s, int enable) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if ((rc = drain_profile(s))) return rc;
    s->profile = enable != 0;
    for (int k = 0; k < 3; ++k) {
        s->prof_ms[k] = 0;
        s->prof_n[k] = 0;
    }
    return ODESAT_OK;
}

extern "C" int odesat_profile_read(odesat_solver *s, double *ms, int64_t *launches) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if ((rc = drain_profile(s))) return rc;
    for (int k = 0; k < 3; ++k) {
        if (ms) ms[k] = s->prof_ms[k];
        if (launches) launches[k] = s->prof_n[k];
    }
    return ODESAT_OK;
}

extern "C" int64_t odesat_clause_kernel_bytes(const odesat_solver *s) {
    // per step over the whole batch: v gathered once (4n), xs/xl read + written (16m), in dtype
    if (!s) return -1;
    return (int64_t)s->B * (s->n + 4 * s->m) * (int64_t)s->tsize;
}
