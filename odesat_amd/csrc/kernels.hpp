// kernels.hpp -- gfx950 device code of the integrator (included once, by odesat_hip.hip).
//
// Layout.  Every per-item array is replica-innermost in groups of W replicas:
// voltages V[g][i][W], clause memories C[g][c][W][2] (xs, xl interleaved per replica, so one clause
// gather of a 16-replica group is one whole 128-byte line), replica r = g*W + j.  A wave covers one "row": LW lanes per
// item, VEC contiguous replicas per lane, W = LW*VEC, 64/LW items per row.  The state (v, xs, xl)
// is double-buffered: group g's current state is in buffer par[g]; a step reads it and writes the
// other buffer (replicas that do not step copy their state across), then k_status flips par[g].
//
// Two algorithms per Euler step (system.rs:141-154 fixed, :111-139 adaptive):
//   FUSED (default)  k_step: one launch per RHS.  Lane = (variable i, replica r): for each incident
//       clause of i in clause order (system.rs:35 Zip order), gather the clause's literal voltages,
//       strict-< min / second-min, C, and add i's contribution G/R (system.rs:43-80) to dv -- the
//       reference's exact accumulation order, so results are bit-identical to the CPU oracle.  The
//       clause's FIRST literal owns the xs/xl update (system.rs:84-85, 94-95) and the sat flag
//       (:88).  No contribution buffer; voltages are re-read from the XCD's L2 (XCD-aware group
//       placement keeps a group's voltage table on one XCD).
//   TWOPASS  k_clause_u / k_clause then k_variable: per clause, write each literal's contribution
//       to a variable-major buffer w; per variable, sum its slots in order.  Kept for A/B.
// FP contraction is OFF in this translation unit: every + and * rounds exactly as written.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/odesat.h"
#include "callio.hpp"

namespace odk {

// ------------------------------------------------------------------------------------------------
// helpers
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

// Non-temporal forms for data with no reuse in the XCD's L2 (clause memories gathered at random,
// state written for the next step): they must not evict the voltage table the gathers hit.
template <typename T, int N> __device__ __forceinline__ Vec<T, N> ldv_nt(const T *p) {
    Vec<T, N> x;
#pragma unroll
    for (int k = 0; k < N; ++k) x.e[k] = __builtin_nontemporal_load(p + k);
    return x;
}
template <typename T, int N> __device__ __forceinline__ void stv_nt(T *p, const Vec<T, N> &x) {
#pragma unroll
    for (int k = 0; k < N; ++k) __builtin_nontemporal_store(x.e[k], p + k);
}

// The topology arrays are never written by a kernel: reading them through the constant address
// space lets wave-uniform indices become scalar (s_load) loads on the scalar cache.
typedef const __attribute__((address_space(4))) int32_t cint32;
__device__ __forceinline__ int32_t ldc(const int32_t *p, size_t i) { return ((cint32 *)p)[i]; }
// 3-SAT incidence record: x = clause << 2 | own literal position, y/z/w = the clause's literals
struct alignas(16) Inc {
    int32_t x, y, z, w;
};
__device__ __forceinline__ Inc ldc4(const Inc *p, size_t i) {
    typedef const __attribute__((address_space(4))) int32_t c32;
    const c32 *q = (const c32 *)(p + i);
    return Inc{q[0], q[1], q[2], q[3]};
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

template <typename T> struct KArgs {
    const int32_t *__restrict__ cptr;  // [m+1]
    const int32_t *__restrict__ lits;  // [L] var<<1 | neg, file order
    const int32_t *__restrict__ wpos;  // [L] slot -> variable-major position (TWOPASS)
    const int32_t *__restrict__ vptr;  // [n+1] variable -> first variable-major position
    const int32_t *__restrict__ pc;    // [L] variable-major position -> clause (FUSED)
    const int32_t *__restrict__ ps;    // [L] variable-major position -> slot (FUSED)
    const Inc *__restrict__ inc;       // [L] 3-SAT incidence records, variable-major (FUSED)
    T *v0, *v1;                        // double-buffered voltages [G][n][W]
    T *c0, *c1;                        // double-buffered clause memories [G][m][W][2] (xs, xl)
    const uint8_t *par;                // [G] which buffer holds group g's current state
    T *w;                              // contributions [chunk groups][L][W] (TWOPASS)
    T *vh, *vf;                        // half / full voltages (adaptive); DERIV: vh = dv
    T *ch, *cf;                        // half / full memories (adaptive); DERIV: ch = (dxs, dxl)
    T *dtr;                            // [Bp] per-replica adaptive dt
    typename Bits<T>::U *err;          // [Bp] max_error bits (non-negative floats order as ints)
    uint32_t *unsat;                   // [Bp] 1 = some clause had C >= gamma this step
    uint8_t *act;                      // [Bp] replica still stepping
    const int32_t *stop;               // first stop step (INT_MAX = none)
    int32_t n, m, L;
    int32_t g0, ng;                    // group range of this launch
    int32_t rows;                      // rows (of 64/LW items) per wave
    int32_t tiles;                     // waves per group
    int32_t bpg;                       // blocks per group (tiles / 4, rounded up)
    int32_t xmode;                     // block -> (group, tile) placement, see Geo::init
    int32_t step;
    T dt, zeta, xl_max;
};

constexpr int WAVES_PER_BLOCK = 4;


// Per-wave geometry.  xmode 1 (ng a multiple of 8) and 2 (ng divides 8) place all blocks of a
// group on the XCDs of one residue class of blockIdx mod 8 (blocks are dealt round-robin over the 8
// XCDs), so a group's voltage table is gathered from one XCD's L2.  Placement is a speed choice
// only: every mapping covers every (group, tile) exactly once.
template <int LW, int VEC> struct Geo {
    static constexpr int W = LW * VEC;   // replicas per group
    static constexpr int IPR = 64 / LW;  // items per wave row
    int gl, g, tile, isub, lin;
    size_t off;  // element offset of this lane's first replica inside an item row
    int r0;      // this lane's first replica
    template <typename A> __device__ __forceinline__ bool init(const A &a) {
        const int lane = threadIdx.x & 63;
        const int b = blockIdx.x;
        int tb;
        if (a.xmode == 1) {
            const int x = b & 7, k = b >> 3;
            gl = x + 8 * (k / a.bpg);
            tb = k % a.bpg;
        } else if (a.xmode == 2) {
            const int sh = 8 / a.ng, x = b & 7, k = b >> 3;
            gl = x % a.ng;
            tb = k * sh + x / a.ng;
        } else {
            gl = b / a.bpg;
            tb = b % a.bpg;
        }
        if (gl >= a.ng || tb >= a.bpg) return false;
        tile = tb * WAVES_PER_BLOCK + (threadIdx.x >> 6);
        if (tile >= a.tiles) return false;
        g = a.g0 + gl;
        lin = lane % LW;
        isub = lane / LW;
        off = (size_t)lin * VEC;
        r0 = g * W + lin * VEC;
        return true;
    }
};

template <typename T> struct Bufs {
    T *vcur, *vnxt, *ccur, *cnxt;
    __device__ __forceinline__ Bufs(const KArgs<T> &a, int g) {
        const bool p = a.par[g] != 0;
        vcur = p ? a.v1 : a.v0;
        vnxt = p ? a.v0 : a.v1;
        ccur = p ? a.c1 : a.c0;
        cnxt = p ? a.c0 : a.c1;
    }
};

// The per-replica prologue.  FUSED kernels and clause kernels see `act` (and, for the second
// adaptive half, the first RHS's sat flag: an allsat replica takes no step, system.rs:122);
// k_variable of the first adaptive half also needs that flag.
template <typename T, int VEC, int MODE, bool SAW_RHS>
__device__ __forceinline__ bool lane_state(const KArgs<T> &a, int r0, bool (&on)[VEC], bool &all_on,
                                           T (&h)[VEC]) {
    bool any = false;
    all_on = true;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        bool o = a.act[r0 + k] != 0;
        if (MODE == M_ADB || (SAW_RHS && MODE == M_ADA)) o = o && a.unsat[r0 + k] != 0;
        on[k] = o;
        any = any || o;
        all_on = all_on && o;
        h[k] = (MODE == M_ADA || MODE == M_ADB) ? a.dtr[r0 + k] : a.dt;
    }
    return __any(any);
}

// :84-85 memory derivatives, then (by mode) the update_state of xs / xl (:94-95), the adaptive
// full / half candidates (:124-128) or the second half step and its max_error terms (:130-132).
// `mem` holds the lane's VEC (xs, xl) pairs; ci is the element offset of the lane's first pair.
// Lanes that do not step copy their current memories into the next buffer.
template <typename T, int VEC, int MODE>
__device__ __forceinline__ void clause_update(const KArgs<T> &a, const Bufs<T> &bf, size_t ci,
                                              const T (&C)[VEC], const Vec<T, 2 * VEC> &mem,
                                              const T (&h)[VEC], const bool (&on)[VEC], bool all_on,
                                              T (&e)[VEC]) {
    const T one = (T)1.0, eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001;
    Vec<T, 2 * VEC> o1, o2;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const T xs_m = mem.e[2 * k], xl_m = mem.e[2 * k + 1];
        const T dxs = (T)20.0 * (xs_m + eps) * (C[k] - (T)0.25);  // :84
        const T dxl = (T)5.0 * (C[k] - (T)0.05);                  // :85
        const T half = (T)0.5 * h[k];
        if (MODE == M_DERIV) {
            o1.e[2 * k] = dxs;
            o1.e[2 * k + 1] = dxl;
        } else if (MODE == M_FIXED) {
            o1.e[2 * k] = on[k] ? dmin(dmax(xs_m + h[k] * dxs, eps), xs_hi) : xs_m;
            o1.e[2 * k + 1] = on[k] ? dmin(dmax(xl_m + h[k] * dxl, one), a.xl_max) : xl_m;
        } else if (MODE == M_ADA) {
            o1.e[2 * k] = dmin(dmax(xs_m + h[k] * dxs, eps), xs_hi);         // full-step clone
            o1.e[2 * k + 1] = dmin(dmax(xl_m + h[k] * dxl, one), a.xl_max);
            o2.e[2 * k] = dmin(dmax(xs_m + half * dxs, eps), xs_hi);         // first half step
            o2.e[2 * k + 1] = dmin(dmax(xl_m + half * dxl, one), a.xl_max);
        } else {
            o1.e[2 * k] = dmin(dmax(xs_m + half * dxs, eps), xs_hi);         // second half step
            o1.e[2 * k + 1] = dmin(dmax(xl_m + half * dxl, one), a.xl_max);
        }
    }
    if (MODE == M_DERIV) {
        stv<T, 2 * VEC>(a.ch + ci, o1);
    } else if (MODE == M_FIXED) {
        stv_nt<T, 2 * VEC>(bf.cnxt + ci, o1);
    } else if (MODE == M_ADA) {
        stv<T, 2 * VEC>(a.cf + ci, o1);
        stv<T, 2 * VEC>(a.ch + ci, o2);
    } else {
        const Vec<T, 2 * VEC> f = ldv<T, 2 * VEC>(a.cf + ci);
#pragma unroll
        for (int k = 0; k < VEC; ++k)  // :101-108 max_error terms (stepping replicas only)
            if (on[k])
                e[k] = dmax(e[k], dmax(dabs(f.e[2 * k] - o1.e[2 * k]), dabs(f.e[2 * k + 1] - o1.e[2 * k + 1])));
        if (!all_on) {  // replicas that take no step keep their state
            const Vec<T, 2 * VEC> c = ldv<T, 2 * VEC>(bf.ccur + ci);
#pragma unroll
            for (int k = 0; k < 2 * VEC; ++k) o1.e[k] = on[k / 2] ? o1.e[k] : c.e[k];
        }
        stv_nt<T, 2 * VEC>(bf.cnxt + ci, o1);
    }
}

// :96 v update by mode, from the variable's current voltage v_old and its dv.
template <typename T, int VEC, int MODE>
__device__ __forceinline__ void variable_update(const KArgs<T> &a, const Bufs<T> &bf, size_t vi,
                                                const Vec<T, VEC> &v_old, const T (&dv)[VEC],
                                                const T (&h)[VEC], const bool (&on)[VEC], bool all_on,
                                                T (&e)[VEC]) {
    Vec<T, VEC> o1, o2;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const T half = (T)0.5 * h[k];
        if (MODE == M_DERIV) {
            o1.e[k] = dv[k];
        } else if (MODE == M_FIXED) {
            o1.e[k] = on[k] ? dmin(dmax(v_old.e[k] + h[k] * dv[k], (T)-1.0), (T)1.0) : v_old.e[k];
        } else if (MODE == M_ADA) {
            o1.e[k] = dmin(dmax(v_old.e[k] + h[k] * dv[k], (T)-1.0), (T)1.0);   // full-step clone
            o2.e[k] = dmin(dmax(v_old.e[k] + half * dv[k], (T)-1.0), (T)1.0);  // first half step
        } else {
            o1.e[k] = dmin(dmax(v_old.e[k] + half * dv[k], (T)-1.0), (T)1.0);  // second half step
        }
    }
    if (MODE == M_DERIV) {
        stv<T, VEC>(a.vh + vi, o1);
    } else if (MODE == M_FIXED) {
        stv_nt<T, VEC>(bf.vnxt + vi, o1);
    } else if (MODE == M_ADA) {
        stv<T, VEC>(a.vf + vi, o1);
        stv<T, VEC>(a.vh + vi, o2);
    } else {
        const Vec<T, VEC> f = ldv<T, VEC>(a.vf + vi);
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            if (on[k]) e[k] = dmax(e[k], dabs(f.e[k] - o1.e[k]));
        if (!all_on) {
            const Vec<T, VEC> c = ldv<T, VEC>(bf.vcur + vi);
#pragma unroll
            for (int k = 0; k < VEC; ++k) o1.e[k] = on[k] ? o1.e[k] : c.e[k];
        }
        stv_nt<T, VEC>(bf.vnxt + vi, o1);
    }
}

template <typename T, int VEC, int MODE>
__device__ __forceinline__ void flush_flags(const KArgs<T> &a, int r0, const bool (&on)[VEC],
                                            const bool (&uns)[VEC], const T (&e)[VEC]) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        if (MODE != M_ADB) {
            if (uns[k]) a.unsat[r0 + k] = 1u;
        } else if (on[k]) {
            atomicMax(&a.err[r0 + k], tobits(e[k]));
        }
    }
}

// dst[i] = src[i] for i = first, first + stride, ... < count (dst in LDS): U loads issued together, then
// their U stores -- one memory round trip per U elements instead of one per element (a plain loop
// waits for each load before its store).
template <int U, typename T>
__device__ __forceinline__ void copy_to_lds(T *dst, const T *src, int first, int count, int stride) {
    if (count <= 0) return;
    for (int i0 = first; i0 < count; i0 += stride * U) {
        T x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = src[min(i0 + u * stride, count - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * stride < count) dst[i0 + u * stride] = x[u];
    }
}

// strict-< min / second-min update (system.rs:50-55), branch-free
template <typename T> __device__ __forceinline__ void minsec(T val, T &mn, T &sec) {
    const bool lt = val < mn;
    sec = lt ? mn : (val < sec ? val : sec);
    mn = lt ? val : mn;
}

// ------------------------------------------------------------------------------------------------
// The 3-SAT incidence stream of one wave (LW = 64: the wave's W replicas of variables [i0, i1)).
// The wave walks the concatenated incidence lists of its variables as ONE stream of batches of RB
// incidences, double-buffered: batch k+1's records, voltage gathers and memory row are in flight
// while batch k computes.  Variable boundaries are crossed inside a batch (uniform branch): the
// finished variable's v update is written and the next variable's row (prefetched one variable
// ahead) becomes current.  Accumulation order per variable is unchanged (position order).
// ------------------------------------------------------------------------------------------------
template <typename T, int VEC, int RB> struct Batch {
    Inc rec[RB];
    Vec<T, VEC> vv[RB][3];
    Vec<T, 2 * VEC> mem[RB];
};

template <typename T, int W, int VEC, int MODE, int RB>
__device__ __forceinline__ void stream_rows3(const KArgs<T> &a, const Bufs<T> &bf, const T *__restrict__ V,
                                             const T *CM, size_t vbase, size_t cbase, int i0, int i1,
                                             const T (&h)[VEC], const bool (&on)[VEC], bool all_on,
                                             bool (&uns)[VEC], T (&e)[VEC]) {
    const T one = (T)1.0, halfc = (T)0.5;
    const int P0 = ldc(a.vptr, i0), P1 = ldc(a.vptr, i1);
    int cur = i0;
    int cur_end = ldc(a.vptr, i0 + 1);
    int next_end = i0 + 1 < i1 ? ldc(a.vptr, i0 + 2) : P1;
    Vec<T, VEC> v_i = ldv<T, VEC>(V + vbase + (size_t)i0 * W);
    Vec<T, VEC> v_nx = ldv<T, VEC>(V + vbase + (size_t)(i0 + 1 < i1 ? i0 + 1 : i0) * W);
    T dv[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) dv[k] = (T)0.0;  // :33

    auto finish = [&]() {  // v update of the current variable, then advance (prefetching one ahead)
        variable_update<T, VEC, MODE>(a, bf, vbase + (size_t)cur * W, v_i, dv, h, on, all_on, e);
        ++cur;
        v_i = v_nx;
        cur_end = next_end;
        if (cur + 1 < i1) {
            next_end = ldc(a.vptr, cur + 2);
            v_nx = ldv<T, VEC>(V + vbase + (size_t)(cur + 1) * W);
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) dv[k] = (T)0.0;
    };
    auto load_recs = [&](Inc (&r)[RB], int q0) {
#pragma unroll
        for (int b = 0; b < RB; ++b) r[b] = ldc4(a.inc, q0 + b < P1 ? q0 + b : P1 - 1);
    };
    auto issue = [&](Batch<T, VEC, RB> &B, const Inc (&r)[RB]) {
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            B.rec[b] = r[b];
            B.vv[b][0] = ldv<T, VEC>(V + vbase + (size_t)(r[b].y >> 1) * W);
            B.vv[b][1] = ldv<T, VEC>(V + vbase + (size_t)(r[b].z >> 1) * W);
            B.vv[b][2] = ldv<T, VEC>(V + vbase + (size_t)(r[b].w >> 1) * W);
        }
#pragma unroll
        for (int b = 0; b < RB; ++b) B.mem[b] = ldv_nt<T, 2 * VEC>(CM + cbase + (size_t)(r[b].x >> 2) * W * 2);
    };
    auto compute = [&](const Batch<T, VEC, RB> &B, int q0) {
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            const int q = q0 + b;
            if (q < P1) {
            while (q >= cur_end) finish();  // crossed into the next variable(s) (degree-0 ones too)
            const int lit[3] = {B.rec[b].y, B.rec[b].z, B.rec[b].w};
            const int own = B.rec[b].x & 3;
            const int c = B.rec[b].x >> 2;
            const int lo = own == 0 ? lit[0] : (own == 1 ? lit[1] : lit[2]);
            const T qo = (lo & 1) ? (T)-1.0 : (T)1.0;
            T C[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                T mn = inf_v<T>(), sec = inf_v<T>();
#pragma unroll
                for (int j = 0; j < 3; ++j) {  // :43-57
                    const T qj = (lit[j] & 1) ? (T)-1.0 : (T)1.0;
                    minsec(one - qj * B.vv[b][j].e[k], mn, sec);
                }
                C[k] = halfc * mn;  // :60
                const T vio = own == 0 ? B.vv[b][0].e[k] : (own == 1 ? B.vv[b][1].e[k] : B.vv[b][2].e[k]);
                const T val = one - qo * vio;
                const T g_ = halfc * qo * (val != mn ? mn : sec);                    // :64-70
                const T xs_m = B.mem[b].e[2 * k], xl_m = B.mem[b].e[2 * k + 1];
                const T t = xl_m * xs_m;
                const T tr = (one + a.zeta * xl_m) * (one - xs_m);
                const T r_ = (C[k] == one - qo * vio) ? halfc * (qo - vio) : (T)0.0;  // :73-77
                dv[k] += t * g_ + tr * r_;                                            // :80
                if (MODE != M_ADB && own == 0) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));
            }
            if (own == 0)  // the clause's first literal owns its memories
                clause_update<T, VEC, MODE>(a, bf, cbase + (size_t)c * W * 2, C, B.mem[b], h, on, all_on, e);
            }
        }
    };

    if (P0 < P1) {
        Batch<T, VEC, RB> A, Bb;
        Inc rn[RB];
        int qa = P0, qb = P0 + RB;
        load_recs(rn, qa);
        issue(A, rn);
        if (qb < P1) load_recs(rn, qb);
        for (;;) {
            const bool hb = qb < P1;
            if (hb) {
                issue(Bb, rn);
                if (qb + RB < P1) load_recs(rn, qb + RB);
            }
            compute(A, qa);
            if (!hb) break;
            qa = qb + RB;
            const bool ha = qa < P1;
            if (ha) {
                issue(A, rn);
                if (qa + RB < P1) load_recs(rn, qa + RB);
            }
            compute(Bb, qb);
            if (!ha) break;
            qb = qa + RB;
        }
    }
    while (cur < i1) finish();  // the last variable(s), degree-0 tails included
}

// ------------------------------------------------------------------------------------------------
// k_step (FUSED): one RHS (+ update) per launch, variable-major.  K > 0: every clause has K
// literals (random k-SAT) -- RB incidences per batch, all their loads issued before the first use.
// K == 0: mixed clause widths, one incidence at a time.
// ------------------------------------------------------------------------------------------------
#ifndef KSTEP_WAVES_PER_EU  // tuning: minimum waves per SIMD the compiler must leave room for (0 = its choice)
#define KSTEP_WAVES_PER_EU 0
#endif
#if KSTEP_WAVES_PER_EU > 0
#define KSTEP_ATTR __attribute__((amdgpu_waves_per_eu(KSTEP_WAVES_PER_EU)))
#else
#define KSTEP_ATTR
#endif
template <typename T, int LW, int VEC, int MODE, int K, int RB = 4>
__global__ __launch_bounds__(256) KSTEP_ATTR void k_step(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    static_assert(K == 0 || K == 3, "incidence records are laid out for 3-SAT");
    constexpr int KK = K > 0 ? K : 1;
    G_ geo;
    if (!geo.init(a)) return;
    if (*a.stop < a.step) return;  // ODESAT_STOP_ANY already triggered
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, false>(a, geo.r0, on, all_on, h)) return;
    const Bufs<T> bf(a, geo.g);
    const T *__restrict__ V = (MODE == M_ADB) ? a.vh : bf.vcur;
    const T *CM = (MODE == M_ADB) ? a.ch : bf.ccur;
    const T one = (T)1.0, halfc = (T)0.5;
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const size_t cbase = ((size_t)geo.g * a.m * W + geo.off) * 2;
    bool uns[VEC];
    T e[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        uns[k] = false;
        e[k] = (T)0.0;
    }
    if constexpr (LW == 64 && K == 3) {
        const int i0 = __builtin_amdgcn_readfirstlane(geo.tile * a.rows);
        const int i1 = min(i0 + a.rows, a.n);
        if (i0 < i1) stream_rows3<T, W, VEC, MODE, RB>(a, bf, V, CM, vbase, cbase, i0, i1, h, on, all_on, uns, e);
        flush_flags<T, VEC, MODE>(a, geo.r0, on, uns, e);
        return;
    }
    for (int row = 0; row < a.rows; ++row) {
        int i = (geo.tile * a.rows + row) * IPR + geo.isub;
        if (LW == 64) i = __builtin_amdgcn_readfirstlane(i);
        if (i >= a.n) break;
        const int p0 = ldc(a.vptr, i), p1 = ldc(a.vptr, i + 1);
        const size_t vi = vbase + (size_t)i * W;
        const Vec<T, VEC> v_i = ldv<T, VEC>(V + vi);
        T dv[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) dv[k] = (T)0.0;  // :33
        if (K > 0) {
            // 3-SAT: one 16-byte incidence record per (variable, clause) feeds every load of the
            // incidence; the records of the next batch are fetched while this batch computes.
            Inc rec[RB], nxt[RB];
#pragma unroll
            for (int b = 0; b < RB; ++b) nxt[b] = ldc4(a.inc, p0 + b < p1 ? p0 + b : p1 - 1);
            for (int p = p0; p < p1; p += RB) {
#pragma unroll
                for (int b = 0; b < RB; ++b) rec[b] = nxt[b];
                Vec<T, VEC> vv[RB][KK];
                Vec<T, 2 * VEC> mem[RB];
#pragma unroll
                for (int b = 0; b < RB; ++b) {
                    vv[b][0] = ldv<T, VEC>(V + vbase + (size_t)(rec[b].y >> 1) * W);
                    if (KK > 1) vv[b][KK > 1 ? 1 : 0] = ldv<T, VEC>(V + vbase + (size_t)(rec[b].z >> 1) * W);
                    if (KK > 2) vv[b][KK > 2 ? 2 : 0] = ldv<T, VEC>(V + vbase + (size_t)(rec[b].w >> 1) * W);
                }
#pragma unroll
                for (int b = 0; b < RB; ++b)
                    mem[b] = ldv_nt<T, 2 * VEC>(CM + cbase + (size_t)(rec[b].x >> 2) * W * 2);
#pragma unroll
                for (int b = 0; b < RB; ++b) {
                    const int q = p + RB + b;
                    nxt[b] = ldc4(a.inc, q < p1 ? q : p1 - 1);
                }
#pragma unroll
                for (int b = 0; b < RB; ++b) {
                    if (p + b >= p1) continue;
                    const int lit[3] = {rec[b].y, rec[b].z, rec[b].w};
                    const int own = rec[b].x & 3;
                    const int c = rec[b].x >> 2;
                    // the incidence's own literal (select chain, no indexed register array)
                    int lo = lit[0];
                    Vec<T, VEC> vo = vv[b][0];
#pragma unroll
                    for (int j = 1; j < KK; ++j)
                        if (own == j) {
                            lo = lit[j];
                            vo = vv[b][j];
                        }
                    const T qo = (lo & 1) ? (T)-1.0 : (T)1.0;
                    T C[VEC];
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        T mn = inf_v<T>(), sec = inf_v<T>();
#pragma unroll
                        for (int j = 0; j < KK; ++j) {  // :43-57
                            const T q = (lit[j] & 1) ? (T)-1.0 : (T)1.0;
                            minsec(one - q * vv[b][j].e[k], mn, sec);
                        }
                        C[k] = halfc * mn;  // :60
                        const T xs_m = mem[b].e[2 * k], xl_m = mem[b].e[2 * k + 1];
                        const T t = xl_m * xs_m;
                        const T tr = (one + a.zeta * xl_m) * (one - xs_m);
                        const T vio = vo.e[k];
                        const T val = one - qo * vio;
                        const T g_ = halfc * qo * (val != mn ? mn : sec);                    // :64-70
                        const T r_ = (C[k] == one - qo * vio) ? halfc * (qo - vio) : (T)0.0;  // :73-77
                        dv[k] += t * g_ + tr * r_;                                            // :80
                        if (MODE != M_ADB && own == 0) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));
                    }
                    if (own == 0)  // the clause's first literal owns its memories
                        clause_update<T, VEC, MODE>(a, bf, cbase + (size_t)c * W * 2, C, mem[b], h, on, all_on, e);
                }
            }
        } else {
            for (int p = p0; p < p1; ++p) {
                const int c = ldc(a.pc, p), s_own = ldc(a.ps, p);
                const int s0 = ldc(a.cptr, c), s1 = ldc(a.cptr, c + 1);
                const size_t ci = cbase + (size_t)c * W * 2;
                const Vec<T, 2 * VEC> mem = ldv<T, 2 * VEC>(CM + ci);
                T mn[VEC], sec[VEC], C[VEC];
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    mn[k] = inf_v<T>();
                    sec[k] = inf_v<T>();
                }
                int lo = 0;
                Vec<T, VEC> vo{};
                for (int s = s0; s < s1; ++s) {  // :43-57
                    const int lit = ldc(a.lits, s);
                    const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
                    const Vec<T, VEC> vv = ldv<T, VEC>(V + vbase + (size_t)(lit >> 1) * W);
                    if (s == s_own) {
                        lo = lit;
                        vo = vv;
                    }
#pragma unroll
                    for (int k = 0; k < VEC; ++k) minsec(one - q * vv.e[k], mn[k], sec[k]);
                }
                const T qo = (lo & 1) ? (T)-1.0 : (T)1.0;
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    C[k] = halfc * mn[k];
                    const T xs_m = mem.e[2 * k], xl_m = mem.e[2 * k + 1];
                    const T t = xl_m * xs_m;
                    const T tr = (one + a.zeta * xl_m) * (one - xs_m);
                    const T val = one - qo * vo.e[k];
                    const T g_ = halfc * qo * (val != mn[k] ? mn[k] : sec[k]);
                    const T r_ = (C[k] == one - qo * vo.e[k]) ? halfc * (qo - vo.e[k]) : (T)0.0;
                    dv[k] += t * g_ + tr * r_;
                    if (MODE != M_ADB && s_own == s0) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));
                }
                if (s_own == s0) clause_update<T, VEC, MODE>(a, bf, ci, C, mem, h, on, all_on, e);
            }
        }
        variable_update<T, VEC, MODE>(a, bf, vi, v_i, dv, h, on, all_on, e);
    }
    flush_flags<T, VEC, MODE>(a, geo.r0, on, uns, e);
}

// Clauses without literals (empty DIMACS lines) have no variable to own them: their memories and
// their (never satisfied) flag are handled here.  Launched only when such clauses exist.
template <typename T, int LW, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_empty_clauses(KArgs<T> a, const int32_t *__restrict__ list, int count) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int per_group = count * LW;
    const int gl = tid / per_group;
    if (gl >= a.ng) return;
    if (*a.stop < a.step) return;
    const int rem = tid - gl * per_group;
    const int c = ldc(list, rem / LW);
    const int lin = rem % LW;
    const int g = a.g0 + gl;
    const int r0 = g * W + lin * VEC;
    bool on[VEC], all_on;
    T h[VEC];
    bool any = false;
    all_on = true;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        bool o = a.act[r0 + k] != 0;
        if (MODE == M_ADB) o = o && a.unsat[r0 + k] != 0;
        on[k] = o;
        any = any || o;
        all_on = all_on && o;
        h[k] = (MODE == M_ADA || MODE == M_ADB) ? a.dtr[r0 + k] : a.dt;
    }
    if (!any) return;
    const Bufs<T> bf(a, g);
    const T *CM = (MODE == M_ADB) ? a.ch : bf.ccur;
    const size_t ci = (((size_t)g * a.m + c) * W + (size_t)lin * VEC) * 2;
    const Vec<T, 2 * VEC> mem = ldv<T, 2 * VEC>(CM + ci);
    T C[VEC], e[VEC];
    bool uns[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        C[k] = (T)0.5 * inf_v<T>();  // min over no literal = +inf (system.rs:43,60)
        e[k] = (T)0.0;
        uns[k] = on[k];
    }
    clause_update<T, VEC, MODE>(a, bf, ci, C, mem, h, on, all_on, e);
    flush_flags<T, VEC, MODE>(a, r0, on, uns, e);
}

// ------------------------------------------------------------------------------------------------
// TWOPASS: k_clause_u / k_clause (system.rs:35-90 per clause, contributions to w) + k_variable
// ------------------------------------------------------------------------------------------------
template <typename T, int LW, int VEC, int MODE, int K>
__global__ __launch_bounds__(256) void k_clause_u(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    constexpr int RB = VEC >= 4 ? 2 : 4;
    G_ geo;
    if (!geo.init(a)) return;
    if (*a.stop < a.step) return;
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, false>(a, geo.r0, on, all_on, h)) return;
    const Bufs<T> bf(a, geo.g);
    const T *__restrict__ V = (MODE == M_ADB) ? a.vh : bf.vcur;
    const T *CM = (MODE == M_ADB) ? a.ch : bf.ccur;
    const T one = (T)1.0, halfc = (T)0.5;
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const size_t cbase = ((size_t)geo.g * a.m * W + geo.off) * 2;
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
        Vec<T, VEC> vv[RB][K];
        Vec<T, 2 * VEC> mem[RB];
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int j = 0; j < K; ++j) vv[b][j] = ldv<T, VEC>(V + vbase + (size_t)(lit[b][j] >> 1) * W);
#pragma unroll
        for (int b = 0; b < RB; ++b) mem[b] = ldv<T, 2 * VEC>(CM + cbase + (size_t)cc[b] * W * 2);
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            if (!ok[b]) continue;
            T C[VEC], mn[VEC], sec[VEC], t[VEC], tr[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                mn[k] = inf_v<T>();
                sec[k] = inf_v<T>();
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const T q = (lit[b][j] & 1) ? (T)-1.0 : (T)1.0;
                    minsec(one - q * vv[b][j].e[k], mn[k], sec[k]);
                }
                C[k] = halfc * mn[k];
                t[k] = mem[b].e[2 * k + 1] * mem[b].e[2 * k];
                tr[k] = (one + a.zeta * mem[b].e[2 * k + 1]) * (one - mem[b].e[2 * k]);
                if (MODE != M_ADB) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const T q = (lit[b][j] & 1) ? (T)-1.0 : (T)1.0;
                Vec<T, VEC> out;
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const T vi = vv[b][j].e[k];
                    const T val = one - q * vi;
                    const T g_ = halfc * q * (val != mn[k] ? mn[k] : sec[k]);
                    const T r_ = (C[k] == one - q * vi) ? halfc * (q - vi) : (T)0.0;
                    out.e[k] = t[k] * g_ + tr[k] * r_;
                }
                stv<T, VEC>(a.w + wbase + (size_t)pos[b][j] * W, out);
            }
            clause_update<T, VEC, MODE>(a, bf, cbase + (size_t)cc[b] * W * 2, C, mem[b], h, on, all_on, e);
        }
    }
    flush_flags<T, VEC, MODE>(a, geo.r0, on, uns, e);
}

template <typename T, int LW, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_clause(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    G_ geo;
    if (!geo.init(a)) return;
    if (*a.stop < a.step) return;
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, false>(a, geo.r0, on, all_on, h)) return;
    const Bufs<T> bf(a, geo.g);
    const T *__restrict__ V = (MODE == M_ADB) ? a.vh : bf.vcur;
    const T *CM = (MODE == M_ADB) ? a.ch : bf.ccur;
    const T one = (T)1.0, halfc = (T)0.5;
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const size_t cbase = ((size_t)geo.g * a.m * W + geo.off) * 2;
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
        const size_t ci = cbase + (size_t)c * W * 2;
        const Vec<T, 2 * VEC> mem = ldv<T, 2 * VEC>(CM + ci);
        T mn[VEC], sec[VEC], C[VEC], t[VEC], tr[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            mn[k] = inf_v<T>();
            sec[k] = inf_v<T>();
        }
        for (int s = s0; s < s1; ++s) {
            const int lit = ldc(a.lits, s);
            const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
            const Vec<T, VEC> vv = ldv<T, VEC>(V + vbase + (size_t)(lit >> 1) * W);
#pragma unroll
            for (int k = 0; k < VEC; ++k) minsec(one - q * vv.e[k], mn[k], sec[k]);
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            C[k] = halfc * mn[k];
            t[k] = mem.e[2 * k + 1] * mem.e[2 * k];
            tr[k] = (one + a.zeta * mem.e[2 * k + 1]) * (one - mem.e[2 * k]);
            if (MODE != M_ADB) uns[k] = uns[k] || (on[k] && !(C[k] < (T)0.25));
        }
        for (int s = s0; s < s1; ++s) {
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
        clause_update<T, VEC, MODE>(a, bf, ci, C, mem, h, on, all_on, e);
    }
    flush_flags<T, VEC, MODE>(a, geo.r0, on, uns, e);
}

template <typename T, int LW, int VEC, int MODE>
__global__ __launch_bounds__(256) void k_variable(KArgs<T> a) {
    using G_ = Geo<LW, VEC>;
    constexpr int W = G_::W, IPR = G_::IPR;
    G_ geo;
    if (!geo.init(a)) return;
    if (*a.stop < a.step) return;
    bool on[VEC], all_on;
    T h[VEC];
    if (!lane_state<T, VEC, MODE, true>(a, geo.r0, on, all_on, h)) return;
    const Bufs<T> bf(a, geo.g);
    const size_t vbase = (size_t)geo.g * a.n * W + geo.off;
    const T *__restrict__ wsrc = a.w + (size_t)geo.gl * a.L * W + geo.off;
    const T *VS = (MODE == M_ADB) ? a.vh : bf.vcur;
    T e[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) e[k] = (T)0.0;
    for (int row = 0; row < a.rows; ++row) {
        int i = (geo.tile * a.rows + row) * IPR + geo.isub;
        if (LW == 64) i = __builtin_amdgcn_readfirstlane(i);
        if (i >= a.n) break;
        const int p0 = ldc(a.vptr, i), p1 = ldc(a.vptr, i + 1);
        const size_t vi = vbase + (size_t)i * W;
        const Vec<T, VEC> v_old = ldv<T, VEC>(VS + vi);
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
        variable_update<T, VEC, MODE>(a, bf, vi, v_old, dv, h, on, all_on, e);
    }
    if (MODE == M_ADB) {
        bool none[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) none[k] = false;
        flush_flags<T, VEC, MODE>(a, geo.r0, on, none, e);
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
    uint8_t *par;
    int32_t r0, r1, W, step, stop_mode, adaptive;
    double tol;
};

template <typename T> __global__ __launch_bounds__(256) void k_status(StatusArgs s) {
    __shared__ uint8_t stepped[256];
    if (*s.stop < s.step) return;  // this step did not run (uniform: stop only moves to >= step here)
    const int r = s.r0 + blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = r < s.r1;
    bool st = false;
    if (valid) {
        auto *err = (typename Bits<T>::U *)s.err;
        T *dtr = (T *)s.dtr;
        // the step's final kernels wrote this replica's next state (else they copied it across)
        st = s.act[r] != 0 && (!s.adaptive || s.unsat[r] != 0u);
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
    // A group's step kernels ran (and wrote its whole next buffer, copying the replicas that did
    // not step) iff some replica of the group stepped: then the group's current buffer flips.
    // Blocks start at multiples of 256 and W divides 256, so a group never straddles blocks.
    stepped[threadIdx.x] = st ? 1 : 0;
    __syncthreads();
    if (valid && r % s.W == 0) {
        bool any = false;
        for (int j = 0; j < s.W && threadIdx.x + j < 256; ++j) any = any || stepped[threadIdx.x + j];
        if (any) s.par[r / s.W] ^= 1;
    }
}

// ------------------------------------------------------------------------------------------------
// init / layout kernels (not on the hot path: group width W is a runtime argument)
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void k_init(T *v, T *cm, const int32_t *cptr, const int32_t *lits, int n, int m, int G, int W, int B,
                       uint64_t seed, int64_t replica0, int zero_v) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nv = (size_t)G * n * W, nc = (size_t)G * m * W;
    if (tid < nv) {
        const int lane = (int)(tid % W);
        const size_t gi = tid / W;
        const int i = (int)(gi % n);
        const int g = (int)(gi / n);
        const int r = g * W + lane;
        v[tid] = (r < B && !zero_v) ? (T)init_voltage(seed, (uint64_t)(replica0 + r), (uint64_t)i) : (T)0.0;
    }
    if (tid < nc) {
        const size_t gi = tid / W;
        const int c = (int)(gi % m);
        bool anyneg = false;  // system.rs:361-372
        for (int s = cptr[c]; s < cptr[c + 1]; ++s) anyneg |= (lits[s] & 1) != 0;
        cm[2 * tid] = anyneg ? (T)1.0 : (T)-1.0;  // xs
        cm[2 * tid + 1] = (T)1.0;                 // xl (main.rs:173)
    }
}

// compact [count][items] f64 <-> layout [G][items][W] (buffer par[g] of the pair) in dtype T;
// imap (clause arrays) maps the caller's clause index to the internal clause order
template <typename T>
__global__ void k_scatter(T *b0, T *b1, const uint8_t *par, const double *src, const int32_t *imap, int items, int W,
                          int stride, int comp, int64_t r0, int64_t count) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)count * items) return;
    const int64_t b = (int64_t)(tid / items);
    const int i = imap ? imap[tid % items] : (int)(tid % items);
    const int64_t r = r0 + b;
    const int64_t g = r / W;
    T *dst = (par && par[g]) ? b1 : b0;
    dst[(((size_t)g * items + i) * W + (r % W)) * stride + comp] = (T)src[tid];
}

template <typename T>
__global__ void k_gather(double *dst, const T *b0, const T *b1, const uint8_t *par, const int32_t *imap, int items,
                         int W, int stride, int comp, int64_t r0, int64_t count) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)count * items) return;
    const int64_t b = (int64_t)(tid / items);
    const int i = imap ? imap[tid % items] : (int)(tid % items);
    const int64_t r = r0 + b;
    const int64_t g = r / W;
    const T *src = (par && par[g]) ? b1 : b0;
    dst[tid] = (double)src[(((size_t)g * items + i) * W + (r % W)) * stride + comp];
}

// (ODK_NO_COMMON_KERNELS: a second translation unit -- wave_k.hip -- includes this header for its
// device helpers; the three non-template kernels below are defined in odesat_hip.hip's only.)
#ifndef ODK_NO_COMMON_KERNELS
// Checkpoint (to_ck) or rollback of one double-buffered state array: group g's words live in buffer
// par[g]; ck holds them group by group.
__global__ void k_group_copy(uint32_t *ck, uint32_t *b0, uint32_t *b1, const uint8_t *par, int64_t gwords, int G,
                             int to_ck) {
    const int64_t total = gwords * G;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t *cur = par[i / gwords] ? b1 : b0;
        if (to_ck) ck[i] = cur[i];
        else cur[i] = ck[i];
    }
}

#endif

#ifndef ODK_NO_COMMON_KERNELS
// Per-call bookkeeping of odesat_simulate, queued on the solver's stream (no host round trip):
// every real replica active, no sat step, no steps done, the adaptive dt restarted at 0.01
// (system.rs:205) when reset_dt, and the stop word cleared.
__global__ void k_begin_call(uint8_t *act, uint32_t *unsat, int64_t *sat_step, int64_t *steps_done, void *dtr,
                             int dtype, int reset_dt, int64_t B, int64_t Bp, int32_t *stop) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r == 0) *stop = 0x7fffffff;
    if (r >= Bp) return;
    act[r] = r < B ? 1 : 0;
    unsat[r] = 0;
    sat_step[r] = -1;
    steps_done[r] = 0;
    if (reset_dt) {
        if (dtype == ODESAT_F64) ((double *)dtr)[r] = 0.01;
        else ((float *)dtr)[r] = 0.01f;
    }
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
#endif

// The exact short forms of one 3-SAT clause on in-range states (the FAST launches of k_resident,
// k_wave, k_solo_fast; onchip.hip's header states the exactness argument).
// q v for q = -1 / +1: the sign bit of v flipped by the literal's sign word (0x80000000 or 0), on the
// high dword in f64
template <typename T> __device__ __forceinline__ T sflip(T x, uint32_t sg) {
    if constexpr (sizeof(T) == 8) {
        return __longlong_as_double((long long)((unsigned long long)__double_as_longlong(x) ^ ((unsigned long long)sg << 32)));
    } else {
        return __uint_as_float(__float_as_uint(x) ^ sg);
    }
}

// -q for the literal's sign word: 1.0 for a negated literal (sg = 0x80000000), -1.0 otherwise
template <typename T> __device__ __forceinline__ T nq_of(uint32_t sg) {
    if constexpr (sizeof(T) == 8) {
        return __hiloint2double((int)(0xBFF00000u ^ sg), 0);
    } else {
        return __uint_as_float(0xBF800000u ^ sg);
    }
}

// the terms (2 x the reference's) of one clause at voltages v, memories product tt; returns mn.
// val_j = 1 - q_j v_j is one fma: q_j v_j = +-v_j is exact, so fma(-q_j, v_j, 1) rounds once, as the
// subtraction does (and a sign flip of a live f64 register pair would cost a copy besides).
template <typename T>
__device__ __forceinline__ T solo_terms(const T (&v)[3], const uint32_t (&sg)[3], T tt, T (&d)[3]) {
    const T one = (T)1.0;
    const T val0 = fma(nq_of<T>(sg[0]), v[0], one), val1 = fma(nq_of<T>(sg[1]), v[1], one),
            val2 = fma(nq_of<T>(sg[2]), v[2], one);  // :47 (f64 legs: neutral, profiles/r05p_solo_terms_fma_ab.txt)
    const T sel0 = dmin(val1, val2), sel1 = dmin(val0, val2), sel2 = dmin(val0, val1);
    d[0] = sflip(tt * sel0, sg[0]);  // 2 xl xs G (:64-70, :80)
    d[1] = sflip(tt * sel1, sg[1]);
    d[2] = sflip(tt * sel2, sg[2]);
    return dmin(sel2, val2);  // :49-57
}

// one memory step of length hx from (xs, xl) with the clause's mn: xs + hx/2 * (2 dxs), xl + hx * dxl
// (:84-85, :94-95; hx2 = hx / 2)
template <typename T>
__device__ __forceinline__ void solo_mem(T xs, T xl, T mn, T hx2, T hx, T xl_max, T &xs_o, T &xl_o) {
    const T eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001;
    const T dxs = ((T)20.0 * (xs + eps)) * (mn - (T)0.5);  // 2 dxs
    const T dxl = (T)2.5 * (mn - (T)0.1);
    xs_o = dmin(dmax(xs + hx2 * dxs, eps), xs_hi);
    xl_o = dmin(dmax(xl + hx * dxl, (T)1.0), xl_max);
}

}  // namespace odk
