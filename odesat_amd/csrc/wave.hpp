// wave.hpp -- ALG_RESIDENT for small 3-SAT instances: one wave per replica, the dv fold variable by
// variable instead of clause tile by clause tile (included by odesat_hip.hip).
//
// The tile kernels fold every dv[i] in the reference's order by running var-disjoint clause tiles
// one after another, so a step costs the depth of the clause-order chains -- 34 tiles of ~5 clauses
// for tests/hard.cnf, 30 of ~35 for config 3 -- whatever the instance's size.  On a small instance
// the whole replica fits in one wave's share of LDS, and the step splits into two phases with no
// order between clauses at all:
//   1. every clause (lane l takes clauses l, l + 64, ...) computes C, its memory update and its
//      three dv terms (system.rs:43-88), and stores each term at its variable-major position:
//      the incidences of variable i, sorted by (clause, literal), occupy [vstart[i], vstart[i+1]);
//   2. every variable (lane l takes l, l + 64, ...) folds its terms in that order from +0 -- the
//      reference's dv[i] += ... sequence exactly (:33, :80) -- and applies :96.
// A single wave needs no barrier between the phases: its LDS operations complete in issue order,
// and wave_sync only keeps the compiler from moving LDS accesses across them.  The state (v, the
// clause memories, the adaptive clone of v and the first pass's C) stays in LDS for a launch, and
// the topology (literal and position records, variable starts) is copied into LDS once per launch
// and shared by the workgroup's WPW waves, so a step reads nothing from the memory hierarchy.
// Arithmetic: the tile kernel's (res_clause3 / res_mem_update) expression for expression, so every
// result is bit-identical to it and to the oracle.
#pragma once

#include "kernels.hpp"
#include "solo_blocks.hpp"

#include <type_traits>

namespace odk {

constexpr int WAVE_NTH = 64;

template <typename T> struct WArgs {
    const int4 *__restrict__ rec4;    // [m] per literal j: (var << 1 | neg) | (variable-major position of
                                      // its term) << 16 -- both below 2^16 whenever k_wave is chosen
    const int32_t *__restrict__ vst;  // [n+1] variable -> first term position
    T *v0, *v1, *c0, *c1;             // state buffers, group width 1
    uint8_t *par;                     // flipped by an out-of-place launch
    T *dtr;
    uint8_t *act;
    int64_t *sat_step, *steps_done;
    int32_t *stop;
    int32_t n, m, L, G;                 // G: replicas (groups of width 1)
    int32_t g0;                         // k_wave: this launch's first replica (a partial round's tail launch)
    uint32_t topo_bytes, rep_bytes;     // LDS: the shared topology, then WPW replicas of rep_bytes
    int32_t step0, nsteps, stop_mode;
    int32_t oop;  // 1: the final state goes to the other buffer and par flips (STOP_ANY replay)
    T dt, zeta, xl_max;
    double tol;
    CallIO io;  // per-call bookkeeping (callio.hpp)
    // k_solo_cv's layout (cv_layout.cpp): per clause slot l + k NL its record (the literals' rec4 fields
    // in the chosen order, w = the clause or -1), each variable's term block (cvblk[n]: the zero block),
    // and the blocks in use (the lanes' sink words follow)
    const int4 *__restrict__ cvrec;
    const int32_t *__restrict__ cvblk;
    int32_t cvnb;
};

// LDS bytes of one replica: v, its full-step clone (adaptive), the terms, the memories and (adaptive)
// each clause's C of the first pass, from which the second pass recomputes the full-step and
// first-half memories with the first pass's expressions -- bit-identical, and 16 bytes per clause
// less than storing them
inline size_t wave_lds_bytes(int64_t n, int64_t m, int64_t L, size_t tsize, bool adaptive) {
    return (((adaptive ? 2 : 1) * (size_t)n + (size_t)L + (adaptive ? 3 : 2) * (size_t)m) * tsize + 15) / 16 * 16;
}
// the topology every wave of a workgroup reads: literal and position records, variable starts
inline size_t wave_topo_bytes(int64_t n, int64_t m) { return ((size_t)m * 16 + (size_t)(n + 1) * 4 + 15) / 16 * 16; }

enum WPass : int { W_FIXED = 0, W_ADA1 = 1, W_ADA2 = 2 };

// One clause's inputs, loaded ahead of its arithmetic.
template <typename T> struct WClause {
    int lit[3], pos[3];
    T v[3], xs, xl, C1;
};

// One clause's arithmetic (system.rs:43-95) for a pass: the three dv terms into d[] (stored at the
// clause's term positions by the caller), C, and by pass the memory update in place (W_FIXED), the
// clause's C kept for the second pass (W_ADA1: the memories stay y) or -- from the first pass's C1 --
// the full-step clone and the first half step of y's memories, then the second half step with its
// max_error terms into e (W_ADA2).  Shared by k_wave and k_solo, so both are the same expressions.
template <typename T, int PK>
__device__ __forceinline__ bool clause_math(const int (&lit)[3], const T (&v)[3], T &xs, T &xl, T &C1, T h, T zeta,
                                            T xl_max, T (&d)[3], T &e) {
    const T one = (T)1.0, halfc = (T)0.5, eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001;
    T q[3], val[3];
    T mn = inf_v<T>(), sec = inf_v<T>();
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // :43-57
        q[j] = (lit[j] & 1) ? (T)-1.0 : (T)1.0;
        val[j] = one - q[j] * v[j];
        minsec(val[j], mn, sec);
    }
    const T C = halfc * mn;  // :60
    T xs_m = xs, xl_m = xl;
    T xs_f = xs_m, xl_f = xl_m;
    if (PK == W_ADA2) {  // y's memories -> the full-step clone and the first half step (:124-128)
        const T half = (T)0.5 * h;
        const T dxs1 = (T)20.0 * (xs_m + eps) * (C1 - (T)0.25);  // :84
        const T dxl1 = (T)5.0 * (C1 - (T)0.05);                  // :85
        xs_f = dmin(dmax(xs_m + h * dxs1, eps), xs_hi);
        xl_f = dmin(dmax(xl_m + h * dxl1, one), xl_max);
        const T xs_h = dmin(dmax(xs_m + half * dxs1, eps), xs_hi);
        const T xl_h = dmin(dmax(xl_m + half * dxl1, one), xl_max);
        xs_m = xs_h;
        xl_m = xl_h;
    }
    const T tt = xl_m * xs_m;
    const T tr = (one + zeta * xl_m) * (one - xs_m);
#pragma unroll
    for (int j = 0; j < 3; ++j) d[j] = tt * (halfc * q[j] * (val[j] != mn ? mn : sec));  // :64-70
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // :73-80 (zero unless C == val_j; adding it keeps the sum exact)
        const T r_ = (C == one - q[j] * v[j]) ? halfc * (q[j] - v[j]) : (T)0.0;
        d[j] = d[j] + tr * r_;
    }
    const T dxs = (T)20.0 * (xs_m + eps) * (C - (T)0.25);  // :84
    const T dxl = (T)5.0 * (C - (T)0.05);                  // :85
    if (PK == W_FIXED) {
        xs = dmin(dmax(xs_m + h * dxs, eps), xs_hi);  // :94-95
        xl = dmin(dmax(xl_m + h * dxl, one), xl_max);
    } else if (PK == W_ADA1) {
        C1 = C;  // the memories stay y until the second pass (an allsat replica takes no step)
    } else {
        const T half = (T)0.5 * h;  // second half step (:130), max_error terms (:132)
        const T xs_n = dmin(dmax(xs_m + half * dxs, eps), xs_hi);
        const T xl_n = dmin(dmax(xl_m + half * dxl, one), xl_max);
        e = dmax(e, dmax(dabs(xs_f - xs_n), dabs(xl_f - xl_n)));
        xs = xs_n;
        xl = xl_n;
    }
    return PK != W_ADA2 && !(C < (T)0.25);  // :88 (unsat)
}

// The max of x over the wave (all 64 lanes active), uniform: a DPP butterfly within each quad, row
// rotations within each row of 16, then the four rows' maxima by readlane.
// (bound_ctrl with old = 0: every lane has a source under these controls, and the form lets the
// compiler fold the move into one v_max_u32_dpp instead of a copy, a v_mov_b32_dpp and the max)
template <int CTRL> __device__ __forceinline__ uint32_t max_dpp(uint32_t x) {
    return max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = max_dpp<0xB1>(x);   // quad_perm [1, 0, 3, 2]
    x = max_dpp<0x4E>(x);   // quad_perm [2, 3, 0, 1]
    x = max_dpp<0x124>(x);  // row_ror:4
    x = max_dpp<0x128>(x);  // row_ror:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
    return max(max(r0, r1), max(r2, r3));
}
__device__ __forceinline__ uint32_t wave_max_bits(uint32_t x) { return wave_max_u32(x); }
__device__ __forceinline__ unsigned long long wave_max_bits(unsigned long long x) {  // (high word, then low word)
    const uint32_t hi = wave_max_u32((uint32_t)(x >> 32));
    const uint32_t lo = wave_max_u32((uint32_t)(x >> 32) == hi ? (uint32_t)x : 0u);
    return ((unsigned long long)hi << 32) | lo;
}

// Phase 1 over the replica's clauses, one lane's share.  Returns whether one of this lane's clauses
// is unsat (:88, W_FIXED / W_ADA1) and raises e to the memories' max_error terms (W_ADA2).
// Lane l of the replica's NL lanes takes clauses l, l + NL, ...  Software-pipelined: the records of
// clause c + 2 NL and the voltages / memories of clause c + NL are loaded before clause c's
// arithmetic and stores (nothing phase 1 stores is read by another
// clause: terms, memories and C are per clause and v is constant), so one wave per SIMD keeps
// three clauses' LDS reads in flight instead of waiting on each clause's dependent load chain.
// FAST (in-range states): solo_terms / solo_mem's exact short forms -- 2 x terms (the fold's caller
// halves h), the first pass keeps mn (= 2 C) for the second.
template <typename T, int PK, int NL, bool FAST>
__device__ __forceinline__ bool lane_clauses(const WArgs<T> &a, const int4 *rec4, const T *vL, T *tL, T *cmL, T *cL,
                                             int l, T h, T &e) {
    bool uns = false;
    if (l >= a.m) return false;  // (NL > m: the lanes without a clause)
    const int last = a.m - 1;
    typedef HIP_vector_type<T, 2> T2;  // a clause's (xs, xl): one 8- / 16-byte LDS access
    auto gather = [&](int c, const int4 &r4, WClause<T> &W) {  // clamped: always loadable
        W.lit[0] = r4.x & 0xffff, W.lit[1] = r4.y & 0xffff, W.lit[2] = r4.z & 0xffff;
        W.pos[0] = (int)((uint32_t)r4.x >> 16), W.pos[1] = (int)((uint32_t)r4.y >> 16), W.pos[2] = (int)((uint32_t)r4.z >> 16);
#pragma unroll
        for (int j = 0; j < 3; ++j) W.v[j] = vL[W.lit[j] >> 1];
        const T2 m2 = reinterpret_cast<const T2 *>(cmL)[c];
        W.xs = m2.x;
        W.xl = m2.y;
        if (PK == W_ADA2) W.C1 = cL[c];
    };
    int4 rn = rec4[min(l + NL, last)];  // the record of the next clause
    WClause<T> W;
    gather(l, rec4[l], W);
    for (int c = l; c < a.m; c += NL) {
        WClause<T> X = W;  // this clause
        const int cn = min(c + NL, last);
        gather(cn, rn, W);       // the next clause's voltages and memories
        rn = rec4[min(c + 2 * NL, last)];
        T d[3];
        if constexpr (FAST) {
            const uint32_t sg[3] = {(uint32_t)X.lit[0] << 31, (uint32_t)X.lit[1] << 31, (uint32_t)X.lit[2] << 31};
            const T hh = (T)0.5 * h, hq = (T)0.25 * h;
            if (PK == W_FIXED) {
                const T mn = solo_terms<T>(X.v, sg, X.xl * X.xs, d);
                solo_mem<T>(X.xs, X.xl, mn, hh, h, a.xl_max, X.xs, X.xl);
                uns = uns || !(mn < (T)0.5);  // :88
            } else if (PK == W_ADA1) {
                X.C1 = solo_terms<T>(X.v, sg, X.xl * X.xs, d);  // mn1 = 2 C1
                uns = uns || !(X.C1 < (T)0.5);
            } else {
                T xsf, xlf, xsh, xlh, xsn, xln;
                solo_mem<T>(X.xs, X.xl, X.C1, hh, h, a.xl_max, xsf, xlf);  // full-step clone (:124-125)
                solo_mem<T>(X.xs, X.xl, X.C1, hq, hh, a.xl_max, xsh, xlh);  // first half step (:128)
                const T mn = solo_terms<T>(X.v, sg, xlh * xsh, d);
                solo_mem<T>(xsh, xlh, mn, hq, hh, a.xl_max, xsn, xln);      // second half step (:130)
                e = dmax(e, dmax(dabs(xsf - xsn), dabs(xlf - xln)));       // :132
                X.xs = xsn;
                X.xl = xln;
            }
        } else {
            uns = clause_math<T, PK>(X.lit, X.v, X.xs, X.xl, X.C1, h, a.zeta, a.xl_max, d, e) || uns;
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) tL[X.pos[j]] = d[j];
        if (PK == W_ADA1) {
            cL[c] = X.C1;
        } else {
            T2 m2;
            m2.x = X.xs;
            m2.y = X.xl;
            reinterpret_cast<T2 *>(cmL)[c] = m2;
        }
    }
    return uns;
}

// Phase 1, wave-uniform result: some clause of this wave is unsat (the caller combines a replica's
// waves).  The ballot runs after every lane's share has returned: taken inside lane_clauses, the
// lanes without a clause (m < NL) would vote among themselves on a divergent path and leave the
// result -- and the step loop's exit -- different across the wave's lanes.
template <typename T, int PK, int NL, bool FAST>
__device__ __forceinline__ bool wave_clauses(const WArgs<T> &a, const int4 *rec4, const T *vL, T *tL, T *cmL, T *cL,
                                             int l, T h, T &e) {
    const bool u = lane_clauses<T, PK, NL, FAST>(a, rec4, vL, tL, cmL, cL, l, h, e);
    return __any(u);
}

// Phase 2 for variable i: dv[i] as the reference's left fold of its terms (:33, :80).  The term
// reads go out four at a time; the adds stay in order.
template <typename T> __device__ __forceinline__ T wave_fold(const int32_t *vst, const T *tL, int i) {
    T dv = (T)0.0;
    const int k1 = vst[i + 1];
    for (int k = vst[i]; k < k1; k += 4) {
        T t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = tL[min(k + u, k1 - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k + u < k1) dv += t[u];
    }
    return dv;
}

// Orders one wave's LDS accesses across the phases: a wave's LDS operations complete in issue
// order, so only the compiler must not move accesses across this point.
__device__ __forceinline__ void wave_sync() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// WPW replicas per workgroup share one LDS copy of the topology; each replica is a team of TW waves
// (NL = 64 TW lanes).  TW = 1: a wave is on its own after the topology copy (its LDS operations
// complete in issue order, so wave_sync only fences the compiler).  TW = 2 (small batches, where one
// wave per replica would leave one wave per SIMD): the team's phases are ordered by workgroup
// barriers, which every wave of the workgroup reaches the same number of times -- a frozen replica's
// team skips the work but not the barriers, and the step loop ends when no team is active.
template <int TW> __device__ __forceinline__ void team_sync() {
    if (TW == 1) wave_sync();
    else __syncthreads();
}

template <typename T, bool ADAPTIVE, int WPW, int TW, bool FAST = false>
__global__ __launch_bounds__(WAVE_NTH * WPW * TW) void k_wave(WArgs<T> a) {
    constexpr int NL = WAVE_NTH * TW;
    extern __shared__ __attribute__((aligned(16))) unsigned char wave_smem[];
    using U = typename Bits<T>::U;
    __shared__ U errL[WPW];
    __shared__ int unsL[WPW * TW];  // TW > 1: each wave's "some clause unsat"
    const int w = threadIdx.x / NL, l = threadIdx.x % NL;
    const int g = a.g0 + (int)blockIdx.x * WPW + w;  // this team's replica (group width 1)
    int4 *rec4 = reinterpret_cast<int4 *>(wave_smem);
    int32_t *vst = reinterpret_cast<int32_t *>(rec4 + a.m);
    copy_to_lds<8>(rec4, a.rec4, (int)threadIdx.x, a.m, NL * WPW);
    copy_to_lds<8>(vst, a.vst, (int)threadIdx.x, a.n + 1, NL * WPW);
    __syncthreads();
    if (l == 0 && g < a.G) io_begin_store<T>(a.io, g, a.act, a.sat_step, a.steps_done, a.dtr, ADAPTIVE, a.stop);
    if (a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0) return;  // an earlier step stopped every replica
    const bool live = g < a.G && io_active(a.io, a.act, g);  // uniform per team
    if (TW == 1 ? !live : !__syncthreads_or(live)) return;
    int act = live;
    int64_t sat = live ? io_sat(a.io, a.sat_step, g) : -1, done = live ? io_done(a.io, a.steps_done, g) : 0;
    T dtr = ADAPTIVE && live ? io_dt<T>(a.io, a.dtr, g) : a.dt;
    // the replica's LDS: memories first (16-byte aligned: read and written as (xs, xl) pairs), the
    // first pass's C (adaptive), v, its full-step clone (adaptive), the terms
    T *cmL = reinterpret_cast<T *>(wave_smem + a.topo_bytes + (size_t)w * a.rep_bytes);
    T *cL = cmL + 2 * a.m;
    T *vL = cL + (ADAPTIVE ? a.m : 0);
    T *vfL = vL + (ADAPTIVE ? a.n : 0);
    T *tL = vfL + a.n;
    const bool p = live && __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;
    if (live) {
        const T *V = (p ? a.v1 : a.v0) + (size_t)g * a.n;
        const T *CM = (p ? a.c1 : a.c0) + (size_t)g * a.m * 2;
        copy_to_lds<8>(vL, V, l, a.n, NL);
        copy_to_lds<8>(cmL, CM, l, 2 * a.m, NL);
    }
    team_sync<TW>();
    const int wi = (int)(threadIdx.x % NL) / WAVE_NTH;  // wave within the team
    auto team_any = [&](bool u) {  // after the next team_sync: some wave of the team saw u
        if (TW == 1) return u;
        if ((threadIdx.x % WAVE_NTH) == 0) unsL[w * TW + wi] = u ? 1 : 0;
        team_sync<TW>();
        bool r = false;
#pragma unroll
        for (int j = 0; j < TW; ++j) r = r || unsL[w * TW + j] != 0;
        return r;
    };
    // Barriers per step (TW > 1): team_any's (phase 1's terms and memories before the fold, and the
    // unsat vote), and the step's closing __syncthreads_or (the fold's voltages before the next
    // step's phase 1, and whether any team still steps); adaptive adds two (the half step's
    // voltages before the second clause pass, its terms before the second fold) and one for the
    // error fold.  The bookkeeping only needs uns, so it runs before the closing barrier.
    for (int k = 0; k < a.nsteps; ++k) {
        const int step = a.step0 + k;
        const T h = dtr;
        T e = (T)0.0;
        bool uns = false;
        const int act0 = act;  // this step's participation; the bookkeeping below may clear act
        bool go = false;
        if (!ADAPTIVE) {  // euler_step_fixed (system.rs:141-154): the update is taken regardless
            if (act0) uns = wave_clauses<T, W_FIXED, NL, FAST>(a, rec4, vL, tL, cmL, cL, l, h, e);
            uns = team_any(uns);
            if (TW == 1) team_sync<TW>();  // (TW > 1: team_any's barrier ordered phase 1's stores)
            const T hv = FAST ? (T)0.5 * h : h;  // FAST: 2 x terms
            if (act0)
                for (int i = l; i < a.n; i += NL) vL[i] = dmin(dmax(vL[i] + hv * wave_fold(vst, tL, i), (T)-1.0), (T)1.0);
        } else {  // euler_step (:111-139)
            if (act0) uns = wave_clauses<T, W_ADA1, NL, FAST>(a, rec4, vL, tL, cmL, cL, l, h, e);
            uns = team_any(uns);
            if (TW == 1) team_sync<TW>();
            if (l == 0) errL[w] = 0;  // last read before the previous step's closing barrier
            go = act0 && uns;  // an allsat replica takes no step (:122)
            const T hf = FAST ? (T)0.5 * h : h, half = FAST ? (T)0.25 * h : (T)0.5 * h;  // FAST: 2 x terms
            if (go)
                for (int i = l; i < a.n; i += NL) {
                    const T d = wave_fold(vst, tL, i), v = vL[i];
                    vfL[i] = dmin(dmax(v + hf * d, (T)-1.0), (T)1.0);   // full-step clone
                    vL[i] = dmin(dmax(v + half * d, (T)-1.0), (T)1.0);  // first half step
                }
            team_sync<TW>();
            if (go) wave_clauses<T, W_ADA2, NL, FAST>(a, rec4, vL, tL, cmL, cL, l, h, e);
            team_sync<TW>();
            if (go)
                for (int i = l; i < a.n; i += NL) {
                    const T vn = dmin(dmax(vL[i] + half * wave_fold(vst, tL, i), (T)-1.0), (T)1.0);  // second half
                    e = dmax(e, dabs(vfL[i] - vn));  // :101-108
                    vL[i] = vn;
                }
            if (go) atomicMax(&errL[w], tobits(e));
        }
        if (act0) {
            done += 1;
            if (!uns) {  // allsat: the fixed step was still taken (:148-152); adaptive took none
                if (sat < 0) sat = step;
                if (a.stop_mode == ODESAT_STOP_EACH) act = 0;                            // simulate() breaks (:193)
                if (a.stop_mode == ODESAT_STOP_ANY && l == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
            }
        }
        if (TW == 1) team_sync<TW>();
        if (TW == 1 ? !act : !__syncthreads_or(act)) break;  // uniform per wave / per workgroup
        if (ADAPTIVE && go) {  // (a stepping team stays active, so it reaches this after the barrier)
            const T error = frombits(errL[w]);  // :133-135 dt <- clamp(dt * sqrt(tol / err), 2^-7, 1e3)
            dtr = dmax(dmin(dtr * dsqrt((T)a.tol / error), (T)1e3), (T)0.0078125);
        }
    }
    team_sync<TW>();
    if (!live) return;
    const bool q = a.oop ? !p : p;
    T *Vo = (q ? a.v1 : a.v0) + (size_t)g * a.n;
    T *CMo = (q ? a.c1 : a.c0) + (size_t)g * a.m * 2;
    for (int i = l; i < a.n; i += NL) Vo[i] = vL[i];
    for (int i = l; i < 2 * a.m; i += NL) CMo[i] = cmL[i];
    if (l == 0) {
        if (a.oop) a.par[g] = (uint8_t)q;
        a.act[g] = (uint8_t)act;
        a.sat_step[g] = sat;
        a.steps_done[g] = done;
        if (ADAPTIVE) a.dtr[g] = dtr;
        io_mirror<T>(a.io, g, sat, done, dtr, ADAPTIVE);
    }
}

// ------------------------------------------------------------------------------------------------
// k_solo -- the latency path for one replica (solve, the criterion benches: B = 1) and small
// batches of tiny formulas.  k_wave's two phases, with everything a lane owns kept in registers
// for the launch: one replica per workgroup, a team of NL = blockDim lanes; lane l owns clauses l,
// l + NL, ... (CPL slots: their literal and term-position records and their memories, plus the
// adaptive pass's C) and variables l, l + NL, ... (VPL slots: the voltage, its term range and the
// adaptive full-step clone).  Per step LDS carries only what crosses lanes -- v for the clause
// gathers, the terms for the fold -- so a step is: the voltage gathers (one round trip), the clause
// arithmetic (clause_math, k_wave's expressions), the term stores, one barrier, the term reads
// (one round trip per 8 terms), the fold and the voltage stores, one barrier.  Bit-identical to
// k_wave and the oracle.
// ------------------------------------------------------------------------------------------------
constexpr int SOLO_MAX_NL = 1024;

// 8 term reads in flight per round (16 measured slower: profiles/r03_solo_sweep2.jsonl -- hard.cnf
// f64 at 256 lanes 1.00 vs 0.81 us per fixed step -- the extra registers and reads cost more than
// the second round trip of the few high-degree variables saves)
template <typename T> __device__ __forceinline__ T solo_fold(const T *tL, int s, int d, int L) {
    T dv = (T)0.0;  // :33, then the reference's left fold of the variable's terms (:80)
    for (int k0 = 0; k0 < d; k0 += 8) {
        T t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = tL[min(s + min(k0 + u, d - 1), L - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k0 + u < d) dv += t[u];
    }
    return dv;
}

// Diagnostic build only (-DSOLO_STAMPS, scripts/build_variant.sh NAME -DSOLO_STAMPS wave_k -- k_solo is
// instantiated in wave_k.hip): per wave, s_memtime
// stamps split each fixed step into the clause pass, the first barrier, the fold and the closing
// barrier; sums in g_solo_stamps (read by odesat_solo_stamps).  Each stamp drains the wave's LDS
// operations: read the SHARES.
#ifdef SOLO_STAMPS
__device__ unsigned long long g_solo_stamps[16 * 8];
__device__ __forceinline__ uint64_t solo_memtime() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define SOLO_STAMP(i)                          \
    do {                                       \
        const uint64_t t_ = solo_memtime();    \
        st_[i] += t_ - st_last;                \
        st_last = t_;                          \
    } while (0)
#else
#define SOLO_STAMP(i) \
    do {              \
    } while (0)
#endif

template <typename T, bool ADAPTIVE, int CPL, int VPL>
__global__ __launch_bounds__(SOLO_MAX_NL) void k_solo(WArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char wave_smem[];
    using U = typename Bits<T>::U;
    __shared__ U errW[SOLO_MAX_NL / 64];
    // per step parity and wave: some clause of the wave is unsat (words of absent waves stay 0)
    __shared__ __attribute__((aligned(16))) int voteW[2][SOLO_MAX_NL / 64];
    const int NL = (int)blockDim.x, l = (int)threadIdx.x, TW = NL / 64;
    const int g = blockIdx.x;  // this workgroup's replica (group width 1)
    if (l == 0 && g < a.G) io_begin_store<T>(a.io, g, a.act, a.sat_step, a.steps_done, a.dtr, ADAPTIVE, a.stop);
    if (a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0) return;  // an earlier step stopped every replica
    if (g >= a.G || !io_active(a.io, a.act, g)) return;                // uniform per workgroup
    T *vL = reinterpret_cast<T *>(wave_smem);
    T *tL = vL + a.n;
    const bool p = __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;
    const T *V = (p ? a.v1 : a.v0) + (size_t)g * a.n;
    const T *CM = (p ? a.c1 : a.c0) + (size_t)g * a.m * 2;
    const int mlast = a.m - 1, nlast = a.n - 1;
    int lit[CPL][3], pos[CPL][3];
    T xs[CPL], xl[CPL], C1[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {  // records and memories of this lane's clauses (clamped: loadable)
        const int c = min(l + k * NL, mlast);
        const int4 r4 = a.rec4[c];
        lit[k][0] = r4.x & 0xffff, lit[k][1] = r4.y & 0xffff, lit[k][2] = r4.z & 0xffff;
        pos[k][0] = (int)((uint32_t)r4.x >> 16), pos[k][1] = (int)((uint32_t)r4.y >> 16);
        pos[k][2] = (int)((uint32_t)r4.z >> 16);
        xs[k] = CM[2 * c];
        xl[k] = CM[2 * c + 1];
        C1[k] = (T)0.0;
    }
    int vs[VPL], vd[VPL];
    T vr[VPL], vf[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {  // this lane's variables: voltage, term range
        const int i = l + j * NL, ii = min(i, nlast);
        vs[j] = a.vst[ii];
        vd[j] = i < a.n ? a.vst[ii + 1] - vs[j] : 0;
        vr[j] = V[ii];
        vf[j] = vr[j];
        if (i < a.n) vL[i] = vr[j];
    }
    if (l < 2 * (SOLO_MAX_NL / 64)) voteW[l >> 4][l & 15] = 0;
    __syncthreads();
    int act = 1;
    int64_t sat = io_sat(a.io, a.sat_step, g), done = io_done(a.io, a.steps_done, g);
    T dtr = ADAPTIVE ? io_dt<T>(a.io, a.dtr, g) : a.dt;
    // phase 1 over this lane's clauses: the voltage gathers of every slot first, then the arithmetic
    auto clauses = [&](auto pk, T h, T &e) -> bool {
        constexpr int PK = decltype(pk)::value;
        T vv[CPL][3];
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) vv[k][j] = vL[lit[k][j] >> 1];
        bool uns = false;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (l + k * NL < a.m) {
                T d[3];
                uns = clause_math<T, PK>(lit[k], vv[k], xs[k], xl[k], C1[k], h, a.zeta, a.xl_max, d, e) || uns;
#pragma unroll
                for (int j = 0; j < 3; ++j) tL[pos[k][j]] = d[j];
            }
        }
        return uns;
    };
    // The unsat vote: each wave's ballot goes to voteW[step parity] before the barrier that orders
    // the clause pass's terms, and every lane reads the TW words after it (one barrier for both; the
    // words of step k are rewritten only after step k + 1's first barrier, which every reader of
    // step k has passed).
    const int w = l >> 6;
    auto vote = [&](bool u, int k) {
        const bool wu = __any(u);
        if ((l & 63) == 0) voteW[k & 1][w] = wu ? 1 : 0;
    };
    auto votes = [&](int k) {  // all 16 words in four 16-byte reads, issued together
        const int4 *vw = reinterpret_cast<const int4 *>(voteW[k & 1]);
        int4 r4[SOLO_MAX_NL / 256];
#pragma unroll
        for (int j = 0; j < SOLO_MAX_NL / 256; ++j) r4[j] = vw[j];
        int r = 0;
#pragma unroll
        for (int j = 0; j < SOLO_MAX_NL / 256; ++j) r |= r4[j].x | r4[j].y | r4[j].z | r4[j].w;
        return r != 0;
    };
#ifdef SOLO_STAMPS
    uint64_t st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = solo_memtime();
#endif
    for (int k = 0; k < a.nsteps; ++k) {
        const int step = a.step0 + k;
        const T h = dtr;
        T e = (T)0.0;
        bool uns, go = false;
        if (!ADAPTIVE) {  // euler_step_fixed (system.rs:141-154): the update is taken regardless
            vote(clauses(std::integral_constant<int, W_FIXED>{}, h, e), k);
            SOLO_STAMP(0);
            __syncthreads();  // the terms (and the votes) before the fold
            SOLO_STAMP(1);
            uns = votes(k);
            const T hv = h;
#pragma unroll
            for (int j = 0; j < VPL; ++j)
                if (l + j * NL < a.n) {
                    vr[j] = dmin(dmax(vr[j] + hv * solo_fold(tL, vs[j], vd[j], a.L), (T)-1.0), (T)1.0);  // :96
                    vL[l + j * NL] = vr[j];
                }
            SOLO_STAMP(2);
        } else {  // euler_step (:111-139)
            vote(clauses(std::integral_constant<int, W_ADA1>{}, h, e), k);
            __syncthreads();
            uns = votes(k);
            go = uns;  // an allsat replica takes no step (:122)
            const T half = (T)0.5 * h, hf = h, hh = half;
            if (go) {
#pragma unroll
                for (int j = 0; j < VPL; ++j)
                    if (l + j * NL < a.n) {
                        const T d = solo_fold(tL, vs[j], vd[j], a.L), v = vr[j];
                        vf[j] = dmin(dmax(v + hf * d, (T)-1.0), (T)1.0);  // full-step clone
                        vr[j] = dmin(dmax(v + hh * d, (T)-1.0), (T)1.0);  // first half step
                        vL[l + j * NL] = vr[j];
                    }
            }
            __syncthreads();  // the half step's voltages before the second pass; the terms read
            if (go) clauses(std::integral_constant<int, W_ADA2>{}, h, e);
            __syncthreads();  // the second pass's terms before its fold
            if (go) {
#pragma unroll
                for (int j = 0; j < VPL; ++j)
                    if (l + j * NL < a.n) {
                        const T vn = dmin(dmax(vr[j] + hh * solo_fold(tL, vs[j], vd[j], a.L), (T)-1.0), (T)1.0);
                        e = dmax(e, dabs(vf[j] - vn));  // :101-108
                        vr[j] = vn;
                        vL[l + j * NL] = vn;
                    }
                U eb = tobits(e);  // non-negative floats order as their bits
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const U o = __shfl_xor(eb, off, 64);
                    eb = o > eb ? o : eb;
                }
                if ((l & 63) == 0) errW[l >> 6] = eb;
            }
        }
        done += 1;
        if (!uns) {  // allsat: the fixed step was still taken (:148-152); adaptive took none
            if (sat < 0) sat = step;
            if (a.stop_mode == ODESAT_STOP_EACH) act = 0;                            // simulate() breaks (:193)
            if (a.stop_mode == ODESAT_STOP_ANY && l == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
        }
        SOLO_STAMP(3);
        __syncthreads();  // the voltages before the next step's gathers (and the error words)
        SOLO_STAMP(4);
        if (ADAPTIVE && go) {  // :133-135 dt <- clamp(dt * sqrt(tol / err), 2^-7, 1e3)
            U eb = errW[0];
            for (int w2 = 1; w2 < TW; ++w2) eb = errW[w2] > eb ? errW[w2] : eb;
            dtr = dmax(dmin(dtr * dsqrt((T)a.tol / frombits(eb)), (T)1e3), (T)0.0078125);
        }
        if (!act) break;  // uniform
    }
#ifdef SOLO_STAMPS
    if ((l & 63) == 0 && g == 0)
        for (int i = 0; i < 8; ++i) g_solo_stamps[(l >> 6) * 8 + i] = st_[i];
#endif
    const bool q = a.oop ? !p : p;
    T *Vo = (q ? a.v1 : a.v0) + (size_t)g * a.n;
    T *CMo = (q ? a.c1 : a.c0) + (size_t)g * a.m * 2;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
        if (l + j * NL < a.n) Vo[l + j * NL] = vr[j];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = l + k * NL;
        if (c < a.m) {
            CMo[2 * c] = xs[k];
            CMo[2 * c + 1] = xl[k];
        }
    }
    if (l == 0) {
        if (a.oop) a.par[g] = (uint8_t)q;
        a.act[g] = (uint8_t)act;
        a.sat_step[g] = sat;
        a.steps_done[g] = done;
        if (ADAPTIVE) a.dtr[g] = dtr;
        io_mirror<T>(a.io, g, sat, done, dtr, ADAPTIVE);
    }
}

// ------------------------------------------------------------------------------------------------
// k_solo_fast -- k_solo on in-range states (the host's `fast` launches: onchip.hip's range, finite
// zeta and dt): solo_fast's exact short arithmetic, and a step laid out for latency --
//   * the terms of variable i sit in a padded block of SOLO_DPAD slots (16-byte aligned, the slots
//     past its degree stay +0), so its fold is SOLO_DPAD / (16 / sizeof(T)) vector reads from one
//     address and a chain of adds whose length is the wave's largest degree (a uniform bound; the
//     added +0 terms change nothing, since dv starts at +0 and is never -0); terms of rank >= SOLO_DPAD
//     go to an overflow area at n SOLO_DPAD + their variable-major position and are folded after;
//   * the memory updates, which nothing in the step waits for, run after the barrier that follows
//     the term stores, under the fold's LDS reads (adaptive: the first pass's clones and half step
//     right after pass 1, the second half step after pass 2).
// Bit-identical to k_solo, k_wave and the oracle (tests/test_gpu_parity.py, tests/test_gpu_fuzz.py).
// ------------------------------------------------------------------------------------------------
// (SOLO_DPAD: solo_blocks.hpp, shared with cv_layout.cpp's bank model)
#ifndef SOLO_FOLD_EARLY
#define SOLO_FOLD_EARLY 1
#endif
// SOLO_DT_LATE=1: an adaptive step's dt update (an f64 divide and square root, system.rs:133-135)
// runs in the next step's first clause pass, between its gathers and its arithmetic (select form, no
// branch, so the two chains share a basic block), instead of after the closing barrier: nothing in
// that pass reads dt.  The last step's update runs after the loop.
#ifndef SOLO_DT_LATE
#define SOLO_DT_LATE 1
#endif

// LDS elements of k_solo_fast: v (rounded up to 16 bytes), the padded term blocks, the overflow area
inline size_t solo_fast_elems(int64_t n, int64_t L, size_t tsize) {
    const int64_t per16 = 16 / (int64_t)tsize;
    return (size_t)((n + per16 - 1) / per16 * per16 + n * SOLO_DPAD + L);
}

template <typename T, bool ADAPTIVE, int CPL, int VPL>
__global__ __launch_bounds__(SOLO_MAX_NL) void k_solo_fast(WArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char wave_smem[];
    using U = typename Bits<T>::U;
    constexpr int PER16 = 16 / (int)sizeof(T);
    typedef T TV __attribute__((ext_vector_type(PER16)));  // 16 bytes of terms
    struct Terms {
        TV t[VPL][SOLO_DPAD / PER16];
    };
    __shared__ U errM[2];  // per step parity: the max_error bits of the step (the waves' LDS atomic max)
    __shared__ __attribute__((aligned(16))) int voteW[2][SOLO_MAX_NL / 64];
    const int NL = (int)blockDim.x, l = (int)threadIdx.x;
    const int g = blockIdx.x;
    if (l == 0 && g < a.G) io_begin_store<T>(a.io, g, a.act, a.sat_step, a.steps_done, a.dtr, ADAPTIVE, a.stop);
    if (a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0) return;  // an earlier step stopped every replica
    if (g >= a.G || !io_active(a.io, a.act, g)) return;                // uniform per workgroup
    const int n = a.n;
    T *vL = reinterpret_cast<T *>(wave_smem);
    T *pL = vL + (n + PER16 - 1) / PER16 * PER16;  // padded blocks, then the overflow area
    for (int i = l; i < n * SOLO_DPAD; i += NL) pL[i] = (T)0.0;
    const bool p = __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;
    const T *V = (p ? a.v1 : a.v0) + (size_t)g * n;
    const T *CM = (p ? a.c1 : a.c0) + (size_t)g * a.m * 2;
    const int mlast = a.m - 1, nlast = n - 1;
    int va[CPL][3], tp[CPL][3];  // voltage index and term slot of each literal
    uint32_t sg[CPL][3];
    T xs[CPL], xl[CPL], mk[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = min(l + k * NL, mlast);
        const int4 r4 = a.rec4[c];
        const int lit[3] = {r4.x & 0xffff, r4.y & 0xffff, r4.z & 0xffff};
        const int pos[3] = {(int)((uint32_t)r4.x >> 16), (int)((uint32_t)r4.y >> 16), (int)((uint32_t)r4.z >> 16)};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int v = lit[j] >> 1, rank = pos[j] - a.vst[v];
            va[k][j] = v;
            tp[k][j] = rank < SOLO_DPAD ? v * SOLO_DPAD + rank : n * SOLO_DPAD + pos[j];
            sg[k][j] = (lit[j] & 1) ? 0x80000000u : 0u;
        }
        xs[k] = CM[2 * c];
        xl[k] = CM[2 * c + 1];
        mk[k] = (T)0.0;
    }
    int vs[VPL], vd[VPL], dw[VPL];  // term range start, degree, the wave's largest degree (uniform)
    T vr[VPL], vf[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int i = l + j * NL, ii = min(i, nlast);
        vs[j] = a.vst[ii];
        vd[j] = i < n ? a.vst[ii + 1] - vs[j] : 0;
        int mx = vd[j];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) mx = max(mx, __shfl_xor(mx, off, 64));
        dw[j] = __builtin_amdgcn_readfirstlane(mx);
        vr[j] = V[ii];
        vf[j] = vr[j];
        if (i < n) vL[i] = vr[j];
    }
    if (l < 2 * (SOLO_MAX_NL / 64)) voteW[l >> 4][l & 15] = 0;
    if (l < 2) errM[l] = 0;
    __syncthreads();
    int act = 1;
    int64_t sat = io_sat(a.io, a.sat_step, g), done = io_done(a.io, a.steps_done, g);
    T dtr = ADAPTIVE ? io_dt<T>(a.io, a.dtr, g) : a.dt;
    const int w = l >> 6;
    auto vote = [&](bool u, int k) {
        const bool wu = __any(u);
        if ((l & 63) == 0) voteW[k & 1][w] = wu ? 1 : 0;
    };
    auto votes = [&](int k) {
        const int4 *vw = reinterpret_cast<const int4 *>(voteW[k & 1]);
        int4 r4[SOLO_MAX_NL / 256];
#pragma unroll
        for (int j = 0; j < SOLO_MAX_NL / 256; ++j) r4[j] = vw[j];
        int r = 0;
#pragma unroll
        for (int j = 0; j < SOLO_MAX_NL / 256; ++j) r |= r4[j].x | r4[j].y | r4[j].z | r4[j].w;
        return r != 0;
    };
    // the clause pass: gathers of every slot first, then `mid` (work that overlaps them), then each
    // slot's terms; mn into mn_o; unsat
    auto clauses = [&](const T (&txs)[CPL], const T (&txl)[CPL], T (&mn_o)[CPL], auto &&mid) -> bool {
        T vv[CPL][3];
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) vv[k][j] = vL[va[k][j]];
        mid();
        bool uns = false;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (l + k * NL < a.m) {
                T d[3];
                mn_o[k] = solo_terms<T>(vv[k], sg[k], txl[k] * txs[k], d);
#pragma unroll
                for (int j = 0; j < 3; ++j) pL[tp[k][j]] = d[j];
                uns = uns || !(mn_o[k] < (T)0.5);  // :88
            }
        return uns;
    };
    // the fold of every variable slot (2 dv: the reference's left fold of the 2x terms)
    auto fold = [&]() {  // the reads of every variable slot's padded block
        Terms r;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const TV *b = reinterpret_cast<const TV *>(pL + (size_t)min(l + j * NL, nlast) * SOLO_DPAD);
#pragma unroll
            for (int q = 0; q < SOLO_DPAD / PER16; ++q) r.t[j][q] = b[q];
        }
        return r;
    };
    auto fold_sum = [&](const Terms &r, T (&dv)[VPL]) {
        const auto &t = r.t;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            T x = (T)0.0 + t[j][0][0];  // :33, the first term
#pragma unroll
            for (int u = 1; u < SOLO_DPAD; ++u)
                if (u < dw[j]) x = x + t[j][u / PER16][u % PER16];  // uniform bound: slots past a degree are +0
            if (dw[j] > SOLO_DPAD)                                  // (uniform) terms of rank >= SOLO_DPAD
                for (int u = SOLO_DPAD; u < vd[j]; ++u) x = x + pL[n * SOLO_DPAD + vs[j] + u];
            dv[j] = x;
        }
    };
    T mn2[CPL], xsf[CPL], xlf[CPL], xsh[CPL], xlh[CPL];
#ifdef SOLO_STAMPS
    uint64_t st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = solo_memtime();
#endif
    auto nop = [] {};
    // :133-135 dt <- clamp(dt * sqrt(tol / err), 2^-7, 1e3), err = the step's max_error (errM)
    auto dt_next = [&](int k) { return dmax(dmin(dtr * dsqrt((T)a.tol / frombits(errM[k & 1])), (T)1e3), (T)0.0078125); };
    bool pend = false;  // SOLO_DT_LATE: the previous step was taken and its dt update is still due
    int klast = 0;
    for (int k = 0; k < a.nsteps; ++k) {
        const int step = a.step0 + k;
        klast = k;
        T h = dtr, hh = (T)0.5 * h, hq = (T)0.25 * h;
        T e = (T)0.0;
        bool uns, go = false;
        if (!ADAPTIVE) {  // euler_step_fixed (system.rs:141-154): the update is taken regardless
            vote(clauses(xs, xl, mk, nop), k);
            __syncthreads();  // the terms (and the votes) before the fold
            const Terms t = fold();
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                if (l + c * NL < a.m) solo_mem<T>(xs[c], xl[c], mk[c], hh, h, a.xl_max, xs[c], xl[c]);
            uns = votes(k);
            T dv[VPL];
            fold_sum(t, dv);
#pragma unroll
            for (int j = 0; j < VPL; ++j)
                if (l + j * NL < n) {
                    vr[j] = dmin(dmax(vr[j] + hh * dv[j], (T)-1.0), (T)1.0);  // :96 (h dv = (h/2) (2 dv))
                    vL[l + j * NL] = vr[j];
                }
        } else {  // euler_step (:111-139)
#if SOLO_DT_LATE
            // the previous step's dt update under this pass's gathers (errM[k - 1] is final: the
            // previous step's closing barrier ordered every wave's atomic max)
            auto late = [&] {
                const T nd = dt_next(k - 1);
                dtr = pend ? nd : dtr;
            };
            vote(clauses(xs, xl, mk, late), k);  // the RHS at y, y's memories
            h = dtr;
            hh = (T)0.5 * h;
            hq = (T)0.25 * h;
#else
            vote(clauses(xs, xl, mk, nop), k);  // the RHS at y, y's memories
#endif
            SOLO_STAMP(0);
            __syncthreads();
            SOLO_STAMP(1);
            // the fold's reads go out with the vote's (one LDS round trip, not two); an allsat
            // replica discards them (SOLO_FOLD_EARLY=0: after the vote, A/B)
#if SOLO_FOLD_EARLY
            const Terms t = fold();
#endif
            uns = votes(k);
            go = uns;  // an allsat replica takes no step (:122)
            if (go) {
#if !SOLO_FOLD_EARLY
                const Terms t = fold();
#endif
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    if (l + c * NL < a.m) {  // the memories' full-step clone and first half step (:124-128)
                        solo_mem<T>(xs[c], xl[c], mk[c], hh, h, a.xl_max, xsf[c], xlf[c]);
                        solo_mem<T>(xs[c], xl[c], mk[c], hq, hh, a.xl_max, xsh[c], xlh[c]);
                    }
                T dv[VPL];
                fold_sum(t, dv);
#pragma unroll
                for (int j = 0; j < VPL; ++j)
                    if (l + j * NL < n) {
                        const T v = vr[j];
                        vf[j] = dmin(dmax(v + hh * dv[j], (T)-1.0), (T)1.0);  // full-step clone
                        vr[j] = dmin(dmax(v + hq * dv[j], (T)-1.0), (T)1.0);  // first half step
                        vL[l + j * NL] = vr[j];
                    }
            }
            SOLO_STAMP(2);
            __syncthreads();  // the half step's voltages before the second pass; the terms read
            SOLO_STAMP(3);
            if (go) clauses(xsh, xlh, mn2, nop);
            SOLO_STAMP(4);
            __syncthreads();  // the second pass's terms before its fold
            SOLO_STAMP(5);
            if (go) {
                const Terms t = fold();
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    if (l + c * NL < a.m) {  // second half step of the memories (:130), max_error (:132)
                        T xsn, xln;
                        solo_mem<T>(xsh[c], xlh[c], mn2[c], hq, hh, a.xl_max, xsn, xln);
                        e = dmax(e, dmax(dabs(xsf[c] - xsn), dabs(xlf[c] - xln)));
                        xs[c] = xsn;
                        xl[c] = xln;
                    }
                T dv[VPL];
                fold_sum(t, dv);
#pragma unroll
                for (int j = 0; j < VPL; ++j)
                    if (l + j * NL < n) {
                        const T vn = dmin(dmax(vr[j] + hq * dv[j], (T)-1.0), (T)1.0);  // second half step
                        e = dmax(e, dabs(vf[j] - vn));  // :101-108
                        vr[j] = vn;
                        vL[l + j * NL] = vn;
                    }
                // (an LDS atomic max from every lane instead: 38 ms per criterion call against 12.6)
                const U eb = wave_max_bits(tobits(e));  // non-negative floats order as their bits
                if ((l & 63) == 0) atomicMax(&errM[k & 1], eb);
            }
            if (l == 0) errM[(k + 1) & 1] = 0;  // read at the start of step k, before this step's first barrier
        }
        done += 1;
        if (!uns) {  // allsat: the fixed step was still taken (:148-152); adaptive took none
            if (sat < 0) sat = step;
            if (a.stop_mode == ODESAT_STOP_EACH) act = 0;                            // simulate() breaks (:193)
            if (a.stop_mode == ODESAT_STOP_ANY && l == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
        }
        if (ADAPTIVE) SOLO_STAMP(6);
        __syncthreads();  // the voltages before the next step's gathers (and the error words)
#if SOLO_DT_LATE
        pend = go;
#else
        if (ADAPTIVE && go) dtr = dt_next(k);
#endif
        if (ADAPTIVE) SOLO_STAMP(7);
        if (!act) break;  // uniform
    }
    if (ADAPTIVE && SOLO_DT_LATE && pend) dtr = dt_next(klast);  // the last step's update
#ifdef SOLO_STAMPS
    if ((l & 63) == 0 && g == 0)
        for (int i = 0; i < 8; ++i) g_solo_stamps[(l >> 6) * 8 + i] = st_[i];
#endif
    const bool q = a.oop ? !p : p;
    T *Vo = (q ? a.v1 : a.v0) + (size_t)g * n;
    T *CMo = (q ? a.c1 : a.c0) + (size_t)g * a.m * 2;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
        if (l + j * NL < n) Vo[l + j * NL] = vr[j];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = l + k * NL;
        if (c < a.m) {
            CMo[2 * c] = xs[k];
            CMo[2 * c + 1] = xl[k];
        }
    }
    if (l == 0) {
        if (a.oop) a.par[g] = (uint8_t)q;
        a.act[g] = (uint8_t)act;
        a.sat_step[g] = sat;
        a.steps_done[g] = done;
        if (ADAPTIVE) a.dtr[g] = dtr;
        io_mirror<T>(a.io, g, sat, done, dtr, ADAPTIVE);
    }
}

// ------------------------------------------------------------------------------------------------
// k_solo_cv -- k_solo_fast with the voltages held by the clauses (round 5, the criterion's latency
// path).  k_solo_fast crosses lanes four times per adaptive step (terms -> fold -> half-step voltages ->
// clause gathers -> terms -> fold -> voltages -> gathers), each crossing an LDS store, a barrier and
// a dependent read.  Here every clause slot keeps the voltages of its own three literals in registers
// and folds their terms itself: variable i's dv is computed by every clause slot that holds i, from
// the same terms in the same order with the same expressions, so every copy is bit-identical to the
// one k_solo_fast's variable slot computes.  A pass is the clause arithmetic, the term stores, ONE
// barrier and the reads of the slot's three padded blocks (SOLO_DPAD terms each, +0 past the degree;
// the host picks this kernel only when no variable has more terms than that); no voltage crosses
// lanes.  Per step: fixed 1 barrier (k_solo_fast 2), adaptive 2 (4).
//   * LDS banks: a block's 16-byte reads from random variables conflict.  Blocks are SOLO_CV_BS
//     slots apart (one 16-byte pad: 80 bytes in f64, 48 in f32), so a block's bank set is one of 16
//     instead of 4; a read past the variable's degree, and every read of a slot without a clause,
//     goes to one shared block of zeros (every lane on it reads the same address: no conflict)
//     instead of the block's +0 padding; and the host places the clauses on lanes, orders each
//     clause's literals and places the blocks so that the lanes of a read's 16-lane groups meet few
//     shared bank sets (cv_layout.cpp).
//   * The two passes (and consecutive fixed steps) use two term areas, so a pass's stores never meet
//     the previous pass's reads: a slow lane's reads of area A finish before it reaches the barrier
//     that the next writer of A must pass first.
//   * The region after the first barrier has no branch: the adaptive step computes its first half
//     whether or not the replica is allsat (only the second half, after the second barrier, commits,
//     under the uniform vote: an allsat replica takes no step, :122), a clause slot past m stores its
//     terms to a sink word of its own lane, and the fold adds every padded slot.  So the term reads
//     go out right after the barrier, under the dt update's divide and square root (system.rs:133-135)
//     and the vote, instead of after them.
//   * Instruction count (the step is VALU-issue bound: ~300 instructions per wave per adaptive step
//     at ~4 cycles, PMC): the two areas sit SOLO_CV_AREA bytes apart, so one set of address VGPRs
//     serves both (the ds offset field); a literal's value 1 - q v is one fma with q v exact (=
//     solo_terms' 1 - flip(v)); VPL = 0 drops the degree-0 code when the formula has none.
//   * The adaptive error's wave max and LDS atomic max run after the second barrier and are read after
//     the next step's first.
//   * Variables of degree 0 (no clause holds them) belong to variable slots l, l + NL, ... that apply
//     the same update with dv = +0 (so a -0 voltage becomes +0 as in k_solo_fast); at the end each
//     variable is written by the slot holding its first incidence (rank 0).
// Bit-identical to k_solo_fast, k_solo, k_wave and the oracle (tests/test_gpu_parity.py,
// tests/test_gpu_fuzz.py).  At most 512 lanes (the three blocks' reads take 48 VGPRs per clause slot
// in f64).
// ------------------------------------------------------------------------------------------------
constexpr int SOLO_CV_MAX_NL = 512;
constexpr uint32_t SOLO_CV_AREA = 32768;  // bytes per term area: the second at a static offset (the ds
                                          // instructions' immediate), so both share the address VGPRs

// A k_solo_cv term area: blocks of SOLO_CV_BS slots (the variables' and the zero block, placed by
// cv_layout.cpp), then a sink word per lane; the blocks that fit SOLO_CV_AREA bytes
// (solo_cv_bs: solo_blocks.hpp)
__host__ __device__ constexpr int solo_cv_blk_cap(size_t tsize) {
    return ((int)(SOLO_CV_AREA / tsize) - SOLO_CV_MAX_NL) / solo_cv_bs(tsize);
}

template <typename T, bool ADAPTIVE, int CPL, int VPL>
__global__ __launch_bounds__(SOLO_CV_MAX_NL) void k_solo_cv(WArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char wave_smem[];
    using U = typename Bits<T>::U;
    constexpr int PER16 = 16 / (int)sizeof(T);
    constexpr int NB = SOLO_DPAD / PER16;  // 16-byte reads per padded block
    constexpr int BS = solo_cv_bs(sizeof(T));  // slots between blocks
    typedef T TV __attribute__((ext_vector_type(PER16)));
    __shared__ U errM[2];  // per step parity: the max_error bits of the step (the waves' LDS atomic max)
    __shared__ __attribute__((aligned(16))) int voteW[2][SOLO_CV_MAX_NL / 64];
    const int NL = (int)blockDim.x, l = (int)threadIdx.x;
    const int g = blockIdx.x;
    if (l == 0 && g < a.G) io_begin_store<T>(a.io, g, a.act, a.sat_step, a.steps_done, a.dtr, ADAPTIVE, a.stop);
    if (a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0) return;  // an earlier step stopped every replica
    if (g >= a.G || !io_active(a.io, a.act, g)) return;                // uniform per workgroup
    const int n = a.n, m = a.m;
    {
        T *P0 = reinterpret_cast<T *>(wave_smem), *P1 = reinterpret_cast<T *>(wave_smem + SOLO_CV_AREA);
        for (int i = l; i < a.cvnb * BS; i += NL) {
            P0[i] = (T)0.0;
            P1[i] = (T)0.0;
        }
    }
    const bool p = __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;
    const T *V = (p ? a.v1 : a.v0) + (size_t)g * n;
    const T *CM = (p ? a.c1 : a.c0) + (size_t)g * m * 2;
    int ci[CPL];                  // the slot's clause (-1: none)
    int vi[CPL][3];               // variable of each literal
    uint32_t tp[CPL][3];          // byte offset of its term slot in an area (a slot past m: its lane's sink word)
    uint32_t ra[CPL][3][NB];      // byte offset of each 16-byte read of its block (the zero block past the degree)
    uint32_t sg[CPL][3];
    T nq[CPL][3];                 // -q_j: 1 for a negated literal, -1 otherwise (val = 1 - q v = fma(nq, v, 1))
    bool ok[CPL], own[CPL][3];    // a clause slot below m; the literal is its variable's first incidence
    T vv[CPL][3], xs[CPL], xl[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int4 r4 = a.cvrec[l + k * NL];  // (a slot without a clause: clause 0's literals, w = -1)
        ci[k] = r4.w;
        ok[k] = r4.w >= 0;
        const int c = ok[k] ? r4.w : 0;
        const int lit[3] = {r4.x & 0xffff, r4.y & 0xffff, r4.z & 0xffff};
        const int pos[3] = {(int)((uint32_t)r4.x >> 16), (int)((uint32_t)r4.y >> 16), (int)((uint32_t)r4.z >> 16)};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int v = lit[j] >> 1, rank = pos[j] - a.vst[v], deg = a.vst[v + 1] - a.vst[v];
            const int b = a.cvblk[v], zb = a.cvblk[n];
            vi[k][j] = v;
            tp[k][j] = (uint32_t)(ok[k] ? b * BS + rank : a.cvnb * BS + l) * (uint32_t)sizeof(T);  // (rank < SOLO_DPAD: host)
#pragma unroll
            for (int q = 0; q < NB; ++q)
                ra[k][j][q] = (uint32_t)((ok[k] && q * PER16 < deg ? b : zb) * BS + q * PER16) * (uint32_t)sizeof(T);
            sg[k][j] = (lit[j] & 1) ? 0x80000000u : 0u;
            nq[k][j] = (lit[j] & 1) ? (T)1.0 : (T)-1.0;
            own[k][j] = ok[k] && rank == 0;
            vv[k][j] = V[v];
        }
        xs[k] = CM[2 * c];
        xl[k] = CM[2 * c + 1];
    }
    bool z0[VPL > 0 ? VPL : 1];  // variable slots of degree 0 (VPL = 0: the formula has none)
    T vr[VPL > 0 ? VPL : 1];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int i = l + j * NL, ii = min(i, n - 1);
        z0[j] = i < n && a.vst[ii + 1] == a.vst[ii];
        vr[j] = V[ii];
    }
    if (l < 2 * (SOLO_CV_MAX_NL / 64)) voteW[l >> 3][l & 7] = 0;
    if (l < 2) errM[l] = 0;
    __syncthreads();
    int act = 1;
    int64_t sat = io_sat(a.io, a.sat_step, g), done = io_done(a.io, a.steps_done, g);
    T dtr = ADAPTIVE ? io_dt<T>(a.io, a.dtr, g) : a.dt;
    const int w = l >> 6;
    auto vote = [&](bool u, int k) {
        const bool wu = __any(u);
        if ((l & 63) == 0) voteW[k & 1][w] = wu ? 1 : 0;
    };
    auto votes = [&](int k) {
        const int4 *vw = reinterpret_cast<const int4 *>(voteW[k & 1]);
        int4 r4[SOLO_CV_MAX_NL / 256];
#pragma unroll
        for (int j = 0; j < SOLO_CV_MAX_NL / 256; ++j) r4[j] = vw[j];
        int r = 0;
#pragma unroll
        for (int j = 0; j < SOLO_CV_MAX_NL / 256; ++j) r |= r4[j].x | r4[j].y | r4[j].z | r4[j].w;
        return r != 0;
    };
    // a pass's clause arithmetic (solo_terms' expressions, the literal's sign by fma: 1 - q v with q v
    // exact) at voltages x with memories (txs, txl): terms into the area at byte offset OFF, mn into
    // mn_o; unsat
    auto terms = [&](auto off_c, const T (&x)[CPL][3], const T (&txs)[CPL], const T (&txl)[CPL], T (&mn_o)[CPL]) -> bool {
        constexpr uint32_t OFF = decltype(off_c)::value;
        bool uns = false;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const T tt = txl[k] * txs[k];
            const T val0 = fma(nq[k][0], x[k][0], (T)1.0), val1 = fma(nq[k][1], x[k][1], (T)1.0),
                    val2 = fma(nq[k][2], x[k][2], (T)1.0);  // :47
            const T sel[3] = {dmin(val1, val2), dmin(val0, val2), dmin(val0, val1)};
            mn_o[k] = dmin(sel[2], val2);  // :49-57
#pragma unroll
            for (int j = 0; j < 3; ++j)
                *reinterpret_cast<T *>(wave_smem + tp[k][j] + OFF) = sflip(tt * sel[j], sg[k][j]);  // 2 xl xs G (:64-70, :80)
            uns = uns || (ok[k] && !(mn_o[k] < (T)0.5));  // :88
        }
        return uns;
    };
    struct Blocks {
        TV t[CPL][3][NB];
    };
    auto reads = [&](auto off_c) {  // every literal's padded block in the area at byte offset OFF
        constexpr uint32_t OFF = decltype(off_c)::value;
        Blocks r;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int q = 0; q < NB; ++q) r.t[k][j][q] = *reinterpret_cast<const TV *>(wave_smem + ra[k][j][q] + OFF);
        return r;
    };
    // 2 dv of every literal's variable: the reference's left fold of the 2x terms (:33, :80).  Every
    // padded slot is added, so the 3 CPL chains interleave: the slots past a degree are +0, which
    // changes no sum (dv starts at +0 and is never -0)
    auto fold = [&](const Blocks &r, T (&dv)[CPL][3]) {
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) dv[k][j] = (T)0.0 + r.t[k][j][0][0];
#pragma unroll
        for (int u = 1; u < SOLO_DPAD; ++u)
#pragma unroll
            for (int k = 0; k < CPL; ++k)
#pragma unroll
                for (int j = 0; j < 3; ++j) dv[k][j] = dv[k][j] + r.t[k][j][u / PER16][u % PER16];
    };
    auto clamp1 = [](T x) { return dmin(dmax(x, (T)-1.0), (T)1.0); };
    const T zero = (T)0.0 + (T)0.0;  // 2 dv of a variable without terms (k_solo_fast's fold of a +0 block)
    using A0 = std::integral_constant<uint32_t, 0>;
    using A1 = std::integral_constant<uint32_t, SOLO_CV_AREA>;
    T mn1[CPL], mn2[CPL];
    auto dt_next = [&](int k) { return dmax(dmin(dtr * dsqrt((T)a.tol / frombits(errM[k & 1])), (T)1e3), (T)0.0078125); };
    bool pend = false;  // the previous step was taken and its dt update is still due
    int klast = 0;
#ifdef SOLO_STAMPS
    uint64_t st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = solo_memtime();
#endif
    // the bookkeeping after step k (uns: some clause unsat); false: the replica stops
    auto book = [&](int k, bool uns) {
        done += 1;
        if (!uns) {  // allsat: the fixed step was still taken (:148-152); adaptive took none
            const int step = a.step0 + k;
            if (sat < 0) sat = step;
            if (a.stop_mode == ODESAT_STOP_EACH) act = 0;                            // simulate() breaks (:193)
            if (a.stop_mode == ODESAT_STOP_ANY && l == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
        }
        SOLO_STAMP(5);
        return act != 0;
    };
    if constexpr (!ADAPTIVE) {  // euler_step_fixed (system.rs:141-154): the update is taken regardless
        const T h = dtr, hh = (T)0.5 * h;
        // one step with its terms in the area at OFF (steps alternate areas: unrolled by two)
        auto step = [&](auto off_c, int k) {
            vote(terms(off_c, vv, xs, xl, mn1), k);
            SOLO_STAMP(0);
            __syncthreads();  // the terms (and the votes) before the fold
            SOLO_STAMP(1);
            const Blocks r = reads(off_c);
            const bool uns = votes(k);
#pragma unroll
            for (int c = 0; c < CPL; ++c) solo_mem<T>(xs[c], xl[c], mn1[c], hh, h, a.xl_max, xs[c], xl[c]);
            T dv[CPL][3];
            fold(r, dv);
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int j = 0; j < 3; ++j) vv[c][j] = clamp1(vv[c][j] + hh * dv[c][j]);  // :96
#pragma unroll
            for (int j = 0; j < VPL; ++j) {
                const T x = clamp1(vr[j] + hh * zero);
                vr[j] = z0[j] ? x : vr[j];
            }
            SOLO_STAMP(2);
            return book(k, uns);
        };
        for (int k = 0; k < a.nsteps; k += 2) {
            if (!step(A0{}, k)) break;
            if (k + 1 < a.nsteps && !step(A1{}, k + 1)) break;
        }
    } else {  // euler_step (:111-139)
        for (int k = 0; k < a.nsteps; ++k) {
            klast = k;
            vote(terms(A0{}, vv, xs, xl, mn1), k);  // the RHS at y, y's memories
            SOLO_STAMP(0);
            __syncthreads();  // B1: the first pass's terms, the votes, the previous step's error
            SOLO_STAMP(1);
            const T nd = dt_next(k - 1);  // (its read first: the divide starts under the blocks' reads)
            const Blocks r1 = reads(A0{});
            const bool uns = votes(k);
            const bool go = uns;  // an allsat replica takes no step (:122)
            dtr = pend ? nd : dtr;
            const T h = dtr, hh = (T)0.5 * h, hq = (T)0.25 * h;
            // the first half of the step whether or not the replica is allsat (so the reads above go
            // out right after B1); only the second half, after B2, commits
            T xsf[CPL], xlf[CPL], xsh[CPL], xlh[CPL], vf[CPL][3], vh[CPL][3];
            T vf0[VPL > 0 ? VPL : 1], vh0[VPL > 0 ? VPL : 1];
#pragma unroll
            for (int c = 0; c < CPL; ++c) {  // the memories' full-step clone and first half step (:124-128)
                solo_mem<T>(xs[c], xl[c], mn1[c], hh, h, a.xl_max, xsf[c], xlf[c]);
                solo_mem<T>(xs[c], xl[c], mn1[c], hq, hh, a.xl_max, xsh[c], xlh[c]);
            }
            T dv[CPL][3];
            fold(r1, dv);
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    vf[c][j] = clamp1(vv[c][j] + hh * dv[c][j]);  // full-step clone
                    vh[c][j] = clamp1(vv[c][j] + hq * dv[c][j]);  // first half step
                }
#pragma unroll
            for (int j = 0; j < VPL; ++j) {
                vf0[j] = clamp1(vr[j] + hh * zero);
                vh0[j] = clamp1(vr[j] + hq * zero);
            }
            terms(A1{}, vh, xsh, xlh, mn2);  // the RHS at the half step
            SOLO_STAMP(2);
            __syncthreads();  // B2: the second pass's terms
            SOLO_STAMP(3);
            if (go) {  // (uniform)
                const Blocks r2 = reads(A1{});
                T ec[CPL];  // each slot's max_error terms (a slot past m does not count)
#pragma unroll
                for (int c = 0; c < CPL; ++c) {  // second half step of the memories (:130), max_error (:132)
                    T xsn, xln;
                    solo_mem<T>(xsh[c], xlh[c], mn2[c], hq, hh, a.xl_max, xsn, xln);
                    ec[c] = dmax(dabs(xsf[c] - xsn), dabs(xlf[c] - xln));
                    xs[c] = xsn;
                    xl[c] = xln;
                }
                fold(r2, dv);
#pragma unroll
                for (int c = 0; c < CPL; ++c)
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const T vn = clamp1(vh[c][j] + hq * dv[c][j]);  // second half step
                        ec[c] = dmax(ec[c], dabs(vf[c][j] - vn));        // :101-108
                        vv[c][j] = vn;
                    }
                T e = (T)0.0;  // (the max of finite non-negative terms: any order)
#pragma unroll
                for (int c = 0; c < CPL; ++c) e = ok[c] ? dmax(e, ec[c]) : e;
#pragma unroll
                for (int j = 0; j < VPL; ++j) {
                    const T vn = clamp1(vh0[j] + hq * zero);
                    const T ev = dmax(e, dabs(vf0[j] - vn));
                    e = z0[j] ? ev : e;
                    vr[j] = z0[j] ? vn : vr[j];
                }
                const U eb = wave_max_bits(tobits(e));  // non-negative floats order as their bits
                if ((l & 63) == 0) atomicMax(&errM[k & 1], eb);  // read after the next step's B1
            }
            if (l == 0) errM[(k + 1) & 1] = 0;  // the previous step's error was read before B2
            pend = go;
            SOLO_STAMP(4);
            if (!book(k, uns)) break;
        }
        __syncthreads();  // the last step's atomic max
        if (pend) dtr = dt_next(klast);
    }
#ifdef SOLO_STAMPS
    if ((l & 63) == 0 && g == 0)
        for (int i = 0; i < 8; ++i) g_solo_stamps[(l >> 6) * 8 + i] = st_[i];
#endif
    const bool q = a.oop ? !p : p;
    T *Vo = (q ? a.v1 : a.v0) + (size_t)g * n;
    T *CMo = (q ? a.c1 : a.c0) + (size_t)g * m * 2;
#pragma unroll
    for (int k = 0; k < CPL; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (own[k][j]) Vo[vi[k][j]] = vv[k][j];
#pragma unroll
    for (int j = 0; j < VPL; ++j)
        if (z0[j]) Vo[l + j * NL] = vr[j];
#pragma unroll
    for (int k = 0; k < CPL; ++k)
        if (ok[k]) {
            CMo[2 * ci[k]] = xs[k];
            CMo[2 * ci[k] + 1] = xl[k];
        }
    if (l == 0) {
        if (a.oop) a.par[g] = (uint8_t)q;
        a.act[g] = (uint8_t)act;
        a.sat_step[g] = sat;
        a.steps_done[g] = done;
        if (ADAPTIVE) a.dtr[g] = dtr;
        io_mirror<T>(a.io, g, sat, done, dtr, ADAPTIVE);
    }
}

// The launches of k_wave / k_solo / k_solo_fast / k_solo_cv live in wave_k.hip, a translation unit of their own
// built with the max-ILP machine scheduler (Makefile WAVE_FLAGS): prep = true sets the
// kernel's dynamic-LDS limit (once per device, outside any timed region), prep = false launches.
template <typename T, bool ADA, int WPW, int TW, bool FAST>
hipError_t wave_launch(bool prep, const WArgs<T> &a, unsigned grid, unsigned block, size_t lds, int lds_max,
                       hipStream_t st);
template <typename T, bool ADA, int CPL, int VPL, bool FAST>
hipError_t solo_launch(bool prep, const WArgs<T> &a, unsigned grid, unsigned block, size_t lds, int lds_max,
                       hipStream_t st);
template <typename T, bool ADA, int CPL, int VPL>
hipError_t solo_cv_launch(bool prep, const WArgs<T> &a, unsigned grid, unsigned block, size_t lds, int lds_max,
                          hipStream_t st);

}  // namespace odk

#ifdef SOLO_STAMPS
// Diagnostic build only: the per-wave stamp sums of replica 0's last k_solo launch, 16 waves x 8.
extern "C" int odesat_solo_stamps(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(odk::g_solo_stamps), sizeof(unsigned long long) * 128, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
