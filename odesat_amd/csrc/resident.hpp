// resident.hpp -- the LDS-resident persistent integrator (ALG_RESIDENT; included by odesat_hip.hip).
//
// One workgroup owns R replicas (the solver's group width W == R) for a launch of `nsteps` Euler
// steps.  Its voltages v[n][R] and derivative accumulators dv[n][R] live in LDS for the launch; per
// step only the clause memories stream through HBM, read once and written once (in place),
// coalesced.
//
// Clause tiles (built on the host): the clauses are stored in an internal order
// made of tiles such that (1) no two clauses of one tile share a variable and (2) for every
// variable, the tiles of its clauses increase in the reference's clause order.  A tile's lanes
// (lane = (clause, replica)) can then add their contributions G/R (system.rs:64-80) straight into
// dv[var] (LDS, no atomics, no contribution buffer): within a tile every dv[i] receives at most
// one clause's terms (in literal order, by one lane), and tiles run in order with a barrier between
// them, so every dv[i] is the reference's left fold over (clause, literal) -- bit-identical.
// After the last tile the variable phase applies :96 and resets dv.  Adaptive steps
// (system.rs:111-139) run two passes per step: the first writes the full-step and first-half
// memories to scratch, the second the second half in place plus max_error.
#pragma once

#include "kernels.hpp"

#include <type_traits>

namespace odk {

// Threads per workgroup: 512 for one replica (two workgroups share a CU), 1024 for R = 2, 4.
template <int R> struct ResShape {
    static constexpr int NTH = R == 1 ? 512 : 1024;
    static constexpr int NL = NTH / R;  // clause lanes = tile capacity in clauses
};
#ifndef RES_DEPTH_F32
#define RES_DEPTH_F32 4
#endif
constexpr int RES_DEPTH = RES_DEPTH_F32;  // tiles in flight per lane (3-SAT register prefetch ring)
// f64 rings (RES_DEPTH_F64; the host pads 3-SAT tilings to a multiple of 4 tiles, so a ring of 8
// ends with a static half block): twice the memory bytes in flight per lane
#ifndef RES_DEPTH_F64
#define RES_DEPTH_F64 8
#endif
template <typename T> constexpr int res_depth() { return sizeof(T) == 8 ? RES_DEPTH_F64 : RES_DEPTH; }
// register-tile launches (RC > 0): the ring beside the register tiles, fixed steps / adaptive steps
#ifndef RES_RC_DEPTH
#define RES_RC_DEPTH 4
#endif
#ifndef RES_RC_DEPTH_ADA
#define RES_RC_DEPTH_ADA 4
#endif

template <typename T> struct RArgs {
    const int4 *__restrict__ cl4;      // [m] 3-SAT: the clause's literals (var << 1 | neg), internal order
    const int32_t *__restrict__ cptr;  // [m+1] internal clause -> first slot
    const int32_t *__restrict__ lits;  // [L] literals by internal slot
    const int32_t *__restrict__ tc;    // [ntiles+1] first internal clause of each tile
    const int32_t *__restrict__ tcw;   // wave-paired tiles (PAIRS): wave w of tile t holds internal clauses
                                       // [tcw[8t+w], tcw[8t+w+1]), padded with m past the last tile
    T *v0, *v1, *c0, *c1;              // state buffers, group layout with W == R
    uint8_t *par;                      // flipped by an out-of-place launch
    T *cf, *ch;                        // adaptive scratch memories (full step, first half)
    T *vf;                             // adaptive full-step voltages in HBM (VFG: LDS holds only v and dv)
    T *dtr;
    uint8_t *act;
    int64_t *sat_step, *steps_done;
    int32_t *stop;
    int32_t n, m, ntiles;
    int32_t step0, nsteps, stop_mode;
    int32_t oop;  // fixed steps: the first step reads the par buffer and writes the other one (the
                  // launch's starting state survives for a STOP_ANY replay), then par flips
    T dt, zeta, xl_max;
    double tol;
    CallIO io;  // per-call bookkeeping (callio.hpp)
};

// Pass kinds: P_FIXED one fixed step in place; P_ADA1 each clause's C to scratch (the memories stay
// y); P_ADA2 recomputes the full-step and first-half candidates from y and that C, then the second
// half in place + max_error against the full-step candidate.
enum Pass : int { P_FIXED = 0, P_ADA1 = 1, P_ADA2 = 2 };

template <typename T, int R> struct ResCtx {
    T *vL, *dvL, *vfL;  // LDS
    T *cf, *ch;         // this group's adaptive scratch: cf holds each clause's first-pass C
    int r, lc;          // this lane's replica and clause-lane index
    int w, wl;          // PAIRS: this lane's wave (uniform) and lane in it
};

// The clause of this lane in tile t, and whether the slot holds one (if not, a valid clause index is
// still returned, for unconditional loads).  Plain tiles: the tile's clauses [tc[t], tc[t+1]) lane by
// lane.  Wave-paired tiles (PAIRS, odesat_hip.hip pair_tiles, as k_onchip runs them): wave w's
// clauses [tcw[8t+w], tcw[8t+w+1]) in its lanes, so a clause that depends on one of the same barrier
// interval sits in the same wave, whose LDS operations complete in issue order.
// PAIRS: 0 = plain tiles; 1 / 2 = wave-paired tiles with pair offset 0 / 1 (a barrier follows tile t iff
// t + PAIRS - 1 is odd).  The offset is a template parameter so that every tile's barrier is static.
template <int PAIRS> __host__ __device__ constexpr bool res_bar_after(int t) { return PAIRS == 0 || ((t + PAIRS - 1) & 1) != 0; }

template <typename T, int R, int PAIRS>
__device__ __forceinline__ int res_slot(const RArgs<T> &a, const ResCtx<T, R> &x, int t, bool &ok) {
    if constexpr (PAIRS != 0) {
        const int c0 = ldc(a.tcw, t * 8 + x.w), c1 = ldc(a.tcw, t * 8 + x.w + 1);
        const int c = c0 + x.wl;
        ok = c < c1;
        return ok ? c : (c1 > 0 ? c1 - 1 : 0);
    } else {
        const int tt = min(t, a.ntiles - 1);
        const int c0 = ldc(a.tc, tt), c1 = ldc(a.tc, tt + 1);
        const int c = c0 + x.lc;
        ok = t < a.ntiles && c < c1;
        return c < c1 ? c : (c1 > 0 ? c1 - 1 : 0);
    }
}

// base + element offset with a 32-bit BYTE offset: lets the compiler use the SGPR-base + 32-bit
// VGPR-offset form of global loads / stores (no 64-bit address arithmetic per lane)
template <typename P> __device__ __forceinline__ P *at(P *base, uint32_t elem) {
    using B = typename std::conditional<std::is_const<P>::value, const char, char>::type;
    return reinterpret_cast<P *>(reinterpret_cast<B *>(base) + (uint32_t)(elem * (uint32_t)sizeof(P)));
}

// Everything one lane loads for one tile (3-SAT): its clause's literals and memories.
template <typename T> struct TileLoad {
    int4 lit;
    Vec<T, 2> mem, full;
    bool ok;
};

// The clause memories stream through HBM once per pass; RES_NT=1 (experiment) moves them with
// non-temporal accesses so they do not evict the clause records every CU re-reads from L2.
#ifndef RES_NT
#define RES_NT 0
#endif
template <typename T> __device__ __forceinline__ Vec<T, 2> res_ldm(const T *p) {
    if constexpr (RES_NT != 0) {
        typedef T t2 __attribute__((ext_vector_type(2)));
        const t2 x = __builtin_nontemporal_load(reinterpret_cast<const t2 *>(p));
        Vec<T, 2> r;
        r.e[0] = x.x;
        r.e[1] = x.y;
        return r;
    } else {
        return ldv<T, 2>(p);
    }
}
// one word of the adaptive C scratch, with the memories' policy
template <typename T> __device__ __forceinline__ T res_ld1(const T *p) {
    if constexpr (RES_NT != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <typename T> __device__ __forceinline__ void res_st1(T *p, T x) {
    if constexpr (RES_NT != 0) __builtin_nontemporal_store(x, p);
    else *p = x;
}
template <typename T> __device__ __forceinline__ void res_stm(T *p, const Vec<T, 2> &v) {
    if constexpr (RES_NT != 0) {
        typedef T t2 __attribute__((ext_vector_type(2)));
        t2 x;
        x.x = v.e[0];
        x.y = v.e[1];
        __builtin_nontemporal_store(x, reinterpret_cast<t2 *>(p));
    } else {
        stv<T, 2>(p, v);
    }
}

// Loads of tile t (t >= ntiles: nothing to do, a valid address is read).  Unconditional, so the
// ring's loads stay in flight across iterations (no control flow for the wait counters to merge).
template <typename T, int R, int PK, int PAIRS = 0>
__device__ __forceinline__ void res_load3(const RArgs<T> &a, const ResCtx<T, R> &x, const T *CM, int t,
                                          TileLoad<T> &ld, bool mem = true) {
    const int cc = res_slot<T, R, PAIRS>(a, x, t, ld.ok);  // a valid clause
    // (one 12-byte load; three separate dword loads from SoA arrays avoid a register copy at the
    // ring's back-edge but measured 4% slower)
    ld.lit = *at(a.cl4, (uint32_t)cc);
    const uint32_t ci = (uint32_t)(cc * R + x.r) * 2u;  // 32-bit offsets from the group's base
    if (mem) ld.mem = res_ldm<T>(at(CM, ci));  // (adaptive: y's memories, untouched until the second pass stores)
    if (PK == P_ADA2 && mem) ld.full.e[0] = res_ld1<T>(at((const T *)x.cf, ci / 2u));  // the first pass's C
}

// The adaptive step's candidates for one clause's memories from y's memories and the first pass's
// C (system.rs:84-85, :124-128): the full-step clone f and the first half step hh.
template <typename T>
__device__ __forceinline__ void res_ada_mems(const RArgs<T> &a, const Vec<T, 2> &y, T C1, T h, Vec<T, 2> &f,
                                             Vec<T, 2> &hh) {
    const T one = (T)1.0, eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001, half = (T)0.5 * h;
    const T dxs = (T)20.0 * (y.e[0] + eps) * (C1 - (T)0.25);  // :84
    const T dxl = (T)5.0 * (C1 - (T)0.05);                    // :85
    f.e[0] = dmin(dmax(y.e[0] + h * dxs, eps), xs_hi);  // full-step clone (:124-125)
    f.e[1] = dmin(dmax(y.e[1] + h * dxl, one), a.xl_max);
    hh.e[0] = dmin(dmax(y.e[0] + half * dxs, eps), xs_hi);  // first half step (:128)
    hh.e[1] = dmin(dmax(y.e[1] + half * dxl, one), a.xl_max);
}

// Memory update of one clause (system.rs:84-85, 94-95 / :124-132); returns the max_error terms.
// copy: a fixed step written out of place -- a replica that does not step copies its memories.
template <typename T, int R, int PK>
__device__ __forceinline__ T res_mem_update(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, uint32_t ci, T C,
                                            const Vec<T, 2> &mem, const Vec<T, 2> &full, bool on, T h,
                                            bool copy) {
    const T one = (T)1.0, eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001;
    const T xs_m = mem.e[0], xl_m = mem.e[1];
    const T dxs = (T)20.0 * (xs_m + eps) * (C - (T)0.25);  // :84
    const T dxl = (T)5.0 * (C - (T)0.05);                  // :85
    T e = (T)0.0;
    if (!on) {
        if (PK == P_FIXED && copy) stv<T, 2>(at(CM, ci), mem);
        return e;
    }
    if (PK == P_FIXED) {
        Vec<T, 2> o;
        o.e[0] = dmin(dmax(xs_m + h * dxs, eps), xs_hi);
        o.e[1] = dmin(dmax(xl_m + h * dxl, one), a.xl_max);
        res_stm<T>(at(CM, ci), o);
    } else if (PK == P_ADA1) {
        // only C: the second pass recomputes the full-step clone and the first half step from it
        // and y's memories (res_ada_mems) -- the same expressions, so the same bits -- which moves
        // 12 bytes per clause less through HBM than storing both candidates
        *at(x.cf, ci / 2u) = C;
    } else {
        const T half = (T)0.5 * h;  // second half step (:130) and max_error terms (:132)
        Vec<T, 2> o;
        o.e[0] = dmin(dmax(xs_m + half * dxs, eps), xs_hi);
        o.e[1] = dmin(dmax(xl_m + half * dxl, one), a.xl_max);
        e = dmax(dabs(full.e[0] - o.e[0]), dabs(full.e[1] - o.e[1]));
        stv<T, 2>(at(CM, ci), o);
    }
    return e;
}

// A clause's three dv terms, computed ahead of the barrier that orders their application.
template <typename T> struct Pend {
    int idx[3];
    T d[3];
    bool ok;
};

// One 3-SAT clause of tile t from its prefetched loads: C, the memories' update and the three dv
// terms (system.rs:43-88).  Voltages are read-only during a pass, so this runs one tile ahead of
// the dv updates.
template <typename T, int R, int PK, bool FAST = false, int PAIRS = 0>
__device__ __forceinline__ void res_clause3(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, int t,
                                            const TileLoad<T> &ld, Pend<T> &P, bool on, T h, bool &uns, T &e,
                                            bool copy) {
    P.ok = ld.ok;
    if (!ld.ok) return;
    if constexpr (FAST) {
        // On in-range states (the host's `fast` launches) the exact short forms of k_solo_fast
        // (kernels.hpp solo_terms): each term tt min(other two values) with the literal's sign, R omitted,
        // 2 x the reference's terms (the variable phases halve h), the memory update from mn
        // (solo_mem); the first adaptive pass keeps mn (= 2 C) in the C scratch.
        bool ok_;
        const int c = res_slot<T, R, PAIRS>(a, x, t, ok_);
        const int lit[3] = {ld.lit.x, ld.lit.y, ld.lit.z};
        T v[3];
        uint32_t sg[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            P.idx[j] = (lit[j] >> 1) * R + x.r;
            sg[j] = (uint32_t)lit[j] << 31;
            v[j] = x.vL[P.idx[j]];
        }
        const uint32_t ci = (uint32_t)(c * R + x.r) * 2u;
        const T hh = (T)0.5 * h, hq = (T)0.25 * h;
        T xs = ld.mem.e[0], xl = ld.mem.e[1], xs_f = xs, xl_f = xl;
        if (PK == P_ADA2) {  // y's memories -> the full-step clone and the first half step (:124-128)
            // (the first pass's mn from the C scratch: recomputing it from y's voltages gathered from HBM
            // measured 22 % slower)
            const T mn1 = ld.full.e[0];
            solo_mem<T>(xs, xl, mn1, hh, h, a.xl_max, xs_f, xl_f);
            solo_mem<T>(ld.mem.e[0], ld.mem.e[1], mn1, hq, hh, a.xl_max, xs, xl);
        }
        const T mn = solo_terms<T>(v, sg, xl * xs, P.d);
        if (PK != P_ADA2) uns = uns || (on && !(mn < (T)0.5));  // :88
        if (!on) {
            if (PK == P_FIXED && copy) stv<T, 2>(at(CM, ci), ld.mem);
            return;
        }
        if (PK == P_FIXED) {
            Vec<T, 2> o;
            solo_mem<T>(xs, xl, mn, hh, h, a.xl_max, o.e[0], o.e[1]);
            res_stm<T>(at(CM, ci), o);
        } else if (PK == P_ADA1) {
            res_st1<T>(at(x.cf, ci / 2u), mn);
        } else {
            Vec<T, 2> o;
            solo_mem<T>(xs, xl, mn, hq, hh, a.xl_max, o.e[0], o.e[1]);  // second half step (:130)
            e = dmax(e, dmax(dabs(xs_f - o.e[0]), dabs(xl_f - o.e[1])));  // :132
            res_stm<T>(at(CM, ci), o);
        }
        return;
    }
    const T one = (T)1.0, halfc = (T)0.5;
    const int c = ldc(a.tc, t) + x.lc;
    const int lit[3] = {ld.lit.x, ld.lit.y, ld.lit.z};
    T v[3], q[3], val[3];
    T mn = inf_v<T>(), sec = inf_v<T>();
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // :43-57
        P.idx[j] = (lit[j] >> 1) * R + x.r;
        q[j] = (lit[j] & 1) ? (T)-1.0 : (T)1.0;
        v[j] = x.vL[P.idx[j]];
        val[j] = one - q[j] * v[j];
        minsec(val[j], mn, sec);
    }
    const T C = halfc * mn;  // :60
    Vec<T, 2> mem = ld.mem, full{};
    if (PK == P_ADA2) res_ada_mems(a, ld.mem, ld.full.e[0], h, full, mem);  // mem <- the first half step
    const T xs_m = mem.e[0], xl_m = mem.e[1];
    const T tt = xl_m * xs_m;
    const T tr = (one + a.zeta * xl_m) * (one - xs_m);
#pragma unroll
    for (int j = 0; j < 3; ++j) P.d[j] = tt * (halfc * q[j] * (val[j] != mn ? mn : sec));  // :64-70
    // :73-80.  R fires only if C == val, i.e. val = mn / 2 -- impossible when 0 < mn < inf (every
    // val >= mn > C).  Then tr * R = +-0 for finite tr, and adding a zero of either sign leaves dv
    // unchanged (dv starts at +0 and a sum of floats is -0 only if both terms are -0), so the wave
    // skips R unless some lane can fire it (|v| > 1 states) or has a non-finite tr.
    const bool quiet = mn > (T)0.0 && mn < inf_v<T>() && dabs(tr) < inf_v<T>();
    if (!__all(quiet)) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const T r_ = (C == one - q[j] * v[j]) ? halfc * (q[j] - v[j]) : (T)0.0;  // :73-77
            P.d[j] = P.d[j] + tr * r_;
        }
    }
    if (PK != P_ADA2) uns = uns || (on && !(C < (T)0.25));  // :88
    e = dmax(e, res_mem_update<T, R, PK>(a, x, CM, (uint32_t)(c * R + x.r) * 2u, C, mem, full, on, h, copy));
}

// :80 for one clause: dv[i_j] += d_j for j = 0, 1, 2 in order.  The three reads are issued
// together; a variable repeated inside the clause takes the running value, as the sequential
// updates would.
template <typename T, int R> __device__ __forceinline__ void res_apply3(const ResCtx<T, R> &x, const Pend<T> &P) {
    if (!P.ok) return;
    // (ds_add_f32 instead of this read-modify-write measured 4.3x slower on MI355X)
    const T o0 = x.dvL[P.idx[0]], o1 = x.dvL[P.idx[1]], o2 = x.dvL[P.idx[2]];
    const T a0 = o0 + P.d[0];
    const T a1 = (P.idx[1] == P.idx[0] ? a0 : o1) + P.d[1];
    const T a2 = (P.idx[2] == P.idx[1] ? a1 : (P.idx[2] == P.idx[0] ? a0 : o2)) + P.d[2];
    x.dvL[P.idx[0]] = a0;
    x.dvL[P.idx[1]] = a1;
    x.dvL[P.idx[2]] = a2;
}

// Tile t, any clause width (empty clauses included); loads issued here.
template <typename T, int R, int PK>
__device__ __forceinline__ void res_clause_any(const RArgs<T> &a, const ResCtx<T, R> &x, const T *CMr, T *CM, int t,
                                               bool on, T h, bool &uns, T &e) {
    const T one = (T)1.0, halfc = (T)0.5;
    const int c = ldc(a.tc, t) + x.lc;
    if (c >= ldc(a.tc, t + 1)) return;
    const int s0 = a.cptr[c], s1 = a.cptr[c + 1];
    const uint32_t ci = (uint32_t)(c * R + x.r) * 2u;
    Vec<T, 2> mem = ldv<T, 2>(CMr + ci);
    Vec<T, 2> full{};
    if (PK == P_ADA2) res_ada_mems(a, Vec<T, 2>(mem), x.cf[ci / 2u], h, full, mem);
    T mn = inf_v<T>(), sec = inf_v<T>();
    for (int s = s0; s < s1; ++s) {
        const int lit = a.lits[s];
        const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
        minsec(one - q * x.vL[(lit >> 1) * R + x.r], mn, sec);
    }
    const T C = halfc * mn;
    const T tt = mem.e[1] * mem.e[0];
    const T tr = (one + a.zeta * mem.e[1]) * (one - mem.e[0]);
    for (int s = s0; s < s1; ++s) {
        const int lit = a.lits[s];
        const int idx = (lit >> 1) * R + x.r;
        const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
        const T vi = x.vL[idx];
        const T val = one - q * vi;
        const T g_ = halfc * q * (val != mn ? mn : sec);
        const T r_ = (C == one - q * vi) ? halfc * (q - vi) : (T)0.0;
        x.dvL[idx] += tt * g_ + tr * r_;
    }
    if (PK != P_ADA2) uns = uns || (on && !(C < (T)0.25));
    e = dmax(e, res_mem_update<T, R, PK>(a, x, CM, ci, C, mem, full, on, h, CMr != CM));
}

// Register-cached tiles (RC > 0; f64 on in-range 3-SAT states, R = 1): the memories of the first RC
// tiles stay in the lane's VGPRs for the whole launch -- read from HBM once at its start and written
// once at its end -- and only the remaining tiles stream through HBM every step, as k_onchip keeps
// every tile (f32) in VGPRs.  Adaptive launches also keep each register tile's first-pass mn there
// (`rmn`, instead of the C scratch).  A register tile's clause: res_clause3's FAST forms with the
// memories in and out of `rmt`, branch-free -- an empty slot (!ld.ok: its literals are a valid
// clause's) computes too, but its terms are never applied, its vote and error are masked and its
// memories are never stored.
template <typename T, int R, int PK>
__device__ __forceinline__ void res_clause3_reg(const RArgs<T> &a, const ResCtx<T, R> &x, const TileLoad<T> &ld,
                                                Pend<T> &P, bool on, T h, bool &uns, T &e, Vec<T, 2> &rmt, T &rmn) {
    P.ok = ld.ok;
    const int lit[3] = {ld.lit.x, ld.lit.y, ld.lit.z};
    T v[3];
    uint32_t sg[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        P.idx[j] = (lit[j] >> 1) * R + x.r;
        sg[j] = (uint32_t)lit[j] << 31;
        v[j] = x.vL[P.idx[j]];
    }
    const T hh = (T)0.5 * h, hq = (T)0.25 * h;
    T xs = rmt.e[0], xl = rmt.e[1], xs_f = xs, xl_f = xl;
    if constexpr (PK == P_ADA2) {  // y's memories -> the full-step clone and the first half step (:124-128)
        solo_mem<T>(rmt.e[0], rmt.e[1], rmn, hh, h, a.xl_max, xs_f, xl_f);
        solo_mem<T>(rmt.e[0], rmt.e[1], rmn, hq, hh, a.xl_max, xs, xl);
    }
    const T mn = solo_terms<T>(v, sg, xl * xs, P.d);
    if constexpr (PK != P_ADA2) uns = uns || (on && ld.ok && !(mn < (T)0.5));  // :88
    if constexpr (PK == P_FIXED) {
        T xs_n, xl_n;
        solo_mem<T>(xs, xl, mn, hh, h, a.xl_max, xs_n, xl_n);
        rmt.e[0] = on ? xs_n : xs;
        rmt.e[1] = on ? xl_n : xl;
    } else if constexpr (PK == P_ADA1) {
        rmn = mn;  // the memories stay y until the second pass
    } else {
        T xs_n, xl_n;
        solo_mem<T>(xs, xl, mn, hq, hh, a.xl_max, xs_n, xl_n);  // second half step (:130)
        const T ec = dmax(e, dmax(dabs(xs_f - xs_n), dabs(xl_f - xl_n)));  // :132
        e = on && ld.ok ? ec : e;
        rmt.e[0] = on ? xs_n : rmt.e[0];
        rmt.e[1] = on ? xl_n : rmt.e[1];
    }
}

// Iteration TT of the pipeline below with a static tile index: tile TT+1's clause from the registers
// (TT+1 < RC) or from its slot, tile TT's terms applied, the slot refilled with tile TT+1+D (its
// memories only if that tile streams).
template <typename T, int R, int PK, bool FAST, int RC, int D, int PAIRS, int TT>
__device__ __forceinline__ void res_iter3_rc(const RArgs<T> &a, const ResCtx<T, R> &x, const T *CMr, T *CM,
                                             TileLoad<T> (&b)[D], Pend<T> &P, bool on, T h, bool &uns, T &e,
                                             Vec<T, 2> (&rm)[RC], T (&rmn)[RC]) {
    Pend<T> Q;
    TileLoad<T> &S = b[(TT + 1) % D];
    if constexpr (TT + 1 < RC) res_clause3_reg<T, R, PK>(a, x, S, Q, on, h, uns, e, rm[TT + 1], rmn[TT + 1]);
    else res_clause3<T, R, PK, FAST, PAIRS>(a, x, CM, TT + 1, S, Q, on, h, uns, e, CMr != CM);
    res_apply3<T, R>(x, P);
    res_load3<T, R, PK, PAIRS>(a, x, CMr, TT + 1 + D, S, TT + 1 + D >= RC);
#ifdef RES_TIMING_PAIRS  // timing-only diagnostic build (results race): a barrier after odd tiles only
    if (TT & 1)
#endif
    if constexpr (res_bar_after<PAIRS>(TT)) __syncthreads();  // PAIRS: after the pair's second tile only
    P = Q;
}
template <typename T, int R, int PK, bool FAST, int RC, int D, int PAIRS, int... Ts>
__device__ __forceinline__ void res_prefix(std::integer_sequence<int, Ts...>, const RArgs<T> &a, const ResCtx<T, R> &x,
                                           const T *CMr, T *CM, TileLoad<T> (&b)[D], Pend<T> &P, bool on, T h,
                                           bool &uns, T &e, Vec<T, 2> (&rm)[RC], T (&rmn)[RC]) {
    (res_iter3_rc<T, R, PK, FAST, RC, D, PAIRS, Ts>(a, x, CMr, CM, b, P, on, h, uns, e, rm, rmn), ...);
}

// One step of the 3-SAT tile pipeline: the terms of tile t+1 are computed from slot S (which is
// then refilled with tile t+1+RES_DEPTH), tile t's terms P are applied to dv, barrier (tile t+1
// may touch the same dv entries).
template <typename T, int R, int PK, bool FAST = false, int D = res_depth<T>(), int PAIRS = 0, bool BAR = true>
__device__ __forceinline__ void res_iter3(const RArgs<T> &a, const ResCtx<T, R> &x, const T *CMr, T *CM, int t,
                                          TileLoad<T> &S, Pend<T> &P, bool on, T h, bool &uns, T &e) {
    Pend<T> Q;
    res_clause3<T, R, PK, FAST, PAIRS>(a, x, CM, t + 1, S, Q, on, h, uns, e, CMr != CM);  // Q.ok = false past the last tile
    res_apply3<T, R>(x, P);
    res_load3<T, R, PK, PAIRS>(a, x, CMr, t + 1 + D, S);
#ifdef RES_TIMING_PAIRS  // timing-only diagnostic build (results race): a barrier after odd tiles only
    if (t & 1)
#endif
    if constexpr (BAR) __syncthreads();  // PAIRS: after the pair's second tile only (res_block)
    P = Q;
}
// Iterations t0 + Is of the pipeline (t0 even), slot (slot0 + Is) % D each, with their static barriers.
template <typename T, int R, int PK, bool FAST, int D, int PAIRS, int... Is>
__device__ __forceinline__ void res_block(std::integer_sequence<int, Is...>, const RArgs<T> &a, const ResCtx<T, R> &x,
                                          const T *CMr, T *CM, int t0, TileLoad<T> (&b)[D], Pend<T> &P, bool on, T h,
                                          bool &uns, T &e) {
    (res_iter3<T, R, PK, FAST, D, PAIRS, res_bar_after<PAIRS>(Is)>(a, x, CMr, CM, t0 + Is, b[(Is + 1) % D], P, on, h, uns,
                                                                   e),
     ...);
}

// One RHS pass over all tiles: dv (LDS) accumulates; memories are read from CMr (or the adaptive
// scratch) and written by kind (P_FIXED: to CM).  Ends with a barrier (dv complete).
template <typename T, int R, int PK, bool K3, bool FAST = false, int RC = 0, int PAIRS = 0>
__device__ __forceinline__ void res_pass(const RArgs<T> &a, const ResCtx<T, R> &x, const T *CMr, T *CM, bool on, T h,
                                         bool &uns, T &e, Vec<T, 2> (&rm)[RC > 0 ? RC : 1], T (&rmn)[RC > 0 ? RC : 1]) {
    const int NT_ = a.ntiles;
    if constexpr (K3) {
        // (register tiles: a ring of RES_RC_DEPTH, whose VGPRs the register tiles need more)
        constexpr int D = RC > 0 ? (PK == P_FIXED ? RES_RC_DEPTH : RES_RC_DEPTH_ADA) : res_depth<T>();
        static_assert(D == 4 || D == 8 || (D == 6 && RC > 0), "the pipeline below is unrolled for 4, 6 or 8 slots");
        static_assert(RC == 0 || (FAST && RC % D == 0 && RC >= D),
                      "register tiles: short-form steps, whole ring blocks (the host needs ntiles > RC + D)");
        // the host pads 3-SAT tilings to a multiple of 4 tiles (empty tiles), so the unrolled loop
        // below runs whole (D = 8: blocks of 8, then at most one static block of 4; D = 6, register
        // tiles only (a sweep point of RES_RC_DEPTH): blocks of 6, then a static block of 4 or 2)
        if (NT_ == 0) {
            __syncthreads();
            return;
        }
        TileLoad<T> b[D];
        Pend<T> P;
#pragma unroll
        for (int i = 0; i < D; ++i) res_load3<T, R, PK, PAIRS>(a, x, CMr, i, b[i], i >= RC);
        int t0 = 0;
        if constexpr (RC > 0) {
            res_clause3_reg<T, R, PK>(a, x, b[0], P, on, h, uns, e, rm[0], rmn[0]);
            res_load3<T, R, PK, PAIRS>(a, x, CMr, D, b[0], D >= RC);
            res_prefix<T, R, PK, FAST, RC, D, PAIRS>(std::make_integer_sequence<int, RC>{}, a, x, CMr, CM, b, P, on, h,
                                                     uns, e, rm, rmn);
            t0 = RC;
        } else {
            res_clause3<T, R, PK, FAST, PAIRS>(a, x, CM, 0, b[0], P, on, h, uns, e, CMr != CM);
            res_load3<T, R, PK, PAIRS>(a, x, CMr, D, b[0]);
        }
        // iteration t computes tile t+1 from slot (t+1) % D (t0 stays even: RC and D are multiples of 4)
        for (; t0 + D <= NT_; t0 += D)
            res_block<T, R, PK, FAST, D, PAIRS>(std::make_integer_sequence<int, D>{}, a, x, CMr, CM, t0, b, P, on, h, uns, e);
        if constexpr (D == 8) {
            if (t0 < NT_)  // four tiles left: slots 1 .. 4
                res_block<T, R, PK, FAST, D, PAIRS>(std::make_integer_sequence<int, 4>{}, a, x, CMr, CM, t0, b, P, on,
                                                    h, uns, e);
        }
        if constexpr (D == 6) {  // (t0 - RC is a multiple of 6 and NT_ - RC is even)
            if (NT_ - t0 == 4)
                res_block<T, R, PK, FAST, D, PAIRS>(std::make_integer_sequence<int, 4>{}, a, x, CMr, CM, t0, b, P, on,
                                                    h, uns, e);
            else if (NT_ - t0 == 2)
                res_block<T, R, PK, FAST, D, PAIRS>(std::make_integer_sequence<int, 2>{}, a, x, CMr, CM, t0, b, P, on,
                                                    h, uns, e);
        }
        if constexpr (PAIRS != 0) __syncthreads();  // dv complete whatever the last tile's parity
    } else {
        for (int t = 0; t < NT_; ++t) {
            res_clause_any<T, R, PK>(a, x, CMr, CM, t, on, h, uns, e);
            __syncthreads();
        }
    }
    if (!K3 && NT_ == 0) __syncthreads();
}

// NTHR threads per workgroup: ResShape<R>::NTH, or one wave (RES_NARROW) for instances whose tile
// chains are deep and narrow (a few dozen clauses per tile): one replica per wave, no idle waves.
// VFG (adaptive steps whose full-step voltage clone does not fit next to v and dv: f64 at n > 6.7 k):
// the clone lives in HBM (a.vf, the replica's own n words), written and read back by the same thread
// in the two variable phases of a step -- 2 n words of traffic per replica-step on top of the memories.
constexpr int RES_NARROW = 64;
// FAST (3-SAT, in-range states): res_clause3's short forms; the terms are 2 x the reference's, so every
// h of the variable phases is halved.
// Diagnostic build only (-DRES_STAMPS, scripts/build_variant.sh ... odesat_hip): per workgroup g < 4096,
// thread 0 records s_memrealtime (100 MHz) at entry, after v is in LDS, after each step k < 60 and
// at the end: g_res_stamps[g][0], [1], [2 + k], [63] (read by odesat_res_stamps; 0 = not reached).
// g_res_clk holds s_memtime (shader clock) at the same points: their ratio is the effective clock.
#ifdef RES_STAMPS
__device__ unsigned long long g_res_stamps[4096 * 64];
__device__ unsigned long long g_res_clk[4096 * 64];
#define RES_STAMP(i)                                                                                \
    do {                                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < 4096) {                                                \
            uint64_t t_, c_;                                                                        \
            asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_), "=s"(c_)::"memory"); \
            g_res_stamps[blockIdx.x * 64 + (i)] = t_;                                               \
            g_res_clk[blockIdx.x * 64 + (i)] = c_;                                                  \
        }                                                                                           \
    } while (0)
#else
#define RES_STAMP(i) do {} while (0)
#endif
template <typename T, int R, bool ADAPTIVE, bool K3, int NTHR, bool VFG = false, bool FAST = false, int RC = 0,
          int PAIRS = 0>
__global__ __launch_bounds__(NTHR) void k_resident(RArgs<T> a) {
    static_assert(!FAST || K3, "the short forms are 3-SAT only (res_clause_any has none)");
    static_assert(RC == 0 || (FAST && R == 1), "register tiles: short-form steps, R = 1");
    static_assert(!PAIRS || (FAST && R == 1 && NTHR == 512), "wave-paired tiles: 8 waves, one replica, short forms");
    extern __shared__ __attribute__((aligned(16))) unsigned char res_smem[];
    using U = typename Bits<T>::U;
    constexpr int NTH = NTHR, NL = NTHR / R;
    __shared__ uint32_t unsL[R];
    __shared__ U errL[R];
    __shared__ T dtL[R];
    __shared__ int actL[R];
    __shared__ int skipL;
    const int g = blockIdx.x;
    const int tid = threadIdx.x;
    RES_STAMP(0);
    ResCtx<T, R> x;
    x.r = tid % R;
    x.lc = tid / R;
    x.w = __builtin_amdgcn_readfirstlane(tid >> 6);
    x.wl = tid & 63;
    const size_t nR = (size_t)a.n * R;
    x.vL = reinterpret_cast<T *>(res_smem);
    x.dvL = x.vL + nR;
    x.vfL = VFG ? a.vf + (size_t)blockIdx.x * nR : x.dvL + nR;
    const bool p = __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;  // uniform: SGPR bases
    const bool oop = !ADAPTIVE && a.oop;
    T *V = (p ? a.v1 : a.v0) + (size_t)g * nR;
    T *CM = (p ? a.c1 : a.c0) + (size_t)g * a.m * R * 2;
    T *CMo = oop ? (p ? a.c0 : a.c1) + (size_t)g * a.m * R * 2 : CM;  // written (out of place: the other buffer)
    const T *CMr = CM;  // read: the launch's first step reads the starting state
    x.cf = ADAPTIVE ? a.cf + (size_t)g * a.m * R * 2 : nullptr;
    x.ch = ADAPTIVE ? a.ch + (size_t)g * a.m * R * 2 : nullptr;
    // per-replica bookkeeping (k_status's job in the other algorithms) lives in thread r < R
    int64_t sat = 0, done = 0;
    T dtr = a.dt;
    int act = 0;
    if (tid < R) {
        const int rg = g * R + tid;
        io_begin_store<T>(a.io, rg, a.act, a.sat_step, a.steps_done, a.dtr, ADAPTIVE, a.stop);
        act = io_active(a.io, a.act, rg);
        sat = io_sat(a.io, a.sat_step, rg);
        done = io_done(a.io, a.steps_done, rg);
        if (ADAPTIVE) dtr = io_dt<T>(a.io, a.dtr, rg);
        actL[tid] = act;
        dtL[tid] = dtr;
        unsL[tid] = 0u;
        errL[tid] = 0;
    }
    if (tid == 0) skipL = a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0;  // an earlier step stopped all
    __syncthreads();
    bool any = false;
#pragma unroll
    for (int j = 0; j < R; ++j) any = any || actL[j] != 0;
    if (skipL || !any) return;  // uniform
    // the register tiles' memories (RC > 0): read once here, written once after the last step
    Vec<T, 2> rm[RC > 0 ? RC : 1];
    T rmn[RC > 0 ? RC : 1];  // adaptive: each register tile's first-pass mn
    auto rm_slot = [&](int t, bool &ok) {  // tile t's slot of this lane (a valid clause when empty)
        const int c = res_slot<T, R, PAIRS>(a, x, t, ok);
        return (uint32_t)(c * R + x.r) * 2u;
    };
#pragma unroll
    for (int t = 0; t < RC; ++t) {
        bool ok;
        rm[t] = res_ldm<T>(at((const T *)CM, rm_slot(t, ok)));
    }
    copy_to_lds<8>(x.vL, V, tid, (int)nR, NTH);
    for (size_t i = tid; i < nR; i += NTH) x.dvL[i] = (T)0.0;  // :33
    __syncthreads();
    RES_STAMP(1);
    for (int k = 0; k < a.nsteps; ++k) {
        const int step = a.step0 + k;
        const bool on = actL[x.r] != 0;
        const T h = dtL[x.r];
        bool uns = false;
        T e = (T)0.0;
        if constexpr (!ADAPTIVE) {  // euler_step_fixed (system.rs:141-154)
            res_pass<T, R, P_FIXED, K3, FAST, RC, PAIRS>(a, x, CMr, CMo, on, h, uns, e, rm, rmn);
            CMr = CMo;
            if (uns) unsL[x.r] = 1u;
            const T hv = FAST ? (T)0.5 * h : h;
            for (int i = x.lc; i < a.n; i += NL) {  // :96, dv restarts at 0 (:33)
                const int idx = i * R + x.r;
                const T d = x.dvL[idx];
                x.dvL[idx] = (T)0.0;
                if (on) x.vL[idx] = dmin(dmax(x.vL[idx] + hv * d, (T)-1.0), (T)1.0);
            }
            __syncthreads();
            if (tid < R && act) {
                done += 1;
                if (unsL[tid] == 0u) {  // allsat: the step was still taken (:148-152)
                    if (sat < 0) sat = step;
                    if (a.stop_mode == ODESAT_STOP_EACH) act = 0;                 // simulate() breaks (:193)
                    if (a.stop_mode == ODESAT_STOP_ANY) atomicMin(a.stop, step);  // simulate_inter (:291)
                }
            }
        } else {  // euler_step (system.rs:111-139), per-replica dt
            res_pass<T, R, P_ADA1, K3, FAST, RC, PAIRS>(a, x, CM, CM, on, h, uns, e, rm, rmn);
            if (uns) unsL[x.r] = 1u;
            __syncthreads();
            const bool st = on && unsL[x.r] != 0u;  // allsat replicas take no step (:122)
            const T half = FAST ? (T)0.25 * h : (T)0.5 * h, hf = FAST ? (T)0.5 * h : h;
            for (int i = x.lc; i < a.n; i += NL) {
                const int idx = i * R + x.r;
                const T d = x.dvL[idx];
                x.dvL[idx] = (T)0.0;
                if (st) {
                    const T v = x.vL[idx];
                    x.vfL[idx] = dmin(dmax(v + hf * d, (T)-1.0), (T)1.0);   // full-step clone
                    x.vL[idx] = dmin(dmax(v + half * d, (T)-1.0), (T)1.0);  // first half step
                }
            }
            __syncthreads();
            bool any_st = false;
#pragma unroll
            for (int j = 0; j < R; ++j) any_st = any_st || (actL[j] != 0 && unsL[j] != 0u);
            if (any_st) {  // uniform
                bool u2 = false;
                res_pass<T, R, P_ADA2, K3, FAST, RC, PAIRS>(a, x, CM, CM, st, h, u2, e, rm, rmn);
                for (int i = x.lc; i < a.n; i += NL) {
                    const int idx = i * R + x.r;
                    const T d = x.dvL[idx];
                    x.dvL[idx] = (T)0.0;
                    if (st) {
                        const T vn = dmin(dmax(x.vL[idx] + half * d, (T)-1.0), (T)1.0);  // second half
                        e = dmax(e, dabs(x.vfL[idx] - vn));                               // :101-108
                        x.vL[idx] = vn;
                    }
                }
                if (st) atomicMax(&errL[x.r], tobits(e));
                __syncthreads();
            }
            if (tid < R && act) {
                done += 1;
                if (unsL[tid] == 0u) {
                    if (sat < 0) sat = step;
                    if (a.stop_mode == ODESAT_STOP_EACH) act = 0;
                    if (a.stop_mode == ODESAT_STOP_ANY) atomicMin(a.stop, step);
                } else {  // :133-135 dt <- clamp(dt * sqrt(tol / err), 2^-7, 1e3)
                    const T error = frombits(errL[tid]);
                    dtr = dmax(dmin(dtr * dsqrt((T)a.tol / error), (T)1e3), (T)0.0078125);
                }
            }
        }
        if (tid < R) {
            unsL[tid] = 0u;
            errL[tid] = 0;
            actL[tid] = act;
            dtL[tid] = dtr;
        }
        __syncthreads();
        if (k < 60) RES_STAMP(2 + k);
        bool still = false;
#pragma unroll
        for (int j = 0; j < R; ++j) still = still || actL[j] != 0;
        if (!still) break;  // uniform
    }
    T *Vo = oop ? (p ? a.v0 : a.v1) + (size_t)g * nR : V;
    if (oop && CMr != CMo) {  // no step ran (every replica of the group stopped at once): carry the memories
        for (size_t i = tid; i < (size_t)a.m * R * 2; i += NTH) CMo[i] = CM[i];
    }
    for (size_t i = tid; i < nR; i += NTH) Vo[i] = x.vL[i];
#pragma unroll
    for (int t = 0; t < RC; ++t) {
        bool ok;
        const uint32_t ci = rm_slot(t, ok);
        if (ok) res_stm<T>(at(CMo, ci), rm[t]);
    }
    if (oop && tid == 0) a.par[g] = (uint8_t)!p;
    if (tid < R) {
        const int rg = g * R + tid;
        a.act[rg] = (uint8_t)act;
        a.sat_step[rg] = sat;
        a.steps_done[rg] = done;
        if (ADAPTIVE) a.dtr[rg] = dtr;
        io_mirror<T>(a.io, rg, sat, done, dtr, ADAPTIVE);
    }
    RES_STAMP(63);
}

}  // namespace odk
