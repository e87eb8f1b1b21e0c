// resident.hpp -- the LDS-resident persistent integrator (ALG_RESIDENT; included by odesat_hip.hip).
//
// One workgroup owns R replicas (the solver's group width W == R) for a whole launch of `nsteps`
// Euler steps.  Its voltages v[n][R] live in LDS for the launch; per step only the clause memories
// stream through HBM, read once and written once (in place), coalesced ([m][R][2] per group).
//
// Per step the clauses are walked in tiles of consecutive clauses:
//   clause phase  lane = (clause, replica): gather the clause's literal voltages from LDS, min /
//                 second-min, C, the memories' update (system.rs:43-95), and each literal's
//                 contribution G/R (:64-80) into a tile buffer w (LDS) at the slot's position in the
//                 tile's variable-sorted order;
//   fold          lane = (segment, replica): a segment is one variable's slots inside the tile; the
//                 lane adds them, in order, to dv[var] (LDS).  Tiles are folded in clause order, so
//                 every dv[i] is the reference's left fold over (clause, literal) -- bit-identical.
// w is double-buffered: tile t+1's clause phase runs between the same two barriers as tile t's
// fold.  After the last tile the variable phase applies :96 and resets dv.
// Adaptive steps (system.rs:111-139) run two such passes per step: the first writes the full-step
// and first-half memories to scratch, the second the second half in place plus max_error.
#pragma once

#include "kernels.hpp"

namespace odk {

constexpr int RES_THREADS = 1024;
constexpr int RES_LIT_BITS = 17;  // packed slot word: (tile-local position << 17) | literal
constexpr int RES_LIT_MASK = (1 << RES_LIT_BITS) - 1;

template <typename T> struct RArgs {
    const int32_t *__restrict__ cl;    // [L] packed slot words, clause-major (file order)
    const int32_t *__restrict__ cptr;  // [m+1]
    const int32_t *__restrict__ tc;    // [ntiles+1] first clause of each tile
    const int32_t *__restrict__ tseg;  // [ntiles+1] first segment of each tile
    const int2 *__restrict__ seg;      // [nseg] {var, start | end << 16} (tile-local positions)
    T *v0, *v1, *c0, *c1;              // state buffers, group layout with W == R
    const uint8_t *par;
    T *cf, *ch;                        // adaptive scratch memories (full step, first half)
    T *dtr;
    uint8_t *act;
    int64_t *sat_step, *steps_done;
    int32_t *stop;
    int32_t n, m, ntiles, ts;          // ts: slot capacity of one tile buffer
    int32_t step0, nsteps, stop_mode;
    T dt, zeta, xl_max;
    double tol;
};

// Everything one lane loads for one tile (3-SAT): its clause's packed slot words and memories,
// and its (at most 3: a tile has <= 3 * NL segments) fold segments.
constexpr int RES_SPL = 3;
template <typename T> struct TileLoad {
    int32_t w0, w1, w2;
    Vec<T, 2> mem, full;
    int2 sg[RES_SPL];
    bool ok;
};

// Pass kinds: P_FIXED one fixed step in place; P_ADA1 full + first half candidates to scratch;
// P_ADA2 second half in place + max_error against the full-step candidate.
enum Pass : int { P_FIXED = 0, P_ADA1 = 1, P_ADA2 = 2 };

template <typename T, int R> struct ResCtx {
    T *vL, *dvL, *vfL, *wL;  // LDS
    T *cf, *ch;              // this group's adaptive scratch memories
    int r, lc;               // this lane's replica and clause-lane index
    static constexpr int NL = RES_THREADS / R;
};

template <typename T, int R, int PK>
__device__ __forceinline__ void res_load3(const RArgs<T> &a, const ResCtx<T, R> &g, const T *CM, int t,
                                          TileLoad<T> &x) {
    constexpr int NL = ResCtx<T, R>::NL;
    const int c = t * NL + g.lc;  // 3-SAT tiles are NL clauses wide
    x.ok = c < a.m;
    const int cc = x.ok ? c : t * NL;  // a valid clause of the tile (every tile is non-empty)
    const int s0 = ldc(a.tseg, t), s1 = ldc(a.tseg, t + 1);
#pragma unroll
    for (int k = 0; k < RES_SPL; ++k) {
        const int sidx = s0 + g.lc + k * NL;
        x.sg[k] = sidx < s1 ? a.seg[sidx] : make_int2(0, 0);
    }
    x.w0 = a.cl[(size_t)cc * 3];
    x.w1 = a.cl[(size_t)cc * 3 + 1];
    x.w2 = a.cl[(size_t)cc * 3 + 2];
    const size_t ci = ((size_t)cc * R + g.r) * 2;
    x.mem = ldv<T, 2>((PK == P_ADA2 ? g.ch : CM) + ci);
    if (PK == P_ADA2) x.full = ldv<T, 2>(g.cf + ci);
}

// Memory update of one clause (system.rs:84-85, 94-95 / :124-132); returns the max_error terms.
template <typename T, int R, int PK>
__device__ __forceinline__ T res_mem_update(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, size_t ci, T C,
                                            const Vec<T, 2> &mem, const Vec<T, 2> &full, bool on, T h) {
    const T one = (T)1.0, eps = (T)0.001, xs_hi = (T)1.0 - (T)0.001;
    const T xs_m = mem.e[0], xl_m = mem.e[1];
    const T dxs = (T)20.0 * (xs_m + eps) * (C - (T)0.25);  // :84
    const T dxl = (T)5.0 * (C - (T)0.05);                  // :85
    T e = (T)0.0;
    if (!on) return e;
    if (PK == P_FIXED) {
        Vec<T, 2> o;
        o.e[0] = dmin(dmax(xs_m + h * dxs, eps), xs_hi);
        o.e[1] = dmin(dmax(xl_m + h * dxl, one), a.xl_max);
        stv<T, 2>(CM + ci, o);
    } else if (PK == P_ADA1) {
        const T half = (T)0.5 * h;
        Vec<T, 2> f, hh;
        f.e[0] = dmin(dmax(xs_m + h * dxs, eps), xs_hi);  // full-step clone (:124-125)
        f.e[1] = dmin(dmax(xl_m + h * dxl, one), a.xl_max);
        hh.e[0] = dmin(dmax(xs_m + half * dxs, eps), xs_hi);  // first half step (:128)
        hh.e[1] = dmin(dmax(xl_m + half * dxl, one), a.xl_max);
        stv<T, 2>(x.cf + ci, f);
        stv<T, 2>(x.ch + ci, hh);
    } else {
        const T half = (T)0.5 * h;  // second half step (:130) and max_error terms (:132)
        Vec<T, 2> o;
        o.e[0] = dmin(dmax(xs_m + half * dxs, eps), xs_hi);
        o.e[1] = dmin(dmax(xl_m + half * dxl, one), a.xl_max);
        e = dmax(dabs(full.e[0] - o.e[0]), dabs(full.e[1] - o.e[1]));
        stv<T, 2>(CM + ci, o);
    }
    return e;
}

// Clause phase of tile t (3-SAT) from prefetched loads.
template <typename T, int R, int PK>
__device__ __forceinline__ void res_clause3(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, int t,
                                            const TileLoad<T> &ld, T *wbuf, bool on, T h, bool &uns, T &e) {
    if (!ld.ok) return;
    const T one = (T)1.0, halfc = (T)0.5;
    const int c = t * ResCtx<T, R>::NL + x.lc;
    const int w[3] = {ld.w0, ld.w1, ld.w2};
    T v[3], q[3], val[3];
    T mn = inf_v<T>(), sec = inf_v<T>();
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // :43-57
        const int lit = w[j] & RES_LIT_MASK;
        q[j] = (lit & 1) ? (T)-1.0 : (T)1.0;
        v[j] = x.vL[(lit >> 1) * R + x.r];
        val[j] = one - q[j] * v[j];
        minsec(val[j], mn, sec);
    }
    const T C = halfc * mn;  // :60
    const T xs_m = ld.mem.e[0], xl_m = ld.mem.e[1];
    const T tt = xl_m * xs_m;
    const T tr = (one + a.zeta * xl_m) * (one - xs_m);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const T g_ = halfc * q[j] * (val[j] != mn ? mn : sec);                  // :64-70
        const T r_ = (C == one - q[j] * v[j]) ? halfc * (q[j] - v[j]) : (T)0.0;  // :73-77
        wbuf[(w[j] >> RES_LIT_BITS) * R + x.r] = tt * g_ + tr * r_;            // :80 term
    }
    if (PK != P_ADA2) uns = uns || (on && !(C < (T)0.25));  // :88
    const T ee = res_mem_update<T, R, PK>(a, x, CM, ((size_t)c * R + x.r) * 2, C, ld.mem, ld.full, on, h);
    e = dmax(e, ee);
}

// Clause phase of tile t, any clause width (empty clauses included); no prefetch.
template <typename T, int R, int PK>
__device__ __forceinline__ void res_clause_any(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, int t, T *wbuf,
                                               bool on, T h, bool &uns, T &e) {
    const T one = (T)1.0, halfc = (T)0.5;
    const int c1 = ldc(a.tc, t + 1);
    for (int c = ldc(a.tc, t) + x.lc; c < c1; c += ResCtx<T, R>::NL) {
        const int s0 = a.cptr[c], s1 = a.cptr[c + 1];
        const size_t ci = ((size_t)c * R + x.r) * 2;
        const Vec<T, 2> mem = ldv<T, 2>((PK == P_ADA2 ? x.ch : CM) + ci);
        Vec<T, 2> full{};
        if (PK == P_ADA2) full = ldv<T, 2>(x.cf + ci);
        T mn = inf_v<T>(), sec = inf_v<T>();
        for (int s = s0; s < s1; ++s) {
            const int lit = a.cl[s] & RES_LIT_MASK;
            const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
            minsec(one - q * x.vL[(lit >> 1) * R + x.r], mn, sec);
        }
        const T C = halfc * mn;
        const T tt = mem.e[1] * mem.e[0];
        const T tr = (one + a.zeta * mem.e[1]) * (one - mem.e[0]);
        for (int s = s0; s < s1; ++s) {
            const int w = a.cl[s];
            const int lit = w & RES_LIT_MASK;
            const T q = (lit & 1) ? (T)-1.0 : (T)1.0;
            const T vi = x.vL[(lit >> 1) * R + x.r];
            const T val = one - q * vi;
            const T g_ = halfc * q * (val != mn ? mn : sec);
            const T r_ = (C == one - q * vi) ? halfc * (q - vi) : (T)0.0;
            wbuf[(w >> RES_LIT_BITS) * R + x.r] = tt * g_ + tr * r_;
        }
        if (PK != P_ADA2) uns = uns || (on && !(C < (T)0.25));
        e = dmax(e, res_mem_update<T, R, PK>(a, x, CM, ci, C, mem, full, on, h));
    }
}

// One fold segment: the variable's slots of the tile, added in order to its dv.
template <typename T, int R>
__device__ __forceinline__ void res_fold_seg(const ResCtx<T, R> &x, int2 sg, const T *wbuf) {
    const int start = sg.y & 0xFFFF, end = (int)((uint32_t)sg.y >> 16);
    if (start >= end) return;
    T d = x.dvL[sg.x * R + x.r];
    for (int p = start; p < end; ++p) d += wbuf[p * R + x.r];
    x.dvL[sg.x * R + x.r] = d;
}

// Fold of tile t (segments loaded here).
template <typename T, int R>
__device__ __forceinline__ void res_fold(const RArgs<T> &a, const ResCtx<T, R> &x, int t, const T *wbuf) {
    const int s0 = ldc(a.tseg, t), s1 = ldc(a.tseg, t + 1);
    for (int s = s0 + x.lc; s < s1; s += ResCtx<T, R>::NL) res_fold_seg<T, R>(x, a.seg[s], wbuf);
}

// One iteration of the 3-SAT tile pipeline: fold tile t-1 (slot P), clause phase of tile t (slot
// Cc), refill slot P with tile t-1+RES_DEPTH, barrier.
constexpr int RES_DEPTH = 4;
template <typename T, int R, int PK>
__device__ __forceinline__ void res_iter3(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, int t, TileLoad<T> &P,
                                          const TileLoad<T> &Cc, bool on, T h, bool &uns, T &e) {
    const int NT_ = a.ntiles;
    if (t > NT_) return;  // uniform
    T *w0 = x.wL, *w1 = x.wL + (size_t)a.ts * R;
    if (t >= 1) {
        const T *wb = ((t - 1) & 1) ? w1 : w0;
#pragma unroll
        for (int k = 0; k < RES_SPL; ++k) res_fold_seg<T, R>(x, P.sg[k], wb);
    }
    if (t < NT_) res_clause3<T, R, PK>(a, x, CM, t, Cc, (t & 1) ? w1 : w0, on, h, uns, e);
    if (t >= 1 && t - 1 + RES_DEPTH < NT_) res_load3<T, R, PK>(a, x, CM, t - 1 + RES_DEPTH, P);
    __syncthreads();
}

// One RHS pass over all tiles: dv (LDS) accumulates; memories are read from the pass's source and
// written by kind.  Ends with a barrier (dv complete, w free).
template <typename T, int R, int PK, bool K3>
__device__ __forceinline__ void res_pass(const RArgs<T> &a, const ResCtx<T, R> &x, T *CM, bool on, T h,
                                         bool &uns, T &e) {
    const int NT_ = a.ntiles;
    if (NT_ == 0) {
        __syncthreads();
        return;
    }
    T *w0 = x.wL, *w1 = x.wL + (size_t)a.ts * R;
    if constexpr (K3) {
        static_assert(RES_DEPTH == 4, "the pipeline below is unrolled for 4 slots");
        TileLoad<T> b0, b1, b2, b3;
        res_load3<T, R, PK>(a, x, CM, 0, b0);
        if (1 < NT_) res_load3<T, R, PK>(a, x, CM, 1, b1);
        if (2 < NT_) res_load3<T, R, PK>(a, x, CM, 2, b2);
        if (3 < NT_) res_load3<T, R, PK>(a, x, CM, 3, b3);
        for (int t0 = 0; t0 <= NT_; t0 += 4) {
            res_iter3<T, R, PK>(a, x, CM, t0, b3, b0, on, h, uns, e);
            res_iter3<T, R, PK>(a, x, CM, t0 + 1, b0, b1, on, h, uns, e);
            res_iter3<T, R, PK>(a, x, CM, t0 + 2, b1, b2, on, h, uns, e);
            res_iter3<T, R, PK>(a, x, CM, t0 + 3, b2, b3, on, h, uns, e);
        }
    } else {
        res_clause_any<T, R, PK>(a, x, CM, 0, w0, on, h, uns, e);
        __syncthreads();
        for (int t = 0; t < NT_; ++t) {
            res_fold<T, R>(a, x, t, (t & 1) ? w1 : w0);
            if (t + 1 < NT_) res_clause_any<T, R, PK>(a, x, CM, t + 1, (t & 1) ? w0 : w1, on, h, uns, e);
            __syncthreads();
        }
    }
}

template <typename T, int R, bool ADAPTIVE, bool K3>
__global__ __launch_bounds__(RES_THREADS) void k_resident(RArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char res_smem[];
    using U = typename Bits<T>::U;
    __shared__ uint32_t unsL[R];
    __shared__ U errL[R];
    __shared__ T dtL[R];
    __shared__ int actL[R];
    __shared__ int skipL;
    const int g = blockIdx.x;
    const int tid = threadIdx.x;
    constexpr int NL = ResCtx<T, R>::NL;
    ResCtx<T, R> x;
    x.r = tid % R;
    x.lc = tid / R;
    const size_t nR = (size_t)a.n * R;
    x.vL = reinterpret_cast<T *>(res_smem);
    x.dvL = x.vL + nR;
    x.vfL = x.dvL + nR;
    x.wL = ADAPTIVE ? x.vfL + nR : x.vfL;
    const bool p = a.par[g] != 0;
    T *V = (p ? a.v1 : a.v0) + (size_t)g * nR;
    T *CM = (p ? a.c1 : a.c0) + (size_t)g * a.m * R * 2;
    x.cf = ADAPTIVE ? a.cf + (size_t)g * a.m * R * 2 : nullptr;
    x.ch = ADAPTIVE ? a.ch + (size_t)g * a.m * R * 2 : nullptr;
    // per-replica bookkeeping (k_status's job in the other algorithms) lives in thread r < R
    int64_t sat = 0, done = 0;
    T dtr = a.dt;
    int act = 0;
    if (tid < R) {
        const int rg = g * R + tid;
        act = a.act[rg];
        sat = a.sat_step[rg];
        done = a.steps_done[rg];
        if (ADAPTIVE) dtr = a.dtr[rg];
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
    for (size_t i = tid; i < nR; i += RES_THREADS) {
        x.vL[i] = V[i];
        x.dvL[i] = (T)0.0;  // :33
    }
    __syncthreads();
    for (int k = 0; k < a.nsteps; ++k) {
        const int step = a.step0 + k;
        const bool on = actL[x.r] != 0;
        const T h = dtL[x.r];
        bool uns = false;
        T e = (T)0.0;
        if (!ADAPTIVE) {  // euler_step_fixed (system.rs:141-154)
            res_pass<T, R, P_FIXED, K3>(a, x, CM, on, h, uns, e);
            if (uns) unsL[x.r] = 1u;
            for (int i = x.lc; i < a.n; i += NL) {  // :96, dv restarts at 0 (:33)
                const int idx = i * R + x.r;
                const T d = x.dvL[idx];
                x.dvL[idx] = (T)0.0;
                if (on) x.vL[idx] = dmin(dmax(x.vL[idx] + h * d, (T)-1.0), (T)1.0);
            }
            __syncthreads();
            if (tid < R && act) {
                done += 1;
                if (unsL[tid] == 0u) {  // allsat: the step was still taken (:148-152)
                    if (sat < 0) sat = step;
                    if (a.stop_mode == ODESAT_STOP_EACH) act = 0;             // simulate() breaks (:193)
                    if (a.stop_mode == ODESAT_STOP_ANY) atomicMin(a.stop, step);  // simulate_inter (:291)
                }
            }
        } else {  // euler_step (system.rs:111-139), per-replica dt
            res_pass<T, R, P_ADA1, K3>(a, x, CM, on, h, uns, e);
            if (uns) unsL[x.r] = 1u;
            __syncthreads();
            const bool st = on && unsL[x.r] != 0u;  // allsat replicas take no step (:122)
            const T half = (T)0.5 * h;
            for (int i = x.lc; i < a.n; i += NL) {
                const int idx = i * R + x.r;
                const T d = x.dvL[idx];
                x.dvL[idx] = (T)0.0;
                if (st) {
                    const T v = x.vL[idx];
                    x.vfL[idx] = dmin(dmax(v + h * d, (T)-1.0), (T)1.0);  // full-step clone
                    x.vL[idx] = dmin(dmax(v + half * d, (T)-1.0), (T)1.0);  // first half step
                }
            }
            __syncthreads();
            bool any_st = false;
#pragma unroll
            for (int j = 0; j < R; ++j) any_st = any_st || (actL[j] != 0 && unsL[j] != 0u);
            if (any_st) {  // uniform
                bool u2 = false;
                res_pass<T, R, P_ADA2, K3>(a, x, CM, st, h, u2, e);
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
        bool still = false;
#pragma unroll
        for (int j = 0; j < R; ++j) still = still || actL[j] != 0;
        if (!still) break;  // uniform
    }
    for (size_t i = tid; i < nR; i += RES_THREADS) V[i] = x.vL[i];
    if (tid < R) {
        const int rg = g * R + tid;
        a.act[rg] = (uint8_t)act;
        a.sat_step[rg] = sat;
        a.steps_done[rg] = done;
        if (ADAPTIVE) a.dtr[rg] = dtr;
    }
}

}  // namespace odk
