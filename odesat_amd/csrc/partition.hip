// partition.hip -- one very large instance split across GPUs (BASELINE configs[4]):
// the fixed Euler step (system.rs:141-154) of a single replica whose clauses are partitioned over
// `world` ranks, one process per GPU.  The collective is the caller's (torch.distributed over RCCL);
// this file provides the per-rank kernels and their C ABI (include/odesat.h, odesat_part_*).
//
// Two partitions (the host builds the local topology, odesat_amd/partition.py):
//   CLAUSES    rank r owns a contiguous slice of the clauses and a full copy of v.  A step writes
//              the PARTIAL dv of every variable (its clauses' terms, folded in clause order) plus
//              its unsat flag; the ranks all-reduce (sum) that vector and apply the same update.
//              The summation order across ranks differs from the reference's fold: results match
//              it within a tolerance (bit-exact at world = 1).
//   VARIABLES  rank r owns variables [v0, v1) and EVERY clause touching them (clauses that span
//              ranks are evaluated -- identically -- by each rank that holds them).  A step folds
//              the complete dv of its own variables in the reference's clause order and writes
//              their updated voltages plus its unsat flag into a send block; the ranks
//              all-gather the blocks, which form the next step's voltage array.  Bit-exact for any
//              world size, and the exchange is half an all-reduce's bytes.
//   CLAUSES_RS rank r owns a slice of the clauses, as CLAUSES, but the all-reduce is split into its
//              two halves (SURVEY.md §8e's alternative): the partial dv of every variable is written
//              in the gathered layout below and reduce-scattered (sum) onto the ranks' variable
//              blocks; each rank updates its own block of voltages, and an all-gather of the blocks
//              rebuilds v.  Same bytes as a ring all-reduce, with the voltage update done once per
//              variable instead of on every rank; tolerance parity as CLAUSES (bit-exact at world 1).
// Gathered voltage layout (VARIABLES, CLAUSES_RS): world blocks of (S voltages, 1 unsat flag), so
// variable i sits at i + i / S.  CLAUSES uses a plain v[n] (stride 0).
//
// Arithmetic: the reference's expressions in the reference's order (system.rs:43-96), f32, with
// the rigidity term -- identical to the oracle's f32 restatement for any state.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <new>
#include <string>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"

using odesat::fail;

// Where the clause kernel puts a literal's term for the variable kernel (w):
//   SLOT    at its literal slot (coalesced stores); the variable kernel gathers it at random;
//   ELL     at its place in the variable kernel's sliced-ELL reads (scattered stores, coalesced reads);
//   REGION  the local variables are cut into `regions` contiguous ranges and region r's terms are
//           stored together, in slot order; the variable kernel folds region r on the blocks
//           b % 8 == r % 8 (one XCD under round-robin placement), so every line of w is fetched into
//           one XCD's L2 and its 16 terms are all read there -- the stores land in runs (a wave's 192
//           terms fall into `regions` runs), the gathers hit L2.  Placement is speed, never results.
enum { TERMS_SLOT = 0, TERMS_ELL = 1, TERMS_REGION = 2 };

// Device bookkeeping of the replica (the partitioned analogue of act / sat_step / steps_done).
struct PartStat {
    int64_t steps_done;  // steps taken (a frozen replica takes no more)
    int64_t sat_step;    // 0-based step whose pre-update state was allsat, -1 = none yet
    int32_t frozen;      // simulate() has stopped (system.rs:193): later steps are no-ops
    int32_t pad;
};

struct odesat_part {
    int device = 0, world = 1;
    int64_t n = 0, m = 0, mloc = 0, L = 0, v0 = 0, v1 = 0, S = 0, voff = 0;
    int32_t *cptr = nullptr, *lits = nullptr, *cstart = nullptr, *deg = nullptr, *islot = nullptr;
    int32_t *tpos = nullptr;  // ELL / REGION term layouts: slot -> the term's position in w
    int terms = 0;            // TERMS_SLOT / TERMS_ELL / TERMS_REGION (odesat_part_create)
    int regions = 0;          // TERMS_REGION: variable ranges, each folded on one XCD
    // every local clause has 3 literals: one literal record per clause (8 bytes, three 21-bit literals,
    // when every literal is below 2^21, else 16 bytes) and its 3 term positions as 3 planes of mloc
    void *lit3 = nullptr;
    int32_t *tpos3 = nullptr;
    bool lit_packed = false;
    int xcd_ranges = 0;  // k_part_clause3 placement: 8 = clause range x on the blocks b with b % 8 == x
    float *xs = nullptr, *xl = nullptr, *w = nullptr;
    PartStat *stat = nullptr;
    int64_t bytes = 0;
};

namespace {

#define PART_TRY(expr)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(ODESAT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

// Folds the previous step's global unsat flag(s) (VARIABLES: the world flag slots of the gathered
// voltages; CLAUSES: dvsum[n] after the all-reduce) into the replica's bookkeeping, then counts the
// step about to be taken.  stop = 1: an allsat step freezes the replica (simulate, system.rs:193).
__global__ void k_part_status(PartStat *st, const float *flags, int64_t stride, int count, int stop, int take) {
    if (threadIdx.x != 0) return;
    if (st->steps_done > 0 && !st->frozen && st->sat_step < 0) {
        float u = 0.0f;
        for (int r = 0; r < count; ++r) u += flags[(int64_t)r * stride];
        if (u == 0.0f) {
            st->sat_step = st->steps_done - 1;
            if (stop) st->frozen = 1;
        }
    }
    if (take && !st->frozen) st->steps_done += 1;
}

// Local clauses, one thread each: C (system.rs:43-60), each literal's term xl xs G + (1 + zeta xl)
// (1 - xs) R into w (:62-80), the memory update (:84-85, :94-95) and the unsat flag (:88).  lits hold
// the voltage's index in v's layout (premapped on the host) << 1 | neg.  The term of slot s goes to
// w[s] (SLOT layout: the variable kernel gathers it) or to w[tpos[s]] (ELL layout: its position in
// the variable kernel's coalesced reads; slots of variables another rank folds go to sink words).
template <bool ELL>
__global__ __launch_bounds__(256) void k_part_clause(const int32_t *__restrict__ cptr, const int32_t *__restrict__ lits,
                                                     const int32_t *__restrict__ tpos, const float *__restrict__ v,
                                                     float *__restrict__ xs, float *__restrict__ xl,
                                                     float *__restrict__ w, int32_t mloc, float dt, float zeta,
                                                     float xl_max, float *__restrict__ unsat,
                                                     const PartStat *__restrict__ st) {
    if (st->frozen) return;  // uniform
    const int32_t c = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    bool uns = false;
    if (c < mloc) {
        const int32_t s0 = cptr[c], s1 = cptr[c + 1];
        const float one = 1.0f, halfc = 0.5f;
        float mn = __builtin_huge_valf(), sec = __builtin_huge_valf();
        for (int32_t s = s0; s < s1; ++s) {  // :43-57, strict <
            const int32_t lit = lits[s];
            const float q = (lit & 1) ? -1.0f : 1.0f;
            const float val = one - q * v[lit >> 1];
            const bool lt = val < mn;
            sec = lt ? mn : (val < sec ? val : sec);
            mn = lt ? val : mn;
        }
        const float C = halfc * mn;  // :60
        const float xs_m = xs[c], xl_m = xl[c];
        for (int32_t s = s0; s < s1; ++s) {  // :62-80
            const int32_t lit = lits[s];
            const float q = (lit & 1) ? -1.0f : 1.0f;
            const float vi = v[lit >> 1];
            const float val = one - q * vi;
            const float g = halfc * q * (val != mn ? mn : sec);
            const float r = (C == one - q * vi) ? halfc * (q - vi) : 0.0f;
            w[ELL ? tpos[s] : s] = xl_m * xs_m * g + (one + zeta * xl_m) * (one - xs_m) * r;
        }
        const float dxs = 20.0f * (xs_m + 0.001f) * (C - 0.25f);  // :84
        const float dxl = 5.0f * (C - 0.05f);                      // :85
        xs[c] = fminf(fmaxf(xs_m + dt * dxs, 0.001f), 1.0f - 0.001f);  // :94
        xl[c] = fminf(fmaxf(xl_m + dt * dxl, one), xl_max);           // :95
        uns = !(C < 0.25f);                                            // :88
    }
    // one flag store per workgroup that has an unsat clause, skipped once the flag is visibly set
    if (__syncthreads_or(uns) && threadIdx.x == 0 && *(volatile float *)unsat == 0.0f) *unsat = 1.0f;
}

// The same for a 3-SAT slice: one literal record per clause (PACK: 8 bytes, literal j in bits
// [21j, 21j + 21); else 16 bytes) and three planes of term positions, so the three voltage gathers
// are independent loads in flight together (the generic loop above chains each gather behind its
// literal's load and the min / second-min update).
// The voltage table is gathered at random and should stay in the XCD's L2; the clause memories and
// the terms stream past it once per step, so they are loaded / stored non-temporally.  XR = 8: the
// (min-variable-sorted) clauses are cut into 8 equal ranges and range x runs on the blocks b with
// b % 8 == x -- under the round-robin block placement one XCD -- so an XCD's gathers touch only the
// voltages from its range's smallest variable up (placement is a speed choice, never correctness).
template <bool ELL, int XR, bool PACK>
__global__ __launch_bounds__(256) void k_part_clause3(const void *__restrict__ lit3, const int32_t *__restrict__ tpos3,
                                                      const float *__restrict__ v, float *__restrict__ xs,
                                                      float *__restrict__ xl, float *__restrict__ w, int32_t mloc,
                                                      float dt, float zeta, float xl_max, float *__restrict__ unsat,
                                                      const PartStat *__restrict__ st) {
    if (st->frozen) return;  // uniform
    int32_t c, cend = mloc;
    if (XR > 1) {
        const int32_t chunk = (mloc + XR - 1) / XR, x = (int32_t)(blockIdx.x % XR);
        c = x * chunk + (int32_t)(blockIdx.x / XR) * (int32_t)blockDim.x + (int32_t)threadIdx.x;
        cend = min(mloc, (x + 1) * chunk);
    } else {
        c = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    }
    bool uns = false;
    if (c < cend) {
        int lit[3];
        if (PACK) {
            const uint64_t r = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(lit3) + c);
            lit[0] = (int)(r & 0x1FFFFF);
            lit[1] = (int)((r >> 21) & 0x1FFFFF);
            lit[2] = (int)(r >> 42);
        } else {
            typedef int i4v __attribute__((ext_vector_type(4)));
            const i4v l4 = __builtin_nontemporal_load(reinterpret_cast<const i4v *>(lit3) + c);
            lit[0] = l4[0], lit[1] = l4[1], lit[2] = l4[2];
        }
        float vv[3], q[3], val[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) vv[j] = v[lit[j] >> 1];
        const float xs_m = __builtin_nontemporal_load(&xs[c]), xl_m = __builtin_nontemporal_load(&xl[c]);
        const float one = 1.0f, halfc = 0.5f;
        float mn = __builtin_huge_valf(), sec = __builtin_huge_valf();
#pragma unroll
        for (int j = 0; j < 3; ++j) {  // :43-57, strict <
            q[j] = (lit[j] & 1) ? -1.0f : 1.0f;
            val[j] = one - q[j] * vv[j];
            const bool lt = val[j] < mn;
            sec = lt ? mn : (val[j] < sec ? val[j] : sec);
            mn = lt ? val[j] : mn;
        }
        const float C = halfc * mn;  // :60
        float t[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {  // :62-80
            const float g = halfc * q[j] * (val[j] != mn ? mn : sec);
            const float r = (C == one - q[j] * vv[j]) ? halfc * (q[j] - vv[j]) : 0.0f;
            t[j] = xl_m * xs_m * g + (one + zeta * xl_m) * (one - xs_m) * r;
        }
        if (ELL) {  // scattered: plain stores (non-temporal scattered stores measured 2x slower)
            w[__builtin_nontemporal_load(&tpos3[c])] = t[0];
            w[__builtin_nontemporal_load(&tpos3[mloc + c])] = t[1];
            w[__builtin_nontemporal_load(&tpos3[2 * (int64_t)mloc + c])] = t[2];
        } else {
            __builtin_nontemporal_store(t[0], &w[3 * c]);
            __builtin_nontemporal_store(t[1], &w[3 * c + 1]);
            __builtin_nontemporal_store(t[2], &w[3 * c + 2]);
        }
        const float dxs = 20.0f * (xs_m + 0.001f) * (C - 0.25f);  // :84
        const float dxl = 5.0f * (C - 0.05f);                      // :85
        __builtin_nontemporal_store(fminf(fmaxf(xs_m + dt * dxs, 0.001f), 1.0f - 0.001f), &xs[c]);  // :94
        __builtin_nontemporal_store(fminf(fmaxf(xl_m + dt * dxl, one), xl_max), &xl[c]);            // :95
        uns = !(C < 0.25f);                                                                          // :88
    }
    if (__syncthreads_or(uns) && threadIdx.x == 0 && *(volatile float *)unsat == 0.0f) *unsat = 1.0f;
}

// Variables [v0, v1), one thread each: dv = the fold of the local terms in clause order (:33, :80).
// The incidences are sliced-ELL: chunk k of 64 variables stores its j-th incidences contiguously
// ([chunk][j][64], padded to the chunk's largest degree): SLOT layout reads the slot there and
// gathers its term, ELL layout reads the term itself there (the clause kernel put it there), both
// coalesced.  CLAUSES (apply == 0): out[i] = partial dv[i].  VARIABLES (apply == 1): out[i - v0] =
// the updated voltage (:96), v[i + voff] being variable i in the gathered layout.  CLAUSES_RS
// (apply == 2): out[i + i / S] = partial dv[i], and block 0's unsat flag (out[S], set by the clause
// kernel) is copied to the other world - 1 blocks' flag slots, so the reduce-scatter hands every
// rank the global count.
// REGION (RG > 0 regions, a multiple of 8): block b runs region x + 8 g (x = b % 8) with bpr blocks
// per region, so every region's variables are folded on one residue class of blockIdx mod 8.
template <bool ELL, bool REGION>
__global__ __launch_bounds__(256) void k_part_var(const int32_t *__restrict__ cstart, const int32_t *__restrict__ deg,
                                                  const int32_t *__restrict__ islot, const float *__restrict__ w,
                                                  const float *__restrict__ v, int32_t voff, int32_t v0, int32_t v1,
                                                  float dt, int apply, float *__restrict__ out,
                                                  const PartStat *__restrict__ st, int32_t RG, int32_t bpr,
                                                  int32_t S, int32_t world) {
    if (apply == 2 && blockIdx.x == 0)
        for (int32_t r = (int32_t)threadIdx.x + 1; r < world; r += (int32_t)blockDim.x)
            out[(int64_t)r * (S + 1) + S] = out[S];  // the clause kernel has finished
    int32_t k;
    if (REGION) {
        const int32_t nv = v1 - v0, x = (int32_t)(blockIdx.x % 8), kk = (int32_t)(blockIdx.x / 8);
        const int32_t r = x + 8 * (kk / bpr);
        if (r >= RG) return;
        const int32_t r0 = (int32_t)((int64_t)r * nv / RG), r1 = (int32_t)((int64_t)(r + 1) * nv / RG);
        k = r0 + (kk % bpr) * (int32_t)blockDim.x + (int32_t)threadIdx.x;
        if (k >= r1) return;
    } else {
        k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    }
    const int32_t i = v0 + k;
    if (i >= v1) return;
    const int32_t oi = apply == 2 ? i + i / S : i;
    if (st->frozen) {  // the replica stopped: v is re-sent unchanged, no dv
        if (apply == 1) out[k] = v[i + voff];
        else out[oi] = 0.0f;
        return;
    }
    const int32_t base = cstart[k >> 6] + (k & 63);
    const int32_t d = deg[k];
    float dv = 0.0f;
    if (ELL) {
        const float *q = w + base;
#pragma unroll 4
        for (int32_t j = 0; j < d; ++j) dv += q[64 * j];
    } else {
        // 8 incidences at a time: their positions, then their terms, are loaded together (clamped to
        // the last one, so the loads are unconditional), then added in order -- the fold stays the
        // reference's left fold; the loop trip count differs per lane, not the order of its adds
        const int32_t *p = islot + base;
        for (int32_t j0 = 0; j0 < d; j0 += 8) {
            int32_t pos[8];
            float t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) pos[u] = p[64 * min(j0 + u, d - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = w[pos[u]];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (j0 + u < d) dv += t[u];
        }
    }
    if (apply == 1) out[k] = fminf(fmaxf(v[i + voff] + dt * dv, -1.0f), 1.0f);
    else out[oi] = dv;
}

// CLAUSES: v[i] = clamp(v[i] + dt * dvsum[i]) after the all-reduce (:96).
__global__ __launch_bounds__(256) void k_part_apply(float *__restrict__ v, const float *__restrict__ dvsum, int32_t n,
                                                    float dt, const PartStat *__restrict__ st) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (st->frozen) return;
    if (i < n) v[i] = fminf(fmaxf(v[i] + dt * dvsum[i], -1.0f), 1.0f);
}

// CLAUSES_RS, after the reduce-scatter: rank r's voltages i in [r S, r S + cnt) (v[i + r] in the
// gathered layout) take the summed dv of its block (:96) into the send block, whose flag slot carries
// the summed unsat count on to the all-gather.
__global__ __launch_bounds__(256) void k_part_reduce_apply(const float *__restrict__ v, const float *__restrict__ blk,
                                                           float *__restrict__ send, int32_t S, int32_t rank,
                                                           int32_t cnt, float dt, const PartStat *__restrict__ st) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k == 0) send[S] = blk[S];
    if (k >= cnt) return;
    const float vi = v[(int64_t)rank * S + k + rank];
    send[k] = st->frozen ? vi : fminf(fmaxf(vi + dt * blk[k], -1.0f), 1.0f);
}

template <typename T> int upload(odesat_part *p, T **dst, const int64_t *src, int64_t count) {
    std::vector<T> h((size_t)count);
    for (int64_t k = 0; k < count; ++k) h[k] = (T)src[k];
    PART_TRY(hipMalloc((void **)dst, std::max<size_t>(16, (size_t)count * sizeof(T))));
    p->bytes += (int64_t)count * (int64_t)sizeof(T);
    if (count) PART_TRY(hipMemcpy(*dst, h.data(), (size_t)count * sizeof(T), hipMemcpyHostToDevice));
    return ODESAT_OK;
}

unsigned blocks_for(int64_t items) { return (unsigned)std::max<int64_t>(1, (items + 255) / 256); }

}  // namespace

extern "C" void odesat_part_destroy(odesat_part *p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    void *ptrs[] = {p->cptr, p->lits, p->cstart, p->deg, p->islot, p->xs, p->xl, p->w, p->stat, p->tpos, p->lit3, p->tpos3};
    for (void *q : ptrs)
        if (q) (void)hipFree(q);
    delete p;
}

extern "C" int odesat_part_create(int device, int world, int64_t n, int64_t m, int64_t mloc, const int64_t *clause_ptr, const int64_t *var,
                                  const uint8_t *neg, int64_t v0, int64_t v1, const int64_t *var_ptr,
                                  const int64_t *inc_slot, int64_t block, odesat_part **out) {
    if (!out) return fail(ODESAT_EINVAL, "null out");
    *out = nullptr;
    // block > 0 with the full range [0, n): CLAUSES_RS (every variable folded, gathered layout)
    if (world < 1 || n <= 0 || m < 0 || mloc < 0 || mloc > m || !clause_ptr || v0 < 0 || v1 < v0 || v1 > n ||
        block < 0 || (block > 0 && v1 - v0 > block && !(v0 == 0 && v1 == n)) || (block > 0 && world * block < n))
        return fail(ODESAT_EINVAL, "bad partition arguments");
    if (n >= (1ll << 29) || m >= INT32_MAX) return fail(ODESAT_EINVAL, "formula too large");
    const int64_t L = clause_ptr[mloc] - clause_ptr[0];
    if (L < 0 || L >= INT32_MAX || (L && (!var || !neg))) return fail(ODESAT_EINVAL, "bad local clause arrays");
    for (int64_t c = 0; c < mloc; ++c)
        if (clause_ptr[c + 1] < clause_ptr[c]) return fail(ODESAT_EINVAL, "clause_ptr must be non-decreasing");
    for (int64_t s = 0; s < L; ++s)
        if (var[s] < 0 || var[s] >= n) return fail(ODESAT_EINVAL, "variable out of range");
    const int64_t nv = v1 - v0;
    if (nv && (!var_ptr || var_ptr[0] != 0)) return fail(ODESAT_EINVAL, "bad var_ptr");
    const int64_t ninc = nv ? var_ptr[nv] : 0;
    for (int64_t k = 0; k < ninc; ++k)
        if (inc_slot[k] < 0 || inc_slot[k] >= L) return fail(ODESAT_EINVAL, "incidence slot out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(ODESAT_EDEVICE, "no HIP device available (odesat_amd has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(ODESAT_EINVAL, "device index out of range");
    PART_TRY(hipSetDevice(device));
    auto *p = new (std::nothrow) odesat_part();
    if (!p) return fail(ODESAT_ENOMEM, "out of memory");
    p->device = device;
    p->world = world;
    p->n = n;
    p->m = m;
    p->mloc = mloc;
    p->L = L;
    p->v0 = v0;
    p->v1 = v1;
    p->S = block;
    // literals carry the voltage's index in v's layout: VARIABLES' gathered blocks put variable i at
    // i + i / S (so no division runs on the device)
    std::vector<int64_t> cp((size_t)mloc + 1), lits((size_t)L);
    for (int64_t c = 0; c <= mloc; ++c) cp[c] = clause_ptr[c] - clause_ptr[0];
    for (int64_t s = 0; s < L; ++s) {
        const int64_t gi = block > 0 ? var[s] + var[s] / block : var[s];
        lits[s] = (gi << 1) | (neg[s] ? 1 : 0);
    }
    // sliced-ELL incidences: chunks of 64 variables, [chunk][j][64], padded with slot 0 (never read:
    // a lane stops at its own degree)
    const int64_t nchunk = (nv + 63) / 64;
    std::vector<int64_t> deg((size_t)std::max<int64_t>(nv, 1), 0), cstart((size_t)nchunk + 1, 0);
    for (int64_t k = 0; k < nv; ++k) deg[k] = var_ptr[k + 1] - var_ptr[k];
    for (int64_t ch = 0; ch < nchunk; ++ch) {
        int64_t mx = 0;
        for (int64_t k = ch * 64; k < std::min(nv, ch * 64 + 64); ++k) mx = std::max(mx, deg[k]);
        cstart[ch + 1] = cstart[ch] + 64 * mx;
    }
    if (cstart[nchunk] >= INT32_MAX) {
        odesat_part_destroy(p);
        return fail(ODESAT_EINVAL, "too many incidences");
    }
    std::vector<int64_t> ell((size_t)std::max<int64_t>(cstart[nchunk], 1), 0);
    for (int64_t k = 0; k < nv; ++k)
        for (int64_t j = 0; j < deg[k]; ++j) ell[cstart[k / 64] + 64 * j + (k % 64)] = inc_slot[var_ptr[k] + j];
    p->voff = block > 0 && v1 - v0 <= block ? v0 / block : 0;
    // term layout: REGION (default), ELL or SLOT (experiment knob PART_TERMS = 0 / 1 / 2)
    {
        const int64_t t = odesat::xp_get("PART_TERMS", 0);
        p->terms = t == 2 ? TERMS_SLOT : (t == 1 ? TERMS_ELL : TERMS_REGION);
    }
    p->regions = 16;
    if (odesat::xp_isset("PART_REGIONS")) p->regions = std::max(8, (int)odesat::xp_get("PART_REGIONS", 16) / 8 * 8);
    const int64_t ell_words = cstart[nchunk];
    // w's size: SLOT L words, ELL the padded sliced-ELL, REGION the in-range incidences; + 64 sink words
    const int64_t ninc_all = nv ? var_ptr[nv] : 0;
    const int64_t wdata = p->terms == TERMS_SLOT ? L : (p->terms == TERMS_ELL ? ell_words : ninc_all);
    std::vector<int64_t> tpos;
    if (p->terms != TERMS_SLOT) {  // slot -> term position; slots of variables outside [v0, v1) -> sink words
        tpos.assign((size_t)std::max<int64_t>(L, 1), 0);
        for (int64_t sl = 0; sl < L; ++sl) tpos[sl] = wdata + (sl & 63);
        if (p->terms == TERMS_ELL) {
            for (int64_t k = 0; k < nv; ++k)
                for (int64_t j = 0; j < deg[k]; ++j) tpos[inc_slot[var_ptr[k] + j]] = cstart[k / 64] + 64 * j + (k % 64);
        } else {  // REGION: region r's terms together, in slot order
            const int64_t RG = p->regions;
            std::vector<int64_t> rcount((size_t)RG + 1, 0), slot_region((size_t)std::max<int64_t>(L, 1), -1);
            for (int64_t k = 0; k < nv; ++k) {
                const int64_t r = std::min(RG - 1, k * RG / nv);
                // the range of region r is [r nv / RG, (r+1) nv / RG): k belongs to the r with r0 <= k < r1
                int64_t rr = r;
                while (rr > 0 && k < rr * nv / RG) --rr;
                while (rr + 1 < RG && k >= (rr + 1) * nv / RG) ++rr;
                for (int64_t j = 0; j < deg[k]; ++j) slot_region[inc_slot[var_ptr[k] + j]] = rr;
                rcount[rr + 1] += deg[k];
            }
            for (int64_t r = 0; r < RG; ++r) rcount[r + 1] += rcount[r];
            std::vector<int64_t> fill(rcount.begin(), rcount.end() - 1);
            for (int64_t sl = 0; sl < L; ++sl)
                if (slot_region[sl] >= 0) tpos[sl] = fill[slot_region[sl]]++;
            for (int64_t q = 0; q < (int64_t)ell.size() && ell_words > 0; ++q) ell[q] = 0;
            for (int64_t k = 0; k < nv; ++k)  // the variable kernel gathers its terms at these positions
                for (int64_t j = 0; j < deg[k]; ++j) ell[cstart[k / 64] + 64 * j + (k % 64)] = tpos[inc_slot[var_ptr[k] + j]];
        }
    }
    int rc;
    if ((rc = upload(p, &p->cptr, cp.data(), mloc + 1)) || (rc = upload(p, &p->lits, lits.data(), L)) ||
        (rc = upload(p, &p->cstart, cstart.data(), nchunk + 1)) || (rc = upload(p, &p->deg, deg.data(), nv)) ||
        (p->terms != TERMS_ELL && (rc = upload(p, &p->islot, ell.data(), ell_words))) ||
        (p->terms != TERMS_SLOT && (rc = upload(p, &p->tpos, tpos.data(), L)))) {
        odesat_part_destroy(p);
        return rc;
    }
    bool k3 = mloc > 0 && L == 3 * mloc;
    for (int64_t c = 0; c < mloc && k3; ++c) k3 = cp[c] == 3 * c;
    if (odesat::xp_get("PART_K3", 1) == 0) k3 = false;
    if (odesat::xp_isset("PART_XCD")) p->xcd_ranges = odesat::xp_get("PART_XCD", 0) != 0 ? 8 : 0;
    if (k3) {  // 3-SAT slice: one literal record per clause, term positions in 3 planes
        bool pack = true;
        for (int64_t q = 0; q < L && pack; ++q) pack = lits[q] < (1 << 21);
        if (odesat::xp_get("PART_PACK", 1) == 0) pack = false;
        p->lit_packed = pack;
        const size_t rb = pack ? 8 : 16;
        std::vector<uint64_t> l8(pack ? (size_t)mloc : 0);
        std::vector<int4> l4(pack ? 0 : (size_t)mloc);
        std::vector<int32_t> t3(p->terms != TERMS_SLOT ? 3 * (size_t)mloc : 0);
        for (int64_t c = 0; c < mloc; ++c) {
            if (pack)
                l8[c] = (uint64_t)lits[3 * c] | (uint64_t)lits[3 * c + 1] << 21 | (uint64_t)lits[3 * c + 2] << 42;
            else
                l4[c] = make_int4((int)lits[3 * c], (int)lits[3 * c + 1], (int)lits[3 * c + 2], 0);
            if (!t3.empty())
                for (int j = 0; j < 3; ++j) t3[j * mloc + c] = (int32_t)tpos[3 * c + j];
        }
        const void *src = pack ? (const void *)l8.data() : (const void *)l4.data();
        if (hipMalloc(&p->lit3, (size_t)mloc * rb) != hipSuccess ||
            hipMemcpy(p->lit3, src, (size_t)mloc * rb, hipMemcpyHostToDevice) != hipSuccess ||
            (!t3.empty() && (hipMalloc((void **)&p->tpos3, t3.size() * 4) != hipSuccess ||
                             hipMemcpy(p->tpos3, t3.data(), t3.size() * 4, hipMemcpyHostToDevice) != hipSuccess))) {
            odesat_part_destroy(p);
            return fail(ODESAT_ENOMEM, "hipMalloc failed");
        }
        p->bytes += mloc * (rb + t3.size() / std::max<int64_t>(mloc, 1) * 4);
    }
    for (float **b : {&p->xs, &p->xl}) {
        if (hipMalloc((void **)b, std::max<size_t>(16, (size_t)mloc * 4)) != hipSuccess) {
            odesat_part_destroy(p);
            return fail(ODESAT_ENOMEM, "hipMalloc failed");
        }
        p->bytes += mloc * 4;
    }
    if (hipMalloc((void **)&p->stat, sizeof(PartStat)) != hipSuccess ||
        hipMemset(p->stat, 0, sizeof(PartStat)) != hipSuccess) {
        odesat_part_destroy(p);
        return fail(ODESAT_ENOMEM, "hipMalloc failed");
    }
    {
        const PartStat s0{0, -1, 0, 0};
        if (hipMemcpy(p->stat, &s0, sizeof(s0), hipMemcpyHostToDevice) != hipSuccess) {
            odesat_part_destroy(p);
            return fail(ODESAT_EDEVICE, "hipMemcpy failed");
        }
    }
    const int64_t wwords = wdata + 64;
    if (hipMalloc((void **)&p->w, std::max<size_t>(16, (size_t)wwords * 4)) != hipSuccess) {
        odesat_part_destroy(p);
        return fail(ODESAT_ENOMEM, "hipMalloc failed");
    }
    p->bytes += wwords * 4;
    *out = p;
    return ODESAT_OK;
}

extern "C" int64_t odesat_part_device_bytes(const odesat_part *p) { return p ? p->bytes : -1; }

extern "C" int odesat_part_set_memories(odesat_part *p, const double *xs, const double *xl) {
    if (!p || !xs || !xl) return fail(ODESAT_EINVAL, "null argument");
    PART_TRY(hipSetDevice(p->device));
    std::vector<float> a((size_t)p->mloc), b((size_t)p->mloc);
    for (int64_t c = 0; c < p->mloc; ++c) {
        a[c] = (float)xs[c];
        b[c] = (float)xl[c];
    }
    if (p->mloc) {
        PART_TRY(hipMemcpy(p->xs, a.data(), p->mloc * 4, hipMemcpyHostToDevice));
        PART_TRY(hipMemcpy(p->xl, b.data(), p->mloc * 4, hipMemcpyHostToDevice));
    }
    return ODESAT_OK;
}

extern "C" int odesat_part_get_memories(odesat_part *p, double *xs, double *xl) {
    if (!p) return fail(ODESAT_EINVAL, "null part");
    PART_TRY(hipSetDevice(p->device));
    PART_TRY(hipDeviceSynchronize());
    std::vector<float> a((size_t)p->mloc), b((size_t)p->mloc);
    if (p->mloc) {
        PART_TRY(hipMemcpy(a.data(), p->xs, p->mloc * 4, hipMemcpyDeviceToHost));
        PART_TRY(hipMemcpy(b.data(), p->xl, p->mloc * 4, hipMemcpyDeviceToHost));
    }
    for (int64_t c = 0; c < p->mloc; ++c) {
        if (xs) xs[c] = a[c];
        if (xl) xl[c] = b[c];
    }
    return ODESAT_OK;
}

// Where the previous step's unsat count(s) live: VARIABLES world flag slots of the gathered v,
// CLAUSES out[n] (the all-reduced partial vector).
static void flag_src(const odesat_part *p, const float *v, const float *out, int apply, const float **f, int64_t *stride,
                     int *count) {
    if (apply) {
        *f = v + p->S;
        *stride = p->S + 1;
        *count = p->world;
    } else {
        *f = out + p->n;
        *stride = 0;
        *count = 1;
    }
}

extern "C" int odesat_part_rhs(odesat_part *p, const float *v, float *out, double dt, double zeta, int apply, int stop,
                               void *stream) {
    if (!p || !v || !out) return fail(ODESAT_EINVAL, "null argument");
    if (apply < 0 || apply > 2) return fail(ODESAT_EINVAL, "apply must be 0 (CLAUSES), 1 (VARIABLES) or 2 (CLAUSES_RS)");
    if (apply != 0 && p->S == 0) return fail(ODESAT_EINVAL, "VARIABLES / CLAUSES_RS need a block size");
    if (apply == 2 && (p->v0 != 0 || p->v1 != p->n)) return fail(ODESAT_EINVAL, "CLAUSES_RS folds every variable");
    // VARIABLES writes out[0 .. v1 - v0) and its flag at out[S]: the slice must fit its send block
    if (apply == 1 && p->v1 - p->v0 > p->S) return fail(ODESAT_EINVAL, "VARIABLES slice wider than its block");
    PART_TRY(hipSetDevice(p->device));
    hipStream_t st = (hipStream_t)stream;
    const float *f;
    int64_t stride;
    int count;
    flag_src(p, v, out, apply, &f, &stride, &count);
    hipLaunchKernelGGL(k_part_status, dim3(1), dim3(64), 0, st, p->stat, f, stride, count, stop ? 1 : 0, 1);
    PART_TRY(hipGetLastError());
    // this step's unsat count goes after the written block: out[S] (send block) or out[n]
    float *unsat = apply ? out + p->S : out + p->n;
    PART_TRY(hipMemsetAsync(unsat, 0, 4, st));
    const float xl_max = 1e4f * (float)p->m;  // system.rs:95, as the oracle's (T)1e4 * (T)m
    if (p->mloc && p->lit3) {
        const unsigned nb = p->xcd_ranges ? 8u * blocks_for((p->mloc + 7) / 8) : blocks_for(p->mloc);
#define PART_C3(E, X, P)                                                                                      \
    hipLaunchKernelGGL((k_part_clause3<E, X, P>), dim3(nb), dim3(256), 0, st, p->lit3, p->tpos3, v, p->xs, p->xl, \
                       p->w, (int32_t)p->mloc, (float)dt, (float)zeta, xl_max, unsat, p->stat)
#define PART_C3P(E, X)                  \
    if (p->lit_packed) PART_C3(E, X, true); \
    else PART_C3(E, X, false)
        const bool scat = p->terms != TERMS_SLOT;
        if (scat && p->xcd_ranges) { PART_C3P(true, 8); }
        else if (scat) { PART_C3P(true, 1); }
        else if (p->xcd_ranges) { PART_C3P(false, 8); }
        else { PART_C3P(false, 1); }
#undef PART_C3P
#undef PART_C3
    } else if (p->mloc) {
        if (p->terms != TERMS_SLOT)
            hipLaunchKernelGGL(k_part_clause<true>, dim3(blocks_for(p->mloc)), dim3(256), 0, st, p->cptr, p->lits,
                               p->tpos, v, p->xs, p->xl, p->w, (int32_t)p->mloc, (float)dt, (float)zeta, xl_max, unsat,
                               p->stat);
        else
            hipLaunchKernelGGL(k_part_clause<false>, dim3(blocks_for(p->mloc)), dim3(256), 0, st, p->cptr, p->lits,
                               p->tpos, v, p->xs, p->xl, p->w, (int32_t)p->mloc, (float)dt, (float)zeta, xl_max, unsat,
                               p->stat);
    }
    PART_TRY(hipGetLastError());
    if (p->v1 > p->v0) {
        const int64_t nv = p->v1 - p->v0;
        const int32_t bpr = (int32_t)((nv / p->regions + 1 + 255) / 256);
        if (p->terms == TERMS_ELL)
            hipLaunchKernelGGL((k_part_var<true, false>), dim3(blocks_for(nv)), dim3(256), 0, st, p->cstart, p->deg,
                               p->islot, p->w, v, (int32_t)p->voff, (int32_t)p->v0, (int32_t)p->v1, (float)dt, apply,
                               out, p->stat, 0, 0, (int32_t)p->S, p->world);
        else if (p->terms == TERMS_REGION)
            hipLaunchKernelGGL((k_part_var<false, true>), dim3((unsigned)(p->regions * bpr)), dim3(256), 0, st,
                               p->cstart, p->deg, p->islot, p->w, v, (int32_t)p->voff, (int32_t)p->v0, (int32_t)p->v1,
                               (float)dt, apply, out, p->stat, (int32_t)p->regions, bpr, (int32_t)p->S, p->world);
        else
            hipLaunchKernelGGL((k_part_var<false, false>), dim3(blocks_for(nv)), dim3(256), 0, st, p->cstart, p->deg,
                               p->islot, p->w, v, (int32_t)p->voff, (int32_t)p->v0, (int32_t)p->v1, (float)dt, apply,
                               out, p->stat, 0, 0, (int32_t)p->S, p->world);
    }
    PART_TRY(hipGetLastError());
    return ODESAT_OK;
}

extern "C" int odesat_part_apply(odesat_part *p, float *v, const float *dvsum, double dt, void *stream) {
    if (!p || !v || !dvsum) return fail(ODESAT_EINVAL, "null argument");
    PART_TRY(hipSetDevice(p->device));
    hipLaunchKernelGGL(k_part_apply, dim3(blocks_for(p->n)), dim3(256), 0, (hipStream_t)stream, v, dvsum,
                       (int32_t)p->n, (float)dt, p->stat);
    PART_TRY(hipGetLastError());
    return ODESAT_OK;
}

extern "C" int odesat_part_reduce_apply(odesat_part *p, const float *v, const float *block, float *send, int rank,
                                        double dt, void *stream) {
    if (!p || !v || !block || !send) return fail(ODESAT_EINVAL, "null argument");
    if (p->S == 0 || p->v0 != 0 || p->v1 != p->n) return fail(ODESAT_EINVAL, "not a CLAUSES_RS slice");
    if (rank < 0 || rank >= p->world) return fail(ODESAT_EINVAL, "rank out of range");
    PART_TRY(hipSetDevice(p->device));
    const int64_t cnt = std::max<int64_t>(0, std::min<int64_t>(p->S, p->n - (int64_t)rank * p->S));
    hipLaunchKernelGGL(k_part_reduce_apply, dim3(blocks_for(std::max<int64_t>(cnt, 1))), dim3(256), 0,
                       (hipStream_t)stream, v, block, send, (int32_t)p->S, rank, (int32_t)cnt, (float)dt, p->stat);
    PART_TRY(hipGetLastError());
    return ODESAT_OK;
}

extern "C" int odesat_part_reset(odesat_part *p, void *stream) {
    if (!p) return fail(ODESAT_EINVAL, "null part");
    PART_TRY(hipSetDevice(p->device));
    const PartStat s0{0, -1, 0, 0};
    PART_TRY(hipMemcpyAsync(p->stat, &s0, sizeof(s0), hipMemcpyHostToDevice, (hipStream_t)stream));
    PART_TRY(hipStreamSynchronize((hipStream_t)stream));
    return ODESAT_OK;
}

extern "C" int odesat_part_status(odesat_part *p, const float *v, const float *out, int apply, int stop, void *stream,
                                  int64_t *steps_done, int64_t *sat_step, int32_t *frozen) {
    if (!p || !v || !out) return fail(ODESAT_EINVAL, "null argument");
    PART_TRY(hipSetDevice(p->device));
    hipStream_t st = (hipStream_t)stream;
    const float *f;
    int64_t stride;
    int count;
    flag_src(p, v, out, apply, &f, &stride, &count);
    hipLaunchKernelGGL(k_part_status, dim3(1), dim3(64), 0, st, p->stat, f, stride, count, stop ? 1 : 0, 0);
    PART_TRY(hipGetLastError());
    PartStat h;
    PART_TRY(hipMemcpyAsync(&h, p->stat, sizeof(h), hipMemcpyDeviceToHost, st));
    PART_TRY(hipStreamSynchronize(st));
    if (steps_done) *steps_done = h.steps_done;
    if (sat_step) *sat_step = h.sat_step;
    if (frozen) *frozen = h.frozen;
    return ODESAT_OK;
}
