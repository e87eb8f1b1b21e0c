// stoch.hip -- the reference's discrete stochastic search (stoch.rs:20-110, the `stoch` command,
// main.rs:206-251) for B independent replicas on one GPU.
//
// One step of one replica (stoch.rs:28-81):
//   every clause c, in order: sat = some literal is true; xl[c] = sat ? max(xl - 1, 1) : xl + 20
//   (u64, saturating); each literal's variable gets tot += xl[c] and, if c is unsat, uns += xl[c];
//   then every variable draws r uniform in [1, tot] and flips when r <= uns.  The step returns
//   "every clause was satisfied" (before the flips, which are then no-ops: uns = 0).
// search (stoch.rs:83-110) starts from v = false, xl = 1 and steps until a step returns true.
//
// Layout (replica fastest, as the FUSED integrator): v[n][B] bytes, xl[m][B] u64, sat[m][B] bytes.
// Per step three kernels: k_stoch_clause (thread per clause x replica: evaluate, update xl, record
// sat), k_stoch_var (thread per variable x replica: sum its incidences' xl -- integer sums, so
// the order does not matter -- then draw and flip), k_stoch_status (bookkeeping, stop policy).
// Declared deviation: the reference draws from thread_rng (OS-seeded, not reproducible); here the
// draw is a counter RNG keyed on (seed, replica, step, variable), r = 1 + mulhi64(h, tot), and the
// oracle (oracle/odesat_oracle.c, oc_stoch_*) uses the same function, so results are bit-exact.
// A variable in no clause makes the reference panic (gen_range(1..=0), stoch.rs:70):
// odesat_stoch_create refuses such a formula with ODESAT_EINVAL.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstdint>
#include <new>
#include <string>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"

using odesat::fail;

#define STOCH_TRY(expr)                                                                       \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(ODESAT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

struct odesat_stoch {
    int device = 0;
    int64_t n = 0, m = 0, L = 0, B = 0;
    hipStream_t stream = nullptr;
    int32_t *cptr = nullptr, *lits = nullptr;  // clause-major literals (var << 1 | neg)
    int32_t *vptr = nullptr, *vinc = nullptr;  // variable-major incidences -> clause
    uint8_t *v = nullptr, *sat = nullptr;      // [n][B], [m][B]
    uint64_t *xl = nullptr;                    // [m][B]
    uint32_t *unsat = nullptr;                 // [B] this step had an unsat clause
    uint8_t *act = nullptr;                    // [B] still searching
    int64_t *steps = nullptr;                  // [B] steps taken since the state was set (RNG step index)
    int64_t *sat_step = nullptr, *done = nullptr;  // [B] per call
    int32_t *topo = nullptr;                   // cptr | lits | vptr | vinc, one block for the wave kernel
    int wpw = 0;                               // wave kernel: replicas (waves) per workgroup; 0 = 3-kernel path
    bool k3 = false;                           // wave kernel: every clause has three literals
    size_t topo_bytes = 0, rep_bytes = 0;      // wave kernel LDS: shared topology, per-replica state
};

namespace {

// splitmix64 finaliser, the counter RNG of the integrator (kernels.hpp mix64) and the oracle
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t stoch_hash(uint64_t seed, uint64_t replica, uint64_t step,
                                                        uint64_t var) {
    uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ULL);
    h = mix64(h ^ (replica * 0xD1B54A32D192ED03ULL + 0x632BE59BD9B4E019ULL));
    h = mix64(h ^ (step * 0xA24BAED4963EE407ULL + 0x9FB21C651E98DF25ULL));
    h = mix64(h ^ (var * 0x8CB92BA72F3D8DD7ULL + 0x9E3779B97F4A7C15ULL));
    return h;
}

__global__ void k_stoch_clause(const int32_t *__restrict__ cptr, const int32_t *__restrict__ lits,
                               const uint8_t *__restrict__ v, uint64_t *__restrict__ xl, uint8_t *__restrict__ sat,
                               uint32_t *__restrict__ unsat, const uint8_t *__restrict__ act, int64_t m, int64_t B) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)m * (size_t)B) return;
    const int64_t r = (int64_t)(tid % (size_t)B), c = (int64_t)(tid / (size_t)B);
    if (!act[r]) return;
    bool s = false;  // stoch.rs:20-25 evaluate_clause
    for (int32_t k = cptr[c]; k < cptr[c + 1]; ++k) {
        const int32_t l = lits[k];
        s = s || ((v[(size_t)(l >> 1) * B + r] != 0) != ((l & 1) != 0));
    }
    uint64_t x = xl[tid];
    x = s ? (x > 1 ? x - 1 : 1) : (x > UINT64_MAX - 20 ? UINT64_MAX : x + 20);  // :47-51
    xl[tid] = x;
    sat[tid] = s ? 1 : 0;
    if (!s) unsat[r] = 1u;
}

__global__ void k_stoch_var(const int32_t *__restrict__ vptr, const int32_t *__restrict__ vinc,
                            const uint64_t *__restrict__ xl, const uint8_t *__restrict__ sat, uint8_t *__restrict__ v,
                            const uint8_t *__restrict__ act, const int64_t *__restrict__ steps, int64_t n, int64_t B,
                            uint64_t seed, int64_t replica0) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)n * (size_t)B) return;
    const int64_t r = (int64_t)(tid % (size_t)B), i = (int64_t)(tid / (size_t)B);
    if (!act[r]) return;
    uint64_t tot = 0, uns = 0;  // :54-59 (u64 sums; wrap-around as a release build)
    for (int32_t k = vptr[i]; k < vptr[i + 1]; ++k) {
        const size_t e = (size_t)vinc[k] * B + r;
        const uint64_t x = xl[e];
        tot += x;
        if (!sat[e]) uns += x;
    }
    const uint64_t h = stoch_hash(seed, (uint64_t)(replica0 + r), (uint64_t)steps[r], (uint64_t)i);
    const uint64_t draw = 1 + __umul64hi(h, tot);  // gen_range(1..=tot) (:70)
    if (draw <= uns) v[tid] ^= 1;                  // :72-74
}

__global__ void k_stoch_status(uint32_t *unsat, uint8_t *act, int64_t *steps, int64_t *sat_step, int64_t *done,
                               int64_t B, int stop) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= B || !act[r]) return;
    const bool all = unsat[r] == 0;
    unsat[r] = 0;
    if (all && sat_step[r] < 0) sat_step[r] = done[r];
    done[r] += 1;
    steps[r] += 1;
    if (all && stop == ODESAT_STOP_EACH) act[r] = 0;  // search breaks (:96-99)
}

// ---- one wave per replica (small formulas): the whole search step in LDS -----------------------
// The workgroup copies the topology (clause starts, literals, variable starts, incidences) into
// LDS once; each of its WPW waves then owns one replica for `nsteps` steps with v, xl and the
// clause flags in LDS.  Phase 1: lane l evaluates clauses l, l+64, ... and updates their memories;
// phase 2 (skipped when every clause is satisfied: no variable can flip then) lane l sums variable
// i's incidences (i = l, l+64, ...), draws and flips.  A wave's LDS operations complete in issue
// order, so the phases need no barrier, only a compiler fence.  The first three stages of the
// counter hash depend only on (seed, replica, step) and are hoisted out of the variable loop; the
// value is the same as stoch_hash's.
struct SArgs {
    const int32_t *topo;
    uint8_t *v;
    uint64_t *xl;
    uint8_t *act;
    int64_t *steps, *sat_step, *done;
    int32_t n, m, L;
    int64_t B;
    uint32_t topo_bytes, rep_bytes;
    int64_t nsteps;
    int stop;
    uint64_t seed;
    int64_t replica0;
};

__device__ __forceinline__ void stoch_wave_sync() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// A step is a chain of dependent LDS round trips (literal -> value, incidence -> memory) with one
// wave per SIMD at B = 1024, so latency, not issue, bounds it: the loops are written to put several
// independent reads in flight at once.  K3 (every clause has three literals, as in the
// configurations) keeps one 16-byte literal record per clause and evaluates four clauses per lane
// iteration; the general form walks clause_ptr.
template <bool K3>
__device__ __forceinline__ bool stoch_clauses(const int32_t *cptr, const int4 *cl4, const int32_t *lits,
                                              const uint8_t *v, uint64_t *xl, uint8_t *sat, uint8_t *flag,
                                              int32_t m, int lane) {
    bool u = false;
    if constexpr (K3) {
        for (int32_t base = 0; base < m; base += 256) {
            int4 l[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t c = base + 64 * j + lane;
                ok[j] = c < m;
                l[j] = cl4[ok[j] ? c : 0];
            }
            uint8_t x0[4], x1[4], x2[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x0[j] = v[l[j].x >> 1];
                x1[j] = v[l[j].y >> 1];
                x2[j] = v[l[j].z >> 1];
            }
            uint64_t x[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = xl[ok[j] ? base + 64 * j + lane : 0];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!ok[j]) continue;
                const bool sj = ((x0[j] != 0) != ((l[j].x & 1) != 0)) || ((x1[j] != 0) != ((l[j].y & 1) != 0)) ||
                                ((x2[j] != 0) != ((l[j].z & 1) != 0));
                uint64_t y = x[j];  // stoch.rs:47-51
                y = sj ? (y > 1 ? y - 1 : 1) : (y > UINT64_MAX - 20 ? UINT64_MAX : y + 20);
                const int32_t c = base + 64 * j + lane;
                xl[c] = y;
                sat[c] = sj ? 1 : 0;
                if (!sj) {  // its variables may flip
                    flag[l[j].x >> 1] = 1;
                    flag[l[j].y >> 1] = 1;
                    flag[l[j].z >> 1] = 1;
                }
                u = u || !sj;
            }
        }
    } else {
        for (int32_t c = lane; c < m; c += 64) {  // stoch.rs:43-52
            bool sj = false;
            for (int32_t q = cptr[c]; q < cptr[c + 1]; ++q) {
                const int32_t l = lits[q];
                sj = sj || ((v[l >> 1] != 0) != ((l & 1) != 0));
            }
            uint64_t y = xl[c];
            y = sj ? (y > 1 ? y - 1 : 1) : (y > UINT64_MAX - 20 ? UINT64_MAX : y + 20);
            xl[c] = y;
            sat[c] = sj ? 1 : 0;
            if (!sj)
                for (int32_t q = cptr[c]; q < cptr[c + 1]; ++q) flag[lits[q] >> 1] = 1;
            u = u || !sj;
        }
    }
    return u;
}

// variable i's sums over its incidences (stoch.rs:54-59), reads issued four at a time; integer
// sums, so the order is free
__device__ __forceinline__ void stoch_sums(const int32_t *vinc, int32_t q, int32_t e, const uint64_t *xl,
                                           const uint8_t *sat, uint64_t &tot, uint64_t &uns) {
    tot = 0;
    uns = 0;
    for (; q + 4 <= e; q += 4) {
        int32_t c[4];
        uint64_t x[4];
        uint8_t f[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = vinc[q + j];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x[j] = xl[c[j]];
            f[j] = sat[c[j]];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            tot += x[j];
            if (!f[j]) uns += x[j];
        }
    }
    for (; q < e; ++q) {
        const int32_t c = vinc[q];
        const uint64_t x = xl[c];
        tot += x;
        if (!sat[c]) uns += x;
    }
}

template <int WPW, bool K3> __global__ __launch_bounds__(64 * WPW) void k_stoch_wave(SArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.topo);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        for (uint32_t w = threadIdx.x; w < a.topo_bytes / 16; w += 64 * WPW) dst[w] = src[w];
    }
    __syncthreads();
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const int64_t r = (int64_t)blockIdx.x * WPW + wv;
    if (r >= a.B || !a.act[r]) return;
    const int32_t n = a.n, m = a.m, L = a.L;
    // topology: K3: cl4[m] | vptr[n+1] | vinc[L]; general: cptr[m+1] | lits[L] | vptr[n+1] | vinc[L]
    const int4 *cl4 = reinterpret_cast<const int4 *>(smem);
    const int32_t *cptr = reinterpret_cast<const int32_t *>(smem);
    const int32_t *lits = cptr + m + 1;
    const int32_t *vptr = K3 ? reinterpret_cast<const int32_t *>(cl4 + m) : lits + L;
    const int32_t *vinc = vptr + n + 1;
    uint8_t *rep = smem + a.topo_bytes + (size_t)wv * a.rep_bytes;
    uint64_t *xl = reinterpret_cast<uint64_t *>(rep);
    uint8_t *sat = rep + (size_t)8 * m, *v = sat + m, *flag = v + n;
    int32_t *list = reinterpret_cast<int32_t *>(rep + (((size_t)9 * m + 2 * n + 3) & ~(size_t)3));
    const int64_t B = a.B;
    for (int32_t i = lane; i < n; i += 64) {
        v[i] = a.v[(size_t)i * B + r];
        flag[i] = 0;
    }
    for (int32_t c = lane; c < m; c += 64) xl[c] = a.xl[(size_t)c * B + r];
    stoch_wave_sync();
    int64_t st = a.steps[r], ss = a.sat_step[r], dn = a.done[r];
    bool active = true;
    const uint64_t h1 = mix64(mix64(a.seed + 0x9E3779B97F4A7C15ULL) ^
                              ((uint64_t)(a.replica0 + r) * 0xD1B54A32D192ED03ULL + 0x632BE59BD9B4E019ULL));
    for (int64_t k = 0; k < a.nsteps; ++k) {
        const bool u = stoch_clauses<K3>(cptr, cl4, lits, v, xl, sat, flag, m, lane);
        stoch_wave_sync();
        const bool unsat = __ballot(u) != 0;
        if (unsat) {  // :54-75
            const uint64_t h3 = mix64(h1 ^ ((uint64_t)st * 0xA24BAED4963EE407ULL + 0x9FB21C651E98DF25ULL));
            // Only a variable of an unsat clause has uns > 0, and the draw is >= 1, so no other
            // variable can flip (its draw is a pure function of the counter, so skipping it
            // changes nothing): compact the flagged variables, then sum, draw and flip those.
            int32_t cnt = 0;
            for (int32_t base = 0; base < n; base += 64) {
                const int32_t i = base + lane;
                const bool f = i < n && flag[i];
                const uint64_t mask = __ballot(f);
                if (f) {
                    list[cnt + __popcll(mask & ((1ull << lane) - 1))] = i;
                    flag[i] = 0;
                }
                cnt += __popcll(mask);
            }
            stoch_wave_sync();
            for (int32_t j = lane; j < cnt; j += 64) {
                const int32_t i = list[j];
                uint64_t tot, uns;
                stoch_sums(vinc, vptr[i], vptr[i + 1], xl, sat, tot, uns);
                const uint64_t h = mix64(h3 ^ ((uint64_t)i * 0x8CB92BA72F3D8DD7ULL + 0x9E3779B97F4A7C15ULL));
                if (1 + __umul64hi(h, tot) <= uns) v[i] ^= 1;
            }
            stoch_wave_sync();
        } else if (ss < 0) {
            ss = dn;
        }
        dn += 1;
        st += 1;
        if (!unsat && a.stop == ODESAT_STOP_EACH) {  // :96-99
            active = false;
            break;
        }
    }
    for (int32_t i = lane; i < n; i += 64) a.v[(size_t)i * B + r] = v[i];
    for (int32_t c = lane; c < m; c += 64) a.xl[(size_t)c * B + r] = xl[c];
    if (lane == 0) {
        a.steps[r] = st;
        a.sat_step[r] = ss;
        a.done[r] = dn;
        if (!active) a.act[r] = 0;
    }
}

__global__ void k_stoch_reset(uint8_t *v, uint64_t *xl, int64_t n, int64_t m, int64_t B, int64_t r0, int64_t count) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nv = (size_t)n * count, total = nv + (size_t)m * count;
    if (tid >= total) return;
    if (tid < nv) {
        v[(tid / count) * B + r0 + tid % count] = 0;  // :89 all false
    } else {
        const size_t t = tid - nv;
        xl[(t / count) * B + r0 + t % count] = 1;  // :90 all ones
    }
}

template <typename T> int dalloc(T **p, size_t count) {
    return hipMalloc((void **)p, std::max<size_t>(16, count * sizeof(T))) == hipSuccess
               ? ODESAT_OK
               : fail(ODESAT_ENOMEM, "odesat_stoch: hipMalloc failed");
}

int stoch_check(odesat_stoch *s) {
    if (!s) return fail(ODESAT_EINVAL, "null stoch search");
    STOCH_TRY(hipSetDevice(s->device));
    return ODESAT_OK;
}

int stoch_reset(odesat_stoch *s, int64_t r0, int64_t count) {
    if (count <= 0) return ODESAT_OK;
    const size_t total = (size_t)(s->n + s->m) * count;
    hipLaunchKernelGGL(k_stoch_reset, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s->stream, s->v, s->xl,
                       s->n, s->m, s->B, r0, count);
    STOCH_TRY(hipGetLastError());
    STOCH_TRY(hipMemsetAsync(s->steps + r0, 0, count * 8, s->stream));
    STOCH_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}


constexpr size_t STOCH_LDS_MAX = 160 * 1024 - 1024;

size_t round16(size_t x) { return (x + 15) & ~(size_t)15; }

// The wave kernel's width: the widest WPW in {8, 4, 2, 1} whose LDS fits and that still gives
// every CU of the device (`cus`) a workgroup; 0 (3-kernel path) when one replica's state and the
// topology do not fit.  The experiment knob STOCH_WAVE = 0 forces the 3-kernel path, STOCH_WPW = w
// forces a width that fits.
int stoch_wave_width(int64_t B, size_t topo, size_t rep, int cus) {
    if (odesat::xp_get("STOCH_WAVE", 1) == 0) return 0;
    auto fits = [&](int w) { return topo + (size_t)w * rep <= STOCH_LDS_MAX; };
    if (!fits(1)) return 0;
    {
        const int64_t w = odesat::xp_get("STOCH_WPW", -1);
        if ((w == 1 || w == 2 || w == 4 || w == 8) && fits((int)w)) return (int)w;
    }
    for (int w : {8, 4, 2}) {
        if (fits(w) && (B + w - 1) / w >= cus) return w;
    }
    return 1;
}

template <int WPW, bool K3> int launch_stoch_wave(odesat_stoch *s, const SArgs &a) {
    const size_t lds = s->topo_bytes + (size_t)WPW * s->rep_bytes;
    STOCH_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_stoch_wave<WPW, K3>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_stoch_wave<WPW, K3>), dim3((unsigned)((s->B + WPW - 1) / WPW)), dim3(64 * WPW), lds, s->stream,
                       a);
    STOCH_TRY(hipGetLastError());
    return ODESAT_OK;
}

template <bool K3> int stoch_wave_launch_k(odesat_stoch *s, const SArgs &a) {
    switch (s->wpw) {
    case 8: return launch_stoch_wave<8, K3>(s, a);
    case 4: return launch_stoch_wave<4, K3>(s, a);
    case 2: return launch_stoch_wave<2, K3>(s, a);
    default: return launch_stoch_wave<1, K3>(s, a);
    }
}

int stoch_wave_launch(odesat_stoch *s, const SArgs &a) {
    return s->k3 ? stoch_wave_launch_k<true>(s, a) : stoch_wave_launch_k<false>(s, a);
}

}  // namespace

extern "C" void odesat_stoch_destroy(odesat_stoch *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    void *ptrs[] = {s->cptr, s->lits, s->vptr, s->vinc, s->v, s->sat, s->xl, s->unsat, s->act, s->steps,
                    s->sat_step, s->done, s->topo};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

extern "C" int odesat_stoch_create(int device, const odesat_cnf *f, int64_t batch, odesat_stoch **out) {
    if (!f || !out) return fail(ODESAT_EINVAL, "odesat_stoch_create: null argument");
    *out = nullptr;
    if (batch <= 0) return fail(ODESAT_EINVAL, "batch must be > 0");
    const int64_t n = f->varnum, m = f->nclauses(), L = f->nliterals();
    if (n <= 0) return fail(ODESAT_EINVAL, "varnum must be > 0");
    if (L >= INT32_MAX || m >= INT32_MAX || n >= INT32_MAX / 2)
        return fail(ODESAT_EINVAL, "formula too large for 32-bit indices");
    std::vector<int32_t> cptr((size_t)m + 1), lits((size_t)std::max<int64_t>(L, 1)), deg((size_t)n + 1, 0);
    for (int64_t c = 0; c <= m; ++c) cptr[c] = (int32_t)f->clause_ptr[c];
    for (int64_t k = 0; k < L; ++k) {
        const int64_t x = f->var[k];
        if (x < 0 || x >= n) return fail(ODESAT_EINVAL, "variable out of range (normalise the formula first)");
        lits[k] = (int32_t)(x << 1 | (f->neg[k] ? 1 : 0));
        deg[x + 1] += 1;
    }
    for (int64_t i = 0; i < n; ++i)
        if (deg[i + 1] == 0)  // gen_range(1..=0) panics (stoch.rs:70)
            return fail(ODESAT_EINVAL, "variable " + std::to_string(i) + " occurs in no clause (stoch.rs:70 panics)");
    for (int64_t i = 0; i < n; ++i) deg[i + 1] += deg[i];
    std::vector<int32_t> vinc((size_t)std::max<int64_t>(L, 1)), pos(deg.begin(), deg.end() - 1);
    for (int64_t c = 0; c < m; ++c)
        for (int64_t k = cptr[c]; k < cptr[c + 1]; ++k) vinc[pos[f->var[k]]++] = (int32_t)c;

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(ODESAT_EDEVICE, "no HIP device available (odesat_amd has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(ODESAT_EINVAL, "bad device index");
    auto *s = new (std::nothrow) odesat_stoch();
    if (!s) return fail(ODESAT_ENOMEM, "out of memory");
    s->device = device;
    s->n = n;
    s->m = m;
    s->L = L;
    s->B = batch;
    int rc = ODESAT_OK;
    auto bail = [&](int code) {
        odesat_stoch_destroy(s);
        return code;
    };
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "hipStreamCreate failed"));
    const size_t B = (size_t)batch;
    if ((rc = dalloc(&s->cptr, m + 1)) || (rc = dalloc(&s->lits, L)) || (rc = dalloc(&s->vptr, n + 1)) ||
        (rc = dalloc(&s->vinc, L)) || (rc = dalloc(&s->v, n * B)) || (rc = dalloc(&s->sat, m * B)) ||
        (rc = dalloc(&s->xl, m * B)) || (rc = dalloc(&s->unsat, B)) || (rc = dalloc(&s->act, B)) ||
        (rc = dalloc(&s->steps, B)) || (rc = dalloc(&s->sat_step, B)) || (rc = dalloc(&s->done, B)))
        return bail(rc);
    if (hipMemcpy(s->cptr, cptr.data(), (m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (L && hipMemcpy(s->lits, lits.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(s->vptr, deg.data(), (n + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (L && hipMemcpy(s->vinc, vinc.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemset(s->unsat, 0, B * 4) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "hipMemcpy failed"));
    {  // the wave kernel's topology block (K3: cl4[m] | vptr | vinc; else cptr | lits | vptr | vinc)
        std::vector<int32_t> topo;
        topo.reserve((size_t)(m + 1 + 2 * L + n + 1 + 4));
        s->k3 = L == 3 * m;
        for (int64_t c = 0; c < m && s->k3; ++c) s->k3 = cptr[c + 1] - cptr[c] == 3;
        if (s->k3) {  // one 16-byte record per clause: three literals and a pad
            for (int64_t c = 0; c < m; ++c) {
                topo.insert(topo.end(), lits.begin() + 3 * c, lits.begin() + 3 * c + 3);
                topo.push_back(0);
            }
        } else {
            topo.insert(topo.end(), cptr.begin(), cptr.end());
            topo.insert(topo.end(), lits.begin(), lits.begin() + L);
        }
        topo.insert(topo.end(), deg.begin(), deg.end());
        topo.insert(topo.end(), vinc.begin(), vinc.begin() + L);
        s->topo_bytes = round16(topo.size() * 4);
        topo.resize(s->topo_bytes / 4, 0);
        // xl[m] u64 | sat[m] | v[n] | flag[n] | (4-aligned) list[n] int32
        s->rep_bytes = round16((((size_t)9 * m + 2 * n + 3) & ~(size_t)3) + (size_t)4 * n);
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
            cus = 256;
        s->wpw = stoch_wave_width(batch, s->topo_bytes, s->rep_bytes, cus);
        if (s->wpw) {
            if ((rc = dalloc(&s->topo, topo.size()))) return bail(rc);
            if (hipMemcpy(s->topo, topo.data(), s->topo_bytes, hipMemcpyHostToDevice) != hipSuccess)
                return bail(fail(ODESAT_EDEVICE, "hipMemcpy failed"));
        }
    }
    if ((rc = stoch_reset(s, 0, batch))) return bail(rc);
    *out = s;
    return ODESAT_OK;
}

extern "C" int odesat_stoch_wave_width(const odesat_stoch *s) { return s ? s->wpw : 0; }

extern "C" int odesat_stoch_reset(odesat_stoch *s, int64_t r0, int64_t count) {
    int rc;
    if ((rc = stoch_check(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    return stoch_reset(s, r0, count);
}

extern "C" int odesat_stoch_set_state(odesat_stoch *s, int64_t r0, int64_t count, const uint8_t *v, const uint64_t *xl) {
    int rc;
    if ((rc = stoch_check(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    if ((rc = stoch_reset(s, r0, count))) return rc;  // the RNG step index restarts too
    const size_t B = (size_t)s->B;
    std::vector<uint8_t> hv((size_t)s->n * B);
    std::vector<uint64_t> hx((size_t)s->m * B);
    STOCH_TRY(hipMemcpy(hv.data(), s->v, hv.size(), hipMemcpyDeviceToHost));
    STOCH_TRY(hipMemcpy(hx.data(), s->xl, hx.size() * 8, hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < count; ++b) {
        if (v)
            for (int64_t i = 0; i < s->n; ++i) hv[(size_t)i * B + r0 + b] = v[b * s->n + i] ? 1 : 0;
        if (xl)
            for (int64_t c = 0; c < s->m; ++c) hx[(size_t)c * B + r0 + b] = xl[b * s->m + c];
    }
    STOCH_TRY(hipMemcpy(s->v, hv.data(), hv.size(), hipMemcpyHostToDevice));
    STOCH_TRY(hipMemcpy(s->xl, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
    return ODESAT_OK;
}

extern "C" int odesat_stoch_get_state(odesat_stoch *s, int64_t r0, int64_t count, uint8_t *v, uint64_t *xl) {
    int rc;
    if ((rc = stoch_check(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    STOCH_TRY(hipStreamSynchronize(s->stream));
    const size_t B = (size_t)s->B;
    if (v) {
        std::vector<uint8_t> hv((size_t)s->n * B);
        STOCH_TRY(hipMemcpy(hv.data(), s->v, hv.size(), hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < count; ++b)
            for (int64_t i = 0; i < s->n; ++i) v[b * s->n + i] = hv[(size_t)i * B + r0 + b];
    }
    if (xl) {
        std::vector<uint64_t> hx((size_t)s->m * B);
        STOCH_TRY(hipMemcpy(hx.data(), s->xl, hx.size() * 8, hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < count; ++b)
            for (int64_t c = 0; c < s->m; ++c) xl[b * s->m + c] = hx[(size_t)c * B + r0 + b];
    }
    return ODESAT_OK;
}

extern "C" int odesat_stoch_search(odesat_stoch *s, uint64_t seed, int64_t replica0, int64_t max_steps, int stop,
                                   int32_t poll_interval, int64_t *first_sat_step, int64_t *steps_done) {
    int rc;
    if ((rc = stoch_check(s))) return rc;
    if (max_steps <= 0) return fail(ODESAT_EINVAL, "max_steps must be > 0");
    if (stop != ODESAT_STOP_EACH && stop != ODESAT_STOP_NONE)
        return fail(ODESAT_EINVAL, "stop must be ODESAT_STOP_EACH or ODESAT_STOP_NONE");
    const int poll = poll_interval > 0 ? poll_interval : 64;
    const size_t B = (size_t)s->B;
    std::vector<uint8_t> ones(B, 1);
    std::vector<int64_t> neg(B, -1);
    STOCH_TRY(hipMemcpyAsync(s->act, ones.data(), B, hipMemcpyHostToDevice, s->stream));
    STOCH_TRY(hipMemcpyAsync(s->sat_step, neg.data(), B * 8, hipMemcpyHostToDevice, s->stream));
    STOCH_TRY(hipMemsetAsync(s->done, 0, B * 8, s->stream));
    STOCH_TRY(hipMemsetAsync(s->unsat, 0, B * 4, s->stream));
    std::vector<uint8_t> act(B);
    if (s->wpw) {
        SArgs a{s->topo, s->v, s->xl, s->act, s->steps, s->sat_step, s->done, (int32_t)s->n, (int32_t)s->m,
                (int32_t)s->L, s->B, (uint32_t)s->topo_bytes, (uint32_t)s->rep_bytes, 0, stop, seed, replica0};
        // one launch per poll interval (EACH) or per 4096 steps (NONE): bounded launch durations
        const int64_t chunk = stop == ODESAT_STOP_EACH ? poll : 4096;
        for (int64_t k = 0; k < max_steps;) {
            a.nsteps = std::min<int64_t>(chunk, max_steps - k);
            if ((rc = stoch_wave_launch(s, a))) return rc;
            k += a.nsteps;
            if (stop == ODESAT_STOP_EACH && k < max_steps) {
                STOCH_TRY(hipMemcpyAsync(act.data(), s->act, B, hipMemcpyDeviceToHost, s->stream));
                STOCH_TRY(hipStreamSynchronize(s->stream));
                if (std::none_of(act.begin(), act.end(), [](uint8_t x) { return x != 0; })) break;
            }
        }
        max_steps = 0;  // the 3-kernel loop below does not run
    }
    const size_t tc = (size_t)s->m * B, tv = (size_t)s->n * B;
    for (int64_t k = 0; k < max_steps; ++k) {
        if (tc)
            hipLaunchKernelGGL(k_stoch_clause, dim3((unsigned)((tc + 255) / 256)), dim3(256), 0, s->stream, s->cptr,
                               s->lits, s->v, s->xl, s->sat, s->unsat, s->act, s->m, s->B);
        hipLaunchKernelGGL(k_stoch_var, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s->stream, s->vptr, s->vinc,
                           s->xl, s->sat, s->v, s->act, s->steps, s->n, s->B, seed, replica0);
        hipLaunchKernelGGL(k_stoch_status, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s->stream, s->unsat,
                           s->act, s->steps, s->sat_step, s->done, s->B, stop);
        STOCH_TRY(hipGetLastError());
        if (stop == ODESAT_STOP_EACH && (k + 1) % poll == 0 && k + 1 < max_steps) {
            STOCH_TRY(hipMemcpyAsync(act.data(), s->act, B, hipMemcpyDeviceToHost, s->stream));
            STOCH_TRY(hipStreamSynchronize(s->stream));
            if (std::none_of(act.begin(), act.end(), [](uint8_t a) { return a != 0; })) break;
        }
    }
    if (first_sat_step) STOCH_TRY(hipMemcpyAsync(first_sat_step, s->sat_step, B * 8, hipMemcpyDeviceToHost, s->stream));
    if (steps_done) STOCH_TRY(hipMemcpyAsync(steps_done, s->done, B * 8, hipMemcpyDeviceToHost, s->stream));
    STOCH_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}
