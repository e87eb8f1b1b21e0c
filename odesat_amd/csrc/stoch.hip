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

}  // namespace

extern "C" void odesat_stoch_destroy(odesat_stoch *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    void *ptrs[] = {s->cptr, s->lits, s->vptr, s->vinc, s->v, s->sat, s->xl, s->unsat, s->act, s->steps,
                    s->sat_step, s->done};
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
    if ((rc = stoch_reset(s, 0, batch))) return bail(rc);
    *out = s;
    return ODESAT_OK;
}

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
    const size_t tc = (size_t)s->m * B, tv = (size_t)s->n * B;
    std::vector<uint8_t> act(B);
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
