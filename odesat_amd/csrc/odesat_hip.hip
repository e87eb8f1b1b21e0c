// odesat_hip.hip -- host side and C ABI of libodesat_hip.so: the MI355X replacement of
// /root/reference/src/system.rs:25-359 (include/odesat.h).  Device code: kernels.hpp.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"
#include "kernels.hpp"
#include "resident.hpp"
#include "wave.hpp"
#include "onchip.hpp"
#include "devattr.hpp"

using odesat::fail;
using namespace odk;

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(ODESAT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

struct odesat_solver {
    int device = 0, dtype = ODESAT_F32;
    int64_t n = 0, m = 0, L = 0, B = 0, Bp = 0;
    int LW = 64, W = 64, G = 1;  // W = LW: one replica per lane
    int chunk_groups = 1;
    int uniform_k = 0;  // every clause has this many literals (0 = mixed widths)
    int schedule = ODESAT_SCHED_AUTO;
    int alg = ODESAT_ALG_FUSED;
    size_t tsize = 4;
    hipStream_t stream = nullptr;
    int32_t *cptr = nullptr, *lits = nullptr, *wpos = nullptr, *vptr = nullptr, *pc = nullptr, *ps = nullptr;
    int32_t *empty = nullptr;  // clauses without literals (FUSED handles them separately)
    Inc *inc = nullptr;        // 3-SAT incidence records, variable-major
    int n_empty = 0;
    void *v[2] = {nullptr, nullptr};   // voltages [G][n][W]
    void *c[2] = {nullptr, nullptr};   // clause memories [G][m][W][2] (xs, xl)
    uint8_t *par = nullptr;  // [G]
    void *w = nullptr;
    void *vh = nullptr, *vf = nullptr, *ch = nullptr, *cf = nullptr;
    void *dtr = nullptr, *err = nullptr;
    // per-call bookkeeping of the persistent kernels (callio.hpp): io_begin -- the next launch starts the
    // call (no k_begin_call); io_mirror -- launches store the results in the pinned host buffers
    bool io_begin = false, io_mirror = false;
    bool check_fault = false;  // this call ran a kernel that may report a fault in stop[1] (k_onchip split barriers)
    uint32_t *unsat = nullptr;
    uint8_t *act = nullptr;
    int64_t *sat_step = nullptr, *steps_done = nullptr;
    int32_t *stop = nullptr;
    // RESIDENT (resident.hpp): group width W == res_R replicas per workgroup; clauses are stored
    // in the internal (tile) order, cmap[original clause] = internal clause
    int res_R = 0;        // 0 = the layout does not admit the resident kernel
    bool res_narrow = false;  // RESIDENT with one wave per workgroup (R = 1, 64-clause tiles)
    bool res_wave = false;    // RESIDENT as k_wave (wave.hpp): small 3-SAT, one wave per replica, variable fold
    int4 *wv_rec4 = nullptr;  // [m] k_wave: literal | variable-major term position << 16, per literal
    int32_t *wv_vst = nullptr;  // [n+1] k_wave: first term position of each variable
    int wv_wpw = 1;             // k_wave: replicas per workgroup sharing the LDS topology
    bool solo = false;          // k_solo (wave.hpp) instead of k_wave: one replica per workgroup, lanes' slots in registers
    int solo_nl = 64, solo_cpl = 1, solo_vpl = 1;  // k_solo: lanes per replica, clause / variable slots per lane
    bool solo_fast = true;      // k_solo's short arithmetic on in-range states (knob SOLO_FAST = 0: the general form)
    bool solo_cv = true;        // k_solo_cv (clause-held voltages) for the short arithmetic when it fits
    bool solo_cv_z0 = false;    // the formula has variables of degree 0 (k_solo_cv's variable slots)
    int4 *cv_rec = nullptr;     // [solo_nl solo_cpl] k_solo_cv's per-slot records (cv_layout.cpp)
    int32_t *cv_blk = nullptr;  // [n + 1] k_solo_cv's term block per variable (n: the zero block)
    int32_t cv_nb = 0;          // blocks in use
    int64_t cv_cost_plain = 0, cv_cost = 0;  // the bank model's LDS cycles per pass, plain / chosen layout
    bool wave_fast = true;      // k_wave's likewise (knob WAVE_FAST = 0)
    bool res_fast = true;       // k_resident's likewise, 3-SAT only (knob RES_FAST = 0)
    bool res_rc = true;         // f64 fixed steps: register-cached tiles (resident.hpp; knob RES_RC = 0)
    int wv_tw = 1;              // k_wave: waves per replica, fixed steps
    int wv_tw_ada = 1;          // ... adaptive steps (four barriers per step instead of two: at most 4)
    int cus = 256;              // the device's CUs (k_wave's device rounds)
    bool wave_tail = true;      // k_wave: a partial last round runs as its own launch, fewer replicas per workgroup
    bool res_ada = false; // adaptive steps run k_resident (else FUSED on the same layout)
    bool res_vfg = false; // ... with the full-step voltage clone in HBM (v and dv fill the LDS)
    int res_ntiles = 0;
    int32_t *res_tc = nullptr, *cmap = nullptr;
    // f64 k_resident on wave-paired tiles (resident.hpp PAIRS): wave w of tile t holds internal clauses
    // [res_tcw[8t+w], res_tcw[8t+w+1]), padded with m; a barrier after tile t iff t + oc_off is odd
    int32_t *res_tcw = nullptr;
    bool res_pairs = false;
    int4 *res_cl4 = nullptr;  // [m] literals of internal clause k (3-SAT)
    // ONCHIP (onchip.hip): same tiles as RESIDENT (R = 1, f32, 3-SAT); tiles [0, oc_tr) keep their
    // memories in VGPRs, [oc_tr, oc_tr + oc_tl) in LDS.  oc_tr == 0: not available
    int oc_tr = 0, oc_tl = 0;
    uint64_t *oc_rec = nullptr;  // [tiles][512] slot-major clause records (onchip::make_rec)
    uint32_t *oc_rec12 = nullptr;  // ONCHIP_REC12: the same in 12 bytes (onchip::make_rec12)
    int32_t *oc_tcp = nullptr;   // [ntp * 8 + 1] wave starts (t * 8 + w) padded with m (static-index loads in k_onchip)
    int64_t oc_rec_bytes = 0;
    bool oc_ada = false;  // ONCHIP also takes adaptive steps (onchip.hpp ADA_*)
    uint32_t oc_poll_limit = 1u << 22;  // split-barrier polls before a wait gives up (knob ONCHIP_POLL_LIMIT)
    int oc_off = 0;  // pair offset of the wave-paired tiles (pair_tiles): barrier after tile t iff t + off is odd
    bool in_range = true;        // every replica's state is in ONCHIP's range (onchip.hip header)
    int64_t bytes = 0;
    // steps run since the last fresh odesat_simulate: odesat_simulate_continue numbers its steps from
    // here and keeps every replica's bookkeeping (sat step, steps done, frozen, adaptive dt)
    int64_t t_base = 0;
    // pinned host staging for polls and results (no pageable copies on the hot path)
    int64_t *h_sat = nullptr, *h_done = nullptr;  // [Bp]
    double *h_dt = nullptr;                       // [Bp] (f32 dt is read into its first half)
    int32_t *h_stop = nullptr;
    uint8_t *h_act = nullptr;                     // [Bp]
    // STOP_ANY replay snapshot of a launch's starting bookkeeping (lazy)
    uint8_t *snap_par = nullptr;
    int64_t *snap_sat = nullptr, *snap_done = nullptr;
    void *snap_dt = nullptr;
    // odesat_checkpoint slot (lazy): the state of every group and the bookkeeping
    void *ck_v = nullptr, *ck_c = nullptr, *ck_dt = nullptr;
    uint8_t *ck_par = nullptr, *ck_act = nullptr;
    int64_t *ck_sat = nullptr, *ck_done = nullptr;
    int32_t *ck_stop = nullptr;
    int64_t ck_t_base = -1;  // -1: no checkpoint taken
    bool ck_in_range = true;
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

// Call f(IC<LW>, IC<1>) with the solver's compile-time layout (one replica per lane: the kernels'
// VEC template parameter, contiguous replicas per lane, is 1 -- round 2 measured 2 and 4 slower).
template <typename T, typename F> int with_layout(const odesat_solver *s, F &&f) {
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
    if ((rc = dmalloc(s, &s->ch, 2 * state_elems(s, s->m) * s->tsize))) return rc;
    if ((rc = dmalloc(s, &s->cf, 2 * state_elems(s, s->m) * s->tsize))) return rc;
    return ODESAT_OK;
}

int ensure_w(odesat_solver *s) {
    if (s->alg != ODESAT_ALG_TWOPASS || s->w) return ODESAT_OK;
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
    a.pc = s->pc;
    a.ps = s->ps;
    a.inc = s->inc;
    a.v0 = (T *)s->v[0];
    a.v1 = (T *)s->v[1];
    a.c0 = (T *)s->c[0];
    a.c1 = (T *)s->c[1];
    a.par = s->par;
    a.w = (T *)s->w;
    a.vh = (T *)s->vh;
    a.vf = (T *)s->vf;
    a.ch = (T *)s->ch;
    a.cf = (T *)s->cf;
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

enum Kern { K_STEP = 0, K_CLAUSE = 1, K_VARIABLE = 2 };

// Grid geometry: rows per wave, waves per group, block placement (XCD-aware when the group count
// and the 8 XCDs divide one another).
template <typename T> unsigned geometry(const odesat_solver *s, KArgs<T> &a, int64_t items, int LW) {
    a.rows = pick_rows(items, a.ng, LW);
    const int64_t ipr = 64 / LW;
    a.tiles = (int)((items + ipr * a.rows - 1) / (ipr * a.rows));
    a.bpg = (a.tiles + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    int64_t blocks;
    if (a.ng >= 8 && a.ng % 8 == 0) {
        a.xmode = 1;
        blocks = (int64_t)a.ng * a.bpg;
    } else if (a.ng < 8 && 8 % a.ng == 0 && a.bpg >= 8 / a.ng) {
        a.xmode = 2;
        const int sh = 8 / a.ng;
        blocks = 8ll * ((a.bpg + sh - 1) / sh);
    } else {
        a.xmode = 0;
        blocks = (int64_t)a.ng * a.bpg;
    }
    (void)s;
    return a.tiles == 0 ? 0u : (unsigned)std::min<int64_t>(blocks, INT_MAX);
}

template <typename T, int LW, int VEC, int MODE>
int launch_kernel(odesat_solver *s, KArgs<T> a, Kern which) {
    const int64_t items = which == K_CLAUSE ? s->m : s->n;
    const unsigned blocks = geometry<T>(s, a, items, LW);
    if (blocks == 0) return ODESAT_OK;
    const dim3 grid(blocks), block(64 * WAVES_PER_BLOCK);
    {
        Timed tm(s, which == K_VARIABLE ? 1 : 0);
        if (which == K_STEP) {
            if (s->uniform_k == 3)
                hipLaunchKernelGGL((k_step<T, LW, VEC, MODE, 3, 4>), grid, block, 0, s->stream, a);
            else
                hipLaunchKernelGGL((k_step<T, LW, VEC, MODE, 0>), grid, block, 0, s->stream, a);
        } else if (which == K_CLAUSE) {
            if (s->uniform_k == 3)
                hipLaunchKernelGGL((k_clause_u<T, LW, VEC, MODE, 3>), grid, block, 0, s->stream, a);
            else
                hipLaunchKernelGGL((k_clause<T, LW, VEC, MODE>), grid, block, 0, s->stream, a);
        } else {
            hipLaunchKernelGGL((k_variable<T, LW, VEC, MODE>), grid, block, 0, s->stream, a);
        }
    }
    HIP_TRY(hipGetLastError());
    if (which == K_STEP && s->n_empty > 0) {  // clauses with no literal (no owning variable)
        const int64_t threads = (int64_t)a.ng * s->n_empty * LW;
        const int64_t nb = (threads + 255) / 256;
        hipLaunchKernelGGL((k_empty_clauses<T, LW, VEC, MODE>), dim3((unsigned)nb), dim3(256), 0, s->stream, a,
                           (const int32_t *)s->empty, s->n_empty);
        HIP_TRY(hipGetLastError());
    }
    return ODESAT_OK;
}

// One RHS(+update) of `MODE` for the groups [gA, gB).
template <typename T, int LW, int VEC, int MODE>
int step_groups(odesat_solver *s, int step, T dt, T zeta, int gA, int gB) {
    KArgs<T> a = make_args<T>(s);
    a.step = step;
    a.dt = dt;
    a.zeta = zeta;
    int rc;
    if (s->alg != ODESAT_ALG_TWOPASS) {  // FUSED (RESIDENT's single steps too)
        a.g0 = gA;
        a.ng = gB - gA;
        return launch_kernel<T, LW, VEC, MODE>(s, a, K_STEP);
    }
    for (int g0 = gA; g0 < gB; g0 += s->chunk_groups) {  // TWOPASS: one contribution buffer per chunk
        a.g0 = g0;
        a.ng = std::min(s->chunk_groups, gB - g0);
        if ((rc = launch_kernel<T, LW, VEC, MODE>(s, a, K_CLAUSE))) return rc;
        if ((rc = launch_kernel<T, LW, VEC, MODE>(s, a, K_VARIABLE))) return rc;
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
    sa.par = s->par;
    sa.r0 = (int32_t)r0;
    sa.r1 = (int32_t)r1;
    sa.W = s->W;
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
        if (!adaptive) return step_groups<T, LW, VEC, M_FIXED>(s, step, (T)dt, (T)zeta, gA, gB);
        const int span = s->alg == ODESAT_ALG_TWOPASS ? s->chunk_groups : gB - gA;
        for (int g0 = gA; g0 < gB; g0 += span) {  // both half steps of one contribution-buffer chunk
            const int g1 = std::min(gB, g0 + span);
            if ((r = step_groups<T, LW, VEC, M_ADA>(s, step, (T)dt, (T)zeta, g0, g1))) return r;
            if ((r = step_groups<T, LW, VEC, M_ADB>(s, step, (T)dt, (T)zeta, g0, g1))) return r;
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

// The CallIO of the next persistent launch: `begin` for the first launch of a folded call only.
CallIO take_io(odesat_solver *s) {
    CallIO io;
    io.B = (int32_t)s->B;
    io.begin = s->io_begin ? 1 : 0;
    s->io_begin = false;
    if (s->io_mirror) {
        io.h_sat = s->h_sat;
        io.h_done = s->h_done;
        io.h_dt = s->h_dt;
    }
    return io;
}

// ---- RESIDENT ---------------------------------------------------------------------------------
constexpr size_t RES_LDS_MAX = 160 * 1024 - 1024;  // dynamic LDS budget (static flags take < 1 KiB)

size_t res_lds_bytes(int64_t n, int R, size_t tsize, bool adaptive) {
    return (adaptive ? 3 : 2) * (size_t)n * R * tsize;  // v, dv (+ the full-step clone of v)
}

bool res_fits(int64_t n, int R, size_t tsize, bool adaptive) {
    return n < (1ll << 24) && res_lds_bytes(n, R, tsize, adaptive) <= RES_LDS_MAX;
}

int res_capacity(int R) {
    switch (R) {
        case 1: return ResShape<1>::NL;
        case 2: return ResShape<2>::NL;
        case 4: return ResShape<4>::NL;
        case 8: return ResShape<8>::NL;
        case 16: return ResShape<16>::NL;
        default: return ResShape<32>::NL;
    }
}

// Var-disjoint clause tiles (resident.hpp): clause c, in the reference's order, goes to the first
// tile after the last tile holding any of its variables that still has room.  Returns the
// internal order perm[k] = original clause and the tile starts, or false when the tiling is
// degenerate (FUSED is then the better kernel).
// the 6 orders of a 3-literal clause: internal slot q holds original literal kP3[code][q]
constexpr int kP3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};

// LDS bank layout of one tile (3-SAT).  A 32-lane half-wave is serviced per LDS cycle and a lane's
// voltage of variable v sits in bank (v*R + r) mod 32, so GS = 32 / R clauses share a half-wave and
// key(v) = v mod GS decides conflicts.  Clauses are dealt to half-wave groups so each group holds
// each key at most ~3 times, then each clause's 3 literals are ordered (min / second-min and the
// G/R terms do not depend on the order of 3 distinct variables) so that each of the 3 gather
// instructions sees distinct keys.  The dv read-modify-write uses the same addresses + a constant.
void bank_layout(const odesat_cnf *f, int R, std::vector<int32_t> &cl, std::vector<uint8_t> &code) {
    const int GS = std::max(1, 32 / R);
    const int64_t s = (int64_t)cl.size();
    if (s == 0) return;
    const int64_t G = (s + GS - 1) / GS;
    std::vector<int> cap((size_t)G, GS), cnt((size_t)G * GS, 0);
    cap[G - 1] = (int)(s - (G - 1) * GS);  // every group but the last is full: groups stay aligned
    std::vector<std::vector<int32_t>> grp((size_t)G);
    auto key = [&](int32_t c, int j) { return (int)(f->var[f->clause_ptr[c] + j] % GS); };
    for (int32_t c : cl) {
        int64_t best = -1;
        long score = LONG_MAX;
        for (int64_t g = 0; g < G; ++g) {
            if ((int)grp[g].size() >= cap[g]) continue;
            int mx = 0, sum = 0;
            for (int j = 0; j < 3; ++j) {
                const int k = cnt[g * GS + key(c, j)];
                mx = std::max(mx, k);
                sum += k;
            }
            const long sc = (long)mx * 1000000 + (long)sum * 1000 + (long)grp[g].size();
            if (sc < score) { score = sc; best = g; }
        }
        grp[best].push_back(c);
        for (int j = 0; j < 3; ++j) cnt[best * GS + key(c, j)] += 1;
    }
    cl.clear();
    std::vector<int> ic(3 * (size_t)GS);
    for (int64_t g = 0; g < G; ++g) {
        std::fill(ic.begin(), ic.end(), 0);
        std::vector<int> pc(grp[g].size(), 0);
        auto distinct = [&](int32_t c) {
            const int64_t b = f->clause_ptr[c];
            return f->var[b] != f->var[b + 1] && f->var[b] != f->var[b + 2] && f->var[b + 1] != f->var[b + 2];
        };
        auto place = [&](size_t i, int sign) {
            for (int q = 0; q < 3; ++q) ic[q * GS + key(grp[g][i], kP3[pc[i]][q])] += sign;
        };
        for (int pass = 0; pass < 3; ++pass) {
            for (size_t i = 0; i < grp[g].size(); ++i) {
                if (pass > 0) place(i, -1);
                int bestp = 0;
                long bs = LONG_MAX;
                for (int pp = 0; pp < (distinct(grp[g][i]) ? 6 : 1); ++pp) {
                    int mx = 0, sum = 0;
                    for (int q = 0; q < 3; ++q) {
                        const int k = ic[q * GS + key(grp[g][i], kP3[pp][q])];
                        mx = std::max(mx, k);
                        sum += k;
                    }
                    const long sc = (long)mx * 1000 + sum;
                    if (sc < bs) { bs = sc; bestp = pp; }
                }
                pc[i] = bestp;
                place(i, +1);
            }
        }
        for (size_t i = 0; i < grp[g].size(); ++i) {
            cl.push_back(grp[g][i]);
            code[grp[g][i]] = (uint8_t)pc[i];
        }
    }
}

// Tile depth of the var-disjoint tiling (build_tiles' greedy, capacity cap) -- its number of tiles.
int64_t tile_count(const odesat_cnf *f, int64_t n, int cap) {
    const int64_t m = f->nclauses();
    std::vector<int32_t> last((size_t)n, -1), fill;
    int32_t first_open = 0;
    for (int64_t c = 0; c < m; ++c) {
        int32_t t = first_open;
        for (int64_t sl = f->clause_ptr[c]; sl < f->clause_ptr[c + 1]; ++sl) t = std::max(t, last[f->var[sl]] + 1);
        while (t < (int32_t)fill.size() && fill[t] >= cap) ++t;
        if (t == (int32_t)fill.size()) fill.push_back(0);
        fill[t] += 1;
        while (first_open < (int32_t)fill.size() && fill[first_open] >= cap) ++first_open;
        for (int64_t sl = f->clause_ptr[c]; sl < f->clause_ptr[c + 1]; ++sl) last[f->var[sl]] = t;
    }
    return (int64_t)fill.size();
}

// RESIDENT replicas per workgroup.  A tile's depth is set by the clause-order chains, not by its
// capacity, so a small instance leaves most of a 512-clause tile empty (config 3, n = 250: ~35
// clauses per tile) and one replica per workgroup wastes the CU.  Then R > 1 replicas share a
// workgroup (tile capacity 1024 / R): the largest R <= 32 that still gives every CU a workgroup and
// whose state (with the adaptive full-step clone) fits in LDS.  Measured on config 3 (adaptive,
// MI355X): B = 1024 R = 1 / 4: 7.2 / 13.9 M replica-steps/s; B = 4096 R = 4 / 16: 14.1 / 48.7 M.
// Instances whose tiles are at least half full keep R = 1 (ONCHIP / RESIDENT at one replica).
int small_instance_width(const odesat_cnf *f, int64_t n, int64_t batch, int device, size_t tsize) {
    const int64_t m = f->nclauses();
    if (m == 0 || odesat::xp_isset("GROUP_WIDTH")) return 1;
    const int64_t nt = tile_count(f, n, ResShape<1>::NL);
    if (2 * m >= nt * (int64_t)ResShape<1>::NL) return 1;
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    int R = 1;
    while (R < 32 && (batch + 2 * R - 1) / (2 * R) >= cus && res_fits(n, 2 * R, tsize, true)) R *= 2;
    return R;
}

// Wave-paired tiles (ONCHIP, onchip.hip: one barrier per PAIR of tiles).  Tiles 2i - off and
// 2i + 1 - off form one barrier interval (off = 0 or 1: with 1, tile 0 is an interval alone), and slots [64w, 64w + 64) of a tile are wave w's.  LDS operations of one
// wave complete in issue order, so a clause may sit in the interval's second tile after a clause
// it shares a variable with in the first tile when both are in the same wave; across waves the
// order still needs the barrier after the pair.  Greedy in the reference's clause order: clause c
// goes to the first tile after the tiles of its variables' last clauses where every one of those
// in the same interval is in one wave w, and w has room (c then takes w); a clause with none there
// takes the least-filled wave.  Each tile stays var-disjoint and every variable's tiles increase in
// clause order, so the tiling is also a RESIDENT tiling.  Config 2: 91 tiles in 46 intervals at
// off = 0, 90 in 46 at off = 1 (plain greedy: 90 tiles, 90 barriers); build_tiles keeps the offset
// with fewer tiles.
constexpr int PAIR_WAVES = 8, PAIR_WAVE_CAP = 64;

void pair_tiles(const odesat_cnf *f, int64_t n, int off, std::vector<int32_t> &tile_of, std::vector<int8_t> &wave_of,
                std::vector<int32_t> &fill) {
    const int64_t m = f->nclauses();
    std::vector<int32_t> lastt((size_t)n, -1);
    std::vector<int8_t> lastw((size_t)n, -1);
    std::vector<std::array<int32_t, PAIR_WAVES>> wf;  // per tile, per wave fill
    tile_of.assign((size_t)m, 0);
    wave_of.assign((size_t)m, 0);
    for (int64_t c = 0; c < m; ++c) {
        const int64_t b = f->clause_ptr[c], e = f->clause_ptr[c + 1];
        int32_t t = 0;
        for (int64_t sl = b; sl < e; ++sl) t = std::max(t, lastt[f->var[sl]] + 1);
        int w = -1;
        for (;;) {
            while ((int32_t)wf.size() <= t) wf.push_back({});
            int want = -1;
            bool split = false;
            for (int64_t sl = b; sl < e; ++sl) {  // last clauses of c's variables in t's interval
                const int32_t lt = lastt[f->var[sl]];
                if (lt >= 0 && (lt + off) / 2 == (t + off) / 2) {
                    const int lw = lastw[f->var[sl]];
                    if (want >= 0 && want != lw) split = true;
                    want = lw;
                }
            }
            if (split) {  // in two waves: only the next interval orders c after both
                t = ((t + off) / 2 + 1) * 2 - off;
                continue;
            }
            if (want >= 0) {
                if (wf[t][want] < PAIR_WAVE_CAP) { w = want; break; }
                ++t;
                continue;
            }
            for (int k = 0; k < PAIR_WAVES; ++k)
                if (wf[t][k] < PAIR_WAVE_CAP && (w < 0 || wf[t][k] < wf[t][w])) w = k;
            if (w >= 0) break;
            ++t;
        }
        wf[t][w] += 1;
        tile_of[c] = t;
        wave_of[c] = (int8_t)w;
        for (int64_t sl = b; sl < e; ++sl) {
            lastt[f->var[sl]] = t;
            lastw[f->var[sl]] = (int8_t)w;
        }
    }
    fill.assign(wf.size(), 0);
    for (size_t t = 0; t < wf.size(); ++t)
        for (int k = 0; k < PAIR_WAVES; ++k) fill[t] += wf[t][k];
    while (!fill.empty() && fill.back() == 0) fill.pop_back();
}

// wst (pairs only): [ntiles * 8 + 1] internal clause of wave w's first slot in tile t at t * 8 + w;
// a tile's clauses are stored wave by wave, so wave w of tile t holds wst[t*8+w+1] - wst[t*8+w].
bool build_tiles(const odesat_cnf *f, int64_t n, int cap, int R, bool k3, bool pairs, std::vector<int32_t> &perm,
                 std::vector<int32_t> &tc, std::vector<uint8_t> &code, std::vector<int32_t> &wst, int &pair_off) {
    const int64_t m = f->nclauses();
    std::vector<int32_t> last((size_t)n, -1), tile_of((size_t)m), fill;
    std::vector<int8_t> wave_of;
    wst.clear();
    pairs = pairs && cap == PAIR_WAVES * PAIR_WAVE_CAP;  // one replica per 512-lane workgroup only
    if (pairs) {
        std::vector<int32_t> t1, f1;
        std::vector<int8_t> w1;
        pair_tiles(f, n, 0, tile_of, wave_of, fill);
        pair_tiles(f, n, 1, t1, w1, f1);
        pair_off = f1.size() < fill.size() ? 1 : 0;
        const int64_t want = odesat::xp_get("PAIR_OFF", -1);  // tests: force the offset
        if (want == 0 || want == 1) pair_off = (int)want;
        if (pair_off) {
            tile_of.swap(t1);
            wave_of.swap(w1);
            fill.swap(f1);
        }
    } else {
        int32_t first_open = 0;  // every tile before it is full
        for (int64_t c = 0; c < m; ++c) {
            int32_t t = 0;
            for (int64_t sl = f->clause_ptr[c]; sl < f->clause_ptr[c + 1]; ++sl) t = std::max(t, last[f->var[sl]] + 1);
            t = std::max(t, first_open);
            while (t < (int32_t)fill.size() && fill[t] >= cap) ++t;
            if (t == (int32_t)fill.size()) fill.push_back(0);
            fill[t] += 1;
            while (first_open < (int32_t)fill.size() && fill[first_open] >= cap) ++first_open;
            tile_of[c] = t;
            for (int64_t sl = f->clause_ptr[c]; sl < f->clause_ptr[c + 1]; ++sl) last[f->var[sl]] = t;
        }
    }
    // a var-disjoint tile holds at most n slots and `cap` clauses: fall back to FUSED only when the
    // tiling is far from that bound (e.g. one variable in every clause)
    const int64_t nt = (int64_t)fill.size(), L = f->nliterals();
    const int64_t bound = std::max<int64_t>((m + cap - 1) / cap, (L + n - 1) / n);
    if (nt > 8 * bound + 16) return false;
    tc.assign((size_t)nt + 1, 0);
    for (int64_t t = 0; t < nt; ++t) tc[t + 1] = tc[t] + fill[t];
    perm.assign((size_t)m, 0);
    code.assign((size_t)m, 0);  // indexed by ORIGINAL clause here; remapped below
    if (pairs) {  // wave by wave inside a tile; the bank layout deals each wave's clauses to its half-waves
        wst.assign((size_t)nt * PAIR_WAVES + 1, 0);
        for (int64_t c = 0; c < m; ++c) wst[(size_t)tile_of[c] * PAIR_WAVES + wave_of[c] + 1] += 1;
        for (size_t i = 1; i < wst.size(); ++i) wst[i] += wst[i - 1];
        std::vector<int32_t> pos(wst.begin(), wst.end() - 1);
        for (int64_t c = 0; c < m; ++c) perm[pos[(size_t)tile_of[c] * PAIR_WAVES + wave_of[c]]++] = (int32_t)c;
        if (k3)
            for (size_t g = 0; g + 1 < wst.size(); ++g) {
                std::vector<int32_t> cl(perm.begin() + wst[g], perm.begin() + wst[g + 1]);
                bank_layout(f, R, cl, code);
                std::copy(cl.begin(), cl.end(), perm.begin() + wst[g]);
            }
    } else {
        std::vector<int32_t> pos(tc.begin(), tc.end() - 1);
        for (int64_t c = 0; c < m; ++c) perm[pos[tile_of[c]]++] = (int32_t)c;  // original order inside a tile
    }
    if (k3 && !pairs) {
        for (int64_t t = 0; t < nt; ++t) {
            std::vector<int32_t> cl(perm.begin() + tc[t], perm.begin() + tc[t + 1]);
            bank_layout(f, R, cl, code);
            std::copy(cl.begin(), cl.end(), perm.begin() + tc[t]);
        }
    }
    std::vector<uint8_t> by_internal((size_t)m);
    for (int64_t k = 0; k < m; ++k) by_internal[k] = code[perm[k]];
    code.swap(by_internal);
    return true;
}

// ONCHIP eligibility and slot-major records (onchip.hpp).  tiles = the padded tile starts, lits =
// the internal-order literals (var << 1 | neg).
int onchip_setup(odesat_solver *s, const std::vector<int32_t> &tiles, const std::vector<int32_t> &wst,
                 const std::vector<int32_t> &lits) {
    if (s->res_R != 1 || s->res_narrow || s->res_wave || s->dtype != ODESAT_F32 || s->uniform_k != 3 || s->n > onchip::MAX_N)
        return ODESAT_OK;
    if (odesat::xp_get("ONCHIP", 1) == 0) return ODESAT_OK;
    const int nt = (int)tiles.size() - 1;
    if (nt == 0 || s->m == 0 || wst.empty()) return ODESAT_OK;  // k_onchip runs wave-paired tiles only
    for (int64_t k = 0; k < s->m; ++k) {  // three distinct variables per clause (independent dv updates)
        const int32_t x = lits[3 * k] >> 1, y = lits[3 * k + 1] >> 1, z = lits[3 * k + 2] >> 1;
        if (x == y || x == z || y == z) return ODESAT_OK;
    }
    const int tl_max = onchip::tl_max(s->n);
    int live = nt;  // tiles up to the last one holding a clause (the tiling is padded to 4 for RESIDENT)
    while (live > 0 && tiles[live] == tiles[live - 1]) --live;
    int tr = 0;
    for (int c : onchip::TR_CHOICES)
        if (c >= live) { tr = c; break; }
    // LDS tiles follow TR_MAX register tiles (their loop continues the 4-deep record ring, so it
    // starts at a multiple of 4; nt is one)
    if (tr == 0 && nt - onchip::TR_MAX <= tl_max) tr = onchip::TR_MAX;
    if (tr == 0) return ODESAT_OK;
    // wave starts (build_tiles): wave w of tile t holds internal clauses [ws[t*8+w], ws[t*8+w+1]),
    // padded with m past the last tile, so the kernel reads a tile's wave bounds at static offsets
    // (a padded tile is empty)
    const int W8 = onchip::WAVES;
    const int ntp = std::max(nt, tr) + 8;
    std::vector<int32_t> ws((size_t)ntp * W8 + 1, (int32_t)s->m);
    std::copy(wst.begin(), wst.end() - 1, ws.begin());
    // slot-major records, padded with empty tiles so every tile a pass touches exists; an empty
    // slot of lane l points all three literals at sink word n + l % 32 (v = 1.0 there)
    std::vector<uint64_t> rec((size_t)ntp * onchip::NTH);
    std::vector<uint32_t> rec12(ONCHIP_REC12 ? rec.size() * 3 : 0);
    for (int t = 0; t < ntp; ++t)
        for (int l = 0; l < onchip::NTH; ++l) {
            const size_t g = (size_t)t * W8 + l / 64;
            const int32_t k = ws[g] + l % 64;
            const size_t i = (size_t)t * onchip::NTH + l;
            uint64_t r;
            if (k < ws[g + 1]) {
                const int32_t *q = &lits[3 * (size_t)k];
                const uint32_t a0 = 4u * (uint32_t)(q[0] >> 1), a1 = 4u * (uint32_t)(q[1] >> 1), a2 = 4u * (uint32_t)(q[2] >> 1);
                r = onchip::make_rec(a0, a1, a2, q[0] & 1, q[1] & 1, q[2] & 1);
                if (ONCHIP_REC12) onchip::make_rec12(a0, a1, a2, q[0] & 1, q[1] & 1, q[2] & 1, &rec12[3 * i]);
            } else {
                const uint32_t sink = 4u * (uint32_t)(s->n + l % onchip::SINKS);
                r = onchip::make_rec(sink, sink, sink, false, false, false) | (uint64_t)onchip::REC_EMPTY << 32;
                if (ONCHIP_REC12) onchip::make_rec12(sink, sink, sink, false, false, false, &rec12[3 * i]);
            }
            rec[i] = r;
        }
    int rc;
    if (ONCHIP_REC12) {
        if ((rc = dmalloc(s, (void **)&s->oc_rec12, rec12.size() * 4))) return rc;
        HIP_TRY(hipMemcpy(s->oc_rec12, rec12.data(), rec12.size() * 4, hipMemcpyHostToDevice));
    }
    s->oc_rec_bytes = (int64_t)(rec.size() * sizeof(uint64_t));
    if ((rc = dmalloc(s, (void **)&s->oc_rec, rec.size() * sizeof(uint64_t)))) return rc;
    HIP_TRY(hipMemcpy(s->oc_rec, rec.data(), rec.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    if ((rc = dmalloc(s, (void **)&s->oc_tcp, ws.size() * 4))) return rc;
    HIP_TRY(hipMemcpy(s->oc_tcp, ws.data(), ws.size() * 4, hipMemcpyHostToDevice));
    s->oc_tr = tr;
    s->oc_tl = tr < live ? nt - tr : 0;
    // adaptive steps on chip: four voltage arrays in LDS, every tile in VGPRs; the first step of a
    // call on a caller-supplied state runs k_resident's adaptive step (res_ada)
    s->oc_ada = s->oc_tl == 0 && s->n <= onchip::ADA_MAX_N && s->res_ada;
    s->oc_ada = s->oc_ada && odesat::xp_get("ONCHIP_ADAPTIVE", 1) != 0;
    s->oc_poll_limit = (uint32_t)std::min<int64_t>(odesat::xp_get("ONCHIP_POLL_LIMIT", 1 << 22), 1 << 22);
    return ODESAT_OK;
}

template <typename T, int R, bool ADA, bool K3, int NTHR = ResShape<R>::NTH, bool VFG = false, bool FAST = false,
          int RC = 0, int PAIRS = 0>
int launch_resident_k(odesat_solver *s, const RArgs<T> &a) {
    const size_t lds = res_lds_bytes(s->n, R, sizeof(T), ADA && !VFG);
    HIP_TRY(odesat::ensure_max_lds(reinterpret_cast<const void *>(&k_resident<T, R, ADA, K3, NTHR, VFG, FAST, RC, PAIRS>),
                                   (int)RES_LDS_MAX));
    {
        Timed tm(s, 0);
        hipLaunchKernelGGL((k_resident<T, R, ADA, K3, NTHR, VFG, FAST, RC, PAIRS>), dim3(s->G), dim3(NTHR), lds, s->stream,
                           a);
    }
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

// replicas [a.g0, g1) of the solver's G
template <typename T, bool ADA, int WPW, int TW, bool FAST> int launch_wave_k(odesat_solver *s, WArgs<T> a, int64_t g1) {
    a.topo_bytes = (uint32_t)wave_topo_bytes(s->n, s->m);
    a.rep_bytes = (uint32_t)wave_lds_bytes(s->n, s->m, s->L, sizeof(T), ADA);
    const size_t lds = a.topo_bytes + (size_t)WPW * a.rep_bytes;
    const unsigned grid = (unsigned)((g1 - a.g0 + WPW - 1) / WPW), block = WAVE_NTH * WPW * TW;
    HIP_TRY((wave_launch<T, ADA, WPW, TW, FAST>(true, a, grid, block, lds, (int)RES_LDS_MAX, s->stream)));
    hipError_t e;
    {
        Timed tm(s, 0);
        e = wave_launch<T, ADA, WPW, TW, FAST>(false, a, grid, block, lds, (int)RES_LDS_MAX, s->stream);
    }
    HIP_TRY(e);
    return ODESAT_OK;
}

template <typename T, bool ADA, int CPL, int VPL, bool FAST> int launch_solo_k(odesat_solver *s, WArgs<T> a) {
    // k_solo_fast on in-range states, k_solo otherwise
    const size_t lds = FAST ? solo_fast_elems(s->n, s->L, sizeof(T)) * sizeof(T) : (size_t)(s->n + s->L) * sizeof(T);
    const unsigned grid = (unsigned)s->G, block = (unsigned)s->solo_nl;
    HIP_TRY((solo_launch<T, ADA, CPL, VPL, FAST>(true, a, grid, block, lds, (int)RES_LDS_MAX, s->stream)));
    hipError_t e;
    {
        Timed tm(s, 0);
        e = solo_launch<T, ADA, CPL, VPL, FAST>(false, a, grid, block, lds, (int)RES_LDS_MAX, s->stream);
    }
    HIP_TRY(e);
    return ODESAT_OK;
}

template <typename T, bool ADA, int CPL, int VPL> int launch_solo_cv_k(odesat_solver *s, WArgs<T> a) {
    const size_t lds = 2 * (size_t)SOLO_CV_AREA;
    const unsigned grid = (unsigned)s->G, block = (unsigned)s->solo_nl;
    if (block > (unsigned)SOLO_CV_MAX_NL) return fail(ODESAT_EINVAL, "k_solo_cv: too many lanes");
    HIP_TRY((solo_cv_launch<T, ADA, CPL, VPL>(true, a, grid, block, lds, (int)RES_LDS_MAX, s->stream)));
    hipError_t e;
    {
        Timed tm(s, 0);
        e = solo_cv_launch<T, ADA, CPL, VPL>(false, a, grid, block, lds, (int)RES_LDS_MAX, s->stream);
    }
    HIP_TRY(e);
    return ODESAT_OK;
}

template <typename T>
int launch_wave(odesat_solver *s, int step0, int nsteps, bool adaptive, double dt, double zeta, double tol,
                int stop_mode, bool oop, bool fast) {
    WArgs<T> a{};
    a.oop = oop ? 1 : 0;
    a.rec4 = s->wv_rec4;
    a.vst = s->wv_vst;
    a.v0 = (T *)s->v[0];
    a.v1 = (T *)s->v[1];
    a.c0 = (T *)s->c[0];
    a.c1 = (T *)s->c[1];
    a.par = s->par;
    a.dtr = (T *)s->dtr;
    a.act = s->act;
    a.sat_step = s->sat_step;
    a.steps_done = s->steps_done;
    a.stop = s->stop;
    a.n = (int32_t)s->n;
    a.m = (int32_t)s->m;
    a.L = (int32_t)s->L;
    a.step0 = step0;
    a.nsteps = nsteps;
    a.stop_mode = stop_mode;
    a.dt = (T)dt;
    a.zeta = (T)zeta;
    a.xl_max = (T)1e4 * (T)s->m;  // system.rs:95
    a.tol = tol;
    a.io = take_io(s);
    a.G = s->G;
    a.cvrec = s->cv_rec;
    a.cvblk = s->cv_blk;
    a.cvnb = s->cv_nb;
    if (s->solo) {
        auto so = [&](auto cc, auto vv) -> int {
            constexpr int CPL = decltype(cc)::value, VPL = decltype(vv)::value;
            if constexpr (CPL <= 2)
                if (fast && s->solo_fast && s->solo_cv) {
                    if (!s->solo_cv_z0)  // no variable of degree 0: no variable slots
                        return adaptive ? launch_solo_cv_k<T, true, CPL, 0>(s, a) : launch_solo_cv_k<T, false, CPL, 0>(s, a);
                    return adaptive ? launch_solo_cv_k<T, true, CPL, VPL>(s, a) : launch_solo_cv_k<T, false, CPL, VPL>(s, a);
                }
            if (fast && s->solo_fast)
                return adaptive ? launch_solo_k<T, true, CPL, VPL, true>(s, a) : launch_solo_k<T, false, CPL, VPL, true>(s, a);
            return adaptive ? launch_solo_k<T, true, CPL, VPL, false>(s, a) : launch_solo_k<T, false, CPL, VPL, false>(s, a);
        };
        switch (s->solo_cpl * 10 + s->solo_vpl) {
            case 11: return so(IC<1>{}, IC<1>{});
            case 12: return so(IC<1>{}, IC<2>{});
            case 21: return so(IC<2>{}, IC<1>{});
            case 22: return so(IC<2>{}, IC<2>{});
            case 41: return so(IC<4>{}, IC<1>{});
            case 42: return so(IC<4>{}, IC<2>{});
            default: return fail(ODESAT_EINVAL, "k_solo shape not available");
        }
    }
    int64_t g1 = s->G;
    auto go = [&](auto ww, auto tw) -> int {
        constexpr int WPW = decltype(ww)::value, TW = decltype(tw)::value;
        if (fast && s->wave_fast)  // in-range states: the short arithmetic (wave.hpp lane_clauses)
            return adaptive ? launch_wave_k<T, true, WPW, TW, true>(s, a, g1) : launch_wave_k<T, false, WPW, TW, true>(s, a, g1);
        return adaptive ? launch_wave_k<T, true, WPW, TW, false>(s, a, g1) : launch_wave_k<T, false, WPW, TW, false>(s, a, g1);
    };
    // (replicas per workgroup, waves per replica): at most 16 waves per workgroup
    auto shape = [&](int wpw, int tw) -> int {
        switch (wpw * 100 + tw) {
            case 401: return go(IC<4>{}, IC<1>{});
            case 402: return go(IC<4>{}, IC<2>{});
            case 404: return go(IC<4>{}, IC<4>{});
            case 201: return go(IC<2>{}, IC<1>{});
            case 202: return go(IC<2>{}, IC<2>{});
            case 204: return go(IC<2>{}, IC<4>{});
            case 208: return go(IC<2>{}, IC<8>{});
            case 101: return go(IC<1>{}, IC<1>{});
            case 102: return go(IC<1>{}, IC<2>{});
            case 104: return go(IC<1>{}, IC<4>{});
            case 108: return go(IC<1>{}, IC<8>{});
            case 116: return go(IC<1>{}, IC<16>{});
            default: return fail(ODESAT_EINVAL, "k_wave shape not available");
        }
    };
    const int wpw = s->wv_wpw, tw = adaptive ? s->wv_tw_ada : s->wv_tw;
    // One workgroup of wpw replicas per CU: the device works in rounds of wpw * cus replicas.  A partial
    // last round at the solver's shape costs a whole one (config 3, B = 1280: 320 workgroups of 4, the
    // last 64 alone in a second round -- DESIGN.md §6.3), so it runs as a launch of its own after the
    // whole rounds, at fewer replicas per workgroup and the wider teams that leaves room for.  Replicas
    // are independent; a STOP_ANY stop is read by the later launch as by a later round of one launch,
    // and the call's replay logic is unchanged.
    // The tail takes the fewest replicas per workgroup that still fit it in one round: when that is
    // wpw itself (more than (wpw / 2) cus replicas left), one launch does as well (measured: config 3,
    // B = 1792, a tail at 2 per workgroup in two rounds was 14 % slower).  Only workgroups of 16 waves
    // are known to run one per CU; smaller ones may share a CU, and a split measured slower there
    // (config 3 adaptive, B = 768: 2 replicas x 4 waves, 11.3 against 9.0 µs per step).
    const int64_t round = (int64_t)wpw * s->cus, g_main = s->G / round * round, rem = s->G - g_main;
    int wpw_t = 1;
    while (wpw_t < wpw && (rem + wpw_t - 1) / wpw_t > s->cus) wpw_t *= 2;
    if (!s->wave_tail || wpw * tw != 16 || wpw_t == wpw || g_main == 0 || rem == 0) return shape(wpw, tw);
    g1 = g_main;
    int rc = shape(wpw, tw);
    if (rc) return rc;
    int tw_t = 16 / wpw_t;
    while (tw_t > 1 && 32 * (int64_t)tw_t > s->m) tw_t /= 2;
    if (adaptive) tw_t = std::min(tw_t, 4);
    a.g0 = (int32_t)g_main;
    g1 = s->G;
    return shape(wpw_t, tw_t);
}

#ifndef RES_RC
#define RES_RC 28  // register-cached tiles of the f64 fixed-step k_resident (4 VGPRs each)
#endif
#ifndef RES_RC_ADA
#define RES_RC_ADA 12  // the same for the f64 adaptive k_resident (VFG; + the first pass's mn)
#endif
template <typename T>
int launch_resident(odesat_solver *s, int step0, int nsteps, bool adaptive, double dt, double zeta, double tol,
                    int stop_mode, bool oop, bool fast) {
    if (s->res_wave) return launch_wave<T>(s, step0, nsteps, adaptive, dt, zeta, tol, stop_mode, oop, fast);
    if (oop && adaptive) return fail(ODESAT_EINVAL, "out-of-place RESIDENT launches are fixed-step only");
    RArgs<T> a{};
    a.oop = oop ? 1 : 0;
    a.cl4 = s->res_cl4;
    a.cptr = s->cptr;
    a.lits = s->lits;
    a.tc = s->res_tc;
    a.tcw = s->res_tcw;
    a.v0 = (T *)s->v[0];
    a.v1 = (T *)s->v[1];
    a.c0 = (T *)s->c[0];
    a.c1 = (T *)s->c[1];
    a.par = s->par;
    a.cf = (T *)s->cf;
    a.ch = (T *)s->ch;
    a.vf = (T *)s->vf;
    a.dtr = (T *)s->dtr;
    a.act = s->act;
    a.sat_step = s->sat_step;
    a.steps_done = s->steps_done;
    a.stop = s->stop;
    a.n = (int32_t)s->n;
    a.m = (int32_t)s->m;
    a.ntiles = s->res_ntiles;
    a.step0 = step0;
    a.nsteps = nsteps;
    a.stop_mode = stop_mode;
    a.dt = (T)dt;
    a.zeta = (T)zeta;
    a.xl_max = (T)1e4 * (T)s->m;  // system.rs:95
    a.tol = tol;
    a.io = take_io(s);
    const bool k3 = s->uniform_k == 3;
    // 3-SAT on in-range states: the short arithmetic (res_clause3's FAST forms)
    const bool f3 = k3 && fast && s->res_fast;
    if (adaptive && s->res_vfg) {  // R = 1: the full-step clone in HBM
        if (s->res_narrow)
            return f3   ? launch_resident_k<T, 1, true, true, RES_NARROW, true, true>(s, a)
                   : k3 ? launch_resident_k<T, 1, true, true, RES_NARROW, true>(s, a)
                        : launch_resident_k<T, 1, true, false, RES_NARROW, true>(s, a);
        if constexpr (std::is_same<T, double>::value) {
            // the first RES_RC_ADA tiles' memories and first-pass mn in VGPRs for the launch (resident.hpp)
            if (f3 && s->res_rc && s->res_ntiles >= RES_RC_ADA + 16)
                return !s->res_pairs ? launch_resident_k<T, 1, true, true, ResShape<1>::NTH, true, true, RES_RC_ADA>(s, a)
                       : s->oc_off
                           ? launch_resident_k<T, 1, true, true, ResShape<1>::NTH, true, true, RES_RC_ADA, 2>(s, a)
                           : launch_resident_k<T, 1, true, true, ResShape<1>::NTH, true, true, RES_RC_ADA, 1>(s, a);
        }
        return f3   ? launch_resident_k<T, 1, true, true, ResShape<1>::NTH, true, true>(s, a)
               : k3 ? launch_resident_k<T, 1, true, true, ResShape<1>::NTH, true>(s, a)
                    : launch_resident_k<T, 1, true, false, ResShape<1>::NTH, true>(s, a);
    }
    if (s->res_narrow) {
        if (adaptive)
            return f3   ? launch_resident_k<T, 1, true, true, RES_NARROW, false, true>(s, a)
                   : k3 ? launch_resident_k<T, 1, true, true, RES_NARROW>(s, a)
                        : launch_resident_k<T, 1, true, false, RES_NARROW>(s, a);
        return f3   ? launch_resident_k<T, 1, false, true, RES_NARROW, false, true>(s, a)
               : k3 ? launch_resident_k<T, 1, false, true, RES_NARROW>(s, a)
                    : launch_resident_k<T, 1, false, false, RES_NARROW>(s, a);
    }
    auto go = [&](auto rr) -> int {
        constexpr int R = decltype(rr)::value, NT = ResShape<R>::NTH;
        if (adaptive)
            return f3   ? launch_resident_k<T, R, true, true, NT, false, true>(s, a)
                   : k3 ? launch_resident_k<T, R, true, true>(s, a)
                        : launch_resident_k<T, R, true, false>(s, a);
        if constexpr (std::is_same<T, double>::value && R == 1) {
            // f64 fixed steps: the first RES_RC tiles' memories in VGPRs for the launch (resident.hpp)
            if (f3 && s->res_rc && s->res_ntiles >= RES_RC + 16)
                return !s->res_pairs ? launch_resident_k<T, 1, false, true, NT, false, true, RES_RC>(s, a)
                       : s->oc_off ? launch_resident_k<T, 1, false, true, NT, false, true, RES_RC, 2>(s, a)
                                   : launch_resident_k<T, 1, false, true, NT, false, true, RES_RC, 1>(s, a);
        }
        return f3   ? launch_resident_k<T, R, false, true, NT, false, true>(s, a)
               : k3 ? launch_resident_k<T, R, false, true>(s, a)
                    : launch_resident_k<T, R, false, false>(s, a);
    };
    switch (s->res_R) {
        case 1: return go(IC<1>{});
        case 2: return go(IC<2>{});
        case 4: return go(IC<4>{});
        case 8: return go(IC<8>{});
        case 16: return go(IC<16>{});
        case 32: return go(IC<32>{});
        default: return fail(ODESAT_EINVAL, "resident layout not available");
    }
}

int launch_onchip(odesat_solver *s, int step0, int nsteps, double dt, double zeta, int stop_mode, bool oop,
                  bool adaptive, double tol) {
    onchip::Args a{};
    a.dtr = (float *)s->dtr;
    a.tol = (float)tol;
    a.oop = oop ? 1 : 0;
    a.rec = s->oc_rec;
    a.rec_bytes = (uint32_t)s->oc_rec_bytes;
    a.rec12 = s->oc_rec12;
    a.rec12_bytes = (uint32_t)(s->oc_rec_bytes / 8 * 12);
    a.lds = onchip::lds_map(s->n);
    a.tc = s->oc_tcp;
    a.v0 = (float *)s->v[0];
    a.v1 = (float *)s->v[1];
    a.c0 = (float *)s->c[0];
    a.c1 = (float *)s->c[1];
    a.par = s->par;
    a.act = s->act;
    a.sat_step = s->sat_step;
    a.steps_done = s->steps_done;
    a.stop = s->stop;
    a.n = (int32_t)s->n;
    a.m = (int32_t)s->m;
    a.ntiles = s->res_ntiles;
    a.tl = s->oc_tl;
    a.step0 = step0;
    a.nsteps = nsteps;
    a.stop_mode = stop_mode;
    a.dt = (float)dt;
    a.xl_max = 1e4f * (float)s->m;  // system.rs:95, as (T)1e4 * (T)m
    a.io = take_io(s);
    a.poll_limit = s->oc_poll_limit;
    {
        Timed tm(s, 0);
        const size_t lds = adaptive ? onchip::LDS_MAX : onchip::lds_bytes(s->n, s->oc_tl);
        HIP_TRY(onchip::launch(s->oc_tr, s->oc_off, a, s->G, lds, s->stream, adaptive));
    }
    s->check_fault = s->check_fault || onchip::split_barriers(adaptive);
    return ODESAT_OK;
}

// fast: every replica's state is in range (onchip.hip's header) and zeta and dt are finite (k_solo's
// short arithmetic, wave.hpp)
int dispatch_resident(odesat_solver *s, int step0, int nsteps, bool adaptive, double dt, double zeta, double tol,
                      int stop_mode, bool oop, bool fast) {
    return s->dtype == ODESAT_F64
               ? launch_resident<double>(s, step0, nsteps, adaptive, dt, zeta, tol, stop_mode, oop, fast)
               : launch_resident<float>(s, step0, nsteps, adaptive, dt, zeta, tol, stop_mode, oop, fast);
}

template <typename T> int deriv_t(odesat_solver *s, double zeta) {
    return with_layout<T>(s, [&](auto lw, auto vec) -> int {
        constexpr int LW = decltype(lw)::value, VEC = decltype(vec)::value;
        return step_groups<T, LW, VEC, M_DERIV>(s, 0, (T)0, (T)zeta, 0, s->G);
    });
}

// compact host-side f64 [count][items] <-> device layout of a buffer pair (par-selected) or a
// single buffer (pair[1] == nullptr)
template <typename T>
int layout_t(odesat_solver *s, void *const pair[2], const double *dsrc, double *ddst, int64_t items, int stride,
             int comp, int64_t r0, int64_t count, bool scatter) {
    const size_t total = (size_t)count * items;
    if (!total) return ODESAT_OK;
    const int threads = 256;
    const size_t blocks = (total + threads - 1) / threads;
    const uint8_t *par = pair[1] ? s->par : nullptr;
    T *b1 = pair[1] ? (T *)pair[1] : (T *)pair[0];
    const int32_t *imap = stride == 2 ? s->cmap : nullptr;  // clause arrays: caller order -> internal order
    if (scatter)
        hipLaunchKernelGGL((k_scatter<T>), dim3((unsigned)blocks), dim3(threads), 0, s->stream, (T *)pair[0], b1, par,
                           dsrc, imap, (int)items, s->W, stride, comp, r0, count);
    else
        hipLaunchKernelGGL((k_gather<T>), dim3((unsigned)blocks), dim3(threads), 0, s->stream, ddst,
                           (const T *)pair[0], (const T *)b1, par, imap, (int)items, s->W, stride, comp, r0, count);
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

int layout(odesat_solver *s, void *const pair[2], const double *dsrc, double *ddst, int64_t items, int stride,
           int comp, int64_t r0, int64_t count, bool scatter) {
    return s->dtype == ODESAT_F64 ? layout_t<double>(s, pair, dsrc, ddst, items, stride, comp, r0, count, scatter)
                                  : layout_t<float>(s, pair, dsrc, ddst, items, stride, comp, r0, count, scatter);
}

// stride 1: a voltage array; stride 2, comp 0 / 1: the xs / xl half of a clause-memory array
int upload_items(odesat_solver *s, void *const pair[2], const double *host, int64_t items, int stride, int comp,
                 int64_t r0, int64_t count) {
    if (!host || !items || !count) return ODESAT_OK;
    void *stage = nullptr;
    const size_t bytes = (size_t)count * items * sizeof(double);
    HIP_TRY(hipMalloc(&stage, bytes));
    hipError_t e = hipMemcpyAsync(stage, host, bytes, hipMemcpyHostToDevice, s->stream);
    int rc = e == hipSuccess ? layout(s, pair, (const double *)stage, nullptr, items, stride, comp, r0, count, true)
                             : fail(ODESAT_EDEVICE, hipGetErrorString(e));
    hipError_t e2 = hipStreamSynchronize(s->stream);
    (void)hipFree(stage);
    if (rc) return rc;
    HIP_TRY(e2);
    return ODESAT_OK;
}

int download_items(odesat_solver *s, void *const pair[2], double *host, int64_t items, int stride, int comp,
                   int64_t r0, int64_t count) {
    if (!host || !items || !count) return ODESAT_OK;
    void *stage = nullptr;
    const size_t bytes = (size_t)count * items * sizeof(double);
    HIP_TRY(hipMalloc(&stage, bytes));
    int rc = layout(s, pair, nullptr, (double *)stage, items, stride, comp, r0, count, false);
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

// v = counter RNG (or 0), xs = init_short_term_memory, xl = 1 into buffer 0; every group's
// current buffer becomes 0
template <typename T> int init_t(odesat_solver *s, uint64_t seed, int64_t replica0, bool zero_v) {
    const size_t total = std::max(state_elems(s, s->n), state_elems(s, s->m));
    if (!total) return ODESAT_OK;
    const int threads = 256;
    const size_t blocks = (total + threads - 1) / threads;
    hipLaunchKernelGGL((k_init<T>), dim3((unsigned)blocks), dim3(threads), 0, s->stream, (T *)s->v[0],
                       (T *)s->c[0], s->cptr, s->lits, (int)s->n, (int)s->m, s->G, s->W, (int)s->B, seed, replica0,
                       zero_v ? 1 : 0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemsetAsync(s->par, 0, s->G, s->stream));
    return ODESAT_OK;
}

int init_dispatch(odesat_solver *s, uint64_t seed, int64_t replica0, bool zero_v) {
    return s->dtype == ODESAT_F64 ? init_t<double>(s, seed, replica0, zero_v)
                                  : init_t<float>(s, seed, replica0, zero_v);
}

double default_zeta(const odesat_solver *s) {  // system.rs:164-173
    const double d = (double)s->m / (double)s->n;
    return d >= 6.0 ? 0.1 : (d >= 4.9 ? 0.01 : 0.001);
}

void pick_chunk(odesat_solver *s, int64_t replicas) {
    // TWOPASS: one chunk's state + contribution buffer stays inside the 256 MiB Infinity Cache
    const int64_t per_group = (s->n + 2 * s->m + s->L) * s->W * (int64_t)s->tsize;
    int64_t groups;
    if (replicas > 0) {
        groups = std::max<int64_t>(1, replicas / s->W);
    } else {
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
extern "C" const char *odesat_version(void) { return "odesat_amd 0.3 (gfx950)"; }

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
    void *ptrs[] = {s->cptr, s->lits, s->wpos, s->vptr, s->pc, s->ps, s->empty, s->inc, s->v[0], s->v[1], s->c[0],
                    s->c[1], s->par, s->w, s->vh, s->vf, s->ch, s->cf, s->dtr, s->err, s->unsat, s->act,
                    s->sat_step, s->stop, s->res_tc, s->res_tcw, s->cmap, s->res_cl4, s->oc_rec, s->oc_rec12, s->oc_tcp, s->wv_rec4, s->wv_vst,
                    s->cv_rec, s->cv_blk};
    for (void *p : ptrs) dfree(p);
    void *snaps[] = {s->snap_par, s->snap_sat, s->snap_done, s->snap_dt, s->ck_v, s->ck_c, s->ck_dt, s->ck_par,
                     s->ck_act, s->ck_sat, s->ck_done, s->ck_stop};
    for (void *p : snaps) dfree(p);
    void *pinned[] = {s->h_sat, s->h_dt, s->h_stop, s->h_act};  // (h_done lies inside h_sat's block)
    for (void *p : pinned)
        if (p) (void)hipHostFree(p);
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
    if (n >= (1ll << 29) || m >= INT_MAX / 4 || L >= INT_MAX || batch >= INT_MAX / 2)
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
    s->uniform_k = m > 0 ? (int)(f->clause_ptr[1] - f->clause_ptr[0]) : 0;
    for (int64_t c = 0; c < m && s->uniform_k; ++c)
        if (f->clause_ptr[c + 1] - f->clause_ptr[c] != s->uniform_k) s->uniform_k = 0;
    if (s->uniform_k != 3) s->uniform_k = 0;  // the specialised kernels are instantiated for 3-SAT
    // layout.  When the voltages of a replica fit in LDS, the group width is the
    // RESIDENT kernel's replicas per workgroup R = 1 (2 and 4 via ODESAT_GROUP_WIDTH) and RESIDENT is
    // the default.  Otherwise W = min(next pow2 >= batch, 64)
    // for FUSED (measured on MI355X, config 2: W = 64 beats 32 / 16 by 1.5-1.7x).
    // ODESAT_GROUP_WIDTH overrides (tuning; RESIDENT only if that width admits it).
    int lw = 1, res_r = 0;
    // k_wave (wave.hpp) for small 3-SAT instances whose replica -- with the adaptive clones --
    // fits in 64 KiB of LDS (two or more waves per CU); the WAVE knob (0/1) overrides, a set
    // GROUP_WIDTH selects the tile kernels (odesat_set_experiment)
    // (its clause records pack a literal and a term position in 16 bits each)
    if (s->uniform_k == 3 && m > 0 && !odesat::xp_isset("GROUP_WIDTH") && 2 * n + 1 < (1 << 16) && L < (1 << 16)) {
        const int64_t ev = odesat::xp_get("WAVE", -1);
        const size_t topo = wave_topo_bytes(n, m), rep = wave_lds_bytes(n, m, L, s->tsize, true);
        s->wv_wpw = topo + 4 * rep <= RES_LDS_MAX ? 4 : (topo + 2 * rep <= RES_LDS_MAX ? 2 : 1);
        // ... and no more than leaves every CU a workgroup: a small batch spreads over the chip one
        // replica per workgroup, each then a team of up to 16 waves (B = 256 on 256 CUs: WPW 4 -> 1)
        {
            int cus = 256;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
                cus = 256;
            s->cus = cus;
            while (s->wv_wpw > 1 && (batch + s->wv_wpw - 1) / s->wv_wpw < cus) s->wv_wpw /= 2;
            s->wave_tail = odesat::xp_get("WAVE_TAIL", 1) != 0;
        }
        s->res_wave = ev >= 0 ? (ev != 0 && topo + rep <= RES_LDS_MAX) : topo + 2 * rep <= RES_LDS_MAX;
        // waves per replica: LDS holds one workgroup (wv_wpw replicas) per CU, so a replica of one
        // wave leaves a lone wave on each SIMD, which issues a VALU instruction every 4 cycles.  A
        // team of TW waves splits the replica's clauses and variables over 64 TW lanes: the workgroup
        // fills 16 waves (4 per SIMD), fewer while the instance has under 32 clauses per wave.
        // Measured (config 3, B = 1024, adaptive / fixed): 59 / 120 M replica-steps/s at TW = 1,
        // 77 / 162 M at TW = 4; hard.cnf (m = 160) at B = 1: 36 / 17 ms per 10 000 steps at TW = 1,
        // 26 / 14 ms at TW = 4.  The WAVE_TEAM knob (1/2/4/8/16) overrides (if the shape exists).
        s->wv_tw = 16 / s->wv_wpw;
        while (s->wv_tw > 1 && 32 * (int64_t)s->wv_tw > m) s->wv_tw /= 2;
        // adaptive steps order their phases with four barriers, fixed ones with two: a wide team pays
        // twice as many (config 3, B = 256, one replica per workgroup: adaptive 42.4 M replica-steps/s
        // at TW = 4 vs 35.7 M at 16; fixed 80.2 M at 4 vs 91.7 M at 16)
        s->wv_tw_ada = std::min(s->wv_tw, 4);
        {
            const int64_t t = odesat::xp_get("WAVE_TEAM", -1);
            if ((t == 1 || t == 2 || t == 4 || t == 8 || t == 16) && t * s->wv_wpw <= 16) s->wv_tw = s->wv_tw_ada = (int)t;
        }
    }
    if (s->res_wave) {
        res_r = lw = 1;
    } else if (res_fits(n, 1, s->tsize, false)) {  // measured (config 2, B = 1024): R = 1 beats R = 2 by 1.13x
        res_r = lw = small_instance_width(f, n, batch, device, s->tsize);
    } else {
        while (lw < batch && lw < 64) lw <<= 1;
    }
    if (odesat::xp_isset("GROUP_WIDTH")) {
        const int want = (int)odesat::xp_get("GROUP_WIDTH", 0);
        if (want == 1 || want == 2 || want == 4 || want == 8 || want == 16 || want == 32 || want == 64) {
            lw = want;
            res_r = (want <= 32 && res_fits(n, want, s->tsize, false)) ? want : 0;
        }
    }
    // One replica per wave (RES_NARROW) when the tile chain is deep and narrow: 64-clause tiles
    // then need barely more tiles than 512-clause ones, and a replica's step costs one wave instead
    // of eight (hard.cnf at B = 1: a step is a chain of ~20 tiles of ~8 clauses).
    // The RES_NARROW knob (0/1) overrides.
    if (res_r == 1 && m > 0 && !s->res_wave) {
        const int64_t ev = odesat::xp_get("RES_NARROW", -1);
        if (ev >= 0) s->res_narrow = ev != 0;
        else s->res_narrow = 4 * tile_count(f, n, RES_NARROW) <= 5 * tile_count(f, n, ResShape<1>::NL);
    }
    // the internal clause order: var-disjoint tiles for RESIDENT, else the file order
    std::vector<int32_t> perm, tiles, wst;
    std::vector<uint8_t> lorder;  // per internal clause: literal order code (kP3), 0 = file order
    // wave-paired tiles where ONCHIP may run (onchip_setup's conditions; k_onchip needs them);
    // the ONCHIP_PAIRS knob = 0: plain tiles (RESIDENT)
    // (f64: k_resident's short-form launches on the same tiles, RES_PAIRS; round 5)
    bool pairs = res_r == 1 && !s->res_narrow && !s->res_wave && s->uniform_k == 3 &&
                 (s->dtype == ODESAT_F32 ? n <= onchip::MAX_N && odesat::xp_get("ONCHIP", 1) != 0
                                         : odesat::xp_get("RES_PAIRS", 1) != 0);
    pairs = pairs && odesat::xp_get("ONCHIP_PAIRS", 1) != 0;
    const int cap = s->res_narrow ? RES_NARROW : res_capacity(res_r);
    if (s->res_wave) {  // no tiles: the file order, one pseudo-tile
        perm.resize(m);
        for (int64_t c = 0; c < m; ++c) perm[c] = (int32_t)c;
        tiles = {0, (int32_t)m};
        lorder.assign(m, 0);
    } else if (res_r > 0 && !build_tiles(f, n, cap, res_r, s->uniform_k == 3, pairs, perm, tiles, lorder, wst, s->oc_off)) {
        res_r = 0;
    } else if (res_r > 0 && pairs && s->dtype == ODESAT_F64 &&
               (odesat::xp_get("RES_RC", 1) == 0 || ((int)tiles.size() + 2) / 4 * 4 < RES_RC_ADA + 16)) {
        // f64: only the register-tile launches run the paired barriers (launch_resident); without them
        // the paired tiling can only cost tiles, so such solvers take the plain tiling
        pairs = false;
        if (!build_tiles(f, n, cap, res_r, s->uniform_k == 3, pairs, perm, tiles, lorder, wst, s->oc_off)) res_r = 0;
    }
    if (res_r != 1) s->res_narrow = false;
    if (res_r == 0 && !odesat::xp_isset("GROUP_WIDTH")) {
        lw = 1;
        while (lw < batch && lw < 64) lw <<= 1;
    }
    if (res_r == 0) {
        perm.resize(m);
        for (int64_t c = 0; c < m; ++c) perm[c] = (int32_t)c;
        lorder.assign(m, 0);
    }
    s->LW = lw;
    s->W = s->LW;
    s->Bp = (batch + s->W - 1) / s->W * s->W;
    s->G = (int)(s->Bp / s->W);
    pick_chunk(s, 0);
    int rc = ODESAT_OK;
    auto bail = [&](int code) {
        odesat_solver_destroy(s);
        return code;
    };
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "hipStreamCreate failed"));

    // topology, in the internal clause order (perm[k] = original clause; cmap is its inverse):
    // clause CSR, packed literals, variable-major slot positions (sorted by ORIGINAL slot, i.e. the
    // reference's clause-then-literal accumulation order) and their inverse
    std::vector<int32_t> cptr(m + 1), lits(L), wpos(L), vptr(n + 1, 0), pc(L), ps(L), empty, cmap(m);
    cptr[0] = 0;
    for (int64_t k = 0; k < m; ++k) {
        const int64_t c = perm[k];
        cmap[c] = (int32_t)k;
        const int64_t len = f->clause_ptr[c + 1] - f->clause_ptr[c];
        cptr[k + 1] = cptr[k] + (int32_t)len;
        for (int64_t q = 0; q < len; ++q) {  // internal slot q holds original literal j
            const int64_t j = len == 3 ? kP3[lorder[k]][q] : q;
            const int64_t so = f->clause_ptr[c] + j;
            lits[cptr[k] + q] = (int32_t)((f->var[so] << 1) | (f->neg[so] ? 1 : 0));
        }
        if (len == 0) empty.push_back((int32_t)k);
    }
    for (int64_t s2 = 0; s2 < L; ++s2) vptr[f->var[s2] + 1] += 1;
    for (int64_t i = 0; i < n; ++i) vptr[i + 1] += vptr[i];
    {
        std::vector<int32_t> fill(vptr.begin(), vptr.end() - 1);
        for (int64_t c = 0; c < m; ++c) {  // original order
            const int32_t k = cmap[c];
            const int64_t len = f->clause_ptr[c + 1] - f->clause_ptr[c];
            for (int64_t j = 0; j < len; ++j) {
                const int32_t p = fill[f->var[f->clause_ptr[c] + j]]++;
                int32_t q = (int32_t)j;  // internal slot of original literal j
                if (len == 3)
                    for (int qq = 0; qq < 3; ++qq)
                        if (kP3[lorder[k]][qq] == j) q = qq;
                const int32_t si = cptr[k] + q;
                wpos[si] = p;
                pc[p] = k;
                ps[p] = si;
            }
        }
    }
    s->n_empty = (int)empty.size();
    std::vector<Inc> inc;
    if (s->uniform_k == 3) {  // {clause << 2 | own literal position, lit0, lit1, lit2} per position
        inc.resize(L);
        for (int64_t p = 0; p < L; ++p) {
            const int32_t c = pc[p], s0 = cptr[c];
            inc[p] = Inc{(c << 2) | (ps[p] - s0), lits[s0], lits[s0 + 1], lits[s0 + 2]};
        }
    }
    if ((rc = dmalloc(s, (void **)&s->cptr, (m + 1) * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->lits, L * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->wpos, L * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->vptr, (n + 1) * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->pc, L * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->ps, L * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->empty, empty.size() * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->inc, inc.size() * 16))) return bail(rc);
    if (hipMemcpy(s->cptr, cptr.data(), (m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (L && hipMemcpy(s->lits, lits.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (L && hipMemcpy(s->wpos, wpos.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (L && hipMemcpy(s->pc, pc.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (L && hipMemcpy(s->ps, ps.data(), L * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (!empty.empty() && hipMemcpy(s->empty, empty.data(), empty.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (!inc.empty() && hipMemcpy(s->inc, inc.data(), inc.size() * 16, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(s->vptr, vptr.data(), (n + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
    if ((rc = dmalloc(s, (void **)&s->cmap, m * 4))) return bail(rc);
    if (m && hipMemcpy(s->cmap, cmap.data(), m * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
    if (res_r > 0) {
        if (s->uniform_k == 3)  // the 3-SAT pipeline is unrolled by 4: pad with empty tiles
            while ((tiles.size() - 1) % 4 != 0) tiles.push_back(tiles.back());
        std::vector<int4> cl4(s->uniform_k == 3 ? m : 0);
        for (size_t k = 0; k < cl4.size(); ++k) cl4[k] = make_int4(lits[3 * k], lits[3 * k + 1], lits[3 * k + 2], 0);
        if ((rc = dmalloc(s, (void **)&s->res_tc, tiles.size() * 4))) return bail(rc);
        if ((rc = dmalloc(s, (void **)&s->res_cl4, cl4.size() * 16))) return bail(rc);
        if (hipMemcpy(s->res_tc, tiles.data(), tiles.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
            (!cl4.empty() && hipMemcpy(s->res_cl4, cl4.data(), cl4.size() * 16, hipMemcpyHostToDevice) != hipSuccess))
            return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
        s->res_R = res_r;
        s->res_ada = res_fits(n, res_r, s->tsize, true);
        s->res_fast = odesat::xp_get("RES_FAST", 1) != 0;
        s->res_rc = odesat::xp_get("RES_RC", 1) != 0;
        // adaptive steps whose clone of v does not fit beside v and dv (f64 at n > 6.7 k, the CLI's
        // default precision and mode on config 2): k_resident with the clone in HBM instead of FUSED
        // on the one-replica layout.  The RES_VFG knob = 0 keeps FUSED.
        if (!s->res_ada && res_r == 1 && !s->res_wave) {
            s->res_vfg = odesat::xp_get("RES_VFG", 1) != 0;
            s->res_ada = s->res_vfg;
        }
        s->res_ntiles = (int)tiles.size() - 1;
        s->alg = ODESAT_ALG_RESIDENT;
        if (s->dtype == ODESAT_F64 && !wst.empty()) {  // the wave table of the paired tiles (k_resident PAIRS)
            std::vector<int32_t> ws((size_t)(s->res_ntiles + 16) * PAIR_WAVES + 1, (int32_t)m);
            std::copy(wst.begin(), wst.end() - 1, ws.begin());
            if ((rc = dmalloc(s, (void **)&s->res_tcw, ws.size() * 4))) return bail(rc);
            if (hipMemcpy(s->res_tcw, ws.data(), ws.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
                return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
            s->res_pairs = true;
        }
        if (s->res_wave) {  // k_wave: variable-major term positions, incidences sorted by (clause, literal)
            std::vector<int32_t> vst((size_t)n + 1, 0), fillc((size_t)n, 0);
            for (int64_t k = 0; k < L; ++k) vst[(lits[k] >> 1) + 1] += 1;
            for (int64_t i = 0; i < n; ++i) vst[i + 1] += vst[i];
            std::vector<int4> rec4((size_t)m);
            for (int64_t c = 0; c < m; ++c) {
                int q[3];
                for (int j = 0; j < 3; ++j) {
                    const int32_t v = lits[3 * c + j] >> 1;
                    q[j] = lits[3 * c + j] | (vst[v] + fillc[v]++) << 16;  // both < 2^16 (selection)
                }
                rec4[c] = make_int4(q[0], q[1], q[2], 0);
            }
            if ((rc = dmalloc(s, (void **)&s->wv_rec4, (size_t)m * 16)) || (rc = dmalloc(s, (void **)&s->wv_vst, (n + 1) * 4)))
                return bail(rc);
            if (hipMemcpy(s->wv_rec4, rec4.data(), (size_t)m * 16, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(s->wv_vst, vst.data(), (n + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
                return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
            s->res_ada = true;  // wave_lds_bytes(adaptive) fits by selection
            // k_solo (wave.hpp): the latency path when k_wave would run one replica per workgroup
            // anyway (small batches, B = 1 for solve): every lane's clause and variable slots in
            // registers.  Lanes: one per clause rounded up to a wave, at least 192 and at most 512
            // (measured, profiles/r03_solo_sweep.jsonl: config 3 at 512 lanes 15-25 % under k_wave's
            // best team, at 1024 no faster and slower in f64 adaptive steps; round 4,
            // profiles/r04ae_solo_lanes.txt: hard.cnf (m = 160) f64 criterion calls 4.64-4.66 / 12.23-12.24
            // ms fixed / adaptive at 192 lanes against 4.85-4.93 / 12.54-12.57 at 256 and 5.6 / 13.4 at 128).
            // The SOLO (0/1) and SOLO_LANES knobs override.
            int64_t nl = std::min<int64_t>(512, std::max<int64_t>(192, (m + 63) / 64 * 64));
            {
                const int64_t want = odesat::xp_get("SOLO_LANES", -1);
                if (want >= 64 && want <= SOLO_MAX_NL && want % 64 == 0) nl = want;
            }
            const int64_t cpl = (m + nl - 1) / nl, vpl = (n + nl - 1) / nl;
            const bool fits = cpl <= 4 && vpl <= 2 && (size_t)(n + L) * s->tsize <= RES_LDS_MAX;
            s->solo = fits && s->wv_wpw == 1;
            if (odesat::xp_isset("SOLO")) s->solo = fits && odesat::xp_get("SOLO", 0) != 0;
            s->solo_nl = (int)nl;
            s->solo_cpl = cpl <= 1 ? 1 : (cpl <= 2 ? 2 : 4);
            s->solo_vpl = (int)vpl;
            // k_solo_fast's padded term blocks must fit as well
            s->solo_fast = solo_fast_elems(n, L, s->tsize) * s->tsize <= RES_LDS_MAX;
            s->solo_fast = s->solo_fast && odesat::xp_get("SOLO_FAST", 1) != 0;
            // k_solo_cv (wave.hpp): the clause slots hold their literals' voltages and fold them
            // themselves (2 barriers per adaptive step instead of 4); up to 2 clause slots per lane,
            // 512 lanes, no variable with more terms than a padded block holds, and its two term
            // areas in LDS.  The SOLO_CV knob (0) turns it off.
            int64_t dmax = 0;
            s->solo_cv_z0 = false;
            for (int64_t i = 0; i < n; ++i) {
                dmax = std::max<int64_t>(dmax, vst[i + 1] - vst[i]);
                s->solo_cv_z0 = s->solo_cv_z0 || vst[i + 1] == vst[i];
            }
            s->solo_cv = s->solo && s->solo_cpl <= 2 && nl <= SOLO_CV_MAX_NL && dmax <= SOLO_DPAD &&
                         n + 1 <= solo_cv_blk_cap(s->tsize) && odesat::xp_get("SOLO_CV", 1) != 0;
            if (s->solo_cv) {  // the lanes' clauses and the term blocks (cv_layout.cpp; knob CV_ITERS = 0: plain)
                const int nslot = (int)nl * s->solo_cpl;
                std::vector<int32_t> sc, so, blk;
                const int iters = (int)odesat::xp_get("CV_ITERS", 20000);
                s->solo_cv = odesat::cv_layout(n, m, lits.data(), vst.data(), (int)nl, s->solo_cpl, (int)s->tsize,
                                               solo_cv_blk_cap(s->tsize), iters, sc, so, blk, &s->cv_cost_plain,
                                               &s->cv_cost);
                if (s->solo_cv) {
                    std::vector<int4> cr((size_t)nslot);
                    for (int t = 0; t < nslot; ++t) {
                        const int c = sc[t] >= 0 ? sc[t] : 0;
                        const int f[3] = {rec4[c].x, rec4[c].y, rec4[c].z};
                        cr[t] = make_int4(f[so[3 * t]], f[so[3 * t + 1]], f[so[3 * t + 2]], sc[t]);
                    }
                    s->cv_nb = 1 + *std::max_element(blk.begin(), blk.end());
                    if ((rc = dmalloc(s, (void **)&s->cv_rec, (size_t)nslot * 16)) ||
                        (rc = dmalloc(s, (void **)&s->cv_blk, (n + 1) * 4)))
                        return bail(rc);
                    if (hipMemcpy(s->cv_rec, cr.data(), (size_t)nslot * 16, hipMemcpyHostToDevice) != hipSuccess ||
                        hipMemcpy(s->cv_blk, blk.data(), (n + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
                        return bail(fail(ODESAT_EDEVICE, "topology upload failed"));
                }
            }
            s->wave_fast = odesat::xp_get("WAVE_FAST", 1) != 0;
        }
        if ((rc = onchip_setup(s, tiles, wst, lits))) return bail(rc);
        if (s->oc_tr > 0) s->alg = ODESAT_ALG_ONCHIP;
    }
    // state (double-buffered)
    for (int b = 0; b < 2; ++b) {
        if ((rc = dmalloc(s, &s->v[b], state_elems(s, n) * s->tsize))) return bail(rc);
        if ((rc = dmalloc(s, &s->c[b], 2 * state_elems(s, m) * s->tsize))) return bail(rc);
    }
    if ((rc = dmalloc(s, (void **)&s->par, s->G))) return bail(rc);
    if ((rc = dmalloc(s, &s->dtr, s->Bp * s->tsize))) return bail(rc);
    if ((rc = dmalloc(s, &s->err, s->Bp * 8))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->unsat, s->Bp * 4))) return bail(rc);
    if ((rc = dmalloc(s, (void **)&s->act, s->Bp))) return bail(rc);
    // sat steps and steps done side by side (one device-to-host copy returns both, finish_simulate)
    if ((rc = dmalloc(s, (void **)&s->sat_step, 2 * s->Bp * 8))) return bail(rc);
    s->steps_done = s->sat_step + s->Bp;
    if ((rc = dmalloc(s, (void **)&s->stop, 16))) return bail(rc);
    if (hipMemset(s->stop, 0, 16) != hipSuccess) return bail(fail(ODESAT_EDEVICE, "memset failed"));  // stop[1]: fault word
    if (hipHostMalloc((void **)&s->h_sat, 2 * s->Bp * 8) != hipSuccess ||
        hipHostMalloc((void **)&s->h_dt, s->Bp * 8) != hipSuccess ||
        hipHostMalloc((void **)&s->h_stop, 16) != hipSuccess || hipHostMalloc((void **)&s->h_act, s->Bp) != hipSuccess)
        return bail(fail(ODESAT_ENOMEM, "hipHostMalloc failed"));
    s->h_done = s->h_sat + s->Bp;
    if (hipMemsetAsync(s->err, 0, s->Bp * 8, s->stream) != hipSuccess)
        return bail(fail(ODESAT_EDEVICE, "memset failed"));
    // default state: v = 0, xs = init_short_term_memory, xl = 1
    if ((rc = init_dispatch(s, 0, 0, true))) return bail(rc);
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

extern "C" int odesat_set_algorithm(odesat_solver *s, int alg) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (alg != ODESAT_ALG_FUSED && alg != ODESAT_ALG_TWOPASS && alg != ODESAT_ALG_RESIDENT && alg != ODESAT_ALG_ONCHIP)
        return fail(ODESAT_EINVAL, "bad algorithm");
    if (alg == ODESAT_ALG_ONCHIP && s->oc_tr == 0)
        return fail(ODESAT_EINVAL, "ONCHIP needs an f32 3-SAT formula whose tiles fit one CU's VGPRs + LDS "
                                   "(group width 1); this solver does not admit it");
    if (alg == ODESAT_ALG_RESIDENT && s->res_R == 0)
        return fail(ODESAT_EINVAL, "RESIDENT needs the voltages of a replica group in LDS: this solver's layout "
                                   "(group width " + std::to_string(s->W) + ") does not admit it");
    s->alg = alg;
    return ODESAT_OK;
}

extern "C" int odesat_get_algorithm(const odesat_solver *s) {
    return s ? s->alg : fail(ODESAT_EINVAL, "null solver");
}

extern "C" int odesat_group_width(const odesat_solver *s) { return s ? s->W : fail(ODESAT_EINVAL, "null solver"); }

// the dispatch of simulate_impl / simulate_resident, named
extern "C" const char *odesat_step_kernel(const odesat_solver *s, int adaptive) {
    if (!s) return nullptr;
    if ((s->alg == ODESAT_ALG_RESIDENT || s->alg == ODESAT_ALG_ONCHIP) && (!adaptive || s->res_ada)) {
        if (s->alg == ODESAT_ALG_ONCHIP && (!adaptive || s->oc_ada)) return "k_onchip";
        return s->res_wave ? (s->solo ? "k_solo" : "k_wave") : "k_resident";
    }
    return s->alg == ODESAT_ALG_TWOPASS ? "k_clause_u" : "k_step";
}

extern "C" int odesat_set_state(odesat_solver *s, int64_t r0, int64_t count, const double *v, const double *xs,
                                const double *xl) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    if ((rc = upload_items(s, s->v, v, s->n, 1, 0, r0, count))) return rc;
    if ((rc = upload_items(s, s->c, xs, s->m, 2, 0, r0, count))) return rc;
    if ((rc = upload_items(s, s->c, xl, s->m, 2, 1, r0, count))) return rc;
    if ((rc = reset_replicas(s, r0, count))) return rc;
    if ((rc = set_stop(s, INT_MAX))) return rc;  // a new state ends the run (and a STOP_ANY stop)
    auto within = [](const double *x, int64_t cnt, double lo, double hi) {
        if (!x) return true;
        for (int64_t i = 0; i < cnt; ++i)
            if (!(x[i] >= lo && x[i] <= hi)) return false;  // NaN fails too
        return true;
    };
    // xs: 0 or 1e-3 <= |xs| <= 1, so |xl xs| is 0 or >= 1e-3 and no term of the short forms
    // (onchip.hip header) can round through a subnormal
    auto within_xs = [](const double *x, int64_t cnt) {
        if (!x) return true;
        for (int64_t i = 0; i < cnt; ++i) {
            const double a = std::fabs(x[i]);
            if (!(a == 0.0 || (a >= 1e-3 && a <= 1.0))) return false;  // NaN fails too
        }
        return true;
    };
    s->in_range = s->in_range && within(v, count * s->n, -1.0, 1.0) && within_xs(xs, count * s->m) &&
                  within(xl, count * s->m, 1.0, 1e30);
    s->t_base = 0;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

extern "C" int odesat_init_state(odesat_solver *s, uint64_t seed, int64_t replica0) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if ((rc = init_dispatch(s, seed, replica0, false))) return rc;
    if ((rc = reset_replicas(s, 0, s->Bp))) return rc;
    if ((rc = set_stop(s, INT_MAX))) return rc;  // a new state ends the run (and a STOP_ANY stop)
    s->in_range = true;  // v in [-1, 1), xs = +-1, xl = 1
    s->t_base = 0;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

extern "C" int odesat_get_state(odesat_solver *s, int64_t r0, int64_t count, double *v, double *xs, double *xl) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (r0 < 0 || count < 0 || r0 + count > s->B) return fail(ODESAT_EINVAL, "replica range out of bounds");
    if ((rc = download_items(s, s->v, v, s->n, 1, 0, r0, count))) return rc;
    if ((rc = download_items(s, s->c, xs, s->m, 2, 0, r0, count))) return rc;
    if ((rc = download_items(s, s->c, xl, s->m, 2, 1, r0, count))) return rc;
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
    void *const vh[2] = {s->vh, nullptr}, *const ch[2] = {s->ch, nullptr};
    if ((rc = download_items(s, vh, dv, s->n, 1, 0, 0, s->B))) return rc;
    if ((rc = download_items(s, ch, dxs, s->m, 2, 0, 0, s->B))) return rc;
    if ((rc = download_items(s, ch, dxl, s->m, 2, 1, 0, s->B))) return rc;
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
    if (!adaptive) s->in_range = true;  // every replica took a clamped step
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

// Results of a simulate call: per-replica bookkeeping through the pinned staging buffers, one sync.
static int finish_simulate(odesat_solver *s, const odesat_params *p, bool adaptive, int64_t t_run,
                           int64_t *first_sat_step, int64_t *steps_done, double *dt_out, int64_t *steps_run) {
    const bool mirrored = s->io_mirror;  // the launches stored the results in the pinned buffers themselves
    s->io_mirror = s->io_begin = false;
    if (!mirrored) {
        if (first_sat_step && steps_done)  // one copy: the two arrays are adjacent (Bp apart)
            HIP_TRY(hipMemcpyAsync(s->h_sat, s->sat_step, (s->Bp + s->B) * 8, hipMemcpyDeviceToHost, s->stream));
        else if (first_sat_step)
            HIP_TRY(hipMemcpyAsync(s->h_sat, s->sat_step, s->B * 8, hipMemcpyDeviceToHost, s->stream));
        else if (steps_done)
            HIP_TRY(hipMemcpyAsync(s->h_done, s->steps_done, s->B * 8, hipMemcpyDeviceToHost, s->stream));
        if (dt_out && adaptive)
            HIP_TRY(hipMemcpyAsync(s->h_dt, s->dtr, s->B * s->tsize, hipMemcpyDeviceToHost, s->stream));
    }
    // the stop word (STOP_ANY) and the fault word beside it (a k_onchip split-barrier wait that gave up)
    const bool fault_check = s->check_fault;
    s->check_fault = false;
    if (p->stop == ODESAT_STOP_ANY || fault_check)
        HIP_TRY(hipMemcpyAsync(s->h_stop, s->stop, 8, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (fault_check && s->h_stop[1] != 0) {
        HIP_TRY(hipMemsetAsync(s->stop + 1, 0, 4, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        return fail(ODESAT_EDEVICE, "k_onchip: a split-barrier wait timed out; the launch's dv updates may have "
                                    "raced, so its results are not returned (re-run the call)");
    }
    // simulate_inter runs T + 1 steps when step T is the first allsat one (system.rs:291): launches
    // after it were no-ops
    if (p->stop == ODESAT_STOP_ANY && *s->h_stop != INT_MAX)
        t_run = std::max<int64_t>(0, std::min<int64_t>(t_run, (int64_t)*s->h_stop - s->t_base + 1));
    if (t_run > 0) s->in_range = true;  // every replica that stepped took a clamped step
    s->t_base += t_run;
    if (steps_run) *steps_run = t_run;
    if (first_sat_step) std::memcpy(first_sat_step, s->h_sat, s->B * 8);
    if (steps_done) std::memcpy(steps_done, s->h_done, s->B * 8);
    if (dt_out) {
        for (int64_t r = 0; r < s->B; ++r)
            dt_out[r] = !adaptive ? p->dt
                                  : (s->dtype == ODESAT_F64 ? s->h_dt[r] : (double)reinterpret_cast<float *>(s->h_dt)[r]);
    }
    return s->profile ? ODESAT_OK : drain_profile(s);
}

// STOP_ANY replay: the bookkeeping a multi-step launch starts from (the state itself survives in the
// other buffer of each group, the launch writing out of place).
static int ensure_snapshot(odesat_solver *s) {
    if (s->snap_par) return ODESAT_OK;
    int rc;
    if ((rc = dmalloc(s, (void **)&s->snap_par, s->G)) || (rc = dmalloc(s, (void **)&s->snap_sat, s->Bp * 8)) ||
        (rc = dmalloc(s, (void **)&s->snap_done, s->Bp * 8)) || (rc = dmalloc(s, &s->snap_dt, s->Bp * s->tsize)))
        return rc;
    return ODESAT_OK;
}

static int snapshot(odesat_solver *s, bool restore) {
    auto cp = [&](void *dst, const void *src, size_t bytes) {
        return hipMemcpyAsync(restore ? const_cast<void *>(src) : dst, restore ? dst : src, bytes,
                              hipMemcpyDeviceToDevice, s->stream);
    };
    HIP_TRY(cp(s->snap_par, s->par, s->G));
    HIP_TRY(cp(s->snap_sat, s->sat_step, s->Bp * 8));
    HIP_TRY(cp(s->snap_done, s->steps_done, s->Bp * 8));
    HIP_TRY(cp(s->snap_dt, s->dtr, s->Bp * s->tsize));
    if (restore) HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)s->stop, INT_MAX, 1, s->stream));
    return ODESAT_OK;
}

static int read_stop(odesat_solver *s, int32_t *out) {
    HIP_TRY(hipMemcpyAsync(s->h_stop, s->stop, 4, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    *out = *s->h_stop;
    return ODESAT_OK;
}

// odesat_simulate for the persistent kernels (RESIDENT / k_wave / ONCHIP): launches of `poll` steps,
// polled at the launch ends.  STOP_ANY (simulate_inter, system.rs:278-294): every replica takes the
// step at which the first one is allsat, and none goes further.  The launches are written out of
// place (the starting state survives in the other buffer of each group); when one finds the first
// allsat step T inside it, the bookkeeping is restored and the launch re-runs from its start to T
// exactly -- bit-identical, the integration being deterministic -- so the multi-step launches cost
// nothing over STOP_NONE until the stop.  RESIDENT's adaptive pass updates in place: one step per
// launch there.
static int simulate_resident(odesat_solver *s, const odesat_params *p, bool adaptive, double zeta, double tol,
                             int poll, int64_t *first_sat_step, int64_t *steps_done, double *dt_out,
                             int64_t *steps_run) {
    int rc = ODESAT_OK;
    // ONCHIP needs in-range states (onchip.hip): when the caller's state may not be, the first step
    // runs RESIDENT, whose clamps bring every state into range.  (The kernel omits the rigidity term
    // and uses med3 clamps: both exact for finite zeta and a finite, normal dt -- onchip.hip.)
    const double adt = std::fabs(p->dt);
    const bool oc = s->alg == ODESAT_ALG_ONCHIP && (!adaptive || s->oc_ada) && std::fabs(zeta) <= 1e6 && adt >= 1e-30 &&
                    adt <= 1e30;
    const bool any = p->stop == ODESAT_STOP_ANY;
    const bool replay = any && (oc || s->res_wave || !adaptive);
    const int per_launch = any && !replay ? 1 : poll;
    const int64_t base = s->t_base;
    if (replay && (rc = ensure_snapshot(s))) return rc;
    const bool finite = std::fabs(zeta) <= 1e6 && adt >= 1e-30 && adt <= 1e30;  // (k_solo's short arithmetic)
    auto launch = [&](int64_t t0, int k, bool oop) -> int {
        const bool use_oc = oc && (t0 > 0 || s->in_range);
        // the RESIDENT stand-in step of an ONCHIP solver on an out-of-range state is a one-step launch
        // (nothing to replay), and adaptive k_resident updates in place: it never runs out of place
        return use_oc ? launch_onchip(s, (int)(base + t0), k, p->dt, zeta, p->stop, oop, adaptive, tol)
                      : dispatch_resident(s, (int)(base + t0), k, adaptive, p->dt, zeta, tol, p->stop,
                                          oop && (s->res_wave || !adaptive), finite && (t0 > 0 || s->in_range));
    };
    int64_t t = 0, next_poll = poll;
    while (t < p->max_steps) {
        const bool use_oc = oc && (t > 0 || s->in_range);
        int k = (int)std::min<int64_t>(std::min<int64_t>(per_launch, next_poll - t), p->max_steps - t);
        if (oc && !use_oc) k = 1;
        if (replay && k > 1 && (rc = snapshot(s, false))) return rc;
        if ((rc = launch(t, k, replay))) return rc;
        const int64_t t0 = t;
        t += k;
        const bool at_poll = t >= next_poll;
        if (at_poll) next_poll += poll;
        if (replay && k > 1) {  // every multi-step launch is polled, the last one too: it may have run past the stop
            // (a one-step launch cannot run past it: later launches see the stop word and do nothing,
            // so those are polled only at the poll interval, below)
            int32_t h_stop = INT_MAX;
            if ((rc = read_stop(s, &h_stop))) return rc;
            if (h_stop == INT_MAX) continue;
            const int64_t T = (int64_t)h_stop - base;  // this call's step index of the first allsat step
            if (T < t - 1) {  // replicas ran past T: back to the launch's start, then exactly to T
                if ((rc = snapshot(s, true))) return rc;
                if ((rc = launch(t0, (int)(T - t0 + 1), true))) return rc;
                t = T + 1;
            }
            break;
        }
        if (!at_poll || p->stop == ODESAT_STOP_NONE || t >= p->max_steps) continue;
        if (any) {
            int32_t h_stop = INT_MAX;
            if ((rc = read_stop(s, &h_stop))) return rc;
            if (h_stop != INT_MAX) break;
        } else {  // STOP_EACH: stop once every replica is frozen
            HIP_TRY(hipMemcpyAsync(s->h_act, s->act, s->Bp, hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            bool live = false;
            for (int64_t r = 0; r < s->B && !live; ++r) live = s->h_act[r] != 0;
            if (!live) break;
        }
    }
    return finish_simulate(s, p, adaptive, t, first_sat_step, steps_done, dt_out, steps_run);
}

static int simulate_impl(odesat_solver *s, const odesat_params *p, bool cont, int64_t *first_sat_step,
                         int64_t *steps_done, double *dt_out, int64_t *steps_run) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (!p) return fail(ODESAT_EINVAL, "null params");
    if (p->dt_policy != ODESAT_DT_PER_REPLICA)
        return fail(ODESAT_EINVAL, "the device runs every replica with its own dt (ODESAT_DT_PER_REPLICA)");
    if (p->max_steps <= 0 || p->max_steps > INT_MAX - 1)
        return fail(ODESAT_EINVAL, "max_steps must be in [1, 2^31-2] (unbounded runs are refused)");
    if (p->stop != ODESAT_STOP_EACH && p->stop != ODESAT_STOP_ANY && p->stop != ODESAT_STOP_NONE)
        return fail(ODESAT_EINVAL, "bad stop policy");
    const bool adaptive = p->adaptive != 0;
    const double tol = p->tol;
    const double zeta = p->zeta < 0 ? default_zeta(s) : p->zeta;
    if ((rc = ensure_w(s))) return rc;
    if (adaptive && (rc = ensure_scratch(s))) return rc;
    // the persistent kernels (simulate_resident) take the call's first-launch bookkeeping reset and, on
    // STOP_NONE calls, the copy of the results into their own launches (callio.hpp); STOP_ANY keeps
    // k_begin_call (its stop word must be reset before any workgroup reads it)
    const bool persistent = (s->alg == ODESAT_ALG_ONCHIP && (!adaptive || s->oc_ada)) ||
                            ((s->alg == ODESAT_ALG_RESIDENT || s->alg == ODESAT_ALG_ONCHIP) && (!adaptive || s->res_ada));
    s->io_begin = s->io_mirror = false;
    if (!cont && persistent && p->stop != ODESAT_STOP_ANY) {
        s->t_base = 0;
        s->io_begin = true;
        s->io_mirror = p->stop == ODESAT_STOP_NONE;
    } else if (!cont) {  // per-call bookkeeping restarts; adaptive dt restarts at 0.01 (:205) -- one async kernel
        s->t_base = 0;
        const int threads = 256;
        hipLaunchKernelGGL(k_begin_call, dim3((unsigned)((s->Bp + threads - 1) / threads)), dim3(threads), 0,
                           s->stream, s->act, s->unsat, s->sat_step, s->steps_done, s->dtr, s->dtype, adaptive ? 1 : 0,
                           s->B, s->Bp, s->stop);
        HIP_TRY(hipGetLastError());
    } else {
        if (s->t_base + p->max_steps > INT_MAX - 1)
            return fail(ODESAT_EINVAL, "continued run exceeds 2^31-2 steps");
        if (p->stop == ODESAT_STOP_ANY) {  // a run that already stopped (simulate_inter broke) stays stopped
            int32_t h_stop = INT_MAX;
            if ((rc = read_stop(s, &h_stop))) return rc;
            if (h_stop != INT_MAX) return finish_simulate(s, p, adaptive, 0, first_sat_step, steps_done, dt_out, steps_run);
        }
    }
    const int poll = p->poll_interval > 0 ? p->poll_interval : 32;
    if (s->alg == ODESAT_ALG_ONCHIP && (!adaptive || s->oc_ada))
        return simulate_resident(s, p, adaptive, zeta, tol, poll, first_sat_step, steps_done, dt_out, steps_run);
    if ((s->alg == ODESAT_ALG_RESIDENT || s->alg == ODESAT_ALG_ONCHIP) && (!adaptive || s->res_ada))
        return simulate_resident(s, p, adaptive, zeta, tol, poll, first_sat_step, steps_done, dt_out, steps_run);
    // Schedule: replicas are independent, so with STOP_EACH / STOP_NONE the batch may be stepped
    // chunk by chunk (all steps of one chunk, then the next).  STOP_ANY needs lock-step.  FUSED has
    // no per-chunk buffer: its chunk is the whole batch unless CHUNK_MAJOR is forced.
    const int chunk = s->alg == ODESAT_ALG_TWOPASS || s->schedule == ODESAT_SCHED_CHUNK_MAJOR ? s->chunk_groups : s->G;
    const bool chunk_major = p->stop != ODESAT_STOP_ANY &&
                             (s->schedule == ODESAT_SCHED_CHUNK_MAJOR ||
                              (s->schedule == ODESAT_SCHED_AUTO && s->G > chunk));
    const int span = chunk_major ? chunk : s->G;
    const int64_t base = s->t_base;
    int64_t t_run = 0;
    for (int gA = 0; gA < s->G; gA += span) {
        const int gB = std::min(s->G, gA + span);
        const int64_t r0 = (int64_t)gA * s->W, r1 = std::min<int64_t>((int64_t)gB * s->W, s->B);
        int64_t t = 0;
        for (; t < p->max_steps; ++t) {
            if ((rc = dispatch_step(s, (int)(base + t), adaptive, p->dt, zeta, tol, p->stop, gA, gB))) return rc;
            if (p->stop != ODESAT_STOP_NONE && (t + 1) % poll == 0 && t + 1 < p->max_steps) {
                // poll the stop condition (results are exact regardless: later launches are no-ops)
                HIP_TRY(hipMemcpyAsync(s->h_stop, s->stop, 4, hipMemcpyDeviceToHost, s->stream));
                HIP_TRY(hipMemcpyAsync(s->h_act + r0, s->act + r0, r1 - r0, hipMemcpyDeviceToHost, s->stream));
                HIP_TRY(hipStreamSynchronize(s->stream));
                if (p->stop == ODESAT_STOP_ANY && *s->h_stop != INT_MAX) { ++t; break; }
                if (p->stop == ODESAT_STOP_EACH) {
                    bool live = false;
                    for (int64_t r = r0; r < r1 && !live; ++r) live = s->h_act[r] != 0;
                    if (!live) { ++t; break; }
                }
            }
        }
        t_run = std::max(t_run, t);
    }
    return finish_simulate(s, p, adaptive, t_run, first_sat_step, steps_done, dt_out, steps_run);
}

extern "C" int odesat_simulate(odesat_solver *s, const odesat_params *p, int64_t *first_sat_step,
                               int64_t *steps_done, double *dt_out, int64_t *steps_run) {
    return simulate_impl(s, p, false, first_sat_step, steps_done, dt_out, steps_run);
}

extern "C" int odesat_simulate_continue(odesat_solver *s, const odesat_params *p, int64_t *first_sat_step,
                                        int64_t *steps_done, double *dt_out, int64_t *steps_run) {
    return simulate_impl(s, p, true, first_sat_step, steps_done, dt_out, steps_run);
}

// ---- batched evaluate_cnf ----------------------------------------------
namespace {

// cnf.rs:246-264 on every replica's assignment (v > 0, system.rs:238): thread (clause c, replica r),
// replicas fastest so a group's W lanes read one voltage row.  unsat[r] = 1 if some clause fails.
template <typename T>
__global__ void k_evaluate(const T *b0, const T *b1, const uint8_t *par, const int32_t *cptr, const int32_t *lits,
                           int64_t n, int64_t m, int W, int64_t B, uint32_t *unsat) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (size_t)m * (size_t)B) return;
    const int64_t r = (int64_t)(tid % (size_t)B), c = (int64_t)(tid / (size_t)B);
    const int64_t g = r / W;
    const T *v = (par[g] ? b1 : b0) + (size_t)g * n * W + (r % W);
    bool sat = false;
    for (int32_t k = cptr[c]; k < cptr[c + 1]; ++k) {
        const int32_t l = lits[k];
        sat = sat || ((v[(size_t)(l >> 1) * W] > (T)0) != ((l & 1) != 0));
    }
    if (!sat) unsat[r] = 1u;
}

// the lowest replica whose assignment satisfies the formula (main.rs:302-307), -1 if none
__global__ void k_first_satisfied(const uint32_t *unsat, int64_t B, int64_t *first) {
    __shared__ int64_t best[256];
    int64_t b = INT64_MAX;
    for (int64_t r = threadIdx.x; r < B; r += blockDim.x)
        if (!unsat[r]) {
            b = r;
            break;
        }
    best[threadIdx.x] = b;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) best[threadIdx.x] = min(best[threadIdx.x], best[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) *first = best[0] == INT64_MAX ? -1 : best[0];
}

template <typename T> int evaluate_t(odesat_solver *s, uint32_t *flags, int64_t *first) {
    HIP_TRY(hipMemsetAsync(flags, 0, (size_t)s->B * 4, s->stream));
    const size_t total = (size_t)s->m * (size_t)s->B;
    if (total) {
        const int threads = 256;
        hipLaunchKernelGGL((k_evaluate<T>), dim3((unsigned)((total + threads - 1) / threads)), dim3(threads), 0,
                           s->stream, (const T *)s->v[0], (const T *)s->v[1], s->par, s->cptr, s->lits, s->n, s->m,
                           s->W, s->B, flags);
        HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_first_satisfied, dim3(1), dim3(256), 0, s->stream, flags, s->B, first);
    HIP_TRY(hipGetLastError());
    return ODESAT_OK;
}

}  // namespace

extern "C" int odesat_evaluate(odesat_solver *s, uint8_t *satisfied, int64_t *first_satisfied) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    uint32_t *flags = nullptr;
    int64_t *first = nullptr;
    // B flags, padded to an 8-byte boundary, then the first-satisfied index
    const int64_t padded = (s->B + 1) & ~int64_t(1);
    HIP_TRY(hipMalloc(&flags, (size_t)padded * 4 + 8));
    first = reinterpret_cast<int64_t *>(flags + padded);
    rc = s->dtype == ODESAT_F64 ? evaluate_t<double>(s, flags, first) : evaluate_t<float>(s, flags, first);
    std::vector<uint32_t> u;
    int64_t f = -1;
    hipError_t e = hipSuccess;
    if (!rc) {
        if (satisfied) {
            u.resize((size_t)s->B);
            e = hipMemcpyAsync(u.data(), flags, (size_t)s->B * 4, hipMemcpyDeviceToHost, s->stream);
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&f, first, 8, hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    }
    (void)hipFree(flags);
    if (rc) return rc;
    HIP_TRY(e);
    if (satisfied)
        for (int64_t r = 0; r < s->B; ++r) satisfied[r] = u[(size_t)r] ? 0 : 1;
    if (first_satisfied) *first_satisfied = f;
    return ODESAT_OK;
}

// ---- checkpoint / rollback ------------------------------------------------------------------
static int checkpoint_copy(odesat_solver *s, bool to_ck) {
    const int threads = 256, blocks = 2048;
    const int64_t vw = (int64_t)s->n * s->W * (int64_t)s->tsize / 4, cw = 2 * (int64_t)s->m * s->W * (int64_t)s->tsize / 4;
    auto cp = [&](void *dst, const void *src, size_t bytes) {
        return hipMemcpyAsync(to_ck ? dst : const_cast<void *>(src), to_ck ? src : dst, bytes, hipMemcpyDeviceToDevice,
                              s->stream);
    };
    if (!to_ck) HIP_TRY(cp(s->ck_par, s->par, s->G));  // the groups' current buffers first
    hipLaunchKernelGGL(k_group_copy, dim3(blocks), dim3(threads), 0, s->stream, (uint32_t *)s->ck_v, (uint32_t *)s->v[0],
                       (uint32_t *)s->v[1], s->par, vw, s->G, to_ck ? 1 : 0);
    HIP_TRY(hipGetLastError());
    if (cw > 0) {
        hipLaunchKernelGGL(k_group_copy, dim3(blocks), dim3(threads), 0, s->stream, (uint32_t *)s->ck_c,
                           (uint32_t *)s->c[0], (uint32_t *)s->c[1], s->par, cw, s->G, to_ck ? 1 : 0);
        HIP_TRY(hipGetLastError());
    }
    if (to_ck) HIP_TRY(cp(s->ck_par, s->par, s->G));
    HIP_TRY(cp(s->ck_act, s->act, s->Bp));
    HIP_TRY(cp(s->ck_sat, s->sat_step, s->Bp * 8));
    HIP_TRY(cp(s->ck_done, s->steps_done, s->Bp * 8));
    HIP_TRY(cp(s->ck_dt, s->dtr, s->Bp * s->tsize));
    HIP_TRY(cp(s->ck_stop, s->stop, 4));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ODESAT_OK;
}

extern "C" int odesat_checkpoint(odesat_solver *s) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (!s->ck_v) {
        if ((rc = dmalloc(s, &s->ck_v, state_elems(s, s->n) * s->tsize)) ||
            (rc = dmalloc(s, &s->ck_c, 2 * state_elems(s, s->m) * s->tsize)) ||
            (rc = dmalloc(s, &s->ck_dt, s->Bp * s->tsize)) || (rc = dmalloc(s, (void **)&s->ck_par, s->G)) ||
            (rc = dmalloc(s, (void **)&s->ck_act, s->Bp)) || (rc = dmalloc(s, (void **)&s->ck_sat, s->Bp * 8)) ||
            (rc = dmalloc(s, (void **)&s->ck_done, s->Bp * 8)) || (rc = dmalloc(s, (void **)&s->ck_stop, 16)))
            return rc;
    }
    if ((rc = checkpoint_copy(s, true))) return rc;
    s->ck_t_base = s->t_base;
    s->ck_in_range = s->in_range;
    return ODESAT_OK;
}

extern "C" int odesat_rollback(odesat_solver *s) {
    int rc;
    if ((rc = check_solver(s))) return rc;
    if (s->ck_t_base < 0) return fail(ODESAT_ESTATE, "odesat_rollback: no checkpoint");
    if ((rc = checkpoint_copy(s, false))) return rc;
    s->t_base = s->ck_t_base;
    s->in_range = s->ck_in_range;
    return ODESAT_OK;
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
    // events for the launches to come, created (and recorded once) here rather than inside a call
    if (s->profile) {
        while (s->pool.size() < 8) {
            hipEvent_t e = nullptr;
            HIP_TRY(hipEventCreate(&e));
            s->pool.push_back(e);
        }
        for (hipEvent_t e : s->pool) HIP_TRY(hipEventRecord(e, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
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
    // Algorithmic bytes per step of the dominant kernel over the whole batch, in dtype.
    // FUSED k_step: v, xs, xl each read and written once (2n + 4m per replica).
    // TWOPASS k_clause: v gathered once (n), xs / xl read + written (4m).
    // RESIDENT / ONCHIP: SURVEY.md §8d's compulsory state traffic, v, xs, xl each read and written
    // once per replica-step (2n + 4m) -- ONCHIP moves it on chip, not through HBM.
    if (!s) return -1;
    const int64_t per = s->alg == ODESAT_ALG_TWOPASS ? s->n + 4 * s->m : 2 * s->n + 4 * s->m;
    return (int64_t)s->B * per * (int64_t)s->tsize;
}

// Test hook (not part of include/odesat.h): the wave-paired tiling the solver would build for a
// 0-based formula (pair_tiles, offset off): tile and wave of every clause, and the tile count.
// tests/test_tiling.py checks its invariants on the CPU -- a race it let through would not show
// reliably on the GPU.
extern "C" int odesat_debug_pair_tiles(const odesat_cnf *f, int off, int32_t *tile_of, int8_t *wave_of,
                                       int32_t *ntiles) {
    if (!f || !tile_of || !wave_of || !ntiles || (off != 0 && off != 1))
        return fail(ODESAT_EINVAL, "odesat_debug_pair_tiles: bad argument");
    const int64_t n = f->varnum;
    for (int64_t v : f->var)
        if (v < 0 || v >= n) return fail(ODESAT_EINVAL, "odesat_debug_pair_tiles: variables must be 0-based below varnum");
    std::vector<int32_t> t, fill;
    std::vector<int8_t> w;
    pair_tiles(f, n, off, t, w, fill);
    std::copy(t.begin(), t.end(), tile_of);
    std::copy(w.begin(), w.end(), wave_of);
    *ntiles = (int32_t)fill.size();
    return ODESAT_OK;
}

#ifdef RES_STAMPS
// Diagnostic build only: the per-workgroup k_resident stamps of the last launch (4096 x 64, resident.hpp).
extern "C" int odesat_res_stamps(unsigned long long *out, int count) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(odk::g_res_stamps), sizeof(unsigned long long) * (size_t)count, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int odesat_res_clk(unsigned long long *out, int count) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(odk::g_res_clk), sizeof(unsigned long long) * (size_t)count, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
