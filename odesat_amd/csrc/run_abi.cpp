// run_abi.cpp -- the one-call boundary of SURVEY.md §8(b): odesat_create / odesat_run /
// odesat_destroy, the C ABI a Rust `extern "C"` block binds in place of simulate / simulate_inter
// (system.rs:156-163, :241-248).  A thin host layer over the solver entry points of
// include/odesat.h: the context owns the normalised formula and a solver sized for the last batch
// it ran; odesat_run copies the caller's replica-innermost f32 states in, integrates, and copies
// the states and per-replica bookkeeping out.  Host buffers stay the caller's; device memory is the
// library's.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"

using odesat::fail;

struct odesat_ctx {
    int device = 0;
    int64_t n = 0, m = 0;
    odesat_cnf *formula = nullptr;
    odesat_solver *solver = nullptr;
    int64_t batch = 0;
};

namespace {

void put_err(char *err, size_t errlen, const char *msg) {
    if (err && errlen) std::snprintf(err, errlen, "%s", msg ? msg : "");
}

// [n][B] f32 (replica-innermost) <-> [B][n] f64 (the solver's replica-major exchange format)
void to_replica_major(const float *src, int64_t items, int64_t B, std::vector<double> &dst) {
    dst.resize((size_t)(items * B));
    for (int64_t i = 0; i < items; ++i)
        for (int64_t b = 0; b < B; ++b) dst[(size_t)(b * items + i)] = (double)src[i * B + b];
}

// steps per bounded call of an unbounded run (the RUN_CHUNK knob overrides: tests force several calls)
int64_t chunk_steps() {
    const int64_t c = odesat::xp_get("RUN_CHUNK", 0);
    return c > 0 ? c : (int64_t)1 << 16;
}

void to_replica_inner(const std::vector<double> &src, int64_t items, int64_t B, float *dst) {
    for (int64_t i = 0; i < items; ++i)
        for (int64_t b = 0; b < B; ++b) dst[i * B + b] = (float)src[(size_t)(b * items + i)];
}

}  // namespace

extern "C" odesat_ctx *odesat_create(int device, int32_t n, int32_t m, const int32_t *clause_ptr, const int32_t *lits,
                                     char *err, size_t errlen) {
    put_err(err, errlen, "");
    if (n <= 0 || m < 0 || (m > 0 && !clause_ptr) || (clause_ptr && clause_ptr[0] != 0)) {
        fail(ODESAT_EINVAL, "odesat_create: bad formula arguments");
        put_err(err, errlen, odesat_last_error());
        return nullptr;
    }
    const int64_t L = m > 0 ? clause_ptr[m] : 0;
    std::vector<int64_t> cp((size_t)m + 1, 0), var((size_t)std::max<int64_t>(L, 1));
    std::vector<uint8_t> neg((size_t)std::max<int64_t>(L, 1));
    for (int32_t c = 0; c < m; ++c) {
        cp[c + 1] = clause_ptr[c + 1];
        if (cp[c + 1] < cp[c]) {
            fail(ODESAT_EINVAL, "odesat_create: clause_ptr must be non-decreasing");
            put_err(err, errlen, odesat_last_error());
            return nullptr;
        }
    }
    for (int64_t s = 0; s < L; ++s) {
        var[s] = lits[s] >> 1;
        neg[s] = (uint8_t)(lits[s] & 1);
        if (var[s] < 0 || var[s] >= n) {
            fail(ODESAT_EINVAL, "odesat_create: literal variable out of [0, n)");
            put_err(err, errlen, odesat_last_error());
            return nullptr;
        }
    }
    auto *x = new (std::nothrow) odesat_ctx();
    if (!x) {
        fail(ODESAT_ENOMEM, "odesat_create: out of memory");
        put_err(err, errlen, odesat_last_error());
        return nullptr;
    }
    x->device = device;
    x->n = n;
    x->m = m;
    if (odesat_cnf_from_arrays(n, m, cp.data(), L ? var.data() : nullptr, L ? neg.data() : nullptr, &x->formula)) {
        put_err(err, errlen, odesat_last_error());
        delete x;
        return nullptr;
    }
    int ndev = 0;
    if (odesat_device_count(&ndev) || device < 0 || device >= ndev) {
        fail(ODESAT_EDEVICE, "odesat_create: no such HIP device (odesat_amd has no CPU fallback)");
        put_err(err, errlen, odesat_last_error());
        odesat_cnf_free(x->formula);
        delete x;
        return nullptr;
    }
    return x;
}

extern "C" void odesat_destroy(odesat_ctx *x) {
    if (!x) return;
    if (x->solver) odesat_solver_destroy(x->solver);
    odesat_cnf_free(x->formula);
    delete x;
}

extern "C" int odesat_run(odesat_ctx *x, const odesat_params *p, int32_t B, const float *v0, const float *xs0,
                          const float *xl0, float *v_out, float *xs_out, float *xl_out, int64_t *first_sat_step,
                          int64_t *steps_done) {
    if (!x || !p) return fail(ODESAT_EINVAL, "odesat_run: null argument");
    if (B <= 0 || !v0 || (x->m > 0 && (!xs0 || !xl0))) return fail(ODESAT_EINVAL, "odesat_run: bad batch or state");
    if (p->dt_policy == ODESAT_DT_SHARED_SERIAL)
        return fail(ODESAT_EINVAL, "odesat_run: ODESAT_DT_SHARED_SERIAL is the serial CPU policy (system.rs:314-326); "
                                   "the device runs every replica with its own dt");
    if (p->max_steps < 0 || (p->max_steps == 0 && p->stop == ODESAT_STOP_NONE))
        return fail(ODESAT_EINVAL, "odesat_run: max_steps must be >= 0 (0 = until the stop condition holds)");
    int rc;
    if (!x->solver || x->batch != B) {
        if (x->solver) odesat_solver_destroy(x->solver);
        x->solver = nullptr;
        if ((rc = odesat_solver_create(x->device, x->formula, B, ODESAT_F32, &x->solver))) return rc;
        x->batch = B;
    }
    std::vector<double> hv, hxs, hxl;
    to_replica_major(v0, x->n, B, hv);
    to_replica_major(xs0, x->m, B, hxs);
    to_replica_major(xl0, x->m, B, hxl);
    if ((rc = odesat_set_state(x->solver, 0, B, hv.data(), x->m ? hxs.data() : nullptr, x->m ? hxl.data() : nullptr)))
        return rc;
    std::vector<int64_t> sat((size_t)B, -1), done((size_t)B, 0);
    odesat_params q = *p;
    if (p->max_steps > 0) {
        if ((rc = odesat_simulate(x->solver, &q, sat.data(), done.data(), nullptr, nullptr))) return rc;
    } else {  // None (system.rs:198, :296): until every replica (EACH) / some replica (ANY) is allsat,
              // one run in bounded calls (odesat_simulate_continue keeps dt, frozen replicas, step count)
        q.max_steps = chunk_steps();
        if ((rc = odesat_simulate(x->solver, &q, sat.data(), done.data(), nullptr, nullptr))) return rc;
        for (;;) {
            bool any = false, all = true;
            for (int32_t b = 0; b < B; ++b) {
                any = any || sat[b] >= 0;
                all = all && sat[b] >= 0;
            }
            if (p->stop == ODESAT_STOP_ANY ? any : all) break;
            if ((rc = odesat_simulate_continue(x->solver, &q, sat.data(), done.data(), nullptr, nullptr))) return rc;
        }
    }
    std::vector<double> ov((size_t)(x->n * B)), oxs((size_t)(x->m * B)), oxl((size_t)(x->m * B));
    if ((rc = odesat_get_state(x->solver, 0, B, ov.data(), x->m ? oxs.data() : nullptr, x->m ? oxl.data() : nullptr)))
        return rc;
    if (v_out) to_replica_inner(ov, x->n, B, v_out);
    if (xs_out) to_replica_inner(oxs, x->m, B, xs_out);
    if (xl_out) to_replica_inner(oxl, x->m, B, xl_out);
    if (first_sat_step) std::copy(sat.begin(), sat.end(), first_sat_step);
    if (steps_done) std::copy(done.begin(), done.end(), steps_done);
    return ODESAT_OK;
}
