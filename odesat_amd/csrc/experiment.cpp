// experiment.cpp -- the experiment knobs of libodesat_hip.so (include/odesat.h odesat_set_experiment).
// Every knob selects a kernel variant or a layout for A/B measurement or for the parity tests that
// drive every path against the oracle; each variant is bit-identical to the default, which is the
// measured best.  No environment variable is read: a caller sets a knob explicitly,
// and it stays set (process-wide) until it is unset or cleared.
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "../../include/odesat.h"
#include "cnf.hpp"

namespace {

// name -> what it forces (read when the object it shapes is created; RUN_CHUNK by odesat_run)
const char *const KNOBS[] = {
    // solver (odesat_solver_create)
    "GROUP_WIDTH",      // replicas per group 1..64 (a power of two); RESIDENT only where that width admits it
    "PAIR_OFF",         // wave-paired tiles: interval offset 0 or 1 instead of the one needing fewer tiles
    "ONCHIP",           // 0: no k_onchip (RESIDENT on plain tiles)
    "ONCHIP_PAIRS",     // 0: plain tiles (RESIDENT) where k_onchip would run
    "ONCHIP_ADAPTIVE",  // 0: adaptive steps of a k_onchip solver on k_resident
    "ONCHIP_POLL_LIMIT",  // split-barrier polls before a wait gives up and fails the call (test of that path)
    "WAVE",             // 1: k_wave where its LDS fits; 0: the tile kernels
    "WAVE_TEAM",        // k_wave waves per replica: 1, 2, 4, 8 or 16
    "WAVE_FAST",        // 0: k_wave's general arithmetic on in-range states
    "WAVE_TAIL",        // 0: a partial last round of k_wave workgroups stays in the main launch
    "SOLO",             // 1 / 0: k_solo instead of / never instead of k_wave
    "SOLO_LANES",       // k_solo lanes per replica (a multiple of 64)
    "SOLO_FAST",        // 0: k_solo's general arithmetic on in-range states
    "SOLO_CV",          // 0: k_solo_fast instead of k_solo_cv (clause-held voltages) on in-range states
    "CV_ITERS",         // k_solo_cv layout search steps (cv_layout.cpp; 0: the plain layout)
    "RES_NARROW",       // 1 / 0: k_resident with one wave (64-clause tiles) per replica / never
    "RES_FAST",         // 0: k_resident's general arithmetic on 3-SAT
    "RES_RC",           // 0: no register-cached tiles in the f64 k_resident
    "RES_VFG",          // 0: f64 adaptive steps whose clone does not fit in LDS on FUSED, not k_resident
    "RES_PAIRS",        // 0: the f64 k_resident on plain tiles (a barrier after every tile) instead of wave-paired ones
    // partition (odesat_part_create)
    "PART_TERMS",       // term layout: 0 REGION, 1 ELL, 2 SLOT
    "PART_REGIONS",     // REGION: ranges (a multiple of 8, >= 8)
    "PART_K3",          // 0: the generic clause kernel on a 3-SAT slice
    "PART_XCD",         // 1: XCD clause ranges for the clause kernel
    "PART_PACK",        // 0: 16-byte literal records instead of the 8-byte packed ones
    // stoch (odesat_stoch_create)
    "STOCH_WAVE",       // 0: the three-kernel path
    "STOCH_WPW",        // k_stoch_wave replicas per workgroup: 1, 2, 4 or 8
    // odesat_run (one-call boundary)
    "RUN_CHUNK",        // steps per bounded call of an unbounded run
};

std::mutex g_mu;
std::map<std::string, int64_t> g_knobs;

bool known(const char *key) {
    for (const char *k : KNOBS)
        if (std::strcmp(k, key) == 0) return true;
    return false;
}

}  // namespace

namespace odesat {

int64_t xp_get(const char *key, int64_t dflt) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_knobs.find(key);
    return it == g_knobs.end() ? dflt : it->second;
}

}  // namespace odesat

extern "C" int odesat_set_experiment(const char *key, int64_t value) {
    if (!key || !known(key)) return odesat::fail(ODESAT_EINVAL, std::string("unknown experiment knob '") + (key ? key : "(null)") + "'");
    std::lock_guard<std::mutex> lk(g_mu);
    if (value < 0) g_knobs.erase(key);
    else g_knobs[key] = value;
    return ODESAT_OK;
}

extern "C" int odesat_get_experiment(const char *key, int64_t *value) {
    if (!key || !known(key) || !value)
        return odesat::fail(ODESAT_EINVAL, std::string("unknown experiment knob '") + (key ? key : "(null)") + "'");
    *value = odesat::xp_get(key, -1);
    return ODESAT_OK;
}

extern "C" void odesat_clear_experiments(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_knobs.clear();
}

extern "C" int odesat_experiment_knob(int i, const char **name) {
    const int n = (int)(sizeof(KNOBS) / sizeof(KNOBS[0]));
    if (i < 0 || i >= n || !name) return ODESAT_EINVAL;
    *name = KNOBS[i];
    return ODESAT_OK;
}
