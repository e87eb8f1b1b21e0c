// cnf.hpp -- host-side formula IR shared by the loader (cnf.cpp) and the solver (odesat_hip.hip).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

struct odesat_cnf {
    int64_t varnum = 0;               // cnf.rs:56 (header varnum, or distinct count without header)
    std::vector<int64_t> clause_ptr;  // [m+1]
    std::vector<int64_t> var;         // [L] variable names (file names before normalisation)
    std::vector<uint8_t> neg;         // [L]
    int64_t nclauses() const { return (int64_t)clause_ptr.size() - 1; }
    int64_t nliterals() const { return (int64_t)var.size(); }
};

namespace odesat {

// thread-local error slot behind odesat_last_error()
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

}  // namespace odesat

namespace odesat {

// Experiment knobs (odesat_set_experiment, experiment.cpp): the value set for `key`, or `dflt` when
// the knob is unset.  Read by the host code when it shapes a solver, a partition or a stoch context.
int64_t xp_get(const char *key, int64_t dflt);
inline bool xp_isset(const char *key) { return xp_get(key, -1) >= 0; }

}  // namespace odesat

namespace odesat {

// k_solo_cv's lane and block placement (cv_layout.cpp): for the 3-SAT formula lits[3 m] (var << 1 |
// neg) with term starts vst[n + 1], nl lanes of cpl clause slots and term blocks 0 .. blk_cap - 1:
// slot_clause[nl cpl] (clause or -1), slot_order[3 nl cpl] (the clause's literal index 0..2 at each
// position),
// blk[n + 1] (each variable's block, blk[n] the zero block), and the bank model's LDS cycles of the
// plain and the chosen layout.  false: no layout (the caller keeps k_solo_fast).
bool cv_layout(int64_t n, int64_t m, const int32_t *lits, const int32_t *vst, int nl, int cpl, int tsize, int blk_cap,
               int iters, std::vector<int32_t> &slot_clause, std::vector<int32_t> &slot_order,
               std::vector<int32_t> &blk, int64_t *cost_plain, int64_t *cost_opt);

}  // namespace odesat
