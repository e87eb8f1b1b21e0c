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
