// cnf.cpp -- DIMACS loader and formula helpers: the C++ replacement of the reference's
// src/cnf.rs:53-315 on the integrator's path (parse, normalise, evaluate, initial memories).
#include <algorithm>
#include <cctype>
#include <climits>
#include <cstring>
#include <string>

#include "../../include/odesat.h"
#include "cnf.hpp"

namespace odesat {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

}  // namespace odesat

using odesat::fail;

extern "C" const char *odesat_last_error(void) { return odesat::g_err.c_str(); }

namespace {

inline bool is_ws(char c) {
    // Rust split_whitespace uses Unicode White_Space; DIMACS files are ASCII.
    return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

// Rust `str::parse::<i32>()`: optional sign, decimal digits, range checked.
bool parse_i32(const char *b, const char *e, int64_t *out) {
    if (b == e) return false;
    bool negative = false;
    if (*b == '+' || *b == '-') {
        negative = *b == '-';
        ++b;
        if (b == e) return false;
    }
    int64_t x = 0;
    for (; b < e; ++b) {
        if (*b < '0' || *b > '9') return false;
        x = x * 10 + (*b - '0');
        if (x > (int64_t)INT_MAX + 1) return false;
    }
    if (negative) x = -x;
    if (x < INT_MIN || x > INT_MAX) return false;
    *out = x;
    return true;
}

// Rust `str::parse::<usize>()`: optional '+', decimal digits.
bool parse_usize(const char *b, const char *e, int64_t *out) {
    if (b == e) return false;
    if (*b == '+') {
        ++b;
        if (b == e) return false;
    }
    int64_t x = 0;
    for (; b < e; ++b) {
        if (*b < '0' || *b > '9') return false;
        if (x > (INT64_MAX - 9) / 10) return false;
        x = x * 10 + (*b - '0');
    }
    *out = x;
    return true;
}

}  // namespace

// cnf.rs:138-172
extern "C" int odesat_cnf_parse(const char *text, size_t len, odesat_cnf **out) {
    if (!out || (!text && len)) return fail(ODESAT_EINVAL, "odesat_cnf_parse: null argument");
    *out = nullptr;
    auto *f = new (std::nothrow) odesat_cnf();
    if (!f) return fail(ODESAT_ENOMEM, "odesat_cnf_parse: out of memory");
    f->clause_ptr.push_back(0);
    bool have_varnum = false;
    int64_t lineno = 0;
    size_t pos = 0;
    // str::lines(): split at '\n', strip one '\r' before it, no empty line after a final '\n'
    while (pos < len) {
        size_t nl = pos;
        while (nl < len && text[nl] != '\n') ++nl;
        const bool terminated = nl < len;
        const char *b = text + pos;
        const char *e = text + nl;
        if (terminated && e > b && e[-1] == '\r') --e;
        pos = terminated ? nl + 1 : nl;
        ++lineno;
        if (e > b && *b == 'c') continue;  // :143
        if (e - b >= 5 && std::memcmp(b, "p cnf", 5) == 0) {  // :146-153
            const char *p = b;
            int tok = 0;
            bool ok = false;
            while (p < e) {
                while (p < e && is_ws(*p)) ++p;
                if (p >= e) break;
                const char *q = p;
                while (q < e && !is_ws(*q)) ++q;
                if (tok == 2) {
                    int64_t vn;
                    if (!parse_usize(p, q, &vn)) break;
                    f->varnum = vn;
                    ok = true;
                    break;
                }
                ++tok;
                p = q;
            }
            if (!ok) {
                delete f;
                return fail(ODESAT_EINVAL, "line " + std::to_string(lineno) +
                                               ": malformed problem line (cnf.rs:151 would panic)");
            }
            have_varnum = true;
            continue;
        }
        // :156-167 clause line: tokens up to "0"
        const char *p = b;
        while (p < e) {
            while (p < e && is_ws(*p)) ++p;
            if (p >= e) break;
            const char *q = p;
            while (q < e && !is_ws(*q)) ++q;
            if (q - p == 1 && *p == '0') break;
            int64_t x;
            if (!parse_i32(p, q, &x)) {
                delete f;
                return fail(ODESAT_EINVAL, "line " + std::to_string(lineno) + ": bad literal '" +
                                               std::string(p, q) + "' (cnf.rs:160 would panic)");
            }
            f->var.push_back(x < 0 ? -x : x);
            f->neg.push_back(x < 0 ? 1 : 0);
            p = q;
        }
        f->clause_ptr.push_back((int64_t)f->var.size());
    }
    if (!have_varnum) {  // CNFFormula::new(.., None): number of distinct variables
        std::vector<int64_t> vs(f->var);
        std::sort(vs.begin(), vs.end());
        f->varnum = (int64_t)(std::unique(vs.begin(), vs.end()) - vs.begin());
    }
    *out = f;
    return ODESAT_OK;
}

extern "C" int odesat_cnf_from_arrays(int64_t varnum, int64_t nclauses, const int64_t *clause_ptr,
                                      const int64_t *var, const uint8_t *neg, odesat_cnf **out) {
    if (!out || nclauses < 0 || !clause_ptr) return fail(ODESAT_EINVAL, "odesat_cnf_from_arrays: bad argument");
    *out = nullptr;
    if (clause_ptr[0] != 0) return fail(ODESAT_EINVAL, "clause_ptr[0] must be 0");
    for (int64_t c = 0; c < nclauses; ++c)
        if (clause_ptr[c + 1] < clause_ptr[c]) return fail(ODESAT_EINVAL, "clause_ptr not monotone");
    const int64_t L = clause_ptr[nclauses];
    if (L > 0 && (!var || !neg)) return fail(ODESAT_EINVAL, "odesat_cnf_from_arrays: null literal arrays");
    auto *f = new (std::nothrow) odesat_cnf();
    if (!f) return fail(ODESAT_ENOMEM, "out of memory");
    f->clause_ptr.assign(clause_ptr, clause_ptr + nclauses + 1);
    f->var.assign(var, var + L);
    f->neg.resize(L);
    for (int64_t s = 0; s < L; ++s) {
        if (var[s] < 0) {
            delete f;
            return fail(ODESAT_EINVAL, "negative variable index");
        }
        f->neg[s] = neg[s] ? 1 : 0;
    }
    if (varnum < 0) {
        std::vector<int64_t> vs(f->var);
        std::sort(vs.begin(), vs.end());
        varnum = (int64_t)(std::unique(vs.begin(), vs.end()) - vs.begin());
    }
    f->varnum = varnum;
    *out = f;
    return ODESAT_OK;
}

extern "C" void odesat_cnf_free(odesat_cnf *cnf) { delete cnf; }
extern "C" int64_t odesat_cnf_varnum(const odesat_cnf *cnf) { return cnf ? cnf->varnum : -1; }
extern "C" int64_t odesat_cnf_nclauses(const odesat_cnf *cnf) { return cnf ? cnf->nclauses() : -1; }
extern "C" int64_t odesat_cnf_nliterals(const odesat_cnf *cnf) { return cnf ? cnf->nliterals() : -1; }

extern "C" int odesat_cnf_export(const odesat_cnf *cnf, int64_t *clause_ptr, int64_t *var, uint8_t *neg) {
    if (!cnf) return fail(ODESAT_EINVAL, "odesat_cnf_export: null formula");
    if (clause_ptr) std::copy(cnf->clause_ptr.begin(), cnf->clause_ptr.end(), clause_ptr);
    if (var) std::copy(cnf->var.begin(), cnf->var.end(), var);
    if (neg) std::copy(cnf->neg.begin(), cnf->neg.end(), neg);
    return ODESAT_OK;
}

// cnf.rs:206-219 (+ apply_variable_mapping :174-199), ascending renaming.
extern "C" int odesat_cnf_normalize(const odesat_cnf *cnf, odesat_cnf **out, int64_t *old_names,
                                    int64_t *k_out) {
    if (!cnf || !out) return fail(ODESAT_EINVAL, "odesat_cnf_normalize: null argument");
    *out = nullptr;
    std::vector<int64_t> names(cnf->var);
    std::sort(names.begin(), names.end());
    names.erase(std::unique(names.begin(), names.end()), names.end());
    auto *f = new (std::nothrow) odesat_cnf();
    if (!f) return fail(ODESAT_ENOMEM, "out of memory");
    f->varnum = cnf->varnum;  // :198 keeps the header varnum
    f->clause_ptr = cnf->clause_ptr;
    f->neg = cnf->neg;
    f->var.resize(cnf->var.size());
    for (size_t s = 0; s < cnf->var.size(); ++s)
        f->var[s] = std::lower_bound(names.begin(), names.end(), cnf->var[s]) - names.begin();
    if (old_names) std::copy(names.begin(), names.end(), old_names);
    if (k_out) *k_out = (int64_t)names.size();
    *out = f;
    return ODESAT_OK;
}

// cnf.rs:246-264
extern "C" int odesat_cnf_evaluate(const odesat_cnf *cnf, const uint8_t *values, int64_t nvalues) {
    if (!cnf || (nvalues > 0 && !values)) return fail(ODESAT_EINVAL, "odesat_cnf_evaluate: null argument");
    const int64_t m = cnf->nclauses();
    for (int64_t c = 0; c < m; ++c) {
        bool ok = false;
        for (int64_t s = cnf->clause_ptr[c]; s < cnf->clause_ptr[c + 1]; ++s) {
            const int64_t v = cnf->var[s];
            const bool val = v < nvalues ? values[v] != 0 : false;
            ok = ok || (cnf->neg[s] ? !val : val);
        }
        if (!ok) return 0;
    }
    return 1;
}

// system.rs:361-372
extern "C" int odesat_cnf_init_short_term_memory(const odesat_cnf *cnf, double *xs) {
    if (!cnf || !xs) return fail(ODESAT_EINVAL, "odesat_cnf_init_short_term_memory: null argument");
    const int64_t m = cnf->nclauses();
    for (int64_t c = 0; c < m; ++c) {
        bool anyneg = false;
        for (int64_t s = cnf->clause_ptr[c]; s < cnf->clause_ptr[c + 1]; ++s) anyneg |= cnf->neg[s] != 0;
        xs[c] = anyneg ? 1.0 : -1.0;
    }
    return ODESAT_OK;
}
