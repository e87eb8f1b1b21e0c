// Host-side fuzz harness for the library's pure C++ parts (the DIMACS loader cnf.cpp, the `solve`
// preprocessing preprocess.cpp, the experiment knobs experiment.cpp), built by
// tests/test_host_sanitizers.py with AddressSanitizer and UndefinedBehaviorSanitizer (host code only:
// GPU sanitizers are not available on the pool).  Every ABI call below must return ODESAT_OK or a
// negative error code without touching memory it does not own.
//   host_fuzz <cases> <seed> [file.cnf ...]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/odesat.h"

namespace {

int fails = 0;
#define CHECK(cond)                                                                     \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            std::fprintf(stderr, "check failed at %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++fails;                                                                    \
        }                                                                               \
    } while (0)

// the whole host pipeline on one parsed formula: export, normalize, evaluate, memories, preprocess,
// the trace and the tri-state evaluation
void pipeline(odesat_cnf *f, std::mt19937_64 &rng) {
    const int64_t n = odesat_cnf_varnum(f), m = odesat_cnf_nclauses(f), L = odesat_cnf_nliterals(f);
    CHECK(m >= 0 && L >= 0);
    std::vector<int64_t> cp((size_t)m + 1), var((size_t)L + 1);
    std::vector<uint8_t> neg((size_t)L + 1);
    CHECK(odesat_cnf_export(f, cp.data(), var.data(), neg.data()) == ODESAT_OK);
    const int64_t maxv = odesat_cnf_max_variable(f);
    odesat_cnf *nf = nullptr;
    std::vector<int64_t> old((size_t)(maxv + 2 > 0 ? maxv + 2 : 1));
    int64_t k = 0;
    if (odesat_cnf_normalize(f, &nf, old.data(), &k) == ODESAT_OK) {
        CHECK(k <= maxv + 1);
        std::vector<double> xs((size_t)m + 1);
        CHECK(odesat_cnf_init_short_term_memory(nf, xs.data()) == ODESAT_OK);
        std::vector<uint8_t> vals((size_t)(k > 0 ? k : 1));
        for (auto &x : vals) x = (uint8_t)(rng() & 1);
        const int r = odesat_cnf_evaluate(nf, vals.data(), k);
        CHECK(r == 0 || r == 1);
        odesat_cnf_free(nf);
    }
    const int64_t nvals = (maxv + 2 > n + 1 ? maxv + 2 : n + 1);
    for (float ratio : {7.0f, 4.2f, 1.0f}) {
        odesat_cnf *red = nullptr;
        odesat_trace *tr = nullptr;
        if (odesat_preprocess(f, ratio, &red, &tr) != ODESAT_OK) continue;
        const int64_t steps = odesat_trace_nsteps(tr);
        for (int64_t i = 0; i < steps; ++i) {
            int32_t kind = -1;
            int64_t v = -1, nc = -1, nl = -1;
            CHECK(odesat_trace_step(tr, i, &kind, &v, &nc, &nl) == ODESAT_OK);
            std::vector<int64_t> scp((size_t)nc + 1), svar((size_t)nl + 1);
            std::vector<uint8_t> sneg((size_t)nl + 1);
            CHECK(odesat_trace_step_clauses(tr, i, scp.data(), svar.data(), sneg.data()) == ODESAT_OK);
        }
        std::vector<uint8_t> tri((size_t)nvals, (uint8_t)ODESAT_UNSET);
        for (auto &x : tri)
            if (rng() % 3 == 0) x = (uint8_t)(rng() & 1);
        const int re = odesat_cnf_evaluate_assign(red, tri.data(), nvals);
        CHECK(re == 0 || re == 1 || re < 0);
        CHECK(odesat_trace_apply(tr, tri.data(), nvals) == ODESAT_OK);
        odesat_trace_free(tr);
        odesat_cnf_free(red);
    }
}

std::string random_dimacs(std::mt19937_64 &rng) {
    const int n = 1 + (int)(rng() % 60), m = (int)(rng() % 200);
    std::string s = "c fuzz\n";
    if (rng() % 4) s += "p cnf " + std::to_string(n) + " " + std::to_string(m) + "\n";
    for (int c = 0; c < m; ++c) {
        const int k = (int)(rng() % 6);  // empty clauses and duplicate literals included
        for (int j = 0; j < k; ++j) {
            const int v = 1 + (int)(rng() % (rng() % 8 == 0 ? 100000 : n));
            s += std::to_string(rng() & 1 ? -v : v) + " ";
        }
        s += "0\n";
    }
    return s;
}

std::string mutate(std::string s, std::mt19937_64 &rng) {
    static const char junk[] = "0123456789- \n\tpcnfx%\r+.e";
    const int edits = 1 + (int)(rng() % 4);
    for (int e = 0; e < edits && !s.empty(); ++e) {
        const size_t at = (size_t)(rng() % s.size());
        switch (rng() % 3) {
            case 0: s[at] = junk[rng() % (sizeof(junk) - 1)]; break;
            case 1: s.erase(at, 1 + rng() % 3); break;
            default: s.insert(at, 1, junk[rng() % (sizeof(junk) - 1)]); break;
        }
    }
    return s;
}

void one_text(const std::string &text, std::mt19937_64 &rng, int64_t &parsed) {
    odesat_cnf *f = nullptr;
    const int rc = odesat_cnf_parse(text.data(), text.size(), &f);
    CHECK(rc == ODESAT_OK || rc < 0);
    if (rc != ODESAT_OK) {
        CHECK(std::strlen(odesat_last_error()) > 0);
        return;
    }
    ++parsed;
    pipeline(f, rng);
    odesat_cnf_free(f);
}

}  // namespace

int main(int argc, char **argv) {
    const int cases = argc > 1 ? std::atoi(argv[1]) : 300;
    std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1);
    int64_t parsed = 0;
    for (int i = 3; i < argc; ++i) {  // the reference's own fixtures, as they are and mutated
        FILE *fh = std::fopen(argv[i], "rb");
        if (!fh) return 2;
        std::string text;
        char buf[4096];
        size_t got;
        while ((got = std::fread(buf, 1, sizeof buf, fh)) > 0) text.append(buf, got);
        std::fclose(fh);
        one_text(text, rng, parsed);
        for (int j = 0; j < 20; ++j) one_text(mutate(text, rng), rng, parsed);
    }
    for (int i = 0; i < cases; ++i) {
        const std::string t = random_dimacs(rng);
        one_text(t, rng, parsed);
        one_text(mutate(t, rng), rng, parsed);
    }
    // the knob registry: unknown keys fail, known keys set / get / clear
    int64_t v = 0;
    CHECK(odesat_set_experiment("NOT_A_KNOB", 1) < 0);
    CHECK(odesat_set_experiment(nullptr, 1) < 0);
    const char *name = nullptr;
    for (int i = 0; odesat_experiment_knob(i, &name) == ODESAT_OK; ++i) {
        CHECK(odesat_set_experiment(name, 3) == ODESAT_OK && odesat_get_experiment(name, &v) == ODESAT_OK && v == 3);
    }
    odesat_clear_experiments();
    std::printf("host_fuzz: %d cases, %lld parsed, %d failed checks\n", cases, (long long)parsed, fails);
    return fails == 0 ? 0 : 1;
}
