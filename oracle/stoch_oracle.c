/*
 * stoch_oracle.c -- CPU restatement of the reference's discrete stochastic search (src/stoch.rs).
 *
 * TEST INFRASTRUCTURE ONLY (see odesat_oracle.h): the checker for odesat_amd/csrc/stoch.hip.
 * Parity status: integer arithmetic followed line by line from stoch.rs; the reference's
 * thread_rng draw is replaced by the counter RNG below (the product's declared deviation), so the
 * GPU must match this bit for bit.  Unpinned by reference-executed outputs (no Rust toolchain).
 */
#include <stdint.h>
#include <string.h>

#include "odesat_oracle.h"

static uint64_t st_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* counter RNG keyed on (seed, replica, step, var) -- the same function as stoch.hip */
uint64_t oc_stoch_hash(uint64_t seed, uint64_t replica, uint64_t step, uint64_t var) {
    uint64_t h = st_mix64(seed + 0x9E3779B97F4A7C15ULL);
    h = st_mix64(h ^ (replica * 0xD1B54A32D192ED03ULL + 0x632BE59BD9B4E019ULL));
    h = st_mix64(h ^ (step * 0xA24BAED4963EE407ULL + 0x9FB21C651E98DF25ULL));
    h = st_mix64(h ^ (var * 0x8CB92BA72F3D8DD7ULL + 0x9E3779B97F4A7C15ULL));
    return h;
}

/* rng.gen_range(1..=tot) (stoch.rs:70), restated as 1 + floor(h * tot / 2^64) */
static uint64_t st_draw(uint64_t h, uint64_t tot) {
    return 1 + (uint64_t)(((unsigned __int128)h * tot) >> 64);
}

/* stoch.rs:20-25 */
static int st_evaluate_clause(const oc_formula *f, int64_t c, const uint8_t *v) {
    for (int64_t s = f->clause_ptr[c]; s < f->clause_ptr[c + 1]; ++s)
        if ((v[f->var[s]] != 0) ^ (f->neg[s] != 0)) return 1;
    return 0;
}

/* stoch.rs:26-81.  slab[var] = (uns, tot) in tot[]/uns[] (n each, caller scratch).  Returns
 * all_clauses_satisfied, or -1 where the reference panics (gen_range(1..=0): a variable in no
 * clause). */
int oc_stoch_step(const oc_formula *f, uint8_t *v, uint64_t *xl, uint64_t seed, uint64_t replica, uint64_t step,
                  uint64_t *tot, uint64_t *uns) {
    int all = 1;
    memset(tot, 0, (size_t)f->varnum * sizeof(uint64_t));  /* :33-37 slab.clear(); insert((0, 0)) */
    memset(uns, 0, (size_t)f->varnum * sizeof(uint64_t));
    for (int64_t c = 0; c < f->nclauses; ++c) {             /* :40-66 */
        const int sat = st_evaluate_clause(f, c, v);
        uint64_t x = xl[c];
        if (sat) {
            const uint64_t y = x == 0 ? 0 : x - 1;           /* saturating_sub(1) */
            x = y > 1 ? y : 1;                               /* .max(1) */
        } else {
            x = x > UINT64_MAX - 20 ? UINT64_MAX : x + 20;   /* saturating_add(ALPHA) */
        }
        xl[c] = x;
        for (int64_t s = f->clause_ptr[c]; s < f->clause_ptr[c + 1]; ++s) {
            tot[f->var[s]] += x;
            if (!sat) uns[f->var[s]] += x;
        }
        if (!sat) all = 0;
    }
    for (int64_t i = 0; i < f->varnum; ++i) {                /* :69-76 */
        if (tot[i] == 0) return -1;
        const uint64_t r = st_draw(oc_stoch_hash(seed, replica, step, (uint64_t)i), tot[i]);
        if (r <= uns[i]) v[i] = !v[i];
    }
    return all;
}

/* stoch.rs:83-110 search, continuing from the caller's (v, xl) (search() itself starts from
 * v = false, xl = 1); steps > 0 bounds the loop.  Returns steps taken (the breaking step included),
 * *sat = 1 if the loop broke on an all-satisfied step, -1 on the panic case. */
int64_t oc_stoch_search(const oc_formula *f, uint8_t *v, uint64_t *xl, uint64_t seed, uint64_t replica, int64_t steps,
                        uint64_t *scratch, int *sat) {
    *sat = 0;
    for (int64_t k = 0; k < steps; ++k) {
        const int r = oc_stoch_step(f, v, xl, seed, replica, (uint64_t)k, scratch, scratch + f->varnum);
        if (r < 0) return -1;
        if (r) {
            *sat = 1;
            return k + 1;
        }
    }
    return steps;
}
