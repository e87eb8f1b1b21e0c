// cv_layout.cpp -- where k_solo_cv (wave.hpp) puts each clause and each variable's term block, chosen on
// the host once per solver so that the kernel's 16-byte LDS reads meet few bank conflicts.
//
// k_solo_cv's clause slot reads its three variables' padded term blocks with one ds_read_b128 per 16
// bytes and literal position.  A ds_read_b128 is serviced in 4 lane groups of 16 (the guide's table:
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}), one LDS cycle per
// group when its lanes hit distinct banks, one more per extra distinct address on a busy bank.  A
// block of SOLO_CV_BS slots starts at bank set (b * BS * tsize / 16) mod 16 of the 16 four-bank sets
// (5 b in f64, 3 b in f32), the read q of a block adds q, and a read past the variable's degree goes
// to the one zero block.  So the read (j, q) of a group costs the largest number of distinct
// variables (or the zero block) that share a bank set -- a "colour" c(v) in 0..15 -- among the 16
// lanes' literal-j variables.  PMC on hard.cnf (profiles/r05k): 328 conflict cycles against 748 LDS
// cycles per adaptive step with the plain layout (clause l on lane l, variable v in block v).
//
// The search (simulated annealing, deterministic) moves clauses between lane slots (the lanes past m
// are free slots), reorders a clause's literals (solo_terms is symmetric in them: its mins are exact)
// and recolours variables; blocks are then handed out per colour (the area holds ~22 blocks of each
// colour).  None of this changes a result: the kernel reads each clause's record, memories and terms
// where the layout says.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"
#include "solo_blocks.hpp"

namespace odesat {

namespace {

// the ds_read_b128 lane group (0..3) of lane i of a wave
int b128_group(int i) {
    const int r = i & 31, hi = i >= 32 ? 2 : 0;
    const bool g0 = r < 4 || (r >= 12 && r < 16) || (r >= 20 && r < 28);
    return hi + (g0 ? 0 : 1);
}

struct Search {
    int n, m, nslots, ngroups, nb_reads;        // nb_reads: 16-byte reads per block (NB)
    int per16;                                  // terms per 16 bytes
    std::vector<int32_t> lits;                  // [m][3] var << 1 | neg
    std::vector<int32_t> deg;                   // [n]
    std::vector<int> slot_clause;               // [nslots] clause or -1
    std::vector<int> clause_slot;               // [m]
    std::vector<uint8_t> perm;                  // [m] literal order (index into PERMS)
    std::vector<int> colour;                    // [n + 1] (n: the zero block)
    std::vector<int> group_of;                  // [nslots]
    std::vector<std::vector<int>> group_slots;  // [ngroups]
    std::vector<std::vector<int>> var_clauses;  // [n]
    std::vector<int> gcost;                     // [ngroups]
    static constexpr int PERMS[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};

    int lit(int c, int j) const { return lits[3 * c + PERMS[perm[c]][j]]; }

    mutable std::vector<uint32_t> seen;  // [n + 1] epoch of the last count of each block address
    mutable uint32_t epoch = 0;
    // LDS cycles of the group's 3 NB reads: per read, the most distinct addresses on one bank set
    int group_cost(int gi) const {
        int total = 0;
        const auto &sl = group_slots[gi];
        for (int j = 0; j < 3; ++j)
            for (int q = 0; q < nb_reads; ++q) {
                ++epoch;
                int cnt[16] = {0}, mx = 1;
                for (int s : sl) {
                    const int c = slot_clause[s];
                    int v = n;  // the zero block
                    if (c >= 0) {
                        const int x = lit(c, j) >> 1;
                        if (q * per16 < deg[x]) v = x;
                    }
                    if (seen[v] != epoch) {
                        seen[v] = epoch;
                        mx = std::max(mx, ++cnt[colour[v]]);
                    }
                }
                total += mx;
            }
        return total;
    }
    long total() const {
        long t = 0;
        for (int g : gcost) t += g;
        return t;
    }
};
constexpr int Search::PERMS[6][3];

struct Rng {
    uint64_t s;
    uint64_t next() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    }
    int below(int k) { return (int)(next() % (uint64_t)k); }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

}  // namespace

bool cv_layout(int64_t n, int64_t m, const int32_t *lits, const int32_t *vst, int nl, int cpl, int tsize, int blk_cap,
               int iters, std::vector<int32_t> &slot_clause, std::vector<int32_t> &slot_order,
               std::vector<int32_t> &blk, int64_t *cost_plain, int64_t *cost_opt) {
    const int bs = solo_cv_bs((size_t)tsize);  // the kernel's own block stride (solo_blocks.hpp)
    const int stride = bs * tsize / 16;   // bank sets per block step (odd: every colour reachable)
    Search S;
    S.n = (int)n;
    S.m = (int)m;
    S.nslots = nl * cpl;
    S.per16 = 16 / tsize;
    S.nb_reads = solo_dpad_reads((size_t)tsize);
    S.lits.assign(lits, lits + 3 * m);
    S.deg.resize(n);
    S.var_clauses.assign(n, {});
    for (int64_t i = 0; i < n; ++i) S.deg[i] = vst[i + 1] - vst[i];
    for (int64_t c = 0; c < m; ++c)
        for (int j = 0; j < 3; ++j) S.var_clauses[lits[3 * c + j] >> 1].push_back((int)c);
    // groups: layer k, wave w, b128 group g
    S.ngroups = cpl * ((nl + 63) / 64) * 4;
    S.group_slots.assign(S.ngroups, {});
    S.group_of.resize(S.nslots);
    for (int s = 0; s < S.nslots; ++s) {
        const int k = s / nl, l = s % nl;
        const int gi = (k * ((nl + 63) / 64) + l / 64) * 4 + b128_group(l & 63);
        S.group_of[s] = gi;
        S.group_slots[gi].push_back(s);
    }
    // the plain layout: clause l + k nl on lane l's slot k, literals as given, variable v in block v
    S.slot_clause.assign(S.nslots, -1);
    S.clause_slot.assign(m, -1);
    for (int64_t c = 0; c < m; ++c) {
        S.slot_clause[c] = (int)c;
        S.clause_slot[c] = (int)c;
    }
    S.perm.assign(m, 0);
    S.colour.resize(n + 1);
    S.seen.assign(n + 1, 0);
    for (int64_t v = 0; v <= n; ++v) S.colour[v] = (int)((v * stride) % 16);
    S.gcost.resize(S.ngroups);
    for (int g = 0; g < S.ngroups; ++g) S.gcost[g] = S.group_cost(g);
    const long plain = S.total();
    long cur = plain;
    // colour capacity: blocks 0 .. blk_cap - 1, each colour class (b stride mod 16) about blk_cap / 16
    std::vector<int> cap(16, 0), used(16, 0);
    for (int b = 0; b < blk_cap; ++b) ++cap[(b * stride) % 16];
    for (int64_t v = 0; v <= n; ++v) ++used[S.colour[v]];
    Rng R{0x9E3779B97F4A7C15ull ^ ((uint64_t)n << 32) ^ (uint64_t)m};
    const double T0 = 2.0, T1 = 0.05;
    std::vector<int> touched;
    for (int it = 0; it < iters && cur > (long)S.ngroups * 3 * S.nb_reads; ++it) {
        const double T = T0 * std::pow(T1 / T0, (double)it / iters);
        const int kind = R.below(4);
        touched.clear();
        if (kind <= 1) {  // swap two slots in different groups
            const int a = R.below(S.nslots), b = R.below(S.nslots);
            if (S.group_of[a] == S.group_of[b] || (S.slot_clause[a] < 0 && S.slot_clause[b] < 0)) continue;
            std::swap(S.slot_clause[a], S.slot_clause[b]);
            touched = {S.group_of[a], S.group_of[b]};
            long d = 0;
            int nc[2];
            for (int t = 0; t < 2; ++t) d += (nc[t] = S.group_cost(touched[t])) - S.gcost[touched[t]];
            if (d <= 0 || R.unit() < std::exp(-d / T)) {
                for (int t = 0; t < 2; ++t) S.gcost[touched[t]] = nc[t];
                cur += d;
                for (int s : {a, b})
                    if (S.slot_clause[s] >= 0) S.clause_slot[S.slot_clause[s]] = s;
            } else {
                std::swap(S.slot_clause[a], S.slot_clause[b]);
            }
        } else if (kind == 2) {  // reorder one clause's literals
            const int c = R.below(S.m), old = S.perm[c];
            S.perm[c] = (uint8_t)R.below(6);
            const int gi = S.group_of[S.clause_slot[c]];
            const int nc = S.group_cost(gi);
            const long d = nc - S.gcost[gi];
            if (d <= 0 || R.unit() < std::exp(-d / T)) {
                S.gcost[gi] = nc;
                cur += d;
            } else {
                S.perm[c] = (uint8_t)old;
            }
        } else {  // recolour a variable (or the zero block)
            const int v = R.below(S.n + 1), to = R.below(16), from = S.colour[v];
            if (to == from || used[to] >= cap[to]) continue;
            S.colour[v] = to;
            if (v == S.n) {
                for (int g = 0; g < S.ngroups; ++g) touched.push_back(g);
            } else {
                for (int c : S.var_clauses[v]) touched.push_back(S.group_of[S.clause_slot[c]]);
                std::sort(touched.begin(), touched.end());
                touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
            }
            std::vector<int> nc(touched.size());
            long d = 0;
            for (size_t t = 0; t < touched.size(); ++t) d += (nc[t] = S.group_cost(touched[t])) - S.gcost[touched[t]];
            if (d <= 0 || R.unit() < std::exp(-d / T)) {
                for (size_t t = 0; t < touched.size(); ++t) S.gcost[touched[t]] = nc[t];
                cur += d;
                --used[from];
                ++used[to];
            } else {
                S.colour[v] = from;
            }
        }
    }
    // blocks: per colour, the lowest free block of that colour
    std::vector<std::vector<int>> free_of(16);
    for (int b = blk_cap - 1; b >= 0; --b) free_of[(b * stride) % 16].push_back(b);
    blk.assign(n + 1, 0);
    for (int64_t v = 0; v <= n; ++v) {
        auto &f = free_of[S.colour[v]];
        if (f.empty()) return false;  // (cannot happen: recolouring respects the capacity)
        blk[v] = f.back();
        f.pop_back();
    }
    slot_clause.assign(S.slot_clause.begin(), S.slot_clause.end());
    slot_order.assign((size_t)S.nslots * 3, 0);
    for (int s = 0; s < S.nslots; ++s) {
        const int c = S.slot_clause[s];
        for (int j = 0; j < 3; ++j) slot_order[3 * s + j] = c >= 0 ? Search::PERMS[S.perm[c]][j] : j;
    }
    if (cost_plain) *cost_plain = plain;
    if (cost_opt) *cost_opt = cur;
    return true;
}

}  // namespace odesat

// Test hook (tests/test_cv_layout.py, no device needed): the layout of a 3-SAT formula (lits[3 m] =
// var << 1 | neg, vst[n + 1] the variable-major term starts) for nl lanes and cpl clause slots per
// lane; slot_clause[nl cpl], slot_order[3 nl cpl] (the clause's literal index at each position),
// blk[n + 1] out, and the model's LDS cycles per pass
// of the plain and the chosen layout.
extern "C" int odesat_cv_layout(int64_t n, int64_t m, const int32_t *lits, const int32_t *vst, int nl, int cpl,
                                int tsize, int blk_cap, int iters, int32_t *slot_clause, int32_t *slot_order,
                                int32_t *blk, int64_t *cost_plain, int64_t *cost_opt) {
    if (n <= 0 || m <= 0 || !lits || !vst || nl <= 0 || nl % 64 || (cpl != 1 && cpl != 2) ||
        (tsize != 4 && tsize != 8) || m > (int64_t)nl * cpl || blk_cap < n + 1)
        return odesat::fail(ODESAT_EINVAL, "odesat_cv_layout: bad arguments");
    std::vector<int32_t> sc, sl, b;
    if (!odesat::cv_layout(n, m, lits, vst, nl, cpl, tsize, blk_cap, iters, sc, sl, b, cost_plain, cost_opt))
        return odesat::fail(ODESAT_EINVAL, "odesat_cv_layout: no layout");
    std::memcpy(slot_clause, sc.data(), sc.size() * 4);
    std::memcpy(slot_order, sl.data(), sl.size() * 4);
    std::memcpy(blk, b.data(), b.size() * 4);
    return ODESAT_OK;
}
