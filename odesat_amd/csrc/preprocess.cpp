// preprocess.cpp -- the reference's CNF preprocessing (cnf.rs:317-840), host C++ behind the C ABI:
// blocked-clause elimination (BCE) and bounded variable elimination by clause distribution toward a
// clause/variable ratio, then subsumption; plus the trace that rebuilds the eliminated variables
// (calculate_trace, cnf.rs:501-519).  This runs once per `solve`, on the host, as in the reference.
//
// Data layout: a clause is its sorted, de-duplicated literal codes (var << 1 | negated), which is the
// order of the reference's BTreeSet<Literal> (Literal derives Ord on (variable, is_negated)), and
// std::vector's lexicographic < is BTreeSet<CNFClauseSet>'s order.  Clauses are interned once (id per
// content); the formula and the per-variable occurrence sets hold ids ordered by content, so every
// iteration visits clauses in the reference's order.
//
// Deterministic where the reference is not: min_ratio_resolvant (cnf.rs:728-745) scans a HashSet of
// candidate variables and keeps the first strict minimum, so ties go to a random variable per run;
// here candidates are scanned in ascending order (the smallest variable wins a tie).  Everything
// else follows the reference operation by operation, including its quirks:
//   * resolvents that come out empty are dropped (cnf.rs:438-440), so (x) with (-x) yields nothing;
//   * a resolvent is dropped as tautological only when a literal of the second clause clashes with
//     one of the first (cnf.rs:429-435); is_blocked then checks the rest with is_tautology;
//   * the clause count in the ratio is usize arithmetic (release build: wraps), divided in f32;
//   * after a variable elimination only the touched variables are candidates (cnf.rs:772-787), so
//     the search stops when none of them stays within the ratio;
//   * the final subsumption removes every clause that strictly contains another (an empty clause
//     subsumes all others), computed here with occurrence lists instead of the O(m^2) scan.
#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <map>
#include <new>
#include <set>
#include <vector>

#include "../../include/odesat.h"
#include "cnf.hpp"

using odesat::fail;

namespace {

using Lit = uint64_t;
using Clause = std::vector<Lit>;

inline uint64_t var_of(Lit l) { return l >> 1; }

// cnf.rs:542-552
bool is_tautology(const Clause &c) {
    for (size_t i = 0; i + 1 < c.size(); ++i)
        if (!(c[i] & 1) && c[i + 1] == (c[i] | 1)) return true;
    return false;
}

bool contains(const Clause &c, Lit l) { return std::binary_search(c.begin(), c.end(), l); }

struct Step {
    int32_t kind;                  // ODESAT_STEP_*
    uint64_t var;
    std::vector<Clause> clauses;   // sorted (BTreeSet order)
};

struct Pre {
    std::vector<Clause> store;           // id -> content
    std::map<Clause, int32_t> ids;       // content -> id
    struct Less {
        const std::vector<Clause> *s;
        bool operator()(int32_t a, int32_t b) const { return (*s)[a] < (*s)[b]; }
    };
    using Set = std::set<int32_t, Less>;
    struct Occ {
        Set pos, neg;
    };
    Set formula{Less{&store}};
    std::map<uint64_t, Occ> idx;         // cnf.rs:381-401 calculate_variable_indices
    uint64_t varnum = 0;
    std::vector<Step> trace;

    int32_t intern(const Clause &c) {
        auto it = ids.find(c);
        if (it != ids.end()) return it->second;
        const int32_t id = (int32_t)store.size();
        store.push_back(c);
        ids.emplace(c, id);
        return id;
    }
    Occ &entry(uint64_t v) {
        auto it = idx.find(v);
        if (it == idx.end()) it = idx.emplace(v, Occ{Set{Less{&store}}, Set{Less{&store}}}).first;
        return it->second;
    }
    void index(int32_t id) {
        for (Lit l : store[id]) {
            Occ &o = entry(var_of(l));
            ((l & 1) ? o.neg : o.pos).insert(id);
        }
    }

    // cnf.rs:403-443 calculate_resolvents: `c` against every clause holding the opposite literal of
    // `v` (the negative side when c holds +v).  fn(resolvent) is called per kept resolvent; it
    // returns false to stop early.
    template <class F>
    void resolvents(const Clause &c, uint64_t v, F &&fn) const {
        auto it = idx.find(v);
        if (it == idx.end()) return;  // the reference indexes var_indices[&v] (always present here)
        const Set &other = contains(c, v << 1) ? it->second.neg : it->second.pos;
        Clause base;
        for (Lit l : c)
            if (var_of(l) != v) base.push_back(l);
        Clause comb;
        for (int32_t o : other) {
            comb = base;
            bool clash = false;
            for (Lit l : store[o]) {
                if (var_of(l) == v) continue;
                if (contains(base, l ^ 1)) {
                    clash = true;
                    break;
                }
                comb.push_back(l);
            }
            if (clash) continue;
            std::sort(comb.begin(), comb.end());
            comb.erase(std::unique(comb.begin(), comb.end()), comb.end());
            if (comb.empty()) continue;
            if (!fn(comb)) return;
        }
    }

    // cnf.rs:586-597 is_blocked: the first literal (in order) whose resolvents are all tautologies
    bool is_blocked(const Clause &c, uint64_t *var) const {
        for (Lit l : c) {
            bool all = true;
            resolvents(c, var_of(l), [&](const Clause &r) { return (all = is_tautology(r)); });
            if (all) {
                *var = var_of(l);
                return true;
            }
        }
        return false;
    }

    // cnf.rs:599-629 eliminate_if_blocked
    bool eliminate_if_blocked(int32_t id, std::set<uint64_t> *changed) {
        uint64_t var = 0;
        if (!is_blocked(store[id], &var)) return false;
        for (Lit l : store[id]) {
            if (changed) changed->insert(var_of(l));
            Occ &o = entry(var_of(l));
            ((l & 1) ? o.neg : o.pos).erase(id);
        }
        formula.erase(id);
        trace.push_back(Step{ODESAT_STEP_BLOCKED_CLAUSE, var, {store[id]}});
        return true;
    }

    // cnf.rs:463-480 calculate_var_resolvents + cnf.rs:736-738 (drop tautologies, subsume)
    std::vector<Clause> var_resolvents(uint64_t v) const {
        std::set<Clause> all;
        auto it = idx.find(v);
        for (int32_t p : it->second.pos)
            resolvents(store[p], v, [&](const Clause &r) {
                all.insert(r);
                return true;
            });
        std::vector<Clause> res;
        for (const Clause &r : all)
            if (!is_tautology(r)) res.push_back(r);
        return subsume_small(res);
    }

    // cnf.rs:521-540 subsume_clauses on a small sorted set: drop every clause that strictly contains
    // another member (the scan compares against the set before any removal)
    static std::vector<Clause> subsume_small(const std::vector<Clause> &s) {
        std::vector<Clause> keep;
        for (size_t i = 0; i < s.size(); ++i) {
            bool sub = false;
            for (size_t j = 0; j < s.size() && !sub; ++j)
                sub = j != i && s[j].size() <= s[i].size() &&
                      std::includes(s[i].begin(), s[i].end(), s[j].begin(), s[j].end());
            if (!sub) keep.push_back(s[i]);
        }
        return keep;
    }

    // cnf.rs:632-722 eliminate_variable
    void eliminate_variable(uint64_t v, const std::vector<Clause> &res, std::set<uint64_t> *changed) {
        auto it = idx.find(v);
        if (it == idx.end()) {
            trace.push_back(Step{ODESAT_STEP_VARIABLE_ELIMINATION, v, {}});
            return;
        }
        Occ occ = std::move(it->second);
        idx.erase(it);
        std::vector<int32_t> orig(occ.pos.begin(), occ.pos.end());
        orig.insert(orig.end(), occ.neg.begin(), occ.neg.end());
        for (int32_t o : orig)
            for (Lit l : store[o]) {
                changed->insert(var_of(l));
                if (var_of(l) == v) continue;
                auto j = idx.find(var_of(l));
                if (j != idx.end()) {
                    j->second.pos.erase(o);
                    j->second.neg.erase(o);
                }
            }
        for (int32_t o : orig) formula.erase(o);
        std::vector<int32_t> rid;
        for (const Clause &r : res) {
            rid.push_back(intern(r));
            formula.insert(rid.back());
        }
        varnum -= 1;  // usize; a release build wraps
        for (int32_t r : rid) index(r);
        std::set<Clause> modified;  // the positive clauses without +v (cnf.rs:709-719)
        for (int32_t p : occ.pos) {
            Clause c = store[p];
            c.erase(std::remove(c.begin(), c.end(), v << 1), c.end());
            modified.insert(c);
        }
        trace.push_back(Step{ODESAT_STEP_VARIABLE_ELIMINATION, v, {modified.begin(), modified.end()}});
    }

    // cnf.rs:725-758 min_ratio_resolvant (candidates ascending; see the header)
    bool min_ratio(const std::set<uint64_t> &cands, float target, uint64_t *best_var,
                   std::vector<Clause> *best_res) const {
        float smallest = FLT_MAX;
        bool found = false;
        for (uint64_t v : cands) {
            auto it = idx.find(v);
            if (it == idx.end()) continue;
            std::vector<Clause> res = var_resolvents(v);
            const uint64_t count =
                (uint64_t)formula.size() - (uint64_t)it->second.pos.size() - (uint64_t)it->second.neg.size() +
                (uint64_t)res.size();
            const uint64_t vars = varnum - 1;
            const float ratio = (float)count / (float)vars;
            if (ratio < smallest) {
                smallest = ratio;
                *best_var = v;
                *best_res = std::move(res);
                found = true;
            }
        }
        return found && !(smallest > target);
    }

    // cnf.rs:521-540 on the whole formula: occurrence lists keyed by each clause's first literal
    void subsume_formula() {
        std::vector<int32_t> cl(formula.begin(), formula.end());
        bool has_empty = false;
        std::map<Lit, std::vector<int32_t>> first;
        for (int32_t c : cl) {
            if (store[c].empty()) has_empty = true;
            else first[store[c][0]].push_back(c);
        }
        std::vector<int32_t> drop;
        for (int32_t c : cl) {
            const Clause &cc = store[c];
            if (cc.empty()) continue;
            bool sub = has_empty;
            for (size_t i = 0; i < cc.size() && !sub; ++i) {
                auto f = first.find(cc[i]);
                if (f == first.end()) continue;
                for (int32_t d : f->second) {
                    const Clause &dd = store[d];
                    if (d != c && dd.size() <= cc.size() && std::includes(cc.begin(), cc.end(), dd.begin(), dd.end())) {
                        sub = true;
                        break;
                    }
                }
            }
            if (sub) drop.push_back(c);
        }
        for (int32_t c : drop) formula.erase(c);
    }

    // cnf.rs:760-831 preprocessing_loop
    void run(float target) {
        std::vector<int32_t> blocked;
        for (int32_t c : formula) {
            uint64_t v;
            if (is_blocked(store[c], &v)) blocked.push_back(c);
        }
        for (int32_t c : blocked) eliminate_if_blocked(c, nullptr);
        std::set<uint64_t> cands;
        for (const auto &kv : idx) cands.insert(kv.first);
        uint64_t v = 0;
        std::vector<Clause> res;
        while (min_ratio(cands, target, &v, &res)) {
            cands.clear();
            eliminate_variable(v, res, &cands);
            for (const Clause &r : res) eliminate_if_blocked(ids.at(r), &cands);
        }
        subsume_formula();
    }
};

}  // namespace

struct odesat_trace {
    std::vector<Step> steps;
};

namespace {

// cnf.rs:266-287 evaluate_cnf_set: a variable read before it has a value gets `false` (entry API),
// every literal of every clause up to the first unsatisfied one is read
bool evaluate_insert(const std::vector<Clause> &clauses, uint8_t *values) {
    for (const Clause &c : clauses) {
        bool ok = false;
        for (Lit l : c) {
            uint8_t &x = values[var_of(l)];
            if (x == ODESAT_UNSET) x = 0;
            ok = ok || ((l & 1) ? x == 0 : x != 0);
        }
        if (!ok) return false;
    }
    return true;
}

}  // namespace

extern "C" int odesat_preprocess(const odesat_cnf *cnf, float target_ratio, odesat_cnf **out,
                                 odesat_trace **trace) {
    if (!cnf || !out || !trace) return fail(ODESAT_EINVAL, "odesat_preprocess: null argument");
    *out = nullptr;
    *trace = nullptr;
    try {
        Pre p;
        p.varnum = (uint64_t)cnf->varnum;
        // cnf.rs:348-361 convert_to_cnf_formula_set
        const int64_t m = cnf->nclauses();
        for (int64_t c = 0; c < m; ++c) {
            Clause cl;
            for (int64_t s = cnf->clause_ptr[c]; s < cnf->clause_ptr[c + 1]; ++s) {
                if (cnf->var[s] < 0) return fail(ODESAT_EINVAL, "odesat_preprocess: negative variable");
                cl.push_back((uint64_t)cnf->var[s] << 1 | (cnf->neg[s] ? 1 : 0));
            }
            std::sort(cl.begin(), cl.end());
            cl.erase(std::unique(cl.begin(), cl.end()), cl.end());
            p.formula.insert(p.intern(cl));
        }
        for (int32_t c : p.formula) p.index(c);
        p.run(target_ratio);
        // cnf.rs:364-379 convert_to_cnf_formula: clauses in set order, varnum carried over
        auto *f = new odesat_cnf();
        f->varnum = (int64_t)p.varnum;
        f->clause_ptr.push_back(0);
        for (int32_t c : p.formula) {
            for (Lit l : p.store[c]) {
                f->var.push_back((int64_t)var_of(l));
                f->neg.push_back((uint8_t)(l & 1));
            }
            f->clause_ptr.push_back((int64_t)f->var.size());
        }
        auto *t = new odesat_trace();
        t->steps = std::move(p.trace);
        *out = f;
        *trace = t;
    } catch (const std::bad_alloc &) {
        return fail(ODESAT_ENOMEM, "odesat_preprocess: out of memory");
    }
    return ODESAT_OK;
}

extern "C" void odesat_trace_free(odesat_trace *t) { delete t; }

extern "C" int64_t odesat_trace_nsteps(const odesat_trace *t) { return t ? (int64_t)t->steps.size() : 0; }

extern "C" int odesat_trace_step(const odesat_trace *t, int64_t i, int32_t *kind, int64_t *var,
                                 int64_t *nclauses, int64_t *nliterals) {
    if (!t || i < 0 || i >= (int64_t)t->steps.size()) return fail(ODESAT_EINVAL, "odesat_trace_step: bad step");
    const Step &s = t->steps[(size_t)i];
    int64_t L = 0;
    for (const Clause &c : s.clauses) L += (int64_t)c.size();
    if (kind) *kind = s.kind;
    if (var) *var = (int64_t)s.var;
    if (nclauses) *nclauses = (int64_t)s.clauses.size();
    if (nliterals) *nliterals = L;
    return ODESAT_OK;
}

extern "C" int odesat_trace_step_clauses(const odesat_trace *t, int64_t i, int64_t *clause_ptr, int64_t *var,
                                         uint8_t *neg) {
    if (!t || i < 0 || i >= (int64_t)t->steps.size())
        return fail(ODESAT_EINVAL, "odesat_trace_step_clauses: bad step");
    int64_t at = 0, k = 0;
    if (clause_ptr) clause_ptr[0] = 0;
    for (const Clause &c : t->steps[(size_t)i].clauses) {
        for (Lit l : c) {
            if (var) var[at] = (int64_t)var_of(l);
            if (neg) neg[at] = (uint8_t)(l & 1);
            ++at;
        }
        if (clause_ptr) clause_ptr[++k] = at;
    }
    return ODESAT_OK;
}

// cnf.rs:501-519 calculate_trace, newest step first
extern "C" int odesat_trace_apply(const odesat_trace *t, uint8_t *values, int64_t nvalues) {
    if (!t || (nvalues > 0 && !values)) return fail(ODESAT_EINVAL, "odesat_trace_apply: null argument");
    for (const Step &s : t->steps) {
        bool ok = s.var < (uint64_t)nvalues;
        for (const Clause &c : s.clauses)
            for (Lit l : c) ok = ok && var_of(l) < (uint64_t)nvalues;
        if (!ok) return fail(ODESAT_EINVAL, "odesat_trace_apply: values[] does not cover the trace's variables");
    }
    for (auto it = t->steps.rbegin(); it != t->steps.rend(); ++it) {
        if (it->kind == ODESAT_STEP_VARIABLE_ELIMINATION) {
            values[it->var] = evaluate_insert(it->clauses, values) ? 0 : 1;
        } else if (!evaluate_insert(it->clauses, values)) {
            values[it->var] = values[it->var] ? 0 : 1;
        }
    }
    return ODESAT_OK;
}

// cnf.rs:246-264 evaluate_cnf with its side effect: variables read without a value get `false`
extern "C" int odesat_cnf_evaluate_assign(const odesat_cnf *cnf, uint8_t *values, int64_t nvalues) {
    if (!cnf || (nvalues > 0 && !values)) return fail(ODESAT_EINVAL, "odesat_cnf_evaluate_assign: null argument");
    for (int64_t v : cnf->var)
        if (v < 0 || v >= nvalues)
            return fail(ODESAT_EINVAL, "odesat_cnf_evaluate_assign: values[] does not cover the formula");
    const int64_t m = cnf->nclauses();
    for (int64_t c = 0; c < m; ++c) {
        bool ok = false;
        for (int64_t s = cnf->clause_ptr[c]; s < cnf->clause_ptr[c + 1]; ++s) {
            uint8_t &x = values[cnf->var[s]];
            if (x == ODESAT_UNSET) x = 0;
            ok = ok || (cnf->neg[s] ? x == 0 : x != 0);
        }
        if (!ok) return 0;
    }
    return 1;
}

extern "C" int64_t odesat_cnf_max_variable(const odesat_cnf *cnf) {
    if (!cnf) return -1;
    int64_t mx = -1;
    for (int64_t v : cnf->var) mx = std::max(mx, v);
    return mx;
}
