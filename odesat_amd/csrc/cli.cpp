// cli.cpp -- the `odesat` command line over libodesat_hip.so: the reference's src/main.rs:12-397
// (clap subcommands solve / batch / inter, their flags, phase banners and output format), with the
// integration on the MI355X through the C ABI (include/odesat.h).
//
//   odesat solve -f FILE [-o OUT] [-t TOL] [-n STEPS] [-s DT] [-l ZETA] [-r RATIO]
//   odesat batch -f FILE -n STEPS -b BATCH [-o OUT] [-t TOL] [-s DT] [-l ZETA]
//   odesat inter -f FILE -b BATCH [-o OUT] [-t TOL] [-n STEPS] [-s DT] [-l ZETA]
//   extra flags: --seed S (initial voltages, counter RNG), --device D, --dtype f64|f32,
//                --gpus G (batch / inter: the B replicas split over GPUs 0..G-1, one host thread each)
//
// Semantics (main.rs):
//   batch (:254-323)  replicas run until their own allsat (all B at once on the device); the first
//                     replica, in index order, whose assignment satisfies the ORIGINAL formula is
//                     reported (the reference's sequential loop breaks there); if none does, the
//                     last replica's assignment is printed with `false`.
//   inter (:326-386)  all replicas stop at the first step any is allsat (simulate_inter); the first
//                     allsat replica of that step, else replica 0 (system.rs:353-358).
//   --gpus G          replica r keeps its global index (initial voltages keyed on it), so the result
//                     is the single-GPU one: batch takes the lowest satisfying global index over the
//                     GPUs; inter runs chunks in lock step from a device checkpoint and every GPU
//                     that ran past the earliest allsat step rolls back and re-runs exactly to it.
//   solve (:143-204)  preprocessing (cnf.rs:317-840, preprocess.cpp) to the -r ratio, one replica
//                     until allsat (unbounded without -n: launched in chunks), calculate_trace.
// Declared deviations: initial voltages come from the reproducible counter RNG (--seed) instead of
// thread_rng; the assignment is rendered in ascending variable order (the reference iterates a
// HashMap); preprocessing ties go to the smallest variable (preprocess.cpp); stoch draws from a
// counter RNG (stoch.hip).
//   stoch (:206-251)  preprocessing, then the discrete search (stoch.rs) of one replica from
//                     v = false, xl = 1 until every clause is satisfied (or -n steps).
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/odesat.h"

namespace {

const char *USAGE =
    "Usage: odesat <COMMAND>\n\n"
    "Commands:\n"
    "  solve  Run a single simulation\n"
    "  stoch  Run a stochastic search search\n"
    "  batch  Run a batch of simulations, sequentially\n"
    "  inter  Run a batch of simulations with their executions interlaced\n\n"
    "Options (per command, main.rs:31-141):\n"
    "  -f, --input <FILE>          Input file containing the CNF formula\n"
    "  -o, --output <FILE>         Optional output file\n"
    "  -t, --tolerance <TOL>       Error tolerance\n"
    "  -n, --step-number <N>       Step number (required by batch)\n"
    "  -s, --step-size <DT>        Step size (overrides tolerance)\n"
    "  -b, --batch-size <B>        Batch size (batch, inter; required)\n"
    "  -l, --learning-rate <ZETA>  Learning rate\n"
    "  -r, --ctv-ratio <R>         Clause-to-Variable Ratio (solve, stoch; default 7)\n"
    "      --seed <S>              Initial-voltage seed (default 42)\n"
    "      --device <D>            GPU index (default 0)\n"
    "      --gpus <G>              batch / inter: split the replicas over GPUs 0..G-1 (default 1)\n"
    "      --dtype <f64|f32>       Integration precision (default f64, the reference's)\n";

struct Opts {
    std::string cmd, input, output;
    bool has_tol = false, has_steps = false, has_dt = false, has_batch = false, has_zeta = false;
    double tol = 1e-3, dt = 0.01, zeta = -1.0, ratio = 7.0;
    int64_t steps = 0, batch = 0;
    uint64_t seed = 42;
    int device = 0, dtype = ODESAT_F64, gpus = 1;
    // hidden test hooks (not in USAGE): steps per bounded call of an unbounded run, and shards that
    // share the visible GPUs round-robin (tests rehearse --gpus G on a one-GPU box)
    int64_t run_chunk = (int64_t)1 << 20;
    bool share_devices = false;
};

[[noreturn]] void usage_error(const std::string &msg) {
    std::fprintf(stderr, "error: %s\n\n%s", msg.c_str(), USAGE);
    std::exit(2);
}

bool parse_f64(const char *s, double *out) {
    char *end = nullptr;
    errno = 0;
    const double x = std::strtod(s, &end);
    if (errno || !end || *end || end == s) return false;
    *out = x;
    return true;
}

bool parse_i64(const char *s, int64_t *out) {
    char *end = nullptr;
    errno = 0;
    const long long x = std::strtoll(s, &end, 10);
    if (errno || !end || *end || end == s || x < 0) return false;
    *out = (int64_t)x;
    return true;
}

Opts parse_args(int argc, char **argv) {
    Opts o;
    if (argc < 2) usage_error("a subcommand is required");
    o.cmd = argv[1];
    if (o.cmd == "-h" || o.cmd == "--help" || o.cmd == "help") {
        std::printf("%s", USAGE);
        std::exit(0);
    }
    if (o.cmd != "solve" && o.cmd != "batch" && o.cmd != "inter" && o.cmd != "stoch")
        usage_error("unrecognized subcommand '" + o.cmd + "'");
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "-h" || a == "--help") {
            std::printf("%s", USAGE);
            std::exit(0);
        }
        if (a == "--share-devices") {  // hidden test hook, takes no value
            o.share_devices = true;
            continue;
        }
        if (i + 1 >= argc) usage_error("a value is required for '" + a + "'");
        const char *val = argv[++i];
        auto f64 = [&](double *dst, bool *has) {
            if (!parse_f64(val, dst)) usage_error("invalid value '" + std::string(val) + "' for '" + a + "'");
            if (has) *has = true;
        };
        auto i64 = [&](int64_t *dst, bool *has) {
            if (!parse_i64(val, dst)) usage_error("invalid value '" + std::string(val) + "' for '" + a + "'");
            if (has) *has = true;
        };
        if (a == "-f" || a == "--input") o.input = val;
        else if (a == "-o" || a == "--output") o.output = val;
        else if (a == "-t" || a == "--tolerance") f64(&o.tol, &o.has_tol);
        else if (a == "-s" || a == "--step-size") f64(&o.dt, &o.has_dt);
        else if (a == "-l" || a == "--learning-rate") f64(&o.zeta, &o.has_zeta);
        else if (a == "-r" || a == "--ctv-ratio") f64(&o.ratio, nullptr);
        else if (a == "-n" || a == "--step-number") i64(&o.steps, &o.has_steps);
        else if (a == "-b" || a == "--batch-size") i64(&o.batch, &o.has_batch);
        else if (a == "--seed") {
            int64_t s = 0;
            i64(&s, nullptr);
            o.seed = (uint64_t)s;
        } else if (a == "--device") {
            int64_t d = 0;
            i64(&d, nullptr);
            o.device = (int)d;
        } else if (a == "--gpus") {
            int64_t g = 0;
            i64(&g, nullptr);
            if (g < 1) usage_error("--gpus must be >= 1");
            o.gpus = (int)g;
        } else if (a == "--run-chunk") {  // hidden test hook
            i64(&o.run_chunk, nullptr);
            if (o.run_chunk < 1) usage_error("--run-chunk must be >= 1");
        } else if (a == "--dtype") {
            if (std::string(val) == "f64") o.dtype = ODESAT_F64;
            else if (std::string(val) == "f32") o.dtype = ODESAT_F32;
            else usage_error("--dtype must be f64 or f32");
        } else {
            usage_error("unexpected argument '" + a + "'");
        }
    }
    if (o.input.empty()) usage_error("the following required arguments were not provided: --input <INPUT>");
    if (o.cmd == "batch" && !o.has_steps)
        usage_error("the following required arguments were not provided: --step-number <STEP_NUMBER>");
    if ((o.cmd == "batch" || o.cmd == "inter") && !o.has_batch)
        usage_error("the following required arguments were not provided: --batch-size <BATCH_SIZE>");
    if (o.cmd == "stoch" && (o.has_tol || o.has_dt || o.has_zeta || o.has_batch))  // StochOpts, main.rs:63-79
        usage_error("stoch takes only --input, --output, --step-number and --ctv-ratio");
    if (o.cmd == "solve" || o.cmd == "stoch") o.batch = 1;
    if (o.batch <= 0) usage_error("--batch-size must be > 0");
    if (o.gpus > 1 && o.cmd != "batch" && o.cmd != "inter") usage_error("--gpus applies to batch and inter");
    if (o.gpus > o.batch) usage_error("--gpus must not exceed --batch-size");
    return o;
}

int die(const char *what) {
    std::fprintf(stderr, "Error: %s: %s\n", what, odesat_last_error());
    return 1;
}

// A reusable barrier for the shard threads (C++17 has no std::barrier).
class Barrier {
  public:
    explicit Barrier(int n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        const uint64_t gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen_ != gen; });
        }
    }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    int n_, count_ = 0;
    uint64_t gen_ = 0;
};

// One GPU's share of the batch: global replicas [r0, r0 + count).
struct Shard {
    int device = 0;
    int64_t r0 = 0, count = 0;
    odesat_solver *s = nullptr;
    std::vector<int64_t> sat, done;
    std::string err;  // non-empty: this shard failed
};

constexpr int64_t NO_STEP = INT64_MAX;
constexpr int64_t ERR_STEP = -2;

int64_t earliest(const std::vector<int64_t> &sat) {
    int64_t t = NO_STEP;
    for (int64_t x : sat)
        if (x >= 0) t = std::min(t, x);
    return t;
}

// The integration of one shard (main.rs:169-176 / :283-292 / :348-360 with the device).  inter
// over several shards (shared != nullptr): chunks in lock step, from a checkpoint; after each the
// shards agree on the earliest allsat step T and a shard that ran past it rolls back and re-runs
// exactly to T (system.rs:291 -- every replica takes step T, none goes further).
void run_shard(const Opts &o, const odesat_cnf *norm, Shard &sh, int nshards, Barrier *bar,
               std::vector<int64_t> *shared, int index) {
    auto failed = [&](const char *what) { sh.err = std::string(what) + ": " + odesat_last_error(); };
    sh.sat.assign((size_t)sh.count, -1);
    sh.done.assign((size_t)sh.count, 0);
    if (odesat_solver_create(sh.device, norm, sh.count, o.dtype, &sh.s)) failed("solver");
    else if (odesat_init_state(sh.s, o.seed, sh.r0)) failed("init");
    odesat_params p{};
    p.adaptive = o.has_dt ? 0 : 1;  // step_size overrides tolerance (main.rs:49)
    p.stop = o.cmd == "inter" ? ODESAT_STOP_ANY : ODESAT_STOP_EACH;
    p.tol = o.tol;
    p.dt = o.dt;
    p.zeta = o.has_zeta ? o.zeta : -1.0;
    const int64_t chunk = o.run_chunk;  // steps per bounded call of an unbounded run
    const bool bounded = o.has_steps || o.cmd == "batch";
    if (nshards == 1 || o.cmd != "inter") {
        if (!sh.err.empty()) return;
        if (bounded) {
            p.max_steps = o.steps;
            if (p.max_steps > 0 && odesat_simulate(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr))
                failed("simulate");
            return;
        }
        // steps = None: until some replica is allsat (system.rs:198, :221, :296, :333) -- one run in
        // bounded calls (dt and the step count carry over)
        p.max_steps = chunk;
        if (odesat_simulate(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr)) return failed("simulate");
        while (earliest(sh.sat) == NO_STEP)
            if (odesat_simulate_continue(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr))
                return failed("simulate");
        return;
    }
    // inter over several shards
    const int64_t total = bounded ? o.steps : INT64_MAX;
    // lock-step chunk: steps between the shards' stop agreements (each chunk starts from a device
    // checkpoint).  The same value is sharding.run_inter's default (odesat_amd/sharding.py).
    constexpr int64_t INTER_LOCKSTEP_CHUNK = 256;
    const int64_t k_lock = std::min<int64_t>(chunk, INTER_LOCKSTEP_CHUNK);
    for (int64_t t = 0; t < total;) {
        const int64_t k = std::min(k_lock, total - t);
        p.max_steps = k;
        int64_t local = ERR_STEP;
        if (sh.err.empty()) {
            const int rc = odesat_checkpoint(sh.s) ? 1
                         : (t == 0 ? odesat_simulate(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr)
                                   : odesat_simulate_continue(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr));
            if (rc) failed("simulate");
            else local = earliest(sh.sat);
        }
        (*shared)[index] = local;
        bar->wait();
        int64_t T = NO_STEP;
        bool err = false;
        for (int64_t x : *shared) {
            err = err || x == ERR_STEP;
            T = std::min(T, x == ERR_STEP ? NO_STEP : x);
        }
        bar->wait();  // every shard has read the slots before they are rewritten
        if (err) return;
        if (T == NO_STEP) {
            t += k;
            continue;
        }
        if (local != T) {  // this shard ran past T: back to the chunk's start, then exactly to T
            p.max_steps = T - t + 1;
            if (odesat_rollback(sh.s) ||
                (t == 0 ? odesat_simulate(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr)
                        : odesat_simulate_continue(sh.s, &p, sh.sat.data(), sh.done.data(), nullptr, nullptr)))
                failed("simulate");
        }
        return;
    }
}

// cnf.rs:289-298 render_variable_map ("{var} {0|1}\n"; ascending, see the header)
std::string render(const std::vector<std::pair<int64_t, bool>> &vals) {
    std::string s;
    for (const auto &kv : vals) s += std::to_string(kv.first) + (kv.second ? " 1\n" : " 0\n");
    return s;
}

}  // namespace

int main(int argc, char **argv) {
    const Opts o = parse_args(argc, argv);
    std::printf("Reading CNF formula from file...\n");
    std::ifstream in(o.input, std::ios::binary);
    if (!in) {
        std::fprintf(stderr, "Error: cannot read %s\n", o.input.c_str());
        return 1;
    }
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string text = ss.str();

    std::printf("Parsing CNF formula...\n");
    odesat_cnf *formula = nullptr;
    if (odesat_cnf_parse(text.data(), text.size(), &formula)) return die("parse");
    // solve: preprocessing (main.rs:162-166, cnf.rs:833-840); batch / inter integrate the parsed formula
    odesat_cnf *reduced = nullptr;
    odesat_trace *trace = nullptr;
    const odesat_cnf *work = formula;
    const bool preprocess = o.cmd == "solve" || o.cmd == "stoch";
    if (preprocess) {
        std::printf("Preprocessing CNF formula...\n");
        if (odesat_preprocess(formula, (float)o.ratio, &reduced, &trace)) return die("preprocess");
        std::printf("Clauses: %" PRId64 " | Vars: %" PRId64 "\n", odesat_cnf_nclauses(reduced),
                    odesat_cnf_varnum(reduced));  // cnf.rs:824-828
        work = reduced;
    } else {
        std::printf("Normalizing CNF formula...\n");
    }
    const int64_t L = odesat_cnf_nliterals(work);
    std::vector<int64_t> names((size_t)std::max<int64_t>(L, 1));
    int64_t k = 0;
    odesat_cnf *norm = nullptr;
    if (odesat_cnf_normalize(work, &norm, names.data(), &k)) return die("normalize");
    const int64_t n = odesat_cnf_varnum(norm);

    std::printf("Simulating...\n");
    std::fflush(stdout);
    // a formula with no variables left (everything eliminated) has an empty state: nothing to
    // integrate, the reference's simulate returns an empty vector at once
    odesat_stoch *st = nullptr;
    std::vector<Shard> shards;
    if (n > 0 && o.cmd == "stoch") {  // stoch.rs:83-110 search
        std::vector<int64_t> sat(1, -1), done(1, 0);
        if (odesat_stoch_create(o.device, norm, 1, &st)) return die("stoch");
        const int64_t chunk = o.has_steps ? o.steps : (int64_t)1 << 16;
        do {
            if (chunk > 0 && odesat_stoch_search(st, o.seed, 0, chunk, ODESAT_STOP_EACH, 0, sat.data(), done.data()))
                return die("search");
        } while (!o.has_steps && sat[0] < 0);
    } else if (n > 0) {
        int ndev = 0;
        if (odesat_device_count(&ndev)) return die("devices");
        // --share-devices lets shards share the visible GPUs round-robin (tests rehearse --gpus G on
        // a one-GPU box); otherwise every shard needs a GPU of its own
        const bool share = o.share_devices;
        if (o.gpus > 1 && o.gpus > ndev && !share) {
            std::fprintf(stderr, "Error: --gpus %d but %d GPU(s) are visible\n", o.gpus, ndev);
            return 1;
        }
        const int G = o.gpus;
        shards.resize((size_t)G);
        for (int d = 0; d < G; ++d) {  // contiguous global ranges, the remainder to the first shards
            const int64_t per = o.batch / G, extra = o.batch % G;
            shards[d].device = G == 1 ? o.device : d % std::max(1, ndev);
            shards[d].count = per + (d < extra ? 1 : 0);
            shards[d].r0 = d * per + std::min<int64_t>(d, extra);
        }
        Barrier bar(G);
        std::vector<int64_t> slots((size_t)G, 0);
        if (G == 1) {
            run_shard(o, norm, shards[0], 1, nullptr, nullptr, 0);
        } else {
            std::vector<std::thread> th;
            for (int d = 0; d < G; ++d) th.emplace_back(run_shard, std::cref(o), norm, std::ref(shards[d]), G, &bar, &slots, d);
            for (auto &x : th) x.join();
        }
        for (auto &sh : shards)
            if (!sh.err.empty()) {
                std::fprintf(stderr, "Error: %s (device %d)\n", sh.err.c_str(), sh.device);
                return 1;
            }
    }
    auto shard_of = [&](int64_t r) -> Shard & {
        for (auto &sh : shards)
            if (r >= sh.r0 && r < sh.r0 + sh.count) return sh;
        return shards.back();
    };
    // the reference's HashMap<usize, bool> as a tri-state array over the file's variable names
    const int64_t top = std::max<int64_t>(odesat_cnf_max_variable(formula), 0) + 1;
    std::vector<uint8_t> vals((size_t)top, ODESAT_UNSET);
    std::vector<uint8_t> a((size_t)std::max<int64_t>(n, 1));
    auto mapped = [&](int64_t r) -> int {  // map_values_by_indices (cnf.rs:301-315); r is a global index
        if (!shards.empty()) {
            Shard &sh = shard_of(r);
            if (odesat_get_assignment(sh.s, r - sh.r0, a.data())) return 1;
        }
        if (st && odesat_stoch_get_state(st, r, 1, a.data(), nullptr)) return 1;
        std::fill(vals.begin(), vals.end(), (uint8_t)ODESAT_UNSET);
        if (shards.empty() && !st) return 0;
        for (int64_t i = 0; i < k && i < n; ++i) vals[(size_t)names[i]] = a[i];
        return 0;
    };
    auto evaluate = [&]() -> bool {  // evaluate_cnf against the ORIGINAL formula (inserts unset reads)
        const int rc = odesat_cnf_evaluate_assign(formula, vals.data(), top);
        if (rc < 0) std::exit(die("evaluate"));
        return rc == 1;
    };
    bool satisfied = false;
    if (o.cmd == "inter") {  // the earliest allsat step, then the lowest global index (system.rs:353-358)
        int64_t win = 0, best = INT64_MAX;
        for (auto &sh : shards)
            for (int64_t b = 0; b < sh.count; ++b)
                if (sh.sat[b] >= 0 && sh.sat[b] < best) {
                    best = sh.sat[b];
                    win = sh.r0 + b;
                }
        if (mapped(win)) return die("assignment");
        satisfied = evaluate();
    } else if (preprocess) {  // solve, stoch
        std::printf("Mapping values...\n");
        if (mapped(0)) return die("assignment");
        if (odesat_trace_apply(trace, vals.data(), top)) return die("trace");  // calculate_trace
        std::printf("Evaluating CNF formula...\n");
        satisfied = evaluate();
    } else {  // batch: each device checks its replicas at once (odesat_evaluate), the lowest
              // satisfying global index wins, then the host re-checks the pick against the input:
              // the first satisfying replica, else the last
        int64_t first = -1;
        for (auto &sh : shards) {
            int64_t f = -1;
            if (odesat_evaluate(sh.s, nullptr, &f)) return die("evaluate");
            if (f >= 0) {
                first = sh.r0 + f;
                break;  // shards hold increasing global ranges
            }
        }
        const int64_t pick = first >= 0 ? first : o.batch - 1;
        // main.rs:279-280: the sequential loop announces every replica it runs, up to the one it keeps
        for (int64_t i = 0; i <= pick; ++i) std::printf("\rRunning simulation %" PRId64 ".", i + 1);
        std::fflush(stdout);
        if (mapped(pick)) return die("assignment");
        satisfied = evaluate();
    }
    std::printf(preprocess ? "Checking if solution vector satisfies formula: %s\n"
                                 : "\nChecking if solution vector satisfies formula: %s\n",
                satisfied ? "true" : "false");
    std::printf("Rendering variable assignments...\n");
    std::vector<std::pair<int64_t, bool>> listed;
    for (int64_t v = 0; v < top; ++v)
        if (vals[(size_t)v] != ODESAT_UNSET) listed.emplace_back(v, vals[(size_t)v] != 0);
    const std::string out = render(listed);
    if (!o.output.empty()) {
        std::printf("Writing results to file...\n");
        std::ofstream f(o.output, std::ios::binary);
        f << out;
        if (!f) {
            std::fprintf(stderr, "Error: cannot write %s\n", o.output.c_str());
            return 1;
        }
    } else {
        std::printf("Variable assignments:\n%s\n", out.c_str());
    }
    for (auto &sh : shards)
        if (sh.s) odesat_solver_destroy(sh.s);
    if (st) odesat_stoch_destroy(st);
    odesat_cnf_free(norm);
    odesat_cnf_free(reduced);
    odesat_trace_free(trace);
    odesat_cnf_free(formula);
    return 0;
}
