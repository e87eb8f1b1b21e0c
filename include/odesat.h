/*
 * odesat.h -- C ABI of libodesat_hip.so, the MI355X-native replacement for odesat's per-step ODE
 * integrator (reference: AHartNtkn/odesat @ 2024-10-24, Rust).
 *
 * The reference has no FFI: its boundary is the Rust library API re-exported by src/lib.rs:1-3
 * (`pub mod cnf; pub mod stoch; pub mod system;`).  Each entry point below names the Rust function
 * it replaces (file:line).  INTEGRATION.md shows the `extern "C"` block a maintainer would add to the
 * Rust crate to bind it.
 *
 * Conventions
 *   - Every `int` function returns ODESAT_OK (0) or a negative ODESAT_E* code; the message is in
 *     odesat_last_error() (thread-local).  No exception crosses the ABI.  (The reference panics on
 *     malformed input, cnf.rs:151,160, and aborts, Cargo.toml:24.)
 *   - Host buffers are caller-owned and copied; device memory is library-owned.
 *   - One odesat_solver per GPU, driven by one host thread.  Multi-GPU = N solvers on N threads or
 *     processes (replicas shard with no collective).
 *   - State arrays at the ABI are replica-major f64: v[B][n], xs[B][m], xl[B][m] -- one Rust
 *     `State` (system.rs:6-11) per replica.  On the device the library keeps its own layout
 *     (replica-innermost) in the solver's dtype (f32 or f64).
 *   - Variables are the normalised 0-based indices of cnf.rs:206-219 (ascending renaming).
 *   - No CPU fallback: every integrator call needs a gfx950 device and fails loudly otherwise.
 */
#ifndef ODESAT_H
#define ODESAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ODESAT_OK 0
#define ODESAT_EINVAL -1   /* bad argument / malformed DIMACS */
#define ODESAT_ENOMEM -2   /* host or device allocation failed */
#define ODESAT_EDEVICE -3  /* HIP runtime error or no usable device */
#define ODESAT_ESTATE -4   /* call not valid in the solver's current state */

#define ODESAT_F32 0
#define ODESAT_F64 1

/* stop policies for odesat_simulate */
#define ODESAT_STOP_EACH 0 /* batch (main.rs:278-308): every replica runs until ITS allsat, then freezes */
#define ODESAT_STOP_ANY 1  /* inter (system.rs:291,308,329,346): all replicas stop at the first step any is allsat */
#define ODESAT_STOP_NONE 2 /* benchmark: run exactly max_steps on every replica, no sat test acts */

typedef struct odesat_cnf odesat_cnf;       /* host-side parsed formula (cnf.rs:53-57 CNFFormula) */
typedef struct odesat_solver odesat_solver; /* device-resident formula + B replica states */

const char *odesat_last_error(void);
const char *odesat_version(void);
/* number of visible HIP devices (0 on a machine without a GPU) */
int odesat_device_count(int *count);

/* ------------------------------------------------------------------ loader (cnf.rs) ---------- */

/* cnf.rs:138-172 parse_dimacs_format (+ CNFFormula::new, cnf.rs:60-77).  Lines starting with 'c'
 * are skipped, "p cnf N ..." sets varnum, every other line is a clause read up to the token "0" (an
 * empty line is an empty clause).  A token that is not an i32 gives ODESAT_EINVAL where the
 * reference panics. */
int odesat_cnf_parse(const char *text, size_t len, odesat_cnf **out);
/* Build a formula from arrays: clause c owns [clause_ptr[c], clause_ptr[c+1]) of var/neg.
 * varnum < 0 means "no header": varnum = number of distinct variables (cnf.rs:63-75). */
int odesat_cnf_from_arrays(int64_t varnum, int64_t nclauses, const int64_t *clause_ptr,
                           const int64_t *var, const uint8_t *neg, odesat_cnf **out);
void odesat_cnf_free(odesat_cnf *cnf);
int64_t odesat_cnf_varnum(const odesat_cnf *cnf);
int64_t odesat_cnf_nclauses(const odesat_cnf *cnf);
int64_t odesat_cnf_nliterals(const odesat_cnf *cnf);
/* copy out the CSR (clause_ptr[m+1], var[L], neg[L]); any pointer may be NULL */
int odesat_cnf_export(const odesat_cnf *cnf, int64_t *clause_ptr, int64_t *var, uint8_t *neg);
/* cnf.rs:206-219 normalize_cnf_variables: distinct variables renamed 0..k-1 in ASCENDING order
 * (declared deviation: the reference iterates a HashSet, a random order per run).  varnum is kept.
 * old_names[k] (may be NULL, else capacity >= number of distinct variables) receives new -> old. */
int odesat_cnf_normalize(const odesat_cnf *cnf, odesat_cnf **out, int64_t *old_names,
                         int64_t *k_out);
/* cnf.rs:246-264 evaluate_cnf: values[var] for var < nvalues, any other variable reads false.
 * Returns 1 (satisfied), 0 (not), or a negative error. */
int odesat_cnf_evaluate(const odesat_cnf *cnf, const uint8_t *values, int64_t nvalues);
/* system.rs:361-372 init_short_term_memory: xs[c] = +1 if clause c has a negated literal, else -1 */
int odesat_cnf_init_short_term_memory(const odesat_cnf *cnf, double *xs);

/* ------------------------------------------------ stochastic search (stoch.rs:20-110) ------- */

/* The `stoch` command's discrete search (stoch.rs; main.rs:206-251) for `batch` independent
 * replicas of a NORMALISED formula on one GPU.  State per replica: v[n] booleans (bytes 0/1) and
 * xl[m] u64; create / reset start every replica from search()'s v = false, xl = 1 (stoch.rs:88-91).
 * Declared deviation: the reference's draw gen_range(1..=tot) uses thread_rng; here
 * r = 1 + mulhi64(h, tot) with h a counter RNG of (seed, replica0 + r, step, var), step = the
 * replica's steps since its state was set.  A variable in no clause (the reference panics at
 * gen_range(1..=0), stoch.rs:70) makes create fail with ODESAT_EINVAL. */
typedef struct odesat_stoch odesat_stoch;
int odesat_stoch_create(int device, const odesat_cnf *normalized, int64_t batch, odesat_stoch **out);
void odesat_stoch_destroy(odesat_stoch *s);
/* v = false, xl = 1, step counter 0 for replicas [r0, r0+count) */
int odesat_stoch_reset(odesat_stoch *s, int64_t r0, int64_t count);
/* replica-major host arrays v[count][n] (0/1), xl[count][m]; either may be NULL (that part is
 * reset); the step counter restarts */
int odesat_stoch_set_state(odesat_stoch *s, int64_t r0, int64_t count, const uint8_t *v, const uint64_t *xl);
int odesat_stoch_get_state(odesat_stoch *s, int64_t r0, int64_t count, uint8_t *v, uint64_t *xl);
/* search (stoch.rs:83-110) on every replica: up to max_steps (> 0) steps; stop = ODESAT_STOP_EACH
 * (a replica stops after its first step that finds every clause satisfied) or ODESAT_STOP_NONE.
 * first_sat_step[B] (0-based step of this call, -1 none) and steps_done[B] may be NULL;
 * poll_interval = steps between host checks of "all stopped" (0 = 64). */
int odesat_stoch_search(odesat_stoch *s, uint64_t seed, int64_t replica0, int64_t max_steps, int stop,
                        int32_t poll_interval, int64_t *first_sat_step, int64_t *steps_done);
/* the kernel search runs on: replicas per workgroup of the one-wave-per-replica kernel (formulas
 * whose topology and one replica's state fit in LDS), or 0 for the three-kernel HBM path */
int odesat_stoch_wave_width(const odesat_stoch *s);

/* ------------------------------------------------------- preprocessing (cnf.rs:317-840) ----- */

/* The `solve` command's preprocessing: repeatedly_resolve_and_update (cnf.rs:833-840) on the set
 * form of the formula (convert_to_cnf_formula_set, cnf.rs:348-361): blocked-clause elimination,
 * bounded variable elimination while the clause/variable ratio stays <= target_ratio, subsumption.
 * out: the reduced formula in set order (convert_to_cnf_formula, cnf.rs:364-379), varnum = input
 * varnum - eliminated variables.  trace: the SimplificationTrace (cnf.rs:560-578).
 * Declared deviation: ties of min_ratio_resolvant (cnf.rs:728-745, a HashSet scan) go to the
 * smallest variable. */
typedef struct odesat_trace odesat_trace;
#define ODESAT_STEP_VARIABLE_ELIMINATION 0 /* cnf.rs:555 (var, positive clauses without +var) */
#define ODESAT_STEP_BLOCKED_CLAUSE 1       /* cnf.rs:556 (var, the removed clause) */
#define ODESAT_UNSET 2                     /* tri-state assignment: no value yet */
int odesat_preprocess(const odesat_cnf *cnf, float target_ratio, odesat_cnf **out,
                      odesat_trace **trace);
void odesat_trace_free(odesat_trace *t);
int64_t odesat_trace_nsteps(const odesat_trace *t);
/* step i: kind, variable, clause and literal counts (any pointer may be NULL) */
int odesat_trace_step(const odesat_trace *t, int64_t i, int32_t *kind, int64_t *var,
                      int64_t *nclauses, int64_t *nliterals);
/* step i's clauses as a CSR: clause_ptr[nclauses+1], var[nliterals], neg[nliterals] (NULL ok) */
int odesat_trace_step_clauses(const odesat_trace *t, int64_t i, int64_t *clause_ptr, int64_t *var,
                              uint8_t *neg);
/* cnf.rs:501-519 calculate_trace on a tri-state assignment values[var] in {0, 1, ODESAT_UNSET}
 * (the reference's HashMap; a variable read while unset becomes 0, as its entry API does).
 * nvalues must exceed every variable of the trace. */
int odesat_trace_apply(const odesat_trace *t, uint8_t *values, int64_t nvalues);
/* cnf.rs:246-264 evaluate_cnf on the tri-state assignment, with its side effect: every variable
 * read (all literals of the clauses up to the first unsatisfied one) that is unset becomes 0.
 * Returns 1 / 0 or a negative error. */
int odesat_cnf_evaluate_assign(const odesat_cnf *cnf, uint8_t *values, int64_t nvalues);
/* the largest variable name in the formula, -1 if it has no literals */
int64_t odesat_cnf_max_variable(const odesat_cnf *cnf);

/* ------------------------------------------------------------- integrator (system.rs) -------- */

/* Upload a NORMALISED formula (every variable < varnum) for `batch` replicas on `device`.
 * dtype = ODESAT_F32 (throughput mode) or ODESAT_F64 (the reference's precision).  The state is
 * initialised to v = 0, xs = init_short_term_memory, xl = 1; use odesat_set_state or
 * odesat_init_state before stepping. */
int odesat_solver_create(int device, const odesat_cnf *normalized, int64_t batch, int dtype,
                         odesat_solver **out);
void odesat_solver_destroy(odesat_solver *s);
int64_t odesat_solver_batch(const odesat_solver *s);
int64_t odesat_solver_varnum(const odesat_solver *s);
int64_t odesat_solver_nclauses(const odesat_solver *s);
/* Device bytes held by the solver. */
int64_t odesat_solver_device_bytes(const odesat_solver *s);

/* Replace replicas [r0, r0+count) with caller states (replica-major f64; values are rounded to
 * the solver dtype).  Marks those replicas active, first_sat_step = -1, adaptive dt = 0.01. */
int odesat_set_state(odesat_solver *s, int64_t r0, int64_t count, const double *v,
                     const double *xs, const double *xl);
/* Device-side initial states for every replica b (global index replica0 + b):
 * v[i] = counter RNG(seed, replica0 + b, i) ~ U[-1,1) (main.rs:171, 285, 353 with a reproducible
 * generator), xs = init_short_term_memory (system.rs:361), xl = 1 (main.rs:173). */
int odesat_init_state(odesat_solver *s, uint64_t seed, int64_t replica0);
/* Copy replicas [r0, r0+count) back (replica-major f64; any pointer may be NULL). */
int odesat_get_state(odesat_solver *s, int64_t r0, int64_t count, double *v, double *xs,
                     double *xl);
/* system.rs:238 / :355: assignment[i] = v[i] > 0 for replica r. */
int odesat_get_assignment(odesat_solver *s, int64_t r, uint8_t *assignment);
/* cnf.rs:246-264 evaluate_cnf of every replica's assignment (v > 0, system.rs:238) against the
 * solver's formula, on the device.  satisfied[B] (may be NULL);
 * first_satisfied = the lowest replica index whose assignment satisfies the formula, -1 if none
 * (batch's pick, main.rs:302-307; may be NULL).  The formula is the normalised one the solver was
 * built from, which without preprocessing is the input with variables renamed. */
int odesat_evaluate(odesat_solver *s, uint8_t *satisfied, int64_t *first_satisfied);

/* system.rs:25-91 compute_derivatives on every replica's current state (no state change).
 * dv[B][n], dxs[B][m], dxl[B][m] (may be NULL), allsat[B] (may be NULL). */
int odesat_compute_derivatives(odesat_solver *s, double zeta, double *dv, double *dxs,
                               double *dxl, uint8_t *allsat);
/* system.rs:141-154 euler_step_fixed on every replica; allsat[B] = pre-update result. */
int odesat_euler_step_fixed(odesat_solver *s, double dt, double zeta, uint8_t *allsat);
/* system.rs:111-139 euler_step on every replica with its own dt: dt[B] in/out (may be NULL: the
 * solver's per-replica dt is used and kept); allsat[B] as returned by the reference. */
int odesat_euler_step(odesat_solver *s, double tol, double *dt, double zeta, uint8_t *allsat);

typedef struct {
    int32_t adaptive;      /* 0: fixed step `dt` (system.rs:190-203); 1: adaptive (:204-234) */
    int32_t stop;          /* ODESAT_STOP_EACH | ODESAT_STOP_ANY | ODESAT_STOP_NONE */
    double tol;            /* adaptive tolerance (reference default 1e-3, system.rs:174) */
    double dt;             /* fixed step size; adaptive starts every replica at 0.01 (:205) */
    double zeta;           /* learning rate; < 0 = density heuristic (system.rs:164-173) */
    int64_t max_steps;     /* > 0 (the reference's None = unbounded is refused) */
    int32_t poll_interval; /* steps between host polls of the stop condition (0 = default 32); with
                              the persistent kernels (RESIDENT / ONCHIP) also the steps per launch */
    int32_t dt_policy;     /* ODESAT_DT_PER_REPLICA (0, the device's) | ODESAT_DT_SHARED_SERIAL (1: the
                              reference's one dt threaded through the replicas, system.rs:314-326; the
                              CPU oracle's policy, refused by the device) */
} odesat_params;
#define ODESAT_DT_PER_REPLICA 0
#define ODESAT_DT_SHARED_SERIAL 1

/* system.rs:156-239 (simulate) applied to every replica at once, or :241-359 (simulate_inter)
 * with stop = ODESAT_STOP_ANY.  Replicas continue from their current state.
 *   first_sat_step[B] : 0-based step at which the replica was allsat, -1 if never (may be NULL)
 *   steps_done[B]     : euler steps applied to the replica in this call (may be NULL)
 *   dt_out[B]         : final adaptive dt per replica (may be NULL)
 *   steps_run         : steps run: the steps launched, or with STOP_ANY after a stop the stop step + 1
 *                       (the reference's simulate_inter steps; may be NULL)
 * Declared deviation: adaptive STOP_ANY uses a per-replica dt; the reference threads ONE dt
 * serially through the replicas (system.rs:314-326), which cannot run in parallel. */
int odesat_simulate(odesat_solver *s, const odesat_params *p, int64_t *first_sat_step,
                    int64_t *steps_done, double *dt_out, int64_t *steps_run);
/* The same run continued for up to p->max_steps more steps (p as in the call that started it): no
 * bookkeeping restarts -- adaptive dt, frozen replicas (STOP_EACH) and a reached stop step (STOP_ANY)
 * carry over, steps are numbered from the run's start (first_sat_step is run-relative, steps_done
 * cumulative).  This is how the reference's unbounded loops (steps = None, system.rs:198, :221,
 * :296, :333) run in bounded calls without leaving its trajectory.  odesat_set_state /
 * odesat_init_state end a run (the next continue numbers steps from 0). */
int odesat_simulate_continue(odesat_solver *s, const odesat_params *p, int64_t *first_sat_step,
                             int64_t *steps_done, double *dt_out, int64_t *steps_run);

/* A device-side checkpoint of every replica's state and bookkeeping, including the position in a
 * continued run (one slot per solver, library-owned memory); odesat_rollback restores it (ODESAT_ESTATE
 * without one).  The sharded inter driver uses it to stop every rank at the global first allsat step
 * (odesat_amd/sharding.py, cli.cpp --gpus). */
int odesat_checkpoint(odesat_solver *s);
int odesat_rollback(odesat_solver *s);

/* Block until all work queued by the solver is done. */
int odesat_synchronize(odesat_solver *s);

/* ------------------------------------------- one-call boundary --------------- */

/* The drop-in for simulate / simulate_inter (system.rs:156-163, :241-248) in one call.
 * odesat_create: a normalised formula as CSR (clause_ptr[m+1], lits = var << 1 | negated, every
 * var < n) for `device`; NULL on error with the message in err[errlen] (and odesat_last_error()).
 * odesat_run: B replicas' f32 states, replica-innermost (v0[n][B], xs0[m][B], xl0[m][B]), are
 * integrated per *p: adaptive 0/1 (FIXED/ADAPTIVE), dt, tol, zeta (< 0: density heuristic),
 * max_steps (0 = the reference's None: until every replica (STOP_EACH) / some replica (STOP_ANY)
 * is allsat), stop, dt_policy (the device runs ODESAT_DT_PER_REPLICA only).  The final states go to
 * v_out / xs_out / xl_out (same layout; any may be NULL), first_sat_step[B] (-1 = never) and
 * steps_done[B].  Host buffers stay the caller's; device memory is the context's. */
typedef struct odesat_ctx odesat_ctx;
odesat_ctx *odesat_create(int device, int32_t n, int32_t m, const int32_t *clause_ptr, const int32_t *lits,
                          char *err, size_t errlen);
int odesat_run(odesat_ctx *ctx, const odesat_params *p, int32_t B, const float *v0, const float *xs0,
               const float *xl0, float *v_out, float *xs_out, float *xl_out, int64_t *first_sat_step,
               int64_t *steps_done);
void odesat_destroy(odesat_ctx *ctx);

/* --------------------------------------------------------------- measurement ----------------- */

/* When enabled, odesat_simulate brackets every launch with HIP events on the solver's stream.
 * odesat_profile_read returns, per kernel class (0 = clause kernel, 1 = variable kernel, 2 = status
 * kernel), the summed device milliseconds and the launch count since the last reset. */
int odesat_profile_enable(odesat_solver *s, int enable);
int odesat_profile_read(odesat_solver *s, double *ms /*[3]*/, int64_t *launches /*[3]*/);
/* Algorithmic bytes per step of the dominant kernel over the whole batch (roofline):
 * FUSED / RESIDENT / ONCHIP (2n + 4m) * dtype bytes per replica (v, xs, xl read and written once),
 * TWOPASS k_clause (n + 4m) * dtype bytes. */
int64_t odesat_clause_kernel_bytes(const odesat_solver *s);
/* Tuning: replicas per chunk (0 = automatic) -- the batch is stepped chunk by chunk so the
 * contribution buffer of one chunk stays resident in the Infinity Cache. */
int odesat_set_chunk_replicas(odesat_solver *s, int64_t replicas);
/* Schedule of odesat_simulate over chunks (results are identical; STOP_ANY is always step-major):
 * AUTO = chunk-major when the batch spans several chunks. */
#define ODESAT_SCHED_AUTO 0
#define ODESAT_SCHED_STEP_MAJOR 1  /* every step: all chunks, then the next step */
#define ODESAT_SCHED_CHUNK_MAJOR 2 /* every chunk: all steps, then the next chunk */
int odesat_set_schedule(odesat_solver *s, int schedule);
/* Per-step algorithm (results are bit-identical):
 * FUSED    = one variable-major kernel per RHS, clauses recomputed from L2-resident voltages;
 * TWOPASS  = clause kernel writing per-literal contributions + variable kernel summing them;
 * RESIDENT = persistent kernel, one workgroup per replica group with its voltages in LDS for many
 *            steps (odesat_simulate only; single-step calls use FUSED).  Available when the
 *            solver's group layout was chosen for it (the default when the voltages fit in LDS). */
#define ODESAT_ALG_FUSED 0
#define ODESAT_ALG_TWOPASS 1
#define ODESAT_ALG_RESIDENT 2
/* ONCHIP   = fixed steps with a replica's WHOLE state on one CU for a launch: v and dv in LDS, the
 *            clause memories in VGPRs + LDS (onchip.hip); per step only the L2-resident clause
 *            records are read.  f32 3-SAT formulas whose tiles fit (config 2's size); the default
 *            when available.  Adaptive steps on such a solver run RESIDENT. */
#define ODESAT_ALG_ONCHIP 3
int odesat_set_algorithm(odesat_solver *s, int alg);
/* The algorithm odesat_simulate uses (ODESAT_ALG_*), and the solver's replica group width. */
int odesat_get_algorithm(const odesat_solver *s);
int odesat_group_width(const odesat_solver *s);
/* The step kernel odesat_simulate launches for fixed (adaptive = 0) or adaptive steps: "k_onchip",
 * "k_resident", "k_wave", "k_step" (FUSED) or "k_clause_u" (TWOPASS); NULL for a null solver. */
const char *odesat_step_kernel(const odesat_solver *s, int adaptive);
/* Experiment knobs: kernel variants and layouts for A/B measurement and for the
 * parity tests that drive every path against the oracle.  Production callers never need them: the
 * defaults are the measured best, and every variant is bit-identical to them.  The library reads no
 * environment variable; a knob is set here, process-wide, and read when the object it shapes is
 * created (solver, partition or stoch context; RUN_CHUNK by each odesat_run).  value >= 0 sets the
 * knob, value < 0 unsets it.  ODESAT_EINVAL for an unknown key.  odesat_get_experiment stores the
 * knob's value, or -1 when it is unset.  odesat_experiment_knob(i) names the i-th knob
 * (ODESAT_EINVAL past the last). */
int odesat_set_experiment(const char *key, int64_t value);
int odesat_get_experiment(const char *key, int64_t *value);
void odesat_clear_experiments(void);
int odesat_experiment_knob(int i, const char **name);

/* Test hook (no device needed): k_solo_cv's lane and LDS block placement (odesat_amd/csrc/cv_layout.cpp)
 * for a 3-SAT formula -- lits[3 m] = var << 1 | neg, vst[n + 1] the variable-major term starts -- on nl
 * lanes (a multiple of 64) of cpl (1 or 2) clause slots, tsize-byte (4 / 8) terms and term blocks
 * 0 .. blk_cap - 1, after `iters` search steps: slot_clause[nl cpl] (clause or -1), slot_order[3 nl cpl]
 * (the clause's literal index 0..2 at each position), blk[n + 1] (blk[n]: the zero block), and the bank model's
 * LDS cycles of the plain and the chosen layout. */
int odesat_cv_layout(int64_t n, int64_t m, const int32_t *lits, const int32_t *vst, int nl, int cpl, int tsize,
                     int blk_cap, int iters, int32_t *slot_clause, int32_t *slot_order, int32_t *blk,
                     int64_t *cost_plain, int64_t *cost_opt);

/* --------------------------------------------- one instance across GPUs ------- */

/* The fixed Euler step (system.rs:141-154) of ONE replica whose formula is partitioned over `world`
 * ranks, one process per GPU; the caller runs the collective (RCCL all-gather / all-reduce on the
 * device buffers; odesat_amd/partition.py builds the local topology below).  Two partitions:
 *   ODESAT_PART_CLAUSES    rank r holds a slice of the clauses and a full v[n].  odesat_part_rhs
 *                          writes the partial dv of every variable (out[0..n)) and the rank's unsat
 *                          count (out[n]); the caller all-reduces (sum) out and calls
 *                          odesat_part_apply.  Matches the reference within a tolerance (the sum
 *                          across ranks reorders the fold; bit-exact at world = 1).
 *   ODESAT_PART_VARIABLES  rank r holds variables [v0, v1) and every clause touching them.
 *                          odesat_part_rhs writes the updated voltages of [v0, v1) (out[0..S)) and
 *                          its unsat count (out[S]); the caller all-gathers the world blocks of
 *                          S + 1 floats, which are the next step's voltages (variable i at
 *                          i + i / S).  Bit-exact for any world size.
 *   ODESAT_PART_CLAUSES_RS rank r holds a slice of the clauses, as CLAUSES, and v in VARIABLES'
 *                          gathered layout (block = S, full range v0 = 0, v1 = n).  odesat_part_rhs
 *                          (apply = 2) writes the partial dv of every variable at out[i + i / S] and
 *                          the rank's unsat count in every block's flag slot; the caller
 *                          reduce-scatters (sum) out onto its block of S + 1 floats, calls
 *                          odesat_part_reduce_apply, and all-gathers the send blocks into v.  The
 *                          all-reduce split into its two halves; tolerance parity
 *                          as CLAUSES (bit-exact at world = 1).
 * world = the number of ranks.  Local topology: clause_ptr[mloc + 1], var[L], neg[L] of the local clauses in the reference's clause
 * order; var_ptr[v1 - v0 + 1] / inc_slot[] = for each variable of [v0, v1), its local literal slots
 * in clause-then-literal order; block = S (VARIABLES) or 0 (CLAUSES, plain v[n]).  m = the global
 * clause count (xl's upper clamp, system.rs:95).  Device pointers v / out / dvsum are the caller's;
 * `stream` is a hipStream_t (NULL = the default stream). */
#define ODESAT_PART_CLAUSES 0
#define ODESAT_PART_VARIABLES 1
#define ODESAT_PART_CLAUSES_RS 2
typedef struct odesat_part odesat_part;
int odesat_part_create(int device, int world, int64_t n, int64_t m, int64_t mloc, const int64_t *clause_ptr,
                       const int64_t *var, const uint8_t *neg, int64_t v0, int64_t v1,
                       const int64_t *var_ptr, const int64_t *inc_slot, int64_t block,
                       odesat_part **out);
void odesat_part_destroy(odesat_part *p);
int64_t odesat_part_device_bytes(const odesat_part *p);
/* the local clauses' memories, in local clause order (f64 host arrays of mloc) */
int odesat_part_set_memories(odesat_part *p, const double *xs, const double *xl);
int odesat_part_get_memories(odesat_part *p, double *xs, double *xl);
/* Enqueue one right-hand side + memory update; apply = 0 (CLAUSES), 1 (VARIABLES) or 2 (CLAUSES_RS).  Before it,
 * the previous step's global unsat count (read from v's flag slots or out[n]) is folded into the
 * replica's bookkeeping; stop = 1: the first allsat step freezes the replica (simulate,
 * system.rs:193) and later steps are no-ops, so callers may poll at any interval. */
int odesat_part_rhs(odesat_part *p, const float *v, float *out, double dt, double zeta, int apply,
                    int stop, void *stream);
/* CLAUSES: v[i] = clamp(v[i] + dt * dvsum[i]) after the all-reduce (system.rs:96) */
int odesat_part_apply(odesat_part *p, float *v, const float *dvsum, double dt, void *stream);
/* CLAUSES_RS: after the reduce-scatter, rank `rank`'s voltages (v[i + rank], i in its block) take the
 * summed dv of `block` (S + 1 floats, the last the summed unsat count) into `send` (S + 1 floats:
 * the updated voltages, then that count), the all-gather's input (system.rs:96). */
int odesat_part_reduce_apply(odesat_part *p, const float *v, const float *block, float *send, int rank,
                             double dt, void *stream);
/* Restart the bookkeeping (steps done 0, no sat step, not frozen). */
int odesat_part_reset(odesat_part *p, void *stream);
/* Fold the last step's unsat count and read the bookkeeping (synchronises `stream`). */
int odesat_part_status(odesat_part *p, const float *v, const float *out, int apply, int stop,
                       void *stream, int64_t *steps_done, int64_t *sat_step, int32_t *frozen);

#ifdef __cplusplus
}
#endif
#endif
