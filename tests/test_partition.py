"""One instance across GPUs (odesat_amd/partition.py, csrc/partition.hip; BASELINE configs[4],
SURVEY.md §8e).

CPU: the local topologies (every rank's fold covers exactly the reference's accumulation of its
variables), and the distributed step at world_size 2 over gloo with the numpy restatement
(oracle/np_oracle.py) standing in for the per-rank kernels: the VARIABLES partition reproduces the
single-process oracle bit for bit, the CLAUSES partition (all-reduce, or CLAUSES_RS: reduce-scatter +
all-gather) within a stated tolerance.
GPU: the HIP kernels, at world 1 and as 2-3 ranks on one device with the exchange done in-process,
against the oracle's f32 restatement: bit-exact (VARIABLES, and CLAUSES at world 1), tolerance
(CLAUSES at world 2); the stop bookkeeping against simulate (system.rs:190-203); and one real
two-process gloo run through TorchComm (scripts/bench_partition.py)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from odesat_amd.partition import CLAUSES, CLAUSES_RS, VARIABLES, block_size, default_zeta, local_topology
from tests.common import oracle_formula

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# CLAUSES at world > 1 sums per-rank partial dv (stated tolerance, max |dv| after 30-40 fixed f32
# steps of dt 0.05 on the fixtures)
CLAUSES_TOL = 1e-5


def _arrays(name):
    f = oracle_formula(name)
    return f.clause_ptr, f.var, f.neg.astype(np.uint8), f.varnum


def _global_incidences(cp, var, i):
    """(clause, literal position) of every occurrence of variable i, in the reference's order."""
    out = []
    for c in range(len(cp) - 1):
        for j, s in enumerate(range(cp[c], cp[c + 1])):
            if var[s] == i:
                out.append((c, j))
    return out


@pytest.mark.parametrize("name", ["rand200", "easy", "small"])
@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("order", ["file", "minvar"])
def test_variables_topology_folds_exactly_the_reference_order(name, world, order):
    """Whatever order the clause kernel processes the local clauses in, every variable's incidences
    are listed in the reference's (clause, literal) order."""
    cp, var, neg, n = _arrays(name)
    m = len(cp) - 1
    seen = []
    for r in range(world):
        t = local_topology(cp, var, neg, n, VARIABLES, r, world, order=order)
        assert t["block"] == block_size(n, world) and t["v1"] - t["v0"] <= t["block"]
        loc = t["clauses"]
        if order == "file":
            assert np.all(np.diff(loc) > 0)  # the reference's clause order
        else:  # ascending smallest variable
            vmin = [int(var[cp[c]:cp[c + 1]].min()) if cp[c + 1] > cp[c] else n for c in loc]
            assert vmin == sorted(vmin)
        touching = {c for c in range(m)
                    if np.any((var[cp[c]:cp[c + 1]] >= t["v0"]) & (var[cp[c]:cp[c + 1]] < t["v1"]))}
        assert set(loc.tolist()) == touching
        lcp = t["clause_ptr"]
        for i in range(t["v0"], t["v1"]):
            slots = t["inc_slot"][t["var_ptr"][i - t["v0"]]:t["var_ptr"][i - t["v0"] + 1]]
            got = []
            for s in slots:
                k = int(np.searchsorted(lcp, s, side="right") - 1)
                assert t["var"][s] == i
                got.append((int(loc[k]), int(s - lcp[k])))
            assert got == _global_incidences(cp, var, i)
        seen.extend(range(t["v0"], t["v1"]))
    assert seen == list(range(n))


@pytest.mark.parametrize("mode", [CLAUSES, CLAUSES_RS])
@pytest.mark.parametrize("world", [1, 2, 5])
def test_clauses_topology_partitions_the_clauses(world, mode):
    cp, var, neg, n = _arrays("rand200")
    m = len(cp) - 1
    allc = []
    for r in range(world):
        t = local_topology(cp, var, neg, n, mode, r, world)
        assert (t["v0"], t["v1"], t["block"]) == (0, n, block_size(n, world) if mode == CLAUSES_RS else 0)
        assert t["var_ptr"][-1] == t["clause_ptr"][-1]  # every local literal is one incidence
        assert sorted(t["clauses"].tolist()) == list(range(r * m // world, (r + 1) * m // world))
        allc.extend(sorted(t["clauses"].tolist()))
    assert allc == list(range(m))


# ------------------------------------------------------------------ gloo, world_size 2 --------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _xs0(cp, neg):
    """system.rs:361-372."""
    return np.array([1.0 if np.any(neg[cp[c]:cp[c + 1]]) else -1.0 for c in range(len(cp) - 1)])


def _emu_step(t, v, xs, xl, dt, zeta, m_global):
    """A rank's kernels restated with np_oracle (f32): partial dv of the local clauses, memories."""
    from oracle import np_oracle as npo
    T = np.float32
    f = npo.Formula(t["clause_ptr"], t["var"], t["neg"].astype(bool), t["n"])
    dv, dxs, dxl, allsat, _ = npo.compute_derivatives(f, v, xs, xl, T(zeta), T)
    xs2 = np.fmin(np.fmax(xs + T(dt) * dxs, T(0.001)), T(1.0) - T(0.001)).astype(T)
    xl2 = np.fmin(np.fmax(xl + T(dt) * dxl, T(1.0)), T(1e4) * T(m_global)).astype(T)
    return dv, xs2, xl2, (0 if allsat else 1)


def _gloo_worker(rank, world, port, out, mode, steps, dt):
    import torch
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import init_voltages
    cp, var, neg, n = _arrays("rand200")
    m = len(cp) - 1
    t = local_topology(cp, var, neg, n, mode, rank, world, order="file")  # the emulation folds in local order
    T = np.float32
    v = init_voltages(7, 0, 1, n)[0].astype(T)
    xs = _xs0(cp, neg).astype(T)[t["clauses"]]
    xl = np.ones(len(t["clauses"]), T)
    zeta = default_zeta(n, m)
    S = t["block"]
    unsat_hist = []
    for _ in range(steps):
        dv, xs, xl, uns = _emu_step(t, v, xs, xl, dt, zeta, m)
        if mode == VARIABLES:
            blk = np.zeros(S + 1, T)
            sl = slice(t["v0"], t["v1"])
            blk[:t["v1"] - t["v0"]] = np.fmin(np.fmax(v[sl] + T(dt) * dv[sl], T(-1.0)), T(1.0))
            blk[S] = uns
            g = torch.zeros(world * (S + 1), dtype=torch.float32)
            td.all_gather_into_tensor(g, torch.from_numpy(blk))
            g = g.numpy().reshape(world, S + 1)
            v = g[:, :S].reshape(-1)[:n].copy()
            unsat_hist.append(float(g[:, S].sum()))
        elif mode == CLAUSES_RS:  # reduce-scatter (gloo: all-reduce, keep own block), update, all-gather
            full = np.zeros(world * (S + 1), T)
            i = np.arange(n)
            full[i + i // S] = dv
            full[S::S + 1] = uns
            buf = torch.from_numpy(full)
            td.all_reduce(buf)
            blk = buf.numpy()[rank * (S + 1):(rank + 1) * (S + 1)]
            own = slice(rank * S, min(n, (rank + 1) * S))
            send = np.zeros(S + 1, T)
            send[:own.stop - own.start] = np.fmin(np.fmax(v[own] + T(dt) * blk[:own.stop - own.start], T(-1.0)), T(1.0))
            send[S] = blk[S]
            g = torch.zeros(world * (S + 1), dtype=torch.float32)
            td.all_gather_into_tensor(g, torch.from_numpy(send))
            g = g.numpy().reshape(world, S + 1)
            v = g[:, :S].reshape(-1)[:n].copy()
            unsat_hist.append(float(g[0, S]))
        else:
            buf = torch.from_numpy(np.concatenate([dv, [T(uns)]]).astype(T))
            td.all_reduce(buf)
            b = buf.numpy()
            v = np.fmin(np.fmax(v + T(dt) * b[:n], T(-1.0)), T(1.0)).astype(T)
            unsat_hist.append(float(b[n]))
    res = {"v": v.astype(np.float64).tolist(), "xs": xs.astype(np.float64).tolist(),
           "xl": xl.astype(np.float64).tolist(), "clauses": t["clauses"].tolist(), "unsat": unsat_hist}
    with open(f"{out}.{rank}", "w") as fh:
        json.dump(res, fh)
    td.destroy_process_group()


@pytest.mark.parametrize("mode", [VARIABLES, CLAUSES, CLAUSES_RS])
def test_two_rank_gloo_step_matches_single_process_oracle(tmp_path, mode):
    import torch.multiprocessing as mp

    from oracle.oracle import Oracle, init_voltages
    world, steps, dt = 2, 40, 0.05
    out = str(tmp_path / "r")
    mp.spawn(_gloo_worker, args=(world, _free_port(), out, mode, steps, dt), nprocs=world, join=True)
    ranks = [json.load(open(f"{out}.{r}")) for r in range(world)]
    cp, var, neg, n = _arrays("rand200")
    m = len(cp) - 1
    o = Oracle(cp, var, neg, n, "f32")
    T = np.float32
    v = init_voltages(7, 0, 1, n)[0].astype(T)
    xs, xl = o.init_short_term_memory(), np.ones(m, T)
    sats = [o.euler_step_fixed(v, xs, xl, T(dt), T(default_zeta(n, m))) for _ in range(steps)]
    for r in ranks:
        loc = np.array(r["clauses"])
        if mode == VARIABLES:  # bit-exact
            assert np.array_equal(np.array(r["v"], T), v)
            assert np.array_equal(np.array(r["xs"], T), xs[loc]) and np.array_equal(np.array(r["xl"], T), xl[loc])
        else:
            assert np.max(np.abs(np.array(r["v"]) - v)) <= CLAUSES_TOL
        assert [u == 0 for u in r["unsat"]] == [bool(s) for s in sats]
    assert ranks[0]["v"] == ranks[1]["v"]  # every rank holds the same voltages


# ------------------------------------------------------------------ GPU (the HIP kernels) ------
def _oracle_run(name, steps, dt, seed=7, stop=False):
    from oracle.oracle import Oracle, init_voltages
    cp, var, neg, n = _arrays(name)
    m = len(cp) - 1
    o = Oracle(cp, var, neg, n, "f32")
    T = np.float32
    v = init_voltages(seed, 0, 1, n)[0].astype(T)
    xs, xl = o.init_short_term_memory(), np.ones(m, T)
    init = (v.copy(), xs.copy(), xl.copy())
    if stop:
        t, sat, _, _, _ = o.simulate(v, xs, xl, dt=T(dt), steps=steps, zeta=T(default_zeta(n, m)))
        return init, (v, xs, xl), t, sat
    sats = [o.euler_step_fixed(v, xs, xl, T(dt), T(default_zeta(n, m))) for _ in range(steps)]
    return init, (v, xs, xl), steps, sats


def _run_parts(name, mode, world, steps, dt, stop=False, poll=7):
    from odesat_amd.partition import LocalComm, PartitionedSolver, step_in_process
    cp, var, neg, n = _arrays(name)
    m = len(cp) - 1
    init, _, _, _ = _oracle_run(name, 0, dt)
    parts = [PartitionedSolver(cp, var, neg, n, mode, comm=LocalComm(r, world)) for r in range(world)]
    for p in parts:
        p.set_state(*init)
    zeta = default_zeta(n, m)
    for k in range(steps):
        step_in_process(parts, dt, zeta, stop)
        if stop and (k + 1) % poll == 0 and parts[0].status(stop)["frozen"]:
            break
    sts = [p.status(stop) for p in parts]
    states = [p.get_state() for p in parts]
    for p in parts:
        p.close()
    return sts, states


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rand200", "easy", "small"])
@pytest.mark.parametrize("mode,world", [(VARIABLES, 1), (VARIABLES, 2), (VARIABLES, 3), (CLAUSES, 1), (CLAUSES, 2),
                                        (CLAUSES_RS, 1), (CLAUSES_RS, 2), (CLAUSES_RS, 3)])
def test_partition_kernels_match_oracle(name, mode, world):
    steps, dt = 30, 0.05
    _, (v, xs, xl), _, sats = _oracle_run(name, steps, dt)
    sts, states = _run_parts(name, mode, world, steps, dt, stop=False)
    exp_sat = next((k for k, s in enumerate(sats) if s), -1)
    for st, (gv, gxs, gxl, loc) in zip(sts, states):
        assert st["steps_done"] == steps
        if mode == VARIABLES or world == 1:
            assert np.array_equal(gv.astype(np.float32), v)
            assert np.array_equal(gxs.astype(np.float32), xs[loc]) and np.array_equal(gxl.astype(np.float32), xl[loc])
            assert st["first_sat_step"] == exp_sat
        else:
            assert np.max(np.abs(gv - v)) <= CLAUSES_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("env", [
    {"PART_TERMS": "slot"}, {"PART_TERMS": "ell"}, {"PART_TERMS": "region"},
    {"PART_PACK": "0"}, {"PART_K3": "0"}, {"PART_XCD": "1"},
    {"PART_REGIONS": "24", "PART_PACK": "0"}])
@pytest.mark.parametrize("mode,world", [(VARIABLES, 2), (CLAUSES, 1), (CLAUSES_RS, 1)])
def test_partition_layouts_match_oracle(xp, env, mode, world):
    """Every term layout / clause record / clause kernel / placement choice (read when a slice is
    created) folds the same terms in the same order: the same bits as the oracle."""
    for k, val in env.items():
        xp.set(k, val)
    steps, dt = 20, 0.05
    _, (v, xs, xl), _, _ = _oracle_run("rand200", steps, dt)
    sts, states = _run_parts("rand200", mode, world, steps, dt, stop=False)
    for st, (gv, gxs, gxl, loc) in zip(sts, states):
        assert st["steps_done"] == steps
        assert np.array_equal(gv.astype(np.float32), v)
        assert np.array_equal(gxs.astype(np.float32), xs[loc]) and np.array_equal(gxl.astype(np.float32), xl[loc])


@pytest.mark.gpu
@pytest.mark.parametrize("mode,world", [(VARIABLES, 2), (CLAUSES, 1), (CLAUSES_RS, 1)])
def test_partition_stop_matches_simulate(mode, world):
    """easy.cnf is SAT: the replica freezes at simulate's stop step, polled every 7 steps."""
    steps, dt = 4000, 0.1
    _, (v, xs, xl), t, sat = _oracle_run("easy", steps, dt, stop=True)
    assert sat
    sts, states = _run_parts("easy", mode, world, steps, dt, stop=True, poll=7)
    for st, (gv, gxs, gxl, loc) in zip(sts, states):
        assert st["frozen"] and st["steps_done"] == t and st["first_sat_step"] == t - 1
        assert np.array_equal(gv.astype(np.float32), v)
        assert np.array_equal(gxs.astype(np.float32), xs[loc])


@pytest.mark.gpu
def test_partition_two_processes_gloo_on_one_device(tmp_path):
    """Two ranks (processes) sharing the box's GPU, exchanging through TorchComm over gloo."""
    out = str(tmp_path / "p.json")
    env = dict(os.environ, ODESAT_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "scripts", "bench_partition.py"), "--fixture", "rand200", "--steps", "30",
           "--warmup", "0", "--dt", "0.05", "--mode", "variables", "--check-out", out, "--gpus", "2"]
    subprocess.run(cmd, check=True, env=env, timeout=240, cwd=ROOT)
    res = json.load(open(out))
    _, (v, _, _), _, _ = _oracle_run("rand200", 30, 0.05)
    assert res["steps_done"] == 30
    assert np.array_equal(np.array(res["v"], np.float32), v)
