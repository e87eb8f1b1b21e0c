"""bench.py's multi-GPU legs at world_size 2 over gloo on the CPU (VERDICT r2 "Next #1"): the code
the driver's SCALE run executes over RCCL -- config 4's sharded inter protocol with its in-run digest,
config 5's three partitions with theirs -- driven with host stand-ins of the device objects
(tests/host_standins.py) on small instances, checked against one process running the C oracle."""
import json
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY4 = dict(n=60, m=150, k=3, seed=11)    # replicas 6..11 are allsat first, at step 205 (rank 1 of 2 x 6)
TINY5 = dict(n=300, m=1260, k=3, seed=5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _args(steps, warmup):
    return SimpleNamespace(steps=steps, warmup=warmup, profile_dir=os.path.join(ROOT, "profiles"), batch=6,
                           dtype="f32", config="config2", config5_graph=0)


BARRIER_DELAY = 0.25  # seconds every barrier of the legs' process group sleeps first (test_bench_multi_gpu_legs_gloo)


def _delay(world):
    """The barrier delay at this world size: 8 gloo ranks on this container's 8 CPUs step the host
    stand-ins slowly enough (config 5's 12 steps took up to ~0.4 s) that the delay grows with them."""
    return BARRIER_DELAY * max(1, world // 2)


class _SlowBarrier:
    """torch.distributed with a barrier that sleeps first: a timed region that reads its clock after
    the closing barrier would grow by the delay."""

    def __init__(self, td, delay):
        self._td, self._delay, self.barriers = td, delay, 0

    def barrier(self):
        import time
        time.sleep(self._delay)
        self.barriers += 1
        self._td.barrier()

    def __getattr__(self, name):
        return getattr(self._td, name)


def _worker(rank, world, port, out, per):
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from odesat_amd import workloads as wl
    from tests.host_standins import HostPart, HostSolver
    wl.CONFIGS["tiny4"], wl.CONFIGS["tiny5"] = TINY4, TINY5
    slow = _SlowBarrier(td, _delay(world))
    r4 = bench.config4_leg(_args(300, 3), world, rank, 0, slow, solver_cls=HostSolver, config="tiny4", batch=per)
    r5 = bench.config5_leg(_args(12, 3), world, rank, 0, slow, part_cls=HostPart, config="tiny5")
    r4["barriers"] = slow.barriers
    if rank == 0:
        with open(out, "w") as fh:
            json.dump({"c4": r4, "c5": r5}, fh)
    td.destroy_process_group()


@pytest.mark.parametrize("world,per", [(2, 6), (4, 3), (8, 2)])
def test_bench_multi_gpu_legs_gloo(tmp_path, world, per):
    """World 2, 4 and 8 -- the driver's SCALE shape (12 replicas at world 2 and 4: the first allsat ones
    on rank 1, resp. ranks 2-3; 16 at world 8: on ranks 3-5)."""
    import torch.multiprocessing as mp

    from odesat_amd import workloads as wl
    from oracle.oracle import Oracle, init_voltages
    out = str(tmp_path / "legs.json")
    mp.spawn(_worker, args=(world, _free_port(), out, per), nprocs=world, join=True)
    res = json.load(open(out))

    # config 4: the sharded protocol stops every replica at the single-process inter stop
    c4 = res["c4"]
    var, neg = wl.random_ksat(TINY4["n"], TINY4["m"], 3, TINY4["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    o = Oracle(cp, v_, n_, TINY4["n"], "f32")
    B = world * per
    v = init_voltages(42, 0, B, o.n).astype(np.float32)
    xs = np.tile(o.init_short_term_memory(), (B, 1))
    xl = np.ones((B, o.m), np.float32)
    t, win, _, _ = o.simulate_inter(v, xs, xl, dt=np.float32(0.01), steps=300)
    assert 0 < t < 300 and win >= per  # rank 1's replica stops the run; rank 0 rolled back
    assert c4["steps_run"] == t and c4["winner"] == {"step": t - 1, "replica": win}
    assert c4["digest"]["match"] and c4["digest"]["ranks_checked"] == world
    assert c4["global_batch"] == B and c4["value"] > 0 and c4["roofline"]["bound"] == "hbm"
    # every barrier slept the delay, and none of that is in a timed region
    delay = _delay(world)
    assert c4["barriers"] >= 4
    assert c4["ms_per_step"] * c4["steps_run"] < 1e3 * delay, c4["ms_per_step"] * c4["steps_run"]
    assert c4["steps_run"] / c4["stop_none_value"] * B * 1e3 < 1e3 * delay, c4["stop_none_value"]

    # config 5: VARIABLES bit-exact against rank 0's world-1 run, the CLAUSES forms within tolerance
    c5 = res["c5"]
    d = c5["digest"]
    assert d["variables_bit_exact"] and d["clauses_within_tol"] and d["clauses_rs_within_tol"]
    assert d["steps"] == 15
    for name in ("clauses", "clauses_rs", "variables"):
        assert c5[name]["value"] > 0 and c5[name]["exchange_bytes_per_rank"] > 0
        assert c5[name]["ms_per_step"] * 12 < 1e3 * delay, (name, c5[name]["ms_per_step"])  # not timed
    assert c5["variables"]["local_clauses_rank0"] < TINY5["m"]  # a share of the clauses


def test_watchdog_prints_the_line_and_ends_the_job_past_the_deadline():
    """A leg that never returns (a collective stuck on one node) costs only that leg: past
    --leg-deadline rank 0 prints the line built so far, marked ("watchdog": the unfinished legs are
    missing), and the process exits with bench.WATCHDOG_EXIT = 0, so a driver that treats a non-zero
    status as a failed run keeps the measured headline."""
    import subprocess
    import sys
    import time
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "res = {}\n"
            "w = bench.Watchdog(0.5, 0, lambda e: {'value': 7.0, **res, **(e or {})})\n"
            "res['f64'] = {'value': 1.0}\n"
            "time.sleep(30)\n" % ROOT)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and time.time() - t0 < 25
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 7.0 and d["f64"] == {"value": 1.0} and "watchdog" in d


def test_watchdog_emits_once_when_the_legs_finish():
    import contextlib
    import io
    import sys
    sys.path.insert(0, ROOT)
    import bench
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        w = bench.Watchdog(60.0, 0, lambda e: {"value": 3.0, **(e or {})})
        w.cancel()
        assert w.emit() and not w.emit()
        w1 = bench.Watchdog(60.0, 1, lambda e: {"value": 3.0})  # other ranks print nothing
        w1.cancel()
        assert w1.emit()
    lines = buf.getvalue().splitlines()
    assert lines == [json.dumps({"value": 3.0})]


class _FakeSolver:
    """The calls time_gpu makes, doing nothing: the timed region then holds only harness cost."""

    def simulate(self, max_steps, poll_interval, **kw):
        return {"steps_run": max_steps, "steps_done": np.full(4, max_steps)}

    def profile(self, on):
        pass

    def profile_read(self):
        return [0.0, 0.0, 0.0], [1, 0, 0]

    def synchronize(self):
        pass


class _SleepDist:
    def __init__(self, delay):
        self.delay, self.barriers = delay, 0

    def barrier(self):
        import time
        time.sleep(self.delay)
        self.barriers += 1


def test_time_gpu_excludes_the_closing_barrier():
    """the headline's timed region ends at the device sync, before the barrier
    (a barrier that sleeps 50 ms must not change the measured time)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from odesat_amd.system import ODESAT_STOP_NONE
    d = _SleepDist(0.05)
    wall, _, _, ran = bench.time_gpu(_FakeSolver(), 20, 5, d, 0, False, ODESAT_STOP_NONE)
    assert d.barriers == 2 and ran == 20  # one barrier opens the region, one follows it
    assert wall < 0.02
    wall0, _, _, _ = bench.time_gpu(_FakeSolver(), 20, 5, None, 0, False, ODESAT_STOP_NONE)
    assert abs(wall - wall0) < 0.02


def test_roofline_reads_the_committed_profiles():
    """The bench line's roofline from the committed PMC fits (profiles/profile_*.json), at the
    driver's shape (20 steps, B = 1024, config 2) with made-up launch times: k_onchip names VALU issue
    and carries its cycle model; the f64 k_resident with register tiles moves fewer bytes than the
    algorithmic convention counts, so its line also carries the rate of the bytes actually moved
    (fabric_traffic, below the algorithmic one) and says why the algorithmic rate can exceed the peak;
    every traffic figure says what the counters count (L2 <-> fabric bytes, Infinity-Cache hits included)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    args = SimpleNamespace(batch=1024, dtype="f32", config="config2", steps=20, profile_dir=os.path.join(ROOT, "profiles"))
    n, m = 10000, 42000
    r = bench.roofline(args, "k_onchip", [1.6, 0.0, 0.0], [1, 0, 0], 1024 * (8 * n + 16 * m))
    assert r["bound"] == "valu" and 0.1 < r["frac"] < 1.0 and r["traffic"] > 0
    assert 0.0 < r["cycle_model"]["valu_floor_frac"] < 1.0
    r64 = bench.roofline(args, "k_resident", [4.7, 0.0, 0.0], [1, 0, 0], 1024 * (8 * n + 16 * m) * 2, dtype="f64")
    assert r64["bound"] == "hbm" and r64["traffic"] < 0.9 * r64["algorithmic_bytes_per_launch"]
    assert 0.0 < r64["fabric_traffic"]["achieved"] < r64["achieved"] and "register tiles" in r64["note"]
    assert "Infinity-Cache hits are included" in r64["traffic_counts"] and "fabric" in r["traffic_counts"]


class _Graph:
    """A captured graph of the host stand-in: replay runs the steps (or raises, as a failed replay)."""

    def __init__(self, ps, steps, fail):
        self.ps, self.steps, self.fail = ps, steps, fail

    def replay(self):
        if self.fail:
            raise RuntimeError("hipGraphLaunch failed (test)")
        for _ in range(self.steps):
            self.ps.step(0.01, self.ps._zeta)


def _capturing_part(fail_capture_ranks=(), fail_replay_ranks=()):
    """HostPart that claims capturable collectives (as PartitionedSolver does over RCCL) and whose
    graph() raises on the given ranks, or returns graphs whose replay raises."""
    from tests.host_standins import HostPart

    class CapPart(HostPart):
        def capturable(self):
            return True

        def graph(self, steps, dt, zeta, stop=True):
            self._zeta = zeta
            if self.comm.rank in fail_capture_ranks:
                raise RuntimeError("stream capture of an RCCL collective failed (test)")
            return _Graph(self, steps, self.comm.rank in fail_replay_ranks)

    return CapPart


@pytest.mark.parametrize("fail", ["capture", "replay", "none"])
def test_config5_leg_graph_failure_steps_eagerly(fail):
    """a partition whose HIP-graph capture (or the probe's first replay) raises is still
    timed, eagerly, with graph_steps 0 and the error text in the leg; the digest and the step count
    hold.  fail = none: the graph path (replays) runs every step too."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from odesat_amd import workloads as wl
    wl.CONFIGS["tiny5"] = TINY5
    part = _capturing_part(fail_capture_ranks=(0,) if fail == "capture" else (),
                           fail_replay_ranks=(0,) if fail == "replay" else ())
    r5 = bench.config5_leg(_args(12, 3), 1, 0, 0, None, part_cls=part, config="tiny5")
    d = r5["digest"]
    assert d["variables_bit_exact"] and d["clauses_within_tol"] and d["clauses_rs_within_tol"] and d["steps"] == 15
    for name in ("clauses", "clauses_rs", "variables"):
        leg = r5[name]
        assert leg["value"] > 0
        if fail == "none":
            assert leg["graph_steps"] == 12 and "graph_error" not in leg
        else:
            assert leg["graph_steps"] == 0 and "(test)" in leg["graph_error"], leg


def _cap_worker(rank, world, port, outdir):
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from odesat_amd import workloads as wl
    wl.CONFIGS["tiny5"] = TINY5
    r5 = bench.config5_leg(_args(12, 3), world, rank, 0, td, part_cls=_capturing_part(fail_capture_ranks=(1,)),
                           config="tiny5")
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as fh:
        json.dump(r5, fh)
    td.destroy_process_group()


def test_config5_leg_one_rank_capture_failure_all_ranks_eager(tmp_path):
    """World 2 over gloo: rank 1's capture fails, rank 0's succeeds; both ranks step eagerly (a MAX
    all-reduce of the failure flag), so the collectives stay matched, and the digest holds."""
    import torch.multiprocessing as mp
    mp.spawn(_cap_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (json.load(open(tmp_path / f"r{r}.json")) for r in (0, 1))
    assert r0["digest"]["variables_bit_exact"] and r0["digest"]["steps"] == 15
    for name in ("clauses", "clauses_rs", "variables"):
        assert r0[name]["graph_steps"] == 0 and r1[name]["graph_steps"] == 0
        assert "another rank" in r0[name]["graph_error"] and "(test)" in r1[name]["graph_error"]
