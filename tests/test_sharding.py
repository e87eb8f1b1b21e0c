"""Multi-GPU path on CPU: replica sharding + the host reductions, world_size 2 over gloo.

The data path has no collective (independent replicas); these tests cover what does cross ranks:
the replica ranges, the max-over-ranks timing reduction and the global first-sat winner of inter /
batch mode.  Each rank integrates its shard with the C oracle (the CPU checker) -- the device
solver's per-rank results are pinned to the oracle by tests/test_gpu_parity.py."""
import json
import os
import socket

import numpy as np
import pytest

from odesat_amd.sharding import (NO_SAT, global_first_sat, global_first_satisfied, local_first_sat, max_over_ranks,
                                  min_over_ranks, shard_range)


def test_shard_range_disjoint_cover():
    world, per = 4, 37
    flat = []
    for r in range(world):
        first, count = shard_range(r, world, per)
        flat.extend(range(first, first + count))
    assert flat == list(range(world * per))
    with pytest.raises(ValueError):
        shard_range(4, 4, 10)


def test_local_first_sat_tie_break():
    assert local_first_sat(np.array([-1, -1]), 10) == (NO_SAT, NO_SAT)
    assert local_first_sat(np.array([7, 3, -1, 3]), 100) == (3, 101)  # earliest step, lowest index
    assert global_first_sat(None, np.array([5, 2]), 0) == (2, 1)
    assert max_over_ranks(None, 1.5) == 1.5
    # batch's rule (main.rs:302-307): the lowest index that satisfies, whatever its sat step
    assert global_first_satisfied(None, np.array([False, True, True]), 40) == 41
    assert global_first_satisfied(None, np.zeros(3, bool), 0) == NO_SAT
    assert min_over_ranks(None, 7) == 7


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out, per, seed, steps):
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import Oracle, init_voltages
    from tests.common import oracle_formula
    f = oracle_formula("easy")
    o = Oracle(f.clause_ptr, f.var, f.neg, f.varnum, "f64")
    r0, cnt = shard_range(rank, world, per)
    v = init_voltages(seed, r0, cnt, o.n)  # keyed on the GLOBAL replica index
    xs = np.tile(o.init_short_term_memory(), (cnt, 1))
    xl = np.ones((cnt, o.m))
    _, sat, _, _ = o.batch_run(v, xs, xl, False, 1e-3, 0.1, steps, 0.001)
    winner = global_first_sat(td, sat, r0)
    wall = max_over_ranks(td, 1.0 + rank)
    # crafted: rank 0 first sat at step 9, rank 1 at step 4 (replica 3) and 4 (replica 1)
    crafted = np.array([9, -1, -1, -1]) if rank == 0 else np.array([-1, 4, -1, 4])
    cw = global_first_sat(td, crafted, r0 if per == 4 else rank * 4)
    none = global_first_sat(td, np.full(3, -1), rank * 3)
    # batch: rank 0 has no satisfying replica, rank 1 its replicas 2 and 3 -> global 4 + 2
    bsat = np.zeros(4, bool) if rank == 0 else np.array([False, False, True, True])
    bw = global_first_satisfied(td, bsat, rank * 4)
    bnone = global_first_satisfied(td, np.zeros(2, bool), rank * 2)
    if rank == 0:
        with open(out, "w") as fh:
            json.dump({"winner": winner, "wall": wall, "crafted": cw, "none": none, "batch": bw, "batch_none": bnone},
                      fh)
    td.destroy_process_group()


@pytest.mark.parametrize("seed", [3, 11])
def test_two_rank_gloo_matches_single_process(tmp_path, seed):
    import torch.multiprocessing as mp

    from oracle.oracle import Oracle, init_voltages
    from tests.common import oracle_formula
    world, per, steps = 2, 4, 400
    out = str(tmp_path / "r.json")
    mp.spawn(_worker, args=(world, _free_port(), out, per, seed, steps), nprocs=world, join=True)
    res = json.load(open(out))
    # single process over all world*per replicas
    f = oracle_formula("easy")
    o = Oracle(f.clause_ptr, f.var, f.neg, f.varnum, "f64")
    B = world * per
    v = init_voltages(seed, 0, B, o.n)
    xs = np.tile(o.init_short_term_memory(), (B, 1))
    xl = np.ones((B, o.m))
    _, sat, _, _ = o.batch_run(v, xs, xl, False, 1e-3, 0.1, steps, 0.001)
    assert tuple(res["winner"]) == local_first_sat(sat, 0)
    assert res["wall"] == 2.0
    assert tuple(res["crafted"]) == (4, 5)  # rank 1's replica 1 -> global 4 + 1
    assert tuple(res["none"]) == (NO_SAT, NO_SAT)
    assert res["batch"] == 6 and res["batch_none"] == NO_SAT


def test_bench_gpus_without_enough_devices_fails_loudly():
    """`bench.py --gpus 2` starts the ranks itself, and refuses when fewer GPUs are visible (here: none)
    instead of quietly timing one device."""
    import subprocess
    import sys
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs are visible")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "GPU(s) are visible" in r.stderr


def test_bench_counts_gpus_without_hip(tmp_path):
    """bench.py's spawn_ranks counts GPUs from the KFD topology (no HIP call in the launcher's parent):
    GPU nodes only (simd_count > 0), whose render node exists, narrowed by *_VISIBLE_DEVICES."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    for node, simd, minor in ((0, 0, None), (1, 256, 128), (2, 256, 129), (3, 256, 130)):
        d = topo / str(node)
        d.mkdir(parents=True)
        lines = [f"simd_count {simd}"] + ([f"drm_render_minor {minor}"] if minor is not None else [])
        (d / "properties").write_text("\n".join(lines) + "\n")
    for minor in (128, 129):  # node 3's render node is not in this container
        (dri / f"renderD{minor}").write_text("")
    assert bench.visible_gpus(str(topo), str(dri), env={}) == 2
    assert bench.visible_gpus(str(topo), str(dri), env={"HIP_VISIBLE_DEVICES": "0"}) == 1
    assert bench.visible_gpus(str(topo), str(dri), env={"ROCR_VISIBLE_DEVICES": ""}) == 2
    assert bench.visible_gpus(str(tmp_path / "none"), str(dri), env={}) is None
