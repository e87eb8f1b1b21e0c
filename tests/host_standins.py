"""Host stand-ins of the device objects bench.py's multi-GPU legs drive, so that those legs run at
world_size > 1 over gloo on a machine without a GPU (tests/test_bench_legs.py).

TEST INFRASTRUCTURE ONLY: they integrate with the C oracle's f32 restatement (oracle/) and the numpy
restatement (oracle/np_oracle.py).  The device solvers themselves are pinned to the same oracle by the
GPU tests (tests/test_gpu_parity.py, tests/test_partition.py); what these stand-ins let a CPU test
check is everything around them: the sharded inter protocol (checkpoint, MIN all-reduce, rollback),
the partitions' collectives over TorchComm, the digests and the bench line's assembly.
"""
import numpy as np

from odesat_amd import _lib
from odesat_amd.partition import CLAUSES, CLAUSES_RS, VARIABLES, local_topology
from odesat_amd.system import ODESAT_STOP_ANY, ODESAT_STOP_EACH
from oracle import np_oracle as npo
from oracle.oracle import Oracle, init_voltages

F32 = np.float32


class HostSolver:
    """odesat_amd.system.Solver's interface over the C f32 oracle: fixed steps only, replicas stepped
    in lock step, the same bookkeeping (run-relative first sat step, steps done, STOP_ANY stop,
    checkpoint / rollback, resume)."""

    def __init__(self, formula, batch, dtype="f32", device=0):
        assert dtype == "f32"
        cp, var, neg = formula.arrays()
        self.o = Oracle(cp, var, neg, formula.varnum, "f32")
        self.batch, self.n, self.m = int(batch), formula.varnum, formula.nclauses
        self.zeta = F32(self.o._fn("default_zeta")(self.o._f))
        self.algorithm = _lib.ODESAT_ALG_FUSED
        self._ms, self._steps, self._prof = 0.0, 0, False
        self._ck = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def close(self):
        pass

    def _reset(self):
        self.t, self.stopped = 0, False
        self.sat = np.full(self.batch, -1, np.int64)
        self.done = np.zeros(self.batch, np.int64)

    def init_state(self, seed, replica0=0):
        self.v = init_voltages(seed, replica0, self.batch, self.n).astype(F32)
        self.xs = np.tile(self.o.init_short_term_memory(), (self.batch, 1))
        self.xl = np.ones((self.batch, self.m), F32)
        self._reset()

    def simulate(self, *, adaptive=False, dt=0.01, tol=1e-3, zeta=None, max_steps=1000, stop=ODESAT_STOP_EACH,
                 poll_interval=0, resume=False):
        import time
        assert not adaptive
        if not resume:
            self._reset()
        z = self.zeta if zeta is None else F32(zeta)
        t0 = time.perf_counter()
        k = 0
        while k < max_steps and not (stop == ODESAT_STOP_ANY and self.stopped):
            for b in range(self.batch):
                if stop == ODESAT_STOP_EACH and self.sat[b] >= 0:
                    continue
                s = self.o.euler_step_fixed(self.v[b], self.xs[b], self.xl[b], F32(dt), z)
                self.done[b] += 1
                if s and self.sat[b] < 0:
                    self.sat[b] = self.t
            self.t += 1
            k += 1
            if stop == ODESAT_STOP_ANY and (self.sat >= 0).any():
                self.stopped = True
        if self._prof:
            self._ms += (time.perf_counter() - t0) * 1e3
            self._steps += k
        return {"first_sat_step": self.sat.copy(), "steps_done": self.done.copy(),
                "dt": np.full(self.batch, dt), "steps_run": k}

    def checkpoint(self):
        self._ck = [x.copy() for x in (self.v, self.xs, self.xl, self.sat, self.done)] + [self.t, self.stopped]

    def rollback(self):
        assert self._ck is not None
        self.v, self.xs, self.xl, self.sat, self.done = (x.copy() for x in self._ck[:5])
        self.t, self.stopped = self._ck[5:]

    def get_state(self, r0=0, count=None):
        count = self.batch - r0 if count is None else count
        sl = slice(r0, r0 + count)
        return (self.v[sl].astype(np.float64), self.xs[sl].astype(np.float64), self.xl[sl].astype(np.float64))

    def synchronize(self):
        pass

    def profile(self, enable):
        self._prof = bool(enable)
        if enable:
            self._ms, self._steps = 0.0, 0

    def profile_read(self):
        return np.array([self._ms, 0.0, 0.0]), np.array([max(self._steps, 1), 0, 0], np.int64)

    def step_kernel(self, adaptive=False):
        return "k_step"

    def clause_kernel_bytes(self):
        return self.batch * (2 * self.n + 4 * self.m) * 4


class HostPart:
    """odesat_amd.partition.PartitionedSolver's interface (one rank of `comm.world`), with the rank's
    kernels restated by np_oracle in f32 and the collectives through the real communicator (TorchComm
    over gloo in the tests).  Local clauses in file order, so the fold order is the reference's."""

    def __init__(self, cp, var, neg, n, mode=VARIABLES, comm=None, device=0, order="file"):
        import torch
        self.comm, self.mode, self.n = comm, int(mode), int(n)
        self.topo = t = local_topology(cp, var, neg, n, mode, comm.rank, comm.world, order="file")
        self.m = t["m"]
        self.f = npo.Formula(t["clause_ptr"], t["var"], t["neg"].astype(bool), self.n)
        S, W = t["block"], comm.world
        z = torch.zeros
        if self.mode == CLAUSES:
            self.v, self.out = z(self.n), z(self.n + 1)
        else:
            self.v = z(W * (S + 1))
            self.out = z(S + 1) if self.mode == VARIABLES else z(W * (S + 1))
            self.blk, self.send = z(S + 1), z(S + 1)
        self.steps = 0

    def _vidx(self):
        i = np.arange(self.n)
        return i if self.mode == CLAUSES else i + i // self.topo["block"]

    def set_state(self, v, xs, xl):
        import torch
        host = np.ones(self.v.numel(), F32)
        host[self._vidx()] = np.asarray(v, np.float64).astype(F32)
        self.v.copy_(torch.from_numpy(host))
        loc = self.topo["clauses"]
        self.xs = np.asarray(xs, np.float64)[loc].astype(F32)
        self.xl = np.asarray(xl, np.float64)[loc].astype(F32)
        self.steps = 0

    def step(self, dt, zeta, stop=True):
        import torch
        T = F32
        v = self.v.numpy()[self._vidx()].copy()
        dv, dxs, dxl, allsat, _ = npo.compute_derivatives(self.f, v, self.xs, self.xl, T(zeta), T)
        self.xs = np.fmin(np.fmax(self.xs + T(dt) * dxs, T(0.001)), T(1.0) - T(0.001)).astype(T)
        self.xl = np.fmin(np.fmax(self.xl + T(dt) * dxl, T(1.0)), T(1e4) * T(self.m)).astype(T)
        uns = T(0.0 if allsat else 1.0)
        S, r, W = self.topo["block"], self.comm.rank, self.comm.world
        clamp = lambda a: np.fmin(np.fmax(a, T(-1.0)), T(1.0)).astype(T)  # noqa: E731
        if self.mode == VARIABLES:
            o = np.zeros(S + 1, T)
            own = slice(self.topo["v0"], self.topo["v1"])
            o[:own.stop - own.start] = clamp(v[own] + T(dt) * dv[own])
            o[S] = uns
            self.out.copy_(torch.from_numpy(o))
            self.comm.all_gather(self.v, self.out)
        elif self.mode == CLAUSES:
            self.out.copy_(torch.from_numpy(np.concatenate([dv, [uns]]).astype(T)))
            self.comm.all_reduce_sum(self.out)
            self.v.copy_(torch.from_numpy(clamp(v + T(dt) * self.out.numpy()[:self.n])))
        else:  # CLAUSES_RS
            full = np.zeros(W * (S + 1), T)
            full[self._vidx()] = dv
            full[S::S + 1] = uns
            self.out.copy_(torch.from_numpy(full))
            self.comm.reduce_scatter_sum(self.blk, self.out)
            b = self.blk.numpy()
            own = slice(r * S, min(self.n, (r + 1) * S))
            snd = np.zeros(S + 1, T)
            snd[:own.stop - own.start] = clamp(v[own] + T(dt) * b[:own.stop - own.start])
            snd[S] = b[S]
            self.send.copy_(torch.from_numpy(snd))
            self.comm.all_gather(self.v, self.send)
        self.steps += 1

    def capturable(self):
        return False

    def status(self, stop=True):
        return {"steps_done": self.steps, "first_sat_step": -1, "frozen": False}

    def get_state(self):
        v = self.v.numpy()[self._vidx()].astype(np.float64)
        return v, self.xs.astype(np.float64), self.xl.astype(np.float64), self.topo["clauses"]

    def exchange_bytes(self):
        S = self.topo["block"]
        return {VARIABLES: 4 * (S + 1), CLAUSES: 4 * (self.n + 1),
                CLAUSES_RS: 4 * self.comm.world * (S + 1) + 4 * (S + 1)}[self.mode]

    def close(self):
        pass
