"""One very large instance across GPUs: BASELINE configs[4] ("single instance n=1M vars m=4.2M
clauses, clause-partitioned across 8 GPUs, RCCL all-reduce on dv each step"), SURVEY.md §8e.

The fixed Euler step of ONE replica (system.rs:141-154, driven like simulate, :156-239) with the
formula split over `world` ranks, one process per GPU.  The per-rank kernels are in
csrc/partition.hip (include/odesat.h, odesat_part_*); this module builds each rank's local topology
on the host and runs the collective through a communicator (torch.distributed over RCCL on GPU
boxes, gloo on CPU, or an in-process stand-in for tests).

Two partitions:
  CLAUSES    (the north star's design) rank r owns a contiguous slice of the clauses and a full v.
             Each step it writes the partial dv of every variable (its clauses' terms, folded in
             clause order) and its unsat count; one all-reduce (sum) of n + 1 floats, then every
             rank applies the same update.  Reordering the fold across ranks makes this match the
             reference within a tolerance (bit-exact at world = 1).
  VARIABLES  rank r owns the variables [r S, (r + 1) S) and every clause touching them (a clause
             spanning ranks is evaluated, identically, by each).  Each step it folds the complete
             dv of its own variables in the reference's order and updates them; one all-gather of
             S + 1 floats per rank (half an all-reduce's traffic) rebuilds v.  Bit-exact for any
             world size.
  CLAUSES_RS the CLAUSES slice with the all-reduce split into its halves: the
             partial dv is reduce-scattered (sum) onto the ranks' variable blocks of S, each rank
             updates its own block, and an all-gather of the blocks rebuilds v (VARIABLES' layout).
             Tolerance parity as CLAUSES (bit-exact at world = 1).
The replica's bookkeeping (steps done, first sat step, frozen after it) lives on the device, so the
host polls the stop condition at any interval without changing results.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import ODESAT_PART_CLAUSES as CLAUSES
from ._lib import ODESAT_PART_CLAUSES_RS as CLAUSES_RS
from ._lib import ODESAT_PART_VARIABLES as VARIABLES
from ._lib import check, lib

__all__ = ["CLAUSES", "CLAUSES_RS", "VARIABLES", "MODES", "block_size", "local_topology", "default_zeta",
           "PartitionedSolver", "TorchComm", "LocalComm", "step_in_process"]

MODES = {"clauses": CLAUSES, "variables": VARIABLES, "clauses_rs": CLAUSES_RS}


def block_size(n: int, world: int) -> int:
    """Variables per rank in the VARIABLES partition (the last block may be short)."""
    return -(-n // world)


def default_zeta(n: int, m: int) -> float:
    """system.rs:164-173: the learning rate from the clause density."""
    d = m / n
    return 0.1 if d >= 6.0 else (0.01 if d >= 4.9 else 0.001)


def local_topology(cp, var, neg, n: int, mode: int, rank: int, world: int, order: str = "minvar") -> dict:
    """Rank `rank`'s share of a normalised formula (clause_ptr cp[m+1], var[L], neg[L]).

    Returns the local clauses (global indices) in the order the clause kernel processes them, their
    CSR, the variable range [v0, v1) this rank folds, and for each of those variables its local
    literal slots in the reference's clause-then-literal order -- the order of its dv accumulation
    (system.rs:35, :62, :80), whatever the processing order.  order = "file" keeps the reference's
    clause order; "minvar" (default) sorts the clauses by their smallest variable, so neighbouring
    threads gather neighbouring voltages and write neighbouring terms (a random instance has no other
    locality to offer)."""
    cp = np.asarray(cp, np.int64)
    var = np.asarray(var, np.int64)
    neg = np.asarray(neg, np.uint8)
    m = len(cp) - 1
    if not (0 <= rank < world):
        raise ValueError("bad rank / world")
    lens_all = np.diff(cp)
    if mode in (CLAUSES, CLAUSES_RS):
        c0, c1 = rank * m // world, (rank + 1) * m // world
        local = np.arange(c0, c1, dtype=np.int64)
        v0, v1, S = 0, n, (block_size(n, world) if mode == CLAUSES_RS else 0)
    elif mode == VARIABLES:
        S = block_size(n, world)
        v0, v1 = min(n, rank * S), min(n, (rank + 1) * S)
        owner = np.repeat(np.arange(m, dtype=np.int64), lens_all)
        touch = np.zeros(m, bool)
        touch[owner[(var >= v0) & (var < v1)]] = True
        # a clause with no literal touches no variable, but it is never satisfied (system.rs:43-57
        # leaves its C at infinity): rank 0 holds it, so its unsat flag reaches the stop check
        touch[lens_all == 0] = rank == 0
        local = np.flatnonzero(touch).astype(np.int64)
    else:
        raise ValueError("mode must be CLAUSES, VARIABLES or CLAUSES_RS")
    if order not in ("file", "minvar"):
        raise ValueError("order must be 'file' or 'minvar'")
    if order == "minvar" and len(local) and len(var):
        owner = np.repeat(np.arange(m, dtype=np.int64), lens_all)
        vmin = np.full(m, n, np.int64)
        np.minimum.at(vmin, owner, var)
        local = local[np.argsort(vmin[local] * m + local)]  # unique keys: = a stable sort by vmin
    lens = lens_all[local]
    lcp = np.zeros(len(local) + 1, np.int64)
    np.cumsum(lens, out=lcp[1:])
    L = int(lcp[-1])
    gslot = np.repeat(cp[local], lens) + (np.arange(L, dtype=np.int64) - np.repeat(lcp[:-1], lens))
    lvar, lneg = var[gslot], neg[gslot]
    sel = np.flatnonzero((lvar >= v0) & (lvar < v1))
    # per variable: ascending global slot = clause, literal order (one argsort of unique int64 keys;
    # np.lexsort over the two columns is 3x slower at config 5's 12.6 M literals)
    inc = sel[np.argsort(lvar[sel] * (int(cp[-1]) + 1) + gslot[sel])]
    counts = np.bincount(lvar[sel] - v0, minlength=v1 - v0)
    vptr = np.zeros(v1 - v0 + 1, np.int64)
    np.cumsum(counts, out=vptr[1:])
    return {"clauses": local, "clause_ptr": lcp, "var": lvar, "neg": lneg, "v0": int(v0), "v1": int(v1),
            "var_ptr": vptr, "inc_slot": inc.astype(np.int64), "block": int(S), "n": int(n), "m": int(m)}


class TorchComm:
    """The collective over a torch.distributed process group (RCCL "nccl" moves device tensors;
    gloo stages them through host memory)."""

    def __init__(self, dist):
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.staged = dist.get_backend() != "nccl"

    def all_gather(self, out, block):
        if self.staged:
            o = out.cpu()
            self.dist.all_gather_into_tensor(o, block.cpu())
            out.copy_(o)
        else:
            self.dist.all_gather_into_tensor(out, block)

    def all_reduce_sum(self, t):
        if self.staged:
            h = t.cpu()
            self.dist.all_reduce(h)
            t.copy_(h)
        else:
            self.dist.all_reduce(t)

    def reduce_scatter_sum(self, block, full):
        """block (this rank's len(full) / world floats) = the sum over ranks of full's block."""
        if self.staged:  # gloo has no reduce-scatter: all-reduce on the host, keep this rank's block
            h = full.cpu()
            self.dist.all_reduce(h)
            k = block.numel()
            block.copy_(h[self.rank * k:(self.rank + 1) * k])
        else:
            self.dist.reduce_scatter_tensor(block, full)


class LocalComm:
    """A single rank (world = 1, no collective), or rank `rank` of `world` when a test drives the
    exchange itself (PartitionedSolver.rhs / .post)."""

    def __init__(self, rank: int = 0, world: int = 1):
        self.rank, self.world = rank, world

    def all_gather(self, out, block):
        assert self.world == 1, "LocalComm gathers only at world = 1"
        out.copy_(block)

    def all_reduce_sum(self, t):
        assert self.world == 1, "LocalComm reduces only at world = 1"

    def reduce_scatter_sum(self, block, full):
        assert self.world == 1, "LocalComm reduces only at world = 1"
        block.copy_(full)


class PartitionedSolver:
    """Rank `comm.rank`'s share of one replica of a normalised formula (f32), on `device`."""

    def __init__(self, cp, var, neg, n: int, mode: int = VARIABLES, comm=None, device: int = 0,
                 order: str = "minvar"):
        import torch
        self.comm = comm or LocalComm()
        self.mode, self.n = int(mode), int(n)
        self.topo = t = local_topology(cp, var, neg, n, mode, self.comm.rank, self.comm.world, order=order)
        self.m = t["m"]
        h = C.c_void_p()
        check(lib().odesat_part_create(int(device), self.comm.world, self.n, self.m, len(t["clauses"]),
                                       _lib.i64ptr(t["clause_ptr"]), _lib.i64ptr(t["var"]), _lib.u8ptr(t["neg"]),
                                       t["v0"], t["v1"], _lib.i64ptr(t["var_ptr"]), _lib.i64ptr(t["inc_slot"]),
                                       t["block"], C.byref(h)))
        self._h = h
        self.dev = torch.device("cuda", device)
        f32 = torch.float32
        if self.mode == VARIABLES:
            S = t["block"]
            self.v = torch.ones(self.comm.world * (S + 1), dtype=f32, device=self.dev)  # gathered layout
            self.out = torch.ones(S + 1, dtype=f32, device=self.dev)                      # send block
        elif self.mode == CLAUSES_RS:
            S = t["block"]
            self.v = torch.ones(self.comm.world * (S + 1), dtype=f32, device=self.dev)    # gathered layout
            self.out = torch.ones(self.comm.world * (S + 1), dtype=f32, device=self.dev)  # partial dv, same layout
            self.blk = torch.ones(S + 1, dtype=f32, device=self.dev)                      # reduce-scatter result
            self.send = torch.ones(S + 1, dtype=f32, device=self.dev)                     # all-gather input
        else:
            self.v = torch.zeros(self.n, dtype=f32, device=self.dev)
            self.out = torch.ones(self.n + 1, dtype=f32, device=self.dev)                 # partial dv + unsat

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().odesat_part_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_bytes(self) -> int:
        return int(lib().odesat_part_device_bytes(self._h))

    # -- state --------------------------------------------------------------------------------
    @property
    def _apply(self) -> int:
        """odesat_part_rhs's apply argument: 0 CLAUSES, 1 VARIABLES, 2 CLAUSES_RS."""
        return {CLAUSES: 0, VARIABLES: 1, CLAUSES_RS: 2}[self.mode]

    def _v_index(self):
        i = np.arange(self.n)
        return i + i // self.topo["block"] if self.mode != CLAUSES else i

    def _stream(self):
        import torch
        return C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def set_state(self, v, xs, xl):
        """Full-size host arrays v[n], xs[m], xl[m] (the reference's State, system.rs:6-11); the
        bookkeeping restarts (no step taken, no sat step)."""
        import torch
        loc = self.topo["clauses"]
        xs_l = np.ascontiguousarray(np.asarray(xs, np.float64)[loc])
        xl_l = np.ascontiguousarray(np.asarray(xl, np.float64)[loc])
        check(lib().odesat_part_set_memories(self._h, _lib.dptr(xs_l), _lib.dptr(xl_l)))
        host = np.ones(self.v.numel(), np.float32)  # VARIABLES flag slots read "unsat" until a step runs
        host[self._v_index()] = np.asarray(v, np.float64).astype(np.float32)
        self.v.copy_(torch.from_numpy(host))
        self.out.fill_(1.0)
        if self.mode == CLAUSES_RS:
            self.blk.fill_(1.0)
            self.send.fill_(1.0)
        check(lib().odesat_part_reset(self._h, self._stream()))

    def get_state(self):
        """(v[n], xs_local, xl_local, local clause indices) as host f64 arrays."""
        import torch
        torch.cuda.synchronize(self.dev)
        v = self.v.cpu().numpy()[self._v_index()].astype(np.float64)
        k = len(self.topo["clauses"])
        xs, xl = np.zeros(k), np.zeros(k)
        check(lib().odesat_part_get_memories(self._h, _lib.dptr(xs), _lib.dptr(xl)))
        return v, xs, xl, self.topo["clauses"]

    # -- stepping -----------------------------------------------------------------------------
    def rhs(self, dt: float, zeta: float, stop: bool = True):
        """The rank's local part of a step: right-hand side + memory update into `out`."""
        check(lib().odesat_part_rhs(self._h, C.c_void_p(self.v.data_ptr()), C.c_void_p(self.out.data_ptr()),
                                    float(dt), float(zeta), self._apply, int(stop), self._stream()))

    def post(self, dt: float):
        """After the (first) collective: CLAUSES applies the summed dv; CLAUSES_RS updates this rank's
        block of voltages from its reduce-scattered dv into the all-gather's send block (VARIABLES'
        gather already is v)."""
        if self.mode == CLAUSES:
            check(lib().odesat_part_apply(self._h, C.c_void_p(self.v.data_ptr()), C.c_void_p(self.out.data_ptr()),
                                          float(dt), self._stream()))
        elif self.mode == CLAUSES_RS:
            check(lib().odesat_part_reduce_apply(self._h, C.c_void_p(self.v.data_ptr()),
                                                 C.c_void_p(self.blk.data_ptr()), C.c_void_p(self.send.data_ptr()),
                                                 self.comm.rank, float(dt), self._stream()))

    def exchange_bytes(self) -> int:
        """Bytes this rank contributes to the step's collective(s): the all-gather's block
        (VARIABLES), the all-reduced vector (CLAUSES), or the reduce-scattered vector plus the
        all-gather's block (CLAUSES_RS)."""
        S = self.topo["block"]
        return {VARIABLES: 4 * (S + 1), CLAUSES: 4 * (self.n + 1),
                CLAUSES_RS: 4 * self.comm.world * (S + 1) + 4 * (S + 1)}[self.mode]

    def step(self, dt: float, zeta: float, stop: bool = True):
        """One fixed Euler step of the whole instance (system.rs:141-154), enqueued on torch's
        current stream: local RHS + memory update, the collective(s), the voltage update.  With stop,
        the first allsat step freezes the replica (later steps are no-ops), as simulate does."""
        self.rhs(dt, zeta, stop)
        if self.mode == VARIABLES:
            self.comm.all_gather(self.v, self.out)
        elif self.mode == CLAUSES_RS:
            self.comm.reduce_scatter_sum(self.blk, self.out)
        else:
            self.comm.all_reduce_sum(self.out)
        self.post(dt)
        if self.mode == CLAUSES_RS:
            self.comm.all_gather(self.v, self.send)

    def status(self, stop: bool = True) -> dict:
        """{steps_done, first_sat_step (-1 = none), frozen}; synchronises the stream."""
        sd, ss, fr = C.c_int64(0), C.c_int64(0), C.c_int32(0)
        check(lib().odesat_part_status(self._h, C.c_void_p(self.v.data_ptr()), C.c_void_p(self.out.data_ptr()),
                                       self._apply, int(stop), self._stream(), C.byref(sd), C.byref(ss),
                                       C.byref(fr)))
        return {"steps_done": sd.value, "first_sat_step": ss.value, "frozen": bool(fr.value)}

    def capturable(self) -> bool:
        """A step can be captured into a HIP graph: world 1, or a device collective (RCCL)."""
        return isinstance(self.comm, LocalComm) or not getattr(self.comm, "staged", True)

    def graph(self, steps: int, dt: float, zeta: float, stop: bool = True):
        """`steps` whole steps (RHS + memory update, the collective, the voltage update) captured into
        one HIP graph (torch.cuda.CUDAGraph over the library's launches and the RCCL call): a replay
        costs one host call instead of three per step."""
        import torch
        if not self.capturable():
            raise ValueError("host-staged collectives (gloo) cannot be captured")
        if not isinstance(self.comm, LocalComm):  # the communicator exists before the capture
            if self.mode == VARIABLES:
                self.comm.all_gather(torch.empty_like(self.v), torch.empty_like(self.out))
            elif self.mode == CLAUSES_RS:
                self.comm.reduce_scatter_sum(torch.empty_like(self.blk), torch.zeros_like(self.out))
                self.comm.all_gather(torch.empty_like(self.v), torch.empty_like(self.send))
            else:
                self.comm.all_reduce_sum(torch.zeros_like(self.out))
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                self.step(dt, zeta, stop)
        return g

    def simulate(self, dt: float = 0.01, steps: int = 1000, zeta: float | None = None, stop: bool = True,
                 poll: int = 32, graph: bool | None = None) -> dict:
        """simulate (system.rs:190-203, fixed step): run until the first allsat step (that step's
        update included, :148-152) or `steps`; the stop condition is polled every `poll` steps
        (exact regardless: a frozen replica does not step).  graph (default: when capturable) replays
        `poll` steps per HIP graph launch.  Returns status()."""
        zeta = default_zeta(self.n, self.m) if zeta is None else zeta
        if graph is None:
            graph = self.capturable() and steps >= poll
        if graph:
            g = self.graph(poll, dt, zeta, stop)
            k = 0
            while k + poll <= steps:
                g.replay()
                k += poll
                if stop and k < steps and self.status(stop)["frozen"]:
                    return self.status(stop)
            for _ in range(steps - k):
                self.step(dt, zeta, stop)
            return self.status(stop)
        for k in range(steps):
            self.step(dt, zeta, stop)
            if stop and (k + 1) % poll == 0 and k + 1 < steps and self.status(stop)["frozen"]:
                break
        return self.status(stop)


def step_in_process(parts, dt: float, zeta: float, stop: bool = True):
    """One step of `world` ranks held by ONE process (parts[r] = rank r, LocalComm(r, world), all on
    the same device): every rank's local kernels, with the collectives done in process by torch ops
    -- the same sums (CLAUSES: the ranks' partials added in rank order) and copies an RCCL call
    would make.  Tests and single-GPU timing of a world's per-rank slices use it."""
    import torch
    mode = parts[0].mode
    for p in parts:
        p.rhs(dt, zeta, stop)
    if mode == VARIABLES:
        g = torch.cat([p.out for p in parts])
        for p in parts:
            p.v.copy_(g)
    elif mode == CLAUSES:
        tot = torch.stack([p.out for p in parts]).sum(0)
        for p in parts:
            p.out.copy_(tot)
    else:
        k = parts[0].blk.numel()
        tot = torch.stack([p.out for p in parts]).sum(0)
        for r, p in enumerate(parts):
            p.blk.copy_(tot[r * k:(r + 1) * k])
    for p in parts:
        p.post(dt)
    if mode == CLAUSES_RS:
        g = torch.cat([p.send for p in parts])
        for p in parts:
            p.v.copy_(g)
