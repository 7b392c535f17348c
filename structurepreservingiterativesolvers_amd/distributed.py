"""Row-partitioned multi-GPU CGMRES: one process per MI355X, RCCL over xGMI.

The reference is single-process; this is the one parallel
strategy the build adds:

* **partition** — field-interleaved contiguous blocks: every field block of
  the field-major vector layout (``swe``: edge RT dofs | interior RT dofs |
  rho; ``lkdv``: u | v | w; ``lkdvRK``: stage x field) is cut into P pieces and
  rank r owns piece r of every field, so halos stay nearest-neighbour.  The
  permutation is internal: inputs are given and outputs returned in the
  reference's ordering.
* **local operator** — the owned rows with columns renumbered
  ``[0, n_local)`` owned, ``[n_local, n_local + n_ghost)`` ghosts (sorted by
  owner).  Each row keeps its entries in the original order, so a local SpMV
  row is bit-identical to the same row of the global SciPy SpMV.
* **halo plan** — ghost requests are exchanged once per operator over a
  gloo side channel (``torch.distributed``); libspis then exchanges ghosts
  with grouped ``ncclSend/ncclRecv`` before every SpMV and all-reduces every
  dot/norm partial array with ``ncclAllReduce`` (include/spis.h).
* every rank runs the same host least-squares on bitwise-identical inputs
  (all-reduced partials, fixed-order sums), so branch decisions agree.

The planning code is plain NumPy and is tested on CPU with world_size 2 gloo
processes (tests/test_distributed.py); the RCCL data path runs in
``bench.py --gpus N`` (one rank per GPU).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import gc
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sps

from . import _lib
from .device import DeviceConstraint  # noqa: F401  (public here for the distributed API)


# ------------------------------------------------------------------------------------------------
# partition + halo planning (host, NumPy)
# ------------------------------------------------------------------------------------------------
class FieldPartition:
    """Field-interleaved contiguous row partition of a field-major vector layout.

    ``field_sizes`` are the consecutive field blocks of the global ordering.
    ``perm[new] = old`` and ``iperm[old] = new``; rank r owns the new indices
    ``[starts[r], starts[r+1])``."""

    def __init__(self, field_sizes, nparts):
        self.field_sizes = [int(s) for s in field_sizes]
        self.nparts = int(nparts)
        self.n = int(sum(self.field_sizes))
        offs = np.concatenate([[0], np.cumsum(self.field_sizes)]).astype(np.int64)
        owned = []
        for r in range(self.nparts):
            pieces = []
            for f, nf in enumerate(self.field_sizes):
                lo = offs[f] + (r * nf) // self.nparts
                hi = offs[f] + ((r + 1) * nf) // self.nparts
                pieces.append(np.arange(lo, hi, dtype=np.int64))
            owned.append(np.concatenate(pieces) if pieces else np.zeros(0, dtype=np.int64))
        self.perm = np.concatenate(owned)
        self.iperm = np.empty(self.n, dtype=np.int64)
        self.iperm[self.perm] = np.arange(self.n, dtype=np.int64)
        self.starts = np.concatenate([[0], np.cumsum([len(o) for o in owned])]).astype(np.int64)

    def owned_old(self, r):
        return self.perm[self.starts[r]:self.starts[r + 1]]

    def n_local(self, r):
        return int(self.starts[r + 1] - self.starts[r])

    def owner_of_new(self, idx_new):
        return np.searchsorted(self.starts, idx_new, side="right") - 1

    def to_local(self, v_global, r):
        """Slice a vector in the reference ordering to rank r's local ordering."""
        return np.ascontiguousarray(np.asarray(v_global)[self.owned_old(r)])

    def from_locals(self, parts):
        """Assemble rank-ordered local vectors back into the reference ordering."""
        out = np.empty(self.n, dtype=np.result_type(*[np.asarray(p).dtype for p in parts]))
        out[self.perm] = np.concatenate([np.asarray(p) for p in parts])
        return out


class LocalOperator:
    """Rank-local rows of a global operator + its ghost columns."""

    def __init__(self, csr, ghosts_new, ghost_owner):
        self.csr = csr                  # n_local x (n_local + n_ghost), int32 indices
        self.ghosts_new = ghosts_new    # new global index of each ghost column
        self.ghost_owner = ghost_owner  # owning rank of each ghost column


def local_operator(A, part: FieldPartition, rank: int) -> LocalOperator:
    """Owned rows of ``A`` (reference ordering) with columns renumbered; entry order kept."""
    A = sps.csr_matrix(A)
    rows = part.owned_old(rank)
    sub = A[rows]  # rows in local order, each row's entries in stored order
    cols_new = part.iperm[sub.indices]
    lo, hi = part.starts[rank], part.starts[rank + 1]
    own = (cols_new >= lo) & (cols_new < hi)
    ghost_cols = np.unique(cols_new[~own])  # sorted by new index == sorted by (owner, index)
    n_local = hi - lo
    local = np.empty(cols_new.shape, dtype=np.int64)
    local[own] = cols_new[own] - lo
    local[~own] = n_local + np.searchsorted(ghost_cols, cols_new[~own])
    csr = sps.csr_matrix(
        (np.ascontiguousarray(sub.data, dtype=np.float64), local.astype(np.int32), sub.indptr.astype(np.int32)),
        shape=(n_local, n_local + len(ghost_cols)),
    )
    return LocalOperator(csr, ghost_cols, part.owner_of_new(ghost_cols))


class HaloPlan:
    """What rank ``rank`` sends to / receives from each neighbour, in neighbour order."""

    def __init__(self, neighbors, send_counts, send_idx, recv_counts, n_ghost):
        self.neighbors = np.asarray(neighbors, dtype=np.int32)
        self.send_counts = np.asarray(send_counts, dtype=np.int32)
        self.send_idx = np.asarray(send_idx, dtype=np.int32)
        self.recv_counts = np.asarray(recv_counts, dtype=np.int32)
        self.n_ghost = int(n_ghost)

    def ctypes_arrays(self):
        return [np.ascontiguousarray(a) for a in (self.neighbors, self.send_counts, self.send_idx, self.recv_counts)]

    def desc(self, keep):
        P = C.POINTER(C.c_int32)
        nb, sc, si, rc = keep
        return _lib.HaloDesc(self.n_ghost, len(nb), nb.ctypes.data_as(P), sc.ctypes.data_as(P),
                             si.ctypes.data_as(P), rc.ctypes.data_as(P))


def halo_plan(op: LocalOperator, part: FieldPartition, rank: int, allgather) -> HaloPlan:
    """Build the halo plan; ``allgather(obj) -> [obj of every rank]`` is the side channel."""
    requests = {}
    for o in np.unique(op.ghost_owner):
        requests[int(o)] = op.ghosts_new[op.ghost_owner == o].astype(np.int64)
    everyone = allgather(requests)
    lo = part.starts[rank]
    sends = {}
    for q, req in enumerate(everyone):
        if q != rank and rank in req:
            sends[q] = (np.asarray(req[rank], dtype=np.int64) - lo).astype(np.int32)
    neighbors = sorted(set(requests) | set(sends))
    send_counts = [len(sends.get(q, ())) for q in neighbors]
    recv_counts = [len(requests.get(q, ())) for q in neighbors]
    send_idx = np.concatenate([sends[q] for q in neighbors if q in sends]) if sends else np.zeros(0, np.int32)
    return HaloPlan(neighbors, send_counts, send_idx, recv_counts, len(op.ghosts_new))


def is_exactly_symmetric(M) -> bool:
    """M equals its transpose entry by entry (values included): K7t's pairing condition."""
    M = sps.csr_matrix(M)
    if M.shape[0] != M.shape[1]:
        return False
    D = (M - M.T).tocsr()
    D.eliminate_zeros()
    return D.nnz == 0


def local_global_ids(op: LocalOperator, part: FieldPartition, rank: int):
    """Global (partition-ordered) index of each local column: owned columns first, in the rows'
    order, then the ghosts."""
    lo = part.starts[rank]
    n_local = op.csr.shape[0]
    return np.concatenate([np.arange(lo, lo + n_local, dtype=np.int64), op.ghosts_new.astype(np.int64)])


def set_global_numbering(Md, op: LocalOperator, part: FieldPartition, rank: int, symmetric: bool):
    gid = np.ascontiguousarray(local_global_ids(op, part, rank))
    _lib.check(Md.ctx.L.spis_matrix_set_global(Md.handle, gid.ctypes.data_as(C.POINTER(C.c_int64)),
                                                1 if symmetric else 0), "spis_matrix_set_global")


def emulate_spmv(op: LocalOperator, plan: HaloPlan, x_local, exchange):
    """NumPy reference of the distributed SpMV data path (for CPU tests):
    ``exchange(send_bufs_by_neighbor) -> recv_bufs_by_neighbor``."""
    sends = {}
    off = 0
    for q, cnt in zip(plan.neighbors, plan.send_counts):
        sends[int(q)] = x_local[plan.send_idx[off:off + cnt]]
        off += cnt
    recvs = exchange(sends)
    ghosts = np.concatenate([recvs[int(q)] for q, c in zip(plan.neighbors, plan.recv_counts) if c > 0]) \
        if plan.n_ghost else np.zeros(0)
    return op.csr @ np.concatenate([x_local, ghosts])


# ------------------------------------------------------------------------------------------------
# runtime: RCCL bootstrap + distributed handles
# ------------------------------------------------------------------------------------------------
@contextlib.contextmanager
def _stdout_to_stderr():
    """File descriptor 1 points at stderr inside the block (native libraries print there too)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _host_collective(dist):
    """spis_host_coll_fn over torch.distributed (gloo): the in-place sum of an all-reduce, and a
    halo exchange's sends / receives to and from each neighbour (non-blocking, then all waited)."""
    import torch

    def coll(_user, op, buf, count, n_nbr, nbr, scnt, rcnt, recv):
        try:
            if op == _lib.COLL_ALLREDUCE:
                if count > 0:
                    dist.all_reduce(torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,))))
                return 0
            sc = [int(scnt[i]) for i in range(n_nbr)]
            rc = [int(rcnt[i]) for i in range(n_nbr)]
            send = np.ctypeslib.as_array(buf, shape=(count,)) if count > 0 else np.zeros(0)
            rv = np.ctypeslib.as_array(recv, shape=(sum(rc),)) if sum(rc) > 0 else np.zeros(0)
            reqs, so, ro = [], 0, 0
            for i in range(n_nbr):
                peer = int(nbr[i])
                if sc[i] > 0:
                    reqs.append(dist.isend(torch.from_numpy(send[so:so + sc[i]]), peer))
                if rc[i] > 0:
                    reqs.append(dist.irecv(torch.from_numpy(rv[ro:ro + rc[i]]), peer))
                so, ro = so + sc[i], ro + rc[i]
            for r in reqs:
                r.wait()
            return 0
        except Exception:  # noqa: BLE001 — reported to the library as a failed collective
            import traceback

            traceback.print_exc()
            return 1

    return _lib.HOST_COLL_FN(coll)


class Comm:
    """torch.distributed (gloo side channel) + the libspis RCCL communicator.

    ``transport="host"`` (or ``SPIS_TRANSPORT=host``) runs the same several-rank code path with the
    collectives staged through host memory and done over gloo (spis_comm_init_host): several
    ranks can then share one GPU (``SPIS_DEVICE``), which RCCL refuses.  For rehearsal and tests,
    not for measurement."""

    def __init__(self, ctx=None, transport=None):
        # gloo reports its peer connections on stdout while the group forms; keep stdout for
        # bench.py's one JSON line
        with _stdout_to_stderr():
            self._init(ctx, transport)

    def _init(self, ctx, transport):
        import torch.distributed as dist

        if not dist.is_initialized():
            if "RANK" not in os.environ and "WORLD_SIZE" not in os.environ:
                # a plain `python` process (no launcher): a one-rank group on a free local port
                import socket

                with socket.socket() as s:
                    s.bind(("127.0.0.1", 0))
                    port = s.getsockname()[1]
                dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
            else:
                dist.init_process_group("gloo", init_method="env://")
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        from .device import get_context

        local_rank = int(os.environ.get("LOCAL_RANK", self.rank))
        # SPIS_DEVICE pins every rank to one device (rehearsing several ranks on a one-GPU box)
        dev = int(os.environ["SPIS_DEVICE"]) if "SPIS_DEVICE" in os.environ else local_rank
        self.ctx = ctx or get_context(dev)
        L = self.ctx.L
        self.transport = transport or os.environ.get("SPIS_TRANSPORT", "rccl")
        if self.transport == "host":
            self._coll = _host_collective(dist)
            _lib.check(L.spis_comm_init_host(self.ctx.handle, self.world, self.rank, self._coll, None),
                       "spis_comm_init_host")
            # the library keeps the raw function pointer on the (process-wide, cached) context:
            # the thunk must live as long as the context, not as long as this Comm
            self.ctx._host_coll = self._coll
        elif self.transport == "rccl":
            uid = (C.c_uint8 * 128)()
            if self.rank == 0:
                _lib.check(L.spis_comm_unique_id(uid), "spis_comm_unique_id")
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0)
            uid = (C.c_uint8 * 128).from_buffer_copy(box[0])
            _lib.check(L.spis_comm_init(self.ctx.handle, self.world, self.rank, uid), "spis_comm_init")
        else:
            raise ValueError(f"unknown transport {self.transport!r} (rccl or host)")
        self.ctx.nranks, self.ctx.rank = self.world, self.rank

    def transport_size(self):
        """(ranks, transport) as the library's communicator reports them (spis_comm_size): RCCL's
        own ncclCommCount for ``rccl``, the count the host transport was given for ``host``."""
        n, t = C.c_int32(0), C.c_int32(0)
        _lib.check(self.ctx.L.spis_comm_size(self.ctx.handle, C.byref(n), C.byref(t)), "spis_comm_size")
        return int(n.value), {0: None, 1: "rccl", 2: "host"}[int(t.value)]

    def allgather(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def barrier(self):
        self.ctx.synchronize()
        self.dist.barrier()

    def max(self, value):
        import torch

        t = torch.tensor([float(value)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


class DistributedSystem:
    """A global operator distributed over the ranks of ``comm`` (every rank passes
    the same global SciPy matrix; each keeps its rows).  ``vector``/``matrix``
    map further global vectors / operators (constraints) onto the partition."""

    def __init__(self, comm: Comm, A_global, field_sizes):
        from .device import DeviceMatrix

        self.comm = comm
        self.part = FieldPartition(field_sizes, comm.world)
        self.rank = comm.rank
        self.n_local = self.part.n_local(self.rank)
        op = local_operator(A_global, self.part, self.rank)
        plan = halo_plan(op, self.part, self.rank, comm.allgather)
        self.A = DeviceMatrix(comm.ctx, op.csr, halo=plan)
        self.op, self.plan = op, plan

    def vector(self, v_global):
        from .device import DeviceVector

        return DeviceVector.from_host(self.part.to_local(v_global, self.rank), ctx=self.comm.ctx)

    def matrix(self, M_global):
        """A further global operator (a constraint matrix) on this partition.  Its local columns'
        global indices and whether M_global is exactly symmetric go to the library
        (spis_matrix_set_global), so the constraint Gram pairs (r, c) with (c, r) across ranks."""
        from .device import DeviceMatrix

        op = local_operator(M_global, self.part, self.rank)
        plan = halo_plan(op, self.part, self.rank, self.comm.allgather)
        Md = DeviceMatrix(self.comm.ctx, op.csr, halo=plan)
        set_global_numbering(Md, op, self.part, self.rank, is_exactly_symmetric(M_global))
        return Md

    def gather(self, x_local):
        """All local pieces -> the global vector in the reference ordering (every rank)."""
        parts = self.comm.allgather(np.asarray(x_local))
        return self.part.from_locals(parts)


# DeviceConstraint (imported above) takes rank-local operators: sysd.matrix / sysd.vector
_DevCon = DeviceConstraint


def swe_fields(M):
    """Field blocks of the synthetic swe ordering (swe/assembly.py): edge RT dofs,
    interior RT dofs, rho — each sliced into pieces by mesh row."""
    return [6 * M * M, 4 * M * M, 2 * M * M]


def lkdv_fields(n):
    """lkdv's field-major ordering u | v | w (``lkdv/lkdv.py:111,122``, lkdv/assembly.py)."""
    return [n // 3] * 3


def lkdvrk_fields(s, n):
    """lkdvRK's stage-major ordering (``lkdvRK/lkdvRK.py:171-172``): stage i's block
    ``zbig[i*dof:(i+1)*dof]``, each field-major u | v | w, so ``3 s`` consecutive stage x field
    blocks.  Cutting every block into P pieces keeps the couplings of ``A = I_s (x) M_t + dt
    (A_GL (x) K)`` (``lkdvRK/lkdvRK.py:107-118``) and of the lifted constraints ``kron(P'P, M)``
    (``lkdvRK/LinearSolver.py:48-49``) between nearest-neighbour ranks: every stage block has the
    same 1-D band structure, and piece r of stage i couples to pieces r-1 .. r+1 of stage j."""
    dof = n // s
    return [dof // 3] * (3 * s)


def distribute_constraints(sysd, conlist):
    """Host class-form constraints ``(M, v, c)`` (reference ordering) -> rank-local device
    constraints: ``M`` by :meth:`DistributedSystem.matrix` (its own halo plan), ``v`` by
    :meth:`DistributedSystem.vector`; an all-zero ``M`` (the ``0*A`` mass) or ``v`` is dropped, as
    ``solvers.cgmres`` does per call."""
    out = []
    for con in conlist:
        M = getattr(con, "M", None)
        Md = None
        if M is not None:
            Ms = sps.csr_matrix(M)
            if Ms.nnz and np.any(Ms.data):
                Md = sysd.matrix(Ms)
        v = getattr(con, "v", None)
        vd = None
        if v is not None:
            va = np.asarray(v, dtype=np.float64).reshape(-1)
            if np.any(va):
                vd = sysd.vector(va)
        out.append(DeviceConstraint(Md, vd, float(np.asarray(getattr(con, "c", 0.0)))))
    return out


def dist_workload(config, P, M_override=None):
    """The global problem of a SURVEY §8 configuration on P ranks: (A, b, host class constraints,
    field blocks, scaling, description, normalisation of the reported value).

    c3: swe weak scaling, ~1.0e6 DoF per GPU (global M = 289 sqrt(P)), mass + energy;
    c5: swe M = 913 (N = 10,002,828) + the synthetic third constraint, strong scaling (restarted);
    c4: lkdvRK GL(3) M = 16,667 (N = 300,006), the three invariants lifted to (M, v, c), strong;
    c2: lkdv DG1, ~1.0e5 DoF per GPU (M = 16,667 P), mass + momentum + energy, weak."""
    if config in ("c3", "c5"):
        from .swe import LinearSolver as ls
        from .swe import assembly

        M = M_override or (913 if config == "c5" else int(round(289 * np.sqrt(P))))
        dic, _ = assembly.linforms(M=M)
        n = dic["A"].shape[0]
        cons = ls.constraints(dic, np.zeros(n))
        desc = f"swe-shaped RT2xDG0 CSR, global N={n:,} DoF (M={M})"
        if config == "c5":
            D, c3 = assembly.extra_constraint(n, dic["z0"], seed=2)
            cons.append(ls._Constraint(D, np.zeros(n), c3))
            desc += ", mass+energy+synthetic constraints (config C5)"
        else:
            desc += ", mass+energy constraints (config C3 per GPU)"
        return dict(A=dic["A"], b=dic["b"], conlist=cons, fields=swe_fields(M), desc=desc,
                    scaling="strong" if config == "c5" else "weak", norm=n / 1002252.0)
    if config == "c4":
        from .lkdvRK import LinearSolver as ls
        from .lkdvRK import assembly

        M = M_override or 16667
        dic, prob = assembly.linforms(M=M, tstages=3)
        n = dic["A"].shape[0]
        return dict(A=dic["A"], b=dic["b"], conlist=ls.constraints(dic, prob, lift=True),
                    fields=lkdvrk_fields(3, n), scaling="strong", norm=1.0,
                    desc=f"lkdvRK GL(3) block-stage CSR (config C4, M={M}), global N={n:,} DoF, 3 invariants "
                         "lifted to (M, v, c) form")
    if config == "c2":
        from .lkdv import LinearSolver as ls
        from .lkdv import assembly

        M = M_override or 16667 * P
        dic, _ = assembly.linforms(M=M)
        n = dic["A"].shape[0]
        return dict(A=dic["A"], b=dic["b"], conlist=ls.constraints(dic, np.zeros(n)), fields=lkdv_fields(n),
                    scaling="weak", norm=n / 100002.0,
                    desc=f"lkdv DG1 CSR, global N={n:,} DoF (M={M}), mass+momentum+energy (config C2 per GPU)")
    raise ValueError(f"no multi-GPU workload for config {config!r}")


# ------------------------------------------------------------------------------------------------
# bench.py --gpus N
# ------------------------------------------------------------------------------------------------
def bench_main(args, metric):
    from . import solvers
    from .device import DeviceVector

    comm = Comm()
    P = comm.world
    want = getattr(args, "gpus", P)
    if P != want:
        raise RuntimeError(f"bench.py --gpus {want} but the process group has {P} rank(s): launch with "
                           "torch.distributed.run --nproc-per-node N, or without a launcher (bench.py then "
                           "spawns the N ranks itself)")
    comm_ranks, comm_transport = comm.transport_size()
    if comm_ranks != P:
        raise RuntimeError(f"the {comm_transport} communicator has {comm_ranks} rank(s), the process group {P}")
    config = getattr(args, "config", "c3")
    wl = dist_workload(config, P, args.M)
    A = wl["A"]
    n_glob = A.shape[0]
    sysd = DistributedSystem(comm, A, wl["fields"])
    ctx = comm.ctx
    if getattr(args, "orthog", "mgs") == "cgs2":
        _lib.check(ctx.L.spis_set_option(ctx.handle, _lib.OPT_ORTHOG, 1), "spis_set_option")
    _lib.check(ctx.L.spis_set_option(ctx.handle, _lib.OPT_DIST_MGS, getattr(args, "dist_mgs", 1)), "spis_set_option")
    if hasattr(args, "nt_basis"):  # bench.py's shared solver flags
        _lib.check(ctx.L.spis_set_option(ctx.handle, _lib.OPT_NT_BASIS, args.nt_basis), "spis_set_option")
    bd = sysd.vector(wl["b"])
    x0d = DeviceVector.from_host(np.zeros(sysd.n_local), ctx=ctx)
    conlist = distribute_constraints(sysd, wl["conlist"])
    cycles = args.cycles if config == "c5" else 1

    def solve():
        if cycles > 1:
            return solvers.cgmres_restarted(sysd.A, bd, x0d, args.k, cycles, tol=args.tol, conlist=conlist)
        return solvers.cgmres(sysd.A, bd, x0d, args.k, tol=args.tol, conlist=conlist)

    # the warm-up holds each result as the timed loop does, so both pooled workspaces exist before
    # the clock starts (bench.py)
    d = None
    for _ in range(args.warmup):
        _, d = solve()
    L = ctx.L
    _lib.check(L.spis_profile_enable(ctx.handle, args.prof_period), "spis_profile_enable")
    gc.collect()
    gc.freeze()  # the set-up's objects out of the collector's walk during the timed loop (bench.py)
    comm.barrier()
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        _, d = solve()
        iters += d["steps"]
    ctx.synchronize()
    t1 = time.perf_counter()
    comm.dist.barrier()
    elapsed = comm.max(t1 - t0)
    ms, cnt = _lib.profile_read(L, ctx.handle)
    _lib.check(L.spis_profile_enable(ctx.handle, 0), "spis_profile_enable")
    nnz_local = int(sysd.op.csr.nnz)
    S = 12 * nnz_local + 4 * (sysd.n_local + 1) + 16 * sysd.n_local
    spmv_ms = ms[_lib.PROF_SPMV] / max(cnt[_lib.PROF_SPMV], 1)
    kname = "spmv_pipe_kernel (Arnoldi SpMV, solvers.py:191; local rows of rank 0)"
    if cnt[_lib.PROF_SPMV_DUAL] > 0:  # fused residual + Arnoldi SpMV: the dominant SpMV launch
        S = 12 * nnz_local + 4 * (sysd.n_local + 1) + 32 * sysd.n_local
        spmv_ms = ms[_lib.PROF_SPMV_DUAL] / cnt[_lib.PROF_SPMV_DUAL]
        kname = ("spmv_pipe_kernel<2048, 4> (true-residual SpMV of x_j, solvers.py:290, fused with the Arnoldi "
                 "SpMV of z_{j+2}, :191; local rows of rank 0)")
    spmv_gbs = S / (spmv_ms * 1e-3) / 1e9 if spmv_ms > 0 else 0.0
    mgs_ms = ms[_lib.PROF_MGS] / max(cnt[_lib.PROF_MGS], 1)
    if comm.rank == 0:
        out = {
            "metric": metric,
            "value": iters * wl["norm"] / elapsed,
            "unit": "iterations/s",
            "n_gpus": P,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": wl["desc"] + f", row-partitioned over {P} GPUs (~{n_glob // P:,} DoF/GPU), "
                            f"CGMRES(k={args.k}, tol={args.tol:g})" + (f" restarted x{cycles}" if cycles > 1 else "")
                            + (f"; value = global iterations x {wl['norm']:.4g} (global DoF / the single-GPU "
                               "config's) / s" if wl["norm"] != 1.0 else "; value = global iterations / s"),
                "config": config,
                # several GPUs: MGS's projections in one-reduce (inverse compact WY) form, K2w
                "orthogonalisation": ("cgs2" if getattr(args, "orthog", "mgs") == "cgs2" else
                                      "mgs-icwy" if getattr(args, "dist_mgs", 1) == 1 else "mgs"),
                "global_dof": n_glob,
                "k": args.k,
                "parallelism": f"row partition x{P}, " + ("RCCL allreduce + halo send/recv" if comm.transport == "rccl" else
                                                          "host-staged gloo collectives (SPIS_TRANSPORT=host: a "
                                                          "rehearsal of the path, not a measurement)"),
                "global_iterations_per_s": iters / elapsed,
                # the communicator's own rank count (ncclCommCount through spis_comm_size)
                "rccl_ranks": comm_ranks if comm_transport == "rccl" else None,
                "comm_ranks": comm_ranks,
                "transport": comm_transport,
                "launch": os.environ.get("SPIS_BENCH_LAUNCH", "torch.distributed.run"),
            },
            "roofline": {
                "kernel": kname,
                "bound": "hbm",
                "achieved": spmv_gbs,
                "peak": 8000.0,
                "unit": "GB/s",
                "frac": spmv_gbs / 8000.0,
                "traffic": None,
                "algorithmic_bytes_per_launch": S,
                "avg_launch_us": 1e3 * spmv_ms,
            },
            "kernels": {"mgs_us_mean": 1e3 * mgs_ms, "spmv_us": 1e3 * spmv_ms},
        }
        # the reference's CPU path on the same global system, at one rank only (several ranks: the
        # N = 1 line carries it, and the other ranks would wait at the barrier for the sample)
        if not args.no_cpu_baseline and P == 1:
            import bench as _bench

            out["cpu_baseline"] = _bench.cpu_baseline(wl, wl["conlist"], args.k, args.tol, args.cpu_budget)
        print(json.dumps(out))
    comm.dist.barrier()
