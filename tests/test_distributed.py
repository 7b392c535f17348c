"""Multi-GPU planning on CPU: field-interleaved partition, local operators with
ghost columns, halo plans exchanged over gloo (world_size 2 processes), and a
NumPy emulation of the distributed data path (halo exchange + local SpMV,
partial-sum all-reduce) checked against the global SciPy results — bit-exact
for the SpMV (entry order is kept per row), identical on every rank for the
reduced dot (fixed-order all-reduce of partial arrays, as libspis does)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from structurepreservingiterativesolvers_amd.distributed import (
    FieldPartition, dist_workload, emulate_spmv, halo_plan, lkdvrk_fields, local_operator, swe_fields)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, problem, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        A, fields, x = _problem(problem)
        part = FieldPartition(fields, world)
        op = local_operator(A, part, rank)

        def allgather(obj):
            o = [None] * world
            dist.all_gather_object(o, obj)
            return o

        plan = halo_plan(op, part, rank, allgather)

        def exchange(sends):
            everyone = allgather({int(q): np.asarray(v) for q, v in sends.items()})
            return {q: everyone[q][rank] for q in range(world) if q != rank and rank in everyone[q]}

        y_local = emulate_spmv(op, plan, part.to_local(x, rank), exchange)
        # reduction exactly as libspis: fixed-size partial arrays summed element-wise across ranks,
        # then summed in a fixed order -> the same scalar on every rank
        xl = part.to_local(x, rank)
        partials = np.zeros(8)
        for i, chunk in enumerate(np.array_split(xl * y_local, 8)):
            partials[i] = chunk.sum()
        import torch
        t = torch.from_numpy(partials)
        dist.all_reduce(t)
        dotv = float(t.numpy().sum())
        ys = allgather(y_local)
        dots = allgather(dotv)
        if rank == 0:
            y = part.from_locals(ys)
            out_q.put((y, dots, int(plan.n_ghost), list(plan.neighbors)))
    finally:
        dist.destroy_process_group()


def _problem(name):
    rng = np.random.default_rng(0)
    if name == "swe":
        from structurepreservingiterativesolvers_amd.swe import assembly
        dic, _ = assembly.linforms(M=12)
        return dic["A"], swe_fields(12), rng.normal(size=dic["A"].shape[0])
    if name in ("lkdvrk", "lkdvrk_lifted"):
        from structurepreservingiterativesolvers_amd.lkdvRK import LinearSolver as rk_ls
        from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra
        dic, prob = ra.linforms(M=40, tstages=3)
        n = dic["A"].shape[0]
        # the operator, or the lifted energy constraint kron(P'P, L - M) (lkdvRK/LinearSolver.py:29-48)
        A = dic["A"] if name == "lkdvrk" else rk_ls.constraints(dic, prob, lift=True)[2].M
        return A, lkdvrk_fields(3, n), rng.normal(size=n)
    from structurepreservingiterativesolvers_amd.lkdv import assembly
    dic, _ = assembly.linforms(M=60)
    n = dic["A"].shape[0]
    return dic["A"], [n // 3] * 3, rng.normal(size=n)


@pytest.mark.parametrize("problem", ["swe", "lkdv", "lkdvrk", "lkdvrk_lifted"])
def test_two_rank_spmv_and_dot(problem):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, problem, q)) for r in range(2)]
    for p in procs:
        p.start()
    y, dots, n_ghost, nbrs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A, fields, x = _problem(problem)
    assert np.array_equal(y, A @ x)  # bit-exact: each local row keeps its entry order
    assert dots[0] == dots[1]
    np.testing.assert_allclose(dots[0], x @ (A @ x), rtol=1e-12)
    if problem == "lkdvrk_lifted":  # kron(P'P, L - M): DG mass blocks couple no cells, so no halo
        assert n_ghost == 0 and nbrs == []
    else:
        assert n_ghost > 0 and nbrs == [1]


def test_partition_roundtrip_and_locality():
    part = FieldPartition(swe_fields(20), 4)
    v = np.arange(part.n, dtype=np.float64)
    parts = [part.to_local(v, r) for r in range(4)]
    assert np.array_equal(part.from_locals(parts), v)
    assert sum(len(p) for p in parts) == part.n
    # field-interleaved: every rank owns a piece of every field block
    offs = np.cumsum([0] + swe_fields(20))
    for r in range(4):
        own = part.owned_old(r)
        for f in range(3):
            assert np.any((own >= offs[f]) & (own < offs[f + 1]))


def test_local_operator_ghosts_are_neighbours_only():
    from structurepreservingiterativesolvers_amd.swe import assembly

    M = 24
    A = assembly.linforms(M=M)[0]["A"]
    part = FieldPartition(swe_fields(M), 4)
    for r in range(4):
        op = local_operator(A, part, r)
        owners = set(op.ghost_owner.tolist())
        assert owners <= {(r - 1) % 4, (r + 1) % 4}, (r, owners)  # strips: periodic neighbours
        assert op.csr.shape[1] == part.n_local(r) + len(op.ghosts_new)
        assert op.csr.indices.dtype == np.int32


@pytest.mark.parametrize("nparts", [2, 4])
def test_lkdvrk_stage_field_partition_nearest_neighbour(nparts):
    """Config C4's row split (lkdvRK GL(3), stage x field blocks): the block-stage operator
    (lkdvRK/lkdvRK.py:107-118) and the lifted constraint matrices kron(P'P, M), kron(P'P, L - M)
    (lkdvRK/LinearSolver.py:29-48, lifted in LinearSolver._lift) only couple a rank to its periodic
    neighbours, every rank owns a piece of every stage x field block, and the local operators'
    rows are the global rows (bit-exact SpMV with the ghosts filled from the global vector)."""
    from structurepreservingiterativesolvers_amd.lkdvRK import LinearSolver as rk_ls
    from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra

    dic, prob = ra.linforms(M=60, tstages=3)
    n = dic["A"].shape[0]
    fields = lkdvrk_fields(3, n)
    assert len(fields) == 9 and sum(fields) == n
    part = FieldPartition(fields, nparts)
    cons = rk_ls.constraints(dic, prob, lift=True)
    rng = np.random.default_rng(1)
    x = rng.normal(size=n)
    offs = np.cumsum([0] + fields)
    for M in (dic["A"], cons[1].M, cons[2].M):
        y = M @ x
        for r in range(nparts):
            op = local_operator(M, part, r)
            owners = set(op.ghost_owner.tolist())
            assert owners <= {(r - 1) % nparts, (r + 1) % nparts}, (r, owners)
            xl = np.concatenate([part.to_local(x, r), x[part.perm[op.ghosts_new]]])
            assert np.array_equal(op.csr @ xl, y[part.owned_old(r)])
    for r in range(nparts):
        own = part.owned_old(r)
        for f in range(len(fields)):
            assert np.any((own >= offs[f]) & (own < offs[f + 1]))


def test_dist_workload_configs():
    """bench.py --gpus N: every SURVEY §8 configuration has a multi-GPU workload (no silent
    fallback to swe): field blocks covering N, class-form constraints, the stated scaling."""
    w = dist_workload("c4", 4, M_override=100)
    assert sum(w["fields"]) == w["A"].shape[0] and len(w["fields"]) == 9
    assert len(w["conlist"]) == 3 and w["scaling"] == "strong" and w["norm"] == 1.0
    w = dist_workload("c3", 2, M_override=20)
    assert sum(w["fields"]) == w["A"].shape[0] and len(w["conlist"]) == 2 and w["scaling"] == "weak"
    w = dist_workload("c5", 2, M_override=20)
    assert len(w["conlist"]) == 3 and w["scaling"] == "strong"
    w = dist_workload("c2", 2, M_override=200)
    assert sum(w["fields"]) == w["A"].shape[0] and len(w["conlist"]) == 3
    with pytest.raises(ValueError):
        dist_workload("c9", 2)


def test_one_reduce_mgs_equals_mgs():
    """The multi-GPU MGS (K2w, kernels.hip icwy_*): h_l = q_l.w - sum_{m<l} h_m G(l, m) from the
    dots q_l.w and the Gram rows G(l, m) = q_l.q_m is MGS's h (solvers.py:193-195) in exact
    arithmetic; in floating point, on an MGS basis, the two agree to roundoff and the updated
    vector is orthogonal to the basis as MGS's is.  A NumPy restatement of the formula (the
    order of the correction terms as icwy_coef_kernel)."""
    rng = np.random.default_rng(5)
    n, k = 4000, 30
    A = np.diag(np.linspace(1, 10, n)) + 0.01 * rng.normal(size=(n, n)) / np.sqrt(n)
    Q = np.zeros((k + 1, n))
    Q[0] = rng.normal(size=n)
    Q[0] /= np.linalg.norm(Q[0])
    for j in range(k):
        w = A @ Q[j]
        # MGS
        wm = w.copy()
        hm = np.zeros(j + 1)
        for i in range(j + 1):
            hm[i] = Q[i] @ wm
            wm = wm - hm[i] * Q[i]
        # one reduce: all dots from the unmodified w and the Gram matrix
        a = Q[: j + 1] @ w
        G = Q[: j + 1] @ Q[: j + 1].T
        h = np.zeros(j + 1)
        for l in range(j + 1):
            t = a[l]
            for m in range(l):
                t -= h[m] * G[l, m]
            h[l] = t
        np.testing.assert_allclose(h, hm, rtol=0, atol=1e-12 * np.linalg.norm(w))
        w1 = w - Q[: j + 1].T @ h
        # orthogonal to the basis to MGS's own level
        assert np.abs(Q[: j + 1] @ w1).max() <= 10 * np.abs(Q[: j + 1] @ wm).max() + 1e-11 * np.linalg.norm(w)
        Q[j + 1] = wm / np.linalg.norm(wm)
