"""Benchmark: CGMRES iterations/sec + Arnoldi-SpMV achieved HBM GB/s (BASELINE.json).

Default workload (BASELINE.json configs[2]): swe-shaped RT2 x DG0 CSR,
N = 12 M^2 = 1,002,252 DoF per GPU (M = 289), 12.5 nnz/row, fp64;
``swe.LinearSolver.cgmresWrapper`` semantics (mass + energy constraints), k = 30, tol = 1e-19
so every solve runs all 30 iterations and the last one is the constrained projection.  One
"step" = one CGMRES(30) solve; inputs (A, b, x0, constraint operators) are resident in HBM
before the timed region.

``--config`` selects the other SURVEY §8 single-GPU configurations (not the driver's line):
  c2  lkdv DG1 M=16,667, N=100,002, 3 constraints (mass, momentum, energy)
  c4  lkdvRK GL(3) M=16,667, N=300,006, the 3 dict constraints lifted to (M, v, c) form
  c5  swe M=913, N=10,002,828, 3 constraints (+ the synthetic third), restarted CGMRES(30),
      one step = one restarted solve of --cycles cycles (default 10)

Multi-GPU (``--gpus N`` under torch.distributed.run, distributed.dist_workload): one global
solve row-partitioned over the N ranks (field-interleaved blocks), RCCL all-reduces (two per
Arnoldi step: MGS's projections in one, the norm in the other) and a halo exchange before every
SpMV.  c3 (default): N x 1,002,252 DoF (weak scaling), ``value`` = iterations x N / time (the
whole job's Mdof-normalised iterations per second), max time over ranks; c4: the C4 lkdvRK GL(3)
problem (N = 300,006) row-split (strong scaling); c5: the C5 swe problem (strong); c2: lkdv with
~1e5 DoF per GPU (weak).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CGMRES iterations/sec + SpMV achieved HBM GB/s, N=10^6 DoF CSR fp64"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def spmv_bytes(n_rows, nnz, col_bytes=4):
    """Algorithmic bytes of one CSR SpMV: fp64 val + int32 col per nnz (int16 with
    the 16-bit column copy, SPIS_OPT_COL16), int32 rowptr, x read once, y written once."""
    return (8 + col_bytes) * nnz + 4 * (n_rows + 1) + 16 * n_rows


def mgs_chain_bytes(n, k, chain):
    """Mean algorithmic bytes of one sampled MGS chain (+ normalise) of a CGMRES(k) solve.  The
    sampled iteration advances by one position per solve (spis.cpp ProfEv, prof_phase), so over
    the timed solves every chain position j = 0 .. k-1 is sampled equally often; the byte count
    is the mean over j of the kernel that runs there:
      K2q (chain 3, (N+1)/2 <= 522,240 pairs): 8 N (j + 3) (w and q_0 .. q_j read, q_{j+1}
          written) + 16 N for the update GEMV it carries from j >= 1 (x0 read, x_{j-1} written);
      K2p (chain 1-2, N/2 <= 2^19): 8 N (j + 3);
      K2b (chain >= 2 beyond): 16 N (j + 1) + 16 N (q_i and q_{i+1} streamed per MGS step, w
          read once, q_{j+1} written);
      one-reduce two-pass MGS (chain 4, and chain 3 beyond K2q): 8 N (j + 2) for the dots (w,
          q_0 .. q_j) + 8 N (j + 3) for the update (q_0 .. q_j and w read, w written) + 16 N for
          the update GEMV it carries from j >= 1 + 16 N for the normalise;
      its one-launch form K2s (chain 3 or 4, N <= 524,288, k <= 32: spis.cpp k2w_small): 8 N
          (j + 2) (w, q_0 .. q_j read once) + 16 N (w' and q_{j+1} written) + 16 N for the GEMV,
          + 8 N_s (j + 2) for the streamed second chunks (N_s ~ N / 2 beyond 262,144) read again;
      per-step launches (chain 0): 32 N (j + 1) + 16 N (y, q_i, q_{i+1} read, y written; the
          normalise reads y, writes q)."""
    tot = 0.0
    k2q = (n + 1) // 2 <= 255 * 512 * 4
    for j in range(k):
        if k2s_used(n, k, chain):
            b = 8 * n * (j + 2) + 16 * n + (16 * n if j >= 1 else 0) + 8 * k2s_reread(n) * (j + 2)
        elif chain == 4 or (chain == 3 and not k2q):
            b = 8 * n * (j + 2) + 8 * n * (j + 3) + (16 * n if j >= 1 else 0) + 16 * n
        elif chain == 3:
            b = 8 * n * (j + 3) + (16 * n if j >= 1 else 0)
        elif chain >= 1 and n // 2 <= 256 * 256 * 8 and not (chain >= 2 and n // 2 > 255 * 256 * 8):
            b = 8 * n * (j + 3)
        elif chain >= 2:
            b = 16 * n * (j + 1) + 16 * n
        else:
            b = 32 * n * (j + 1) + 16 * n
        tot += b
    return tot / k


def k2s_used(n, k, chain):
    """One GPU: does the library take K2s, the one-launch one-reduce MGS (spis.cpp k2w_small and
    arnoldi_post_icwy: chain 3 or 4, k <= 32, N within its 1024 resident 256-row workgroups, one
    register chunk each, and as many streamed second chunks: kernels.hip icwy_onepass_max_n)?"""
    return chain in (3, 4) and k <= 32 and n <= 2 * 256 * 1024


def k2s_reread(n):
    """Elements K2s reads twice (its streamed second chunks, dots then update): beyond 1024 chunks of
    256 rows each workgroup takes two chunks (kernels.hip launch_icwy_onepass), the second streamed."""
    chunks = (n + 255) // 256
    return 0 if chunks <= 1024 else max(0, n - 256 * ((chunks + 1) // 2))


def orthog_label(n, k, chain, orthog):
    """The arithmetic the run's orthogonalisation actually performs (variants that do
    not round as MGS does are reported as such): "mgs" for per-step MGS and the K2p chain (MGS's
    rounding), "mgs-lag2" for K2q (MGS with each dot taken two steps early by the distributive
    law), "mgs-icwy" for K2w / K2s (MGS's projections in inverse-compact-WY one-reduce form), or
    "cgs2"."""
    if orthog == "cgs2":
        return "cgs2"
    if k2s_used(n, k, chain) or chain == 4 or (chain == 3 and (n + 1) // 2 > 255 * 512 * 4):
        return "mgs-icwy"
    return "mgs-lag2" if chain == 3 else "mgs"


def mgs_one_read_bytes(n, k):
    """Mean bytes of an Arnoldi step's orthogonalisation with the basis read ONCE: w and q_0 ..
    q_j read, q_{j+1} written (8 N (j + 3)), + 16 N for the update GEMV it carries from j >= 1.
    The figure a two-pass kernel (K2w: dots, then update) is also quoted against."""
    return sum(8 * n * (j + 3) + (16 * n if j >= 1 else 0) for j in range(k)) / k


def dual_bytes(n_rows, nnz, col_bytes=4):
    """Algorithmic bytes of the fused residual + Arnoldi SpMV: the matrix once, x_j and b read
    (true residual, solvers.py:290), z_{j+2} read and w written (Arnoldi, :191)."""
    return (8 + col_bytes) * nnz + 4 * (n_rows + 1) + 32 * n_rows


def k_per_solve(k):
    """MGS chains per CGMRES(k) solve (one per Arnoldi step)."""
    return k


def kernels_sha256():
    import hashlib

    with open(os.path.join(ROOT, "structurepreservingiterativesolvers_amd", "csrc", "kernels.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def load_traffic(args, c16, pipe):
    """Per-launch PMC bytes from profiles/r06_traffic_<config>.json (tools/r06_pmc.sh; else r05, r04), with the
    reason when there are none: the file must have been measured on this csrc/kernels.hip (SHA-256)
    with this run's SpMV and chain options, on the configuration's default size."""
    for rnd in ("r06", "r05", "r04"):  # the newest round's file that exists
        path = os.path.join(ROOT, "profiles", f"{rnd}_traffic_{args.config}.json")
        if os.path.exists(path):
            break
    if args.M is not None:
        return {}, "no PMC traffic for a non-default mesh size"
    if not os.path.exists(path):
        return {}, f"no {os.path.relpath(path, ROOT)}"
    with open(path) as f:
        t = json.load(f)
    if t.get("kernels_sha256") != kernels_sha256():
        return {}, f"{os.path.relpath(path, ROOT)} was measured on another kernels.hip (git {t.get('git_rev')})"
    want = {"spmv_pipe": pipe, "col16": bool(c16), "slab_key": args.slab_key, "chain": args.chain,
            "nt_basis": args.nt_basis, "orthog": args.orthog, "fuse": not args.no_fuse}
    if t.get("options") != want:
        return {}, f"{os.path.relpath(path, ROOT)} was measured with options {t.get('options')}, this run {want}"
    return t.get("bytes_per_launch", {}), f"{os.path.relpath(path, ROOT)} (git {t.get('git_rev')})"


def cpu_baseline(dic, conlist, k, tol, budget_s, method="cgmres"):  # dic: the workload (A, b)
    """The oracle (CPU restatement of the reference solvers.cgmres, NumPy/SciPy +
    SLSQP exactly as the reference) on the same workload, bounded sample."""
    import oracle

    try:
        from threadpoolctl import threadpool_info

        blas_threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        blas_threads = 1
    cores = len(os.sched_getaffinity(0))  # the host cores this process may run on
    x0 = np.zeros_like(dic["b"])
    iters = 0
    solves = 0
    t0 = time.perf_counter()
    while True:
        if method == "cgmres_p":
            _, d = oracle.cgmres_p(dic["A"], dic["b"], x0, k, conlist=conlist)
            iters += len(d["res"])
        else:
            _, d = oracle.cgmres(dic["A"], dic["b"], x0, k, tol=tol, conlist=conlist)
            iters += d["steps"]
        solves += 1
        if time.perf_counter() - t0 > budget_s or solves >= 3:
            break
    dt = time.perf_counter() - t0
    return {
        "value": iters / dt,
        "unit": "iterations/s",
        "cores": int(cores),
        "blas_threads": int(blas_threads),
        "kind": "port",
        "sample": f"{solves} full {'CGMRES_P' if method == 'cgmres_p' else 'CGMRES'}({k}) solve(s) of the same "
                  f"N={len(x0)} system ({iters} iterations, "
                  f"{dt:.1f} s); SciPy csr_matvec single-threaded, OpenBLAS {blas_threads} threads on "
                  f"{cores} affinity cores",
    }


def build_workload(args):
    """A, b and the reference-form constraint list of the selected SURVEY §8 configuration."""
    x0 = None
    if args.config in ("c3", "c5"):
        from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls
        from structurepreservingiterativesolvers_amd.swe import assembly

        M = args.M or (289 if args.config == "c3" else 913)
        dic, _ = assembly.linforms(M=M)
        x0 = np.zeros(dic["A"].shape[0])
        conlist = ls.constraints(dic, x0)
        desc = f"swe-shaped RT2xDG0 CSR (config {args.config.upper()}, M={M}), mass+energy constraints"
        if args.config == "c5":
            D, c3 = assembly.extra_constraint(len(x0), dic["z0"], seed=2)
            conlist.append(ls._Constraint(D, np.zeros(len(x0)), c3))
            desc += " + synthetic third constraint (seed 2)"
        return {"A": dic["A"], "b": dic["b"], "conlist": conlist, "desc": desc, "dic": dic,
                "cycles": args.cycles if args.config == "c5" else 1}
    if args.config == "c2":
        from structurepreservingiterativesolvers_amd.lkdv import LinearSolver as ls
        from structurepreservingiterativesolvers_amd.lkdv import assembly

        M = args.M or 16667
        dic, _ = assembly.linforms(M=M)
        conlist = ls.constraints(dic, np.zeros(dic["A"].shape[0]))
        return {"A": dic["A"], "b": dic["b"], "conlist": conlist, "cycles": 1,
                "desc": f"lkdv DG1 (config C2, M={M}), mass+momentum+energy constraints"}
    from structurepreservingiterativesolvers_amd.lkdvRK import LinearSolver as ls
    from structurepreservingiterativesolvers_amd.lkdvRK import assembly

    M = args.M or 16667
    dic, prob = assembly.linforms(M=M, tstages=3)
    conlist = ls.constraints(dic, prob, lift=True)
    return {"A": dic["A"], "b": dic["b"], "conlist": conlist, "cycles": 1,
            "desc": f"lkdvRK GL(3) block-stage (config C4, M={M}), 3 invariants lifted to (M, v, c) form"}


def spawn_ranks(n, script=None, argv=None):
    """``bench.py --gpus N`` started without a launcher: start the N ranks as child processes of
    this one (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1 rendezvous), forward rank 0's
    JSON line and return the exit status (non-zero if any rank failed).  Runs before anything here
    touches HIP: this process only waits on its children."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]

    def die_with_parent():  # a rank outlives no parent (PR_SET_PDEATHSIG = SIGKILL)
        import ctypes

        ctypes.CDLL(None).prctl(1, signal.SIGKILL)

    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPIS_BENCH_LAUNCH="bench.py spawn")
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)]
                                      + list(sys.argv[1:] if argv is None else argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      preexec_fn=die_with_parent))

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    out = []  # rank 0's stdout, drained as it comes so a full pipe never stalls the rank
    import threading

    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read().decode()), daemon=True)
    reader.start()
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            if p.poll() not in (None, 0):
                failed = (r, p.returncode)
                break
        else:
            time.sleep(0.2)
    if failed is None:
        failed = next(((r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0), None)
    if failed is not None:  # a rank died: its peers would wait in a collective forever
        stop_all()
        print(f"bench.py: rank {failed[0]} of {n} exited with status {failed[1]}", file=sys.stderr)
        return failed[1] if failed[1] > 0 else 1
    reader.join()
    sys.stdout.write("".join(out))
    sys.stdout.flush()
    return 0


def wrapper_rate(wl, args, reps=30, warm=3):
    """SURVEY §8(d)'s it/s as defined there: ``dict['steps']`` / wall time of the drop-in call
    ``swe.LinearSolver.cgmresWrapper(dic, x0, k, tol)`` (reference ``swe/LinearSolver.py:12-49``) on
    host SciPy/NumPy inputs, warm (the operator uploads cached by the warm-up calls, as a
    time-stepping caller sees them; only the matrix upload is excluded).  Each call still uploads
    b, x0 and the constraint vectors, re-verifies the cached matrices against their full contents
    and downloads x; the host phases are reported beside the rate (solvers._PHASES)."""
    from structurepreservingiterativesolvers_amd import device, solvers
    from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls

    dic = wl["dic"]
    x0 = np.zeros(dic["A"].shape[0])
    d = None
    for _ in range(warm):
        _, d = ls.cgmresWrapper(dic, x0, args.k, tol=args.tol)
    solvers._PHASES = {}
    iters = 0
    t0 = time.perf_counter()
    for _ in range(reps):
        _, d = ls.cgmresWrapper(dic, x0, args.k, tol=args.tol)
        iters += d["steps"]
    el = time.perf_counter() - t0
    ph, solvers._PHASES = solvers._PHASES, None
    t1 = time.perf_counter()
    for M in (dic["A"], dic["L"]):
        device.content_digest(M)
    hash_ms = 1e3 * (time.perf_counter() - t1)
    per = {k: 1e3 * v / reps for k, v in ph.items()}
    return {
        "call": f"swe.LinearSolver.cgmresWrapper(dic, x0=zeros, k={args.k}, tol={args.tol:g}) on SciPy/NumPy inputs",
        "value": iters / el,
        "unit": "iterations/s",
        "ms_per_call": 1e3 * el / reps,
        "calls": reps,
        "h2d_ms": per.get("h2d", 0.0),
        "verify_ms": hash_ms,
        "verify_wait_ms": per.get("verify_wait", 0.0),
        "d2h_ms": per.get("d2h", 0.0),
        "phases_ms": per,
        "verify_threads": device._HASH_THREADS,
    }


def main():
    if "RANK" not in os.environ and "WORLD_SIZE" not in os.environ:
        # --gpus N > 1 with no launcher: this process becomes the parent of N ranks
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        known, _ = pre.parse_known_args()
        if known.gpus > 1:
            sys.exit(spawn_ranks(known.gpus))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c5"],
                    help="SURVEY §8 configuration (c3 = the BASELINE.json line)")
    ap.add_argument("--M", type=int, default=None, help="mesh size override (swe: N = 12 M^2 per GPU)")
    ap.add_argument("--cycles", type=int, default=10, help="restart cycles for c5")
    ap.add_argument("--k", type=int, default=30)
    ap.add_argument("--tol", type=float, default=1e-19)
    ap.add_argument("--method", default="cgmres", choices=["cgmres", "cgmres_p"],
                    help="cgmres (the BASELINE line) or cgmres_p (solvers.py:328-445: constraint i enforced from "
                         "step i, every step constrained)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wrapper", action="store_true", help="skip the drop-in wrapper call's rate (c3)")
    ap.add_argument("--no-cold", action="store_true", help="skip the standalone cold-cache SpMV timing")
    ap.add_argument("--force-distributed", action="store_true",
                    help="use the row-partitioned RCCL path even for one rank (plumbing check)")
    ap.add_argument("--dist-mgs", type=int, default=1, choices=[0, 1],
                    help="several GPUs (SPIS_OPT_DIST_MGS): 1 MGS's projections in one all-reduce per Arnoldi "
                         "step, 0 one all-reduce per projection")
    ap.add_argument("--no-fuse", action="store_true", help="separate residual and Arnoldi SpMV launches")
    ap.add_argument("--chain", type=int, default=3, choices=[0, 1, 2, 3, 4],
                    help="MGS chain (SPIS_OPT_MGS_CHAIN): 0 per-step launches, 1 persistent chain gathered by "
                         "workgroup 0, 2 with a dedicated gathering workgroup, 3 pipelined (dots two steps early), "
                         "4 one-reduce two-pass MGS carrying the update GEMV")
    ap.add_argument("--nt-basis", type=int, default=2, choices=[0, 1, 2],
                    help="MGS basis loads nontemporal (SPIS_OPT_NT_BASIS): 0 never, 1 always, 2 auto")
    ap.add_argument("--gram", default="mfma", choices=["generic", "csr", "mfma", "mfma_full"],
                    help="constraint reduction (SPIS_OPT_CON_GRAM)")
    ap.add_argument("--spmv-pipe", default="auto", choices=["off", "stride", "xcd", "auto", "xcd_natural"],
                    help="solver SpMV kernels (SPIS_OPT_SPMV_PIPE): unpipelined, pipelined grid-stride, "
                         "pipelined XCD-local walk (slab order / natural order)")
    ap.add_argument("--col16", type=int, default=1, choices=[0, 1, 2],
                    help="16-bit column copy for the pipelined SpMV: 1 beyond the Infinity Cache, 2 always, 0 never")
    ap.add_argument("--slab-key", type=int, default=1, choices=[0, 1],
                    help="SpMV row blocks of a slab by position (SPIS_OPT_SLAB_KEY, at upload): 1 groups side by "
                         "side, 0 group after group")
    ap.add_argument("--orthog", default="mgs", choices=["mgs", "cgs2"],
                    help="mgs = the reference's MGS (the BASELINE line); cgs2 = the opt-in low-sync option")
    ap.add_argument("--prof-period", type=int, default=10,
                    help="time every n-th iteration's kernels with HIP events inside the timed region")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 or world > 1 or args.force_distributed:
        from structurepreservingiterativesolvers_amd import distributed

        return distributed.bench_main(args, METRIC)

    from structurepreservingiterativesolvers_amd import _lib, solvers
    from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints, device_matrix,
                                                                get_context)

    wl = build_workload(args)
    A = wl["A"]
    n = A.shape[0]
    ctx = get_context(0)
    opt = {_lib.OPT_SLAB_KEY: args.slab_key, _lib.OPT_FUSE_SPMV: 0 if args.no_fuse else 1,
           _lib.OPT_ORTHOG: 1 if args.orthog == "cgs2" else 0, _lib.OPT_MGS_CHAIN: args.chain,
           _lib.OPT_NT_BASIS: args.nt_basis, _lib.OPT_COL16: args.col16,
           _lib.OPT_CON_GRAM: {"generic": 0, "csr": 1, "mfma": 2, "mfma_full": 3}[args.gram],
           _lib.OPT_SPMV_PIPE: {"off": 0, "stride": 1, "xcd": 2, "auto": 5, "xcd_natural": 7}[args.spmv_pipe]}
    for k, v in opt.items():
        _lib.check(ctx.L.spis_set_option(ctx.handle, k, v), "spis_set_option")
    Ad = device_matrix(A, ctx=ctx)  # inputs resident in HBM before timing (the operator, b, x0, constraints)
    bd = DeviceVector.from_host(wl["b"], ctx=ctx)
    x0 = np.zeros(n)
    x0d = DeviceVector.from_host(x0, ctx=ctx)
    conlist = wl["conlist"]
    conlist_dev = device_constraints(conlist, ctx=ctx)

    if args.method == "cgmres_p":
        if wl["cycles"] > 1:
            raise ValueError("cgmres_p is not restarted")

        def solve():
            return solvers.cgmres_p(Ad, bd, x0d, args.k, conlist=conlist_dev)
    elif wl["cycles"] > 1:
        def solve():
            return solvers.cgmres_restarted(Ad, bd, x0d, args.k, wl["cycles"], tol=args.tol, conlist=conlist_dev)
    else:
        def solve():
            return solvers.cgmres(Ad, bd, x0d, args.k, tol=args.tol, conlist=conlist_dev)

    # the warm-up holds each result until the next call returns, as the timed loop does: a result
    # keeps its workspace (the lazy iterates), so the loop runs on two pooled workspaces, and both
    # are allocated before the clock starts (else the second timed solve allocates one, ~1.3 ms)
    d = None
    for _ in range(args.warmup):
        _, d = solve()
    ctx.synchronize()
    L = ctx.L
    import ctypes as C

    _lib.check(L.spis_profile_enable(ctx.handle, args.prof_period), "spis_profile_enable")
    ctx.synchronize()
    # the set-up's objects (assembled matrices, oracle imports) leave the collector's generations,
    # so a full collection inside the timed loop does not walk them (one run's host time between
    # solves read 302 instead of 48 us)
    gc.collect()
    gc.freeze()
    t0 = time.perf_counter()
    iters = 0
    outside = 0.0  # host time per solve outside spis_solve (Python wrapper, result objects)
    for _ in range(args.steps):
        ts = time.perf_counter()
        _, d = solve()
        st = d["x"].stamps if "x" in d and hasattr(d["x"], "stamps") else None
        if st is not None:
            outside += (time.perf_counter() - ts) - (st[4 * args.k + 1] - st[4 * args.k])
        iters += d["steps"] if "steps" in d else len(d["res"])
    ctx.synchronize()
    t1 = time.perf_counter()
    ms, cnt = _lib.profile_read(L, ctx.handle)
    _lib.check(L.spis_profile_enable(ctx.handle, 0), "spis_profile_enable")
    elapsed = t1 - t0

    # the 16-bit column copy (SPIS_OPT_COL16, as the library decides: the swe matrices have one)
    c16 = args.col16 == 2 or (args.col16 == 1 and 12 * A.nnz > 256 * 1024 * 1024 and args.config in ("c3", "c5"))
    cb = 2 if c16 else 4
    S = spmv_bytes(n, A.nnz, cb)
    spmv_ms = ms[_lib.PROF_SPMV] / max(cnt[_lib.PROF_SPMV], 1)
    spmv_gbs = S / (spmv_ms * 1e-3) / 1e9 if spmv_ms > 0 else 0.0
    SD = dual_bytes(n, A.nnz, cb)
    dual_ms = ms[_lib.PROF_SPMV_DUAL] / max(cnt[_lib.PROF_SPMV_DUAL], 1)
    dual_gbs = SD / (dual_ms * 1e-3) / 1e9 if dual_ms > 0 else 0.0
    mgs_ms = ms[_lib.PROF_MGS] / max(cnt[_lib.PROF_MGS], 1)
    mgs_b = mgs_chain_bytes(n, args.k, args.chain if args.orthog == "mgs" else -1)
    mgs_gbs = mgs_b / (mgs_ms * 1e-3) / 1e9 if mgs_ms > 0 and args.orthog == "mgs" else None
    res_ms = ms[_lib.PROF_SPMV_RES] / max(cnt[_lib.PROF_SPMV_RES], 1)
    gemv_ms = ms[_lib.PROF_GEMV] / max(cnt[_lib.PROF_GEMV], 1)
    fused = cnt[_lib.PROF_SPMV_DUAL] > 0
    pipe = args.spmv_pipe
    if pipe == "auto":  # as the library decides (SPIS_OPT_SPMV_PIPE 5): the XCD-local walk, on the
        # slab-ordered table when the upload found one (the swe configs), else while val/col fit
        # the 256 MB Infinity Cache
        pipe = "xcd" if args.config in ("c3", "c5") or 12 * A.nnz <= 256 * 1024 * 1024 else "stride"
    kname = {"off": "spmv_dual_kernel", "stride": "spmv_pipe_kernel<2048, 4> (grid-stride walk)",
             "xcd": "spmv_pipe_kernel<2048, 4> (XCD-local walk, slab order)",
             "xcd_natural": "spmv_pipe_kernel<2048, 4> (XCD-local walk, natural block order)"}[pipe]
    if c16 and pipe != "off":
        kname = kname.replace(", 4>", ", 4, true>").replace(")", ", 16-bit columns)")
    # PMC traffic (profiles/r04_traffic_<config>.json, tools/archive/r04_pmc.sh): used only when it was
    # measured on this kernels.hip and these SpMV / chain options (load_traffic checks both)
    tr, tr_note = load_traffic(args, c16, pipe)
    if fused:  # the SpMV of the north star: true residual of x_j fused with the Arnoldi SpMV of z_{j+2}
        roof_spmv = {"kernel": kname + ": true-residual SpMV of x_j, solvers.py:290, fused with the "
                                       "Arnoldi SpMV of z_{j+2}, :191; matrix read once",
                     "bound": "hbm", "achieved": dual_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": dual_gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": SD,
                     "avg_launch_us": 1e3 * dual_ms, "launches": int(cnt[_lib.PROF_SPMV_DUAL])}
    else:
        roof_spmv = {"kernel": kname.replace(", 4", ", 1") + ": Arnoldi SpMV, solvers.py:191",
                     "bound": "hbm", "achieved": spmv_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": spmv_gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": S,
                     "avg_launch_us": 1e3 * spmv_ms, "launches": int(cnt[_lib.PROF_SPMV])}
    roof_spmv["traffic"] = tr.get("dual_solver" if fused else "arnoldi_solver")
    roof_spmv["traffic_cold"] = tr.get("dual_cold" if fused else "arnoldi_cold")
    # the MGS chain (+ normalise, + the update GEMV it carries): its launches' mean algorithmic bytes
    # over the sampled chain positions / their mean duration (mgs_chain_bytes)
    chain_name = {3: "mgs_chain_lag_kernel<8, PER, 5, 2, FX, NT> (K2q: MGS, dots two steps early)",
                  4: "icwy_dot + cgs_update + normalise (K2w: one-reduce two-pass MGS)"}.get(args.chain, "MGS chain")
    if args.chain == 3 and (n + 1) // 2 > 255 * 512 * 4:
        chain_name = "icwy_dot + cgs_update + normalise (K2w: one-reduce two-pass MGS, beyond K2q's capacity)"
    if args.orthog == "mgs" and k2s_used(n, args.k, args.chain):
        chain_name = "icwy_onepass_kernel (K2s: one-reduce MGS in one launch, basis slices in registers)"
    roof_mgs = {"kernel": chain_name + ": solvers.py:193-198 (+ the update GEMV of :287)", "bound": "hbm",
                "achieved": mgs_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": None if mgs_gbs is None else mgs_gbs / HBM_PEAK_GBS,
                "algorithmic_bytes_per_launch": mgs_b, "avg_launch_us": 1e3 * mgs_ms,
                "launches": int(cnt[_lib.PROF_MGS]), "traffic": tr.get("mgs_solver"),
                "orthogonalisation": orthog_label(n, args.k, args.chain, args.orthog)}
    if roof_mgs["orthogonalisation"] == "mgs-icwy" and mgs_ms > 0:
        # the one-read figure beside the kernel's own byte model (two passes for K2w)
        b1 = mgs_one_read_bytes(n, args.k)
        roof_mgs["one_read_bytes_per_launch"] = b1
        roof_mgs["achieved_one_read"] = b1 / (mgs_ms * 1e-3) / 1e9
        roof_mgs["frac_one_read"] = roof_mgs["achieved_one_read"] / HBM_PEAK_GBS
    # the dominant kernel by GPU time per solve (the contract's roofline object); the other beside it
    t_mgs = mgs_ms * k_per_solve(args.k)
    t_spmv = (dual_ms if fused else spmv_ms) * max(args.k - 2, 1)
    mgs_dominant = roof_mgs["frac"] is not None and t_mgs >= t_spmv
    roof = dict(roof_mgs if mgs_dominant else roof_spmv)
    roof["share_of_solve_kernel_time"] = "dominant by time per solve: MGS chain %.0f us vs SpMV %.0f us" % (
        1e3 * t_mgs, 1e3 * t_spmv)
    roof["traffic_note"] = tr_note
    # the same launch standalone (spis_spmv_bench: the solver's table, walk and grid), back to back
    # and behind a 1 GiB cache-evicting read, so the fraction is also quoted with the matrix and
    # the vectors coming from HBM, not from the 256 MB Infinity Cache
    if not args.no_cold:
        kind = 1 if fused else 0
        bytes_l = SD if fused else S
        us = {}
        for cold in (0, 1):
            v = C.c_double()
            _lib.check(L.spis_spmv_bench(ctx.handle, device_matrix(A, ctx=ctx).handle, kind, cold, 20, C.byref(v)),
                       "spis_spmv_bench")
            us[cold] = v.value
        roof_spmv["standalone_warm_us"] = us[0]
        roof_spmv["avg_launch_us_cold"] = us[1]
        roof_spmv["achieved_cold"] = bytes_l / (us[1] * 1e-6) / 1e9
        roof_spmv["frac_cold"] = roof_spmv["achieved_cold"] / HBM_PEAK_GBS
    out = {
        "metric": METRIC,
        "value": iters / elapsed,
        "unit": "iterations/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": wl["desc"] + f", N={n:,} DoF, nnz={A.nnz:,}, "
                        + (f"CGMRES_P(k={args.k}, every step constrained)" if args.method == "cgmres_p" else
                           f"CGMRES(k={args.k}, tol={args.tol:g})")
                        + (f" restarted x{wl['cycles']}" if wl["cycles"] > 1 else ""),
            "method": args.method,
            "config": args.config,
            "orthogonalisation": orthog_label(n, args.k, args.chain, args.orthog),
            "global_dof": n,
            "k": args.k,
            "parallelism": "single GPU",
        },
        "roofline": roof,
        "roofline_spmv": roof_spmv,
        "kernels": {
            "spmv_arnoldi_us": 1e3 * spmv_ms,
            "spmv_arnoldi_GBs": spmv_gbs,
            "spmv_dual_us": 1e3 * dual_ms,
            "spmv_dual_GBs": dual_gbs,
            "spmv_residual_us": 1e3 * res_ms,
            "mgs_chain_us_mean": 1e3 * mgs_ms,
            "mgs_chain_GBs": mgs_gbs,
            "gemv_us_mean": 1e3 * gemv_ms,
            "iteration_us": 1e6 * elapsed / max(iters, 1),
            "host_outside_solve_us": 1e6 * outside / args.steps,
        },
    }
    if args.config == "c3" and args.method == "cgmres" and not args.no_wrapper:
        out["wrapper"] = wrapper_rate(wl, args)
        out["wrapper"]["frac_of_value"] = out["wrapper"]["value"] / out["value"]
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl, conlist, args.k, args.tol, args.cpu_budget, args.method)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
