"""One rank of a several-rank solve through libspis's distributed code path (run by
tests/test_gpu_multirank.py, one process per rank, all on GPU 0 with SPIS_TRANSPORT=host).

    RANK=r WORLD_SIZE=P MASTER_ADDR=127.0.0.1 MASTER_PORT=... SPIS_DEVICE=0 SPIS_TRANSPORT=host \
        python tests/multirank_worker.py OUT_PREFIX PROBLEM M K [CYCLES]

PROBLEM is a bench workload (distributed.dist_workload) at mesh size M: swe (config C3's shape:
mass + energy), lkdv (C2's: mass + momentum + energy), c4 (lkdvRK GL(3), stage x field
partition, the three invariants lifted to (M, v, c)), c5 (swe + the synthetic third constraint).
CYCLES > 1 restarts CGMRES(K) from the previous cycle's x[-1] (C5's restart loop).

Writes OUT_PREFIX.<rank>.npz with, per cycle c: the cycle's start x0 and every iterate (gathered
to the global ordering), the residual history, the branch trace, the step count, and the last
constrained step's LS inputs (H, beta, y_{k-2}, y_{k-1}, the reduced constraint terms), as this
rank saw them."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIG = {"swe": "c3", "lkdv": "c2", "c4": "c4", "c5": "c5"}


def main():
    out, problem, M, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    cycles = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    from structurepreservingiterativesolvers_amd import distributed as D
    from structurepreservingiterativesolvers_amd import solvers
    from structurepreservingiterativesolvers_amd.device import DeviceVector

    comm = D.Comm()
    try:
        w = D.dist_workload(CONFIG[problem], comm.world, M_override=M)
        sysd = D.DistributedSystem(comm, w["A"], w["fields"])
        bd = sysd.vector(w["b"])
        conlist = D.distribute_constraints(sysd, w["conlist"])
        x = DeviceVector.from_host(np.zeros(sysd.n_local), ctx=comm.ctx)
        rec = dict(cycles=cycles, n_ghost=sysd.A.n_ghost)
        for c in range(cycles):
            rec[f"x0_{c}"] = sysd.gather(x.numpy())
            xf, d = solvers.cgmres(sysd.A, bd, x, k, tol=1e-19, conlist=conlist)
            its = d["x"]
            rec[f"X_{c}"] = np.stack([sysd.gather(its[i].numpy()) for i in range(len(its))])
            rec[f"x_{c}"] = sysd.gather(xf.numpy())
            rec[f"res_{c}"] = np.asarray(d["res"])
            rec[f"steps_{c}"] = d["steps"]
            trace = its.trace
            rec[f"trace_j_{c}"] = np.array([t[0] for t in trace])
            rec[f"trace_b_{c}"] = np.array([t[1] for t in trace])
            if d["steps"] == k and trace and trace[-1][1] != "uncon":
                rec[f"H_{c}"] = its.hessenberg(k)
                rec[f"beta_{c}"] = its.beta
                rec[f"y0_{c}"] = np.concatenate([its.y[k - 2], [0.0]])
                rec[f"y_{c}"] = its.y[k - 1]
                for ci in range(len(conlist)):
                    p, t0, t1, t2 = its.constraint_terms(ci)
                    rec[f"t0_{c}_{ci}"], rec[f"t1_{c}_{ci}"], rec[f"t2_{c}_{ci}"] = t0, t1, t2
            x = xf
        np.savez(f"{out}.{comm.rank}.npz", **rec)
        comm.barrier()
    finally:
        comm.dist.destroy_process_group()


if __name__ == "__main__":
    main()
