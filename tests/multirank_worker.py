"""One rank of a several-rank solve through libspis's distributed code path (run by
tests/test_gpu_multirank.py, one process per rank, all on GPU 0 with SPIS_TRANSPORT=host).

    RANK=r WORLD_SIZE=P MASTER_ADDR=127.0.0.1 MASTER_PORT=... SPIS_DEVICE=0 SPIS_TRANSPORT=host \
        python tests/multirank_worker.py OUT_PREFIX PROBLEM M K

Writes OUT_PREFIX.<rank>.npz: the gathered final iterate and the middle one, the residual history,
the branch trace and the step count, as this rank saw them."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    out, problem, M, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    from structurepreservingiterativesolvers_amd import distributed as D
    from structurepreservingiterativesolvers_amd import solvers
    from structurepreservingiterativesolvers_amd.device import DeviceVector

    comm = D.Comm()
    try:
        if problem == "swe":
            from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls
            from structurepreservingiterativesolvers_amd.swe import assembly

            dic, _ = assembly.linforms(M=M)
            fields = D.swe_fields(M)
        else:
            from structurepreservingiterativesolvers_amd.lkdv import LinearSolver as ls
            from structurepreservingiterativesolvers_amd.lkdv import assembly

            dic, _ = assembly.linforms(M=M)
            fields = D.lkdv_fields(dic["A"].shape[0])
        n = dic["A"].shape[0]
        cons = ls.constraints(dic, np.zeros(n))
        sysd = D.DistributedSystem(comm, dic["A"], fields)
        bd = sysd.vector(dic["b"])
        x0d = DeviceVector.from_host(np.zeros(sysd.n_local), ctx=comm.ctx)
        conlist = D.distribute_constraints(sysd, cons)
        xf, d = solvers.cgmres(sysd.A, bd, x0d, k, tol=1e-19, conlist=conlist)
        its = d["x"]
        mid = len(its) // 2
        x_final = sysd.gather(np.asarray(xf.numpy() if hasattr(xf, "numpy") else xf))
        x_mid = sysd.gather(np.asarray(its[mid].numpy() if hasattr(its[mid], "numpy") else its[mid]))
        trace = its.trace
        np.savez(f"{out}.{comm.rank}.npz", x=x_final, x_mid=x_mid, mid=mid, res=np.asarray(d["res"]),
                 steps=d["steps"], trace_j=np.array([t[0] for t in trace]),
                 trace_b=np.array([t[1] for t in trace]), n_ghost=sysd.A.n_ghost)
        comm.barrier()
    finally:
        comm.dist.destroy_process_group()


if __name__ == "__main__":
    main()
