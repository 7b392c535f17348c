"""MI355X-native CGMRES/FGMRES inner loop of the structure-preserving
iterative solvers (reference: JamesJackaman/StructurePreservingIterativeSolvers).

* :mod:`.solvers`    — drop-in ``cgmres`` / ``gmres`` / ``cgmres_p`` (reference ``solvers.py``)
* :mod:`.heat`, :mod:`.lkdv`, :mod:`.lkdvRK`, :mod:`.swe` — ``LinearSolver`` wrappers
  (same signatures as the reference's) and synthetic ``assembly.linforms``
* :mod:`.primitives` — single HIP kernels (SpMV, BLAS-1, GEMV, Gram)
* :mod:`.distributed` — row-partitioned multi-GPU solve (RCCL over xGMI)

The compute path is ``libspis.so`` (HIP, gfx950) behind the C-ABI in
``include/spis.h``; importing this package does not touch the GPU.
"""
__version__ = "0.1.0"
