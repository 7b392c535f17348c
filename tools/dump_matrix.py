"""Dump the bench matrix (swe-shaped, config C3) as raw int32/float64 files for tools/kbench."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 289
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/kbench_mat"
dic, _ = assembly.linforms(M=M)
A = dic["A"]
os.makedirs(out, exist_ok=True)
np.array([A.shape[0], A.nnz], dtype=np.int64).tofile(f"{out}/shape.bin")
A.indptr.astype(np.int32).tofile(f"{out}/indptr.bin")
A.indices.astype(np.int32).tofile(f"{out}/indices.bin")
A.data.astype(np.float64).tofile(f"{out}/data.bin")
print("dumped", A.shape, A.nnz)
