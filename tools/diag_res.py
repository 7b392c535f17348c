import sys, numpy as np
sys.path.insert(0,'.')
from structurepreservingiterativesolvers_amd import solvers
from structurepreservingiterativesolvers_amd.device import set_option
from structurepreservingiterativesolvers_amd.swe import LinearSolver as swe_ls
from structurepreservingiterativesolvers_amd.swe import assembly as sa
import oracle
dic, _ = sa.linforms(M=30)
cons = swe_ls.constraints(dic, np.zeros_like(dic["b"]))
A, b = dic["A"], dic["b"]
xr, dr = oracle.cgmres(A, b, np.zeros_like(b), 25, tol=1e-19, conlist=cons)
print("oracle", np.asarray(dr["res"])[-3:])
for gram in ("ell","mfma"):
  set_option("ell_gram", gram)
  for pipe in ("off","stride","xcd","stride2","xcd2"):
    set_option("spmv_pipe", pipe)
    x, d = solvers.cgmres(A, b, np.zeros_like(b), 25, tol=1e-19, conlist=cons)
    r=np.asarray(d["res"])
    print(gram, pipe, r[-3:], np.linalg.norm(x-xr)/np.linalg.norm(xr))
set_option("spmv_pipe","auto"); set_option("ell_gram","mfma")
