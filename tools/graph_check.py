import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams
from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
from mpi_cuda_sartsolver_amd.utils.synthetic import host_problem
dev = torch.device("cuda", 0)
A, g, _ = host_problem(2048, 4096, seed=3)
kw = dict(max_iterations=40, conv_tolerance=0.0)
xr, _, _ = sart_gpu_semantics(A, g, **kw)
for fused in (True, False):
    for graph in (True, False):  # graph first: the first chunk of a fresh engine must not be captured
        s = SARTSolver(DenseRTM.from_dense(A, device=dev), None, None, SolverParams(**kw), allow_zero_tolerance=True,
                       use_fused=fused, use_graph=graph)
        r = s.solve(g)
        print(f"fused={fused} graph={graph} it={r.iterations} rel={np.linalg.norm(r.solution - xr) / np.linalg.norm(xr):.3e}", flush=True)
