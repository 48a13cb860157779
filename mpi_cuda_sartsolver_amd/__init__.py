"""mpi_cuda_sartsolver_amd -- MI355X-native constrained SART tomographic reconstruction.

Same capabilities, CLI and HDF5 formats as vsnever/mpi-cuda-sartsolver, re-designed for AMD MI355X
(gfx950): hand-written CDNA4 HIP kernels (fused single-pass SART sweep, MFMA multi-frame projections),
one process per GPU over torch.distributed/RCCL, device-resident convergence control, and a native
C++ runtime for HDF5 I/O, the CLI and the fp64 CPU solver.

Layout:
  ops/       native module loaders, device state view
  models/    RTM shard, SART solvers (GPU linear/log, multi-frame, CPU), Laplacian, fp64 oracles
  parallel/  row partition, communicators (RCCL / gloo / single process)
  io/        HDF5 inputs/outputs (native), composite image streamer, solution writer, voxel grids
  utils/     config, timing/profiling, synthetic problems
"""
__version__ = "0.1.0"
