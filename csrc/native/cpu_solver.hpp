// CPU SART solvers (the --use_cpu path): fp64 arithmetic over the fp32 RTM shard, host collectives.
//
// Reference: SARTSolverMPI / LogSARTSolverMPI (reference sartsolver.cpp:133-339). gpu_semantics = false
// reproduces the reference CPU path exactly (no normalisation; the cold start back-projects the raw
// measurement including negative, saturated pixels; no 1e-7 clamp in linear mode; 1e-100 clamp and
// epsilon in log mode). gpu_semantics = true evaluates the GPU semantics in fp64 (the oracle).
// The O(P*V) loops are the OpenMP kernels of cpu_kernels.hpp.
#pragma once

#include <cstdint>
#include <vector>

#include "host_comm.hpp"
#include "sparse_csr.hpp"
#include "solver_params.hpp"

namespace sart {

class CpuSolver {
   public:
    // A: row-major fp32 [P x ld] (not owned), comm: host collectives (not owned).
    CpuSolver(const float* A, int64_t P, int64_t V, int64_t ld, HostComm* comm, const SolverParams& params,
              bool gpu_semantics = false);
    // sparse shard: the CSR rows (P x V) and their transpose (owned copies); forward and back-projection as two
    // passes over the non-zeros
    CpuSolver(HostCsr rows, HostComm* comm, const SolverParams& params, bool gpu_semantics = false);
    bool sparse() const { return sparse_; }
    void set_laplacian(const Csr& L);
    SolveInfo solve(const double* g, const double* x0, double* x_out);
    const std::vector<double>& ray_density() const { return rho_; }
    const std::vector<double>& ray_length() const { return ell_; }

   private:
    void penalty(const std::vector<double>& x, std::vector<double>& pen) const;
    void init_scales();
    void backproject(const double* w, double* out) const;
    const float* A_;
    bool sparse_ = false;
    HostCsr rows_, cols_;
    int64_t P_, V_, ld_;
    HostComm* comm_;
    SolverParams p_;
    bool gpu_;
    Csr L_;
    bool has_lap_ = false;
    std::vector<double> rho_, ell_, rho_s_, inv_len_;
    std::vector<char> dvalid_;
};

}  // namespace sart
