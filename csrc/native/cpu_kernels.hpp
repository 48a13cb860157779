// fp64 CPU projection kernels over an fp32 row-major RTM shard (the --use_cpu path).
//
// Reference: the CPU solvers run O(P*V) triple loops single-threaded, with the back-projection
// striding down columns of a row-major matrix (reference sartsolver.cpp:38-56, 191-220). Here every
// kernel streams rows contiguously and is parallel over rows (OpenMP); the back-projection keeps one
// fp64 accumulator per thread and reduces them in a fixed order, so the result does not depend on
// scheduling (it depends only on the thread count).
#pragma once

#include <cstdint>

namespace sart {

int cpu_num_threads();
void cpu_set_num_threads(int n);

// rho[v] = sum_p A[p,v], ell[p] = sum_v A[p,v] (fp64)
void cpu_raysums(const float* A, int64_t P, int64_t V, int64_t ld, double* rho, double* ell);
// f[p] = sum_v A[p,v] x[v]; returns sum_p f[p]^2
double cpu_forward(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, double* f);
// out[v] = sum_p A[p,v] w[p]
void cpu_backproject(const float* A, int64_t P, int64_t V, int64_t ld, const double* w, double* out);
// One read of A per SART iteration (the CPU counterpart of the GPU fused sweep): per row, f[p] = A[p,:] x, then
// w_p = a[p] f[p] (log) or a[p] (g[p] - f[p]) (linear) and out += A[p,:]^T w_p while the row is still in cache.
// Returns sum_p f[p]^2. out: the back-projection of the NEXT iteration's weights (x is the iterate after this
// iteration's update).
double cpu_sweep(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, const double* g, const double* a,
                 bool logmode, double* f, double* out);

// Sparse shard (the --rtm_format sparse CPU path): CSR rows and CSC columns of the same matrix (sparse_csr.hpp).
// Every row / column sum runs in its entries' order, one output per loop iteration: the results do not depend on
// the thread count.
struct HostCsr;
void cpu_sparse_raysums(const HostCsr& rows, const HostCsr& cols, double* rho, double* ell);
double cpu_csr_forward(const HostCsr& rows, const double* x, double* f);  // returns sum_p f[p]^2
void cpu_csc_backproject(const HostCsr& cols, const double* w, double* out);

}  // namespace sart
