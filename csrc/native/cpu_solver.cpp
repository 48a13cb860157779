#include "cpu_solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <numeric>
#include <stdexcept>
#include <string>

#include "cpu_kernels.hpp"

namespace sart {

CpuSolver::CpuSolver(const float* A, int64_t P, int64_t V, int64_t ld, HostComm* comm, const SolverParams& params,
                     bool gpu_semantics)
    : A_(A), P_(P), V_(V), ld_(ld), comm_(comm), p_(params), gpu_(gpu_semantics) {
    validate_params(p_);
    if (!comm_) throw std::invalid_argument("CpuSolver: communicator required");
    rho_.assign(V_, 0.0);
    ell_.assign(P_, 0.0);
    cpu_raysums(A_, P_, V_, ld_, rho_.data(), ell_.data());  // (reference sartsolver.cpp:38-56)
    init_scales();
}

CpuSolver::CpuSolver(HostCsr rows, HostComm* comm, const SolverParams& params, bool gpu_semantics)
    : A_(nullptr), sparse_(true), rows_(std::move(rows)), P_(rows_.nrows), V_(rows_.ncols), ld_(rows_.ncols),
      comm_(comm), p_(params), gpu_(gpu_semantics) {
    validate_params(p_);
    if (!comm_) throw std::invalid_argument("CpuSolver: communicator required");
    cols_ = csr_transpose(rows_);
    rho_.assign(V_, 0.0);
    ell_.assign(P_, 0.0);
    cpu_sparse_raysums(rows_, cols_, rho_.data(), ell_.data());
    init_scales();
}

void CpuSolver::backproject(const double* w, double* out) const {
    if (sparse_)
        cpu_csc_backproject(cols_, w, out);
    else
        cpu_backproject(A_, P_, V_, ld_, w, out);
}

void CpuSolver::init_scales() {
    comm_->all_reduce_host(rho_.data(), (size_t)V_, ReduceOp::kSum);
    dvalid_.assign(V_, 0);
    rho_s_.assign(V_, 1.0);
    inv_len_.assign(P_, 0.0);
    for (int64_t v = 0; v < V_; ++v) {
        if (gpu_) {  // fp32 thresholds on fp32-rounded sums, as the GPU kernels compare
            const float r32 = (float)rho_[v];
            dvalid_[v] = r32 > (float)p_.ray_density_threshold;
            rho_s_[v] = dvalid_[v] ? (double)r32 : 1.0;
        } else {
            dvalid_[v] = rho_[v] > p_.ray_density_threshold;
            rho_s_[v] = dvalid_[v] ? rho_[v] : 1.0;
        }
    }
    for (int64_t q = 0; q < P_; ++q) {
        if (gpu_) {
            const float l32 = (float)ell_[q];
            // fp32 reciprocal, as the kernels (sart_update.hip k_prep_rows) and the fp32 oracle
            inv_len_[q] = l32 > (float)p_.ray_length_threshold ? (double)(1.0f / (l32 > 0 ? l32 : 1.0f)) : 0.0;
        } else {
            inv_len_[q] = ell_[q] > p_.ray_length_threshold ? 1.0 / (ell_[q] != 0 ? ell_[q] : 1.0) : 0.0;
        }
    }
}

void CpuSolver::set_laplacian(const Csr& L) {
    has_lap_ = L.nnz() > 0 && p_.beta_laplace > 0;
    if (has_lap_ && L.n != V_) throw std::invalid_argument("Laplacian and ray-transfer matrices have different number of voxels.");
    L_ = L;
}

void CpuSolver::penalty(const std::vector<double>& x, std::vector<double>& pen) const {
    // beta * L x (linear) or beta * L log x (log), one row per iteration of a parallel loop (each row's sum in CSR
    // order: the result does not depend on the thread count) (reference sartsolver.cpp:190-199, 287-296)
    const bool lg = p_.logarithmic;
    const double beta = p_.beta_laplace;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < V_; ++r) {
        double s = 0.0;
        for (int64_t k = L_.row_ptr[r]; k < L_.row_ptr[r + 1]; ++k) {
            const double xv = x[L_.col[k]];
            s += (double)L_.val[k] * (lg ? std::log(xv) : xv);
        }
        pen[r] = beta * s;
    }
}

SolveInfo CpuSolver::solve(const double* g, const double* x0, double* x_out) {
    const auto t0 = std::chrono::steady_clock::now();
    const bool lg = p_.logarithmic;
    double norm = 1.0, eps = 1e-100, clamp = lg ? 1e-100 : -1.0;
    std::vector<double> gw(g, g + P_);
    if (gpu_) {
        double mx = -std::numeric_limits<double>::infinity();
        for (int64_t q = 0; q < P_; ++q) mx = std::max(mx, g[q]);
        norm = comm_->all_reduce_scalar(mx, ReduceOp::kMax);
        if (!(norm > 0)) norm = 1.0;
        for (int64_t q = 0; q < P_; ++q) gw[q] = (double)(float)(g[q] / norm);
        eps = clamp = 1e-7;
    }
    double gs = 0.0;
    for (int64_t q = 0; q < P_; ++q)
        if (g[q] > 0) gs += g[q] * g[q];
    const double G = comm_->all_reduce_scalar(gs, ReduceOp::kSum) / (norm * norm);
    std::vector<double> a(P_), w(P_), f(P_), red(V_), x(V_), O, pen(V_, 0.0);  // red: one-off back-projections
    for (int64_t q = 0; q < P_; ++q) a[q] = gw[q] >= 0 ? inv_len_[q] : 0.0;
    if (!x0) {  // cold start (reference sartsolver.cpp:150-160)
        for (int64_t q = 0; q < P_; ++q) w[q] = gpu_ ? std::max(gw[q], 0.0) : gw[q];
        backproject(w.data(), red.data());
        comm_->all_reduce_host(red.data(), (size_t)V_, ReduceOp::kSum);
        for (int64_t v = 0; v < V_; ++v) x[v] = dvalid_[v] ? red[v] / rho_s_[v] : 0.0;
    } else {
        for (int64_t v = 0; v < V_; ++v) x[v] = x0[v] / norm;
    }
    if (clamp > 0)
        for (auto& xv : x) xv = std::max(xv, clamp);
    if (lg) {
        O.assign(V_, 0.0);
        for (int64_t q = 0; q < P_; ++q) w[q] = a[q] * gw[q];
        backproject(w.data(), O.data());
        comm_->all_reduce_host(O.data(), (size_t)V_, ReduceOp::kSum);
        for (int64_t v = 0; v < V_; ++v)
            if (!dvalid_[v]) O[v] = 0.0;
    }
    // One read of A per iteration (cpu_sweep): the sweep after an update computes that iterate's forward
    // projection (for the convergence test) and, from it, the next iteration's back-projection, as the GPU fused
    // sweep does. red[0, V) and the sum of f^2 (red[V]) travel in one host all-reduce per iteration (the reference
    // runs two: sartsolver.cpp:206, 222).
    // SART_CPU_TWO_PASS=1: the forward and the back-projection as two reads of A (A/B measurements only)
    std::vector<double> redF(V_ + 1);
    const char* tp = std::getenv("SART_CPU_TWO_PASS");
    const bool two_pass = tp && *tp && std::atoi(tp) != 0;
    auto sweep = [&]() {
        if (sparse_) {  // two passes over the non-zeros (rows, then columns)
            redF[V_] = cpu_csr_forward(rows_, x.data(), f.data());
            for (int64_t q = 0; q < P_; ++q) w[q] = lg ? a[q] * f[q] : a[q] * (gw[q] - f[q]);
            cpu_csc_backproject(cols_, w.data(), redF.data());
        } else if (two_pass) {
            redF[V_] = cpu_forward(A_, P_, V_, ld_, x.data(), f.data());
            for (int64_t q = 0; q < P_; ++q) w[q] = lg ? a[q] * f[q] : a[q] * (gw[q] - f[q]);
            cpu_backproject(A_, P_, V_, ld_, w.data(), redF.data());
        } else {
            redF[V_] = cpu_sweep(A_, P_, V_, ld_, x.data(), gw.data(), a.data(), lg, f.data(), redF.data());
        }
        comm_->all_reduce_host(redF.data(), (size_t)V_ + 1, ReduceOp::kSum);
    };
    sweep();  // the start value's forward projection and the first back-projection
    SolveInfo info;
    info.status = -1;
    info.iterations = p_.max_iterations;
    double conv_prev = 0.0, conv = 0.0;
    for (int it = 0; it < p_.max_iterations; ++it) {
        if (has_lap_) penalty(x, pen);
        const double* red_ = redF.data();
        if (lg) {
#pragma omp parallel for schedule(static)
            for (int64_t v = 0; v < V_; ++v) {
                const double Fv = dvalid_[v] ? red_[v] : 0.0;
                x[v] = x[v] * std::pow((O[v] + eps) / (Fv + eps), p_.relaxation) * std::exp(-pen[v]);
            }
        } else {
#pragma omp parallel for schedule(static)
            for (int64_t v = 0; v < V_; ++v) {
                const double d = (dvalid_[v] ? p_.relaxation / rho_s_[v] * red_[v] : 0.0) - pen[v];
                const double xn = x[v] + d;
                x[v] = gpu_ ? std::max(xn, 0.0) : (std::signbit(xn) ? 0.0 : xn);
            }
        }
        sweep();
        const double F = redF[V_];
        conv = G != 0 ? (G - F) / G : 0.0;
        if (!std::isfinite(conv)) {
            info.nonfinite = true;
            info.iterations = it + 1;
            break;
        }
        if (it && std::abs(conv - conv_prev) < p_.conv_tolerance) {
            info.status = 0;
            info.iterations = it + 1;
            break;
        }
        conv_prev = conv;
    }
    for (int64_t v = 0; v < V_; ++v) x_out[v] = x[v] * norm;
    info.convergence = conv;
    info.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return info;
}

}  // namespace sart
