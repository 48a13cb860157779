// Solver parameters, results and the Laplacian CSR shared by the GPU engine and the CPU solver.
#pragma once

#include <cstdint>
#include <vector>

namespace sart {

// Reference defaults (sartsolver.hpp:64-66; the CLI overrides beta_laplace with 2e-2, arguments.cpp:125).
struct SolverParams {
    bool logarithmic = false;
    double ray_density_threshold = 1e-6;
    double ray_length_threshold = 1e-6;
    double conv_tolerance = 1e-5;
    double beta_laplace = 1e-2;
    double relaxation = 1.0;
    int max_iterations = 2000;
    bool allow_zero_tolerance = false;  // benchmarks: run exactly max_iterations
};

// Same checks and messages as the reference setters (sartsolver.cpp:61-123); throws std::invalid_argument.
void validate_params(const SolverParams& p);

struct SolveInfo {
    int status = -1;          // 0 SUCCESS, -1 MAX_ITERATIONS_EXCEEDED (reference sartsolver.cpp:16-17)
    int iterations = 0;
    double convergence = 0.0; // last (G - ||A x||^2) / G
    bool used_fused = false;
    int fused_variant = -1;
    int fallbacks = 0;        // persistent-kernel protocol timeouts survived during this solve
    int comm_fallbacks = 0;   // device all-reduce timeouts survived (the frame re-solved on the base communicator)
    const char* comm = "";    // device communicator that produced the result (static string)
    bool nonfinite = false;   // the iteration produced NaN/Inf and was stopped
    double ms = 0.0;
    int sweeps = 0;           // sweeps executed on the device (iterations + the final decision sweep)
    double comm_ms = -1.0;    // GPU time inside the per-sweep all-reduces (EngineConfig::time_collectives; else -1)
    int warm_from = -1;       // multi-frame time series: index of the frame whose iterate started this one
                              // (-1: the caller's x0, or cold)
    int warm_iter = -1;       // the update count of that iterate (its final count when it had finished)
    bool warm_live = false;   // that frame was still in flight (its iterate extrapolated along its last update)
    // per-frame breakdown of ms (single-frame engine): host + device setup of the frame (normalisation, H2D of g
    // and x0, cold-start back-projection) up to the first queued sweep, the sweep loop up to the final state
    // check, the read-back of x (D2H and de-normalisation); sweeps queued in total (the chunks past the
    // convergence sweep run as no-op sweeps)
    double setup_ms = 0.0, iterate_ms = 0.0, finish_ms = 0.0;
    int queued_sweeps = 0;
};

// CSR over n rows (row_ptr int64, col int32, val fp32), from the reference's sorted-flat-index COO
// (laplacian.cpp:34-91).
struct Csr {
    int64_t n = 0;
    std::vector<int64_t> row_ptr;
    std::vector<int32_t> col;
    std::vector<float> val;
    int64_t nnz() const { return (int64_t)val.size(); }
};
Csr csr_from_coo(int64_t n, const std::vector<uint64_t>& i, const std::vector<uint64_t>& j,
                 const std::vector<float>& v);

}  // namespace sart
