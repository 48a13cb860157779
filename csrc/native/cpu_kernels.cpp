#include "cpu_kernels.hpp"

#include <omp.h>

#include <algorithm>
#include <vector>

namespace sart {

int cpu_num_threads() { return omp_get_max_threads(); }
void cpu_set_num_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
}

void cpu_raysums(const float* A, int64_t P, int64_t V, int64_t ld, double* rho, double* ell) {
    const int nt = omp_get_max_threads();
    std::vector<double> acc((size_t)nt * V, 0.0);
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        double* mine = acc.data() + (size_t)tid * V;
#pragma omp for schedule(static)
        for (int64_t p = 0; p < P; ++p) {
            const float* row = A + p * ld;
            double s = 0.0;
            for (int64_t v = 0; v < V; ++v) {
                const double a = row[v];
                s += a;
                mine[v] += a;
            }
            ell[p] = s;
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < V; ++v) {
        double s = 0.0;
        for (int t = 0; t < nt; ++t) s += acc[(size_t)t * V + v];
        rho[v] = s;
    }
}

double cpu_forward(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, double* f) {
    double f2 = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : f2)
    for (int64_t p = 0; p < P; ++p) {
        const float* row = A + p * ld;
        double s = 0.0;
        for (int64_t v = 0; v < V; ++v) s += (double)row[v] * x[v];
        f[p] = s;
        f2 += s * s;
    }
    return f2;
}

void cpu_backproject(const float* A, int64_t P, int64_t V, int64_t ld, const double* w, double* out) {
    const int nt = omp_get_max_threads();
    std::vector<double> acc((size_t)nt * V, 0.0);
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        double* mine = acc.data() + (size_t)tid * V;
#pragma omp for schedule(static)
        for (int64_t p = 0; p < P; ++p) {
            const double wp = w[p];
            if (wp == 0.0) continue;
            const float* row = A + p * ld;
            for (int64_t v = 0; v < V; ++v) mine[v] += (double)row[v] * wp;
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < V; ++v) {
        double s = 0.0;
        for (int t = 0; t < nt; ++t) s += acc[(size_t)t * V + v];
        out[v] = s;
    }
}

}  // namespace sart
