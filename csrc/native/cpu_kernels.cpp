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

namespace {
// fp64 row dot in a fixed order: eight interleaved partial sums (independent add chains the compiler vectorises;
// one chain is latency-bound at ~4 cycles per element), combined pairwise
inline double row_dot(const float* row, const double* x, int64_t V) {
    double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t v = 0;
    for (; v + 8 <= V; v += 8)
        for (int k = 0; k < 8; ++k) s[k] += (double)row[v + k] * x[v + k];
    for (; v < V; ++v) s[v & 7] += (double)row[v] * x[v];
    return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}
}  // namespace

double cpu_forward(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, double* f) {
    double f2 = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : f2)
    for (int64_t p = 0; p < P; ++p) {
        const double s = row_dot(A + p * ld, x, V);
        f[p] = s;
        f2 += s * s;
    }
    return f2;
}

double cpu_sweep(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, const double* g, const double* a,
                 bool logmode, double* f, double* out) {
    const int nt = omp_get_max_threads();
    std::vector<double> acc((size_t)nt * V, 0.0);
    std::vector<double> f2t((size_t)nt, 0.0);
    // rows in blocks of ~128 KiB of A: the block's dot products first (independent rows keep the FMA pipes busy; a
    // row's back-projection depends on its own dot), then its back-projection while the block is in L2
    const int64_t rb = std::max<int64_t>(1, std::min<int64_t>(64, (128 << 10) / std::max<int64_t>(1, 4 * V)));
    const int64_t nblk = (P + rb - 1) / rb;
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        double* mine = acc.data() + (size_t)tid * V;
        double f2 = 0.0;
        double wb[64];
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nblk; ++b) {
            const int64_t p0 = b * rb, p1 = std::min(P, p0 + rb);
            for (int64_t p = p0; p < p1; ++p) {
                const double s = row_dot(A + p * ld, x, V);
                f[p] = s;
                f2 += s * s;
                wb[p - p0] = logmode ? a[p] * s : a[p] * (g[p] - s);
            }
            for (int64_t p = p0; p < p1; ++p) {
                const double wp = wb[p - p0];
                if (wp == 0.0) continue;
                const float* row = A + p * ld;
                for (int64_t v = 0; v < V; ++v) mine[v] += (double)row[v] * wp;
            }
        }
        f2t[tid] = f2;
    }
    double f2 = 0.0;
    for (int t = 0; t < nt; ++t) f2 += f2t[t];  // fixed order
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < V; ++v) {
        double s = 0.0;
        for (int t = 0; t < nt; ++t) s += acc[(size_t)t * V + v];
        out[v] = s;
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
