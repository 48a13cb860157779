#include "cpu_kernels.hpp"

#include "sparse_csr.hpp"

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
// The inner loops are built three times (AVX-512, AVX2, baseline SSE2) and picked at load time (GCC target_clones:
// the library is compiled here and runs on whatever host the GPU box has). Floating-point contraction is off for
// this library (_build.py), so every clone gives the same bits.
#define SART_CPU_CLONES __attribute__((target_clones("avx512f", "avx2", "default")))

// out[r] = A[r,:] . x for n consecutive rows: fp64 sums in a fixed order per row (eight interleaved partial sums --
// independent add chains the compiler vectorises; one chain is latency-bound at ~4 cycles per element -- combined
// pairwise); four rows at a time share each load of x.
SART_CPU_CLONES __attribute__((noinline)) void block_dots(const float* A, int64_t ld, int64_t n, int64_t V,
                                                          const double* x, double* out) {
    int64_t r = 0;
    for (; r + 4 <= n; r += 4) {
        const float* r0 = A + r * ld;
        const float* r1 = r0 + ld;
        const float* r2 = r1 + ld;
        const float* r3 = r2 + ld;
        double s0[8] = {}, s1[8] = {}, s2[8] = {}, s3[8] = {};
        int64_t v = 0;
        for (; v + 8 <= V; v += 8)
            for (int k = 0; k < 8; ++k) {
                const double xv = x[v + k];
                s0[k] += (double)r0[v + k] * xv;
                s1[k] += (double)r1[v + k] * xv;
                s2[k] += (double)r2[v + k] * xv;
                s3[k] += (double)r3[v + k] * xv;
            }
        for (; v < V; ++v) {
            s0[v & 7] += (double)r0[v] * x[v];
            s1[v & 7] += (double)r1[v] * x[v];
            s2[v & 7] += (double)r2[v] * x[v];
            s3[v & 7] += (double)r3[v] * x[v];
        }
        double* ss[4] = {s0, s1, s2, s3};
        for (int q = 0; q < 4; ++q) {
            const double* s = ss[q];
            out[r + q] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        }
    }
    for (; r < n; ++r) {
        const float* row = A + r * ld;
        double s[8] = {};
        int64_t v = 0;
        for (; v + 8 <= V; v += 8)
            for (int k = 0; k < 8; ++k) s[k] += (double)row[v + k] * x[v + k];
        for (; v < V; ++v) s[v & 7] += (double)row[v] * x[v];
        out[r] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    }
}

// acc[v] += sum_j A[rows[j], v] w[j] over the n listed rows of a block (weights already non-zero), four rows per
// pass over acc: one load and one store of the fp64 accumulator per four matrix elements instead of per element.
SART_CPU_CLONES __attribute__((noinline)) void block_axpy(const float* A, int64_t ld, const int32_t* rows,
                                                          const double* w, int64_t n, int64_t V, double* acc) {
    int64_t j = 0;
    for (; j + 4 <= n; j += 4) {
        const float* r0 = A + rows[j] * ld;
        const float* r1 = A + rows[j + 1] * ld;
        const float* r2 = A + rows[j + 2] * ld;
        const float* r3 = A + rows[j + 3] * ld;
        const double w0 = w[j], w1 = w[j + 1], w2 = w[j + 2], w3 = w[j + 3];
        for (int64_t v = 0; v < V; ++v)
            acc[v] += ((double)r0[v] * w0 + (double)r1[v] * w1) + ((double)r2[v] * w2 + (double)r3[v] * w3);
    }
    for (; j < n; ++j) {
        const float* row = A + rows[j] * ld;
        const double wj = w[j];
        for (int64_t v = 0; v < V; ++v) acc[v] += (double)row[v] * wj;
    }
}

// rows per block: ~128 KiB of A (a block's dot products, then its back-projection while it is still in L2)
inline int64_t rows_per_block(int64_t V) {
    return std::max<int64_t>(4, std::min<int64_t>(64, (128 << 10) / std::max<int64_t>(1, 4 * V)));
}

// out[v] = sum over threads of acc[t][v], in thread order
void reduce_threads(const std::vector<double>& acc, int nt, int64_t V, double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < V; ++v) {
        double s = 0.0;
        for (int t = 0; t < nt; ++t) s += acc[(size_t)t * V + v];
        out[v] = s;
    }
}
}  // namespace

double cpu_forward(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, double* f) {
    const int nt = omp_get_max_threads();
    std::vector<double> f2t((size_t)nt, 0.0);
    const int64_t rb = rows_per_block(V), nblk = (P + rb - 1) / rb;
#pragma omp parallel
    {
        double f2 = 0.0;
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nblk; ++b) {
            const int64_t p0 = b * rb, p1 = std::min(P, p0 + rb);
            block_dots(A + p0 * ld, ld, p1 - p0, V, x, f + p0);
            for (int64_t p = p0; p < p1; ++p) f2 += f[p] * f[p];
        }
        f2t[omp_get_thread_num()] = f2;
    }
    double f2 = 0.0;
    for (int t = 0; t < nt; ++t) f2 += f2t[t];  // fixed order
    return f2;
}

double cpu_sweep(const float* A, int64_t P, int64_t V, int64_t ld, const double* x, const double* g, const double* a,
                 bool logmode, double* f, double* out) {
    const int nt = omp_get_max_threads();
    std::vector<double> acc((size_t)nt * V, 0.0);
    std::vector<double> f2t((size_t)nt, 0.0);
    const int64_t rb = rows_per_block(V), nblk = (P + rb - 1) / rb;
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        double* mine = acc.data() + (size_t)tid * V;
        double f2 = 0.0;
        double wb[64];
        int32_t rows[64];
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nblk; ++b) {
            const int64_t p0 = b * rb, p1 = std::min(P, p0 + rb);
            block_dots(A + p0 * ld, ld, p1 - p0, V, x, f + p0);
            int64_t n = 0;
            for (int64_t p = p0; p < p1; ++p) {
                const double s = f[p];
                f2 += s * s;
                const double wp = logmode ? a[p] * s : a[p] * (g[p] - s);
                if (wp != 0.0) {
                    wb[n] = wp;
                    rows[n++] = (int32_t)(p - p0);
                }
            }
            block_axpy(A + p0 * ld, ld, rows, wb, n, V, mine);
        }
        f2t[tid] = f2;
    }
    double f2 = 0.0;
    for (int t = 0; t < nt; ++t) f2 += f2t[t];  // fixed order
    reduce_threads(acc, nt, V, out);
    return f2;
}

void cpu_backproject(const float* A, int64_t P, int64_t V, int64_t ld, const double* w, double* out) {
    const int nt = omp_get_max_threads();
    std::vector<double> acc((size_t)nt * V, 0.0);
    const int64_t rb = rows_per_block(V), nblk = (P + rb - 1) / rb;
#pragma omp parallel
    {
        double* mine = acc.data() + (size_t)omp_get_thread_num() * V;
        double wb[64];
        int32_t rows[64];
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nblk; ++b) {
            const int64_t p0 = b * rb, p1 = std::min(P, p0 + rb);
            int64_t n = 0;
            for (int64_t p = p0; p < p1; ++p)
                if (w[p] != 0.0) {
                    wb[n] = w[p];
                    rows[n++] = (int32_t)(p - p0);
                }
            block_axpy(A + p0 * ld, ld, rows, wb, n, V, mine);
        }
    }
    reduce_threads(acc, nt, V, out);
}

namespace {
inline double sparse_row_dot(const HostCsr& a, int64_t r, const double* x) {
    double s = 0.0;
    for (int64_t k = a.ptr[r]; k < a.ptr[r + 1]; ++k) s += (double)a.val[k] * x[a.idx[k]];
    return s;
}
}  // namespace

void cpu_sparse_raysums(const HostCsr& rows, const HostCsr& cols, double* rho, double* ell) {
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < rows.nrows; ++r) {
        double s = 0.0;
        for (int64_t k = rows.ptr[r]; k < rows.ptr[r + 1]; ++k) s += rows.val[k];
        ell[r] = s;
    }
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < cols.nrows; ++c) {
        double s = 0.0;
        for (int64_t k = cols.ptr[c]; k < cols.ptr[c + 1]; ++k) s += cols.val[k];
        rho[c] = s;
    }
}

double cpu_csr_forward(const HostCsr& rows, const double* x, double* f) {
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t r = 0; r < rows.nrows; ++r) f[r] = sparse_row_dot(rows, r, x);
    double f2 = 0.0;
    for (int64_t r = 0; r < rows.nrows; ++r) f2 += f[r] * f[r];  // row order
    return f2;
}

void cpu_csc_backproject(const HostCsr& cols, const double* w, double* out) {
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t c = 0; c < cols.nrows; ++c) out[c] = sparse_row_dot(cols, c, w);
}

}  // namespace sart
