#include "sparse_csr.hpp"

#include <omp.h>

#include <algorithm>
#include <numeric>
#include <stdexcept>
#include <string>

namespace sart {

HostCsr csr_from_entries(int64_t nrows, int64_t ncols, const std::vector<int64_t>& rows,
                         const std::vector<int32_t>& cols, const std::vector<float>& vals) {
    if (rows.size() != cols.size() || rows.size() != vals.size())
        throw std::invalid_argument("csr_from_entries: rows, cols and values differ in length");
    if (ncols > INT32_MAX) throw std::invalid_argument("csr_from_entries: more than 2^31 - 1 columns");
    const size_t n = vals.size();
    std::vector<int64_t> count(nrows + 1, 0);
    for (size_t t = 0; t < n; ++t) {
        if (rows[t] < 0 || rows[t] >= nrows || cols[t] < 0 || cols[t] >= ncols)
            throw std::invalid_argument("csr_from_entries: entry (" + std::to_string(rows[t]) + ", " +
                                        std::to_string(cols[t]) + ") outside the matrix");
        ++count[rows[t] + 1];
    }
    std::partial_sum(count.begin(), count.end(), count.begin());
    // stable counting sort by row: the entries of a row keep their input order
    std::vector<size_t> order(n);
    {
        std::vector<int64_t> next(count.begin(), count.end() - 1);
        for (size_t t = 0; t < n; ++t) order[next[rows[t]]++] = t;
    }
    HostCsr a;
    a.nrows = nrows;
    a.ncols = ncols;
    a.ptr.assign(nrows + 1, 0);
    a.idx.reserve(n);
    a.val.reserve(n);
    std::vector<size_t> rowv;
    for (int64_t r = 0; r < nrows; ++r) {
        rowv.assign(order.begin() + count[r], order.begin() + count[r + 1]);
        std::stable_sort(rowv.begin(), rowv.end(), [&](size_t p, size_t q) { return cols[p] < cols[q]; });
        for (size_t k = 0; k < rowv.size(); ++k) {
            if (k + 1 < rowv.size() && cols[rowv[k + 1]] == cols[rowv[k]]) continue;  // a later duplicate wins
            const float v = vals[rowv[k]];
            if (v == 0.0f) continue;
            a.idx.push_back(cols[rowv[k]]);
            a.val.push_back(v);
        }
        a.ptr[r + 1] = (int64_t)a.val.size();
    }
    return a;
}

void csr_validate(const HostCsr& a, const char* who) {
    const std::string w(who);
    if (a.nrows < 0 || a.ncols < 0) throw std::invalid_argument(w + ": negative shape");
    if (a.ncols > INT32_MAX) throw std::invalid_argument(w + ": more than 2^31 - 1 columns");
    if ((int64_t)a.ptr.size() != a.nrows + 1) throw std::invalid_argument(w + ": row pointer needs nrows + 1 entries");
    if (a.idx.size() != a.val.size()) throw std::invalid_argument(w + ": column indices and values differ in length");
    if (a.ptr[0] != 0 || a.ptr[a.nrows] != (int64_t)a.idx.size())
        throw std::invalid_argument(w + ": row pointer must start at 0 and end at the number of entries");
    for (int64_t r = 0; r < a.nrows; ++r)
        if (a.ptr[r + 1] < a.ptr[r])
            throw std::invalid_argument(w + ": row pointer decreases at row " + std::to_string(r));
    for (size_t k = 0; k < a.idx.size(); ++k)
        if (a.idx[k] < 0 || (int64_t)a.idx[k] >= a.ncols)
            throw std::invalid_argument(w + ": column index " + std::to_string(a.idx[k]) + " outside [0, " +
                                        std::to_string(a.ncols) + ")");
}

HostCsr csr_transpose(const HostCsr& a) {
    if (a.nrows > INT32_MAX) throw std::invalid_argument("csr_transpose: more than 2^31 - 1 rows");
    // a malformed CSR (user arrays through SparseRTM) would index outside the buffers below, and its device copy
    // would make the gather kernels read outside x / Xt
    csr_validate(a, "csr_transpose");
    HostCsr t;
    t.nrows = a.ncols;
    t.ncols = a.nrows;
    t.ptr.assign(a.ncols + 1, 0);
    t.idx.resize(a.idx.size());
    t.val.resize(a.val.size());
    // Threads take contiguous row blocks of about equal entry counts: per-thread column counts, turned in place into
    // each thread's cursors (a column's start plus the earlier blocks' entries), so every column's entries still come
    // out in row order (the sequential transpose's result, bitwise). At most 4 threads: the cursors are 8 bytes per
    // column and thread, host memory on top of the CSR + CSC. A small matrix runs on one thread.
    const int64_t nnz = a.nnz();
    const int nth = nnz < (1 << 20) ? 1 : std::max(1, std::min(omp_get_max_threads(), 4));
    std::vector<int64_t> rcut(nth + 1, a.nrows);
    rcut[0] = 0;
    for (int q = 1, r = 0; q < nth; ++q) {
        const int64_t goal = nnz * q / nth;
        while (r < a.nrows && a.ptr[r] < goal) ++r;
        rcut[q] = r;
    }
    std::vector<int64_t> cur((size_t)nth * a.ncols, 0);
#pragma omp parallel num_threads(nth)
    {
        const int q = omp_get_thread_num();
        int64_t* cq = cur.data() + (size_t)q * a.ncols;
        for (int64_t k = a.ptr[rcut[q]]; k < a.ptr[rcut[q + 1]]; ++k) ++cq[a.idx[k]];
    }
    for (int64_t c = 0, base = 0; c < a.ncols; ++c) {
        t.ptr[c] = base;
        for (int q = 0; q < nth; ++q) {
            const int64_t n = cur[(size_t)q * a.ncols + c];
            cur[(size_t)q * a.ncols + c] = base;
            base += n;
        }
        t.ptr[c + 1] = base;
    }
#pragma omp parallel num_threads(nth)
    {
        const int q = omp_get_thread_num();
        int64_t* next = cur.data() + (size_t)q * a.ncols;
        for (int64_t r = rcut[q]; r < rcut[q + 1]; ++r)
            for (int64_t k = a.ptr[r]; k < a.ptr[r + 1]; ++k) {
                const int64_t d = next[a.idx[k]]++;
                t.idx[d] = (int32_t)r;
                t.val[d] = a.val[k];
            }
    }
    return t;
}

}  // namespace sart
