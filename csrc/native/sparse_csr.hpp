// Host CSR matrices for the sparse RTM path (csrc/kernels/sparse.hip): built from the input's COO datasets (or from
// the non-zeros of dense datasets) by RtmReader::read_csr, transposed once per shard for the device CSC copy.
#pragma once

#include <cstdint>
#include <vector>

namespace sart {

struct HostCsr {
    int64_t nrows = 0, ncols = 0;
    std::vector<int64_t> ptr;  // [nrows + 1]
    std::vector<int32_t> idx;  // column of each entry, ascending within a row
    std::vector<float> val;
    int64_t nnz() const { return (int64_t)val.size(); }
    double density() const { return nrows && ncols ? (double)val.size() / ((double)nrows * (double)ncols) : 0.0; }
};

// Row-major entries (row, col, value) appended in input order -> CSR: rows ascending, columns ascending within a
// row; an entry repeated at the same (row, col) keeps the LAST value appended (what scattering the entries into a
// dense shard in that order leaves); exact zeros are dropped. Throws std::invalid_argument on an index out of range.
HostCsr csr_from_entries(int64_t nrows, int64_t ncols, const std::vector<int64_t>& rows,
                         const std::vector<int32_t>& cols, const std::vector<float>& vals);
// Throws std::invalid_argument unless ptr has nrows + 1 non-decreasing entries from 0 to nnz and every column index
// lies in [0, ncols) (who: the caller's name in the message).
void csr_validate(const HostCsr& a, const char* who);
// A^T in CSR form (= A in CSC form): entries of each column in ascending row order. Validates a first (csr_validate).
HostCsr csr_transpose(const HostCsr& a);

}  // namespace sart
