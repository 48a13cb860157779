#include "solver_params.hpp"

#include <algorithm>
#include <numeric>
#include <stdexcept>

namespace sart {

void validate_params(const SolverParams& c) {
    if (c.ray_density_threshold < 0) throw std::invalid_argument("Ray density threshold must be non-negative.");
    if (c.ray_length_threshold < 0) throw std::invalid_argument("Ray length threshold must be non-negative.");
    if (c.conv_tolerance < 0 || (c.conv_tolerance == 0 && !c.allow_zero_tolerance))
        throw std::invalid_argument("Convolution tolerance must be positive.");
    if (c.beta_laplace < 0) throw std::invalid_argument("Attribute beta_laplace must be non-negative.");
    if (!(c.relaxation > 0 && c.relaxation <= 1.0))
        throw std::invalid_argument("Attribute relaxation must be within (0, 1] interval.");
    if (c.max_iterations <= 0) throw std::invalid_argument("Attribute max_iterations must be positive.");
}

Csr csr_from_coo(int64_t n, const std::vector<uint64_t>& i, const std::vector<uint64_t>& j,
                 const std::vector<float>& v) {
    if (i.size() != j.size() || i.size() != v.size())
        throw std::invalid_argument("i, j and value arrays must have the same length");
    std::vector<size_t> order(i.size());
    std::iota(order.begin(), order.end(), size_t(0));
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return i[a] * (uint64_t)n + j[a] < i[b] * (uint64_t)n + j[b];
    });
    Csr c;
    c.n = n;
    c.row_ptr.assign(n + 1, 0);
    c.col.resize(i.size());
    c.val.resize(i.size());
    for (size_t k = 0; k < order.size(); ++k) {
        const size_t o = order[k];
        if ((int64_t)i[o] >= n || (int64_t)j[o] >= n) throw std::invalid_argument("Laplacian index out of range");
        c.row_ptr[i[o] + 1]++;
        c.col[k] = (int32_t)j[o];
        c.val[k] = v[o];
    }
    for (int64_t r = 0; r < n; ++r) c.row_ptr[r + 1] += c.row_ptr[r];
    return c;
}

}  // namespace sart
