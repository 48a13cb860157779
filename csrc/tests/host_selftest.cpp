// Self-test of the native host runtime, built with AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/test_sanitizers.py; SURVEY 5.2: the reference has no sanitizer coverage). Exercises the CLI parser,
// time intervals, partitioning, CSR conversion, the host communicator, the fp64 CPU kernels and solver,
// and an HDF5 round trip (fixture writers -> validation -> row reader -> composite image -> solution
// writer -> reader). Exit code 0 = all checks passed.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../native/config.hpp"
#include "../native/cpu_kernels.hpp"
#include "../native/cpu_solver.hpp"
#include "../native/fixtures.hpp"
#include "../native/frames.hpp"
#include "../native/host_comm.hpp"
#include "../native/inputs.hpp"
#include "../native/solver_params.hpp"

using namespace sart;

static int failures = 0;
#define CHECK(cond)                                                             \
    do {                                                                        \
        if (!(cond)) {                                                          \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                         \
        }                                                                       \
    } while (0)

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    // CLI
    Config c = parse_arguments({"-m", "50", "-c", "1e-6", "-L", "-o", "out.h5", "a.h5", "b.h5"});
    CHECK(c.max_iterations == 50 && c.logarithmic && c.input_files.size() == 2 && c.output_file == "out.h5");
    bool threw = false;
    try {
        parse_arguments({"-R", "3", "a.h5", "b.h5"});
    } catch (const std::exception&) {
        threw = true;
    }
    CHECK(threw);
    auto iv = parse_time_intervals("0:1:0.1, 2:3");
    CHECK(iv.size() == 2 && iv[0][2] == 0.1);
    // partition
    uint64_t total = 0;
    for (int r = 0; r < 7; ++r) total += block_partition(100, 7, r).size;
    CHECK(total == 100 && block_partition(100, 7, 0).size == 15 && block_partition(100, 7, 6).offset == 86);
    // CSR
    Csr L = csr_from_coo(4, {2, 0, 1, 0}, {1, 0, 1, 3}, {1.f, 2.f, 3.f, 4.f});
    CHECK(L.row_ptr == (std::vector<int64_t>{0, 2, 3, 4, 4}) && L.col[1] == 3 && L.val[3] == 1.f);
    // CPU solver vs its own invariants on a consistent system
    const int64_t P = 300, V = 120;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    std::vector<float> A(P * V);
    for (auto& a : A) a = U(rng);
    std::vector<double> xt(V), g(P, 0.0), x(V);
    for (auto& v : xt) v = U(rng) + 0.1;
    for (int64_t p = 0; p < P; ++p)
        for (int64_t v = 0; v < V; ++v) g[p] += (double)A[p * V + v] * xt[v];
    auto comm = make_local_host_comm();
    for (int lg = 0; lg < 2; ++lg) {
        SolverParams sp;
        sp.logarithmic = lg;
        sp.max_iterations = 400;
        sp.conv_tolerance = 1e-9;
        CpuSolver s(A.data(), P, V, V, comm.get(), sp, lg == 1);
        const SolveInfo info = s.solve(g.data(), nullptr, x.data());
        std::vector<double> f(P);
        cpu_forward(A.data(), P, V, V, x.data(), f.data());
        double num = 0, den = 0;
        for (int64_t p = 0; p < P; ++p) num += (f[p] - g[p]) * (f[p] - g[p]), den += g[p] * g[p];
        CHECK(info.iterations > 0 && std::sqrt(num / den) < 5e-2);
    }
    // HDF5 round trip
    RtmFileSpec r;
    r.path = dir + "/selftest_rtm.h5";
    r.camera_name = "cam";
    r.wavelength = 500;
    r.frame_h = 4, r.frame_w = 5;
    r.frame_mask.assign(20, 1);
    r.frame_mask[3] = 0;
    r.npixel = 19, r.nvoxel = 8;
    r.value.resize(19 * 8);
    for (auto& v : r.value) v = U(rng);
    r.nx = 2, r.ny = 2, r.nz = 2;
    for (uint64_t i = 0; i < 2; ++i)
        for (uint64_t j = 0; j < 2; ++j)
            for (uint64_t k = 0; k < 2; ++k) r.vi.push_back(i), r.vj.push_back(j), r.vk.push_back(k),
                                              r.vvalue.push_back((int32_t)(i * 4 + j * 2 + k));
    write_rtm_file(r);
    std::vector<double> frames(3 * 20, 1.0);
    write_image_file(dir + "/selftest_img.h5", "cam", 500, {0.0, 0.1, 0.2}, frames, 4, 5);
    InputSet in = validate_inputs({r.path, dir + "/selftest_img.h5"}, "with_reflections", 50.0);
    CHECK(in.npixel == 19 && in.nvoxel == 8 && in.camera_names.size() == 1);
    std::vector<float> rows(19 * 8, 0.f);
    read_rtm_rows(in.rtm_files, in.rtm_name, 8, 0, 19, rows.data(), 8);
    CHECK(rows == r.value);
    {  // sparse path: CSR of the same rows (read_csr), its transpose, and the one-read CPU sweep
        RtmReader rd(in.rtm_files, in.rtm_name, 8);
        const HostCsr a = rd.read_csr(2, 17);
        CHECK(a.nrows == 15 && a.ncols == 8 && (int64_t)a.ptr.size() == 16);
        bool same = true;
        for (int64_t i = 0; i < 15; ++i)
            for (int64_t k = a.ptr[i]; k < a.ptr[i + 1]; ++k) same = same && a.val[k] == r.value[(i + 2) * 8 + a.idx[k]];
        CHECK(same && a.nnz() == 15 * 8);
        const HostCsr t = csr_transpose(a);
        CHECK(t.nrows == 8 && t.ncols == 15 && t.nnz() == a.nnz() && t.ptr[8] == a.nnz());
        const HostCsr d = csr_from_entries(3, 4, {2, 0, 2, 0}, {1, 3, 1, 0}, {1.f, 2.f, 5.f, 0.f});
        CHECK(d.ptr == (std::vector<int64_t>{0, 1, 1, 2}) && d.val[1] == 5.f && d.idx[0] == 3);
        std::vector<double> xx(8, 1.0), gg(19, 1.0), aa(19, 0.5), ff(19), oo(8);
        const double f2 = cpu_sweep(rows.data(), 19, 8, 8, xx.data(), gg.data(), aa.data(), false, ff.data(), oo.data());
        CHECK(std::isfinite(f2) && f2 > 0);
    }
    CompositeImage ci(in.image_files, in.frame_masks, parse_time_intervals(""), 19, 0);
    CHECK(ci.nframe() == 3 && ci.frame(1).size() == 19);
    {
        SolutionWriter w(dir + "/selftest_sol.h5", in.camera_names, 8, 2, false);
        for (int k = 0; k < 3; ++k) w.add(std::vector<double>(8, k), 0, 0.1 * k, {0.1 * k}, 5);
    }
    StoredSolutions st = read_solution_file(dir + "/selftest_sol.h5");
    CHECK(st.time.size() == 3 && st.last_solution.size() == 8 && st.last_solution[0] == 2.0);
    if (failures) std::fprintf(stderr, "%d check(s) failed\n", failures);
    else std::printf("host selftest OK\n");
    return failures ? 1 : 0;
}
