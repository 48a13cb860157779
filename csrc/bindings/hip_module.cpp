// Python bindings of the gfx950 SART kernels (module mpi_cuda_sartsolver_amd._lib._sart_hip).
//
// The interface is deliberately ABI-neutral: device pointers and HIP streams are passed as integers
// (torch.Tensor.data_ptr(), torch.cuda.Stream.cuda_stream), so this module links only against the
// HIP runtime and works with any PyTorch-ROCm build. Launch functions never allocate, copy or
// synchronise, so callers may capture them into HIP graphs.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "../kernels/sart_common.hpp"

namespace py = pybind11;

namespace sart {
// projection.hip
int64_t forward_num_blocks(int64_t nrows_pad);
void launch_forward(int epi, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                    const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                    const SartState* st, hipStream_t stream);
void launch_rowsum_f64(const float* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream);
int backproject_num_splits(int64_t ld, int64_t nrows);
void launch_backproject(const float* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                        const SartState* st, hipStream_t stream);
void launch_colsum_f64(const float* A, int64_t ld, int64_t nrows, int nsplit, double* partial, hipStream_t stream);
void launch_reduce_partials(const float* partial, int64_t ld, int nsplit, const float* scale, float* out,
                            const double* Fpart, int64_t nF, float* Fout, const SartState* st, hipStream_t stream);
void launch_reduce_partials_f64(const double* partial, int64_t ld, int nsplit, double* out, hipStream_t stream);
// sart_update.hip
void launch_prep_rows(const double* g, int64_t nrows, int64_t nrows_pad, double inv_s, const float* ray_length,
                      float len_thres, float* ghat, float* arow, float* gpos, float* wo, hipStream_t stream);
void launch_init_solution(float* x, int64_t n, int64_t n_pad, const float* src_f32, const double* src_f64,
                          double scale, hipStream_t stream);
void launch_penalty(bool logx, const int64_t* row_ptr, const int32_t* col, const float* val, int64_t n, float beta,
                    const float* x, float* pen, const SartState* st, hipStream_t stream);
void launch_decide(SartState* st, const float* Fslot, hipStream_t stream);
void launch_update_linear(float* x, const float* d, const float* pen, int64_t n, const SartState* st,
                          hipStream_t stream);
void launch_update_log(float* x, const float* O, const float* Fv, const float* pen, float alpha, int64_t n,
                       const SartState* st, hipStream_t stream);
void launch_state_begin(SartState* st, double G, double tol, int max_iter, hipStream_t stream);
// synth.hip
void launch_synth_matrix(float* A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols, int64_t row_offset,
                         uint64_t seed, float lo, float hi, hipStream_t stream);
void launch_synth_vector(double* out, int64_t n, int64_t offset, uint64_t seed, double lo, double hi,
                         hipStream_t stream);
// fused_sweep.hip
int fused_pick_k(int64_t ld);
int fused_tile_rows(int K, int variant);
void fused_set_schedule(int sched);
int fused_get_schedule();
void fused_set_trace(unsigned long long* buf, long long tiles);
std::vector<int> fused_debug_map(int nblocks);
int fused_fpart_per_block(int variant);
void fused_set_debug(int flags);
std::vector<unsigned long long> fused_debug_stats(int nblocks);
void launch_fused_sweep(bool logmode, int K, int variant, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                        const float* x, const float* ghat, const float* arow, float* partial, double* Fpart,
                        uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt, hipStream_t stream);
// multiframe.hip
int mf_forward_num_splits(int64_t ld, int64_t nrows_pad);
int mf_backproject_num_splits(int64_t ld, int64_t nrows);
void launch_mf_forward(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* X, int64_t ldx,
                       float* Fout, int nsplit, hipStream_t stream);
void launch_mf_backproject(const float* A, int64_t ld, int64_t nrows, const float* W, int nsplit, float* partial,
                           hipStream_t stream);
}  // namespace sart

template <typename T>
static T* P(uintptr_t p) {
    return reinterpret_cast<T*>(p);
}
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

PYBIND11_MODULE(_sart_hip, m) {
    m.doc() = "Hand-written gfx950 (CDNA4) HIP kernels of the SART solver";

    m.def("arch", []() { return std::string("gfx950"); });
    m.def("state_nbytes", []() { return (int)sizeof(sart::SartState); });

    m.def("device_info", [](int dev) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) throw std::runtime_error("hipGetDeviceProperties failed");
        py::dict d;
        d["name"] = std::string(prop.name);
        d["gcnArchName"] = std::string(prop.gcnArchName);
        d["multiProcessorCount"] = prop.multiProcessorCount;
        d["totalGlobalMem"] = (int64_t)prop.totalGlobalMem;
        d["l2CacheSize"] = prop.l2CacheSize;
        d["clockRate_kHz"] = prop.clockRate;
        d["memoryClockRate_kHz"] = prop.memoryClockRate;
        d["memoryBusWidth"] = prop.memoryBusWidth;
        return d;
    });

    m.def("forward_num_blocks", &sart::forward_num_blocks);
    m.def("forward", [](int epi, uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t x,
                        uintptr_t ghat, uintptr_t arow, uintptr_t out_f, uintptr_t out_w, uintptr_t Fpart,
                        uintptr_t st, uintptr_t stream) {
        sart::launch_forward(epi, P<const float>(A), ld, nrows, nrows_pad, P<const float>(x), P<const float>(ghat),
                             P<const float>(arow), P<float>(out_f), P<float>(out_w), P<double>(Fpart),
                             P<const sart::SartState>(st), S(stream));
    });
    m.def("rowsum_f64", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t out, uintptr_t stream) {
        sart::launch_rowsum_f64(P<const float>(A), ld, nrows, P<double>(out), S(stream));
    });
    m.def("backproject_num_splits", &sart::backproject_num_splits);
    m.def("backproject", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t w, int nsplit, uintptr_t partial,
                            uintptr_t st, uintptr_t stream) {
        sart::launch_backproject(P<const float>(A), ld, nrows, P<const float>(w), nsplit, P<float>(partial),
                                 P<const sart::SartState>(st), S(stream));
    });
    m.def("colsum_f64", [](uintptr_t A, int64_t ld, int64_t nrows, int nsplit, uintptr_t partial, uintptr_t stream) {
        sart::launch_colsum_f64(P<const float>(A), ld, nrows, nsplit, P<double>(partial), S(stream));
    });
    m.def("reduce_partials", [](uintptr_t partial, int64_t ld, int nsplit, uintptr_t scale, uintptr_t out,
                                uintptr_t Fpart, int64_t nF, uintptr_t Fout, uintptr_t st, uintptr_t stream) {
        sart::launch_reduce_partials(P<const float>(partial), ld, nsplit, P<const float>(scale), P<float>(out),
                                     P<const double>(Fpart), nF, P<float>(Fout), P<const sart::SartState>(st),
                                     S(stream));
    });
    m.def("reduce_partials_f64", [](uintptr_t partial, int64_t ld, int nsplit, uintptr_t out, uintptr_t stream) {
        sart::launch_reduce_partials_f64(P<const double>(partial), ld, nsplit, P<double>(out), S(stream));
    });
    m.def("prep_rows", [](uintptr_t g, int64_t nrows, int64_t nrows_pad, double inv_s, uintptr_t ray_length,
                          float len_thres, uintptr_t ghat, uintptr_t arow, uintptr_t gpos, uintptr_t wo,
                          uintptr_t stream) {
        sart::launch_prep_rows(P<const double>(g), nrows, nrows_pad, inv_s, P<const float>(ray_length), len_thres,
                               P<float>(ghat), P<float>(arow), P<float>(gpos), P<float>(wo), S(stream));
    });
    m.def("init_solution", [](uintptr_t x, int64_t n, int64_t n_pad, uintptr_t src_f32, uintptr_t src_f64,
                              double scale, uintptr_t stream) {
        sart::launch_init_solution(P<float>(x), n, n_pad, P<const float>(src_f32), P<const double>(src_f64), scale,
                                   S(stream));
    });
    m.def("penalty", [](bool logx, uintptr_t row_ptr, uintptr_t col, uintptr_t val, int64_t n, float beta,
                        uintptr_t x, uintptr_t pen, uintptr_t st, uintptr_t stream) {
        sart::launch_penalty(logx, P<const int64_t>(row_ptr), P<const int32_t>(col), P<const float>(val), n, beta,
                             P<const float>(x), P<float>(pen), P<const sart::SartState>(st), S(stream));
    });
    m.def("decide", [](uintptr_t st, uintptr_t Fslot, uintptr_t stream) {
        sart::launch_decide(P<sart::SartState>(st), P<const float>(Fslot), S(stream));
    });
    m.def("update_linear", [](uintptr_t x, uintptr_t d, uintptr_t pen, int64_t n, uintptr_t st, uintptr_t stream) {
        sart::launch_update_linear(P<float>(x), P<const float>(d), P<const float>(pen), n,
                                   P<const sart::SartState>(st), S(stream));
    });
    m.def("update_log", [](uintptr_t x, uintptr_t O, uintptr_t Fv, uintptr_t pen, float alpha, int64_t n,
                           uintptr_t st, uintptr_t stream) {
        sart::launch_update_log(P<float>(x), P<const float>(O), P<const float>(Fv), P<const float>(pen), alpha, n,
                                P<const sart::SartState>(st), S(stream));
    });
    m.def("state_begin", [](uintptr_t st, double G, double tol, int max_iter, uintptr_t stream) {
        sart::launch_state_begin(P<sart::SartState>(st), G, tol, max_iter, S(stream));
    });
    m.def("synth_matrix", [](uintptr_t A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols,
                             int64_t row_offset, uint64_t seed, float lo, float hi, uintptr_t stream) {
        sart::launch_synth_matrix(P<float>(A), ld, nrows_pad, nrows, ncols, row_offset, seed, lo, hi, S(stream));
    });
    m.def("synth_vector", [](uintptr_t out, int64_t n, int64_t offset, uint64_t seed, double lo, double hi,
                             uintptr_t stream) {
        sart::launch_synth_vector(P<double>(out), n, offset, seed, lo, hi, S(stream));
    });
    m.def("fused_pick_k", &sart::fused_pick_k);
    m.def("fused_tile_rows", &sart::fused_tile_rows);
    m.def("fused_set_schedule", &sart::fused_set_schedule);
    m.def("fused_get_schedule", &sart::fused_get_schedule);
    m.def("fused_debug_map", &sart::fused_debug_map);
    m.def("fused_set_trace", [](uintptr_t buf, long long tiles) {
        sart::fused_set_trace(reinterpret_cast<unsigned long long*>(buf), tiles);
    });
    m.def("fused_fpart_per_block", &sart::fused_fpart_per_block);
    m.def("fused_set_debug", &sart::fused_set_debug);
    m.def("fused_debug_stats", &sart::fused_debug_stats);
    m.def("fused_sweep", [](bool logmode, int K, int variant, uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                            uintptr_t x, uintptr_t ghat, uintptr_t arow, uintptr_t partial, uintptr_t Fpart,
                            uintptr_t gran, int I, int J, uintptr_t st, uintptr_t xcnt, uintptr_t stream) {
        sart::launch_fused_sweep(logmode, K, variant, P<const float>(A), ld, nrows, nrows_pad, P<const float>(x),
                                 P<const float>(ghat), P<const float>(arow), P<float>(partial), P<double>(Fpart),
                                 P<uint64_t>(gran), I, J, P<sart::SartState>(st), P<unsigned>(xcnt), S(stream));
    });
    m.def("mf_forward_num_splits", &sart::mf_forward_num_splits);
    m.def("mf_backproject_num_splits", &sart::mf_backproject_num_splits);
    m.def("mf_forward", [](uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t X, int64_t ldx,
                           uintptr_t Fout, int nsplit, uintptr_t stream) {
        sart::launch_mf_forward(P<const float>(A), ld, nrows, nrows_pad, P<const float>(X), ldx, P<float>(Fout),
                                nsplit, S(stream));
    });
    m.def("mf_backproject", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t W, int nsplit, uintptr_t partial,
                               uintptr_t stream) {
        sart::launch_mf_backproject(P<const float>(A), ld, nrows, P<const float>(W), nsplit, P<float>(partial),
                                    S(stream));
    });
}
