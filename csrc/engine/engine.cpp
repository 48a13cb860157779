#include "engine.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>

#include <unistd.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../kernels/launchers.hpp"

namespace sart {

namespace {

constexpr int kEpiPlain = 0, kEpiLinear = 1, kEpiLog = 2;

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Rank of this process among the ranks that asked for fault injection (SART_FAULT_RANK: only that rank
// injects; unset: every rank).
bool fault_rank_selected(int rank) {
    const char* e = std::getenv("SART_FAULT_RANK");
    return !(e && *e) || std::atoi(e) == rank;
}

}  // namespace

int ranks_sharing_device(Communicator* comm, int device) { return ranks_sharing_device(comm->host(), device); }

bool device_shared_across_ranks(Communicator* comm, int device) { return ranks_sharing_device(comm, device) > 1; }

double fused_min_bytes_from_env() {
    const char* e = std::getenv("SART_FUSED_MIN_MB");
    return ((e && *e) ? std::atof(e) : 128.0) * 1024.0 * 1024.0;
}

RoctxRange::RoctxRange(const char* name) { roctxRangePushA(name); }
RoctxRange::~RoctxRange() { roctxRangePop(); }

template <typename T>
void DeviceArray<T>::resize(size_t n) {
    release();
    if (n == 0) return;
    hip_ok(hipMalloc(reinterpret_cast<void**>(&p_), n * sizeof(T)), "hipMalloc");
    hip_ok(hipMemset(p_, 0, n * sizeof(T)), "hipMemset");
    // hipMemset is ordered on the null stream only; the engine's stream is non-blocking, so wait here or
    // the zero fill may land after the first kernel that writes the buffer
    hip_ok(hipDeviceSynchronize(), "hipMemset sync");
    n_ = n;
}

template <typename T>
void DeviceArray<T>::release() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
}

template class DeviceArray<float>;
template class DeviceArray<double>;
template class DeviceArray<SartState>;
template class DeviceArray<MfState>;
template class DeviceArray<MfQueue>;
template class DeviceArray<uint64_t>;
template class DeviceArray<unsigned>;
template class DeviceArray<int64_t>;
template class DeviceArray<int32_t>;
template class DeviceArray<bf16_t>;

Engine::Engine(int device, const void* A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel, int64_t ld,
               Communicator* comm, const EngineConfig& cfg, const SparseRtm* sparse)
    : device_(device), A_(A), P_(nrows), Pp_(nrows_pad), V_(nvoxel), ld_(ld), comm_(comm), cfg_(cfg) {
    validate_params(cfg_);
    if (!comm_) throw std::invalid_argument("Engine: communicator required");
    if (sparse) {
        if (cfg_.column_shard || cfg_.rtm_bf16)
            throw std::invalid_argument("Engine: a sparse shard is a row shard of fp32 values");
        if (!sparse->row_ptr || !sparse->col_ptr)
            throw std::invalid_argument("Engine: sparse shard needs its CSR and CSC arrays");
        sparse_ = true;
        sp_ = *sparse;
        // lanes per row / column from the mean entries per row / column, fixed for the engine's life
        if (!sp_.lanes_rows) sp_.lanes_rows = sparse_lanes(nrows_pad ? (double)sp_.nnz / (double)nrows_pad : 0.0);
        if (!sp_.lanes_cols) sp_.lanes_cols = sparse_lanes(nvoxel ? (double)sp_.nnz / (double)nvoxel : 0.0);
    } else if (!A_) {
        throw std::invalid_argument("Engine: dense shard pointer required");
    }
    if (ld_ % 64 || ld_ < V_ || Pp_ % 64 || Pp_ < P_)
        throw std::invalid_argument("Engine: ld and nrows_pad must be multiples of 64 covering the shard");
    cfg_.check_interval = std::max(1, cfg_.check_interval);
    if (cfg_.column_shard) {
        if (cfg_.nvoxel_total <= 0) cfg_.nvoxel_total = V_;
        if (cfg_.col_offset < 0 || cfg_.col_offset + V_ > cfg_.nvoxel_total)
            throw std::invalid_argument("Engine: column shard outside [0, nvoxel_total)");
    }
    set_device();
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");  // the shard may have been filled on another stream
    hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    for (auto& e : ev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hstate_), 2 * sizeof(SartState)), "hipHostMalloc");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hg_), std::max<int64_t>(P_, 1) * sizeof(double)), "hipHostMalloc");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hx0_), std::max<int64_t>(V_, 1) * sizeof(double)), "hipHostMalloc");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hxo_), std::max<int64_t>(V_, 1) * sizeof(float)), "hipHostMalloc");
    hipDeviceProp_t prop;
    hip_ok(hipGetDeviceProperties(&prop, device_), "hipGetDeviceProperties");
    num_cus_ = prop.multiProcessorCount;
    if (cfg_.fused_schedule >= 0) fused_set_schedule(cfg_.fused_schedule);
    if (const char* fi = std::getenv("SART_FAULT_INJECT"); fi && *fi && cfg_.fault_inject == 0)
        cfg_.fault_inject = std::atoi(fi);
    if (const char* fn = std::getenv("SART_FAULT_NAN"); fn && *fn && cfg_.fault_nan_sweep < 0)
        cfg_.fault_nan_sweep = std::atoi(fn);
    if (const char* t = std::getenv("SART_TAIL_FUSED"); t && *t) tail_fused_ = std::atoi(t) != 0;

    // the sparse back-projection writes complete column sums: one partial row
    nsplit_ = sparse_ ? 1 : backproject_num_splits(ld_, Pp_, cfg_.rtm_bf16 ? 2 : 4);
    comm_buf_.resize(ld_ + 64);  // [0, ld) correction, [ld] ||A x||^2
    x_.resize(ld_);
    pen_.resize(ld_);
    if (cfg_.logarithmic) O_.resize(ld_);
    for (auto* b : {&ghat_, &arow_, &gpos_, &wo_, &w_, &fitted_}) b->resize(Pp_);
    g64_.resize(Pp_);
    x064_.resize(std::max<int64_t>(V_, 1));
    st_.resize(1);
    xcnt_.resize(16);
    ticket_.resize(1);
    xprev_.resize(ld_);
    use_fused_ = false;
    // The fused sweep is a persistent grid whose workgroups must all be co-resident. Ranks sharing one GPU
    // (one-GPU rehearsals of an N-rank run) therefore plan their grids on disjoint shares of the CUs: with
    // SART_FUSED_SHARED=1 each rank's geometry targets num_cus / (ranks per GPU) CUs (8 XCDs x CUs per XCD,
    // every workgroup one CU by its LDS), so the grids of all ranks fit side by side; without it ranks that share
    // a GPU use the two-pass kernels. EngineConfig::fused_max_cus / SART_FUSED_CUS caps the plan explicitly.
    // Decided from device identity, identically on every rank of the group.
    ranks_per_device_ = cfg_.column_shard ? 1 : ranks_sharing_device(comm_, device_);
    shared_device_ = ranks_per_device_ > 1;
    const char* fs = std::getenv("SART_FUSED_SHARED");
    const bool fused_ok_shared = fs && std::string(fs) == "1";
    if (shared_device_ && cfg_.use_fused && !fused_ok_shared && comm_->rank() == 0)
        std::fprintf(stderr, "sart: %d ranks share GPUs; using the two-pass kernels (SART_FUSED_SHARED=1 splits the "
                             "CUs between their fused sweeps)\n", comm_->size());
    plan_cus_ = num_cus_;
    if (shared_device_) plan_cus_ = num_cus_ / ranks_per_device_;
    if (const char* c = std::getenv("SART_FUSED_CUS"); c && *c && cfg_.fused_max_cus <= 0) cfg_.fused_max_cus = std::atoi(c);
    if (cfg_.fused_max_cus > 0) plan_cus_ = std::min(plan_cus_, cfg_.fused_max_cus);
    plan_cus_ = plan_cus_ / 8 * 8;  // whole CUs per XCD
    // bf16 storage: the fused sweep exists as variant 6 only (else the two-pass kernels)
    const double abytes = (double)Pp_ * (double)ld_ * (cfg_.rtm_bf16 ? 2.0 : 4.0);
    if (cfg_.use_fused && !sparse_ && !cfg_.column_shard && abytes >= cfg_.fused_min_bytes && plan_cus_ >= 8 &&
        (!shared_device_ || fused_ok_shared) && (!cfg_.rtm_bf16 || cfg_.fused_variant == 6)) {
        geom_ = fused_geometry(ld_, plan_cus_, cfg_.fused_variant, cfg_.rows_per_tile, !cfg_.rtm_bf16, !cfg_.rtm_bf16);
        if (cfg_.rtm_bf16 && (cfg_.rows_per_tile == 0 || cfg_.rows_per_tile == 4)) {
            // wide bf16 tiles (8 KB per wave per step, like fp32) where the width allows; SART_BF16_WIDE=0 keeps
            // the narrow tiles
            const char* w = std::getenv("SART_BF16_WIDE");
            const FusedGeometry gw = fused_geometry_bf16_wide(ld_, plan_cus_);
            if (gw.valid() && !(w && std::string(w) == "0")) geom_ = gw;
        }
        use_fused_ = geom_.valid() && (!cfg_.rtm_bf16 || geom_.variant == 6);
    }
    // Every rank runs the fused sweep or none does: shards of different heights can land on both sides of
    // fused_min_bytes, and a rank on the two-pass kernels would then see its peers' protocol errors (the error
    // word rides in the all-reduce) without a fused sweep of its own to fall back from.
    if (comm_->size() > 1 && !cfg_.column_shard) {
        const double off = comm_->host().all_reduce_scalar(use_fused_ ? 0.0 : 1.0, ReduceOp::kMax);
        if (off > 0.0 && use_fused_) {
            use_fused_ = false;
            geom_ = FusedGeometry{};
        }
    }
    alloc_fused();
    ray_sums();
    // the fp32 collectives of a solve: row shards reduce the voxel correction (+ ||A x||^2 and the error word) per
    // sweep and ld-long vectors per frame; column shards the pixel vector A x (and x when there is a Laplacian)
    if (comm_->size() > 1) {
        if (cfg_.column_shard)
            comm_->prepare({P_, cfg_.nvoxel_total});
        else
            comm_->prepare({ld_ + 2, ld_});
    }
}

Engine::~Engine() {
    set_device();
    drop_graph();
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& pool : cev_)
        for (auto& e : pool) (void)hipEventDestroy(e);
    if (hstate_) (void)hipHostFree(hstate_);
    for (void* p : {static_cast<void*>(hg_), static_cast<void*>(hx0_), static_cast<void*>(hxo_)})
        if (p) (void)hipHostFree(p);
    if (stream_) (void)hipStreamDestroy(stream_);
}

void Engine::set_device() const { hip_ok(hipSetDevice(device_), "hipSetDevice"); }

void Engine::drop_graph() {
    if (graph_) (void)hipGraphExecDestroy(graph_);
    graph_ = nullptr;
    warm_ = false;
}

void Engine::alloc_fused() {
    nF_fused_ = use_fused_ ? (int64_t)geom_.grid * fused_fpart_per_block(geom_.variant) : 0;
    const ChainPlan plan = use_fused_ ? fused_chain_plan(geom_, Pp_, fused_split_schedule(geom_.K, cfg_.rtm_bf16))
                                      : ChainPlan{};
    chain_tiles_ = plan.chain_tiles;
    fused_blocks_ = use_fused_ ? plan.blocks : 0;
    const int64_t n_part = std::max<int64_t>(nsplit_, use_fused_ ? fused_blocks_ : 1);
    if ((int64_t)partial_.size() < n_part * ld_) partial_.resize(n_part * ld_);
    const int64_t nF = std::max<int64_t>({forward_num_blocks(Pp_), (int64_t)weights_num_blocks(Pp_), nF_fused_, 1});
    if ((int64_t)Fpart_.size() < nF) Fpart_.resize(nF);
    if (use_fused_) {
        const int64_t ng = std::max<int64_t>(Pp_ * geom_.J, fused_granules(Pp_, geom_.J, geom_.xl));
        if ((int64_t)gran_.size() < ng) gran_.resize(ng);
    }
}

void DeviceRaySums::compute(const void* A, int64_t P, int64_t Pp, int64_t V, int64_t ld, Communicator* comm,
                            const SolverParams& p, hipStream_t stream, bool col_shard, bool a_bf16) {
    // rho_v = sum_p A[p, v] (fp64, all-reduced), l_p = sum_v A[p, v] (fp64, local): on the device instead of
    // the reference's host loops (sartsolver.cpp:38-56); scales with the reference's fp32 semantics
    RoctxRange r("sart::ray_sums");
    ell64.resize(Pp);
    rho64.resize(ld);
    ray_len.resize(Pp);
    for (auto* b : {&dinv, &dscale, &dmask}) b->resize(ld);
    const int nsplit = backproject_num_splits(ld, Pp, a_bf16 ? 2 : 4);
    {
        DeviceArray<double> part((size_t)nsplit * ld);
        if (a_bf16) {
            launch_rowsum_f64(static_cast<const bf16_t*>(A), ld, P, ell64.get(), stream);
            launch_colsum_f64(static_cast<const bf16_t*>(A), ld, P, nsplit, part.get(), stream);
        } else {
            launch_rowsum_f64(static_cast<const float*>(A), ld, P, ell64.get(), stream);
            launch_colsum_f64(static_cast<const float*>(A), ld, P, nsplit, part.get(), stream);
        }
        launch_reduce_partials_f64(part.get(), ld, nsplit, rho64.get(), stream);
        hip_ok(hipStreamSynchronize(stream), "ray sums");
    }
    if (col_shard)
        comm->all_reduce(ell64.get(), (size_t)P, ReduceOp::kSum, stream);
    else
        comm->all_reduce(rho64.get(), (size_t)ld, ReduceOp::kSum, stream);
    launch_f64_to_f32(ell64.get(), ray_len.get(), Pp, stream);
    launch_density_scales(rho64.get(), V, ld, (float)p.ray_density_threshold, (float)p.relaxation, dinv.get(),
                          dscale.get(), dmask.get(), stream);
    hip_ok(hipStreamSynchronize(stream), "ray sums");
}

std::vector<double> DeviceRaySums::density(int64_t V) const {
    std::vector<double> h(V);
    if (V) hip_ok(hipMemcpy(h.data(), rho64.get(), V * sizeof(double), hipMemcpyDeviceToHost), "D2H");
    return h;
}

std::vector<double> DeviceRaySums::length(int64_t P) const {
    std::vector<double> h(P);
    if (P) hip_ok(hipMemcpy(h.data(), ell64.get(), P * sizeof(double), hipMemcpyDeviceToHost), "D2H");
    return h;
}

void DeviceRaySums::compute_sparse(const SparseRtm& s, int64_t P, int64_t Pp, int64_t V, int64_t ld,
                                   Communicator* comm, const SolverParams& p, hipStream_t stream) {
    RoctxRange r("sart::ray_sums");
    ell64.resize(Pp);  // zero-filled: padded rows / columns stay 0
    rho64.resize(ld);
    ray_len.resize(Pp);
    for (auto* b : {&dinv, &dscale, &dmask}) b->resize(ld);
    launch_csr_rowsum_f64(s, P, ell64.get(), stream);
    launch_csc_colsum_f64(s, V, rho64.get(), stream);
    comm->all_reduce(rho64.get(), (size_t)ld, ReduceOp::kSum, stream);
    launch_f64_to_f32(ell64.get(), ray_len.get(), Pp, stream);
    launch_density_scales(rho64.get(), V, ld, (float)p.ray_density_threshold, (float)p.relaxation, dinv.get(),
                          dscale.get(), dmask.get(), stream);
    hip_ok(hipStreamSynchronize(stream), "ray sums");
}

void Engine::ray_sums() {
    if (sparse_)
        rs_.compute_sparse(sp_, P_, Pp_, V_, ld_, comm_, cfg_, stream_);
    else
        rs_.compute(A_, P_, Pp_, V_, ld_, comm_, cfg_, stream_, cfg_.column_shard, cfg_.rtm_bf16);
}

void Engine::fwd(int epi, const float* x, float* out_f, float* out_w, double* Fpart, const SartState* st) {
    const float* ghat = epi == kEpiPlain ? nullptr : ghat_.get();
    const float* arow = epi == kEpiPlain ? nullptr : arow_.get();
    if (sparse_)
        launch_csr_forward(epi, sp_, P_, Pp_, x, ghat, arow, out_f, out_w, Fpart, st, stream_);
    else if (cfg_.rtm_bf16)
        launch_forward(epi, static_cast<const bf16_t*>(A_), ld_, P_, Pp_, x, ghat, arow, out_f, out_w, Fpart, st,
                       stream_);
    else
        launch_forward(epi, static_cast<const float*>(A_), ld_, P_, Pp_, x, ghat, arow, out_f, out_w, Fpart, st,
                       stream_);
}

void Engine::bwd(const float* w, const SartState* st) {
    if (sparse_)
        launch_csc_backproject(sp_, V_, w, partial_.get(), st, stream_);  // nsplit_ == 1
    else if (cfg_.rtm_bf16)
        launch_backproject(static_cast<const bf16_t*>(A_), ld_, P_, w, nsplit_, partial_.get(), st, stream_);
    else
        launch_backproject(static_cast<const float*>(A_), ld_, P_, w, nsplit_, partial_.get(), st, stream_);
}

std::vector<double> Engine::ray_density() const {
    set_device();
    return rs_.density(V_);
}

std::vector<double> Engine::ray_length() const {
    set_device();
    return rs_.length(P_);
}

void Engine::set_laplacian(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t nnz) {
    set_device();
    drop_graph();
    has_lap_ = false;
    if (nnz <= 0 || cfg_.beta_laplace <= 0) return;
    if (cfg_.column_shard) {
        // full L (nvoxel_total rows, global column indices): keep this shard's rows, gather x for the columns
        const int64_t n = cfg_.nvoxel_total, r0 = cfg_.col_offset;
        if (row_ptr[n] != nnz) throw std::invalid_argument("Laplacian CSR row pointer does not match nnz");
        const int64_t k0 = row_ptr[r0], k1 = row_ptr[r0 + V_];
        std::vector<int64_t> rp(V_ + 1);
        for (int64_t i = 0; i <= V_; ++i) rp[i] = row_ptr[r0 + i] - k0;
        lap_rp_.resize(V_ + 1);
        hip_ok(hipMemcpy(lap_rp_.get(), rp.data(), (V_ + 1) * sizeof(int64_t), hipMemcpyHostToDevice), "H2D");
        if (k1 > k0) {
            lap_col_.resize(k1 - k0);
            lap_val_.resize(k1 - k0);
            hip_ok(hipMemcpy(lap_col_.get(), col + k0, (k1 - k0) * sizeof(int32_t), hipMemcpyHostToDevice), "H2D");
            hip_ok(hipMemcpy(lap_val_.get(), val + k0, (k1 - k0) * sizeof(float), hipMemcpyHostToDevice), "H2D");
        }
        xg_.resize((size_t)(n + 63) / 64 * 64);
        has_lap_ = true;
        return;
    }
    if (row_ptr[V_] != nnz) throw std::invalid_argument("Laplacian CSR row pointer does not match nnz");
    lap_rp_.resize(V_ + 1);
    lap_col_.resize(nnz);
    lap_val_.resize(nnz);
    hip_ok(hipMemcpy(lap_rp_.get(), row_ptr, (V_ + 1) * sizeof(int64_t), hipMemcpyHostToDevice), "H2D");
    hip_ok(hipMemcpy(lap_col_.get(), col, nnz * sizeof(int32_t), hipMemcpyHostToDevice), "H2D");
    hip_ok(hipMemcpy(lap_val_.get(), val, nnz * sizeof(float), hipMemcpyHostToDevice), "H2D");
    has_lap_ = true;
}

double Engine::setup_frame(const double* g, const double* x0, bool x0_on_device) {
    RoctxRange r("sart::setup_frame");
    // normalisation by the global maximum and sum_{g > 0} g^2 (reference sartsolver_cuda.cpp:146-157);
    // the reference divides by zero when every pixel is <= 0, we keep norm = 1 then.
    // the previous frame's copies out of the pinned buffers have completed (solve() synchronises the stream)
    // eight interleaved max / sum chains combined pairwise (fixed order): one serial chain is bound by the
    // add latency (65536 pixels: 67 us; eight: 23 us with the copy into pinned memory in the same pass)
    double mx8[8], gs8[8];
    for (int k = 0; k < 8; ++k) mx8[k] = -std::numeric_limits<double>::infinity(), gs8[k] = 0.0;
    // a non-finite pixel is masked like a saturated one (k_prep_rows)
    auto acc = [](double v, double& m, double& q) {
        const bool ok = std::isfinite(v);
        m = ok && v > m ? v : m;
        q += (ok && v > 0) ? v * v : 0.0;
    };
    int64_t i0 = 0;
    for (; i0 + 8 <= P_; i0 += 8)
#pragma GCC unroll 8
        for (int k = 0; k < 8; ++k) {
            const double v = g[i0 + k];
            hg_[i0 + k] = v;  // into pinned memory in the same pass
            acc(v, mx8[k], gs8[k]);
        }
    for (; i0 < P_; ++i0) {
        hg_[i0] = g[i0];
        acc(g[i0], mx8[i0 & 7], gs8[i0 & 7]);
    }
    const double mx = std::max(std::max(std::max(mx8[0], mx8[1]), std::max(mx8[2], mx8[3])),
                               std::max(std::max(mx8[4], mx8[5]), std::max(mx8[6], mx8[7])));
    const double gs = ((gs8[0] + gs8[1]) + (gs8[2] + gs8[3])) + ((gs8[4] + gs8[5]) + (gs8[6] + gs8[7]));
    const bool cols = cfg_.column_shard;  // every rank holds every pixel: the sums are already global
    double norm = cols ? mx : comm_->host().all_reduce_scalar(mx, ReduceOp::kMax);
    if (!(norm > 0)) norm = 1.0;
    double G = (cols ? gs : comm_->host().all_reduce_scalar(gs, ReduceOp::kSum)) / (norm * norm);
    if (!(G > 0)) G = 1.0;
    if (P_) hip_ok(hipMemcpyAsync(g64_.get(), hg_, P_ * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D g");
    launch_prep_rows(g64_.get(), P_, Pp_, 1.0 / norm, rs_.ray_len.get(), (float)cfg_.ray_length_threshold, ghat_.get(),
                     arow_.get(), gpos_.get(), wo_.get(), stream_);
    if (!x0) {
        // cold start x0 = [rho > tau] A^T max(ghat, 0) / rho (reference sart_kernels.cu:22-60)
        bwd(gpos_.get(), nullptr);
        launch_reduce_partials(partial_.get(), ld_, nsplit_, rs_.dinv.get(), comm_buf_.get(), nullptr, 0, nullptr,
                               nullptr, stream_);
        if (!cols) comm_->all_reduce(comm_buf_.get(), (size_t)ld_, ReduceOp::kSum, stream_);
        launch_init_solution(x_.get(), V_, ld_, comm_buf_.get(), nullptr, 1.0, stream_);
    } else if (x0_on_device) {
        launch_rescale_solution(x_.get(), V_, ld_, last_norm_, 1.0 / norm, stream_);
    } else {
        std::memcpy(hx0_, x0, V_ * sizeof(double));
        hip_ok(hipMemcpyAsync(x064_.get(), hx0_, V_ * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D x0");
        launch_init_solution(x_.get(), V_, ld_, nullptr, x064_.get(), 1.0 / norm, stream_);
    }
    if (cfg_.logarithmic) {
        // frame-constant observed back-projection O = [rho > tau] A^T (a ghat), reduced once per frame
        bwd(wo_.get(), nullptr);
        launch_reduce_partials(partial_.get(), ld_, nsplit_, rs_.dmask.get(), O_.get(), nullptr, 0, nullptr, nullptr,
                               stream_);
        if (!cols) comm_->all_reduce(O_.get(), (size_t)ld_, ReduceOp::kSum, stream_);
    }
    launch_state_begin(st_.get(), G, cfg_.conv_tolerance, cfg_.max_iterations, stream_);
    // per-XCD tickets of the first fused sweep (variant 6); later sweeps get them zeroed by the update kernel
    if (use_fused_ && geom_.variant == 6) hip_ok(hipMemsetAsync(xcnt_.get(), 0, 16 * sizeof(unsigned), stream_), "memset");
    return norm;
}

void Engine::sweep() {
    SartState* st = st_.get();
    const float* scale = cfg_.logarithmic ? rs_.dmask.get() : rs_.dscale.get();
    float* Fslot = comm_buf_.get() + ld_;
    if (cfg_.column_shard) {
        sweep_columns();
        return;
    }
    unsigned* xcnt = (use_fused_ && geom_.variant == 6) ? xcnt_.get() : nullptr;  // zeroed by setup / update
    const int nsplit = use_fused_ ? (int)fused_blocks_ : nsplit_;
    const int64_t nF = use_fused_ ? nF_fused_ : (sparse_ ? csr_forward_num_blocks(sp_, Pp_) : forward_num_blocks(Pp_));
    // One rank: the reduction of the partial rows, the decision and the update are one kernel (nothing to
    // all-reduce in between); every workgroup sums the nF sweep partials, so only while nF stays small.
    const bool one_tail = tail_fused_ && comm_->size() == 1 && nF <= 4096;
    if (use_fused_) {
        if (cfg_.rtm_bf16)  // variant 6, K = rows per tile
            launch_fused_sweep_bf16(cfg_.logarithmic, geom_.K, static_cast<const bf16_t*>(A_), ld_, P_, Pp_, x_.get(),
                                    ghat_.get(), arow_.get(), partial_.get(), Fpart_.get(), gran_.get(), geom_.I,
                                    geom_.J, st, xcnt_.get(), stream_, geom_.cpl, chain_tiles_, geom_.kw, geom_.xl);
        else
            launch_fused_sweep(cfg_.logarithmic, geom_.K, geom_.variant, static_cast<const float*>(A_), ld_, P_, Pp_,
                               x_.get(), ghat_.get(), arow_.get(), partial_.get(), Fpart_.get(), gran_.get(), geom_.I,
                               geom_.J, st, xcnt_.get(), stream_, chain_tiles_, geom_.kw, geom_.xl);
    } else {
        fwd(cfg_.logarithmic ? kEpiLog : kEpiLinear, x_.get(), nullptr, w_.get(), Fpart_.get(), st);
        bwd(w_.get(), st);
    }
    const float* pen = nullptr;
    if (has_lap_) {
        launch_penalty(cfg_.logarithmic, lap_rp_.get(), lap_col_.get(), lap_val_.get(), V_, (float)cfg_.beta_laplace,
                       x_.get(), pen_.get(), st, stream_);
        pen = pen_.get();
    }
    bool updated = false;
    if (comm_->size() > 1) {  // [0, ld) corrections, [ld] ||A x||^2, [ld + 1] error word: one collective
        comm_begin();          // (p2p: formed from the partial rows, pushed, and the update applied by one kernel)
        UpdateArgs u;
        u.st = st;
        u.x = x_.get();
        u.O = O_.get();
        u.pen = pen;
        u.alpha = (float)cfg_.relaxation;
        u.n = V_;
        u.xcnt = xcnt;
        u.xprev = xprev_.get();
        u.ticket = ticket_.get();
        u.logmode = cfg_.logarithmic;
        updated = comm_->reduce_all_reduce_update(ReduceSrc{partial_.get(), ld_, nsplit, scale, Fpart_.get(), nF, st},
                                                  comm_buf_.get(), u, stream_);
        comm_end();
    } else if (!one_tail) {
        launch_reduce_partials(partial_.get(), ld_, nsplit, scale, comm_buf_.get(), Fpart_.get(), nF, Fslot, st,
                               stream_);
    }
    if (updated) {
    } else if (one_tail)
        launch_reduce_decide_update(cfg_.logarithmic, st, partial_.get(), ld_, nsplit, scale, Fpart_.get(), nF,
                                    x_.get(), O_.get(), pen, (float)cfg_.relaxation, V_, xcnt, xprev_.get(),
                                    ticket_.get(), stream_);
    else
        launch_decide_update(cfg_.logarithmic, st, Fslot, x_.get(), comm_buf_.get(), O_.get(), pen,
                             (float)cfg_.relaxation, V_, xcnt, xprev_.get(), ticket_.get(), stream_);
    if (cfg_.fault_nan_sweep >= 0 && host_sweep_ == cfg_.fault_nan_sweep)  // fault injection (tests)
        hip_ok(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(x_.get()), 0x7fc00000, 1, stream_), "inject NaN");
    ++host_sweep_;
}

void Engine::sweep_columns() {
    // f_r = A_r x_r -> all-reduce (pixel vector) -> weights and ||f||^2 (identical on every rank) ->
    // local back-projection, penalty (x all-gathered when there is a Laplacian), decision and update.
    SartState* st = st_.get();
    const float* scale = cfg_.logarithmic ? rs_.dmask.get() : rs_.dscale.get();
    float* Fslot = comm_buf_.get() + ld_;
    fwd(kEpiPlain, x_.get(), fitted_.get(), nullptr, nullptr, st);
    if (comm_->size() > 1) {
        comm_begin();
        comm_->all_reduce(fitted_.get(), (size_t)P_, ReduceOp::kSum, stream_);
        comm_end();
    }
    launch_weights(cfg_.logarithmic, fitted_.get(), ghat_.get(), arow_.get(), P_, Pp_, w_.get(), Fpart_.get(), st,
                   stream_);
    bwd(w_.get(), st);
    launch_reduce_partials(partial_.get(), ld_, nsplit_, scale, comm_buf_.get(), Fpart_.get(),
                           weights_num_blocks(Pp_), Fslot, st, stream_);
    const float* pen = nullptr;
    if (has_lap_) {
        const float* xfull = x_.get();
        if (comm_->size() > 1) {
            hip_ok(hipMemsetAsync(xg_.get(), 0, xg_.size() * sizeof(float), stream_), "memset");
            launch_copy_slice(x_.get(), V_, xg_.get(), cfg_.col_offset, stream_);
            comm_begin();
            comm_->all_reduce(xg_.get(), (size_t)cfg_.nvoxel_total, ReduceOp::kSum, stream_);
            comm_end();
            xfull = xg_.get();
        }
        launch_penalty(cfg_.logarithmic, lap_rp_.get(), lap_col_.get(), lap_val_.get(), V_, (float)cfg_.beta_laplace,
                       xfull, pen_.get(), st, stream_);
        pen = pen_.get();
    }
    launch_decide_update(cfg_.logarithmic, st, Fslot, x_.get(), comm_buf_.get(), O_.get(), pen, (float)cfg_.relaxation,
                         V_, nullptr, xprev_.get(), ticket_.get(), stream_);
}

bool Engine::timing_collectives() const { return cfg_.time_collectives && !cfg_.use_graph && comm_->size() > 1; }

void Engine::comm_begin() {
    if (!timing_collectives()) return;
    auto& pool = cev_[cur_slot_];
    const size_t k = (size_t)cev_used_[cur_slot_] * 2;
    while (pool.size() < k + 2) {
        hipEvent_t e;
        hip_ok(hipEventCreate(&e), "hipEventCreate");
        pool.push_back(e);
    }
    hip_ok(hipEventRecord(pool[k], stream_), "hipEventRecord");
}

void Engine::comm_end() {
    if (!timing_collectives()) return;
    const size_t k = (size_t)cev_used_[cur_slot_] * 2;
    hip_ok(hipEventRecord(cev_[cur_slot_][k + 1], stream_), "hipEventRecord");
    ++cev_used_[cur_slot_];
}

void Engine::collect_comm(int slot) {  // the chunk of `slot` has completed
    for (int i = 0; i < cev_used_[slot]; ++i) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, cev_[slot][2 * i], cev_[slot][2 * i + 1]) == hipSuccess) comm_ms_ += ms;
    }
    cev_used_[slot] = 0;
}

void Engine::run_chunk(int n) {
    RoctxRange r("sart::chunk");
    // Capture only after an eager chunk with the current kernels: launchers configure function attributes
    // (dynamic LDS above 64 KiB) on first use, which must not happen inside a capture.
    const bool graphable = cfg_.use_graph && !graph_failed_ && warm_ && comm_->graph_capturable() &&
                           n == cfg_.check_interval;
    if (graphable && !graph_) {
        hipGraph_t g = nullptr;
        bool ok = hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) == hipSuccess;
        if (ok) {
            try {
                for (int i = 0; i < n; ++i) sweep();
            } catch (...) {
                ok = false;
            }
            ok = (hipStreamEndCapture(stream_, &g) == hipSuccess) && ok && g;
        }
        if (ok) ok = hipGraphInstantiate(&graph_, g, nullptr, nullptr, 0) == hipSuccess;
        if (g) (void)hipGraphDestroy(g);
        if (!ok) {
            (void)hipGetLastError();
            graph_ = nullptr;
            graph_failed_ = true;
        }
    }
    if (graphable && graph_) {
        hip_ok(hipGraphLaunch(graph_, stream_), "hipGraphLaunch");
    } else {
        for (int i = 0; i < n; ++i) sweep();
        warm_ = true;
    }
}

bool Engine::fallback() {
    RoctxRange r("sart::fallback");
    // A persistent sweep gave up waiting (SartState.error, set on every rank by the all-reduced error word):
    // XCD-local groups (variant 6) -> generic groups (variant 3) -> two-pass kernels. The frame is re-solved from
    // scratch. A rank whose own kernels are already the two-pass ones re-solves on them: its peers step down
    // their chains and re-solve too, so every rank enters the same number of collectives.
    drop_graph();
    if (use_fused_ && geom_.variant == 6 && !cfg_.rtm_bf16) {
        const FusedGeometry g3 = fused_geometry(ld_, plan_cus_, 3, 0);
        if (g3.valid()) {
            std::fprintf(stderr, "sart: fused sweep variant 6 timed out (unexpected workgroup placement); using variant 3\n");
            geom_ = g3;
            alloc_fused();
            return true;
        }
    }
    if (use_fused_) {
        std::fprintf(stderr, "sart: fused sweep protocol timeout; switching to the two-pass kernels\n");
        use_fused_ = false;
    }
    return true;
}

bool device_comm_failed_anywhere(Communicator* comm) {
    // The P2P all-reduce of one rank can time out while its peers complete the same call (they received every
    // flag), so whether a frame must be re-solved is agreed over the host communicator after every solve, while
    // a degradable device path is active (one host scalar per frame).
    if (comm->size() <= 1 || !comm->degradable()) return false;
    const bool mine = comm->device_failed();
    return comm->host().all_reduce_scalar(mine ? 1.0 : 0.0, ReduceOp::kMax) > 0.0;
}

bool Engine::comm_failed_anywhere() { return device_comm_failed_anywhere(comm_); }

SolveInfo Engine::solve(const double* g, const double* x0, double* x_out, bool x0_is_last) {
    RoctxRange range("sart::solve");
    set_device();
    // a re-solve (fallback, device all-reduce failure) starts from the host x0: x_ has moved by then
    bool x0_on_device = x0 && x0_is_last && last_x_on_device_;
    last_x_on_device_ = false;
    const auto t0 = std::chrono::steady_clock::now();
    // Row shards align the ranks in setup_frame's host collectives; column shards have none there, so while a
    // device path with a timeout is active a barrier keeps a rank that was busy between frames (rank 0 writing
    // the output) from counting against its peers' first all-reduce timeout.
    if (cfg_.column_shard && comm_->size() > 1 && comm_->degradable()) comm_->host().barrier();
    SolveInfo info;
    const int max_sweeps = cfg_.max_iterations + 1;
    auto ms_since = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    };
    std::chrono::steady_clock::time_point t_iter = t0;
    while (true) {
        norm_ = setup_frame(g, x0, x0_on_device);
        x0_on_device = false;
        info.setup_ms = ms_since(t0);
        t_iter = std::chrono::steady_clock::now();
        host_sweep_ = 0;
        // Fault injection (tests): report a protocol timeout from the device in the first sweep of this solve,
        // through the same path as a real one (error word -> all-reduce -> k_decide on every rank).
        if (use_fused_ && injected_ < cfg_.fault_inject && fault_rank_selected(comm_->rank())) {
            ++injected_;
            hip_ok(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&st_.get()->error), 16, 1, stream_), "inject");
        }
        int enqueued = 0, issued = 0, checked = 0;
        bool error = false;
        comm_ms_ = 0.0;
        cev_used_[0] = cev_used_[1] = 0;
        // Chunk sizes. A warm-started frame of a time series needs about as many sweeps as the one before it, so
        // its first chunk holds that many + 1 and the chunk queued behind it (to keep the GPU busy while the first
        // is checked) only 2; later chunks are check_interval long. Sweeps queued past the decision return at once
        // but still cost their launches (~3 x 3 us): with full chunks a sparse 64k x 64k frame of 8 sweeps of 33 us
        // queued 24 of them. Results are unchanged (the decision and the update are on the device).
        const int pred = (x0 && last_sweeps_ > 0) ? last_sweeps_ : 0;
        auto chunk = [&](int k) {
            if (pred && k == 0) return std::min(cfg_.check_interval, pred + 1);
            if (pred && k == 1) return std::min(cfg_.check_interval, 2);
            return cfg_.check_interval;
        };
        auto issue = [&]() {
            const int n = std::min(chunk(issued), max_sweeps - enqueued);
            cur_slot_ = issued & 1;
            run_chunk(n);
            enqueued += n;
            const int slot = issued & 1;
            hip_ok(hipMemcpyAsync(hstate_ + slot, st_.get(), sizeof(SartState), hipMemcpyDeviceToHost, stream_),
                   "D2H state");
            hip_ok(hipEventRecord(ev_[slot], stream_), "event");
            ++issued;
        };
        issue();
        while (true) {
            if (enqueued < max_sweeps) issue();  // keep the GPU busy while the previous chunk is checked
            const int slot = checked & 1;
            hip_ok(hipEventSynchronize(ev_[slot]), "event sync");
            collect_comm(slot);
            SartState s = hstate_[slot];
            ++checked;
            if (s.error) {  // bit 8 (collective) is set on every rank in the same sweep
                error = true;
                break;
            }
            if (s.done || (checked == issued && enqueued >= max_sweeps)) break;
        }
        hip_ok(hipStreamSynchronize(stream_), "solve");
        info.queued_sweeps = enqueued;
        collect_comm(0);  // chunks issued after the last check
        collect_comm(1);
        if (comm_failed_anywhere()) {
            // a device all-reduce timed out somewhere (its output is NaN there): every rank switches to the base
            // communicator and re-solves the frame; a second failure on the base path is fatal
            ++info.comm_fallbacks;
            const bool had = comm_->degrade();
            if (comm_->rank() == 0)
                std::fprintf(stderr, "sart: device all-reduce timed out; re-solving on %s\n", comm_->backend());
            if (!had || info.comm_fallbacks > 1) throw std::runtime_error("SART engine: device all-reduce failed");
            drop_graph();
            continue;
        }
        comm_->check();
        if (error) {
            ++info.fallbacks;
            if (info.fallbacks > 4 || !fallback())
                throw std::runtime_error("SART engine: persistent sweep failed without fallback");
            continue;
        }
        break;
    }
    info.iterate_ms = ms_since(t_iter);
    const auto t_fin = std::chrono::steady_clock::now();
    SartState s;
    hip_ok(hipMemcpy(&s, st_.get(), sizeof(SartState), hipMemcpyDeviceToHost), "D2H state");
    // NaN/Inf guard: x of the failing sweep is non-finite; return the last finite iterate (saved by the update
    // of the previous sweep), unless the very first sweep failed (no update yet: nothing better to return)
    const bool rollback = (s.flags & 1) != 0 && s.sweep >= 2;
    if (V_) {
        hip_ok(hipMemcpyAsync(hxo_, rollback ? xprev_.get() : x_.get(), V_ * sizeof(float), hipMemcpyDeviceToHost,
                              stream_),
               "D2H x");
        hip_ok(hipStreamSynchronize(stream_), "D2H x");
    }
    for (int64_t i = 0; i < V_; ++i) x_out[i] = (double)hxo_[i] * norm_;  // reference sartsolver_cuda.cpp:264-265
    last_x_on_device_ = !rollback;
    last_norm_ = norm_;
    info.status = s.status == kSuccess ? kSuccess : kMaxIterationsExceeded;
    info.iterations = s.iterations;
    info.convergence = s.conv_last;
    info.nonfinite = (s.flags & 1) != 0;
    info.used_fused = use_fused_;
    info.comm = comm_->backend();
    info.fused_variant = use_fused_ ? geom_.variant : -1;
    info.sweeps = s.sweep;
    last_sweeps_ = s.sweep;
    info.comm_ms = timing_collectives() ? comm_ms_ : -1.0;
    info.finish_ms = ms_since(t_fin);
    info.ms = ms_since(t0);
    return info;
}

void Engine::forward(const double* x, double* f) {
    set_device();
    std::vector<float> xf(ld_, 0.f);
    for (int64_t i = 0; i < V_; ++i) xf[i] = (float)x[i];
    DeviceArray<float> xd(ld_);
    hip_ok(hipMemcpyAsync(xd.get(), xf.data(), ld_ * sizeof(float), hipMemcpyHostToDevice, stream_), "H2D");
    fwd(kEpiPlain, xd.get(), fitted_.get(), nullptr, nullptr, nullptr);
    if (cfg_.column_shard && comm_->size() > 1) comm_->all_reduce(fitted_.get(), (size_t)P_, ReduceOp::kSum, stream_);
    std::vector<float> fh(P_);
    if (P_) hip_ok(hipMemcpyAsync(fh.data(), fitted_.get(), P_ * sizeof(float), hipMemcpyDeviceToHost, stream_), "D2H");
    hip_ok(hipStreamSynchronize(stream_), "forward");
    for (int64_t i = 0; i < P_; ++i) f[i] = fh[i];
}

}  // namespace sart
