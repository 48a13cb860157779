#include "multiframe.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>

#include "../kernels/launchers.hpp"

namespace sart {

namespace {
void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

int MultiFrameEngine::batch_width(int frames) { return frames <= 16 ? 16 : (frames <= 32 ? 32 : 64); }

MultiFrameEngine::MultiFrameEngine(int device, const void* A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel,
                                   int64_t ld, Communicator* comm, const EngineConfig& cfg)
    : device_(device), A_(A), bf16_(cfg.rtm_bf16), P_(nrows), Pp_(nrows_pad), V_(nvoxel), ld_(ld), comm_(comm),
      cfg_(cfg) {
    validate_params(cfg_);
    if (!comm_) throw std::invalid_argument("MultiFrameEngine: communicator required");
    if (ld_ % 64 || ld_ < V_ || Pp_ % 64 || Pp_ < P_)
        throw std::invalid_argument("MultiFrameEngine: ld and nrows_pad must be multiples of 64 covering the shard");
    cfg_.check_interval = std::max(1, cfg_.check_interval);
    nf_ = batch_width(cfg_.mf_frames);
    const int NF = nf_;
    set_device();
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hstate_), 2 * sizeof(MfState)), "hipHostMalloc");
    for (auto& e : ev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hg_), std::max<int64_t>(P_, 1) * NF * sizeof(double)),
           "hipHostMalloc");
    nsf_ = mf_forward_num_splits(ld_, Pp_);
    nsb_ = bf16_ ? mf_backproject_b16_num_splits(ld_, P_) : mf_backproject_num_splits(ld_, P_);
    nwb_ = mf_weights_num_blocks(Pp_);
    X_.resize((size_t)NF * ld_);
    Xprev_.resize((size_t)NF * ld_);
    Fs_.resize((size_t)nsf_ * Pp_ * NF);
    W_.resize((size_t)Pp_ * NF);
    part_.resize((size_t)nsb_ * ld_ * NF);
    buf_.resize((size_t)NF * ld_ + NF);  // [nf][ld] correction + [nf] ||A x||^2: one all-reduce per sweep
    pen_.resize((size_t)NF * ld_);
    if (cfg_.logarithmic) O_.resize((size_t)NF * ld_);
    for (auto* b : {&ghat_, &arow_, &gpos_, &wo_}) b->resize((size_t)Pp_ * NF);
    g64_.resize((size_t)Pp_ * NF);
    norm64_.resize(NF);
    G64_.resize(NF);
    F2part_.resize((size_t)nwb_ * NF);
    st_.resize(1);
    if (bf16_) {
        for (auto* b : {&Xh_, &Xl_}) b->resize((size_t)NF * ld_);
        for (auto* b : {&Wh_, &Wl_}) b->resize((size_t)NF * Pp_);
    }
    rs_.compute(A_, P_, Pp_, V_, ld_, comm_, cfg_, stream_, false, bf16_);
    // chunks of the overlapped back-projection / all-reduce pipeline (several ranks only): SART_MF_CHUNKS
    // (default 4) voxel ranges aligned to the back-projection's voxel tile, each >= 1 MiB of corrections
    int nchunks = 1;
    if (comm_->size() > 1) {
        const char* e = std::getenv("SART_MF_CHUNKS");
        nchunks = (e && *e) ? std::max(1, std::atoi(e)) : 4;
        const int64_t min_vox = std::max<int64_t>(1, (1 << 20) / (4 * NF));
        nchunks = (int)std::max<int64_t>(1, std::min<int64_t>(nchunks, ld_ / min_vox));
    }
    const int64_t align = bf16_ ? mf_backproject_b16_vox_align(ld_) : mf_backproject_vox_align(ld_, NF);
    chunks_.assign(1, 0);
    for (int c = 1; c < nchunks; ++c) {
        const int64_t v = (ld_ * c / nchunks) / align * align;
        if (v > chunks_.back() && v < ld_) chunks_.push_back(v);
    }
    chunks_.push_back(ld_);
    if (chunks_.size() > 2) {
        hip_ok(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking), "hipStreamCreate");
        cev_.resize(chunks_.size() - 1);
        for (auto& e : cev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        hip_ok(hipEventCreateWithFlags(&comm_done_, hipEventDisableTiming), "hipEventCreate");
    }
}

MultiFrameEngine::~MultiFrameEngine() {
    set_device();
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (comm_stream_) (void)hipStreamSynchronize(comm_stream_);
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : cev_)
        if (e) (void)hipEventDestroy(e);
    if (comm_done_) (void)hipEventDestroy(comm_done_);
    if (comm_stream_) (void)hipStreamDestroy(comm_stream_);
    if (hstate_) (void)hipHostFree(hstate_);
    if (hg_) (void)hipHostFree(hg_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

void MultiFrameEngine::set_device() const { hip_ok(hipSetDevice(device_), "hipSetDevice"); }

void MultiFrameEngine::set_laplacian(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t nnz) {
    set_device();
    has_lap_ = false;
    if (nnz <= 0 || cfg_.beta_laplace <= 0) return;
    if (row_ptr[V_] != nnz) throw std::invalid_argument("Laplacian CSR row pointer does not match nnz");
    lap_rp_.resize(V_ + 1);
    lap_col_.resize(nnz);
    lap_val_.resize(nnz);
    hip_ok(hipMemcpy(lap_rp_.get(), row_ptr, (V_ + 1) * sizeof(int64_t), hipMemcpyHostToDevice), "H2D");
    hip_ok(hipMemcpy(lap_col_.get(), col, nnz * sizeof(int32_t), hipMemcpyHostToDevice), "H2D");
    hip_ok(hipMemcpy(lap_val_.get(), val, nnz * sizeof(float), hipMemcpyHostToDevice), "H2D");
    has_lap_ = true;
}

void MultiFrameEngine::forward() {
    if (bf16_) {
        launch_mf_split_x(X_.get(), (int64_t)nf_ * ld_, Xh_.get(), Xl_.get(), stream_);
        launch_mf_forward_b16(static_cast<const bf16_t*>(A_), ld_, P_, Pp_, Xh_.get(), Xl_.get(), Fs_.get(), nsf_, nf_,
                              stream_);
    } else {
        launch_mf_forward(static_cast<const float*>(A_), ld_, P_, Pp_, X_.get(), ld_, Fs_.get(), nsf_, nf_, stream_);
    }
}

void MultiFrameEngine::backproject(const float* W, bool split_w, int64_t v0, int64_t v1) {
    if (bf16_) {
        if (split_w) launch_mf_split_w(W, Pp_, nf_, Pp_, Wh_.get(), Wl_.get(), stream_);
        launch_mf_backproject_b16(static_cast<const bf16_t*>(A_), ld_, P_, Wh_.get(), Wl_.get(), Pp_, nsb_,
                                  part_.get(), nf_, stream_, v0, v1);
    } else {
        launch_mf_backproject(static_cast<const float*>(A_), ld_, P_, W, nsb_, part_.get(), nf_, stream_, v0, v1);
    }
}

void MultiFrameEngine::sweep() {
    const int NF = nf_;
    MfState* st = st_.get();
    float* D = buf_.get();                     // [ld][nf] voxel-major corrections
    float* F2 = buf_.get() + (int64_t)NF * ld_;  // [nf] ||A x||^2, all-reduced with the last chunk
    const float* scale = cfg_.logarithmic ? rs_.dmask.get() : rs_.dscale.get();
    forward();
    launch_mf_weights(Fs_.get(), nsf_, Pp_, ghat_.get(), arow_.get(), cfg_.logarithmic, W_.get(), F2part_.get(),
                      NF, stream_);
    const int nc = (int)chunks_.size() - 1;
    if (comm_->size() > 1 && nc > 1) {
        // Overlap: the back-projection runs chunk by chunk over the voxel axis on the compute
        // stream; the all-reduce of chunk c (a contiguous [v0, v1) x nf slice of the voxel-major corrections)
        // runs on the comm stream as soon as its collect has finished, next to the back-projection of the later
        // chunks. All compute chunks are queued first so that a host-staged all-reduce, which blocks this thread,
        // still overlaps with them.
        for (int c = 0; c < nc; ++c) {
            const int64_t v0 = chunks_[c], v1 = chunks_[c + 1];
            backproject(W_.get(), c == 0, v0, v1);
            const bool last = c == nc - 1;
            launch_mf_collect(part_.get(), nsb_, ld_, v0, v1, scale, D, last ? F2part_.get() : nullptr, nwb_,
                              last ? F2 : nullptr, NF, stream_);
            hip_ok(hipEventRecord(cev_[c], stream_), "event");
        }
        for (int c = 0; c < nc; ++c) {
            const int64_t v0 = chunks_[c], v1 = chunks_[c + 1];
            hip_ok(hipStreamWaitEvent(comm_stream_, cev_[c], 0), "wait chunk");
            const size_t n = (size_t)(v1 - v0) * NF + (c == nc - 1 ? (size_t)NF : 0);
            comm_->all_reduce(D + v0 * NF, n, ReduceOp::kSum, comm_stream_);
        }
        hip_ok(hipEventRecord(comm_done_, comm_stream_), "event");
    } else {
        backproject(W_.get(), true, 0, ld_);
        launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, scale, D, F2part_.get(), nwb_, F2, NF, stream_);
        if (comm_->size() > 1) comm_->all_reduce(buf_.get(), (size_t)NF * ld_ + NF, ReduceOp::kSum, stream_);
    }
    const float* pen = nullptr;
    if (has_lap_) {  // needs X only: runs while the last chunks are being reduced
        launch_mf_penalty(lap_rp_.get(), lap_col_.get(), lap_val_.get(), V_, (float)cfg_.beta_laplace,
                          cfg_.logarithmic, X_.get(), ld_, pen_.get(), st, NF, stream_);
        pen = pen_.get();
    }
    if (comm_->size() > 1 && nc > 1) hip_ok(hipStreamWaitEvent(stream_, comm_done_, 0), "wait all-reduce");
    launch_mf_decide(st, F2, stream_);
    launch_mf_update(X_.get(), D, O_.get(), pen, (float)cfg_.relaxation, cfg_.logarithmic, V_, ld_, st, NF, stream_,
                     Xprev_.get());
}

void MultiFrameEngine::solve_group(const double* g, int B, double* x_out, SolveInfo* info, const double* x0) {
    RoctxRange range("sart::mf_solve");
    const int NF = nf_;
    const auto t0 = std::chrono::steady_clock::now();
    // host: layout [rows][nf], per-frame maxima and sums of squares (reference sartsolver_cuda.cpp:146-157)
    double mx[kMfMaxFrames], gs[kMfMaxFrames];
    for (int f = 0; f < NF; ++f) mx[f] = -std::numeric_limits<double>::infinity(), gs[f] = 0.0;
    for (int64_t p = 0; p < P_; ++p)
        for (int f = 0; f < NF; ++f) {
            double v = f < B ? g[(int64_t)f * P_ + p] : 0.0;
            if (!std::isfinite(v)) v = -1.0;  // non-finite pixel: masked like a saturated one
            hg_[p * NF + f] = v;
            if (f < B) {
                mx[f] = std::max(mx[f], v);
                if (v > 0) gs[f] += v * v;
            }
        }
    comm_->host().all_reduce_host(mx, NF, ReduceOp::kMax);
    comm_->host().all_reduce_host(gs, NF, ReduceOp::kSum);
    double norm[kMfMaxFrames], G[kMfMaxFrames];
    for (int f = 0; f < NF; ++f) {
        norm[f] = (f < B && mx[f] > 0) ? mx[f] : 1.0;
        G[f] = gs[f] / (norm[f] * norm[f]);
        if (!(G[f] > 0)) G[f] = 1.0;
    }
    if (P_) hip_ok(hipMemcpyAsync(g64_.get(), hg_, P_ * NF * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D g");
    hip_ok(hipMemcpyAsync(norm64_.get(), norm, NF * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D norm");
    hip_ok(hipMemcpyAsync(G64_.get(), G, NF * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D G");
    launch_mf_prep(g64_.get(), P_, Pp_, norm64_.get(), rs_.ray_len.get(), (float)cfg_.ray_length_threshold,
                   ghat_.get(), arow_.get(), gpos_.get(), wo_.get(), NF, stream_);
    if (x0) {  // warm start: x_prev / s per frame, clamped (reference sartsolver_cuda.cpp:176-180)
        if ((int64_t)x064_.size() < V_) x064_.resize(std::max<int64_t>(V_, 1));
        if (V_) hip_ok(hipMemcpyAsync(x064_.get(), x0, V_ * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D x0");
        launch_mf_init_warm(X_.get(), x064_.get(), norm64_.get(), V_, ld_, B, NF, stream_);
    } else {
        // cold start x0 = max([rho > tau] A^T max(ghat, 0) / rho, 1e-7) per frame (reference sart_kernels.cu:22-60)
        backproject(gpos_.get(), true, 0, ld_);
        launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, nullptr, buf_.get(), nullptr, 0, nullptr, NF, stream_);
        comm_->all_reduce(buf_.get(), (size_t)NF * ld_, ReduceOp::kSum, stream_);
        launch_mf_init(X_.get(), buf_.get(), rs_.dinv.get(), V_, ld_, B, NF, stream_);
    }
    if (cfg_.logarithmic) {  // frame-constant observed back-projection, reduced once per batch
        backproject(wo_.get(), true, 0, ld_);
        launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, rs_.dmask.get(), O_.get(), nullptr, 0, nullptr, NF, stream_);
        comm_->all_reduce(O_.get(), (size_t)NF * ld_, ReduceOp::kSum, stream_);
    }
    launch_mf_state_begin(st_.get(), G64_.get(), B, cfg_.conv_tolerance, cfg_.max_iterations, NF, stream_);
    // Chunks of check_interval sweeps, pipelined like Engine::solve: chunk c + 1 is queued before the state
    // after chunk c is read, so the GPU never drains between chunks (sweeps after all_done are no-ops).
    const int max_sweeps = cfg_.max_iterations + 1;
    int enqueued = 0, issued = 0, checked = 0;
    auto issue = [&]() {
        const int n = std::min(cfg_.check_interval, max_sweeps - enqueued);
        {
            RoctxRange r("sart::mf_chunk");
            for (int i = 0; i < n; ++i) sweep();
        }
        enqueued += n;
        const int slot = issued & 1;
        hip_ok(hipMemcpyAsync(hstate_ + slot, st_.get(), sizeof(MfState), hipMemcpyDeviceToHost, stream_), "D2H state");
        hip_ok(hipEventRecord(ev_[slot], stream_), "event");
        ++issued;
    };
    issue();
    while (true) {
        if (enqueued < max_sweeps) issue();
        const int slot = checked & 1;
        hip_ok(hipEventSynchronize(ev_[slot]), "mf chunk");
        ++checked;
        if (hstate_[slot].all_done || (checked == issued && enqueued >= max_sweeps)) break;
    }
    std::vector<float> xh((size_t)NF * ld_), xp;
    hip_ok(hipMemcpyAsync(xh.data(), X_.get(), xh.size() * sizeof(float), hipMemcpyDeviceToHost, stream_), "D2H X");
    hip_ok(hipMemcpyAsync(hstate_, st_.get(), sizeof(MfState), hipMemcpyDeviceToHost, stream_), "D2H state");
    hip_ok(hipStreamSynchronize(stream_), "mf solve");
    if (hstate_->flags) {  // NaN/Inf guard: frames that stopped on a non-finite iterate return the last finite one
        xp.resize(xh.size());
        hip_ok(hipMemcpy(xp.data(), Xprev_.get(), xp.size() * sizeof(float), hipMemcpyDeviceToHost), "D2H Xprev");
    }
    comm_->check();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int f = 0; f < B; ++f) {
        const bool rollback = (hstate_->rollback >> f) & 1;
        const float* src = rollback ? xp.data() : xh.data();
        for (int64_t v = 0; v < V_; ++v) x_out[(int64_t)f * V_ + v] = (double)src[(size_t)f * ld_ + v] * norm[f];
        info[f].status = hstate_->status[f] == kSuccess ? kSuccess : kMaxIterationsExceeded;
        info[f].iterations = hstate_->iters[f];
        info[f].convergence = hstate_->conv[f];
        info[f].nonfinite = (hstate_->flags >> f) & 1;
        info[f].used_fused = false;
        info[f].ms = ms / B;
    }
}

std::vector<SolveInfo> MultiFrameEngine::solve_batch(const double* g, int nframes, double* x_out, const double* x0,
                                                     bool chain) {
    set_device();
    std::vector<SolveInfo> out(std::max(nframes, 0));
    const double* warm = x0;
    for (int b0 = 0; b0 < nframes; b0 += nf_) {
        const int B = std::min(nf_, nframes - b0);
        solve_group(g + (int64_t)b0 * P_, B, x_out + (int64_t)b0 * V_, out.data() + b0, warm);
        // time-series warm start: the next group starts from this group's last solution (if it is finite)
        const double* last = x_out + (int64_t)(b0 + B - 1) * V_;
        warm = chain && std::all_of(last, last + V_, [](double v) { return std::isfinite(v); }) ? last : nullptr;
    }
    return out;
}

}  // namespace sart
