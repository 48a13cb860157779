#include "multiframe.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <thread>

#include "../kernels/launchers.hpp"

namespace sart {

namespace {
void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

int MultiFrameEngine::batch_width(int frames) {
    return frames <= 16 ? 16 : (frames <= 32 ? 32 : (frames <= 64 ? 64 : 128));
}

MultiFrameEngine::MultiFrameEngine(int device, const void* A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel,
                                   int64_t ld, Communicator* comm, const EngineConfig& cfg, const SparseRtm* sparse)
    : device_(device), A_(A), bf16_(cfg.rtm_bf16), P_(nrows), Pp_(nrows_pad), V_(nvoxel), ld_(ld), comm_(comm),
      cfg_(cfg) {
    validate_params(cfg_);
    if (sparse) {
        if (bf16_) throw std::invalid_argument("MultiFrameEngine: a sparse shard holds fp32 values");
        if (!sparse->row_ptr || !sparse->col_ptr)
            throw std::invalid_argument("MultiFrameEngine: sparse shard needs its CSR and CSC arrays");
        sparse_ = true;
        sp_ = *sparse;
        cfg_.mf_split_a = 0;  // fp32 SpMM: no operand splits
    } else if (!A_) {
        throw std::invalid_argument("MultiFrameEngine: dense shard pointer required");
    }
    if (const char* fn = std::getenv("SART_FAULT_NAN"); fn && *fn && cfg_.fault_nan_sweep < 0)
        cfg_.fault_nan_sweep = std::atoi(fn);
    if (!comm_) throw std::invalid_argument("MultiFrameEngine: communicator required");
    if (ld_ % 64 || ld_ < V_ || Pp_ % 64 || Pp_ < P_)
        throw std::invalid_argument("MultiFrameEngine: ld and nrows_pad must be multiples of 64 covering the shard");
    cfg_.check_interval = std::max(1, cfg_.check_interval);
    nf_ = batch_width(cfg_.mf_frames);
    if (!bf16_) {
        int m = cfg_.mf_split_a;
        if (m < 0) {
            const char* e = std::getenv("SART_MF_X3");
            m = (e && *e) ? (std::atoi(e) != 0) : (nf_ >= 32);
        }
        x3_ = m != 0;
    }
    // split-A back-projection: f16 pairs (three products) unless SART_MF_BWD16=0 (bf16 hi + mid + lo, six); split-A
    // forward: f16 pairs unless SART_MF_FWD16=0 (bf16 hi + lo, whose 2^-17 per product is not fp32-grade on rows
    // dominated by a few entries: tests/test_gpu_realistic.py)
    if (sparse_) x3_ = false;
    if (const char* e = std::getenv("SART_MF_BWD16"); x3_) h16_ = !(e && *e && std::atoi(e) == 0);
    if (const char* e = std::getenv("SART_MF_FWD16"); x3_) fwd16_ = !(e && *e && std::atoi(e) == 0);
    // 128 columns (8 MFMA column groups) exist for bf16 storage and for split-A with the f16-pair back-projection;
    // the fp32 MFMA and three-piece bf16 back-projection paths take 64-frame batches
    if (nf_ == 128 && !(sparse_ || bf16_ || (x3_ && h16_))) nf_ = 64;
    const int NF = nf_;
    split_ = bf16_ || x3_;
    if (split_) {  // X planes blocked [ld / 32][nf][32] for the forward (SART_MF_XBLK=0: frame-major, A/B runs)
        const char* e = std::getenv("SART_MF_XBLK");
        xblk_ = !(e && *e && std::atoi(e) == 0);
    }
    if (const char* e = std::getenv("SART_MF_LAST_BWD"); e && *e) skip_last_bwd_ = std::atoi(e) == 0;
    set_device();
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hstate_), 2 * sizeof(MfState)), "hipHostMalloc");
    for (auto& e : ev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hg_), std::max<int64_t>(P_, 1) * NF * sizeof(double)),
           "hipHostMalloc");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hx_), (size_t)NF * ld_ * sizeof(float)), "hipHostMalloc");
    hip_ok(hipEventCreateWithFlags(&ev_copy_, hipEventDisableTiming), "hipEventCreate");
    nsf_ = mf_forward_num_splits(ld_, Pp_, bf16_ ? 512 : 0);  // bf16 storage: ~512 workgroups (see the back-projection)
    nsb_ = split_ ? mf_backproject_b16_num_splits(ld_, P_, x3_) : mf_backproject_num_splits(ld_, P_);
    if (sparse_) {  // the SpMM kernels write complete sums
        nsf_ = nsb_ = 1;
        Xt_.resize((size_t)ld_ * NF);
        pw_ = mf_sparse_plane_width(NF);
        if (mf_sparse_needs_w_planes(NF, pw_)) Wt_.resize((size_t)Pp_ * NF);  // cold-start / log operands re-laid
    }
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
    G64_.resize(NF);
    F2part_.resize((size_t)nwb_ * NF);
    st_.resize(1);
    if (split_) {
        for (auto* b : {&Xh_, &Xl_}) b->resize((size_t)NF * ld_);
        if (h16_) {
            W16_.resize((size_t)2 * NF * Pp_);
            wmax_.resize(NF);
            wscale_.resize(NF);
            csc_.resize((size_t)2 * ld_);
            DeviceArray<unsigned> cmax;
            cmax.resize(ld_);
            launch_mf_col_scales(static_cast<const float*>(A_), ld_, Pp_, cmax.get(), csc_.get(), stream_);
            hip_ok(hipStreamSynchronize(stream_), "column scales");
        }
        if (fwd16_) {
            rsc_.resize((size_t)2 * Pp_);
            xinv_.resize(NF);
            xmax_.resize(NF);
            launch_mf_row_scales(static_cast<const float*>(A_), ld_, Pp_, rsc_.get(), stream_);
        }
        if (!h16_) {
            Wh_.resize((size_t)(x3_ ? 2 : 1) * NF * Pp_);  // split-A: hi and mid planes
            Wl_.resize((size_t)NF * Pp_);
        }
    }
    if (sparse_)
        rs_.compute_sparse(sp_, P_, Pp_, V_, ld_, comm_, cfg_, stream_);
    else
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
    const int64_t align = split_ ? mf_backproject_b16_vox_align(ld_, x3_) : mf_backproject_vox_align(ld_, NF);
    chunks_.assign(1, 0);
    for (int c = 1; c < nchunks; ++c) {
        const int64_t v = (ld_ * c / nchunks) / align * align;
        if (v > chunks_.back() && v < ld_) chunks_.push_back(v);
    }
    chunks_.push_back(ld_);
    if (comm_->size() > 1) {  // the fp32 collectives of a sweep (p2p auto mode times exactly these sizes)
        std::vector<int64_t> sizes{(int64_t)NF * ld_ + NF, (int64_t)NF * ld_, (int64_t)NF};
        for (size_t c = 0; c + 1 < chunks_.size(); ++c)
            sizes.push_back((chunks_[c + 1] - chunks_[c]) * NF + (c + 2 == chunks_.size() ? NF : 0));
        comm_->prepare(sizes);
    }
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
    if (hx_) (void)hipHostFree(hx_);
    if (ev_copy_) (void)hipEventDestroy(ev_copy_);
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

std::string MultiFrameEngine::forward_split() const {
    if (sparse_) return "sparse-fp32";
    return bf16_ ? "bf16-storage" : (!x3_ ? "fp32" : (fwd16_ ? "f16x2" : "bf16x2"));
}

std::string MultiFrameEngine::backproject_split() const {
    if (sparse_) return "sparse-fp32";
    return bf16_ ? "bf16-storage" : (!x3_ ? "fp32" : (h16_ ? "f16x2" : "bf16x3"));
}

void MultiFrameEngine::forward() {
    if (sparse_) {
        launch_mf_sparse_forward(sp_, P_, Pp_, X_.get(), ld_, Xt_.get(), Fs_.get(), nf_, pw_, stream_, g_mf_skip);
        return;
    }
    if (fwd16_) {
        uint16_t* x1 = reinterpret_cast<uint16_t*>(Xh_.get());
        uint16_t* x2 = reinterpret_cast<uint16_t*>(Xl_.get());
        launch_mf_split_x16(X_.get(), ld_, nf_, x1, x2, xmax_.get(), xinv_.get(), stream_, true, xblk_);
        launch_mf_forward_h16(static_cast<const float*>(A_), ld_, P_, Pp_, x1, x2, Fs_.get(), nsf_, nf_, stream_, xblk_,
                              rsc_.get(), xinv_.get());
        return;
    }
    if (split_) {
        launch_mf_split_x(X_.get(), (int64_t)nf_ * ld_, Xh_.get(), Xl_.get(), stream_, x3_, xblk_ ? ld_ : 0);
        if (bf16_)
            launch_mf_forward_b16(static_cast<const bf16_t*>(A_), ld_, P_, Pp_, Xh_.get(), Xl_.get(), Fs_.get(), nsf_,
                                  nf_, stream_, xblk_);
        else
            launch_mf_forward_x3(static_cast<const float*>(A_), ld_, P_, Pp_, Xh_.get(), Xl_.get(), Fs_.get(), nsf_,
                                 nf_, stream_, xblk_);
    } else {
        launch_mf_forward(static_cast<const float*>(A_), ld_, P_, Pp_, X_.get(), ld_, Fs_.get(), nsf_, nf_, stream_);
    }
}

void MultiFrameEngine::backproject(const float* W, bool split_w, int64_t v0, int64_t v1, bool have_max, float* out,
                                   const float* oscale) {
    if (sparse_) {
        // W_ comes from the weights kernel already in frame-order planes (sweep); the cold-start operands (gpos_,
        // wo_) are re-laid here
        if (mf_sparse_needs_w_planes(nf_, pw_) && W != W_.get()) {
            if (split_w) launch_mf_w_planes(W, Pp_, nf_, pw_, Wt_.get(), stream_, g_mf_skip);
            W = Wt_.get();
        }
        launch_mf_sparse_backproject(sp_, V_, W, Pp_, out ? out : part_.get(), out ? oscale : nullptr, nf_, pw_, v0,
                                     v1, stream_, g_mf_skip);
        return;
    }
    if (h16_) {
        uint16_t* w1 = W16_.get();
        uint16_t* w2 = W16_.get() + (size_t)nf_ * Pp_;
        if (split_w)
            launch_mf_split_w16(W, Pp_, nf_, Pp_, w1, w2, wmax_.get(), 1.f, wscale_.get(), stream_, have_max);
        launch_mf_backproject_h16(static_cast<const float*>(A_), ld_, P_, w1, w2, Pp_, nsb_, part_.get(), nf_, stream_,
                                  v0, v1, csc_.get(), wscale_.get());
    } else if (split_) {
        if (split_w) launch_mf_split_w(W, Pp_, nf_, Pp_, Wh_.get(), Wl_.get(), stream_, x3_);
        if (bf16_)
            launch_mf_backproject_b16(static_cast<const bf16_t*>(A_), ld_, P_, Wh_.get(), Wl_.get(), Pp_, nsb_,
                                      part_.get(), nf_, stream_, v0, v1);
        else
            launch_mf_backproject_x3(static_cast<const float*>(A_), ld_, P_, Wh_.get(), Wl_.get(), Pp_, nsb_,
                                     part_.get(), nf_, stream_, v0, v1);
    } else {
        launch_mf_backproject(static_cast<const float*>(A_), ld_, P_, W, nsb_, part_.get(), nf_, stream_, v0, v1);
    }
}

void MultiFrameEngine::sweep(bool last) {
    const int NF = nf_;
    MfState* st = st_.get();
    const MfSkipScope skip(&st->all_done);  // every slot done: the sweep's heavy kernels return at once
    float* D = buf_.get();                     // [ld][nf] voxel-major corrections
    float* F2 = buf_.get() + (int64_t)NF * ld_;  // [nf] ||A x||^2, all-reduced with the last chunk
    const float* scale = cfg_.logarithmic ? rs_.dmask.get() : rs_.dscale.get();
    forward();
    // f16-pair back-projection: the weights kernel also leaves each frame's max |w| (its f16 scale) in wmax_
    launch_mf_weights(Fs_.get(), nsf_, Pp_, ghat_.get(), arow_.get(), cfg_.logarithmic, W_.get(), F2part_.get(),
                      NF, stream_, h16_ ? wmax_.get() : nullptr,
                      sparse_ && mf_sparse_needs_w_planes(NF, pw_) ? pw_ : 0);
    if (last && skip_last_bwd_) {
        // every running frame is decided at max_iter here (its update is skipped on all_done): ||A x||^2 only
        launch_mf_collect(part_.get(), nsb_, ld_, 0, 0, scale, D, F2part_.get(), nwb_, F2, NF, stream_);
        if (comm_->size() > 1) comm_->all_reduce(F2, (size_t)NF, ReduceOp::kSum, stream_);
        launch_mf_decide(st, F2, stream_);
        ++host_sweep_;
        return;
    }
    // D[v0, v1) = scale * A^T W and, with the last chunk, the per-frame ||A x||^2: a sparse shard's SpMM writes the
    // scaled sums itself (the collect then only sums F2part)
    auto bwd_collect = [&](int64_t v0, int64_t v1, bool first, bool lastc) {
        if (sparse_) {
            backproject(W_.get(), first, v0, v1, true, D, scale);
            if (lastc) launch_mf_collect(part_.get(), nsb_, ld_, 0, 0, scale, D, F2part_.get(), nwb_, F2, NF, stream_);
            return;
        }
        backproject(W_.get(), first, v0, v1, true);
        launch_mf_collect(part_.get(), nsb_, ld_, v0, v1, scale, D, lastc ? F2part_.get() : nullptr, nwb_,
                          lastc ? F2 : nullptr, NF, stream_);
    };
    const int nc = (int)chunks_.size() - 1;
    if (comm_->size() > 1 && nc > 1) {
        // Overlap: the back-projection runs chunk by chunk over the voxel axis on the compute
        // stream; the all-reduce of chunk c (a contiguous [v0, v1) x nf slice of the voxel-major corrections)
        // runs on the comm stream as soon as its collect has finished, next to the back-projection of the later
        // chunks. All compute chunks are queued first so that a host-staged all-reduce, which blocks this thread,
        // still overlaps with them.
        for (int c = 0; c < nc; ++c) {
            const int64_t v0 = chunks_[c], v1 = chunks_[c + 1];
            const bool last = c == nc - 1;
            bwd_collect(v0, v1, c == 0, last);
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
        bwd_collect(0, ld_, true, true);
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
    if (cfg_.fault_nan_sweep >= 0 && host_sweep_ == cfg_.fault_nan_sweep)  // fault injection (tests): slot 0
        hip_ok(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(X_.get()), 0x7fc00000, 1, stream_), "inject NaN");
    ++host_sweep_;
}

// Continuous batching. The batch's nf columns are slots: every slot holds one frame, and a slot whose frame has
// finished (converged, non-finite, or max_iter) is refilled with the next frame between two sweeps, so no
// sweep works on finished frames while frames are waiting (the former group-by-group solve ran every group
// as long as its slowest frame). All ranks see the same device state (it follows all-reduced sums), so they
// admit the same frames at the same chunk.
// Start values: the first frames start from x0 (or cold); later frames of a time series (chain) from the
// solution of the latest frame finished before them (SolveInfo::warm_from), otherwise cold (--no_guess).
// The chunks of check_interval sweeps stay pipelined: chunk c + 1 is queued before the state after chunk c
// is read, so a refill decided on chunk c's state is queued after chunk c + 1 and the slot's new frame is
// visible in the states from chunk c + 2 on.
void MultiFrameEngine::admit(const double* g, const std::vector<int>& slots, const std::vector<int>& frames,
                             const double* warm, const float* dev_src, double src_norm,
                             std::vector<double>& slot_norm) {
    const int NF = nf_;
    const int k = (int)slots.size();
    if (k == 0) return;
    // per-frame maxima and positive sums of squares over all ranks' pixels (reference sartsolver_cuda.cpp:146-157)
    double mx[kMfMaxFrames], gs[kMfMaxFrames];
    auto scan = [&](int q) {  // one frame, pixels in order (the sum is deterministic whatever thread runs it)
        double m = -std::numeric_limits<double>::infinity(), s = 0.0;
        const double* gq = g + (int64_t)frames[q] * P_;
        double* hq = hg_ + (int64_t)q * P_;
        for (int64_t p = 0; p < P_; ++p) {
            double v = gq[p];
            if (!std::isfinite(v)) v = -1.0;  // non-finite pixel: masked like a saturated one
            hq[p] = v;
            m = std::max(m, v);
            if (v > 0) s += v * v;
        }
        mx[q] = m, gs[q] = s;
    };
    // frames on host threads when the batch is large (64 frames x 245760 pixels: 12 ms on one thread per solve)
    const int nth = (int)std::min<int64_t>({k, 8, std::max<int64_t>(1, (int64_t)k * P_ / (1 << 20))});
    if (nth > 1) {
        std::vector<std::thread> pool;
        for (int t = 0; t < nth; ++t)
            pool.emplace_back([&, t] {
                for (int q = t; q < k; q += nth) scan(q);
            });
        for (auto& th : pool) th.join();
    } else {
        for (int q = 0; q < k; ++q) scan(q);
    }
    comm_->host().all_reduce_host(mx, k, ReduceOp::kMax);
    comm_->host().all_reduce_host(gs, k, ReduceOp::kSum);
    MfSlots sl{};
    sl.n = k;
    for (int q = 0; q < k; ++q) {
        sl.slot[q] = slots[q];
        sl.norm[q] = mx[q] > 0 ? mx[q] : 1.0;
        sl.G[q] = gs[q] / (sl.norm[q] * sl.norm[q]);
        if (!(sl.G[q] > 0)) sl.G[q] = 1.0;
        slot_norm[slots[q]] = sl.norm[q];
    }
    if (P_) hip_ok(hipMemcpyAsync(g64_.get(), hg_, (size_t)k * P_ * sizeof(double), hipMemcpyHostToDevice, stream_),
                   "H2D g");
    launch_mf_prep_slots(g64_.get(), P_, Pp_, sl, rs_.ray_len.get(), (float)cfg_.ray_length_threshold, ghat_.get(),
                         arow_.get(), gpos_.get(), wo_.get(), NF, stream_);
    if (warm) {  // x = x_prev / s, clamped (reference sartsolver_cuda.cpp:176-180)
        if (V_) hip_ok(hipMemcpyAsync(x064_.get(), warm, V_ * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D x0");
        launch_mf_init_slots_warm(X_.get(), x064_.get(), sl, V_, ld_, stream_);
    } else if (dev_src) {  // copied first: a new frame may enter the source's own slot
        if (V_) hip_ok(hipMemcpyAsync(xsrc_.get(), dev_src, V_ * sizeof(float), hipMemcpyDeviceToDevice, stream_), "D2D");
        launch_mf_init_slots_scaled(X_.get(), xsrc_.get(), src_norm, sl, V_, ld_, stream_);
    } else {  // x0 = max([rho > tau] A^T max(ghat, 0) / rho, 1e-7) (reference sart_kernels.cu:22-60)
        backproject(gpos_.get(), true, 0, ld_);
        launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, nullptr, buf_.get(), nullptr, 0, nullptr, NF, stream_);
        comm_->all_reduce(buf_.get(), (size_t)NF * ld_, ReduceOp::kSum, stream_);
        launch_mf_init_slots_cold(X_.get(), buf_.get(), rs_.dinv.get(), sl, V_, ld_, NF, stream_);
    }
    if (cfg_.logarithmic) {  // frame-constant observed back-projection of the new frames
        backproject(wo_.get(), true, 0, ld_);
        launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, rs_.dmask.get(), Otmp_.get(), nullptr, 0, nullptr, NF,
                          stream_);
        comm_->all_reduce(Otmp_.get(), (size_t)NF * ld_, ReduceOp::kSum, stream_);
        launch_mf_copy_slots(O_.get(), Otmp_.get(), sl, ld_, NF, stream_);
    }
    launch_mf_slot_reset(st_.get(), sl, stream_);
}

std::vector<SolveInfo> MultiFrameEngine::solve_batch(const double* g, int nframes, double* x_out, const double* x0,
                                                     bool chain) {
    // a device all-reduce that timed out on some rank (P2P: a peer never arrived) is agreed over the host
    // communicator; every rank then switches to the base communicator and re-solves the batch once
    for (int attempt = 0;; ++attempt) {
        std::vector<SolveInfo> out = solve_batch_once(g, nframes, x_out, x0, chain);
        if (!device_comm_failed_anywhere(comm_)) {
            comm_->check();
            for (auto& info : out) {
                info.comm_fallbacks = attempt;
                info.comm = comm_->backend();
            }
            return out;
        }
        const bool had = comm_->degrade();
        if (comm_->rank() == 0)
            std::fprintf(stderr, "sart: device all-reduce timed out; re-solving the batch on %s\n", comm_->backend());
        if (!had || attempt >= 1) throw std::runtime_error("MultiFrameEngine: device all-reduce failed");
    }
}

std::vector<SolveInfo> MultiFrameEngine::solve_batch_once(const double* g, int nframes, double* x_out,
                                                          const double* x0, bool chain) {
    set_device();
    RoctxRange range("sart::mf_solve");
    const int NF = nf_;
    std::vector<SolveInfo> out(std::max(nframes, 0));
    if (nframes <= 0) return out;
    const auto t0 = std::chrono::steady_clock::now();
    host_sweep_ = 0;
    if ((int64_t)x064_.size() < V_) x064_.resize(std::max<int64_t>(V_, 1));
    if (cfg_.logarithmic && (int64_t)Otmp_.size() < (int64_t)NF * ld_) Otmp_.resize((size_t)NF * ld_);
    if ((int64_t)xsrc_.size() < ld_) xsrc_.resize(ld_);
    // every slot starts empty (done) with finite zero columns
    for (auto* b : {&X_, &Xprev_, &ghat_, &arow_, &gpos_, &wo_})
        hip_ok(hipMemsetAsync(b->get(), 0, b->size() * sizeof(float), stream_), "memset");
    if (cfg_.logarithmic) hip_ok(hipMemsetAsync(O_.get(), 0, O_.size() * sizeof(float), stream_), "memset");
    hip_ok(hipMemsetAsync(G64_.get(), 0, G64_.size() * sizeof(double), stream_), "memset");
    launch_mf_state_begin(st_.get(), G64_.get(), 0, cfg_.conv_tolerance, cfg_.max_iterations, NF, stream_);

    std::vector<int> slot_frame(NF, -1), slot_valid(NF, 0), frame_warm(nframes, -1);
    std::vector<double> slot_norm(NF, 1.0), frame_norm(nframes, 1.0);
    int next = 0, finished = 0, latest = -1;  // latest: highest-index frame finished with a finite solution
    int issued = 0, checked = 0;
    // frames whose solution is being copied back (finalised at the next state check, after the copy)
    struct Pending {
        int frame, slot;
        bool rollback;
    };
    std::vector<Pending> pend;
    auto finalize = [&]() {
        for (const Pending& pd : pend) {
            const float* src = hx_ + (size_t)pd.slot * ld_;
            double* dst = x_out + (int64_t)pd.frame * V_;
            for (int64_t v = 0; v < V_; ++v) dst[v] = (double)src[v] * frame_norm[pd.frame];
            bool finite = true;
            for (int64_t v = 0; v < V_ && finite; ++v) finite = std::isfinite(dst[v]);
            if (finite && pd.frame > latest) latest = pd.frame;
            ++finished;
        }
        pend.clear();
    };
    // dev: the best finished frame whose solution is still only on the device (collected at this check)
    struct DevSrc {
        int frame = -1, slot = -1;
        bool prev = false;
    };
    auto fill = [&](const std::vector<int>& free_slots, const DevSrc& dev) {
        std::vector<int> slots, frames;
        for (int f : free_slots) {
            if (next >= nframes) break;
            slots.push_back(f);
            frames.push_back(next++);
        }
        if (slots.empty()) return;
        const double* warm = nullptr;
        const float* dsrc = nullptr;
        double dnorm = 1.0;
        int wsrc = -1;
        if (issued == 0) {
            warm = x0;  // the first frames: the caller's start value (or cold)
        } else if (chain && dev.frame > latest) {
            dsrc = (dev.prev ? Xprev_.get() : X_.get()) + (size_t)dev.slot * ld_;
            dnorm = frame_norm[dev.frame];
            wsrc = dev.frame;
        } else if (chain && latest >= 0) {
            warm = x_out + (int64_t)latest * V_;
            wsrc = latest;
        }
        admit(g, slots, frames, warm, dsrc, dnorm, slot_norm);
        for (size_t q = 0; q < slots.size(); ++q) {
            slot_frame[slots[q]] = frames[q];
            slot_valid[slots[q]] = issued;  // states from the next chunk on describe this frame
            frame_warm[frames[q]] = wsrc;
        }
    };
    // Sweeps are queued in chunks of at most check_interval, and never past the last sweep a running frame can
    // need: a frame admitted after `enq` queued sweeps has made its final decision by sweep enq + max_iter + 1
    // (its slot keeps the device sweep counter running), so a fixed-iteration batch queues exactly the sweeps
    // it uses.
    int64_t enq = 0;
    std::vector<int64_t> slot_end(NF, 0);
    auto issue = [&]() {
        int64_t bound = 0;
        for (int f = 0; f < NF; ++f)
            if (slot_frame[f] >= 0) bound = std::max(bound, slot_end[f] - enq);
        const int n = (int)std::min<int64_t>(cfg_.check_interval, bound);
        if (n <= 0) return false;
        {
            RoctxRange r("sart::mf_chunk");
            // the chunk that reaches the bound ends with the batch's final sweep (its frames are all decided there)
            for (int i = 0; i < n; ++i) sweep(i == bound - 1);
        }
        enq += n;
        const int slot = issued & 1;
        hip_ok(hipMemcpyAsync(hstate_ + slot, st_.get(), sizeof(MfState), hipMemcpyDeviceToHost, stream_), "D2H state");
        hip_ok(hipEventRecord(ev_[slot], stream_), "event");
        ++issued;
        return true;
    };
    auto admitted = [&]() {  // after fill(): the end bound of the slots that just took frames
        for (int f = 0; f < NF; ++f)
            if (slot_frame[f] >= 0 && slot_valid[f] == issued) slot_end[f] = enq + cfg_.max_iterations + 1;
    };
    std::vector<int> all(NF);
    for (int f = 0; f < NF; ++f) all[f] = f;
    fill(all, DevSrc{});
    admitted();
    issue();
    while (finished < nframes) {
        issue();  // keep the next chunk in flight while frames run
        if (!pend.empty()) {  // the solutions copied at the previous check
            hip_ok(hipEventSynchronize(ev_copy_), "mf copy");
            finalize();
            if (finished >= nframes) break;
        }
        if (checked >= issued) throw std::runtime_error("MultiFrameEngine: no chunk in flight and frames unfinished");
        const int c = checked++;
        hip_ok(hipEventSynchronize(ev_[c & 1]), "mf chunk");
        const MfState S = hstate_[c & 1];
        std::vector<int> freed;
        DevSrc best;
        for (int f = 0; f < NF; ++f) {
            const int fr = slot_frame[f];
            if (fr < 0 || c < slot_valid[f] || !S.done[f]) continue;
            const bool rollback = (S.rollback[f >> 6] >> (f & 63)) & 1;
            SolveInfo& info = out[fr];
            info.status = S.status[f] == kSuccess ? kSuccess : kMaxIterationsExceeded;
            info.iterations = S.iters[f];
            info.convergence = S.conv[f];
            info.nonfinite = (S.flags[f >> 6] >> (f & 63)) & 1;
            info.used_fused = false;
            info.warm_from = frame_warm[fr];
            frame_norm[fr] = slot_norm[f];
            const float* src = (rollback ? Xprev_.get() : X_.get()) + (size_t)f * ld_;
            hip_ok(hipMemcpyAsync(hx_ + (size_t)f * ld_, src, V_ * sizeof(float), hipMemcpyDeviceToHost, stream_),
                   "D2H x");
            pend.push_back({fr, f, rollback});
            if (!(info.nonfinite && !rollback) && fr > best.frame) best = DevSrc{fr, f, rollback};
            slot_frame[f] = -1;
            freed.push_back(f);
        }
        if (!freed.empty()) {
            hip_ok(hipEventRecord(ev_copy_, stream_), "event");  // the copies, before the refills' work
            fill(freed, best);
            admitted();
        }
    }
    hip_ok(hipStreamSynchronize(stream_), "mf solve");
    if (comm_stream_) hip_ok(hipStreamSynchronize(comm_stream_), "mf comm");
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto& info : out) info.ms = ms / nframes;
    return out;
}

}  // namespace sart
