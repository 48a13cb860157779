#include "multiframe.hpp"

#include <algorithm>
#include <exception>
#include <mutex>
#include <deque>
#include <condition_variable>
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
double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
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
    hip_ok(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking), "hipStreamCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hsnap_), 2 * sizeof(Snap)), "hipHostMalloc");
    for (auto& e : ev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventCreateWithFlags(&ev_copy_, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventCreateWithFlags(&ev_stage_, hipEventDisableTiming), "hipEventCreate");
    // device refill: a queue and an output ring of 2 nf entries each (staging and draining run a chunk behind the
    // sweeps, ~nf frames finish per chunk at ~8 sweeps per frame); sweeps per host check (SART_MF_CHUNK, default
    // min(check_interval, 4): the host check no longer gates a refill, only the staging and the drain)
    // queue and output ring: 4 nf entries (at most 256), down to 2 nf where their pinned host rows (fp64 pixels /
    // fp32 voxels) would pass 1 GiB
    qcap_ = rcap_ = std::min(kMfQueueMax, 4 * NF);
    while (qcap_ > 2 * NF && (double)qcap_ * Pp_ * 8 > 1073741824.0) qcap_ /= 2;
    while (rcap_ > 2 * NF && (double)rcap_ * ld_ * 4 > 1073741824.0) rcap_ /= 2;
    {  // sweeps per chunk: ~1.5 ms of estimated sweep time (dense: two reads of A at ~5 TB/s; sparse: two gathers over
       // the entries; plus ~13 launches), at least min(check_interval, 4): the host's per-chunk work (snapshot,
       // drain, staging) must hide behind the chunk in flight when sweeps are short (sparse shards)
        const double bytes = sparse ? 2.0 * (double)sparse->nnz * 8.0 : 2.0 * (double)Pp_ * ld_ * (bf16_ ? 2 : 4);
        const double t_sweep = bytes / 5e12 + 13 * 4e-6;
        chunk_ = (int)std::min<double>(32, std::max<double>(std::min(cfg_.check_interval, 4), std::ceil(1.5e-3 / t_sweep)));
    }
    if (const char* e = std::getenv("SART_MF_CHUNK"); e && *e) chunk_ = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("SART_MF_GRAPH"); e && *e) use_graph_ = std::atoi(e) != 0;
    // admissions per sweep of a time series (SART_MF_ADMIT_CAP; 0: any): a frame admitted together with others
    // starts from the same source iterate, so a burst of admissions starts frames far from their predecessors
    admit_cap_ = std::max(1, NF / 4);
    if (const char* e = std::getenv("SART_MF_ADMIT_CAP"); e && *e) admit_cap_ = std::max(0, std::atoi(e));
    // chain sources: the newest frame with at least 3 updates, extrapolated along its last update by 4 x (linear mode):
    // a young iterate's slowest modes decay by ~rho = 0.86 per sweep on the 64k ray-traced series, so x + c (x - x_prev)
    // with c ~ rho / (1 - rho) removes most of the error it would pass on, once its fast modes are gone (>= 3 updates).
    // Measured there at 64 frames: 27.8 -> 22.9 iterations per frame, 253 -> 290 frames/s
    // (profiles/series_r6_raytraced_64k_refill_policies*.jsonl; SART_MF_SRC_AGE / SART_MF_SRC_EXTRAP override)
    src_age_ = 3;
    src_extrap_ = 4.0;
    if (const char* e = std::getenv("SART_MF_SRC_AGE"); e && *e) src_age_ = std::max(0, std::atoi(e));
    // A/B knobs of the chain: SART_MF_SRC_FINISHED=1 (sources: finished frames only), SART_MF_LEAD=0 (no lead frame)
    if (const char* e = std::getenv("SART_MF_SRC_FINISHED"); e && *e) src_finished_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SART_MF_LEAD"); e && *e) lead_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SART_MF_SRC_EXTRAP"); e && *e) src_extrap_ = std::atof(e);
    // drift across the frame gap (linear mode): a source is >= src_age sweeps old, so frames newer than it are already
    // in flight and an admitted frame sits several frames of drift away from its source; the start adds that many
    // times the per-frame change between the two newest finished solutions (MfQueue::drift; SART_MF_DRIFT)
    if (const char* e = std::getenv("SART_MF_DRIFT"); e && *e) drift_ = std::atof(e);
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hg64_), (size_t)qcap_ * Pp_ * sizeof(double)), "hipHostMalloc");
    std::memset(hg64_, 0, (size_t)qcap_ * Pp_ * sizeof(double));  // padding rows stay zero
    g64q_.resize((size_t)qcap_ * Pp_);
    sstats_.resize((size_t)2 * NF);
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&hx_), (size_t)rcap_ * ld_ * sizeof(float)), "hipHostMalloc");
    q_.resize(1);
    ghq_.resize((size_t)qcap_ * Pp_);
    ring_.resize((size_t)rcap_ * ld_);
    xlast_.resize(ld_);
    xlast2_.resize(ld_);
    if (cfg_.logarithmic) oq_.resize((size_t)qcap_ * ld_);
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
    drop_graph();
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (comm_stream_) (void)hipStreamSynchronize(comm_stream_);
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : cev_)
        if (e) (void)hipEventDestroy(e);
    if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
    if (comm_done_) (void)hipEventDestroy(comm_done_);
    if (comm_stream_) (void)hipStreamDestroy(comm_stream_);
    if (hsnap_) (void)hipHostFree(hsnap_);
    if (hg64_) (void)hipHostFree(hg64_);
    if (hx_) (void)hipHostFree(hx_);
    if (ev_copy_) (void)hipEventDestroy(ev_copy_);
    if (ev_stage_) (void)hipEventDestroy(ev_stage_);
    if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
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

void MultiFrameEngine::sweep() {
    const int NF = nf_;
    MfState* st = st_.get();
    MfQueue* q = q_.get();
    const MfSkipScope skip(&st->all_done);  // every slot done: the sweep's heavy kernels return at once
    // the back-projection (and its operand split) also returns when every running frame is decided at max_iter in
    // this sweep (mf_plan's skip_bwd): its corrections would be discarded; the collect still sums ||A x||^2
    const int* bskip = skip_last_bwd_ ? &q->skip_bwd : &st->all_done;
    float* D = buf_.get();                     // [ld][nf] voxel-major corrections
    float* F2 = buf_.get() + (int64_t)NF * ld_;  // [nf] ||A x||^2, all-reduced with the last chunk
    const float* scale = cfg_.logarithmic ? rs_.dmask.get() : rs_.dscale.get();
    forward();
    // f16-pair back-projection: the weights kernel also leaves each frame's max |w| (its f16 scale) in wmax_
    launch_mf_weights(Fs_.get(), nsf_, Pp_, ghat_.get(), arow_.get(), cfg_.logarithmic, W_.get(), F2part_.get(),
                      NF, stream_, h16_ ? wmax_.get() : nullptr,
                      sparse_ && mf_sparse_needs_w_planes(NF, pw_) ? pw_ : 0);
    // D[v0, v1) = scale * A^T W and, with the last chunk, the per-frame ||A x||^2: a sparse shard's SpMM writes the
    // scaled sums itself (the collect then only sums F2part)
    auto bwd_collect = [&](int64_t v0, int64_t v1, bool first, bool lastc) {
        if (sparse_) {
            {
                const MfSkipScope sb(bskip);
                backproject(W_.get(), first, v0, v1, true, D, scale);
            }
            if (lastc) launch_mf_collect(part_.get(), nsb_, ld_, 0, 0, scale, D, F2part_.get(), nwb_, F2, NF, stream_);
            return;
        }
        {
            const MfSkipScope sb(bskip);
            backproject(W_.get(), first, v0, v1, true);
        }
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
    launch_mf_decide(st, F2, stream_, q);
    launch_mf_update(X_.get(), D, O_.get(), pen, (float)cfg_.relaxation, cfg_.logarithmic, V_, ld_, st, NF, stream_,
                     Xprev_.get(), q, &rf_);
    launch_mf_admit_rows(q, ghq_.get(), P_, Pp_, rs_.ray_len.get(), (float)cfg_.ray_length_threshold, ghat_.get(),
                         arow_.get(), NF, stream_);
    if (cfg_.fault_nan_sweep >= 0 && host_sweep_ == cfg_.fault_nan_sweep)  // fault injection (tests): slot 0
        hip_ok(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(X_.get()), 0x7fc00000, 1, stream_), "inject NaN");
    ++host_sweep_;
}

void MultiFrameEngine::drop_graph() {
    if (graph_) (void)hipGraphExecDestroy(graph_);
    graph_ = nullptr;
}

void MultiFrameEngine::run_chunk() {
    RoctxRange r("sart::mf_chunk");
    // capture only after an eager chunk with the current kernels (launchers may set function attributes on first
    // use, which must not happen inside a capture); the captured update kernel holds rf_ by value
    const bool graphable = use_graph_ && !graph_failed_ && warm_chunk_ && comm_->size() == 1 &&
                           comm_->graph_capturable() && cfg_.fault_nan_sweep < 0;
    if (graph_ && (!graphable || graph_chunk_ != chunk_ || std::memcmp(&graph_rf_, &rf_, sizeof(rf_)) != 0))
        drop_graph();
    if (graphable && !graph_) {
        hipGraph_t g = nullptr;
        bool ok = hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) == hipSuccess;
        if (ok) {
            try {
                for (int i = 0; i < chunk_; ++i) sweep();
            } catch (...) {
                ok = false;
            }
            ok = (hipStreamEndCapture(stream_, &g) == hipSuccess) && ok && g;
        }
        if (ok) ok = hipGraphInstantiate(&graph_, g, nullptr, nullptr, 0) == hipSuccess;
        if (g) (void)hipGraphDestroy(g);
        if (!ok) {  // eager launches from now on (the capture queued nothing)
            (void)hipGetLastError();
            graph_ = nullptr;
            graph_failed_ = true;
        } else {
            graph_rf_ = rf_;
            graph_chunk_ = chunk_;
        }
    }
    if (graphable && graph_) {
        hip_ok(hipGraphLaunch(graph_, stream_), "hipGraphLaunch");
        host_sweep_ += chunk_;
    } else {
        for (int i = 0; i < chunk_; ++i) sweep();
        warm_chunk_ = true;
    }
}

void MultiFrameEngine::refill() {
    const int NF = nf_;
    float* D = buf_.get();
    launch_mf_decide(st_.get(), D + (int64_t)NF * ld_, stream_, q_.get());  // every slot done: the plan only
    launch_mf_update(X_.get(), D, O_.get(), nullptr, (float)cfg_.relaxation, cfg_.logarithmic, V_, ld_, st_.get(), NF,
                     stream_, Xprev_.get(), q_.get(), &rf_);
    launch_mf_admit_rows(q_.get(), ghq_.get(), P_, Pp_, rs_.ray_len.get(), (float)cfg_.ray_length_threshold,
                         ghat_.get(), arow_.get(), NF, stream_);
}

void MultiFrameEngine::stage(int64_t first, int64_t e0, int k, const FrameSource& src, bool cold) {
    const int NF = nf_;
    if (k <= 0) return;
    if (k > NF) throw std::logic_error("MultiFrameEngine::stage: at most nf frames per call");
    RoctxRange r("sart::mf_stage");
    // the frames' raw pixels straight into the pinned queue rows, then to the device on the copy stream (one or two
    // runs of ring positions), next to the sweeps; normalisation and scalars on the device (k_mf_stage_*)
    const auto ts = std::chrono::steady_clock::now();
    for (int j = 0; j < k; ++j) src(first + e0 + j, hg64_ + (size_t)((e0 + j) % qcap_) * Pp_);
    stats_.host_src_ms += ms_since(ts);
    for (int j = 0; j < k;) {
        const int pos = (int)((e0 + j) % qcap_);
        const int run = std::min(k - j, qcap_ - pos);
        if (P_)
            hip_ok(hipMemcpyAsync(g64q_.get() + (size_t)pos * Pp_, hg64_ + (size_t)pos * Pp_,
                                  (size_t)run * Pp_ * sizeof(double), hipMemcpyHostToDevice, copy_stream_),
                   "H2D queue");
        j += run;
    }
    hip_ok(hipEventRecord(ev_stage_, copy_stream_), "event");
    hip_ok(hipStreamWaitEvent(stream_, ev_stage_, 0), "wait staging");
    // per-frame maxima and positive sums of squares over all ranks' pixels (reference sartsolver_cuda.cpp:146-157)
    launch_mf_stage_stats(g64q_.get(), e0, qcap_, k, P_, Pp_, sstats_.get(), NF, stream_);
    if (comm_->size() > 1) {
        comm_->all_reduce(sstats_.get(), (size_t)k, ReduceOp::kMax, stream_);
        comm_->all_reduce(sstats_.get() + NF, (size_t)k, ReduceOp::kSum, stream_);
    }
    launch_mf_stage_norm(q_.get(), g64q_.get(), ghq_.get(), sstats_.get(), e0, first + e0, cold, k, P_, Pp_, NF, stream_);
    if (cold || cfg_.logarithmic) {
        // one batched back-projection of the k staged frames (columns 0 .. k - 1): cold starts
        // x0 = max([rho > tau] A^T max(ghat, 0) / rho, 1e-7) (reference sart_kernels.cu:22-60) and / or the
        // frame-constant observed back-projection O = mask A^T (a ghat) of log mode
        const float thr = (float)cfg_.ray_length_threshold;
        launch_mf_stage_ops(ghq_.get(), e0, qcap_, k, P_, Pp_, rs_.ray_len.get(), thr, gpos_.get(),
                            cfg_.logarithmic ? wo_.get() : nullptr, NF, stream_);
        if (cold) {
            backproject(gpos_.get(), true, 0, ld_);
            launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, nullptr, buf_.get(), nullptr, 0, nullptr, NF, stream_);
            if (comm_->size() > 1) comm_->all_reduce(buf_.get(), (size_t)NF * ld_, ReduceOp::kSum, stream_);
            launch_mf_stage_cols(buf_.get(), rs_.dinv.get(), e0, qcap_, k, V_, ld_, NF, x0q_.get(), stream_);
        }
        if (cfg_.logarithmic) {
            backproject(wo_.get(), true, 0, ld_);
            launch_mf_collect(part_.get(), nsb_, ld_, 0, ld_, rs_.dmask.get(), buf_.get(), nullptr, 0, nullptr, NF,
                              stream_);
            if (comm_->size() > 1) comm_->all_reduce(buf_.get(), (size_t)NF * ld_, ReduceOp::kSum, stream_);
            launch_mf_stage_cols(buf_.get(), nullptr, e0, qcap_, k, V_, ld_, NF, oq_.get(), stream_);
        }
    }
    launch_mf_publish(q_.get(), e0 + k, stream_);
}

std::vector<SolveInfo> MultiFrameEngine::solve_batch(const double* g, int nframes, double* x_out, const double* x0,
                                                     bool chain, double* starts) {
    std::vector<SolveInfo> out(std::max(nframes, 0));
    if (nframes <= 0) return out;
    const auto t0 = std::chrono::steady_clock::now();
    if (starts) {  // the start value of every frame (normalised on the device; de-normalised below)
        set_device();
        starts_.resize((size_t)nframes * ld_);
        rf_.starts = starts_.get();
    }
    try {
        solve_series(
            nframes, [&](int64_t k, double* dst) { std::memcpy(dst, g + k * P_, (size_t)P_ * sizeof(double)); },
            [&](int64_t k, const double* x, const SolveInfo& info) {
                std::memcpy(x_out + k * V_, x, (size_t)V_ * sizeof(double));
                out[k] = info;
            },
            x0, chain);
    } catch (...) {
        rf_.starts = nullptr;
        throw;
    }
    if (starts) {
        rf_.starts = nullptr;
        std::vector<float> h((size_t)nframes * ld_);
        hip_ok(hipMemcpy(h.data(), starts_.get(), h.size() * sizeof(float), hipMemcpyDeviceToHost), "D2H starts");
        for (int k = 0; k < nframes; ++k)
            for (int64_t v = 0; v < V_; ++v)
                starts[(size_t)k * V_ + v] = (double)h[(size_t)k * ld_ + v] * frame_norm_[k];
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto& info : out) info.ms = ms / nframes;
    return out;
}

void MultiFrameEngine::solve_series(int64_t nframes, const FrameSource& src, const FrameSink& sink, const double* x0,
                                    bool chain) {
    set_device();
    RoctxRange range("sart::mf_series");
    stats_ = SeriesStats{};
    if (nframes <= 0) return;
    if (nframes > std::numeric_limits<int32_t>::max()) throw std::invalid_argument("solve_series: too many frames");
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<char> delivered((size_t)nframes, 0);
    frame_norm_.assign((size_t)nframes, 1.0);
    std::vector<double> newest;  // the newest delivered finite solution (a re-solve's chain start)
    int64_t newest_frame = -1;
    int64_t first = 0;
    for (int attempt = 0;; ++attempt) {
        const bool failed = series_once(first, nframes, src, sink, attempt == 0 ? x0 : (newest_frame >= 0 && chain ? newest.data() : x0),
                                        chain, delivered, attempt, newest, newest_frame);
        if (!failed) break;
        const bool had = comm_->degrade();
        if (comm_->rank() == 0)
            std::fprintf(stderr, "sart: device all-reduce timed out; re-solving the undelivered frames on %s\n",
                         comm_->backend());
        if (!had || attempt >= 1) throw std::runtime_error("MultiFrameEngine: device all-reduce failed");
        ++stats_.restarts;
        while (first < nframes && delivered[first]) ++first;
    }
    comm_->check();
    stats_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

bool MultiFrameEngine::series_once(int64_t first, int64_t nframes, const FrameSource& src, const FrameSink& sink,
                                   const double* x0, bool chain, std::vector<char>& delivered, int attempt,
                                   std::vector<double>& newest, int64_t& newest_frame) {
    const int NF = nf_;
    const int64_t n = nframes - first;  // frames of this pass: queue entry e = frame first + e
    host_sweep_ = 0;
    // cold starts are staged for every frame without --chain, and for the first nf frames of a chain without x0
    // (later ones start from a frame in flight)
    const bool any_cold = !(chain && x0);
    if (any_cold && x0q_.size() == 0) x0q_.resize((size_t)qcap_ * ld_);
    if ((int64_t)x064_.size() < V_) x064_.resize(std::max<int64_t>(V_, 1));
    rf_.ring = ring_.get();
    rf_.xlast = xlast_.get();
    rf_.xlast2 = xlast2_.get();
    rf_.x0 = x064_.get();
    rf_.x0q = x0q_.size() ? x0q_.get() : nullptr;
    rf_.oq = oq_.size() ? oq_.get() : nullptr;
    // every slot starts empty (done) with finite zero columns
    for (auto* b : {&X_, &Xprev_, &ghat_, &arow_})
        hip_ok(hipMemsetAsync(b->get(), 0, b->size() * sizeof(float), stream_), "memset");
    if (cfg_.logarithmic) hip_ok(hipMemsetAsync(O_.get(), 0, O_.size() * sizeof(float), stream_), "memset");
    hip_ok(hipMemsetAsync(G64_.get(), 0, G64_.size() * sizeof(double), stream_), "memset");
    launch_mf_state_begin(st_.get(), G64_.get(), 0, cfg_.conv_tolerance, cfg_.max_iterations, NF, stream_);
    const int64_t x0_below = x0 ? (chain ? std::numeric_limits<int64_t>::max() : first + NF) : 0;
    launch_mf_queue_begin(q_.get(), qcap_, rcap_, chain, chain ? admit_cap_ : 0, src_age_, x0_below, src_finished_,
                          chain && !x0 && lead_, (float)src_extrap_, stream_, chain ? (float)drift_ : 0.f);
    if (x0 && V_) hip_ok(hipMemcpyAsync(x064_.get(), x0, V_ * sizeof(double), hipMemcpyHostToDevice, stream_), "H2D x0");
    stats_.chunk = chunk_;
    stats_.admit_cap = chain ? admit_cap_ : 0;
    stats_.src_age = src_age_;
    stats_.src_finished = src_finished_;
    stats_.src_extrap = src_extrap_;
    stats_.drift = chain ? drift_ : 0.0;
    stats_.lead = chain && !x0 && lead_;

    int64_t staged = 0;
    // stage while the queue has room for a unit (nf with a back-projection), up to `limit` frames
    auto stage_upto = [&](int64_t head, int64_t limit) {
        while (staged < std::min(n, limit)) {
            // the first nf frames start from x0 (or cold without it); later ones cold (!chain) or chained
            const bool cold = chain ? (!x0 && staged < NF) : (!x0 || staged >= NF);
            const int64_t lim = staged < NF ? NF - staged : NF;  // no unit straddles frame nf
            const int64_t room = qcap_ - (staged - head);
            const int64_t unit = (cold || cfg_.logarithmic) ? std::min<int64_t>(lim, n - staged)
                                                            : std::max<int64_t>(1, std::min<int64_t>(NF / 4, n - staged));
            if (room < unit) return;
            const int k = (int)std::min<int64_t>({room, lim, n - staged});
            const auto ts = std::chrono::steady_clock::now();
            stage(first, staged, k, src, cold);
            stats_.host_stage_ms += ms_since(ts);
            staged += k;
        }
    };
    stage_upto(0, NF);  // the first nf frames: the first chunk starts as soon as they are read; the rest next to it
    refill();

    int issued = 0, checked = 0;
    auto issue = [&]() {
        run_chunk();
        const int slot = issued & 1;
        hip_ok(hipMemcpyAsync(&hsnap_[slot].st, st_.get(), sizeof(MfState), hipMemcpyDeviceToHost, stream_), "D2H state");
        hip_ok(hipMemcpyAsync(&hsnap_[slot].q, q_.get(), sizeof(MfQueue), hipMemcpyDeviceToHost, stream_), "D2H queue");
        hip_ok(hipEventRecord(ev_[slot], stream_), "event");
        ++issued;
    };
    struct Pending {
        MfFinish log;
        int pos;
    };
    // Delivery thread: finished frames are de-normalised and handed to the sink (the driver's writer) next to the
    // series thread, which only issues chunks, stages frames and queues the output-ring copies (at ~2000 sparse
    // frames/s the sink alone took a third of the series thread's time, profiles/series_r6_sparse*).
    struct Batch {
        hipEvent_t ev;  // the batch's copies into hx_
        std::vector<Pending> items;
    };
    std::mutex dm;
    std::condition_variable dcv;
    std::deque<Batch> dq;
    bool dstop = false;
    std::exception_ptr derr;
    int64_t dcount = 0, warm_age = 0;  // entries delivered (FIFO: entries [0, dcount) are done with hx_)
    std::thread deliver([&] {
        try {
            hip_ok(hipSetDevice(device_), "hipSetDevice");
            std::vector<double> x(std::max<int64_t>(V_, 1));
            for (;;) {
                Batch b;
                {
                    std::unique_lock<std::mutex> lk(dm);
                    dcv.wait(lk, [&] { return dstop || !dq.empty(); });
                    if (dq.empty()) return;
                    b = std::move(dq.front());
                    dq.pop_front();
                }
                const auto tw = std::chrono::steady_clock::now();
                const hipError_t se = hipEventSynchronize(b.ev);
                (void)hipEventDestroy(b.ev);
                hip_ok(se, "mf copy");
                for (const Pending& pd : b.items) {
                    const MfFinish& L = pd.log;
                    const float* hs = hx_ + (size_t)pd.pos * ld_;
                    for (int64_t v = 0; v < V_; ++v) x[v] = (double)hs[v] * L.norm;
                    stats_.busy_slot_sweeps += L.iters + 1;
                    stats_.mean_iterations += L.iters;
                    if (L.warm_from >= 0) ++stats_.chained, warm_age += (L.frame - L.warm_from);
                    if (L.frame < 0 || L.frame >= nframes || delivered[L.frame]) continue;
                    SolveInfo info;
                    info.status = L.status;
                    info.iterations = L.iters;
                    info.convergence = L.conv;
                    info.nonfinite = (L.flags & 1) != 0;
                    info.used_fused = false;
                    info.warm_from = L.warm_from;
                    info.warm_iter = L.warm_iter;
                    info.warm_live = L.warm_live != 0;
                    info.comm_fallbacks = attempt;
                    info.comm = comm_->backend();
                    info.sweeps = L.iters + 1;
                    frame_norm_[L.frame] = L.norm;
                    delivered[L.frame] = 1;
                    sink(L.frame, x.data(), info);
                    if (L.frame > newest_frame && !info.nonfinite) {
                        newest.assign(x.begin(), x.begin() + V_);
                        newest_frame = L.frame;
                    }
                }
                stats_.host_deliver_ms += ms_since(tw);
                std::lock_guard<std::mutex> lk(dm);
                dcount += (int64_t)b.items.size();
                dcv.notify_all();
            }
        } catch (...) {
            std::lock_guard<std::mutex> lk(dm);
            derr = std::current_exception();
            dcv.notify_all();
        }
    });
    struct JoinDelivery {  // also on an exception of the series thread (a source that throws, a HIP error)
        std::thread& t;
        std::mutex& m;
        std::condition_variable& cv;
        bool& stop;
        std::deque<Batch>& q;
        ~JoinDelivery() {
            {
                std::lock_guard<std::mutex> lk(m);
                stop = true;
            }
            cv.notify_all();
            if (t.joinable()) t.join();
            for (Batch& b : q) (void)hipEventDestroy(b.ev);
        }
    } join_delivery{deliver, dm, dcv, dstop, dq};
    auto check_delivery = [&]() {
        std::lock_guard<std::mutex> lk(dm);
        if (derr) std::rethrow_exception(derr);
    };
    issue();
    stage_upto(0, n);
    issue();
    bool failed = false;
    int64_t seen_fin = 0;
    while (seen_fin < n) {
        check_delivery();
        if (checked >= issued) throw std::runtime_error("MultiFrameEngine: no chunk in flight and frames unfinished");
        const int c = checked++;
        const auto tw = std::chrono::steady_clock::now();
        hip_ok(hipEventSynchronize(ev_[c & 1]), "mf chunk");
        stats_.host_wait_ms += ms_since(tw);
        const MfQueue& Q = hsnap_[c & 1].q;
        const int64_t fin = Q.fin, head = Q.q_head;
        std::vector<Pending> fresh;
        for (int64_t e = seen_fin; e < fin; ++e) {
            const int pos = (int)(e % rcap_);
            fresh.push_back({Q.log[pos], pos});
        }
        if (device_comm_failed_anywhere(comm_)) {  // collective: every rank sees the same device state
            failed = true;
            break;
        }
        if (!fresh.empty()) {
            {  // hx_ position of entry e is free once entry e - rcap has been delivered
                const auto tw2 = std::chrono::steady_clock::now();
                std::unique_lock<std::mutex> lk(dm);
                dcv.wait(lk, [&] { return derr || fin - 1 - rcap_ < dcount; });
                if (derr) std::rethrow_exception(derr);
                stats_.host_wait_ms += ms_since(tw2);
            }
            // solutions from the output ring on the copy stream (the chunk that wrote them has completed: its
            // snapshot was read), next to the sweeps; the ring positions are free again once the copies are done
            for (const Pending& pd : fresh)
                hip_ok(hipMemcpyAsync(hx_ + (size_t)pd.pos * ld_, ring_.get() + (size_t)pd.pos * ld_,
                                      V_ * sizeof(float), hipMemcpyDeviceToHost, copy_stream_),
                       "D2H x");
            seen_fin = fin;
            Batch b;
            hip_ok(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming), "hipEventCreate");
            hip_ok(hipEventRecord(b.ev, copy_stream_), "event");
            hip_ok(hipStreamWaitEvent(stream_, b.ev, 0), "wait ring copies");
            launch_mf_drained(q_.get(), seen_fin, stream_);
            b.items = std::move(fresh);
            std::lock_guard<std::mutex> lk(dm);
            dq.push_back(std::move(b));
            dcv.notify_all();
        }
        stage_upto(head, n);
        if (fin < n) issue();  // frames left to finish on the device (a chunk still in flight may finish them)
    }
    {  // every handed-over frame delivered (or the delivery failed)
        std::unique_lock<std::mutex> lk(dm);
        dcv.wait(lk, [&] { return derr || dcount >= seen_fin; });
    }
    check_delivery();
    hip_ok(hipStreamSynchronize(stream_), "mf series");
    if (comm_stream_) hip_ok(hipStreamSynchronize(comm_stream_), "mf comm");
    hip_ok(hipStreamSynchronize(copy_stream_), "mf copy stream");
    if (!failed) {
        const MfState& S = hsnap_[(issued - 1) & 1].st;
        const int64_t finished = dcount;
        stats_.sweeps = S.sweep;
        stats_.queued_sweeps = (int64_t)issued * chunk_;
        stats_.frames = finished;
        if (finished) stats_.mean_iterations /= finished;
        if (stats_.chained) stats_.mean_warm_age = (double)warm_age / stats_.chained;
        if (stats_.sweeps > 0) stats_.slot_util = (double)stats_.busy_slot_sweeps / ((double)stats_.sweeps * NF);
    }
    return failed;
}

}  // namespace sart
