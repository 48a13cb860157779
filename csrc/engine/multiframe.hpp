// Native multi-frame engine: up to nf = 16, 32, 64 or 128 independent frames solved together on the matrix cores
// (csrc/kernels/multiframe.hip, multiframe_bf16.hip, multiframe_glue.hip; 128 on the 16-bit paths only). The reference solves a time series strictly
// frame by frame (reference main.cpp:131-140), streaming the RTM twice per iteration per frame; batching
// turns A.x and A^T.w into skinny GEMMs (nf right-hand sides) that reuse every byte of A nf times. Every frame
// keeps its own normalisation, saturation mask, convergence history, status and iteration count; frames
// that finish are retired and their slots refilled on the device in the same sweep (solve_series). Frames are
// cold-started (like --no_guess), or warm-started as a time series: each frame starts from the current iterate of
// the newest frame in flight (the reference's frame k-1 -> k warm start, main.cpp:127-139, pipelined: the
// predecessor need not have converged yet).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../kernels/sart_common.hpp"
#include "../native/solver_params.hpp"
#include "comm.hpp"
#include "engine.hpp"

namespace sart {

class MultiFrameEngine {
   public:
    // A: fp32 [nrows_pad][ld], or bf16 when cfg.rtm_bf16 (bf16 MFMA projections, multiframe_bf16.hip); fp32
    // shards run on fp32 MFMA (multiframe.hip) or split into bf16 on the bf16 matrix cores (cfg.mf_split_a)
    // sparse: the shard as device CSR + CSC arrays instead (A null; not owned): fp32 SpMM projections on the
    // frames' fp32 state (csrc/kernels/sparse.hip), no operand splits
    MultiFrameEngine(int device, const void* A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel, int64_t ld,
                     Communicator* comm, const EngineConfig& cfg, const SparseRtm* sparse = nullptr);
    ~MultiFrameEngine();
    MultiFrameEngine(const MultiFrameEngine&) = delete;
    MultiFrameEngine& operator=(const MultiFrameEngine&) = delete;

    void set_laplacian(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t nnz);
    // A series of nframes frames through batch_frames() slots with device-side refill: the sweep in which a frame
    // finishes retires it and admits the next staged frame into its slot (MfQueue, mf_plan in multiframe_glue.hip).
    // src(k, dst): frame k's pixels of this rank (host fp64, nrows) -- asked once per frame in increasing order
    // (again for the frames not delivered yet when a device all-reduce failure makes every rank re-solve them).
    // sink(k, x, info): frame k finished (x: nvoxel, de-normalised); frames finish out of order, each is delivered
    // once. x0 (optional, nvoxel, de-normalised): start value when no chain source exists (chain), or of the first
    // batch_frames() frames (!chain); null: cold. chain (time series): every frame starts from the current iterate
    // of the newest frame in flight or finished (SolveInfo::warm_from / warm_iter), rescaled to its own
    // normalisation; otherwise frames cold-start. Collective over the communicator.
    using FrameSource = std::function<void(int64_t k, double* dst)>;
    using FrameSink = std::function<void(int64_t k, const double* x, const SolveInfo& info)>;
    void solve_series(int64_t nframes, const FrameSource& src, const FrameSink& sink, const double* x0 = nullptr,
                      bool chain = false);
    // g: nframes x nrows (host fp64, frame-major); x_out: nframes x nvoxel: solve_series over an array.
    // starts (optional, nframes x nvoxel): each frame's start value, de-normalised (tests of the chain semantics)
    std::vector<SolveInfo> solve_batch(const double* g, int nframes, double* x_out, const double* x0 = nullptr,
                                       bool chain = false, double* starts = nullptr);
    // counters of the last solve_series (--profile): sweeps the device ran with a frame in some slot, sweeps queued,
    // slot-sweeps spent on frames (sum of sweeps per frame) over nf x sweeps, staged frames, restarts
    struct SeriesStats {
        int64_t frames = 0, sweeps = 0, queued_sweeps = 0, busy_slot_sweeps = 0, chained = 0;
        double slot_util = 0.0, mean_iterations = 0.0, mean_warm_age = 0.0, ms = 0.0;
        // host time of the series thread: waiting for the GPU (chunk / copy events), staging frames (of which in
        // the source callback: reading), delivering finished frames (de-normalisation and the sink)
        double host_wait_ms = 0.0, host_stage_ms = 0.0, host_src_ms = 0.0, host_deliver_ms = 0.0;
        int chunk = 0, admit_cap = 0, src_age = 0, restarts = 0;
        bool src_finished = false, lead = false;
        double src_extrap = 0.0;
        double drift = 0.0;
    };
    const SeriesStats& series_stats() const { return stats_; }
    int64_t nrows() const { return P_; }
    int64_t nvoxel() const { return V_; }
    int batch_frames() const { return nf_; }
    bool split_a() const { return x3_; }  // fp32 shard on the bf16 matrix cores
    bool sparse() const { return sparse_; }
    // the operand pieces of the split-A projections ("f16x2" range-safe f16 pairs, "bf16x2" / "bf16x3" bf16 pieces),
    // "fp32" (fp32 MFMA) or "bf16-storage"
    std::string forward_split() const;
    std::string backproject_split() const;
    // 16, 32, 64 or 128: the smallest batch width that holds `frames` (128 for anything larger; the constructor
    // takes 64 where the path has no 128-column kernels)
    static int batch_width(int frames);

   private:
    // one pass over frames [first, nframes) (frames already delivered are solved again but not re-delivered);
    // true when a device all-reduce failed on some rank (agreed over the host communicator)
    bool series_once(int64_t first, int64_t nframes, const FrameSource& src, const FrameSink& sink, const double* x0,
                     bool chain, std::vector<char>& delivered, int attempt, std::vector<double>& newest,
                     int64_t& newest_frame);
    // queue entries [e0, e0 + k) = frames first + e0 .. (k <= nf): normalisation over all ranks, normalised pixels
    // into the queue (copy stream), cold starts (cold) and the observed back-projection (log) by one batched
    // back-projection, then published to the plan
    void stage(int64_t first, int64_t e0, int k, const FrameSource& src, bool cold);
    // every sweep ends with the decision + refill plan, the update (with retire / start values) and the admitted
    // frames' pixel columns. The final sweep of a frame decided at max_iter skips its back-projection (q->skip_bwd:
    // reference sartsolver_cuda.cpp:231-262 runs max_iter back-projections after the initial guess)
    void sweep();
    void refill();  // the plan, start values and pixel columns without a sweep (the first admissions)
    // chunk_ sweeps: replayed from a HIP graph captured after one eager chunk (one rank, no fault injection;
    // re-captured when the refill buffers change; SART_MF_GRAPH=0: eager launches)
    void run_chunk();
    void drop_graph();
    void set_device() const;
    // F = A X (Fs_ split-K partials); the bf16 engine first writes the X planes
    void forward();
    // part_ = A^T W for voxels [v0, v1) (W in the back-projection layout); the bf16 engine reads the W planes,
    // written from W when split_w
    // have_max: wmax_ already holds the max |w| per frame (the weights kernel of this sweep)
    // sparse shards with `out`: the scaled sums straight into out (oscale[v] * sum, voxel-major [ld][nf]: the
    // collect's D, so the sweep's collect only sums ||A x||^2)
    void backproject(const float* W, bool split_w, int64_t v0, int64_t v1, bool have_max = false,
                     float* out = nullptr, const float* oscale = nullptr);

    int device_;
    const void* A_;
    bool sparse_ = false;
    SparseRtm sp_{};
    DeviceArray<float> Xt_;  // sparse: X voxel-major planes [nf / PW][ld][PW] for the row gathers
    DeviceArray<float> Wt_;  // sparse: W as frame-order planes [nf / PW][rows][PW] (launch_mf_w_planes)
    int pw_ = 64;            // sparse: frames per SpMM plane (mf_sparse_plane_width, fixed at construction)
    bool bf16_ = false;
    bool x3_ = false;     // fp32 shard on the bf16 matrix cores (EngineConfig::mf_split_a)
    bool split_ = false;  // X / W enter as hi + lo bf16 planes (bf16_ || x3_)
    bool xblk_ = false;   // X planes blocked [ld / 32][nf][32] (launch_mf_split_x / forward xblk)
    int64_t P_, Pp_, V_, ld_;
    Communicator* comm_;
    EngineConfig cfg_;
    hipStream_t stream_ = nullptr;
    int nf_ = 16;
    int nsf_ = 1, nsb_ = 1, nwb_ = 1;
    DeviceRaySums rs_;
    DeviceArray<float> X_, Xprev_, Fs_, W_, part_, buf_, pen_, O_, ghat_, arow_, gpos_, wo_;
    DeviceArray<double> G64_, F2part_, x064_;
    DeviceArray<bf16_t> Xh_, Xl_, Wh_, Wl_;  // bf16 / split-A engine: hi / lo operand planes
    // split-A back-projection on f16 pairs (launch_mf_backproject_h16): planes w1 | w2 ([2][nf][Pp] f16 bits),
    // per-frame max scratch and 1 / s_f, and the per-column power-of-two scales of the shard (csc_: [2][ld])
    bool h16_ = false;
    DeviceArray<bf16_t> W16_;
    DeviceArray<unsigned> wmax_;
    DeviceArray<float> wscale_, csc_;
    // split-A forward on f16 pairs (launch_mf_forward_h16, default with split-A; SART_MF_FWD16=0: bf16 hi + lo
    // pieces): X planes in Xh_ / Xl_ (f16 bits), per-row scales of the shard (rsc_: [2][Pp]), per-frame 1 / s_f
    bool fwd16_ = false;
    DeviceArray<float> rsc_, xinv_;
    DeviceArray<unsigned> xmax_;
    DeviceArray<MfState> st_;
    DeviceArray<int64_t> lap_rp_;
    DeviceArray<int32_t> lap_col_;
    DeviceArray<float> lap_val_;
    bool has_lap_ = false;
    // overlapped back-projection / all-reduce (several ranks): voxel chunk bounds, comm stream, events
    std::vector<int64_t> chunks_;
    hipStream_t comm_stream_ = nullptr;
    std::vector<hipEvent_t> cev_;
    hipEvent_t comm_done_ = nullptr;
    // device refill: queue (normalised pixels ghq_ [qcap][Pp], cold starts x0q_ / observed back-projections oq_
    // [qcap][ld] when staged), output ring ring_ [rcap][ld], xlast_ [ld], and the plan state q_
    int qcap_ = 32, rcap_ = 32, chunk_ = 4, admit_cap_ = 0, src_age_ = 0;
    bool src_finished_ = false, lead_ = true;
    hipGraphExec_t graph_ = nullptr;
    MfRefill graph_rf_{};
    int graph_chunk_ = 0;
    bool use_graph_ = true, graph_failed_ = false, warm_chunk_ = false;
    double src_extrap_ = 0.0;
    double drift_ = 0.0;  // drift-extrapolated chain starts (MfQueue::drift; SART_MF_DRIFT)
    DeviceArray<MfQueue> q_;
    DeviceArray<float> ghq_, x0q_, oq_, ring_, xlast_, xlast2_, starts_;
    MfRefill rf_{};
    std::vector<double> frame_norm_;  // the last series' normalisation per frame (solve_batch's starts)
    struct Snap {
        MfState st;
        MfQueue q;
    };
    Snap* hsnap_ = nullptr;      // pinned [2]: state after each of the two chunks in flight
    hipEvent_t ev_[2] = {nullptr, nullptr};
    double* hg64_ = nullptr;     // pinned [qcap][Pp]: the queue's raw pixels (the source writes them here; H2D source)
    DeviceArray<double> g64q_, sstats_;  // device copy [qcap][Pp]; per-frame max / sum of squares [2][nf]
    float* hx_ = nullptr;        // pinned [rcap][ld]: solutions of finished frames (D2H target)
    hipStream_t copy_stream_ = nullptr;
    hipEvent_t ev_copy_ = nullptr, ev_stage_ = nullptr;
    bool skip_last_bwd_ = true;  // SART_MF_LAST_BWD=1: run the final sweep's back-projection anyway (A/B)
    int host_sweep_ = 0;         // sweeps queued in the current series (EngineConfig::fault_nan_sweep)
    SeriesStats stats_;
};

}  // namespace sart
