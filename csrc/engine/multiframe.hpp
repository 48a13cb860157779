// Native multi-frame engine: up to nf = 16, 32, 64 or 128 independent frames solved together on the matrix cores
// (csrc/kernels/multiframe.hip, multiframe_bf16.hip, multiframe_glue.hip; 128 on the 16-bit paths only). The reference solves a time series strictly
// frame by frame (reference main.cpp:131-140), streaming the RTM twice per iteration per frame; batching
// turns A.x and A^T.w into skinny GEMMs (nf right-hand sides) that reuse every byte of A nf times. Every frame
// keeps its own normalisation, saturation mask, convergence history, status and iteration count; frames
// that finish are frozen while the others continue. Groups are cold-started (like --no_guess), or warm-
// started as a time series: group k + 1 starts from the solution of group k's last frame (the reference's
// frame-to-frame warm start, main.cpp:127-139, applied per group of batch_frames() frames).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
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
    // g: nframes x nrows (host fp64, frame-major); x_out: nframes x nvoxel. batch_frames() slots, refilled with
    // the next frame as soon as a slot's frame finishes (continuous batching). x0 (optional, nvoxel,
    // de-normalised like a solution): start value of the first batch_frames() frames (null: cold). chain: every
    // later frame starts from the solution of the latest frame finished before it (time series; the index is
    // SolveInfo::warm_from); otherwise later frames cold-start.
    std::vector<SolveInfo> solve_batch(const double* g, int nframes, double* x_out, const double* x0 = nullptr,
                                       bool chain = false);
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
    std::vector<SolveInfo> solve_batch_once(const double* g, int nframes, double* x_out, const double* x0, bool chain);
    // frames[q] of g into slots[q] (normalisation, prep, start value, log observed back-projection, state)
    // Start value: warm (host, de-normalised), else dev_src (a finished frame's normalised solution still on
    // the device, normalisation src_norm), else cold.
    void admit(const double* g, const std::vector<int>& slots, const std::vector<int>& frames, const double* warm,
               const float* dev_src, double src_norm, std::vector<double>& slot_norm);
    // last: the batch's final sweep (every running frame reaches max_iter at its decision): forward, ||A x||^2 and
    // the decision only; its back-projection and update would be discarded (reference sartsolver_cuda.cpp:231-262
    // runs max_iter back-projections after the initial guess)
    void sweep(bool last = false);
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
    DeviceArray<double> g64_, G64_, F2part_, x064_;
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
    MfState* hstate_ = nullptr;  // pinned [2]: state after each of the two chunks in flight
    hipEvent_t ev_[2] = {nullptr, nullptr};
    double* hg_ = nullptr;       // pinned [k][rows] staging of the frames entering slots
    float* hx_ = nullptr;        // pinned [nf][ld]: solutions of finished frames, per slot
    hipEvent_t ev_copy_ = nullptr;
    bool skip_last_bwd_ = true;  // SART_MF_LAST_BWD=1: run the final sweep's back-projection anyway (A/B)
    int host_sweep_ = 0;         // sweeps queued in the current solve_batch (EngineConfig::fault_nan_sweep)
    DeviceArray<float> Otmp_;    // log mode: observed back-projection of the frames entering slots
    DeviceArray<float> xsrc_;    // [ld] copy of the finished frame that warm-starts a refill
};

}  // namespace sart
