// Native per-GPU SART engine: owns the device workspaces of one rank's solver and
// runs whole frame solves in C++ -- ray sums, frame setup, the sweep loop (fused single-pass sweep with
// the v6 -> v3 -> two-pass fallback chain, or the two-pass kernels), the per-iteration all-reduce and the
// device-side convergence decision -- without Python in the loop.
//
// Reference parity: BaseSARTSolverMPICuda / SARTSolverMPICuda / LogSARTSolverMPICuda
// (reference sartsolver_cuda.cpp:78-354, ray sums sartsolver.cpp:20-58, parameter checks :61-123);
// iteration semantics in mpi_cuda_sartsolver_amd/models/sart.py.
//
// MI355X specifics: every buffer is allocated once per engine (the reference mallocs 5 buffers per
// frame, sartsolver_cuda.cpp:160-191); the host reads the 128-byte SartState once per chunk of
// `check_interval` sweeps, with the next chunk already queued, so the GPU never drains between chunks;
// a chunk is captured once into a HIP graph and replayed (local and RCCL communicators).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../kernels/launchers.hpp"
#include "../kernels/sart_common.hpp"
#include "../native/solver_params.hpp"
#include "comm.hpp"
#include "geometry.hpp"

namespace sart {

struct EngineConfig : SolverParams {
    int check_interval = 16;
    bool use_fused = true;
    int fused_variant = 6;
    int rows_per_tile = 0;   // 0: default (fused_geometry)
    int fused_schedule = -1; // -1: keep the launcher's default
    // Opt-in (SART_GRAPH=1): bitwise equal to eager chunks (tests/test_gpu_solver.py), but measured no
    // faster for the two-pass kernels and 13-28 % slower for the fused sweep at 8k x 16k and 16k x 64k
    // (profiles/graph_check_r1.jsonl): launches are already hidden behind the queued chunk.
    bool use_graph = false;
    // The fused sweep is used only for shards of at least this many bytes (the drivers pass 128 MiB:
    // below ~100 MB the two-pass kernels are faster, e.g. 40.6 vs 60.2 us per iteration at 2048 x 4096).
    double fused_min_bytes = 0;
    // Fault injection (tests; env SART_FAULT_INJECT=N): report a persistent-sweep protocol timeout in the
    // first N solves, exercising the v6 -> v3 -> two-pass fallback chain end to end.
    int fault_inject = 0;
    // Fault injection (tests; env SART_FAULT_NAN=k): write NaN into x after sweep k of every solve (eager
    // chunks), exercising the NaN/Inf guard's rollback to the last finite iterate. -1: off.
    int fault_nan_sweep = -1;
    // Multi-frame engine: frames per batch (16, 32, 64 or 128; MultiFrameEngine rounds other values up).
    int mf_frames = 16;
    // Column (voxel) shard instead of the reference's row (pixel) shard: this rank holds ALL
    // pixel rows for voxels [col_offset, col_offset + nvoxel) of nvoxel_total, and gets the full
    // measurement. Per sweep the partial forward projections (a pixel vector) are all-reduced instead of
    // the corrections (a voxel vector); the back-projection and the update are local. Two-pass kernels
    // only (the fused sweep needs complete row dots on one GPU). With a Laplacian, x is all-gathered
    // every sweep for the penalty of the local rows.
    bool column_shard = false;
    int64_t col_offset = 0;
    int64_t nvoxel_total = 0;  // 0: nvoxel
    // Observability: bracket every per-sweep all-reduce with timing events and report the GPU
    // time spent in collectives (SolveInfo::comm_ms). Eager chunks only (ignored with use_graph).
    bool time_collectives = false;
    // Storage precision of the shard: A holds bf16 bit patterns instead of fp32 (half the
    // HBM bytes per sweep, twice the matrix per GPU); products, sums and every vector stay fp32 / fp64. Ray
    // sums are taken over the stored (rounded) values, so the solve is exact SART for the bf16 matrix.
    // Fused sweep variant 6 (bf16 register tiles, fp32 LDS ring), the two-pass kernels, or the bf16 MFMA
    // multi-frame kernels.
    bool rtm_bf16 = false;
    // Multi-frame engine with an fp32 shard: run the projections on the bf16 matrix cores with A split into
    // hi + lo bf16 in registers (three products per element; multiframe_bf16.hip, "split-A") instead of fp32
    // MFMA. 1: on, 0: off, -1: env SART_MF_X3 (0 / 1), else on for batches of 32 and 64 frames (where fp32
    // MFMA bounds the sweep; at 16 frames both paths are HBM-bound).
    int mf_split_a = -1;
    // Fused sweep: plan the persistent grid for at most this many CUs (0: all; env SART_FUSED_CUS). Ranks that
    // share a GPU (SART_FUSED_SHARED=1) plan for num_cus / (ranks per GPU) each.
    int fused_max_cus = 0;
};

// roctx range (rocprofv3 --marker-trace) for the lifetime of the object.
struct RoctxRange {
    explicit RoctxRange(const char* name);
    ~RoctxRange();
};

template <typename T>
class DeviceArray {
   public:
    DeviceArray() = default;
    explicit DeviceArray(size_t n) { resize(n); }
    ~DeviceArray() { release(); }
    DeviceArray(const DeviceArray&) = delete;
    DeviceArray& operator=(const DeviceArray&) = delete;
    void resize(size_t n);  // zero-filled
    void release();
    T* get() const { return p_; }
    size_t size() const { return n_; }

   private:
    T* p_ = nullptr;
    size_t n_ = 0;
};

// Column / row sums of the shard and the per-voxel / per-pixel scales derived from them (device, fp64
// accumulation, global column sums all-reduced): shared by the single- and multi-frame engines.
struct DeviceRaySums {
    // col_shard: the shard holds all rows of some columns, so the row sums are all-reduced instead
    // A: fp32 shard, or bf16 bit patterns when a_bf16
    void compute(const void* A, int64_t P, int64_t Pp, int64_t V, int64_t ld, Communicator* comm,
                 const SolverParams& p, hipStream_t stream, bool col_shard = false, bool a_bf16 = false);
    // the same from a sparse shard (CSR row sums, CSC column sums)
    void compute_sparse(const SparseRtm& s, int64_t P, int64_t Pp, int64_t V, int64_t ld, Communicator* comm,
                        const SolverParams& p, hipStream_t stream);
    std::vector<double> density(int64_t V) const;  // host copies
    std::vector<double> length(int64_t P) const;
    DeviceArray<double> rho64, ell64;
    DeviceArray<float> ray_len, dinv, dscale, dmask;
};

// The largest number of ranks of `comm` that drive one physical GPU (boot id + host name + PCI bus id), identical
// on every rank; 1 when every rank has a GPU of its own. Collective.
int ranks_sharing_device(Communicator* comm, int device);
bool device_shared_across_ranks(Communicator* comm, int device);  // ranks_sharing_device(...) > 1

// Collective, after a synchronised solve: true on every rank when a degradable device all-reduce (P2P) failed on
// some rank (then every rank calls comm->degrade() and re-solves). One host scalar while P2P is active, else free.
bool device_comm_failed_anywhere(Communicator* comm);

// SART_FUSED_MIN_MB (default 128): the drivers' threshold for EngineConfig::fused_min_bytes.
double fused_min_bytes_from_env();

class Engine {
   public:
    // A: device pointer to the row-major shard [nrows_pad x ld] (fp32, or bf16 with cfg.rtm_bf16), zero
    // padded (not owned).
    // sparse: the shard as device CSR + CSC arrays instead (A null; csrc/kernels/sparse.hip, not owned): the two-pass
    // sweep on sparse kernels, row shards of fp32 values only
    Engine(int device, const void* A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel, int64_t ld,
           Communicator* comm, const EngineConfig& cfg, const SparseRtm* sparse = nullptr);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    // CSR Laplacian over nvoxel rows (host arrays, copied). Ignored when beta_laplace == 0 or nnz == 0.
    void set_laplacian(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t nnz);
    // One frame: g = this rank's pixels (host fp64, nrows), x0 = warm start (host fp64, nvoxel) or null,
    // x_out = solution (host fp64, nvoxel, de-normalised).
    // x0_is_last: x0 is this engine's previous x_out (the reference's frame k-1 -> k warm start): the start value
    // is rescaled from the copy still on the device (no host copy and upload; bitwise the same start value)
    SolveInfo solve(const double* g, const double* x0, double* x_out, bool x0_is_last = false);
    // f = A x for this shard (host fp64 in/out).
    void forward(const double* x, double* f);

    bool use_fused() const { return use_fused_; }
    const FusedGeometry& geometry() const { return geom_; }
    const EngineConfig& config() const { return cfg_; }
    hipStream_t stream() const { return stream_; }
    int num_cus() const { return num_cus_; }
    int64_t nrows() const { return P_; }
    int64_t nvoxel() const { return V_; }
    std::vector<double> ray_density() const;  // fp64 (nvoxel): global (row shard) / this shard's voxels (column)
    std::vector<double> ray_length() const;   // fp64 (nrows): this shard's pixels (row shard) / global (column)
    bool column_shard() const { return cfg_.column_shard; }
    bool sparse() const { return sparse_; }
    int64_t nnz() const { return sparse_ ? sp_.nnz : 0; }
    bool shared_device() const { return shared_device_; }
    int ranks_per_device() const { return ranks_per_device_; }
    int plan_cus() const { return plan_cus_; }  // CUs the fused geometry was planned for
    double last_norm() const { return norm_; }

   private:
    void ray_sums();
    void alloc_fused();
    double setup_frame(const double* g, const double* x0, bool x0_on_device = false);
    void sweep();
    void sweep_columns();
    // two-pass kernels on the shard in its storage type: forward (epilogue epi) and split-K back-projection
    // into partial_
    void fwd(int epi, const float* x, float* out_f, float* out_w, double* Fpart, const SartState* st);
    void bwd(const float* w, const SartState* st);
    void run_chunk(int n);
    bool fallback();  // steps the fused-sweep fallback chain (re-solve on the current kernels at its end)
    bool comm_failed_anywhere();  // collective: a degradable device all-reduce failed on some rank
    void drop_graph();
    void set_device() const;

    int device_;
    const void* A_;
    bool sparse_ = false;
    SparseRtm sp_{};
    int64_t P_, Pp_, V_, ld_;
    Communicator* comm_;
    EngineConfig cfg_;
    hipStream_t stream_ = nullptr;
    int num_cus_ = 0;
    bool use_fused_ = false;
    FusedGeometry geom_;
    int nsplit_ = 0;
    int64_t nF_fused_ = 0;
    int64_t chain_tiles_ = 0;     // fused sweep chain_tiles (T = 1 fold period / T >= 2 segment length), 0 = off
    int64_t fused_blocks_ = 0;   // partial-sum rows written by the fused sweep (I, or I * T * segments)
    double norm_ = 1.0;
    int last_sweeps_ = 0;  // sweeps of the previous solve: the first chunk of a warm-started one
    bool last_x_on_device_ = false;  // x_ holds the previous solve's returned solution (no rollback since)
    double last_norm_ = 1.0;

    // comm_buf_: [0, ld) the reduced correction, [ld] ||A x||^2, [ld + 1] the error word of the last sweep, EXCEPT
    // after a one-rank sweep on the one-kernel tail (k_reduce_decide_update keeps them in registers): its contents
    // are then undefined (stale). Nothing reads it after a solve; a diagnostic that does must use SART_TAIL_FUSED=0.
    DeviceArray<float> partial_, comm_buf_, x_, pen_, O_, ghat_, arow_, gpos_, wo_, w_, fitted_;
    DeviceArray<float> xprev_;  // x before the last update (NaN/Inf guard rollback)
    bool shared_device_ = false;
    int ranks_per_device_ = 1;
    int plan_cus_ = 0;
    DeviceArray<double> Fpart_, g64_, x064_;
    DeviceRaySums rs_;
    DeviceArray<SartState> st_;
    DeviceArray<uint64_t> gran_;
    DeviceArray<unsigned> xcnt_;
    DeviceArray<unsigned> ticket_;  // k_decide_update's arrival ticket (0 between sweeps)
    DeviceArray<float> xg_;  // column shard + Laplacian: all-gathered x (nvoxel_total, padded)
    DeviceArray<int64_t> lap_rp_;
    DeviceArray<int32_t> lap_col_;
    DeviceArray<float> lap_val_;
    bool has_lap_ = false;

    // time_collectives: event pairs around the all-reduces of the chunk in each pipeline slot
    std::vector<hipEvent_t> cev_[2];
    int cev_used_[2] = {0, 0};
    int cur_slot_ = 0;
    double comm_ms_ = 0.0;
    bool timing_collectives() const;
    void comm_begin();
    void comm_end();
    void collect_comm(int slot);

    SartState* hstate_ = nullptr;  // pinned [2]
    // pinned per-frame staging (the frame's pixels in, x0 in, the solution out): asynchronous copies instead of
    // the runtime's staged pageable ones (profiles/series_r5_*.jsonl: setup / finish per frame)
    double* hg_ = nullptr;
    double* hx0_ = nullptr;
    float* hxo_ = nullptr;
    hipEvent_t ev_[2] = {nullptr, nullptr};
    hipGraphExec_t graph_ = nullptr;
    bool graph_failed_ = false;
    bool tail_fused_ = true;  // one rank: reduce + decide + update in one kernel (SART_TAIL_FUSED=0: three)
    bool warm_ = false;  // an eager chunk ran with the current kernels
    int injected_ = 0;
    int host_sweep_ = 0;  // sweeps enqueued in the current solve (fault_nan_sweep)
};

}  // namespace sart
