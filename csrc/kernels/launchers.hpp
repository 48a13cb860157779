// Host launchers of the gfx950 SART kernels (csrc/kernels/*.hip). Launchers never allocate, copy or
// synchronise, so they may be captured into HIP graphs; every one checks hipGetLastError.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "sart_common.hpp"

namespace sart {
// projection.hip (RTM in fp32, or bf16 storage with fp32 products and sums)
int64_t forward_num_blocks(int64_t nrows_pad);
void launch_forward(int epi, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                    const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                    const SartState* st, hipStream_t stream);
void launch_forward(int epi, const bf16_t* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                    const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                    const SartState* st, hipStream_t stream);
void launch_rowsum_f64(const float* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream);
void launch_rowsum_f64(const bf16_t* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream);
int backproject_num_splits(int64_t ld, int64_t nrows, int elem_bytes = 4);
void launch_backproject(const float* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                        const SartState* st, hipStream_t stream);
void launch_backproject(const bf16_t* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                        const SartState* st, hipStream_t stream);
void launch_colsum_f64(const float* A, int64_t ld, int64_t nrows, int nsplit, double* partial, hipStream_t stream);
void launch_colsum_f64(const bf16_t* A, int64_t ld, int64_t nrows, int nsplit, double* partial, hipStream_t stream);
// sparse.hip: a sparse RTM shard held twice on the device, as CSR (rows: the forward projection and the row sums) and
// CSC (columns: the back-projection and the column sums), so both projections are gathers with one writer per output
// (no atomics: bitwise reproducible). Indices are 32-bit column / row numbers, offsets 64-bit.
struct SparseRtm {
    const int64_t* row_ptr = nullptr;  // [nrows + 1]
    const int32_t* col = nullptr;      // [nnz]
    const float* val = nullptr;        // [nnz]
    const int64_t* col_ptr = nullptr;  // [nvoxel + 1]
    const int32_t* row = nullptr;      // [nnz]
    const float* cval = nullptr;       // [nnz]
    int64_t nnz = 0;
    // lanes per row / column (4, 8, 16 or 32; 0: sparse_lanes()): one power-of-two group of a wave per row, so short
    // rows do not leave most of a wave idle (set once per engine: the forward's Fpart layout depends on it)
    int lanes_rows = 0, lanes_cols = 0;
};
// lanes per row for rows of `avg` entries on average (env SART_SPARSE_LANES overrides)
int sparse_lanes(double avg);
// fp64 ||f||^2 partials of launch_csr_forward: one per 256 / lanes_rows rows
int64_t csr_forward_num_blocks(const SparseRtm& s, int64_t nrows_pad);
// f = A x with the epilogues of launch_forward (kEpiPlain / kEpiLinear / kEpiLog); Fpart: csr_forward_num_blocks
// fp64 partial sums of f^2
void launch_csr_forward(int epi, const SparseRtm& s, int64_t nrows, int64_t nrows_pad, const float* x,
                        const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                        const SartState* st, hipStream_t stream);
// out[v] = sum_p A[p, v] w[p] for v < nvoxel (one split: out is a partial row of k_reduce_partials)
void launch_csc_backproject(const SparseRtm& s, int64_t nvoxel, const float* w, float* out, const SartState* st,
                            hipStream_t stream);
// multi-frame engine, sparse shard: F [nrows_pad][nf] = A X^T (X frame-major [nf][ld], copied voxel-major into Xt
// [nf / PW][ld][PW] first, PW = pw (mf_sparse_plane_width); padded rows written 0) and part [v][nf] = sum_p A[p][v]
// W[p][f] for v in [v0, v1) (columns >= nvoxel written 0; times scale[v] when given). W: the back-projection
// layout of launch_mf_weights ([wrows][nf], mf_bp_slot), or with mf_sparse_needs_w_planes(nf, pw) the frame-order
// planes [nf / PW][wrows][PW] (launch_mf_w_planes, or launch_mf_weights with wplane = PW).
// frames per SpMM plane for an nf-frame batch (64, or nf below; SART_MF_SPARSE_PW = 16 / 32 / 64 overrides): read
// once by the engine, which lays X and W out for it
int mf_sparse_plane_width(int nf);
bool mf_sparse_needs_w_planes(int nf, int pw);
void launch_mf_sparse_forward(const SparseRtm& s, int64_t nrows, int64_t nrows_pad, const float* X, int64_t ld,
                              float* Xt, float* Fout, int nf, int pw, hipStream_t stream, const int* skip);
void launch_mf_sparse_backproject(const SparseRtm& s, int64_t nvoxel, const float* W, int64_t wrows, float* part,
                                  const float* scale, int nf, int pw, int64_t v0, int64_t v1, hipStream_t stream,
                                  const int* skip);
void launch_mf_w_planes(const float* W, int64_t rows, int nf, int pw, float* Wt, hipStream_t stream,
                        const int* skip);
void launch_csr_rowsum_f64(const SparseRtm& s, int64_t nrows, double* out, hipStream_t stream);
void launch_csc_colsum_f64(const SparseRtm& s, int64_t nvoxel, double* out, hipStream_t stream);
// fp32 -> bf16, round to nearest even (n a multiple of 4)
void launch_f32_to_bf16(const float* src, int64_t n, bf16_t* dst, hipStream_t stream);
// Fout (optional): Fout[0] = sum of Fpart (fp32), Fout[1] = st->error (the sweep's error word, reduced with it)
void launch_reduce_partials(const float* partial, int64_t ld, int nsplit, const float* scale, float* out,
                            const double* Fpart, int64_t nF, float* Fout, const SartState* st, hipStream_t stream);
void launch_reduce_partials_f64(const double* partial, int64_t ld, int nsplit, double* out, hipStream_t stream);
// sart_update.hip
void launch_prep_rows(const double* g, int64_t nrows, int64_t nrows_pad, double inv_s, const float* ray_length,
                      float len_thres, float* ghat, float* arow, float* gpos, float* wo, hipStream_t stream);
void launch_init_solution(float* x, int64_t n, int64_t n_pad, const float* src_f32, const double* src_f64,
                          double scale, hipStream_t stream);
// x = fp32((x a) b), clamped (a warm start from the solution left on the device by the previous solve)
void launch_rescale_solution(float* x, int64_t n, int64_t n_pad, double a, double b, hipStream_t stream);
void launch_penalty(bool logx, const int64_t* row_ptr, const int32_t* col, const float* val, int64_t n, float beta,
                    const float* x, float* pen, const SartState* st, hipStream_t stream);
void launch_decide(SartState* st, const float* Fslot, hipStream_t stream);
// launch_decide + launch_update_{linear,log} in one kernel (d = the reduced corrections, or Fv for log with O the
// observed back-projection); ticket: one device word, 0 between launches (re-armed by the kernel itself).
void launch_decide_update(bool logmode, SartState* st, const float* Fslot, float* x, const float* d, const float* O,
                          const float* pen, float alpha, int64_t n, unsigned* xcnt, float* xprev, unsigned* ticket,
                          hipStream_t stream);
// One rank: launch_reduce_partials (into registers, not d) + launch_decide_update in one kernel; x is bitwise the
// two-launch x. nF: the Fpart partials every workgroup sums (keep it small, e.g. the fused sweep's grid).
void launch_reduce_decide_update(bool logmode, SartState* st, const float* partial, int64_t ld, int nsplit,
                                 const float* scale, const double* Fpart, int64_t nF, float* x, const float* O,
                                 const float* pen, float alpha, int64_t n, unsigned* xcnt, float* xprev,
                                 unsigned* ticket, hipStream_t stream);
// xcnt (optional): fused-sweep ticket counters to zero for the next sweep; xprev (optional): receives x
// before the update (rollback point of the NaN/Inf guard)
void launch_update_linear(float* x, const float* d, const float* pen, int64_t n, const SartState* st,
                          hipStream_t stream, unsigned* xcnt = nullptr, float* xprev = nullptr);
void launch_update_log(float* x, const float* O, const float* Fv, const float* pen, float alpha, int64_t n,
                       const SartState* st, hipStream_t stream, unsigned* xcnt = nullptr, float* xprev = nullptr);
void launch_state_begin(SartState* st, double G, double tol, int max_iter, hipStream_t stream);
// w = a (ghat - f) (linear) or a f (log) from a complete forward projection f; Fpart[block] = sum f^2 (fp64)
int weights_num_blocks(int64_t nrows_pad);
void launch_weights(bool logmode, const float* f, const float* ghat, const float* arow, int64_t nrows,
                    int64_t nrows_pad, float* w, double* Fpart, const SartState* st, hipStream_t stream);
// dst[offset + i] = src[i] for i < n (gather of a column shard's slice into a full-length vector)
void launch_copy_slice(const float* src, int64_t n, float* dst, int64_t offset, hipStream_t stream);
void launch_density_scales(const double* rho, int64_t n, int64_t n_pad, float thres, float alpha, float* dinv,
                           float* dscale, float* dmask, hipStream_t stream);
void launch_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t stream);
// synth.hip
void launch_synth_matrix(float* A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols, int64_t row_offset,
                         uint64_t seed, float lo, float hi, hipStream_t stream);
// block [row_offset, +nrows) x [col_offset, +ncols) of a global nrows_total x ncols_total synthetic matrix
void launch_synth_matrix_block(float* A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols,
                               int64_t row_offset, int64_t col_offset, int64_t ncols_total, uint64_t seed, float lo,
                               float hi, hipStream_t stream);
void launch_synth_vector(double* out, int64_t n, int64_t offset, uint64_t seed, double lo, double hi,
                         hipStream_t stream);
// fused_sweep.hip
int fused_pick_k(int64_t ld);
int fused_tile_rows(int K, int variant);
void fused_set_schedule(int sched);
int fused_get_schedule();
int fused_last_schedule();
// granule buffer entries (uint64) of a variant-6 sweep: chip-wide groups pad each tile's row to 16 granules
int64_t fused_granules(int64_t nrows_pad, int J, bool xl);  // pipeline schedule the last variant-6 launch ran (T / kw / chip-wide pick it), -1: v3
void fused_set_trace(unsigned long long* buf, long long tiles);
std::vector<int> fused_debug_map(int nblocks);
int fused_fpart_per_block(int variant);
void fused_set_debug(int flags);
std::vector<unsigned long long> fused_debug_stats(int nblocks);
void launch_fused_sweep(bool logmode, int K, int variant, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                        const float* x, const float* ghat, const float* arow, float* partial, double* Fpart,
                        uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt, hipStream_t stream,
                        int64_t chain_tiles = 0, int kw = 8, bool xl = true);
// kw (variant 6): lane-vectors per lane per row, slab = 1024 kw / T columns (8, or 7 / 6 at the default
// schedules: widths whose 8-KiB-slab count leaves CUs idle; FusedGeometry::kw).
// chain_tiles (variant 6; 0 = off): T = 1: every ~chain_tiles tiles a compute wave folds its fp32 back-projection
// chain into a second register set (two-level sums). T >= 2 with a split schedule (fused_split_schedule): the
// row groups run in segments of chain_tiles tiles (a multiple of kChainAlign); segment s writes the partial
// blocks (s * T + row) * I + gi, so partial must hold I * T * segments rows of ld floats (fused_chain_plan).
constexpr int64_t kChainAlign = 140;  // lcm of the register-slot counts RS (4, 5, 7) of the T >= 2 pipelines
bool fused_split_schedule(int T, bool bf16);
// bf16-stored RTM: the variant 6 sweep with bf16 tiles (T = rows per tile of the variant 6 geometry; cpl = bf16
// columns per lane per k-slot: 4 (8-byte loads, slab 8192 / T) or 8 (16-byte loads at T = 4 / 2, "wide": slab
// 2048 kw / T with kw = 5 ... 8 lane-vectors per lane, 16384 / T at kw 8))
void launch_fused_sweep_bf16(bool logmode, int T, const bf16_t* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                             const float* x, const float* ghat, const float* arow, float* partial, double* Fpart,
                             uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt, hipStream_t stream,
                             int cpl = 4, int64_t chain_tiles = 0, int kw = 8, bool xl = true);
// p2p_allreduce.hip: one-shot push all-reduce through IPC-mapped peer buffers (at most 8 ranks, fp32).
// Receive buffer of every rank: [2 parities][kP2pMaxRanks sources][cap] floats; flags: [sources][blocks].
constexpr int kP2pMaxRanks = 8;
constexpr int kP2pMaxBlocks = 1024;
struct P2pArgs {
    float* recv[kP2pMaxRanks];      // rank j's receive buffer as mapped in this process
    unsigned* flags[kP2pMaxRanks];  // rank j's flag array as mapped in this process
    const unsigned* abort_word;     // this rank's abort word: set remotely by a peer that aborts
    // workgroups per call (0: kP2pMaxBlocks). Identical on every rank. Ranks sharing one GPU (one-GPU rehearsals)
    // use few: every workgroup spins until its peers' chunks arrive, and the spinning workgroups of all ranks must
    // leave room for the peers' persistent sweeps and their own all-reduce kernels.
    int max_blocks;
};
int64_t p2p_chunk(int64_t n, int max_blocks = kP2pMaxBlocks);  // elements per workgroup
// op: 0 sum, 1 max. `epoch` strictly increases by one per call on every rank (starts at 1).
// skip_flags (fault injection, tests): push the data but raise no flag, so the peers time out in this call.
void launch_p2p_allreduce(const float* in, float* out, int64_t n, const P2pArgs& a, int rank, int nranks,
                          unsigned epoch, int64_t cap, int op, unsigned* err, double timeout_s, hipStream_t stream,
                          bool skip_flags = false);
// The per-sweep vector of the single-frame engine before its all-reduce, as launch_reduce_partials writes it:
// v[i] = scale[i] * sum_s partial[s][i] for i < ld (scale nullptr: 1), v[ld] = sum Fpart[0:nF] (fp64 -> fp32),
// v[ld + 1] = st->error (st nullptr: 0). partial: nsplit rows of ld floats, 16-byte aligned, ld % 64 == 0.
struct ReduceSrc {
    const float* partial = nullptr;
    int64_t ld = 0;
    int nsplit = 0;
    const float* scale = nullptr;
    const double* Fpart = nullptr;
    int64_t nF = 0;
    const SartState* st = nullptr;
};
// The SART update after the per-sweep all-reduce (launch_decide_update's operands), for the P2P kernel's fused tail
struct UpdateArgs {
    SartState* st = nullptr;
    float* x = nullptr;
    const float* O = nullptr;    // log mode: the observed back-projection
    const float* pen = nullptr;  // optional
    float alpha = 1.f;
    int64_t n = 0;               // voxels
    unsigned* xcnt = nullptr;    // optional: per-XCD tickets of the next fused sweep, zeroed here
    float* xprev = nullptr;      // optional: the iterate before the update (NaN/Inf rollback point)
    unsigned* ticket = nullptr;  // the last workgroup to arrive writes the new state
    bool logmode = false;
};
// launch_reduce_partials + launch_p2p_allreduce (sum) of its ld + 2 floats in ONE kernel: each workgroup forms its
// chunk of v in registers and pushes it. out (ld + 2 floats) receives the all-reduced v, bitwise the two-launch result.
// upd (optional): also launch_decide_update in the same kernel -- every workgroup takes ||A x||^2 and the error word
// from the tail slots of all ranks (its own rank's tail computed locally), decides, and updates its chunk's voxels
// (x, state and xprev bitwise those of the separate launch). At N > 1 a SART iteration is then the sweep plus this
// one kernel, as at N = 1 (k_reduce_decide_update).
void launch_p2p_reduce_allreduce(const ReduceSrc& src, float* out, const P2pArgs& a, int rank, int nranks,
                                 unsigned epoch, int64_t cap, unsigned* err, double timeout_s, hipStream_t stream,
                                 bool skip_flags = false, const UpdateArgs* upd = nullptr);
// multiframe.hip (nf = frames per batch: 16, 32 or 64; the 16-bit kernels of multiframe_bf16.hip also take 128)
// target: workgroups to aim for (0: 1024, or SART_MF_FWD_BLOCKS)
int mf_forward_num_splits(int64_t ld, int64_t nrows_pad, int target = 0);
int mf_backproject_num_splits(int64_t ld, int64_t nrows);
void mf_set_depth(int d);  // 1..3: register-ring depth of the MFMA projections; 0: default
void mf_set_rows(int rt);  // 2 or 4: 16-row tiles per wave of the MFMA forward projection; 0: default
void mf_set_vox(int vt);   // 1 or 2: 64-voxel tiles per wave of the MFMA back-projection; 0: default
void launch_mf_forward(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* X, int64_t ldx,
                       float* Fout, int nsplit, int nf, hipStream_t stream);
// voxel range [v0, v1) (default: the whole row), aligned to mf_backproject_vox_align
int mf_backproject_vox_align(int64_t ld, int nf);
void launch_mf_backproject(const float* A, int64_t ld, int64_t nrows, const float* W, int nsplit, float* partial,
                           int nf, hipStream_t stream, int64_t v0 = 0, int64_t v1 = -1);
// multiframe_glue.hip
// No-op sweeps of the multi-frame engine: while a MfSkipScope is alive on the calling thread, the heavy multi-frame
// kernels (projections, weights, collect, operand splits) launched from it return at once when *skip != 0 (the
// device flag MfState::all_done: every slot's frame is done and the sweep would change nothing).
extern thread_local const int* g_mf_skip;
struct MfSkipScope {
    explicit MfSkipScope(const int* p) : prev(g_mf_skip) { g_mf_skip = p; }
    ~MfSkipScope() { g_mf_skip = prev; }
    MfSkipScope(const MfSkipScope&) = delete;
    MfSkipScope& operator=(const MfSkipScope&) = delete;
    const int* prev;
};
// bf16-stored RTM (multiframe_bf16.hip): the same projections on v_mfma_f32_16x16x32_bf16 with the fp32
// operand (X or W) split into hi + lo bf16 planes (k_mf_split_x: X [nf][ld] -> planes [nf][ld]; k_mf_split_w:
// W [rows][16][nf / 16] -> frame-major planes [nf][ldw], ldw >= rows rounded up to 32).
// xblk: X planes in the blocked layout [ld / 32][nf][32] (launch_mf_split_x with ld > 0), else frame-major [nf][ld]
void launch_mf_forward_b16(const bf16_t* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const bf16_t* Xh,
                           const bf16_t* Xl, float* Fout, int nsplit, int nf, hipStream_t stream, bool xblk = false);
// a32: the split-A kernels (fp32 A split into hi + lo bf16 in registers, three products; launch_mf_*_x3)
int mf_backproject_b16_num_splits(int64_t ld, int64_t nrows, bool a32 = false);
int mf_backproject_b16_vox_align(int64_t ld, bool a32 = false);  // voxel-range alignment of the launchers below
void launch_mf_backproject_b16(const bf16_t* A, int64_t ld, int64_t nrows, const bf16_t* Wh, const bf16_t* Wl,
                               int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream, int64_t v0 = 0,
                               int64_t v1 = -1);
void launch_mf_forward_x3(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const bf16_t* Xh,
                          const bf16_t* Xl, float* Fout, int nsplit, int nf, hipStream_t stream, bool xblk = false);
// Wh: hi and mid planes ([2][nf][ldw], launch_mf_split_w with three), Wl: lo plane
void launch_mf_backproject_x3(const float* A, int64_t ld, int64_t nrows, const bf16_t* Wh, const bf16_t* Wl,
                              int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream, int64_t v0 = 0,
                              int64_t v1 = -1);
// perm: the split-A forward's k order (launch_mf_forward_x3 reads planes written with perm = true). ld > 0: X is
// [nf = n / ld][ld] and the planes are written blocked, [ld / 32][nf][32] (the forward's xblk layout)
void launch_mf_split_x(const float* X, int64_t n, bf16_t* hi, bf16_t* lo, hipStream_t stream, bool perm = false,
                       int64_t ld = 0);
// fp16-pair back-projection operands: frame-major planes w1, w2 ([nf][ldw] of f16 bits) of w s_f with a per-frame
// power-of-two scale s_f (from the frame's max |w|, wmax: nf words of scratch), inv_scale[f] = 1 / (a_scale s_f)
// have_max: wmax already holds the frames' max |w| (launch_mf_weights with wmax), else it is computed here
void launch_mf_split_w16(const float* W, int64_t nrows_pad, int nf, int64_t ldw, uint16_t* w1, uint16_t* w2,
                         unsigned* wmax, float a_scale, float* inv_scale, hipStream_t stream, bool have_max = false);
// power-of-two scale 2^(14 - e) for max |A| = m 2^e over n floats (1 if A is zero); synchronises the stream
float absmax_pow2_scale(const float* A, int64_t n, unsigned* scratch, hipStream_t stream);
// split-A back-projection on f16 pairs (two pieces of A s_v and of W s_f, three v_mfma_f32_16x16x32_f16 products,
// fp32 accumulation, the output scaled by 1 / s_v and inv_scale[f] = 1 / s_f): W1 / W2 from launch_mf_split_w16
// (a_scale 1), csc from launch_mf_col_scales
void launch_mf_backproject_h16(const float* A, int64_t ld, int64_t nrows, const uint16_t* W1, const uint16_t* W2,
                               int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream, int64_t v0,
                               int64_t v1, const float* csc, const float* inv_scale);
// Range-safe f16 scales (multiframe_glue.hip): powers of two per row (rsc: [nrows_pad] scales then their inverses)
// and per column (csc: [ld] then [ld]; scratch: ld words) of an fp32 shard
void launch_mf_row_scales(const float* A, int64_t ld, int64_t nrows_pad, float* rsc, hipStream_t stream);
void launch_mf_col_scales(const float* A, int64_t ld, int64_t nrows_pad, unsigned* scratch, float* csc,
                          hipStream_t stream);
// X [nf][ld] -> f16 pieces of X s_f (per-frame power-of-two scale from max |X[f]|; xmax: nf words of scratch,
// xinv[f] = 1 / s_f), in the layout of launch_mf_split_x (perm; blocked = the ld > 0 layout)
void launch_mf_split_x16(const float* X, int64_t ld, int nf, uint16_t* x1, uint16_t* x2, unsigned* xmax, float* xinv,
                         hipStream_t stream, bool perm, bool blocked);
// split-A forward on f16 pairs: A s_p (rsc, per row) times X s_f (launch_mf_split_x16), three f16 products, the
// output scaled by 1 / (s_p s_f)
void launch_mf_forward_h16(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const uint16_t* X1,
                           const uint16_t* X2, float* Fout, int nsplit, int nf, hipStream_t stream, bool xblk,
                           const float* rsc, const float* xinv);
// three: hi [nf][ldw] then mid [nf][ldw] in `hi` (2 nf ldw elements), lo: the split-A back-projection's planes
void launch_mf_split_w(const float* W, int64_t nrows_pad, int nf, int64_t ldw, bf16_t* hi, bf16_t* lo,
                       hipStream_t stream, bool three = false);
int mf_weights_num_blocks(int64_t nrows_pad);
// wmax (optional, nf words): also the per-frame max |w| over finite weights (zeroed here first; as k_mf_wmax)
void launch_mf_weights(const float* Fs, int nsplit, int64_t nrows_pad, const float* ghat, const float* arow,
                       bool logmode, float* W, double* F2part, int nf, hipStream_t stream, unsigned* wmax = nullptr,
                       int wplane = 0);
// D[v][f] (voxel-major) for v in [v0, v1); F2out (optional) = per-frame sums of F2part
void launch_mf_collect(const float* part, int nsplit, int64_t ld, int64_t v0, int64_t v1, const float* scale, float* D,
                       const double* F2part, int nF2, float* F2out, int nf, hipStream_t stream);
void launch_mf_penalty(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t n, float beta, bool logx,
                       const float* X, int64_t ld, float* pen, const MfState* st, int nf, hipStream_t stream);
// q (optional): the device refill plan follows the decisions (mf_plan, MultiFrameEngine::solve_series)
void launch_mf_decide(MfState* st, const float* F2, hipStream_t stream, MfQueue* q = nullptr);
// Xprev (optional): receives X before the update (NaN/Inf guard rollback). q / rf: the refill of this sweep's plan
// (retired iterates into the ring, start values and log O of the admitted frames)
void launch_mf_update(float* X, const float* D, float* O, const float* pen, float alpha, bool logmode,
                      int64_t nvox, int64_t ld, const MfState* st, int nf, hipStream_t stream, float* Xprev = nullptr,
                      const MfQueue* q = nullptr, const MfRefill* rf = nullptr);
// device refill: ghat / arow columns of the admitted frames from the staged pixels ghq [qcap][nrows_pad]
void launch_mf_admit_rows(const MfQueue* q, const float* ghq, int64_t nrows, int64_t nrows_pad, const float* ray_length,
                          float len_thres, float* ghat, float* arow, int nf, hipStream_t stream);
// back-projection operands (gpos, and wo unless null) of k staged entries, columns j < k (layout of k_mf_prep_slots)
void launch_mf_stage_ops(const float* ghq, int64_t e0, int qcap, int k, int64_t nrows, int64_t nrows_pad,
                         const float* ray_length, float len_thres, float* gpos, float* wo, int nf, hipStream_t stream);
// columns j < k of a reduced voxel-major D [ld][nf] into rows (e0 + j) % qcap of out [qcap][ld]: cold starts
// max(D dinv, 1e-7) with dinv, else copies
void launch_mf_stage_cols(const float* D, const float* dinv, int64_t e0, int qcap, int k, int64_t nvox, int64_t ld,
                          int nf, float* out, hipStream_t stream);
// staging on the device: raw fp64 pixels g64q [qcap][nrows_pad] of k entries -> per-frame max / positive sum of squares
// (stats [2][nf], all-reduced by the caller) -> the queue metadata and the normalised pixels ghq [qcap][nrows_pad]
void launch_mf_stage_stats(const double* g64q, int64_t e0, int qcap, int k, int64_t nrows, int64_t nrows_pad,
                           double* stats, int nf, hipStream_t stream);
void launch_mf_stage_norm(MfQueue* q, const double* g64q, float* ghq, const double* stats, int64_t e0, int64_t frame0,
                          bool cold, int k, int64_t nrows, int64_t nrows_pad, int nf, hipStream_t stream);
void launch_mf_publish(MfQueue* q, int64_t q_tail, hipStream_t stream);
void launch_mf_drained(MfQueue* q, int64_t drained, hipStream_t stream);
void launch_mf_queue_begin(MfQueue* q, int qcap, int rcap, bool chain, int admit_cap, int src_age, int64_t x0_below,
                           bool src_finished, bool lead, float src_extrap, hipStream_t stream, float drift = 0.f);
void launch_mf_state_begin(MfState* st, const double* G, int nused, double tol, int max_iter, int nf,
                           hipStream_t stream);
}  // namespace sart
