// sartsolver -- native driver binary: same CLI, input validation, frame loop, output file
// and console output as the reference binary (reference main.cpp:25-151), MI355X-first:
//
//   * one process per GPU, any launcher that sets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
//     MASTER_PORT (torchrun --no-python, mpirun via OMPI_COMM_WORLD_*, or bin/sartsolver); one process
//     runs without any launcher. Rank -> GPU = LOCAL_RANK % device count (reference: rank % count,
//     sartsolver_cuda.cpp:96-98).
//   * per-iteration reductions on device buffers (csrc/engine/comm.cpp): the one-shot P2P all-reduce over
//     xGMI or RCCL; host scalars over the TCP or MPI bootstrap (mpiexec launches use MPI_COMM_WORLD); the
//     --use_cpu path uses the host communicator alone.
//   * every rank streams only its pixel rows from HDF5 straight into HBM through two pinned staging
//     buffers (the reference keeps the whole shard in host RAM, raytransfer.hpp:20); with
//     --parallel_read all ranks read at once, otherwise in turn (reference main.cpp:78-86).
//   * the next composite frame is read on a helper thread while the current one is solved.
//   * a fatal error on any rank aborts the communicators instead of leaving peers blocked in a
//     collective (the reference calls std::exit on one rank).
// Extensions: --resume, --two_pass, --profile FILE (JSON lines per frame: iterations, convergence, it/s,
// GFLOPS, RTM GB/s, GPU time in the all-reduces, communicators), --batch_frames N (N
// frames solved together by the multi-frame MFMA engine; batches warm-start from the previous batch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <future>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <stdexcept>
#include <string>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <csignal>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../engine/comm.hpp"
#include "../engine/engine.hpp"
#include "../engine/geometry.hpp"
#include "../engine/multiframe.hpp"
#include "../kernels/launchers.hpp"
#include "../native/config.hpp"
#include "../native/cpu_solver.hpp"
#include "../native/frames.hpp"
#include "../native/h5.hpp"
#include "../native/host_comm.hpp"
#include "../native/inputs.hpp"
#include "../native/solver_params.hpp"

using namespace sart;

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

bool file_exists(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0;
}

// Device-resident row shard [nrows_pad x ld] filled by streaming HDF5 row blocks through two pinned
// buffers: block k+1 is read on a helper thread while block k is copied host -> HBM. bf16 (--rtm_bf16):
// each block lands in an fp32 staging buffer in HBM and is rounded into the bf16 shard on the device.
struct DeviceShard {
    void* A = nullptr;  // fp32, or bf16 bit patterns when bf16
    bool bf16 = false;
    int64_t nrows = 0, nrows_pad = 0, nvoxel = 0, ld = 0;
    ~DeviceShard() {
        if (A) (void)hipFree(A);
    }
};

// Load-path observability (--profile's first line): wall time of the whole load, the summed HDF5 read time of the
// reader, the summed GPU time of the host -> HBM copies, the time the copy loop waited for a read (read-bound) and for
// a staging buffer to drain (copy-bound), and the resident-set high-water mark before / after, the baseline taken after
// the HIP runtime's one-time set-up (the loader's own host memory is the two pinned staging blocks). With the double
// buffer working, wall ~ max(read, h2d) + one block.
struct LoadStats {
    // setup_s: device allocation, pinned staging and opening the files (before the first block read)
    double wall_s = 0, setup_s = 0, read_s = 0, h2d_s = 0, wait_read_s = 0, wait_copy_s = 0;
    uint64_t bytes = 0, blocks = 0, rows_per_block = 0, staging_bytes = 0, rows_per_read = 0;
    double rss_hwm_before_mb = 0, rss_hwm_after_mb = 0, rss_after_setup_mb = 0, rss_after_first_read_mb = 0;
    // setup checkpoints (VmHWM, MiB): after the device allocation, after its zero fill, after the pinned staging
    double rss_after_malloc_mb = 0, rss_after_memset_mb = 0, rss_after_pinned_mb = 0;
};

double rss_hwm_mb() {  // VmHWM of this process, MiB (0 where /proc is unavailable)
    std::ifstream f("/proc/self/status");
    std::string line;
    while (std::getline(f, line))
        if (line.rfind("VmHWM:", 0) == 0) return std::atof(line.c_str() + 6) / 1024.0;
    return 0.0;
}

double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// col0 / ncols: only that voxel block of every row (--partition_voxels), read as a column hyperslab.
std::unique_ptr<DeviceShard> load_device_shard(const InputSet& in, uint64_t row0, uint64_t nrows, size_t block_bytes,
                                               uint64_t col0 = 0, uint64_t ncols = 0, bool bf16 = false,
                                               LoadStats* stats = nullptr) {
    LoadStats ls;
    // The HIP runtime's one-time host footprint is not the loader's: its first kernel launch (code objects, device
    // queues: ~0.4 GB of resident memory on the MI355X box), its first pitched host -> device copy and the copy
    // stream itself (~0.19 GB: the stream's device queue) are paid here, before the baseline is taken
    // (profiles/load_r5_rss_checkpoints*.jsonl); what the load adds after it is the loader's own memory.
    hip_ok(hipFree(nullptr), "hipFree");
    hipStream_t s;
    hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    {
        void* d = nullptr;
        float* h = nullptr;
        hip_ok(hipMalloc(&d, 1 << 20), "hipMalloc(warm-up)");
        hip_ok(hipHostMalloc(reinterpret_cast<void**>(&h), 4096), "hipHostMalloc(warm-up)");
        hip_ok(hipMemsetAsync(d, 0, 1 << 20, s), "hipMemset(warm-up)");
        hip_ok(hipMemcpy2DAsync(d, 4096, h, 1024, 1024, 4, hipMemcpyHostToDevice, s), "hipMemcpy2D(warm-up)");
        hip_ok(hipStreamSynchronize(s), "warm-up sync");
        (void)hipHostFree(h);
        (void)hipFree(d);
    }
    ls.rss_hwm_before_mb = rss_hwm_mb();
    const auto t_load = std::chrono::steady_clock::now();
    auto sh = std::make_unique<DeviceShard>();
    sh->bf16 = bf16;
    if (ncols == 0) ncols = in.nvoxel - col0;
    sh->nrows = (int64_t)nrows;
    sh->nvoxel = (int64_t)ncols;
    sh->ld = choose_ld(sh->nvoxel, 0.10, !bf16);  // bf16 shards keep the 8-KiB slabs of their tiles
    sh->nrows_pad = (sh->nrows + 63) / 64 * 64;
    const size_t bytes = (size_t)sh->nrows_pad * sh->ld * (bf16 ? sizeof(bf16_t) : sizeof(float));
    hip_ok(hipMalloc(&sh->A, bytes), "hipMalloc(RTM shard)");
    ls.rss_after_malloc_mb = rss_hwm_mb();
    // on the copy stream: a fill on the null stream would bring up that stream's device queue (~0.19 GB resident)
    hip_ok(hipMemsetAsync(sh->A, 0, bytes, s), "hipMemset(RTM shard)");
    hip_ok(hipStreamSynchronize(s), "hipMemset sync");
    ls.rss_after_memset_mb = rss_hwm_mb();
    const uint64_t V = ncols;  // staging row length: the column window only
    RtmReader reader(in.rtm_files, in.rtm_name, in.nvoxel, col0, col0 + ncols);
    if (const char* e = std::getenv("SART_RTM_ROWS_PER_READ"); e && *e) {
        ls.rows_per_read = (uint64_t)std::max(0ll, std::atoll(e));
        reader.set_rows_per_read(ls.rows_per_read);
    }
    const uint64_t rows_per_block = std::max<uint64_t>(1, std::min<uint64_t>(nrows, block_bytes / (4 * V)));
    ls.rows_per_block = rows_per_block;
    ls.staging_bytes = 2 * rows_per_block * V * sizeof(float);
    float* buf[2] = {nullptr, nullptr};
    for (auto& b : buf) hip_ok(hipHostMalloc(reinterpret_cast<void**>(&b), rows_per_block * V * sizeof(float)), "hipHostMalloc");
    ls.rss_after_pinned_mb = rss_hwm_mb();
    // bf16: fp32 staging rows [rows_per_block x ld], padding columns zero (the 2-D copies write ncols only)
    DeviceArray<float> stage;
    if (bf16) stage.resize(rows_per_block * (size_t)sh->ld);
    hipEvent_t ev[2];
    for (auto& e : ev) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    bool ev_used[2] = {false, false};
    std::vector<std::pair<uint64_t, uint64_t>> blocks;
    for (uint64_t r = 0; r < nrows; r += rows_per_block) blocks.emplace_back(r, std::min(nrows, r + rows_per_block));
    // timing events around every block copy (GPU time of the H2D traffic)
    std::vector<hipEvent_t> tev(2 * blocks.size(), nullptr);
    for (auto& e : tev) hip_ok(hipEventCreate(&e), "hipEventCreate");
    std::vector<double> read_s(blocks.size(), 0.0);  // one slot per block: written by whichever thread reads it
    auto read_into = [&](size_t k, float* b) {
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t r0 = blocks[k].first, r1 = blocks[k].second;
        std::memset(b, 0, (r1 - r0) * V * sizeof(float));  // sparse COO rows are scattered into zeros
        reader.read(row0 + r0, row0 + r1, b, V);  // one reader: sparse arrays are read once per shard
        read_s[k] = seconds_since(t0);
    };
    auto release = [&]() {
        for (auto& e : tev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : ev) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(s);
        for (auto& b : buf) (void)hipHostFree(b);
    };
    ls.setup_s = seconds_since(t_load);
    ls.rss_after_setup_mb = rss_hwm_mb();
    try {
        if (!blocks.empty()) read_into(0, buf[0]);
        ls.rss_after_first_read_mb = rss_hwm_mb();
        for (size_t k = 0; k < blocks.size(); ++k) {
            float* cur = buf[k % 2];
            std::future<void> next;
            if (k + 1 < blocks.size()) {
                const int nb = (k + 1) % 2;
                if (ev_used[nb]) {  // the staging buffer of block k + 1 still feeds the copy of block k - 1
                    const auto tw = std::chrono::steady_clock::now();
                    hip_ok(hipEventSynchronize(ev[nb]), "event sync");
                    ls.wait_copy_s += seconds_since(tw);
                }
                next = std::async(std::launch::async, read_into, k + 1, buf[nb]);
            }
            const uint64_t r0 = blocks[k].first, nr = blocks[k].second - blocks[k].first;
            float* dst = bf16 ? stage.get() : static_cast<float*>(sh->A) + r0 * sh->ld;
            hip_ok(hipEventRecord(tev[2 * k], s), "event");
            hip_ok(hipMemcpy2DAsync(dst, sh->ld * sizeof(float), cur, V * sizeof(float), ncols * sizeof(float), nr,
                                    hipMemcpyHostToDevice, s),
                   "H2D RTM block");
            hip_ok(hipEventRecord(tev[2 * k + 1], s), "event");
            if (bf16)  // stream-ordered: the next block's copy into the staging rows waits for this conversion
                launch_f32_to_bf16(stage.get(), (int64_t)nr * sh->ld, static_cast<bf16_t*>(sh->A) + r0 * sh->ld, s);
            hip_ok(hipEventRecord(ev[k % 2], s), "event");
            ev_used[k % 2] = true;
            if (next.valid()) {
                const auto tw = std::chrono::steady_clock::now();
                next.get();
                ls.wait_read_s += seconds_since(tw);
            }
        }
        hip_ok(hipStreamSynchronize(s), "RTM upload");
    } catch (...) {
        (void)hipStreamSynchronize(s);
        release();
        throw;
    }
    for (size_t k = 0; k < blocks.size(); ++k) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, tev[2 * k], tev[2 * k + 1]) == hipSuccess) ls.h2d_s += 1e-3 * ms;
        ls.read_s += read_s[k];
    }
    release();
    ls.blocks = blocks.size();
    ls.bytes = nrows * V * sizeof(float);
    ls.wall_s = seconds_since(t_load);
    ls.rss_hwm_after_mb = rss_hwm_mb();
    if (stats) *stats = ls;
    return sh;
}

// Sparse device shard (--rtm_format): the rows' non-zeros as CSR + CSC (csrc/kernels/sparse.hip). Read through
// RtmReader::read_csr (COO arrays of sparse datasets, non-zeros of dense row blocks), transposed on the host, copied
// once; host memory is the two CSR copies of the shard, freed after the upload.
struct DeviceSparseShard {
    DeviceArray<int64_t> rp, cp;
    DeviceArray<int32_t> col, row;
    DeviceArray<float> val, cval;
    int64_t nrows = 0, nvoxel = 0, nnz = 0;
    SparseRtm view() const {
        SparseRtm s;
        s.row_ptr = rp.get();
        s.col = col.get();
        s.val = val.get();
        s.col_ptr = cp.get();
        s.row = row.get();
        s.cval = cval.get();
        s.nnz = nnz;
        return s;
    }
};

std::unique_ptr<DeviceSparseShard> load_sparse_shard(const InputSet& in, uint64_t row0, uint64_t nrows,
                                                     LoadStats* stats) {
    LoadStats ls;
    // The HIP runtime's one-time host footprint first, as in load_device_shard: each device queue comes up with its
    // first command, ~0.19 GB resident apiece on the MI355X box whatever the shard size -- the null stream's (the
    // fills of DeviceArray::resize, which the engine runs anyway), the copy stream's and the copy engine's, which a
    // small copy does not use (profiles/sparse_load_rss_r6.jsonl: +0.19 / +0.41 GB after the CSR + CSC without
    // these). The baseline is taken after them.
    hip_ok(hipFree(nullptr), "hipFree");
    hipStream_t s;
    hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    constexpr size_t kStage = (size_t)16 << 20;  // two pinned 16-MiB staging buffers (the upload's only host memory)
    char* stg[2] = {nullptr, nullptr};
    hipEvent_t ev[2];
    {
        DeviceArray<float> d;
        d.resize(kStage / sizeof(float));  // (null-stream fill)
        void* h = nullptr;
        hip_ok(hipHostMalloc(&h, kStage), "hipHostMalloc(warm-up)");
        for (auto& e : ev) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        hip_ok(hipMemsetAsync(d.get(), 0, kStage, s), "hipMemset(warm-up)");
        hip_ok(hipMemcpyAsync(d.get(), h, kStage, hipMemcpyHostToDevice, s), "hipMemcpy(warm-up)");
        for (auto& e : ev) hip_ok(hipEventRecord(e, s), "hipEventRecord");
        hip_ok(hipStreamSynchronize(s), "warm-up sync");
        (void)hipHostFree(h);
    }
    ls.rss_hwm_before_mb = rss_hwm_mb();
    const auto t0 = std::chrono::steady_clock::now();
    RtmReader reader(in.rtm_files, in.rtm_name, in.nvoxel);
    const HostCsr a = reader.read_csr(row0, row0 + nrows);
    ls.rss_after_first_read_mb = rss_hwm_mb();  // (streamed COO chunks: the CSR and the reader's 20 MB of chunks)
    const HostCsr t = csr_transpose(a);
    ls.rss_after_setup_mb = rss_hwm_mb();  // CSR + CSC
    ls.read_s = seconds_since(t0);
    auto sh = std::make_unique<DeviceSparseShard>();
    sh->nrows = (int64_t)nrows;
    sh->nvoxel = (int64_t)in.nvoxel;
    sh->nnz = a.nnz();
    const size_t n = (size_t)std::max<int64_t>(1, sh->nnz);
    sh->rp.resize(a.ptr.size());
    sh->cp.resize(t.ptr.size());
    sh->col.resize(n);
    sh->row.resize(n);
    sh->val.resize(n);
    sh->cval.resize(n);
    const auto t1 = std::chrono::steady_clock::now();
    for (auto& b : stg) hip_ok(hipHostMalloc(reinterpret_cast<void**>(&b), kStage), "hipHostMalloc");
    // through the pinned buffers, double-buffered: a pageable hipMemcpy of a large array stages through the
    // runtime's own pinned memory, which stays resident after the load
    int k = 0;
    auto up = [&](void* d, const void* h, size_t bytes) {
        for (size_t o = 0; o < bytes; o += kStage, k ^= 1) {
            const size_t m = std::min(kStage, bytes - o);
            hip_ok(hipEventSynchronize(ev[k]), "hipEventSynchronize");  // the copy that last used this buffer
            std::memcpy(stg[k], static_cast<const char*>(h) + o, m);
            hip_ok(hipMemcpyAsync(static_cast<char*>(d) + o, stg[k], m, hipMemcpyHostToDevice, s), "H2D sparse RTM");
            hip_ok(hipEventRecord(ev[k], s), "hipEventRecord");
        }
    };
    up(sh->rp.get(), a.ptr.data(), a.ptr.size() * sizeof(int64_t));
    up(sh->cp.get(), t.ptr.data(), t.ptr.size() * sizeof(int64_t));
    up(sh->col.get(), a.idx.data(), a.idx.size() * sizeof(int32_t));
    up(sh->val.get(), a.val.data(), a.val.size() * sizeof(float));
    up(sh->row.get(), t.idx.data(), t.idx.size() * sizeof(int32_t));
    up(sh->cval.get(), t.val.data(), t.val.size() * sizeof(float));
    hip_ok(hipStreamSynchronize(s), "H2D sparse RTM sync");
    for (auto& e : ev) (void)hipEventDestroy(e);
    for (auto& b : stg) (void)hipHostFree(b);
    (void)hipStreamDestroy(s);
    ls.staging_bytes = 2 * kStage;
    ls.h2d_s = seconds_since(t1);
    ls.blocks = 1;
    ls.rows_per_block = nrows;
    ls.bytes = (uint64_t)sh->nnz * 16 + (a.ptr.size() + t.ptr.size()) * sizeof(int64_t);
    ls.wall_s = seconds_since(t0);
    ls.rss_hwm_after_mb = rss_hwm_mb();
    if (stats) *stats = ls;
    return sh;
}

std::string json_escape(const std::string& s) {
    std::string o;
    for (char c : s) o += (c == '"' || c == '\\') ? std::string("\\") + c : std::string(1, c);
    return o;
}

}  // namespace

int main(int argc, char** argv) {
    // Started by the Python entry point (cli.py sets SART_PARENT_PID): die with it. cli.py forwards SIGTERM /
    // SIGINT / SIGHUP itself; this covers a parent killed with SIGKILL, so no orphan keeps the GPU or sits in a
    // collective. A parent that is already gone (a race with the prctl) ends the driver at once.
    if (const char* pp = std::getenv("SART_PARENT_PID"); pp && *pp) {
        (void)::prctl(PR_SET_PDEATHSIG, SIGTERM);
        if ((long)::getppid() != std::atol(pp)) return 1;
    }
    std::vector<std::string> args(argv + 1, argv + argc);
    Config cfg;
    std::vector<std::array<double, 4>> intervals;
    InputSet in;
    try {
        cfg = parse_arguments(args);
        if (cfg.help) {
            std::cout << usage() << std::endl;
            return 0;
        }
        intervals = parse_time_intervals(cfg.time_range);
        // metadata validation on every rank, before any communicator exists (reference main.cpp:27-59)
        in = validate_inputs(cfg.input_files, cfg.raytransfer_name, cfg.wavelength_threshold);
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }

    const bool gpu = !cfg.use_cpu;
    const EnvWorld w = env_world();
    int device = 0;
    std::unique_ptr<Communicator> dcomm;
    std::unique_ptr<HostComm> hcomm;
    HostComm* host = nullptr;
    try {
        if (gpu) {
            int ndev = 0;
            if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
                throw std::runtime_error("No GPU available: run with --use_cpu or on an MI355X node.");
            device = w.local_rank % ndev;
            hip_ok(hipSetDevice(device), "hipSetDevice");
            dcomm = comm_from_env(device);
            host = &dcomm->host();
        } else {
            hcomm = host_comm_from_env();
            host = hcomm.get();
        }
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    const int rank = host->rank(), size = host->size();

    try {
        // --partition_voxels: every rank holds all pixels of a block of voxels (EngineConfig::column_shard)
        const bool cols = gpu && cfg.partition_voxels;
        const Block vblk = cols ? block_partition(in.nvoxel, size, rank) : Block{0, in.nvoxel};
        const Block blk = cols ? Block{0, in.npixel} : block_partition(in.npixel, size, rank);  // reference main.cpp:67-68
        if (blk.size == 0 || vblk.size == 0)
            throw std::runtime_error("rank " + std::to_string(rank) + " owns no " + (cols ? "voxels" : "pixels") +
                                     ": use at most " + std::to_string(cols ? in.nvoxel : in.npixel) + " ranks");
        CompositeImage image(in.image_files, in.frame_masks, intervals, blk.size, blk.offset);
        image.set_max_cache_size((uint64_t)cfg.max_cached_frames);

        SolverParams params;
        params.logarithmic = cfg.logarithmic;
        params.ray_density_threshold = cfg.ray_density_threshold;
        params.ray_length_threshold = cfg.ray_length_threshold;
        params.conv_tolerance = cfg.conv_tolerance;
        params.beta_laplace = cfg.beta_laplace;
        params.relaxation = cfg.relaxation;
        params.max_iterations = cfg.max_iterations;
        validate_params(params);
        Csr lap;
        if (!cfg.laplacian_file.empty()) {
            const LaplacianCOO coo = read_laplacian(cfg.laplacian_file, in.nvoxel);
            lap = csr_from_coo((int64_t)in.nvoxel, coo.i, coo.j, coo.value);
        }

        std::unique_ptr<DeviceShard> dshard;
        std::unique_ptr<DeviceSparseShard> sshard;
        std::vector<float> hshard;
        // --rtm_format: the single-frame GPU solver on pixel-row shards of fp32 values can keep a sparse RTM sparse
        // (decided from the files' metadata: the same on every rank)
        bool sparse = false;
        if (!cols && !cfg.rtm_bf16 && cfg.rtm_format != "dense") {
            const double dens = rtm_sparse_density(in.rtm_files, in.rtm_name, in.npixel, in.nvoxel);
            // auto: the sparse kernels read 16 bytes per non-zero and sweep (CSR + CSC, index + value) against 4 bytes
            // per element for the dense fused sweep; measured at 32768 x 32768 (uniform random positions): sparse /
            // dense fused it/s 11268 / 1525 at 1 %, 3038 / 1532 at 4.9 %, 2031 / 1534 at 9.5 %, 1336 / 1531 at 18 %
            // (profiles/sparse_r5_density_breakeven.jsonl): auto takes the sparse path up to 10 %
            sparse = cfg.rtm_format == "sparse" || (dens >= 0.0 && dens <= 0.10);
        }
        LoadStats lstats;
        size_t block_bytes = (size_t)256 << 20;  // per staging buffer (two of them)
        if (const char* e = std::getenv("SART_RTM_BLOCK_MB"); e && *e)
            block_bytes = (size_t)std::max(1.0, std::atof(e) * 1048576.0);
        HostCsr hcsr;  // --use_cpu with a sparse shard
        int64_t cpu_nnz = 0;
        auto load = [&]() {
            if (sparse && !gpu) {  // (the CPU solver's CSR alone; the load line as on the GPU path)
                lstats.rss_hwm_before_mb = rss_hwm_mb();
                const auto t0 = std::chrono::steady_clock::now();
                hcsr = RtmReader(in.rtm_files, in.rtm_name, in.nvoxel).read_csr(blk.offset, blk.offset + blk.size);
                lstats.wall_s = lstats.read_s = seconds_since(t0);
                cpu_nnz = hcsr.nnz();
                lstats.bytes = (uint64_t)cpu_nnz * 8 + hcsr.ptr.size() * sizeof(int64_t);
                lstats.rss_hwm_after_mb = rss_hwm_mb();
            }
            else if (sparse)
                sshard = load_sparse_shard(in, blk.offset, blk.size, &lstats);
            else if (gpu)
                dshard = load_device_shard(in, blk.offset, blk.size, block_bytes, vblk.offset, vblk.size,
                                           cfg.rtm_bf16, &lstats);
            else {
                hshard.assign(blk.size * in.nvoxel, 0.f);
                RtmReader(in.rtm_files, in.rtm_name, in.nvoxel)
                    .read(blk.offset, blk.offset + blk.size, hshard.data(), in.nvoxel);
            }
        };
        if (cfg.parallel_read || size == 1) {
            load();
        } else {
            for (int r = 0; r < size; ++r) {  // serialized reads (reference main.cpp:80-85)
                if (r == rank) load();
                host->barrier();
            }
        }
        if (gpu && rank == 0)  // the HDF5 -> HBM load of this rank's shard (all ranks: the --profile load line)
            std::cout << "RTM loaded in: " << lstats.wall_s << " s (" << lstats.bytes / 1e9 << " GB, "
                      << (lstats.wall_s > 0 ? lstats.bytes / 1e9 / lstats.wall_s : 0.0) << " GB/s"
                      << (sparse ? ", sparse: " + std::to_string(sshard->nnz) + " non-zeros" : std::string()) << ")"
                      << std::endl;

        // the single-frame engine (frame by frame; with --batch_frames it solves a cold time series' first frame)
        auto make_engine = [&](double tol_factor) {
            std::unique_ptr<Engine> e;
            EngineConfig ec;
            static_cast<SolverParams&>(ec) = params;
            ec.conv_tolerance *= tol_factor;
            ec.use_fused = !cfg.two_pass;
            ec.fused_min_bytes = fused_min_bytes_from_env();
            if (const char* v = std::getenv("SART_FUSED_VARIANT"); v && *v) ec.fused_variant = std::atoi(v);
            ec.time_collectives = !cfg.profile_file.empty();  // --profile: GPU time in the all-reduces per frame
            if (cols) {
                ec.column_shard = true;
                ec.col_offset = (int64_t)vblk.offset;
                ec.nvoxel_total = (int64_t)in.nvoxel;
            }
            if (sparse) {
                const SparseRtm view = sshard->view();
                e = std::make_unique<Engine>(device, nullptr, sshard->nrows, (sshard->nrows + 63) / 64 * 64,
                                             sshard->nvoxel, (sshard->nvoxel + 63) / 64 * 64, dcomm.get(), ec, &view);
            } else {
                ec.rtm_bf16 = dshard->bf16;
                e = std::make_unique<Engine>(device, dshard->A, dshard->nrows, dshard->nrows_pad, dshard->nvoxel,
                                             dshard->ld, dcomm.get(), ec);
            }
            if (lap.nnz()) e->set_laplacian(lap.row_ptr.data(), lap.col.data(), lap.val.data(), lap.nnz());
            return e;
        };
        std::unique_ptr<Engine> engine, lead_engine;
        // the lead frame stops at lead_tol x the tolerance and hands its iterate to the batch, where it finishes next
        // to the frames chained from it (1: it finishes on the single-frame engine; SART_MF_LEAD_TOL)
        double lead_tol = 1.0;
        std::unique_ptr<MultiFrameEngine> mf;
        std::unique_ptr<CpuSolver> cpu;
        const bool batched = gpu && cfg.batch_frames > 1;
        if (batched) {
            EngineConfig ec;
            static_cast<SolverParams&>(ec) = params;
            ec.mf_frames = cfg.batch_frames;  // batch width 16, 32, 64 or 128 (rounded up; 128: bf16 storage and f16-pair split-A)
            if (sparse) {  // fp32 SpMM projections of the CSR / CSC shard
                const SparseRtm view = sshard->view();
                mf = std::make_unique<MultiFrameEngine>(device, nullptr, sshard->nrows, (sshard->nrows + 63) / 64 * 64,
                                                        sshard->nvoxel, (sshard->nvoxel + 63) / 64 * 64, dcomm.get(),
                                                        ec, &view);
            } else {
                ec.rtm_bf16 = dshard->bf16;  // bf16 MFMA projections
                mf = std::make_unique<MultiFrameEngine>(device, dshard->A, dshard->nrows, dshard->nrows_pad,
                                                        dshard->nvoxel, dshard->ld, dcomm.get(), ec);
            }
            if (lap.nnz()) mf->set_laplacian(lap.row_ptr.data(), lap.col.data(), lap.val.data(), lap.nnz());
            // a cold time series' first frame: the single-frame engine, built with the set-up (before the frame loop's
            // clock, like the frame-by-frame engine); dropped after that frame (SART_MF_LEAD_ENGINE=0: none)
            const char* le = std::getenv("SART_MF_LEAD_ENGINE");
            if (const char* lt = std::getenv("SART_MF_LEAD_TOL"); lt && *lt) lead_tol = std::max(1.0, std::atof(lt));
            if (!cfg.no_guess && !(le && *le && std::atoi(le) == 0)) lead_engine = make_engine(lead_tol);
        } else if (gpu) {
            engine = make_engine(1.0);
        } else {
            if (sparse)
                cpu = std::make_unique<CpuSolver>(std::move(hcsr), host, params, false);
            else
                cpu = std::make_unique<CpuSolver>(hshard.data(), (int64_t)blk.size, (int64_t)in.nvoxel,
                                                  (int64_t)in.nvoxel, host, params, false);
            if (lap.nnz()) cpu->set_laplacian(lap);
        }

        // rank 0 owns the output (reference main.cpp:115-125, solution.cpp)
        std::unique_ptr<SolutionWriter> writer;
        VoxelGrid voxelgrid;
        double skip_until = -std::numeric_limits<double>::infinity();
        std::vector<double> warm;
        bool appended = false;
        if (rank == 0) {
            if (cfg.resume && file_exists(cfg.output_file)) {
                const StoredSolutions st = read_solution_file(cfg.output_file);
                if (!st.time.empty()) {
                    appended = true;
                    skip_until = st.time.back();
                    warm = st.last_solution;
                }
            }
            writer = std::make_unique<SolutionWriter>(cfg.output_file, in.camera_names, in.nvoxel,
                                                      (uint64_t)cfg.max_cached_solutions, appended);
            voxelgrid.read(in.rtm_files.begin()->second, "rtm/voxel_map");
            for (const auto& m : voxelgrid.warnings) std::cerr << "warning: " << m << std::endl;
        }
        host->broadcast_host(&skip_until, sizeof(skip_until), 0);
        int has_warm = (!cfg.no_guess && !warm.empty()) ? 1 : 0;
        host->broadcast_host(&has_warm, sizeof(has_warm), 0);
        if (has_warm) {
            warm.resize(in.nvoxel);
            host->broadcast_host(warm.data(), warm.size() * sizeof(double), 0);
        } else {
            warm.clear();
        }
        std::ofstream profile;
        if (rank == 0 && !cfg.profile_file.empty()) profile.open(cfg.profile_file);
        if ((gpu || sparse) && !cfg.profile_file.empty()) {
            // first profile line: the HDF5 -> HBM load (slowest rank's wall time; totals over ranks)
            double mx[4] = {lstats.wall_s, lstats.rss_hwm_after_mb - lstats.rss_hwm_before_mb, lstats.setup_s,
                            (double)lstats.bytes};
            double sm[5] = {(double)lstats.bytes, lstats.read_s, lstats.h2d_s, lstats.wait_read_s, lstats.wait_copy_s};
            host->all_reduce_host(mx, 4, ReduceOp::kMax);
            host->all_reduce_host(sm, 5, ReduceOp::kSum);
            if (profile.is_open())
                profile << "{\"load\": true, \"load_s\": " << mx[0] << ", \"rtm_GB\": " << sm[0] / 1e9
                        << ", \"load_GBps\": " << (mx[0] > 0 ? sm[0] / 1e9 / mx[0] : 0.0)
                        << ", \"setup_s\": " << mx[2]
                        << ", \"read_s\": " << sm[1] << ", \"h2d_s\": " << sm[2] << ", \"wait_read_s\": " << sm[3]
                        << ", \"wait_copy_s\": " << sm[4] << ", \"ranks\": " << size
                        << ", \"parallel_read\": " << ((cfg.parallel_read || size == 1) ? "true" : "false")
                        << ", \"rank0\": {\"load_s\": " << lstats.wall_s << ", \"setup_s\": " << lstats.setup_s
                        << ", \"read_s\": " << lstats.read_s
                        << ", \"h2d_s\": " << lstats.h2d_s << ", \"blocks\": " << lstats.blocks
                        << ", \"rows_per_block\": " << lstats.rows_per_block
                        << ", \"rows_per_read\": " << lstats.rows_per_read
                        << ", \"staging_MB\": " << lstats.staging_bytes / 1048576.0
                        << ", \"rss_hwm_before_MB\": " << lstats.rss_hwm_before_mb
                        << ", \"rss_hwm_after_malloc_MB\": " << lstats.rss_after_malloc_mb
                        << ", \"rss_hwm_after_memset_MB\": " << lstats.rss_after_memset_mb
                        << ", \"rss_hwm_after_pinned_MB\": " << lstats.rss_after_pinned_mb
                        << ", \"rss_hwm_after_setup_MB\": " << lstats.rss_after_setup_mb
                        << ", \"rss_hwm_after_first_read_MB\": " << lstats.rss_after_first_read_mb
                        << ", \"rss_hwm_after_MB\": " << lstats.rss_hwm_after_mb << "}"
                        << ", \"rss_growth_MB_max\": " << mx[1] << ", \"shard_MB_max\": " << mx[3] / 1048576.0
                        << ", \"sparse\": " << (in.has_sparse ? "true" : "false")
                        << ", \"rtm_format\": \"" << (sparse ? "sparse" : "dense") << "\""
                        << ", \"nnz\": " << (sparse ? (gpu ? sshard->nnz : cpu_nnz) : 0) << ", \"driver\": \"native\"}\n";
        }

        std::vector<uint64_t> frames;
        for (uint64_t i = 0; i < image.nframe(); ++i)
            if (image.frame_time(i) > skip_until + 1e-12) frames.push_back(i);
        const size_t nframes_total = frames.size();
        const auto t_loop = std::chrono::steady_clock::now();
        if (batched) {
            // --batch_frames N: N slots on the matrix cores, refilled on the device (MultiFrameEngine::solve_series):
            // the sweep in which a frame finishes admits the next staged frame into its slot. The whole series is one
            // stream: a reader thread keeps up to 4 N frames read ahead, the engine stages them into its device queue
            // while earlier frames sweep, and finished frames (out of order) are written in time order. Without
            // --no_guess the frames form a warm-started time series -- each starts from the current iterate of the
            // newest frame in flight, rescaled (the resumed solution starts the first ones); with --no_guess every
            // frame cold-starts.
            const int64_t nfr = (int64_t)frames.size();
            const int64_t ahead = 4 * (int64_t)cfg.batch_frames;
            std::vector<double> bwarm = cfg.no_guess ? std::vector<double>() : warm;
            std::mutex mu, io_mu;
            std::condition_variable cv;
            std::map<int64_t, std::vector<double>> ready;  // frames read ahead, by series index
            int64_t consumed = 0, reader_next = 0;
            double reader_ms = 0.0, sink_ms = 0.0;  // (--profile: the reader thread's frame reads, rank 0's writes)
            bool stop = false;
            std::exception_ptr read_err;
            std::thread reader([&] {
                try {
                    for (int64_t k = 0; k < nfr; ++k) {
                        {
                            std::unique_lock<std::mutex> lk(mu);
                            cv.wait(lk, [&] { return stop || k < consumed + ahead; });
                            if (stop) return;
                        }
                        std::vector<double> f;
                        const auto tr = std::chrono::steady_clock::now();
                        {
                            std::lock_guard<std::mutex> io(io_mu);
                            f = image.frame(frames[k]);
                        }
                        const double rms =
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count();
                        std::lock_guard<std::mutex> lk(mu);
                        reader_ms += rms;
                        ready.emplace(k, std::move(f));
                        reader_next = k + 1;
                        cv.notify_all();
                    }
                } catch (...) {
                    std::lock_guard<std::mutex> lk(mu);
                    read_err = std::current_exception();
                    stop = true;
                    cv.notify_all();
                }
            });
            struct ReaderJoin {
                std::thread& t;
                std::mutex& m;
                std::condition_variable& c;
                bool& stop;
                ~ReaderJoin() {
                    {
                        std::lock_guard<std::mutex> lk(m);
                        stop = true;
                    }
                    c.notify_all();
                    if (t.joinable()) t.join();
                }
            } join_reader{reader, mu, cv, stop};
            // A cold time series: its first frame is solved alone by the single-frame engine (the fused sweep, half
            // the time of a batched sweep) and starts the chain as a converged source -- frames chained from a cold
            // start's young iterates would carry its error for ~100 frames (profiles/series_r6_*). SART_MF_LEAD_ENGINE=0:
            // the multi-frame engine's own lead frame instead (MfQueue::lead).
            int64_t off = 0;
            int lead_iters = -1;
            if (lead_engine && bwarm.empty() && nfr > 0) {
                const auto t0 = std::chrono::steady_clock::now();
                std::vector<double> g0, x0s(in.nvoxel);
                {  // frame 0 from the reader thread (which goes on reading the next frames meanwhile)
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return read_err || ready.count(0); });
                    if (read_err) std::rethrow_exception(read_err);
                    g0 = std::move(ready[0]);
                    ready.erase(0);
                    consumed = 1;
                    cv.notify_all();
                }
                SolveInfo info = lead_engine->solve(g0.data(), nullptr, x0s.data());
                lead_engine.reset();
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                if (rank == 0 && !(lead_tol > 1.0)) {
                    writer->add(x0s, info.status, image.frame_time(frames[0]), image.camera_frame_time(frames[0]),
                                info.iterations);
                    std::cout << "Processed in: " << ms << " ms" << std::endl;
                    if (profile.is_open())
                        profile << "{\"frame\": " << frames[0] << ", \"time\": " << image.frame_time(frames[0])
                                << ", \"status\": " << info.status << ", \"iterations\": " << info.iterations
                                << ", \"convergence\": " << info.convergence << ", \"ms\": " << ms
                                << ", \"batch\": " << cfg.batch_frames << ", \"warm_from\": -1, \"warm_iter\": -1"
                                << ", \"lead\": true, \"fused\": " << (info.used_fused ? "true" : "false")
                                << ", \"driver\": \"native\"}\n";
                }
                if (std::all_of(x0s.begin(), x0s.end(), [](double v) { return std::isfinite(v); })) bwarm = x0s;
                lead_iters = info.iterations;
                // handover (lead_tol > 1): frame 0 is solved on in the batch from this iterate (its reported update
                // count includes the lead's), as are the first frames chained from it; else the lead is frame 0
                off = (lead_tol > 1.0 && !bwarm.empty()) ? 0 : 1;
            }
            lead_engine.reset();  // (a resumed series starts from the stored solution instead)
            const size_t npix = (size_t)mf->nrows();
            auto src = [&](int64_t j, double* dst) {  // series index j = frame off + j
                const int64_t k = j + off;
                std::vector<double> f;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return read_err || ready.count(k) || k < reader_next; });
                    if (read_err) std::rethrow_exception(read_err);
                    auto it = ready.find(k);
                    if (it != ready.end()) {
                        f = std::move(it->second);
                        ready.erase(it);
                    }
                    consumed = std::max(consumed, k + 1);
                    cv.notify_all();
                }
                if (f.empty()) {  // asked again (a re-solve after a device all-reduce failure): read it here
                    std::lock_guard<std::mutex> io(io_mu);
                    f = image.frame(frames[k]);
                }
                if (f.size() != npix) throw std::runtime_error("frame size does not match the shard's pixels");
                std::copy(f.begin(), f.end(), dst);
            };
            // rank 0: finished frames written in time order
            std::map<int64_t, std::pair<std::vector<double>, SolveInfo>> done;
            int64_t written = off;
            auto t_prev = std::chrono::steady_clock::now();
            auto sink = [&](int64_t j, const double* xs, const SolveInfo& info) {
                if (rank != 0) return;
                const auto tsk = std::chrono::steady_clock::now();
                struct Acc {
                    double& ms;
                    std::chrono::steady_clock::time_point t;
                    ~Acc() { ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count(); }
                } acc{sink_ms, tsk};
                SolveInfo fi = info;
                if (fi.warm_from >= 0) {
                    fi.warm_from += (int)off;
                } else if (lead_iters >= 0 && j + off == 0) {  // the lead frame, finished in the batch (handover)
                    fi.iterations += lead_iters;
                } else if (lead_iters >= 0) {  // started from the lead frame's solution / handed-over iterate
                    fi.warm_from = 0;
                    fi.warm_iter = lead_iters;
                    fi.warm_live = false;
                }
                done.emplace(j + off, std::make_pair(std::vector<double>(xs, xs + in.nvoxel), fi));
                for (auto it = done.find(written); it != done.end(); it = done.find(written)) {
                    const uint64_t cur = frames[written];
                    const SolveInfo& fi = it->second.second;
                    writer->add(it->second.first, fi.status, image.frame_time(cur), image.camera_frame_time(cur),
                                fi.iterations);
                    const auto now = std::chrono::steady_clock::now();
                    const double ms = std::chrono::duration<double, std::milli>(now - t_prev).count();
                    t_prev = now;
                    std::cout << "Processed in: " << ms << " ms" << std::endl;
                    if (fi.nonfinite) std::cerr << "warning: frame " << cur << ": non-finite iterate, stopped" << std::endl;
                    if (profile.is_open())
                        profile << "{\"frame\": " << cur << ", \"time\": " << image.frame_time(cur)
                                << ", \"status\": " << fi.status << ", \"iterations\": " << fi.iterations
                                << ", \"convergence\": " << fi.convergence << ", \"ms\": " << ms
                                << ", \"batch\": " << cfg.batch_frames << ", \"warm_from\": "
                                << (fi.warm_from >= 0 ? (int64_t)frames[fi.warm_from] : -1)
                                << ", \"warm_iter\": " << fi.warm_iter << ", \"warm_live\": " << (fi.warm_live ? 1 : 0)
                                << ", \"comm_fallbacks\": " << fi.comm_fallbacks
                                << ", \"driver\": \"native\"}\n";
                    done.erase(it);
                    ++written;
                }
            };
            mf->solve_series(nfr - off, src, sink, bwarm.empty() ? nullptr : bwarm.data(), !cfg.no_guess);
            if (rank == 0 && profile.is_open()) {
                const auto& ss = mf->series_stats();
                profile << "{\"series\": true, \"frames\": " << ss.frames << ", \"sweeps\": " << ss.sweeps
                        << ", \"queued_sweeps\": " << ss.queued_sweeps << ", \"slot_util\": " << ss.slot_util
                        << ", \"mean_iterations\": " << ss.mean_iterations << ", \"chained\": " << ss.chained
                        << ", \"mean_warm_age\": " << ss.mean_warm_age << ", \"series_ms\": " << ss.ms
                        << ", \"chunk\": " << ss.chunk << ", \"admit_cap\": " << ss.admit_cap
                        << ", \"src_age\": " << ss.src_age << ", \"src_finished\": " << (ss.src_finished ? 1 : 0)
                        << ", \"lead\": " << (ss.lead ? 1 : 0) << ", \"src_extrap\": " << ss.src_extrap << ", \"drift\": " << ss.drift
                        << ", \"restarts\": " << ss.restarts << ", \"host_wait_ms\": " << ss.host_wait_ms
                        << ", \"host_stage_ms\": " << ss.host_stage_ms << ", \"host_src_ms\": " << ss.host_src_ms
                        << ", \"host_deliver_ms\": " << ss.host_deliver_ms << ", \"reader_ms\": " << reader_ms
                        << ", \"sink_ms\": " << sink_ms
                        << ", \"batch\": " << mf->batch_frames() << ", \"driver\": \"native\"}\n";
            }
            frames.clear();
        }
        if (cols && !warm.empty())  // this rank's voxels of the stored solution
            warm = std::vector<double>(warm.begin() + vblk.offset, warm.begin() + vblk.offset + vblk.size);
        std::vector<double> solution = warm, x(vblk.size), xfull(cols ? in.nvoxel : 0);
        const char* wd = std::getenv("SART_WARM_ON_DEVICE");
        const bool warm_dev = !(wd && *wd && std::atoi(wd) == 0);
        std::future<std::vector<double>> fut;
        if (!frames.empty()) fut = std::async(std::launch::async, [&image, i = frames[0]]() { return image.frame(i); });
        for (size_t k = 0; k < frames.size(); ++k) {
            const uint64_t cur = frames[k];
            const auto tf = std::chrono::steady_clock::now();
            std::vector<double> frame = fut.get();
            const double wait_frame_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf).count();
            if (k + 1 < frames.size())  // prefetch the next composite frame during the solve
                fut = std::async(std::launch::async, [&image, i = frames[k + 1]]() { return image.frame(i); });
            const auto t0 = std::chrono::steady_clock::now();
            const double* x0 = (cfg.no_guess || solution.empty()) ? nullptr : solution.data();
            // from frame 1 on, a warm start is the engine's own previous solution: rescaled on the device
            // (SART_WARM_ON_DEVICE=0: through the host copy, for A/B runs)
            const SolveInfo info = gpu ? engine->solve(frame.data(), x0, x.data(), k > 0 && x0 != nullptr && warm_dev)
                                       : cpu->solve(frame.data(), x0, x.data());
            if (info.fallbacks)
                std::cerr << "warning: fused sweep fell back " << info.fallbacks << " time(s)" << std::endl;
            if (info.comm_fallbacks && rank == 0)
                std::cerr << "warning: frame " << cur << ": device all-reduce timed out; re-solved on "
                          << (dcomm ? dcomm->backend() : "the base communicator") << std::endl;
            if (info.nonfinite) std::cerr << "warning: frame " << cur << ": non-finite iterate, stopped" << std::endl;
            solution = x;
            if (cols) {  // gather the voxel blocks (zero-filled sum over ranks)
                std::fill(xfull.begin(), xfull.end(), 0.0);
                std::copy(x.begin(), x.end(), xfull.begin() + vblk.offset);
                host->all_reduce_host(xfull.data(), xfull.size(), ReduceOp::kSum);
            }
            if (rank == 0) {
                const auto tw = std::chrono::steady_clock::now();
                writer->add(cols ? xfull : x, info.status, image.frame_time(cur), image.camera_frame_time(cur),
                            info.iterations);
                const auto t1 = std::chrono::steady_clock::now();
                const double writer_ms = std::chrono::duration<double, std::milli>(t1 - tw).count();
                const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
                std::cout << "Processed in: " << ms << " ms" << std::endl;  // reference main.cpp:132-137
                if (profile.is_open())
                {
                    // throughput of the solve (4 P V flop and one or two reads of every rank's shard per sweep)
                    const double sweeps = gpu ? (double)info.sweeps : (double)info.iterations;
                    const double secs = info.ms > 0 ? 1e-3 * info.ms : 1e-3 * ms;
                    const double pv = (double)in.npixel * (double)in.nvoxel;
                    const double reads = gpu && info.used_fused ? 1.0 : 2.0;
                    const double elem = gpu && cfg.rtm_bf16 ? 2.0 : 4.0;  // bytes per stored RTM element
                    profile << "{\"frame\": " << cur << ", \"time\": " << image.frame_time(cur)
                            << ", \"status\": " << info.status << ", \"iterations\": " << info.iterations
                            << ", \"convergence\": " << info.convergence << ", \"sweeps\": " << sweeps
                            << ", \"iters_per_s\": " << sweeps / secs << ", \"gflops\": " << 4.0 * pv * sweeps / secs / 1e9
                            << ", \"rtm_GBps\": " << reads * elem * pv * sweeps / secs / 1e9
                            << ", \"comm_ms\": " << info.comm_ms << ", \"comm_fallbacks\": " << info.comm_fallbacks
                            << ", \"ms\": " << ms << ", \"solve_ms\": " << info.ms
                            << ", \"setup_ms\": " << info.setup_ms << ", \"iterate_ms\": " << info.iterate_ms
                            << ", \"finish_ms\": " << info.finish_ms << ", \"writer_ms\": " << writer_ms
                            << ", \"queued_sweeps\": " << info.queued_sweeps << ", \"wait_frame_ms\": " << wait_frame_ms
                            << ", \"fused\": " << (info.used_fused ? "true" : "false")
                            << ", \"ranks\": " << size << ", \"comm\": \"" << json_escape(host->backend())
                            << "\", \"device_comm\": \"" << json_escape(dcomm ? dcomm->describe() : "none")
                            << "\", \"driver\": \"" << json_escape("native") << "\"}\n";
                }
            }
            // --no_guess, or a frame whose iterate stayed non-finite (the NaN/Inf guard returned the last finite
            // iterate when there was one): the next frame cold-starts instead of inheriting NaN
            if (cfg.no_guess ||
                (info.nonfinite && !std::all_of(x.begin(), x.end(), [](double v) { return std::isfinite(v); })))
                solution.clear();
        }
        if (rank == 0) {
            writer->flush();
            if (!appended) voxelgrid.write(cfg.output_file, "voxel_map");
            // the whole frame loop (reads not hidden by the prefetch, solves, output, the final flush)
            if (nframes_total) {
                const double loop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_loop).count();
                std::cout << "Frames processed: " << nframes_total << " in " << loop_s << " s ("
                          << nframes_total / loop_s << " frames/s)" << std::endl;
            }
        }
        host->barrier();
    } catch (const std::exception& e) {
        std::cerr << "rank " << rank << ": " << e.what() << std::endl;
        if (dcomm) dcomm->abort();
        else if (host) host->abort();
        std::fflush(nullptr);
        std::_Exit(1);
    }
    return 0;
}
