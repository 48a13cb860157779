#include "comm.hpp"

#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <thread>
#include <vector>

#include "../kernels/launchers.hpp"

namespace sart {

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void nccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

class LocalComm final : public Communicator {
   public:
    LocalComm() : host_(make_local_host_comm()) {}
    HostComm& host() override { return *host_; }
    const char* backend() const override { return "local"; }
    void all_reduce(float*, size_t, ReduceOp, hipStream_t) override {}
    void all_reduce(double*, size_t, ReduceOp, hipStream_t) override {}
    bool graph_capturable() const override { return true; }

   private:
    std::unique_ptr<HostComm> host_;
};

class StagedComm final : public Communicator {
   public:
    explicit StagedComm(std::unique_ptr<HostComm> h, std::string note = "") : host_(std::move(h)), note_(std::move(note)) {}
    HostComm& host() override { return *host_; }
    const char* backend() const override { return "staged"; }
    std::string describe() const override { return note_.empty() ? std::string("staged") : "staged (" + note_ + ")"; }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t s) override { staged(dev, n, op, s); }
    void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t s) override { staged(dev, n, op, s); }

   private:
    template <typename T>
    void staged(T* dev, size_t n, ReduceOp op, hipStream_t stream) {
        if (host_->size() == 1 || n == 0) return;
        std::vector<T> h(n);
        hip_ok(hipMemcpyAsync(h.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost, stream), "staged D2H");
        hip_ok(hipStreamSynchronize(stream), "staged sync");
        host_->all_reduce_host(h.data(), n, op);
        hip_ok(hipMemcpyAsync(dev, h.data(), n * sizeof(T), hipMemcpyHostToDevice, stream), "staged H2D");
        hip_ok(hipStreamSynchronize(stream), "staged sync");
    }
    std::unique_ptr<HostComm> host_;
    std::string note_;
};

class RcclComm final : public Communicator {
   public:
    explicit RcclComm(std::unique_ptr<HostComm> boot) : host_(std::move(boot)) {}
    // The communicator of this rank, brought up NON-blocking (ncclConfig_t::blocking = 0) and polled against a
    // deadline (SART_RCCL_INIT_TIMEOUT_S, default 120 s): a peer that never enters the init (crashed, hung, or the
    // SART_FAULT_RCCL_INIT_SKIP fault) makes this rank abort its half-built communicator and report failure instead
    // of blocking forever in ncclCommInitRank. "" on success, else the error (the communicator stays unusable).
    std::string init(int device, const std::string& uid, double timeout_s) {
        try {
            if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: bad unique id");
            ncclUniqueId id;
            std::memcpy(&id, uid.data(), sizeof(id));
            hip_ok(hipSetDevice(device), "hipSetDevice");
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            const ncclResult_t r = ncclCommInitRankConfig(&comm_, host_->size(), id, host_->rank(), &cfg);
            if (r != ncclSuccess && r != ncclInProgress) nccl_ok(r, "ncclCommInitRankConfig");
            if (!comm_) throw std::runtime_error("ncclCommInitRankConfig: no communicator");
            wait_ready(timeout_s, "ncclCommInitRankConfig");
        } catch (const std::exception& e) {
            if (comm_) (void)ncclCommAbort(comm_);  // (abort: a destroy would wait for the peers)
            comm_ = nullptr;
            return e.what();
        }
        return "";
    }
    // a non-blocking communicator's call may return before its work is enqueued (ncclInProgress): poll to a deadline
    void wait_ready(double timeout_s, const char* what) {
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
        for (;;) {
            ncclResult_t st = ncclInProgress;
            nccl_ok(ncclCommGetAsyncError(comm_, &st), "ncclCommGetAsyncError");
            if (st == ncclSuccess) return;
            if (st != ncclInProgress) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(st));
            if (std::chrono::steady_clock::now() > deadline)
                throw std::runtime_error(std::string(what) + ": not complete after " + std::to_string((int)timeout_s) +
                                         " s (a peer never joined?)");
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    void destroy() {
        if (comm_) (void)ncclCommDestroy(comm_);
        comm_ = nullptr;
    }
    std::unique_ptr<HostComm> take_host() { return std::move(host_); }
    ~RcclComm() override { destroy(); }
    HostComm& host() override { return *host_; }
    const char* backend() const override { return "rccl"; }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        if (n) enqueued(ncclAllReduce(dev, dev, n, ncclFloat32, nop(op), comm_, stream));
    }
    void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        if (n) enqueued(ncclAllReduce(dev, dev, n, ncclFloat64, nop(op), comm_, stream));
    }
    bool graph_capturable() const override { return true; }
    void abort() override {
        if (comm_) {
            (void)ncclCommAbort(comm_);
            comm_ = nullptr;
        }
        host_->abort();
    }

   private:
    static ncclRedOp_t nop(ReduceOp op) { return op == ReduceOp::kSum ? ncclSum : ncclMax; }
    void enqueued(ncclResult_t r) {  // (the first collective connects the peers: bounded like the init)
        if (r == ncclInProgress)
            wait_ready(env_seconds("SART_RCCL_INIT_TIMEOUT_S", 120.0), "ncclAllReduce");
        else
            nccl_ok(r, "ncclAllReduce");
    }
    static double env_seconds(const char* name, double dflt) {
        const char* e = std::getenv(name);
        return (e && *e) ? std::atof(e) : dflt;
    }
    std::unique_ptr<HostComm> host_;
    ncclComm_t comm_ = nullptr;
};


// ---- p2p: one-shot push all-reduce through IPC-mapped peer buffers (csrc/kernels/p2p_allreduce.hip) ----
double env_double(const char* name, double dflt) {
    const char* e = std::getenv(name);
    return (e && *e) ? std::atof(e) : dflt;
}

}  // namespace

void Communicator::reduce_all_reduce(const ReduceSrc& src, float* out, hipStream_t stream) {
    launch_reduce_partials(src.partial, src.ld, src.nsplit, src.scale, out, src.Fpart, src.nF, out + src.ld, src.st,
                           stream);
    all_reduce(out, (size_t)src.ld + 2, ReduceOp::kSum, stream);
}

namespace {

class P2pComm final : public Communicator {
   public:
    P2pComm(int device, std::shared_ptr<Communicator> base) : base_(std::move(base)), device_(device) {
        const auto t0 = std::chrono::steady_clock::now();
        HostComm& h = base_->host();
        rank_ = h.rank();
        n_ = h.size();
        const char* m = std::getenv("SART_P2P");
        mode_ = (m && *m) ? m : "auto";
        cap_ = std::max<int64_t>(1024, (int64_t)(env_double("SART_P2P_MAX_BYTES", 2.0 * 1024 * 1024) / 4) / 4 * 4);
        // a healthy peer is at most a few sweeps behind (the host collectives of every frame's setup align the
        // ranks first), so a P2P wait this long means the peer is gone or stuck: the engines then switch to the
        // base communicator and re-solve the frame (device_failed / degrade)
        timeout_s_ = env_double("SART_P2P_TIMEOUT_S", 60.0);
        // start-up calls (self-test, probes) give up sooner: a failure there only means "no P2P"
        setup_timeout_s_ = std::min(timeout_s_, env_double("SART_P2P_SETUP_TIMEOUT_S", 10.0));
        if (const char* f = std::getenv("SART_P2P_FUSED_REDUCE"); f && *f) fused_reduce_ = std::atoi(f) != 0;
        if (const char* f = std::getenv("SART_P2P_FUSED_UPDATE"); f && *f) fused_update_ = std::atoi(f) != 0;
        if (const char* f = std::getenv("SART_FAULT_P2P"); f && *f) {
            const char* fr = std::getenv("SART_FAULT_RANK");
            if (!(fr && *fr) || std::atoi(fr) == rank_) fault_call_ = std::atoll(f);
        }
        if (mode_ == "0" || mode_ == "off") {
            finish(false, "p2p off (SART_P2P=0)");
            return;
        }
        if (n_ < 2 || n_ > kP2pMaxRanks) {
            finish(false, "p2p needs 2.." + std::to_string(kP2pMaxRanks) + " ranks");
            return;
        }
        if (!agree(same_host())) {
            finish(false, "p2p off: ranks span several hosts");
            return;
        }
        hip_ok(hipSetDevice(device_), "hipSetDevice");
        // Ranks sharing one GPU (one-GPU rehearsals): every P2P workgroup spins until its peers' chunks arrive, so
        // the spinning workgroups of all ranks together must leave the CUs their peers' persistent sweeps need:
        // 32 / (ranks per GPU) workgroups per call (4 at 8 ranks). One rank per GPU: up to kP2pMaxBlocks.
        rpd_ = ranks_sharing_device(h, device_);
        args_.max_blocks = rpd_ > 1 ? std::max(1, 32 / rpd_) : kP2pMaxBlocks;
        if (rpd_ > 1 && rank_ == 0) {
            // the GPU maps 24 compute queues at once (KFD num_cp_queues); more and the processes are time-sliced, and
            // a P2P call then waits out a time slice for a descheduled peer (measured 10.3 ms instead of 111 us at 8
            // ranks with HIP's default 4 queues per process: profiles/bench_r4_n8_rehearsal_one_gpu_q{4,1}.json)
            const char* q = std::getenv("GPU_MAX_HW_QUEUES");
            const int hwq = (q && *q) ? std::atoi(q) : 4;
            if (rpd_ * hwq > 24)
                std::fprintf(stderr, "sart: %d ranks share one GPU with %d hardware queues each (%d > 24 mapped at once): "
                             "processes are time-sliced; set GPU_MAX_HW_QUEUES=%d\n", rpd_, hwq, rpd_ * hwq,
                             std::max(1, 12 / rpd_));
        }
        if (const char* b = std::getenv("SART_P2P_BLOCKS"); b && *b) args_.max_blocks = std::max(1, std::atoi(b));
        hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
        const bool mapped = agree(map_peers());
        t_map_ = seconds_since(t0);
        if (!mapped) {
            finish(false, "p2p off: IPC mapping failed (" + err_msg_ + ")");
            return;
        }
        const auto t1 = std::chrono::steady_clock::now();
        const bool tested = self_test();
        t_test_ = seconds_since(t1);
        if (!tested) {
            finish(false, "p2p off: self-test failed (" + (err_msg_.empty() ? "on another rank" : err_msg_) + ")");
            return;
        }
        if (mode_ == "1" || mode_ == "on") {
            finish(true, "p2p (forced, self-test ok)");
            return;
        }
        finish(true, "p2p self-test ok; auto: sizes the engine announces are timed against " +
                         std::string(base_->backend()));
    }
    ~P2pComm() override {
        (void)hipSetDevice(device_);
        if (stream_) (void)hipStreamSynchronize(stream_);
        for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
        if (mem_) (void)hipFree(mem_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }
    HostComm& host() override { return base_->host(); }
    const char* backend() const override { return active_ ? "p2p" : base_->backend(); }
    std::string describe() const override {
        char buf[160];
        std::snprintf(buf, sizeof(buf), " [p2p setup %.0f ms: map %.0f, self-test %.0f, probes %.0f; %d ranks/GPU, %d blocks]",
                      1e3 * setup_seconds(), 1e3 * t_map_, 1e3 * t_test_, 1e3 * t_probe_, rpd_, args_.max_blocks);
        std::string table;
        for (const auto& p : probes_) {
            char cell[96];
            std::snprintf(cell, sizeof(cell), "%s%lld: %.1f/%.1f", table.empty() ? "" : ", ", (long long)p.n, p.us_p2p,
                          p.us_base);
            table += cell;
        }
        std::string sel = why_;
        if (active_ && auto_mode()) {
            std::string won;
            for (const auto& p : probes_)
                if (p.p2p) won += (won.empty() ? "" : ",") + std::to_string(p.n);
            sel = won.empty() ? std::string(base_->backend()) + " (auto: p2p won at no announced size)"
                              : "p2p at floats " + won + ", " + base_->backend() + " otherwise (auto)";
        }
        if (!table.empty()) sel += " (rank 0, us p2p/" + std::string(base_->backend()) + " at floats " + table + ")";
        const std::string bd = base_->describe();
        if (bd != base_->backend()) sel += "; base: " + bd;  // e.g. staged after a failed RCCL bring-up
        return sel + buf;
    }
    double setup_seconds() const override { return t_map_ + t_test_ + t_probe_; }
    void prepare(const std::vector<int64_t>& sizes) override {
        if (!active_ || !auto_mode()) return;
        std::vector<int64_t> todo;
        for (int64_t n : sizes)
            if (n > 0 && n <= cap_ && !probed(n) && std::find(todo.begin(), todo.end(), n) == todo.end())
                todo.push_back(n);
        // every rank must probe the same sizes in the same order: agree on the count (a mismatch is a caller bug)
        double cnt[2] = {(double)todo.size(), -(double)todo.size()};
        base_->host().all_reduce_host(cnt, 2, ReduceOp::kMax);
        if (cnt[0] != -cnt[1]) throw std::runtime_error("p2p prepare: ranks announced different message sizes");
        if (todo.empty()) return;
        const auto t0 = std::chrono::steady_clock::now();
        std::sort(todo.begin(), todo.end());
        std::vector<double> us(2 * todo.size(), 0.0);
        for (size_t i = 0; i < todo.size(); ++i) {
            const int64_t n = todo[i];
            us[2 * i] = time_us([&](float* b) { p2p(b, n, 0, stream_, setup_timeout_s_); }, n);
            us[2 * i + 1] = time_us([&](float* b) { base_->all_reduce(b, (size_t)n, ReduceOp::kSum, stream_); }, n);
        }
        base_->host().broadcast_host(us.data(), us.size() * sizeof(double), 0);  // rank 0 decides
        // a probe call that timed out on any rank leaves that rank's device path failed: P2P off everywhere
        const bool ok = agree(err_words().first == 0);
        for (size_t i = 0; i < todo.size(); ++i)
            probes_.push_back(Probe{todo[i], us[2 * i], us[2 * i + 1], ok && us[2 * i] < us[2 * i + 1]});
        std::sort(probes_.begin(), probes_.end(), [](const Probe& a, const Probe& b) { return a.n < b.n; });
        t_probe_ += seconds_since(t0);
        if (!ok) {
            active_ = false;
            why_ = std::string(base_->backend()) + " (p2p off: a probe call timed out)";
        }
    }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        // the choice depends only on n (identical on every rank), never on this rank's pointer alignment
        if (use_p2p((int64_t)n)) {
            // SART_FAULT_P2P=k (tests): from its k-th P2P all-reduce on, this process raises no flags (a peer whose
            // device path stopped; a single missing flag would heal at the next call, flags being monotonic), only
            // on SART_FAULT_RANK when that is set
            const bool skip = fault_call_ > 0 && ++calls_ >= fault_call_;
            p2p(dev, (int64_t)n, op == ReduceOp::kSum ? 0 : 1, stream, -1.0, skip);
        } else
            base_->all_reduce(dev, n, op, stream);
    }
    void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        base_->all_reduce(dev, n, op, stream);
    }
    void reduce_all_reduce(const ReduceSrc& src, float* out, hipStream_t stream) override {
        // SART_P2P_FUSED_REDUCE=0: two launches (the A/B baseline); same fault injection as all_reduce
        if (fused_reduce_ && use_p2p(src.ld + 2)) {
            const bool skip = fault_call_ > 0 && ++calls_ >= fault_call_;
            launch_p2p_reduce_allreduce(src, out, args_, rank_, n_, ++epoch_, cap_, err_, timeout_s_, stream, skip);
        } else {
            Communicator::reduce_all_reduce(src, out, stream);
        }
    }
    bool reduce_all_reduce_update(const ReduceSrc& src, float* out, const UpdateArgs& upd, hipStream_t stream) override {
        // SART_P2P_FUSED_UPDATE=0: the update in its own launch (the A/B baseline); same fault injection as all_reduce
        if (fused_reduce_ && fused_update_ && use_p2p(src.ld + 2)) {
            const bool skip = fault_call_ > 0 && ++calls_ >= fault_call_;
            launch_p2p_reduce_allreduce(src, out, args_, rank_, n_, ++epoch_, cap_, err_, timeout_s_, stream, skip,
                                        &upd);
            return true;
        }
        reduce_all_reduce(src, out, stream);
        return false;
    }
    bool graph_capturable() const override { return !active_ && base_->graph_capturable(); }  // epoch is an argument
    void abort() override {
        // tell every peer: their P2P kernels stop polling for this rank at once instead of at the timeout
        const unsigned one = 1;
        for (int r = 0; r < n_; ++r)
            if (r != rank_ && tail_[r]) (void)hipMemcpy(tail_[r] + 1, &one, sizeof(one), hipMemcpyHostToDevice);
        base_->abort();
    }
    void check() override {
        if (err_ && active_) {
            const auto e = err_words();
            if (e.second) throw std::runtime_error("p2p all-reduce: a peer aborted");
            if (e.first) throw std::runtime_error("p2p all-reduce: a peer did not arrive within SART_P2P_TIMEOUT_S");
        }
        base_->check();
    }
    bool device_failed() override {
        if (!err_ || !active_) return false;
        const auto e = err_words();
        return e.first != 0 && e.second == 0;  // a timeout; a peer's abort is fatal (check() throws)
    }
    bool degradable() const override { return active_; }
    bool degrade() override {
        if (!active_) return false;
        why_ = std::string(base_->backend()) + " (p2p disabled after a p2p all-reduce timeout; was: " + describe() + ")";
        active_ = false;
        return true;
    }

   private:
    struct Probe {
        int64_t n;
        double us_p2p, us_base;
        bool p2p;
    };
    static double seconds_since(std::chrono::steady_clock::time_point t0) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    bool auto_mode() const { return !(mode_ == "1" || mode_ == "on"); }
    bool probed(int64_t n) const {
        for (const auto& p : probes_)
            if (p.n == n) return true;
        return false;
    }
    // forced: every vector that fits the slots; auto: the decision at the smallest probed size >= n (a vector a
    // few floats shorter than a probed one, e.g. the cold start's ld next to the sweep's ld + 2, goes the same way)
    bool use_p2p(int64_t n) const {
        if (!active_ || n <= 0 || n > cap_) return false;
        if (!auto_mode()) return true;
        for (const auto& p : probes_)  // sorted by n
            if (p.n >= n) return p.p2p;
        return false;
    }
    std::pair<unsigned, unsigned> err_words() {  // {timeout, abort}
        unsigned e[2] = {0, 0};
        if (err_) hip_ok(hipMemcpy(e, err_, sizeof(e), hipMemcpyDeviceToHost), "p2p error word");
        return {e[0], e[1]};
    }
    void finish(bool active, const std::string& why) {
        active_ = active;
        why_ = why;
    }
    bool agree(bool ok) {  // every rank learns whether all succeeded
        double bad = ok ? 0.0 : 1.0;
        base_->host().all_reduce_host(&bad, 1, ReduceOp::kMax);
        return bad == 0.0;
    }
    bool same_host() {
        char mine[256] = {0};
        (void)gethostname(mine, sizeof(mine) - 1);
        bool same = true;
        for (int r = 0; r < n_; ++r) {
            char other[256];
            std::memcpy(other, mine, sizeof(mine));
            base_->host().broadcast_host(other, sizeof(other), r);
            same = same && std::memcmp(other, mine, sizeof(mine)) == 0;
        }
        return same;
    }
    bool map_peers() {
        const size_t recv_bytes = (size_t)2 * kP2pMaxRanks * (size_t)cap_ * sizeof(float);
        const size_t flag_bytes = (size_t)kP2pMaxRanks * kP2pMaxBlocks * sizeof(unsigned);
        hipIpcMemHandle_t hdl;
        std::memset(&hdl, 0, sizeof(hdl));
        bool ok = true;
        try {
            hip_ok(hipExtMallocWithFlags(&mem_, recv_bytes + flag_bytes + 256, hipDeviceMallocUncached),
                   "hipExtMallocWithFlags(uncached)");
            hip_ok(hipMemset(mem_, 0, recv_bytes + flag_bytes + 256), "hipMemset");
            hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
            err_ = reinterpret_cast<unsigned*>(static_cast<char*>(mem_) + recv_bytes + flag_bytes);
            args_.abort_word = err_ + 1;
            hip_ok(hipIpcGetMemHandle(&hdl, mem_), "hipIpcGetMemHandle");
        } catch (const std::exception& e) {
            ok = false;
            err_msg_ = e.what();
        }
        // every rank's handle in one gather (a sum of one nonzero slot per rank) instead of n broadcasts
        std::vector<unsigned char> all((size_t)n_ * sizeof(hdl), 0);
        std::memcpy(all.data() + (size_t)rank_ * sizeof(hdl), &hdl, sizeof(hdl));
        std::vector<double> words(all.size());
        for (size_t i = 0; i < all.size(); ++i) words[i] = all[i];
        base_->host().all_reduce_host(words.data(), words.size(), ReduceOp::kSum);
        for (int r = 0; r < n_ && ok; ++r) {
            hipIpcMemHandle_t h;
            for (size_t i = 0; i < sizeof(h); ++i)
                reinterpret_cast<unsigned char*>(&h)[i] = (unsigned char)words[(size_t)r * sizeof(h) + i];
            void* p = mem_;
            if (r != rank_) {
                if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    (void)hipGetLastError();
                    ok = false;
                    err_msg_ = "hipIpcOpenMemHandle of rank " + std::to_string(r);
                    break;
                }
                opened_.push_back(p);
            }
            args_.recv[r] = static_cast<float*>(p);
            args_.flags[r] = reinterpret_cast<unsigned*>(static_cast<char*>(p) + recv_bytes);
            tail_[r] = reinterpret_cast<unsigned*>(static_cast<char*>(p) + recv_bytes + flag_bytes);  // {err, abort}
        }
        return ok;  // the caller's agree() is also the barrier: every flag array is zeroed before any push
    }
    void p2p(float* dev, int64_t n, int op, hipStream_t stream, double timeout_s = -1, bool skip_flags = false) {
        launch_p2p_allreduce(dev, dev, n, args_, rank_, n_, ++epoch_, cap_, op, err_,
                             timeout_s > 0 ? timeout_s : timeout_s_, stream, skip_flags);
    }
    // Exact checks: integer-valued sums / maxima, and random fp32 data against the rank-order sum (the kernel's
    // result must be bitwise identical to ((v0 + v1) + v2) + ... on every rank). Every rank runs every call (a
    // failed call on one rank makes its later calls fail fast; its peers time out at most once, after
    // setup_timeout_s_), and the ranks agree once at the end.
    bool self_test() {
        float* d = nullptr;
        if (!agree(hipMalloc(reinterpret_cast<void**>(&d), (size_t)cap_ * sizeof(float)) == hipSuccess)) {
            (void)hipGetLastError();
            if (d) (void)hipFree(d);
            err_msg_ = "hipMalloc";
            return false;
        }
        const int64_t sizes[] = {1, 4099, std::min<int64_t>(cap_, 65537)};
        int call = 0;
        bool good = true;
        for (int64_t n : sizes) {
            for (int kind = 0; kind < 3; ++kind, ++call) {  // 0 integer sum, 1 integer max, 2 random fp32 sum
                try {
                    std::vector<float> mine((size_t)n), want((size_t)n), got((size_t)n);
                    for (int64_t i = 0; i < n; ++i) {
                        float acc = 0.f;
                        for (int r = 0; r < n_; ++r) {
                            const float v = value(kind, r, i, call);
                            if (r == rank_) mine[(size_t)i] = v;
                            acc = r == 0 ? v : (kind == 1 ? std::max(acc, v) : acc + v);
                        }
                        want[(size_t)i] = acc;
                    }
                    hip_ok(hipMemcpy(d, mine.data(), (size_t)n * sizeof(float), hipMemcpyHostToDevice), "H2D");
                    p2p(d, n, kind == 1 ? 1 : 0, stream_, setup_timeout_s_);
                    hip_ok(hipStreamSynchronize(stream_), "p2p self-test");
                    hip_ok(hipMemcpy(got.data(), d, (size_t)n * sizeof(float), hipMemcpyDeviceToHost), "D2H");
                    if (err_words().first) throw std::runtime_error("peer timeout");
                    if (std::memcmp(got.data(), want.data(), (size_t)n * sizeof(float)) != 0)
                        throw std::runtime_error("mismatch at n=" + std::to_string(n) + " kind " + std::to_string(kind));
                } catch (const std::exception& ex) {
                    if (good) err_msg_ = ex.what();
                    good = false;
                }
            }
        }
        (void)hipFree(d);
        return agree(good);
    }
    static float value(int kind, int r, int64_t i, int call) {
        if (kind < 2) return (float)((r + 1) * ((i * 7 + call) % 251));
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + (uint64_t)(r + 1) * 0xBF58476D1CE4E5B9ull + (uint64_t)call;
        z = (z ^ (z >> 31)) * 0x94D049BB133111EBull;
        return (float)((double)(z >> 40) / (double)(1ull << 24) * 2.0 - 1.0);
    }
    // mean microseconds per call over 10 calls after 2 warm-up calls (host barrier before timing)
    double time_us(const std::function<void(float*)>& f, int64_t n) {
        float* d = nullptr;
        hip_ok(hipMalloc(reinterpret_cast<void**>(&d), (size_t)n * sizeof(float)), "hipMalloc");
        hip_ok(hipMemset(d, 0, (size_t)n * sizeof(float)), "hipMemset");
        hip_ok(hipDeviceSynchronize(), "sync");
        for (int i = 0; i < 2; ++i) f(d);
        hip_ok(hipStreamSynchronize(stream_), "sync");
        base_->host().barrier();
        hipEvent_t e0, e1;
        hip_ok(hipEventCreate(&e0), "event");
        hip_ok(hipEventCreate(&e1), "event");
        hip_ok(hipEventRecord(e0, stream_), "event");
        for (int i = 0; i < 10; ++i) f(d);
        hip_ok(hipEventRecord(e1, stream_), "event");
        hip_ok(hipEventSynchronize(e1), "event");
        float ms = 0.f;
        hip_ok(hipEventElapsedTime(&ms, e0, e1), "event");
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipFree(d);
        return 1e3 * ms / 10.0;
    }

    std::shared_ptr<Communicator> base_;
    int device_ = 0, rank_ = 0, n_ = 1, rpd_ = 1;
    std::string mode_;
    int64_t cap_ = 0;
    std::vector<Probe> probes_;  // auto mode: announced sizes, sorted by n
    double timeout_s_ = 60.0, setup_timeout_s_ = 10.0;
    double t_map_ = 0.0, t_test_ = 0.0, t_probe_ = 0.0;
    int64_t fault_call_ = 0, calls_ = 0;  // SART_FAULT_P2P
    bool active_ = false;
    std::string why_, err_msg_;
    hipStream_t stream_ = nullptr;
    void* mem_ = nullptr;
    unsigned* err_ = nullptr;
    std::vector<void*> opened_;
    P2pArgs args_{};
    unsigned* tail_[kP2pMaxRanks] = {};  // {err, abort} words of every rank as mapped here
    unsigned epoch_ = 0;
    bool fused_reduce_ = true;  // reduce_all_reduce in one kernel
    bool fused_update_ = true;  // ... with the sweep's decision and update (reduce_all_reduce_update)
};

}  // namespace

int ranks_sharing_device(HostComm& host, int device) {
    const int n = host.size();
    if (n <= 1) return 1;
    // identity of the physical GPU: boot id + host name + PCI bus id (device ordinals differ under per-rank
    // HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES and LOCAL_WORLD_SIZE is launcher-specific; containers on
    // different nodes can share a host name and bus ids, but not the kernel's boot id)
    char bus[64] = {0};
    hip_ok(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, device), "hipDeviceGetPCIBusId");
    char hn[256] = {0};
    (void)gethostname(hn, sizeof(hn) - 1);
    char boot[64] = {0};
    if (FILE* f = std::fopen("/proc/sys/kernel/random/boot_id", "r")) {
        if (!std::fgets(boot, sizeof(boot), f)) boot[0] = 0;
        std::fclose(f);
    }
    uint64_t h = 1469598103934665603ull;  // FNV-1a over "boot/host/bus"
    for (const char* p : {static_cast<const char*>(boot), "/", static_cast<const char*>(hn), "/",
                          static_cast<const char*>(bus)})
        for (; *p; ++p) h = (h ^ (unsigned char)*p) * 1099511628211ull;
    std::vector<double> keys((size_t)n, 0.0);
    keys[(size_t)host.rank()] = (double)(h >> 12) + 1.0;  // < 2^53: exact in fp64; one nonzero slot per rank
    host.all_reduce_host(keys.data(), keys.size(), ReduceOp::kSum);
    std::sort(keys.begin(), keys.end());
    int most = 1;  // the largest number of ranks on one GPU (identical on every rank)
    for (size_t i = 0, j = 0; i < keys.size(); i = j) {
        for (j = i; j < keys.size() && keys[j] == keys[i]; ++j) {
        }
        most = std::max(most, (int)(j - i));
    }
    return most;
}

std::unique_ptr<Communicator> make_local_comm() { return std::make_unique<LocalComm>(); }

std::unique_ptr<Communicator> make_staged_comm(std::unique_ptr<HostComm> host) {
    return std::make_unique<StagedComm>(std::move(host));
}

std::string rccl_unique_id() {
    ncclUniqueId id;
    nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::unique_ptr<Communicator> make_rccl_comm(int device, const std::string& uid, std::unique_ptr<HostComm> bootstrap) {
    auto rc = std::make_unique<RcclComm>(std::move(bootstrap));
    // SART_FAULT_RCCL_INIT=1 (tests): the RCCL bring-up fails on every rank (no rank calls ncclCommInitRank), or,
    // with SART_FAULT_RANK, on that rank only (it still takes part in the collective init and reports failure
    // afterwards). SART_FAULT_RCCL_INIT_SKIP=<rank>: that rank never enters the init, so its peers wait in theirs
    // until the deadline (SART_RCCL_INIT_TIMEOUT_S) -- an uncooperative failure
    const char* f = std::getenv("SART_FAULT_RCCL_INIT");
    const char* fr = std::getenv("SART_FAULT_RANK");
    const char* fs = std::getenv("SART_FAULT_RCCL_INIT_SKIP");
    const bool inject = f && *f && std::atoi(f) != 0;
    const bool inject_all = inject && !(fr && *fr);
    const bool skip = fs && *fs && std::atoi(fs) == rc->host().rank();
    const double timeout_s = env_double("SART_RCCL_INIT_TIMEOUT_S", 120.0);
    std::string err = inject_all ? std::string("injected (SART_FAULT_RCCL_INIT)")
                      : skip     ? std::string("injected: never entered the init (SART_FAULT_RCCL_INIT_SKIP)")
                                 : rc->init(device, uid, timeout_s);
    if (inject && !inject_all && std::atoi(fr) == rc->host().rank()) {
        rc->destroy();
        err = "injected (SART_FAULT_RCCL_INIT)";
    }
    // every rank learns whether all brought RCCL up; if any did not, all continue on device buffers staged
    // through the host communicator (which the P2P all-reduce then wraps: it needs only IPC), instead of a
    // failed run. The second word carries the lowest failing rank (max of -rank).
    double fail[2] = {err.empty() ? 0.0 : 1.0, err.empty() ? -1e9 : -(double)rc->host().rank()};
    rc->host().all_reduce_host(fail, 2, ReduceOp::kMax);
    if (fail[0] == 0.0) return rc;
    rc->destroy();
    const int first = (int)(-fail[1]);
    std::string note = "RCCL init failed on rank " + std::to_string(first) + (err.empty() ? "" : ": " + err) +
                       "; collectives staged through host memory";
    if (rc->host().rank() == 0) std::fprintf(stderr, "sart: %s\n", note.c_str());
    return std::make_unique<StagedComm>(rc->take_host(), note);
}

std::unique_ptr<Communicator> comm_from_env(int device) {
    auto host = host_comm_from_env();
    if (host->size() <= 1) return make_local_comm();
    const char* be = std::getenv("SART_DIST_BACKEND");
    const char* p2p = std::getenv("SART_P2P");
    if (be && (std::string(be) == "tcp" || std::string(be) == "gloo")) {
        auto staged = make_staged_comm(std::move(host));
        const char* wrap = std::getenv("SART_P2P_WRAP_STAGED");  // tests on one GPU
        if ((p2p && std::string(p2p) == "1") || (wrap && std::string(wrap) == "1"))
            return make_p2p_comm(device, std::move(staged));
        return staged;
    }
    std::string uid(128, '\0');
    if (host->rank() == 0) uid = rccl_unique_id();
    host->broadcast_host(uid.data(), uid.size(), 0);
    return make_p2p_comm(device, make_rccl_comm(device, uid, std::move(host)));
}

std::unique_ptr<Communicator> make_p2p_comm(int device, std::shared_ptr<Communicator> base) {
    return std::make_unique<P2pComm>(device, std::move(base));
}

}  // namespace sart
