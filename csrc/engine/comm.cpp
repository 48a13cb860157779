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
    explicit StagedComm(std::unique_ptr<HostComm> h) : host_(std::move(h)) {}
    HostComm& host() override { return *host_; }
    const char* backend() const override { return "staged"; }
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
};

class RcclComm final : public Communicator {
   public:
    RcclComm(int device, const std::string& uid, std::unique_ptr<HostComm> boot) : host_(std::move(boot)) {
        if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: bad unique id");
        ncclUniqueId id;
        std::memcpy(&id, uid.data(), sizeof(id));
        hip_ok(hipSetDevice(device), "hipSetDevice");
        nccl_ok(ncclCommInitRank(&comm_, host_->size(), id, host_->rank()), "ncclCommInitRank");
    }
    ~RcclComm() override {
        if (comm_) (void)ncclCommDestroy(comm_);
    }
    HostComm& host() override { return *host_; }
    const char* backend() const override { return "rccl"; }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        if (n) nccl_ok(ncclAllReduce(dev, dev, n, ncclFloat32, nop(op), comm_, stream), "ncclAllReduce");
    }
    void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        if (n) nccl_ok(ncclAllReduce(dev, dev, n, ncclFloat64, nop(op), comm_, stream), "ncclAllReduce");
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
        t_start_ = std::chrono::steady_clock::now();
        HostComm& h = base_->host();
        rank_ = h.rank();
        n_ = h.size();
        const char* m = std::getenv("SART_P2P");
        const std::string mode = (m && *m) ? m : "auto";
        cap_ = std::max<int64_t>(1024, (int64_t)(env_double("SART_P2P_MAX_BYTES", 2.0 * 1024 * 1024) / 4) / 4 * 4);
        // a healthy peer is at most a few sweeps behind (the host collectives of every frame's setup align the
        // ranks first), so a P2P wait this long means the peer is gone or stuck: the engines then switch to the
        // base communicator and re-solve the frame (device_failed / degrade)
        timeout_s_ = env_double("SART_P2P_TIMEOUT_S", 60.0);
        if (const char* f = std::getenv("SART_P2P_FUSED_REDUCE"); f && *f) fused_reduce_ = std::atoi(f) != 0;
        if (const char* f = std::getenv("SART_FAULT_P2P"); f && *f) {
            const char* fr = std::getenv("SART_FAULT_RANK");
            if (!(fr && *fr) || std::atoi(fr) == rank_) fault_call_ = std::atoll(f);
        }
        if (mode == "0" || mode == "off") {
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
        hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
        if (!agree(map_peers())) {
            finish(false, "p2p off: IPC mapping failed (" + err_msg_ + ")");
            return;
        }
        if (!agree(self_test())) {
            finish(false, "p2p off: self-test failed (" + (err_msg_.empty() ? "on another rank" : err_msg_) + ")");
            return;
        }
        if (mode == "1" || mode == "on") {
            finish(true, "p2p (forced, self-test ok)");
            return;
        }
        // auto: rank 0 times both at message sizes around the engine's (V + 1 floats: 64k .. 256k voxels);
        // the P2P path serves vectors up to the largest probed size at which it won (rank 0 decides)
        const int64_t probes[] = {4097, 65537, 262145, 524288};
        double pick[1 + 2 * 4] = {0.0};
        std::string table;
        for (int i = 0; i < 4; ++i) {
            const int64_t n = probes[i];
            if (n > cap_) break;
            const double tp = time_us([&](float* b) { p2p(b, n, 0, stream_); }, n);
            const double tb = time_us([&](float* b) { base_->all_reduce(b, (size_t)n, ReduceOp::kSum, stream_); }, n);
            pick[1 + 2 * i] = tp;
            pick[2 + 2 * i] = tb;
            if (tp < tb) pick[0] = (double)n;
        }
        h.broadcast_host(pick, sizeof(pick), 0);
        for (int i = 0; i < 4 && probes[i] <= cap_; ++i) {
            char cell[96];
            std::snprintf(cell, sizeof(cell), "%s%lld: %.1f/%.1f", i ? ", " : "", (long long)probes[i], pick[1 + 2 * i],
                          pick[2 + 2 * i]);
            table += cell;
        }
        max_n_ = (int64_t)pick[0];
        char buf[96];
        std::snprintf(buf, sizeof(buf), "p2p up to %lld floats, %s above", (long long)max_n_, base_->backend());
        finish(max_n_ > 0, (max_n_ > 0 ? std::string(buf) : std::string(base_->backend())) +
                               " (auto, rank 0, us p2p/" + base_->backend() + " at floats " + table + ")");
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
    std::string describe() const override { return why_; }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        // the choice depends only on n (identical on every rank), never on this rank's pointer alignment
        if (active_ && n > 0 && (int64_t)n <= max_n_) {
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
        if (active_ && fused_reduce_ && src.ld + 2 <= max_n_) {
            const bool skip = fault_call_ > 0 && ++calls_ >= fault_call_;
            launch_p2p_reduce_allreduce(src, out, args_, rank_, n_, ++epoch_, cap_, err_, timeout_s_, stream, skip);
        } else {
            Communicator::reduce_all_reduce(src, out, stream);
        }
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
        active_ = false;
        why_ = std::string(base_->backend()) + " (p2p disabled after a p2p all-reduce timeout; was: " + why_ + ")";
        return true;
    }

   private:
    std::pair<unsigned, unsigned> err_words() {  // {timeout, abort}
        unsigned e[2] = {0, 0};
        hip_ok(hipMemcpy(e, err_, sizeof(e), hipMemcpyDeviceToHost), "p2p error word");
        return {e[0], e[1]};
    }
    void finish(bool active, const std::string& why) {
        active_ = active;
        // start-up cost (IPC mapping, self-test, auto probe) on this rank, reported with the selection
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start_).count();
        char buf[64];
        std::snprintf(buf, sizeof(buf), " [p2p setup %.0f ms]", ms);
        why_ = why + buf;
        if (active && max_n_ == 0) max_n_ = cap_;  // forced on: every vector that fits the slots
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
        for (int r = 0; r < n_; ++r) {  // every rank takes part in every broadcast, even after a failure
            hipIpcMemHandle_t h = hdl;
            base_->host().broadcast_host(&h, sizeof(h), r);
            if (!ok) continue;
            void* p = mem_;
            if (r != rank_) {
                if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    (void)hipGetLastError();
                    ok = false;
                    err_msg_ = "hipIpcOpenMemHandle of rank " + std::to_string(r);
                    continue;
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
    // Exact checks: integer-valued sums / maxima, and random fp32 data against the rank-order sum (the
    // kernel's result must be bitwise identical to ((v0 + v1) + v2) + ... on every rank), both parities.
    bool self_test() {
        float* d = nullptr;
        if (!agree(hipMalloc(reinterpret_cast<void**>(&d), (size_t)cap_ * sizeof(float)) == hipSuccess)) {
            (void)hipGetLastError();
            if (d) (void)hipFree(d);
            err_msg_ = "hipMalloc";
            return false;
        }
        const int64_t sizes[] = {1, 5, 1024, 4099, std::min<int64_t>(cap_, 65537)};
        int call = 0;
        for (int64_t n : sizes) {
            for (int kind = 0; kind < 3; ++kind, ++call) {  // 0 integer sum, 1 integer max, 2 random fp32 sum
                bool good = true;
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
                    p2p(d, n, kind == 1 ? 1 : 0, stream_, std::min(timeout_s_, 30.0));
                    hip_ok(hipStreamSynchronize(stream_), "p2p self-test");
                    hip_ok(hipMemcpy(got.data(), d, (size_t)n * sizeof(float), hipMemcpyDeviceToHost), "D2H");
                    unsigned e = 0;
                    hip_ok(hipMemcpy(&e, err_, sizeof(e), hipMemcpyDeviceToHost), "D2H");
                    if (e) throw std::runtime_error("peer timeout");
                    if (std::memcmp(got.data(), want.data(), (size_t)n * sizeof(float)) != 0)
                        throw std::runtime_error("mismatch at n=" + std::to_string(n) + " kind " + std::to_string(kind));
                } catch (const std::exception& ex) {
                    good = false;
                    err_msg_ = ex.what();
                }
                if (!agree(good)) {  // every rank leaves the test at the same call
                    (void)hipFree(d);
                    return false;
                }
            }
        }
        (void)hipFree(d);
        return true;
    }
    static float value(int kind, int r, int64_t i, int call) {
        if (kind < 2) return (float)((r + 1) * ((i * 7 + call) % 251));
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + (uint64_t)(r + 1) * 0xBF58476D1CE4E5B9ull + (uint64_t)call;
        z = (z ^ (z >> 31)) * 0x94D049BB133111EBull;
        return (float)((double)(z >> 40) / (double)(1ull << 24) * 2.0 - 1.0);
    }
    // mean microseconds per call over 20 calls after 3 warm-up calls (host barrier before timing)
    double time_us(const std::function<void(float*)>& f, int64_t n) {
        float* d = nullptr;
        hip_ok(hipMalloc(reinterpret_cast<void**>(&d), (size_t)n * sizeof(float)), "hipMalloc");
        hip_ok(hipMemset(d, 0, (size_t)n * sizeof(float)), "hipMemset");
        hip_ok(hipDeviceSynchronize(), "sync");
        for (int i = 0; i < 3; ++i) f(d);
        hip_ok(hipStreamSynchronize(stream_), "sync");
        base_->host().barrier();
        hipEvent_t e0, e1;
        hip_ok(hipEventCreate(&e0), "event");
        hip_ok(hipEventCreate(&e1), "event");
        hip_ok(hipEventRecord(e0, stream_), "event");
        for (int i = 0; i < 20; ++i) f(d);
        hip_ok(hipEventRecord(e1, stream_), "event");
        hip_ok(hipEventSynchronize(e1), "event");
        float ms = 0.f;
        hip_ok(hipEventElapsedTime(&ms, e0, e1), "event");
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipFree(d);
        return 1e3 * ms / 20.0;
    }

    std::shared_ptr<Communicator> base_;
    int device_ = 0, rank_ = 0, n_ = 1;
    int64_t cap_ = 0;
    int64_t max_n_ = 0;  // P2P for n <= max_n_ (auto: largest probed size at which it beat the base)
    double timeout_s_ = 60.0;
    int64_t fault_call_ = 0, calls_ = 0;  // SART_FAULT_P2P
    std::chrono::steady_clock::time_point t_start_;
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
};

}  // namespace

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
    return std::make_unique<RcclComm>(device, uid, std::move(bootstrap));
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
