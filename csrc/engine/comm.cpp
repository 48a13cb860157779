#include "comm.hpp"

#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

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
    if (be && (std::string(be) == "tcp" || std::string(be) == "gloo")) return make_staged_comm(std::move(host));
    std::string uid(128, '\0');
    if (host->rank() == 0) uid = rccl_unique_id();
    host->broadcast_host(uid.data(), uid.size(), 0);
    return make_rccl_comm(device, uid, std::move(host));
}

}  // namespace sart
