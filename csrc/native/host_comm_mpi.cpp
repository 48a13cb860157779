// MPI backend of the host collectives: the reference's own transport, host MPI_Allreduce /
// MPI_Bcast / MPI_Barrier on MPI_COMM_WORLD (reference sartsolver.cpp:47,158-329; main.cpp:63-65,84,148).
//
// Used when the job is started by an MPICH-family launcher (mpiexec / mpirun of MPICH, Intel MPI, Cray
// MPICH: PMI_RANK / PMI_SIZE in the environment) or when SART_HOST_COMM=mpi; it then also bootstraps RCCL
// (unique-id broadcast) across nodes without a MASTER_ADDR. libmpi is loaded at run time with dlopen
// (SART_MPI_LIB, else libmpi.so.12 on the loader path or /opt/conda/lib), so the build has no MPI
// dependency; the handles below are the MPICH ABI constants (mpi.h of MPICH 3.x / 4.x).
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "host_comm.hpp"

namespace sart {

namespace {

// MPICH ABI (mpi.h): handles are plain ints
using MPI_Comm = int;
using MPI_Datatype = int;
using MPI_Op = int;
constexpr MPI_Comm kCommWorld = 0x44000000;
constexpr MPI_Datatype kByte = 0x4c00010d, kFloat = 0x4c00040a, kDouble = 0x4c00080b;
constexpr MPI_Op kMax = 0x58000001, kSum = 0x58000003;
void* const kInPlace = reinterpret_cast<void*>(-1);

struct MpiApi {
    void* lib = nullptr;
    int (*Initialized)(int*) = nullptr;
    int (*Init)(int*, char***) = nullptr;
    int (*Finalized)(int*) = nullptr;
    int (*Finalize)() = nullptr;
    int (*Comm_rank)(MPI_Comm, int*) = nullptr;
    int (*Comm_size)(MPI_Comm, int*) = nullptr;
    int (*Allreduce)(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm) = nullptr;
    int (*Bcast)(void*, int, MPI_Datatype, int, MPI_Comm) = nullptr;
    int (*Barrier)(MPI_Comm) = nullptr;
    int (*Abort)(MPI_Comm, int) = nullptr;

    static MpiApi& get() {
        static MpiApi api;
        if (!api.lib) api.load();
        return api;
    }

   private:
    template <typename F>
    void sym(F& f, const char* name) {
        f = reinterpret_cast<F>(dlsym(lib, name));
        if (!f) throw std::runtime_error(std::string("mpi host comm: symbol ") + name + " missing");
    }
    void load() {
        std::string tried;
        const char* env = std::getenv("SART_MPI_LIB");
        for (const char* cand : {env, "libmpi.so.12", "/opt/conda/lib/libmpi.so.12", "libmpi.so"}) {
            if (!cand || !*cand) continue;
            lib = dlopen(cand, RTLD_NOW | RTLD_GLOBAL);
            if (lib) break;
            tried += std::string(" ") + cand;
        }
        if (!lib) throw std::runtime_error("mpi host comm: cannot load libmpi (tried" + tried + "); set SART_MPI_LIB");
        sym(Initialized, "MPI_Initialized");
        sym(Init, "MPI_Init");
        sym(Finalized, "MPI_Finalized");
        sym(Finalize, "MPI_Finalize");
        sym(Comm_rank, "MPI_Comm_rank");
        sym(Comm_size, "MPI_Comm_size");
        sym(Allreduce, "MPI_Allreduce");
        sym(Bcast, "MPI_Bcast");
        sym(Barrier, "MPI_Barrier");
        sym(Abort, "MPI_Abort");
    }
};

void mpi_ok(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string("mpi host comm: ") + what + " failed (" + std::to_string(rc) + ")");
}

class MpiHostComm final : public HostComm {
   public:
    MpiHostComm() : api_(MpiApi::get()) {
        int init = 0;
        mpi_ok(api_.Initialized(&init), "MPI_Initialized");
        if (!init) {
            mpi_ok(api_.Init(nullptr, nullptr), "MPI_Init");
            owner_ = true;
        }
        mpi_ok(api_.Comm_rank(kCommWorld, &rank_), "MPI_Comm_rank");
        mpi_ok(api_.Comm_size(kCommWorld, &size_), "MPI_Comm_size");
    }
    ~MpiHostComm() override {
        int fin = 0;
        if (owner_ && api_.Finalized(&fin) == 0 && !fin) (void)api_.Finalize();
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    const char* backend() const override { return "mpi"; }
    void all_reduce_host(double* v, size_t n, ReduceOp op) override { reduce(v, n, kDouble, op); }
    void all_reduce_host(float* v, size_t n, ReduceOp op) override { reduce(v, n, kFloat, op); }
    void broadcast_host(void* buf, size_t nbytes, int root) override {
        char* p = static_cast<char*>(buf);
        for (size_t off = 0; off < nbytes;) {  // int counts: chunks below 2 GiB
            const int c = (int)std::min<size_t>(nbytes - off, (size_t)1 << 30);
            mpi_ok(api_.Bcast(p + off, c, kByte, root, kCommWorld), "MPI_Bcast");
            off += (size_t)c;
        }
    }
    void barrier() override { mpi_ok(api_.Barrier(kCommWorld), "MPI_Barrier"); }
    void abort() override { (void)api_.Abort(kCommWorld, 1); }

   private:
    void reduce(void* v, size_t n, MPI_Datatype t, ReduceOp op) {
        const size_t esz = t == kDouble ? 8 : 4;
        char* p = static_cast<char*>(v);
        for (size_t off = 0; off < n;) {
            const int c = (int)std::min<size_t>(n - off, (size_t)1 << 28);
            mpi_ok(api_.Allreduce(kInPlace, p + off * esz, c, t, op == ReduceOp::kSum ? kSum : kMax, kCommWorld),
                   "MPI_Allreduce");
            off += (size_t)c;
        }
    }
    MpiApi& api_;
    int rank_ = 0, size_ = 1;
    bool owner_ = false;
};

}  // namespace

std::unique_ptr<HostComm> make_mpi_host_comm() { return std::make_unique<MpiHostComm>(); }

bool mpi_launch_detected() {
    const char* sel = std::getenv("SART_HOST_COMM");
    if (sel && *sel) return std::string(sel) == "mpi";
    // MPICH-family launchers export PMI_*; torchrun exports RANK (and is served by the TCP backend)
    const char* pmi = std::getenv("PMI_SIZE");
    const char* rank = std::getenv("RANK");
    return pmi && *pmi && std::atoi(pmi) > 1 && !(rank && *rank);
}

}  // namespace sart
