// MPI backend of the host collectives: the reference's own transport, host MPI_Allreduce /
// MPI_Bcast / MPI_Barrier on MPI_COMM_WORLD (reference sartsolver.cpp:47,158-329; main.cpp:63-65,84,148).
//
// Used when the job is started by an MPI launcher (MPICH family: PMI_RANK / PMI_SIZE; Open MPI:
// OMPI_COMM_WORLD_*) without torchrun's RANK, or when SART_HOST_COMM=mpi; it then also bootstraps RCCL
// (unique-id broadcast) across nodes without a MASTER_ADDR. libmpi is loaded at run time with dlopen
// (SART_MPI_LIB, else libmpi.so.12 (MPICH) / libmpi.so.40 (Open MPI) on the loader path or /opt/conda/lib),
// so the build has no MPI dependency. The two ABIs differ in their handles, so the library is identified
// with MPI_Get_library_version:
//   * MPICH ABI (MPICH, Intel MPI, Cray MPICH): handles are ints (mpi.h constants), MPI_IN_PLACE = -1;
//   * Open MPI (the reference's SDCC stack, reference README.md:42-44): handles are pointers to the
//     predefined objects ompi_mpi_comm_world, ompi_mpi_float, ompi_mpi_op_sum, ... (resolved with dlsym),
//     MPI_IN_PLACE = 1.
#include <dlfcn.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "host_comm.hpp"

namespace sart {

namespace {

enum class MpiAbi { kMpich, kOpenMpi };

// Both ABIs pass handles in one integer register (int or pointer); Handle carries either. Each function is
// bound with the parameter types of the detected ABI.
using Handle = uintptr_t;

struct MpiApi {
    void* lib = nullptr;
    MpiAbi abi = MpiAbi::kMpich;
    std::string version;
    Handle comm_world = 0, byte = 0, f32 = 0, f64 = 0, op_sum = 0, op_max = 0;
    void* in_place = nullptr;
    int (*Initialized)(int*) = nullptr;
    int (*Init)(int*, char***) = nullptr;
    int (*Finalized)(int*) = nullptr;
    int (*Finalize)() = nullptr;
    // MPICH-ABI signatures (int handles)
    int (*Comm_rank_i)(int, int*) = nullptr;
    int (*Comm_size_i)(int, int*) = nullptr;
    int (*Allreduce_i)(const void*, void*, int, int, int, int) = nullptr;
    int (*Bcast_i)(void*, int, int, int, int) = nullptr;
    int (*Barrier_i)(int) = nullptr;
    int (*Abort_i)(int, int) = nullptr;
    // Open MPI signatures (pointer handles)
    int (*Comm_rank_p)(void*, int*) = nullptr;
    int (*Comm_size_p)(void*, int*) = nullptr;
    int (*Allreduce_p)(const void*, void*, int, void*, void*, void*) = nullptr;
    int (*Bcast_p)(void*, int, void*, int, void*) = nullptr;
    int (*Barrier_p)(void*) = nullptr;
    int (*Abort_p)(void*, int) = nullptr;

    static MpiApi& get() {
        static MpiApi api;
        if (!api.lib) api.load();
        return api;
    }

    int comm_rank(int* r) const {
        return abi == MpiAbi::kMpich ? Comm_rank_i((int)comm_world, r) : Comm_rank_p((void*)comm_world, r);
    }
    int comm_size(int* s) const {
        return abi == MpiAbi::kMpich ? Comm_size_i((int)comm_world, s) : Comm_size_p((void*)comm_world, s);
    }
    int allreduce(void* buf, int n, Handle type, Handle op) const {
        if (abi == MpiAbi::kMpich) return Allreduce_i(in_place, buf, n, (int)type, (int)op, (int)comm_world);
        return Allreduce_p(in_place, buf, n, (void*)type, (void*)op, (void*)comm_world);
    }
    int bcast(void* buf, int n, int root) const {
        if (abi == MpiAbi::kMpich) return Bcast_i(buf, n, (int)byte, root, (int)comm_world);
        return Bcast_p(buf, n, (void*)byte, root, (void*)comm_world);
    }
    int barrier() const { return abi == MpiAbi::kMpich ? Barrier_i((int)comm_world) : Barrier_p((void*)comm_world); }
    int abort_all(int code) const {
        return abi == MpiAbi::kMpich ? Abort_i((int)comm_world, code) : Abort_p((void*)comm_world, code);
    }

   private:
    template <typename F>
    void sym(F& f, const char* name) {
        f = reinterpret_cast<F>(dlsym(lib, name));
        if (!f) throw std::runtime_error(std::string("mpi host comm: symbol ") + name + " missing");
    }
    Handle object(const char* name) {
        void* p = dlsym(lib, name);
        if (!p) throw std::runtime_error(std::string("mpi host comm: Open MPI object ") + name + " missing");
        return reinterpret_cast<Handle>(p);
    }
    void load() {
        std::string tried;
        const char* env = std::getenv("SART_MPI_LIB");
        // the launcher names the ABI to try first: Open MPI's mpirun exports OMPI_*, the MPICH family PMI_*
        // (a singleton MPI_Init of the other library would make every process rank 0 of 1)
        const char* ompi = std::getenv("OMPI_COMM_WORLD_SIZE");
        const bool open_mpi_first = ompi && *ompi;
        const char* first = open_mpi_first ? "libmpi.so.40" : "libmpi.so.12";
        const char* second = open_mpi_first ? "libmpi.so.12" : "libmpi.so.40";
        const char* first_c = open_mpi_first ? "/opt/conda/lib/libmpi.so.40" : "/opt/conda/lib/libmpi.so.12";
        const char* second_c = open_mpi_first ? "/opt/conda/lib/libmpi.so.12" : "/opt/conda/lib/libmpi.so.40";
        for (const char* cand : {env, first, first_c, second, second_c, "libmpi.so"}) {
            if (!cand || !*cand) continue;
            lib = dlopen(cand, RTLD_NOW | RTLD_GLOBAL);
            if (lib) break;
            tried += std::string(" ") + cand;
        }
        if (!lib) throw std::runtime_error("mpi host comm: cannot load libmpi (tried" + tried + "); set SART_MPI_LIB");
        int (*get_version)(char*, int*) = nullptr;
        sym(get_version, "MPI_Get_library_version");
        char buf[8192] = {0};  // >= MPI_MAX_LIBRARY_VERSION_STRING of both ABIs
        int len = 0;
        if (get_version(buf, &len) == 0) version.assign(buf, (size_t)std::max(0, std::min(len, (int)sizeof(buf))));
        abi = (version.find("Open MPI") != std::string::npos || dlsym(lib, "ompi_mpi_comm_world")) ? MpiAbi::kOpenMpi
                                                                                                   : MpiAbi::kMpich;
        sym(Initialized, "MPI_Initialized");
        sym(Init, "MPI_Init");
        sym(Finalized, "MPI_Finalized");
        sym(Finalize, "MPI_Finalize");
        if (abi == MpiAbi::kMpich) {
            // mpi.h of MPICH 3.x / 4.x
            comm_world = 0x44000000, byte = 0x4c00010d, f32 = 0x4c00040a, f64 = 0x4c00080b;
            op_max = 0x58000001, op_sum = 0x58000003;
            in_place = reinterpret_cast<void*>(-1);
            sym(Comm_rank_i, "MPI_Comm_rank");
            sym(Comm_size_i, "MPI_Comm_size");
            sym(Allreduce_i, "MPI_Allreduce");
            sym(Bcast_i, "MPI_Bcast");
            sym(Barrier_i, "MPI_Barrier");
            sym(Abort_i, "MPI_Abort");
        } else {
            // mpi.h of Open MPI 4.x / 5.x: MPI_COMM_WORLD = &ompi_mpi_comm_world, ...
            comm_world = object("ompi_mpi_comm_world");
            byte = object("ompi_mpi_byte");
            f32 = object("ompi_mpi_float");
            f64 = object("ompi_mpi_double");
            op_sum = object("ompi_mpi_op_sum");
            op_max = object("ompi_mpi_op_max");
            in_place = reinterpret_cast<void*>(1);
            sym(Comm_rank_p, "MPI_Comm_rank");
            sym(Comm_size_p, "MPI_Comm_size");
            sym(Allreduce_p, "MPI_Allreduce");
            sym(Bcast_p, "MPI_Bcast");
            sym(Barrier_p, "MPI_Barrier");
            sym(Abort_p, "MPI_Abort");
        }
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
        mpi_ok(api_.comm_rank(&rank_), "MPI_Comm_rank");
        mpi_ok(api_.comm_size(&size_), "MPI_Comm_size");
        // the world must be the launcher's: a library of the other MPI family initialises as a singleton
        for (const char* var : {"OMPI_COMM_WORLD_SIZE", "PMI_SIZE"}) {
            const char* v = std::getenv(var);
            if (v && *v && std::atoi(v) != size_)
                throw std::runtime_error(std::string("mpi host comm: MPI_Comm_size is ") + std::to_string(size_) +
                                         " but the launcher set " + var + "=" + v + " (" + api_.version.substr(0, 60) +
                                         "): point SART_MPI_LIB at the launcher's libmpi");
        }
    }
    ~MpiHostComm() override {
        int fin = 0;
        if (owner_ && api_.Finalized(&fin) == 0 && !fin) (void)api_.Finalize();
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    const char* backend() const override { return api_.abi == MpiAbi::kMpich ? "mpi" : "mpi(openmpi)"; }
    void all_reduce_host(double* v, size_t n, ReduceOp op) override { reduce(v, n, api_.f64, 8, op); }
    void all_reduce_host(float* v, size_t n, ReduceOp op) override { reduce(v, n, api_.f32, 4, op); }
    void broadcast_host(void* buf, size_t nbytes, int root) override {
        char* p = static_cast<char*>(buf);
        for (size_t off = 0; off < nbytes;) {  // int counts: chunks below 2 GiB
            const int c = (int)std::min<size_t>(nbytes - off, (size_t)1 << 30);
            mpi_ok(api_.bcast(p + off, c, root), "MPI_Bcast");
            off += (size_t)c;
        }
    }
    void barrier() override { mpi_ok(api_.barrier(), "MPI_Barrier"); }
    void abort() override { (void)api_.abort_all(1); }

   private:
    void reduce(void* v, size_t n, Handle t, size_t esz, ReduceOp op) {
        char* p = static_cast<char*>(v);
        for (size_t off = 0; off < n;) {
            const int c = (int)std::min<size_t>(n - off, (size_t)1 << 28);
            mpi_ok(api_.allreduce(p + off * esz, c, t, op == ReduceOp::kSum ? api_.op_sum : api_.op_max),
                   "MPI_Allreduce");
            off += (size_t)c;
        }
    }
    const MpiApi& api_;
    int rank_ = 0, size_ = 1;
    bool owner_ = false;
};

}  // namespace

std::unique_ptr<HostComm> make_mpi_host_comm() { return std::make_unique<MpiHostComm>(); }

std::string mpi_library_version() { return MpiApi::get().version; }

bool mpi_launch_detected() {
    const char* sel = std::getenv("SART_HOST_COMM");
    if (sel && *sel) return std::string(sel) == "mpi";
    // MPICH-family launchers export PMI_*, Open MPI's mpirun OMPI_COMM_WORLD_*; torchrun exports RANK (and is
    // served by the TCP backend)
    const char* rank = std::getenv("RANK");
    if (rank && *rank) return false;
    for (const char* var : {"PMI_SIZE", "OMPI_COMM_WORLD_SIZE"}) {
        const char* v = std::getenv(var);
        if (v && *v && std::atoi(v) > 1) return true;
    }
    return false;
}

}  // namespace sart
