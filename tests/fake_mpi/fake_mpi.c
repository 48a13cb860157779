/* Fake libmpi for the ABI tests of csrc/native/host_comm_mpi.cpp (tests/test_mpi_abi.py): one process that
 * pretends to be rank 0 of 2. The "peer" contributes 1 to every SUM element and 100 to every MAX element, so
 * the test sees whether the right datatype and operation reached the library. Every handle is checked
 * against this ABI's values; a mismatch aborts the process (exit 3).
 * Build with -DOMPI_ABI for Open MPI's ABI (pointer handles to predefined objects, MPI_IN_PLACE = 1),
 * without it for the MPICH ABI (int handles, MPI_IN_PLACE = -1). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void fail(const char* what) {
    fprintf(stderr, "fake_mpi: bad %s\n", what);
    exit(3);
}

#ifdef OMPI_ABI
struct ompi_obj { int tag; };
struct ompi_obj ompi_mpi_comm_world = {1}, ompi_mpi_byte = {2}, ompi_mpi_float = {3}, ompi_mpi_double = {4},
                ompi_mpi_op_sum = {5}, ompi_mpi_op_max = {6};
typedef void* H;
#define COMM_WORLD ((H)&ompi_mpi_comm_world)
#define T_BYTE ((H)&ompi_mpi_byte)
#define T_FLOAT ((H)&ompi_mpi_float)
#define T_DOUBLE ((H)&ompi_mpi_double)
#define OP_SUM ((H)&ompi_mpi_op_sum)
#define OP_MAX ((H)&ompi_mpi_op_max)
#define IN_PLACE ((void*)1)
static const char* kVersion = "Open MPI v4.1.0 (fake, tests/fake_mpi)";
#else
typedef int H;
#define COMM_WORLD 0x44000000
#define T_BYTE 0x4c00010d
#define T_FLOAT 0x4c00040a
#define T_DOUBLE 0x4c00080b
#define OP_SUM 0x58000003
#define OP_MAX 0x58000001
#define IN_PLACE ((void*)-1)
static const char* kVersion = "MPICH Version: 3.3.2 (fake, tests/fake_mpi)";
#endif

static int initialized = 0, finalized = 0;
int MPI_Get_library_version(char* v, int* len) {
    strcpy(v, kVersion);
    *len = (int)strlen(kVersion);
    return 0;
}
int MPI_Initialized(int* f) { *f = initialized; return 0; }
int MPI_Init(int* argc, char*** argv) { (void)argc; (void)argv; initialized = 1; return 0; }
int MPI_Finalized(int* f) { *f = finalized; return 0; }
int MPI_Finalize(void) { finalized = 1; return 0; }
int MPI_Comm_rank(H c, int* r) { if (c != COMM_WORLD) fail("comm"); *r = 0; return 0; }
int MPI_Comm_size(H c, int* s) { if (c != COMM_WORLD) fail("comm"); *s = 2; return 0; }
int MPI_Allreduce(const void* s, void* r, int n, H t, H op, H c) {
    if (s != IN_PLACE) fail("MPI_IN_PLACE");
    if (c != COMM_WORLD) fail("comm");
    if (op != OP_SUM && op != OP_MAX) fail("op");
    for (int i = 0; i < n; ++i) {
        if (t == T_DOUBLE) {
            double* d = (double*)r;
            d[i] = op == OP_SUM ? d[i] + 1.0 : (d[i] > 100.0 ? d[i] : 100.0);
        } else if (t == T_FLOAT) {
            float* f = (float*)r;
            f[i] = op == OP_SUM ? f[i] + 1.0f : (f[i] > 100.0f ? f[i] : 100.0f);
        } else {
            fail("datatype");
        }
    }
    return 0;
}
int MPI_Bcast(void* b, int n, H t, int root, H c) {
    (void)b; (void)n;
    if (t != T_BYTE) fail("bcast datatype");
    if (c != COMM_WORLD || root < 0 || root > 1) fail("bcast comm/root");
    return 0;
}
int MPI_Barrier(H c) { if (c != COMM_WORLD) fail("comm"); return 0; }
int MPI_Abort(H c, int code) { (void)c; exit(code); }
