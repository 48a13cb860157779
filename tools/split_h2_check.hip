// Bitwise check of the f16-pair split (multiframe_bf16.hip::split_h2, v_fma_mix in inline asm) against the plain
// scale / convert / subtract formulation, over random fp32 values whose scaled magnitude spans the f16 range
// (normal, subnormal and flushed-to-zero residuals, both signs, zeros). Prints mismatches and exits 1 on any.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 halfx2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split_asm(unsigned x, unsigned y, float s, unsigned& p1, unsigned& p2) {
    asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
        "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
        "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(p1), "=&v"(p2)
        : "v"(__uint_as_float(x)), "v"(__uint_as_float(y)), "v"(s));
}
__device__ __forceinline__ void split_ref(unsigned x, unsigned y, float s, unsigned& p1, unsigned& p2) {
    const float a = __uint_as_float(x) * s, b = __uint_as_float(y) * s;
    const halfx2_t h = {(_Float16)a, (_Float16)b};
    p1 = __builtin_bit_cast(unsigned, h);
    const halfx2_t l = {(_Float16)(a - (float)h.x), (_Float16)(b - (float)h.y)};
    p2 = __builtin_bit_cast(unsigned, l);
}
__global__ void k(const uint2* in, const float* sc, uint4* o, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 v = in[i];
    unsigned p1, p2, q1, q2;
    split_asm(v.x, v.y, sc[i], p1, p2);
    split_ref(v.x, v.y, sc[i], q1, q2);
    o[i] = make_uint4(p1, p2, q1, q2);
}

int main() {
    const int n = 1 << 22;
    std::mt19937_64 rng(7);
    std::vector<uint2> in(n);
    std::vector<float> sc(n);
    for (int i = 0; i < n; ++i) {
        // scaled magnitude 2^e with e in [-40, 15]: normal f16, subnormal f16 and below; the scale 2^k, k in [-30, 30]
        const int k = (int)(rng() % 61) - 30;
        auto val = [&]() {
            const int e = (int)(rng() % 56) - 40;
            float m = 1.0f + (float)(rng() >> 40) / (float)(1ull << 24);
            float v = std::ldexp(m, e - k);
            if (rng() % 2) v = -v;
            if (rng() % 97 == 0) v = 0.0f;
            unsigned u;
            std::memcpy(&u, &v, 4);
            return u;
        };
        in[i] = make_uint2(val(), val());
        sc[i] = std::ldexp(1.0f, k);
    }
    uint2* din;
    float* dsc;
    uint4* dout;
    if (hipMalloc(&din, n * sizeof(uint2)) || hipMalloc(&dsc, n * sizeof(float)) || hipMalloc(&dout, n * sizeof(uint4)))
        return 2;
    hipMemcpy(din, in.data(), n * sizeof(uint2), hipMemcpyHostToDevice);
    hipMemcpy(dsc, sc.data(), n * sizeof(float), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, din, dsc, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<uint4> out(n);
    hipMemcpy(out.data(), dout, n * sizeof(uint4), hipMemcpyDeviceToHost);
    long bad = 0;
    for (int i = 0; i < n; ++i)
        if (out[i].x != out[i].z || out[i].y != out[i].w) {
            if (bad < 10)
                std::printf("mismatch %d: in %08x %08x s %g asm %08x %08x ref %08x %08x\n", i, in[i].x, in[i].y,
                            sc[i], out[i].x, out[i].y, out[i].z, out[i].w);
            ++bad;
        }
    std::printf("{\"split_h2_check\": true, \"n_pairs\": %d, \"mismatches\": %ld}\n", n, bad);
    return bad ? 1 : 0;
}
