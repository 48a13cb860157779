// Rounding behaviour of v_dot2c_f32_bf16 on gfx950: D = a.lo * b.lo + a.hi * b.hi + c against the exact
// (fp64) value of the same operands. Prints the mean signed error in ulps of the result (0 for round to
// nearest even, about -0.5 for round toward zero) and the max |error|.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

__global__ void k_dot2(const unsigned* a, const unsigned* b, const float* c, float* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, a[i]), __builtin_bit_cast(bf2, b[i]), c[i],
                                                 false);
}

static float bf(unsigned short h) {
    unsigned u = (unsigned)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

int main() {
    const int n = 1 << 20;
    std::vector<unsigned> a(n), b(n);
    std::vector<float> c(n), out(n);
    srand(7);
    auto rb = [] { return (unsigned short)(0x3f00 + (rand() & 0xff)); };  // bf16 in [0.5, 2)
    for (int i = 0; i < n; ++i) {
        a[i] = rb() | ((unsigned)rb() << 16);
        b[i] = rb() | ((unsigned)rb() << 16);
        c[i] = 1000.0f * (float)rand() / RAND_MAX;  // a running sum much larger than the products
    }
    unsigned *da, *db;
    float *dc, *dout;
    hipMalloc(&da, n * 4), hipMalloc(&db, n * 4), hipMalloc(&dc, n * 4), hipMalloc(&dout, n * 4);
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_dot2, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dout, n);
    hipMemcpy(out.data(), dout, n * 4, hipMemcpyDeviceToHost);
    double sum = 0, mx = 0, fsum = 0;
    for (int i = 0; i < n; ++i) {
        const double exact = (double)bf(a[i] & 0xffff) * bf(b[i] & 0xffff) + (double)bf(a[i] >> 16) * bf(b[i] >> 16) + c[i];
        const double ulp = std::ldexp(1.0, std::ilogb(exact) - 23);
        const double e = ((double)out[i] - exact) / ulp;
        const float fma2 = std::fma(bf(a[i] >> 16), bf(b[i] >> 16), std::fma(bf(a[i] & 0xffff), bf(b[i] & 0xffff), c[i]));
        fsum += ((double)fma2 - exact) / ulp;
        sum += e;
        mx = std::max(mx, std::fabs(e));
    }
    printf("{\"op\": \"v_dot2c_f32_bf16\", \"mean_err_ulp\": %.4f, \"max_abs_err_ulp\": %.4f, \"two_fma_mean_err_ulp\": %.4f}\n",
           sum / n, mx, fsum / n);
    return 0;
}
