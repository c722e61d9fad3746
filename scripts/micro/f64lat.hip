// f64 VALU latency/throughput probe: dependent vs independent v_fma_f64 chains,
// one wave per SIMD, cycles from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CHAINS>
__global__ __launch_bounds__(64) void k(double* out, unsigned long long* cyc, double a, double b) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x + c;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
#pragma unroll
        for (int u = 0; u < 16 / CHAINS; ++u)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fma(x[c], a, b);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    double* o; unsigned long long* c;
    (void)hipMalloc(&o, 4096 * 64 * 8); (void)hipMalloc(&c, 4096 * 8);
    static unsigned long long h[4096];
    auto run = [&](auto kern, const char* name, int blocks) {
        for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, o, c, 1.0000001, 0.5);
        hipDeviceSynchronize();
        hipMemcpy(h, c, blocks * 8, hipMemcpyDeviceToHost);
        double m = 0; for (int i = 0; i < blocks; ++i) m += h[i]; m /= blocks;
        printf("{\"probe\": \"%s\", \"blocks\": %d, \"cycles_per_fma\": %.2f}\n", name, blocks, m / (256.0 * 16));
    };
    for (int blocks : {256, 1024, 2048}) {
        run(k<1>, "dep1", blocks); run(k<2>, "dep2", blocks); run(k<4>, "dep4", blocks);
        run(k<8>, "dep8", blocks); run(k<16>, "indep16", blocks);
    }
    return 0;
}
