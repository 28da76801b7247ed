// Issue rate and dependent latency of v_mfma_f64_16x16x4f64 / v_mfma_f32_16x16x4f32 on gfx950
// (one wave per SIMD, 256 CUs): cycles per MFMA with 1 (dependent chain) and 4 independent
// accumulators. hipcc --offload-arch=gfx950 -O3 tools/ubench7.hip -o tools/ubench7
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) k64(double a, double b, double* out, long long* cyc, int iters) {
    d4 c[NACC];
    for (int q = 0; q < NACC; ++q) c[q] = d4{0, 0, 0, 0};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[q], 0, 0, 0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int q = 0; q < NACC; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NACC>
__global__ void __launch_bounds__(256) k32(float a, float b, float* out, long long* cyc, int iters) {
    f4 c[NACC];
    for (int q = 0; q < NACC; ++q) c[q] = f4{0, 0, 0, 0};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[q], 0, 0, 0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int q = 0; q < NACC; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K, class T>
void run(const char* name, K kern, int nacc, T a, T b) {
    const int blocks = 256, iters = 4096;
    T* out;
    long long* cyc;
    hipMalloc(&out, blocks * 256 * sizeof(T));
    hipMalloc(&cyc, blocks * sizeof(long long));
    kern<<<blocks, 256>>>(a, b, out, cyc, iters);
    hipDeviceSynchronize();
    kern<<<blocks, 256>>>(a, b, out, cyc, iters);
    hipDeviceSynchronize();
    long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks; ++i) mean += (double)h[i];
    mean /= blocks;
    printf("%-8s acc=%d: %.1f cycles per MFMA per wave (s_memtime ticks)\n", name, nacc, mean / ((double)iters * nacc));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run("f64", k64<1>, 1, 1.0, 1e-9);
    run("f64", k64<4>, 4, 1.0, 1e-9);
    run("f64", k64<8>, 8, 1.0, 1e-9);
    run("f32", k32<1>, 1, 1.0f, 1e-9f);
    run("f32", k32<4>, 4, 1.0f, 1e-9f);
    return 0;
}
