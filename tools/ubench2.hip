// Micro-benchmark: one 1024-thread workgroup copying a table global -> LDS (prologue cost)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d2 __attribute__((ext_vector_type(2)));

template <int U>
__global__ void __launch_bounds__(1024) k_copy(const d2* __restrict__ src, int n2, unsigned long long* out, int rep) {
    extern __shared__ d2 lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int b = threadIdx.x; b < n2; b += U * blockDim.x) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * blockDim.x;
            v[u] = src[i < n2 ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * blockDim.x;
            if (i < n2) lds[i] = v[u];
        }
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[rep] = t1 - t0 + (lds[7].x == 12345.0);
}

__global__ void __launch_bounds__(1024) k_scalar(const double* __restrict__ src, int n, unsigned long long* out, int rep) {
    extern __shared__ double ldsd[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = threadIdx.x; i < n; i += blockDim.x) ldsd[i] = src[i];
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[rep] = t1 - t0 + (ldsd[7] == 12345.0);
}

int main() {
    const int n = 10240;  // doubles (80 KB)
    double* src;
    hipMalloc(&src, n * sizeof(double));
    hipMemset(src, 0, n * sizeof(double));
    unsigned long long* out;
    hipMalloc(&out, 64 * sizeof(unsigned long long));
    unsigned long long h[64];
    hipFuncSetAttribute((const void*)k_copy<8>, hipFuncAttributeMaxDynamicSharedMemorySize, n * 8);
    hipFuncSetAttribute((const void*)k_copy<1>, hipFuncAttributeMaxDynamicSharedMemorySize, n * 8);
    hipFuncSetAttribute((const void*)k_scalar, hipFuncAttributeMaxDynamicSharedMemorySize, n * 8);
    for (int r = 0; r < 8; ++r) k_copy<8><<<1, 1024, n * 8>>>((const d2*)src, n / 2, out, r);
    hipMemcpy(h, out, 64, hipMemcpyDeviceToHost);
    printf("d2 x8 batched:");
    for (int r = 0; r < 8; ++r) printf(" %llu", h[r] * 10);
    printf(" ns\n");
    for (int r = 0; r < 8; ++r) k_copy<1><<<1, 1024, n * 8>>>((const d2*)src, n / 2, out, r);
    hipMemcpy(h, out, 64, hipMemcpyDeviceToHost);
    printf("d2 x1 loop:");
    for (int r = 0; r < 8; ++r) printf(" %llu", h[r] * 10);
    printf(" ns\n");
    for (int r = 0; r < 8; ++r) k_scalar<<<1, 1024, n * 8>>>(src, n, out, r);
    hipMemcpy(h, out, 64, hipMemcpyDeviceToHost);
    printf("scalar loop:");
    for (int r = 0; r < 8; ++r) printf(" %llu", h[r] * 10);
    printf(" ns\n");
    return 0;
}
