// Micro-benchmarks of the latencies the dependent dynamics sweep is built from (gfx950):
// workgroup barrier, dependent LDS read, dependent global (L2-hit) read, xor-shuffle.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_barrier(int iters, unsigned long long* out) {
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = clock64();
    for (int i = 0; i < iters; ++i) __syncthreads();
    const long long c1 = clock64();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = c1 - c0; }
}

__global__ void k_lds_chain(int iters, unsigned long long* out) {
    __shared__ int buf[1024];
    buf[threadIdx.x] = (threadIdx.x + 1) & 1023;
    __syncthreads();
    int p = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = clock64();
    for (int i = 0; i < iters; ++i) p = buf[p];
    const long long c1 = clock64();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = p; }
}

__global__ void k_glb_chain(const int* __restrict__ nxt, int iters, unsigned long long* out) {
    int p = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = clock64();
    for (int i = 0; i < iters; ++i) p = nxt[p];
    const long long c1 = clock64();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = p; }
}

__global__ void k_shfl_chain(int iters, unsigned long long* out) {
    double v = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = clock64();
    for (int i = 0; i < iters; ++i) v = __shfl_xor(v, 1, 64) + 1.0;
    const long long c1 = clock64();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = (unsigned long long)v; }
}

// barrier + LDS write/read round trip (one "phase" hand-off)
__global__ void k_handoff(int iters, unsigned long long* out) {
    __shared__ double buf[1024];
    double v = threadIdx.x;
    buf[threadIdx.x] = v;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = clock64();
    for (int i = 0; i < iters; ++i) {
        v = buf[(threadIdx.x + 1) & 1023] + 1.0;
        __syncthreads();
        buf[threadIdx.x] = v;
        __syncthreads();
    }
    const long long c1 = clock64();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = (unsigned long long)v; }
}

int main() {
    unsigned long long* d_out;
    hipMalloc(&d_out, 64);
    int* d_nxt;
    std::vector<int> h(64);
    for (int i = 0; i < 64; ++i) h[i] = (i + 1) & 63;
    hipMalloc(&d_nxt, 64 * sizeof(int));
    hipMemcpy(d_nxt, h.data(), 64 * sizeof(int), hipMemcpyHostToDevice);
    unsigned long long r[4];
    const int it = 10000;
    auto report = [&](const char* name, int iters) {
        hipMemcpy(r, d_out, 32, hipMemcpyDeviceToHost);
        printf("%-28s %8.1f ns/op  %8.1f clk/op  (clk/ns %.2f)\n", name, r[0] * 10.0 / iters, (double)r[1] / iters,
               (double)r[1] / (r[0] * 10.0));
    };
    for (int threads : {64, 256, 1024}) {
        for (int rep = 0; rep < 2; ++rep) k_barrier<<<1, threads>>>(it, d_out);
        hipDeviceSynchronize();
        char nm[64];
        snprintf(nm, 64, "barrier (%d thr)", threads);
        report(nm, it);
    }
    for (int rep = 0; rep < 2; ++rep) k_lds_chain<<<1, 64>>>(it, d_out);
    hipDeviceSynchronize();
    report("dependent LDS read", it);
    for (int rep = 0; rep < 3; ++rep) k_glb_chain<<<1, 64>>>(d_nxt, it, d_out);
    hipDeviceSynchronize();
    report("dependent global read (L2)", it);
    for (int rep = 0; rep < 2; ++rep) k_shfl_chain<<<1, 64>>>(it, d_out);
    hipDeviceSynchronize();
    report("dependent shfl_xor+add", it);
    for (int threads : {256, 1024}) {
        for (int rep = 0; rep < 2; ++rep) k_handoff<<<1, threads>>>(it, d_out);
        hipDeviceSynchronize();
        char nm[64];
        snprintf(nm, 64, "LDS handoff 2 barriers (%d)", threads);
        report(nm, it);
    }
    return 0;
}
