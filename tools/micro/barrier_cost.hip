// Diagnostics: cycles per iteration of the k_dr level skeleton pieces on one workgroup of 512
// lanes (8 waves): a bare LDS barrier, a counted vmcnt wait through a 64-way switch, the
// scalar index arithmetic of a level, and an LDS-DMA issue. hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
#define VM(n) case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vm(int n) {
    switch (n < 15 ? n : 15) { VM(0) VM(1) VM(2) VM(3) VM(4) VM(5) VM(6) VM(7) VM(8) VM(9) VM(10) VM(11) VM(12) VM(13) VM(14)
        default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break; }
}
__device__ __forceinline__ int ipow(int b, int e) { int v = 1; for (int i = 0; i < e; ++i) v *= b; return v; }

__global__ void __launch_bounds__(512) k(int mode, int iters, int C, unsigned long long* out, int* sink) {
    __shared__ double lds[4096];
    int acc = 0;
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (mode == 1) wait_vm((i * 7) & 15);
        if (mode == 2) acc += (ipow(C, i & 7) - 1) / (C - 1) + ipow(C, (i + 3) & 7);
        if (mode == 3) acc += (int)lds[(threadIdx.x * 3 + i) & 4095];
        if (mode == 4) {
            double v = lds[(threadIdx.x + i) & 4095];
            lds[(threadIdx.x + 64 + i) & 4095] = v + 1.0;
        }
        lds_sync();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r0; }
    if (acc == 12345) sink[0] = acc;
}

int main() {
    unsigned long long* out; int* sink;
    hipMalloc(&out, 4096 * 8); hipMalloc(&sink, 4);
    const char* names[] = {"barrier", "wait_vm + barrier", "index math + barrier", "lds read + barrier", "lds rw + barrier"};
    for (int grid : {1, 256}) for (int mode = 0; mode < 5; ++mode) {
        const int iters = 1000;
        for (int rep = 0; rep < 3; ++rep) k<<<grid, 512>>>(mode, iters, 2, out, sink);
        hipDeviceSynchronize();
        unsigned long long h[2];
        hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        printf("grid %3d %-22s %8.1f cycles / iteration\n", grid, names[mode], (double)h[0] / iters);
    }
    return 0;
}
