// LDS-DMA issue-structure probe: B blocks x 512 threads, each stages 8 KB (512 16-B
// chunks) from its slice into LDS in R regions of 512/R chunks, each region issued
// either by wave (r mod 8) (spread) or all by wave 0, then stores the slice back.
// Reports us/launch over 200 back-to-back launches.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) double ldsd;
typedef __attribute__((address_space(1))) double glbd;

__global__ void __launch_bounds__(512) k_probe(const double* __restrict__ src, double* __restrict__ out, int R,
                                               int spread, int wait_each) {
    extern __shared__ __attribute__((aligned(16))) double sm_[];
    ldsd* sm = (ldsd*)sm_;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int per = 1024, rch = 512 / R;
    const double* s = src + (size_t)blockIdx.x * per;
    for (int r = 0; r < R; ++r) {
        const int owner = spread ? (r & 7) : 0;
        if (wave != owner) continue;
        for (int c0 = 0; c0 < rch; c0 += 64) {
            const int ch = c0 + lane;
            if (ch < rch)
                __builtin_amdgcn_global_load_lds((const glbd*)(s + r * 2 * rch) + 2 * ch, sm + r * 2 * rch + 2 * c0, 16, 0, 0);
        }
        if (wait_each) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int e = threadIdx.x; e < per; e += blockDim.x) out[(size_t)blockIdx.x * per + e] = sm[e] * 1.0000001;
}

int main() {
    for (int B : {256, 2048}) {
        double *src, *out;
        hipMalloc(&src, (size_t)B * 1024 * 8 + 64);
        hipMalloc(&out, (size_t)B * 1024 * 8 + 64);
        hipMemset(src, 0, (size_t)B * 1024 * 8);
        for (int R : {1, 8, 16, 32, 64}) {
            for (int spread = 0; spread < 2; ++spread) {
                for (int we = 0; we < 2; ++we) {
                    auto launch = [&]() { k_probe<<<B, 512, 8192>>>(src, out, R, spread, we); };
                    for (int i = 0; i < 10; ++i) launch();
                    hipEvent_t e0, e1;
                    hipEventCreate(&e0);
                    hipEventCreate(&e1);
                    hipEventRecord(e0);
                    for (int i = 0; i < 200; ++i) launch();
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    printf("B %5d  R %2d (%3d chunks/region)  %s  %s: %7.2f us/launch\n", B, R, 512 / R,
                           spread ? "spread " : "wave 0 ", we ? "wait-each" : "no-wait  ", ms * 1e3 / 200);
                }
            }
        }
        hipFree(src);
        hipFree(out);
    }
    return 0;
}
