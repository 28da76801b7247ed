// Staging-cost probe: B blocks, each stages `per` doubles from its own slice into LDS
// (a) LDS-DMA in 1 region, (b) LDS-DMA in R regions, (c) plain global_load -> ds_write,
// then stores them back. Per-launch time (200 back-to-back) and block 0's in-kernel
// timeline (start, after issue, after wait) in ns, from s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) double ldsd;
typedef __attribute__((address_space(1))) double glbd;

template <int V>
__global__ void __launch_bounds__(512) k_probe(const double* __restrict__ src, double* __restrict__ out, int per,
                                               int regions, unsigned long long* st) {
    extern __shared__ __attribute__((aligned(16))) double sm_[];
    ldsd* sm = (ldsd*)sm_;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const double* s = src + (size_t)blockIdx.x * per;
    if (V == 0 || V == 1) {
        const int R = V == 0 ? 1 : regions;
        const int rlen = per / R;  // doubles per region (even)
        int rot = 0;
        for (int r = 0; r < R; ++r) {
            const int chunks = rlen / 2;
            const int g0 = ((wave - rot) % nw + nw) % nw;
            for (int c0 = g0 * 64; c0 < chunks; c0 += nw * 64) {
                const int ch = c0 + lane;
                if (ch < chunks)
                    __builtin_amdgcn_global_load_lds((const glbd*)(s + r * rlen) + 2 * ch, sm + r * rlen + 2 * c0, 16, 0, 0);
            }
            rot += (chunks + 63) >> 6;
        }
    } else {
        for (int e = threadIdx.x; e < per; e += blockDim.x) sm[e] = ((const glbd*)s)[e];
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    for (int e = threadIdx.x; e < per; e += blockDim.x) out[(size_t)blockIdx.x * per + e] = sm[e] * 1.0000001;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st[0] = t0;
        st[1] = t1;
        st[2] = t2;
        st[3] = __builtin_amdgcn_s_memrealtime();
    }
}

int main() {
    unsigned long long* st;
    hipMalloc(&st, 64);
    unsigned long long h[4];
    for (int B : {256, 512, 2048}) {
        for (int per : {1024, 4096}) {
            double *src, *out;
            hipMalloc(&src, (size_t)B * per * 8 + 64);
            hipMalloc(&out, (size_t)B * per * 8 + 64);
            hipMemset(src, 0, (size_t)B * per * 8);
            for (int v = 0; v < 3; ++v) {
                for (int R : {1, 12}) {
                    if (v != 1 && R != 1) continue;
                    auto launch = [&]() {
                        if (v == 0) k_probe<0><<<B, 512, per * 8>>>(src, out, per, R, st);
                        else if (v == 1) k_probe<1><<<B, 512, per * 8>>>(src, out, per, R, st);
                        else k_probe<2><<<B, 512, per * 8>>>(src, out, per, R, st);
                    };
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
                    hipMemcpy(h, st, 32, hipMemcpyDeviceToHost);
                    printf("B %5d per %5d (%3d KB) %s R %2d: %7.2f us/launch  blk0: issue %5lld ns  wait %5lld ns  store %5lld ns\n",
                           B, per, per * 8 / 1024, v == 2 ? "regs" : "DMA ", R, ms * 1e3 / 200, (long long)(h[1] - h[0]) * 10,
                           (long long)(h[2] - h[1]) * 10, (long long)(h[3] - h[2]) * 10);
                }
            }
            hipFree(src);
            hipFree(out);
        }
    }
    // empty-kernel floor
    for (int B : {256, 512, 2048}) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        for (int i = 0; i < 200; ++i) k_probe<2><<<B, 512, 64>>>(nullptr, nullptr, 0, 1, st);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("empty B %5d: %7.2f us/launch\n", B, ms * 1e3 / 200);
    }
    return 0;
}
