// Floor of a "stage-then-compute" block structure: grid of B blocks x 256 threads, each
// block: scalar table load, LDS-DMA of S KB, barrier, light compute from LDS, coalesced store.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) double ldsd;
typedef __attribute__((address_space(1))) double glbd;

template <int VARIANT>
__global__ void __launch_bounds__(256) k_stage(const double* __restrict__ src, const int4* __restrict__ tbl,
                                               double* __restrict__ out, int per_block, const int* done) {
    extern __shared__ __attribute__((aligned(16))) double sm_[];
    ldsd* sm = (ldsd*)sm_;
    if (*done) return;
    const int4 r = tbl[blockIdx.x];
    const int base = r.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int chunks = per_block / 2;
    if (VARIANT == 0) {
        for (int c0 = wave * 64; c0 < chunks; c0 += 4 * 64) {
            const int ch = c0 + lane;
            if (ch < chunks)
                __builtin_amdgcn_global_load_lds((const glbd*)src + base + 2 * ch, sm + 2 * c0, 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    } else {
        for (int e = threadIdx.x; e < per_block; e += 256) sm[e] = src[base + e];
        __syncthreads();
    }
    double acc = 0.0;
    for (int k = 0; k < 20; ++k) acc = fma(sm[(threadIdx.x + k * 7) % per_block], 1.0001, acc);
    for (int e = threadIdx.x; e < per_block; e += 256) out[base + e] = sm[e] + acc * 1e-30;
}

int main() {
    const int per = 640;  // doubles per block (5 KB)
    unsigned long long h[8];
    (void)h;
    for (int B : {512, 1024, 2300, 4600}) {
        double *src, *out;
        int4* tbl;
        int* done;
        hipMalloc(&src, (size_t)B * per * 8 + 64);
        hipMalloc(&out, (size_t)B * per * 8 + 64);
        hipMalloc(&tbl, B * 16);
        hipMalloc(&done, 4);
        hipMemset(done, 0, 4);
        hipMemset(src, 0, (size_t)B * per * 8);
        int4* ht = new int4[B];
        for (int b = 0; b < B; ++b) ht[b] = make_int4(b * per, 0, 0, 0);
        hipMemcpy(tbl, ht, B * 16, hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int v = 0; v < 2; ++v) {
            for (int i = 0; i < 10; ++i) {
                if (v == 0) k_stage<0><<<B, 256, per * 8>>>(src, tbl, out, per, done);
                else k_stage<1><<<B, 256, per * 8>>>(src, tbl, out, per, done);
            }
            hipEventRecord(e0);
            for (int i = 0; i < 200; ++i) {
                if (v == 0) k_stage<0><<<B, 256, per * 8>>>(src, tbl, out, per, done);
                else k_stage<1><<<B, 256, per * 8>>>(src, tbl, out, per, done);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("blocks %5d  %s  %7.2f us/launch  (%.1f GB/s in+out)\n", B, v == 0 ? "DMA " : "regs", ms * 1e3 / 200,
                   2.0 * B * per * 8 / (ms / 200 * 1e-3) / 1e9);
        }
        hipFree(src); hipFree(out); hipFree(tbl); hipFree(done);
        delete[] ht;
    }
    return 0;
}
