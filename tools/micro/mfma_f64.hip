// Microbenchmark (tools/micro): cycles of v_mfma_f64_16x16x4f64 chains as the CP tiles use them
// (k_cp6 / k_drc: an R = 20 product = 2 row blocks x 5 k-steps, two accumulators interleaved).
//   mode 0: A fragments from registers;  mode 1: A fragments read from LDS before each product
//   (WL::fresh, the tiles' form);  waves: 1..8 waves of the workgroup each run the chain.
// Prints cycles (s_memtime) per product (10 MFMAs) for the first wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) double ldsd;

template <int MODE>
__global__ void k_chain(double* out, long long* cyc, int reps, int nwave) {
    __shared__ double frag[10 * 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int e = threadIdx.x; e < 640; e += blockDim.x) frag[e] = 1e-3 * (e % 7);
    __syncthreads();
    if (wv >= nwave) return;
    double a[10], b[5];
    for (int q = 0; q < 10; ++q) a[q] = 1e-3 * (q + lane);
    for (int q = 0; q < 5; ++q) b[q] = 1e-2 * (q + lane);
    v4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (MODE == 1) {
            const ldsd* base = (const ldsd*)frag;
            asm volatile("" : "+v"(base));
            for (int q = 0; q < 10; ++q) a[q] = base[q * 64 + lane];
        }
        #pragma unroll
        for (int s = 0; s < 5; ++s) {
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2 * s], b[s], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2 * s + 1], b[s], acc1, 0, 0, 0);
        }
        // the next product depends on this one (as the SOC output feeds the L^T product)
        b[0] = acc0[0] + acc1[1];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc0[0] + acc0[1] + acc0[2] + acc0[3] + acc1[0] + acc1[3];
    if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
}

int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 4096 * sizeof(double));
    hipMalloc(&cyc, sizeof(long long));
    for (int mode = 0; mode < 2; ++mode)
        for (int nw : {1, 2, 4, 8}) {
            long long c = 0;
            for (int rep = 0; rep < 3; ++rep) {
                if (mode == 0) k_chain<0><<<256, 512>>>(out, cyc, 200, nw);
                else k_chain<1><<<256, 512>>>(out, cyc, 200, nw);
                hipDeviceSynchronize();
            }
            hipMemcpy(&c, cyc, sizeof(long long), hipMemcpyDeviceToHost);
            printf("mode %d (%s) waves %d: %lld cycles per 10-MFMA product\n", mode,
                   mode ? "fragments from LDS" : "fragments in registers", nw, c);
        }
    return 0;
}
