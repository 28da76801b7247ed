// Diagnostics: cycles per k_dr level (raocp_dynr.hip's back_level / fwd_level, included) on
// one workgroup of 512 lanes over LDS of random data, per node count, with the LDS barrier
// after each level. hipcc --offload-arch=gfx950 -O3 -I../../raocp-toolbox_amd/csrc
#include "raocp_dynr.hip"
#include <cstdio>

namespace raocp {
namespace {
template <int MODE, int CNT>
__global__ void __launch_bounds__(512) k_level(int iters, unsigned long long* out, double* sink) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    ldsd* sm = (ldsd*)smem_;
    for (int i = threadIdx.x; i < 16384; i += 512) sm[i] = 1e-3 * (double)((i * 37) % 101);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) back_level<20, 8, 2, 512, 1, CNT>(sm, sm + 2048, sm + 6144, 28, sm + 10240, 1.0);
        if (MODE == 1) fwd_level<20, 8, 2, 512, 1, CNT>(sm + 12288, sm + 2048, sm + 6144, 28, sm + 10240);
        if (MODE == 2) back_level<20, 8, 2, 512, 4, CNT>(sm, sm + 2048, sm + 6144, 28, sm + 10240, 1.0);
        lds_sync();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (sm[threadIdx.x] == 12345.0) sink[0] = 1.0;
}
template <int MODE, int CNT>
void run(unsigned long long* out, double* sink, const char* name) {
    const int iters = 1000;
    (void)hipFuncSetAttribute((const void*)k_level<MODE, CNT>, hipFuncAttributeMaxDynamicSharedMemorySize, 16384 * 8);
    for (int rep = 0; rep < 3; ++rep) k_level<MODE, CNT><<<1, 512, 16384 * 8>>>(iters, out, sink);
    (void)hipDeviceSynchronize();
    unsigned long long h = 0;
    (void)hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    printf("%-18s cnt %2d: %8.1f cycles / level\n", name, CNT, (double)h / iters);
}
}  // namespace
}  // namespace raocp

int main() {
    using namespace raocp;
    unsigned long long* out;
    double* sink;
    (void)hipMalloc(&out, 4096 * 8);
    (void)hipMalloc(&sink, 8);
    run<0, 1>(out, sink, "back UMAX 1");
    run<0, 2>(out, sink, "back UMAX 1");
    run<0, 8>(out, sink, "back UMAX 1");
    run<0, 32>(out, sink, "back UMAX 1");
    run<2, 8>(out, sink, "back UMAX 4");
    run<2, 32>(out, sink, "back UMAX 4");
    run<1, 1>(out, sink, "fwd UMAX 1");
    run<1, 8>(out, sink, "fwd UMAX 1");
    return 0;
}
