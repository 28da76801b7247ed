// Layout check of v_mfma_f64_16x16x4f64 on gfx950: D = A (16x4) B (4x16) with
// A fragment lane l -> A[l % 16][l / 16], B fragment lane l -> B[l / 16][l % 16];
// prints where D[i][j] lands (lane, element) by matching against the host product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_mfma(const double* A, const double* B, double* out) {
    const int l = threadIdx.x;
    const double a = A[(l % 16) * 4 + l / 16];  // A row-major 16x4
    const double b = B[(l / 16) * 16 + l % 16];  // B row-major 4x16
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int v = 0; v < 4; ++v) out[l * 4 + v] = c[v];
}

int main() {
    double hA[64], hB[64], hD[256], out[256];
    for (int i = 0; i < 64; ++i) { hA[i] = 1.0 + i * 0.37; hB[i] = 2.0 - i * 0.11; }
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += hA[i * 4 + k] * hB[k * 16 + j];
            hD[i * 16 + j] = s;
        }
    double *A, *B, *O;
    hipMalloc(&A, 512); hipMalloc(&B, 512); hipMalloc(&O, 2048);
    hipMemcpy(A, hA, 512, hipMemcpyHostToDevice);
    hipMemcpy(B, hB, 512, hipMemcpyHostToDevice);
    k_mfma<<<1, 64>>>(A, B, O);
    hipMemcpy(out, O, 2048, hipMemcpyDeviceToHost);
    int ok = 0, guess = 0;
    for (int l = 0; l < 64; ++l)
        for (int v = 0; v < 4; ++v) {
            const int i = 4 * (l / 16) + v, j = l % 16;  // guessed layout
            if (fabs(out[l * 4 + v] - hD[i * 16 + j]) <= 1e-12 * fabs(hD[i * 16 + j])) ++guess;
            for (int q = 0; q < 256; ++q)
                if (out[l * 4 + v] == hD[q]) { ++ok; if (l < 2 || l == 16) printf("lane %2d v %d -> D[%d][%d]\n", l, v, q / 16, q % 16); break; }
        }
    printf("exact matches %d / 256, guessed layout (row 4*(l/16)+v, col l%%16) within 1e-12: %d / 256\n", ok, guess);
    return 0;
}
