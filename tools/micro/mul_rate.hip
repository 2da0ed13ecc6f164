// Issue cost of 32-bit integer multiplies on gfx950 (tools/micro: measurements behind DESIGN.md choices).
// Every lane runs 8 independent chains of N steps of one op; 4 waves per SIMD on every CU.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t n, uint32_t c) {
    uint32_t x[8];
    for (int q = 0; q < 8; q++) x[q] = threadIdx.x * 8u + q + blockIdx.x;
    for (uint32_t i = 0; i < n; i++) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
            if (OP == 0) x[q] = x[q] + c;
            if (OP == 1) x[q] = x[q] * c;                                   // v_mul_lo_u32
            if (OP == 2) x[q] = __umul24(x[q], c);            // v_mul_u32_u24 (24-bit)
            if (OP == 3) x[q] = __builtin_amdgcn_alignbit(x[q], x[q], c);   // rotate
            if (OP == 4) x[q] = __umulhi(x[q], c);                          // v_mul_hi_u32
        }
    }
    uint32_t s = 0;
    for (int q = 0; q < 8; q++) s ^= x[q];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP> float run(uint32_t *d, uint32_t n, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, n, 0x9E3779B1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, n, 0x9E3779B1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}
int main() {
    const int blocks = 256 * 4;   // 4 waves per SIMD... x4 per block of 256
    const uint32_t n = 4096;
    uint32_t *d; hipMalloc(&d, blocks * 256 * 4);
    const double ops = (double)blocks * 4 * 8 * n;   // wave-instructions
    const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_u32_u24", "v_alignbit_b32", "v_mul_hi_u32"};
    float t[5] = {run<0>(d, n, blocks), run<1>(d, n, blocks), run<2>(d, n, blocks), run<3>(d, n, blocks), run<4>(d, n, blocks)};
    for (int i = 0; i < 5; i++)
        printf("%-16s %.3f ms  %.2f cycles per wave-instruction per SIMD at 2.4 GHz\n", names[i], t[i],
               t[i] * 1e-3 * 2.4e9 / (ops / 1024.0));
    return 0;
}
