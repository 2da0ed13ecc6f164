// Diagnostic (GPU box): the bound of the finish pass's copy -- int16 staging -> int32 ids -- as plain streaming
// kernels over the cfg2 volume (209M ids), against which the finish kernel's 0.29 ms is read.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/copy_bound.hip -o tools/micro/copy_bound && ./tools/micro/copy_bound
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void widen_flat(const int16_t *__restrict__ src, int32_t *__restrict__ dst, uint64_t n) {
    // 8 ids per thread: one 16-byte load, two 16-byte stores
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i + 8 <= n) {
        const int4 v = *reinterpret_cast<const int4 *>(src + i);
        const int16_t *h = reinterpret_cast<const int16_t *>(&v);
        int4 a = make_int4(h[0], h[1], h[2], h[3]), b = make_int4(h[4], h[5], h[6], h[7]);
        *reinterpret_cast<int4 *>(dst + i) = a;
        *reinterpret_cast<int4 *>(dst + i + 4) = b;
    }
}

// per string of 256 staging slots: copy its first cnt ids to a packed output (one wave per string, 4 ids per lane)
__global__ void per_string(const int16_t *__restrict__ src, int32_t *__restrict__ dst, const uint32_t *__restrict__ cnt,
                           const uint64_t *__restrict__ pre, uint32_t n_str) {
    const uint32_t s = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (s >= n_str) return;
    const uint32_t c = cnt[s];
    const uint64_t o = pre[s];
    const int16_t *p = src + (uint64_t)s * 256;
    int32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t k = lane + 64 * u;
        v[u] = k < c ? p[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t k = lane + 64 * u;
        if (k < c) dst[o + k] = v[u];
    }
}

int main() {
    const uint32_t n_str = 1000000;
    const uint64_t slots = (uint64_t)n_str * 256, n_ids = (uint64_t)n_str * 209;
    int16_t *src; int32_t *dst; uint32_t *cnt; uint64_t *pre;
    hipMalloc(&src, slots * 2); hipMalloc(&dst, slots * 4); hipMalloc(&cnt, n_str * 4); hipMalloc(&pre, n_str * 8);
    hipMemset(src, 1, slots * 2);
    uint32_t *hc = new uint32_t[n_str]; uint64_t *hp = new uint64_t[n_str]; uint64_t acc = 0;
    for (uint32_t s = 0; s < n_str; s++) { hc[s] = 190 + (s * 2654435761u) % 40; hp[s] = acc; acc += hc[s]; }
    hipMemcpy(cnt, hc, n_str * 4, hipMemcpyHostToDevice); hipMemcpy(pre, hp, n_str * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        float ms;
        hipEventRecord(e0);
        for (int k = 0; k < 10; k++) widen_flat<<<(unsigned)((n_ids / 8 + 255) / 256), 256>>>(src, dst, n_ids);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
        printf("widen_flat  %llu ids: %.4f ms  (%.2f TB/s of 6 B per id)\n", (unsigned long long)n_ids, ms / 10, n_ids * 6.0 / (ms / 10 * 1e-3) / 1e12);
        hipEventRecord(e0);
        for (int k = 0; k < 10; k++) per_string<<<(n_str + 7) / 8, 512>>>(src, dst, cnt, pre, n_str);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
        printf("per_string  %llu ids: %.4f ms  (%.2f TB/s of 6 B per id)\n", (unsigned long long)acc, ms / 10, acc * 6.0 / (ms / 10 * 1e-3) / 1e12);
    }
    return 0;
}
