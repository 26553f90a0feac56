// Scatter-pattern probe (debug tool, not part of the library): one stable LSD-like scatter of
// 256 M keys whose digit takes 256 (or 16) values per 4096-key tile, written as two u32 arrays
// (key, position) or as one array of u64 records.  Destinations come from a precomputed
// permutation with the LSD pass's run structure, so only the write pattern is measured.
//   hipcc --offload-arch=gfx950 -O3 -o tools/scatter_probe tools/scatter_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
typedef uint32_t u32;
typedef uint64_t u64;

// element i (tile order, wave-quarter layout as k_lsd_scatter_w) goes to dst[i]
__global__ __launch_bounds__(256) void k_sc2(const u32* K, const u32* dst, u32* Ko, u32* Po) {
    const u32 t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 q0 = t * 4096 + w * 1024;
    u32 k[16], d[16];
#pragma unroll
    for (u32 j = 0; j < 16; ++j) {
        k[j] = K[q0 + j * 64 + lane];
        d[j] = dst[q0 + j * 64 + lane];
    }
#pragma unroll
    for (u32 j = 0; j < 16; ++j) {
        Ko[d[j]] = k[j];
        Po[d[j]] = q0 + j * 64 + lane;
    }
}
__global__ __launch_bounds__(256) void k_sc64(const u32* K, const u32* dst, u64* R) {
    const u32 t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 q0 = t * 4096 + w * 1024;
    u32 k[16], d[16];
#pragma unroll
    for (u32 j = 0; j < 16; ++j) {
        k[j] = K[q0 + j * 64 + lane];
        d[j] = dst[q0 + j * 64 + lane];
    }
#pragma unroll
    for (u32 j = 0; j < 16; ++j) R[d[j]] = ((u64)(q0 + j * 64 + lane) << 32) | k[j];
}

int main() {
    const u32 n = 1u << 28, T = 4096, nt = n / T, bs = 1u << 20, tpb = bs / T;
    std::vector<u32> hk(n), hd(n);
    for (int nv : {256, 16}) {
        uint64_t s = 88172645463325252ull;
        for (u32 i = 0; i < n; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            hk[i] = (u32)(s % nv);
        }
        // stable counting-sort destinations per 1 MiB block (tile-major within a digit)
        for (u32 b = 0; b < n / bs; ++b) {
            std::vector<u32> cnt((size_t)nv * tpb, 0);
            for (u32 i = 0; i < bs; ++i) cnt[(size_t)hk[b * bs + i] * tpb + i / T]++;
            u32 acc = b * bs;
            for (auto& c : cnt) { const u32 v = c; c = acc; acc += v; }
            for (u32 i = 0; i < bs; ++i) hd[b * bs + i] = cnt[(size_t)hk[b * bs + i] * tpb + i / T]++;
        }
        // the kernels read element (tile t, wave w, step j, lane) at index t*4096 + w*1024 + j*64 + lane,
        // which is tile order already
        u32 *dK, *dD, *dKo, *dPo;
        u64* dR;
        CK(hipMalloc(&dK, (size_t)n * 4));
        CK(hipMalloc(&dD, (size_t)n * 4));
        CK(hipMalloc(&dKo, (size_t)n * 4));
        CK(hipMalloc(&dPo, (size_t)n * 4));
        CK(hipMalloc(&dR, (size_t)n * 8));
        CK(hipMemcpy(dK, hk.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dD, hd.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        auto run = [&](const char* name, auto launch) -> int {
            for (int i = 0; i < 3; ++i) launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int i = 0; i < 10; ++i) launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%3d digit values  %-28s %7.3f ms\n", nv, name, ms / 10);
            return 0;
        };
        run("two u32 arrays", [&] { k_sc2<<<nt, 256>>>(dK, dD, dKo, dPo); });
        run("one u64 record array", [&] { k_sc64<<<nt, 256>>>(dK, dD, dR); });
        CK(hipFree(dK)); CK(hipFree(dD)); CK(hipFree(dKo)); CK(hipFree(dPo)); CK(hipFree(dR));
    }
    return 0;
}
