// Read-bandwidth probe (debug tool, not part of the library): how fast can a 1 GiB array of
// u32 keys be streamed in the access shapes of the LSD histogram pass?  Prints GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe tools/bw_probe.hip && ./tools/bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32;
constexpr u32 T = 4096;  // elements per tile

// plain read: each workgroup reads its 16 KB tile (4 x uint4 per thread), xor-reduces
__global__ __launch_bounds__(256) void k_read(const uint4* K, u32* out) {
    const uint4* p = K + (size_t)blockIdx.x * (T / 4);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[q * 256 + threadIdx.x];
    u32 x = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) x ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    if (x == 0x12345678u) out[0] = x;
}

// the histogram pass's shape: per-wave LDS histograms of one byte digit, 256 counts written
template <int P>
__global__ __launch_bounds__(256) void k_hist(const uint4* K, u32* hist) {
    __shared__ u32 h[4][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i][tid] = 0;
    __syncthreads();
    const uint4* p = K + (size_t)blockIdx.x * (T / 4);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[q * 256 + tid];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        atomicAdd(&h[w][(v[q].x >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].y >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].z >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].w >> (8 * P)) & 255], 1u);
    }
    __syncthreads();
    hist[(size_t)blockIdx.x * 256 + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

// the same with the tile's loads issued before the LDS clear (no barrier ahead of them)
template <int P>
__global__ __launch_bounds__(256) void k_hist_early(const uint4* K, u32* hist) {
    __shared__ u32 h[4][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
    const uint4* p = K + (size_t)blockIdx.x * (T / 4);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[q * 256 + tid];
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i][tid] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        atomicAdd(&h[w][(v[q].x >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].y >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].z >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].w >> (8 * P)) & 255], 1u);
    }
    __syncthreads();
    hist[(size_t)blockIdx.x * 256 + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

// two tiles per workgroup, the second tile's loads in flight while the first is counted
template <int P>
__global__ __launch_bounds__(256) void k_hist2(const uint4* K, u32* hist) {
    __shared__ u32 h[2][4][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
    const uint4* p = K + (size_t)blockIdx.x * (2 * T / 4);
    uint4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = p[q * 256 + tid];
#pragma unroll
    for (int i = 0; i < 4; ++i) h[0][i][tid] = h[1][i][tid] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        u32* hh = h[q >> 2][w];
        atomicAdd(&hh[(v[q].x >> (8 * P)) & 255], 1u);
        atomicAdd(&hh[(v[q].y >> (8 * P)) & 255], 1u);
        atomicAdd(&hh[(v[q].z >> (8 * P)) & 255], 1u);
        atomicAdd(&hh[(v[q].w >> (8 * P)) & 255], 1u);
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t)
        hist[((size_t)blockIdx.x * 2 + t) * 256 + tid] = h[t][0][tid] + h[t][1][tid] + h[t][2][tid] + h[t][3][tid];
}

// the histogram with the per-(block, part) totals of k_lsd_hist (16 tiles per part: 16 workgroups
// add into the same 256 counters)
template <int P>
__global__ __launch_bounds__(256) void k_hist_parts(const uint4* K, u32* hist, u32* parts) {
    __shared__ u32 h[4][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i][tid] = 0;
    __syncthreads();
    const uint4* p = K + (size_t)blockIdx.x * (T / 4);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[q * 256 + tid];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        atomicAdd(&h[w][(v[q].x >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].y >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].z >> (8 * P)) & 255], 1u);
        atomicAdd(&h[w][(v[q].w >> (8 * P)) & 255], 1u);
    }
    __syncthreads();
    const u32 c = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
    hist[(size_t)blockIdx.x * 256 + tid] = c;
    if (c) atomicAdd(&parts[(size_t)(blockIdx.x >> 4) * 256 + tid], c);
}

// 4 copies per wave (lane & 3): a same-value instruction hits 4 addresses of 16 lanes each
template <int P>
__global__ __launch_bounds__(256) void k_hist_c4(const uint4* K, u32* hist) {
    __shared__ u32 h[16][257];
    const u32 tid = threadIdx.x, cp = (tid >> 6) * 4 + (tid & 3);
#pragma unroll
    for (int i = 0; i < 16; ++i) h[i][tid] = 0;
    __syncthreads();
    const uint4* p = K + (size_t)blockIdx.x * (T / 4);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[q * 256 + tid];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        atomicAdd(&h[cp][(v[q].x >> (8 * P)) & 255], 1u);
        atomicAdd(&h[cp][(v[q].y >> (8 * P)) & 255], 1u);
        atomicAdd(&h[cp][(v[q].z >> (8 * P)) & 255], 1u);
        atomicAdd(&h[cp][(v[q].w >> (8 * P)) & 255], 1u);
    }
    __syncthreads();
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) c += h[i][tid];
    hist[(size_t)blockIdx.x * 256 + tid] = c;
}

// one hot value per wave (the digit of the wave's first element): its lanes are counted by a
// ballot into a register, only the other lanes go to the LDS atomics
template <int P>
__global__ __launch_bounds__(256) void k_hist_hot(const uint4* K, u32* hist) {
    __shared__ u32 h[4][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i][tid] = 0;
    __syncthreads();
    const uint4* p = K + (size_t)blockIdx.x * (T / 4);
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[q * 256 + tid];
    const u32 hot = __builtin_amdgcn_readfirstlane((v[0].x >> (8 * P)) & 255);
    u32 nh = 0;
    auto add = [&](u32 k) {
        const u32 d = (k >> (8 * P)) & 255;
        const bool is = d == hot;
        nh += (u32)__popcll(__ballot(is));
        if (!is) atomicAdd(&h[w][d], 1u);
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        add(v[q].x);
        add(v[q].y);
        add(v[q].z);
        add(v[q].w);
    }
    if ((tid & 63) == 0 && nh) atomicAdd(&h[w][hot], nh);
    __syncthreads();
    hist[(size_t)blockIdx.x * 256 + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

int main() {
    const size_t n = (size_t)1 << 28;  // 256 M keys = 1 GiB
    const u32 nt = (u32)(n / T);
    std::vector<u32> hk(n);
    // text-like digits: 6-bit codes with a skewed distribution packed 5 per key
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < n; ++i) {
        u32 k = 0;
        for (int c = 0; c < 5; ++c) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            const u32 r = (u32)s & 1023;
            const u32 code = r < 512 ? (r & 7) : r < 800 ? 8 + (r & 15) : (r % 50);
            k = (k << 6) | code;
        }
        hk[i] = k << 2;
    }
    uint4* dk;
    u32 *dh, *dout;
    CK(hipMalloc(&dk, n * 4));
    CK(hipMalloc(&dh, (size_t)nt * 256 * 4));
    CK(hipMalloc(&dout, 64));
    CK(hipMemcpy(dk, hk.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) -> int {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        const int R = 20;
        for (int i = 0; i < R; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        printf("%-24s %8.3f ms  %7.1f GB/s (keys read)\n", name, ms, n * 4 / (ms * 1e6));
        return 0;
    };
    run("read uint4 tiles", [&] { k_read<<<nt, 256>>>(dk, dout); });
    run("hist digit 0", [&] { k_hist<0><<<nt, 256>>>(dk, dh); });
    run("hist digit 2", [&] { k_hist<2><<<nt, 256>>>(dk, dh); });
    run("hist early digit 2", [&] { k_hist_early<2><<<nt, 256>>>(dk, dh); });
    run("hist 2 tiles digit 2", [&] { k_hist2<2><<<nt / 2, 256>>>(dk, dh); });
    run("hist c4 digit 2", [&] { k_hist_c4<2><<<nt, 256>>>(dk, dh); });
    run("hist hot digit 2", [&] { k_hist_hot<2><<<nt, 256>>>(dk, dh); });
    u32* dp;
    CK(hipMalloc(&dp, (size_t)(nt / 16 + 1) * 256 * 4));
    run("hist + part totals", [&] { k_hist_parts<2><<<nt, 256>>>(dk, dh, dp); });
    // concentrated digits: 60 % of the keys share digit 2's value
    for (size_t i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        if (((u32)s & 1023) < 614) hk[i] = (hk[i] & ~0x00FF0000u) | 0x00200000u;
    }
    CK(hipMemcpy(dk, hk.data(), n * 4, hipMemcpyHostToDevice));
    run("hist 60% one digit", [&] { k_hist<2><<<nt, 256>>>(dk, dh); });
    run("hist c4 60%", [&] { k_hist_c4<2><<<nt, 256>>>(dk, dh); });
    run("hist hot 60%", [&] { k_hist_hot<2><<<nt, 256>>>(dk, dh); });
    run("hist+parts 60% one digit", [&] { k_hist_parts<2><<<nt, 256>>>(dk, dh, dp); });
    for (size_t i = 0; i < n; ++i) hk[i] = (hk[i] & ~0x00FF0000u) | 0x00200000u;
    CK(hipMemcpy(dk, hk.data(), n * 4, hipMemcpyHostToDevice));
    run("hist 100% one digit", [&] { k_hist<2><<<nt, 256>>>(dk, dh); });
    run("hist c4 100%", [&] { k_hist_c4<2><<<nt, 256>>>(dk, dh); });
    run("hist hot 100%", [&] { k_hist_hot<2><<<nt, 256>>>(dk, dh); });
    return 0;
}
