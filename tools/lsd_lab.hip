// Round-0 LSD laboratory (stand-alone, not part of the library): times variants of the
// per-block stable sort of 60-bit rotation keys on 256 MiB of text, solo, and checks them
// against a host stable sort on a few blocks.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lsd_lab.hip -o build/lsd_lab
//   python -c "..." > /tmp/text.bin ; build/lsd_lab /tmp/text.bin [variant]
// Keys: C = 10 six-bit codes of the block's rotation starting at each position
// (wrapping at the block end), left-aligned in 64 bits: KA = low 32 bits, KB = high 32.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "HIP %s at %d: %s\n", hipGetErrorString(e), __LINE__, #x); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr u32 BS = 1u << 20;  // block size
constexpr u32 C = 10, W = 6, SH = 4;

__global__ void k_keys(const u8* text, const u8* code, u32 N, u32* KA, u32* KB) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const u32 b0 = p & ~(BS - 1), bn = min(BS, N - b0);
    u64 key = 0;
    for (u32 k = 0; k < C; ++k) {
        u32 q = p - b0 + k;
        if (q >= bn) q -= bn;
        key = (key << W) | code[text[b0 + q]];
    }
    key <<= SH;
    KA[p] = (u32)key;
    KB[p] = (u32)(key >> 32);
}

// ---------------------------------------------------------------------------------
// Variant S: one workgroup sweeps one block through all 8 passes (no histogram passes,
// no launches between passes).  NT threads = NW waves; chunks of CH = NW * 64 * SPW
// elements; wave w owns the contiguous CH / NW elements of a chunk (SPW steps of 64).
// Records (KA, KB, P) in three SoA arrays, ping-pong between two sets.
// ---------------------------------------------------------------------------------
template <int NW, int SPW>
__global__ __launch_bounds__(NW * 64) void k_sweep(u32 N, const u32* KA0, const u32* KB0, u32* A1, u32* B1, u32* P1,
                                                  u32* A2, u32* B2, u32* P2) {
    constexpr u32 NT = NW * 64, CH = NT * SPW, PW = CH / NW;
    __shared__ u32 hist[8][256];
    __shared__ u32 run[256];
    __shared__ u16 wc[NW][256];
    __shared__ u32 wb[NW][256];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 b = blockIdx.x;
    const u32 base = b * BS, n = min(BS, N - base);
    for (u32 i = tid; i < 8 * 256; i += NT) (&hist[0][0])[i] = 0;
    for (u32 i = tid; i < NW * 256; i += NT) (&wc[0][0])[i] = 0;
    __syncthreads();
    // all 8 digit histograms (the block's digit counts do not change between passes)
    for (u32 i = tid * 4; i < n; i += NT * 4) {
        const uint4 a = *reinterpret_cast<const uint4*>(KA0 + base + i);
        const uint4 c = *reinterpret_cast<const uint4*>(KB0 + base + i);
        const u32 av[4] = {a.x, a.y, a.z, a.w}, cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (i + e >= n) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                atomicAdd(&hist[q][(av[e] >> (8 * q)) & 255], 1u);
                atomicAdd(&hist[4 + q][(cv[e] >> (8 * q)) & 255], 1u);
            }
        }
    }
    __syncthreads();
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int p = 0; p < 8; ++p) {
        // run[d] = block base + exclusive prefix of digit counts
        if (tid < 64) {
            u32 v[4], s = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = hist[p][tid * 4 + q], s += v[q];
            u32 inc = s;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 t = __shfl_up(inc, o);
                if (lane >= o) inc += t;
            }
            u32 ex = inc - s;
#pragma unroll
            for (int q = 0; q < 4; ++q) run[tid * 4 + q] = base + ex, ex += v[q];
        }
        __syncthreads();
        const u32 *sa, *sb, *sp;
        u32 *da, *db, *dp;
        if (p == 0) sa = KA0, sb = KB0, sp = nullptr;
        else if (p & 1) sa = A1, sb = B1, sp = P1;
        else sa = A2, sb = B2, sp = P2;
        if (p & 1) da = A2, db = B2, dp = P2;
        else da = A1, db = B1, dp = P1;
        const u32 sh = 8 * (p & 3);
        for (u32 c0 = 0; c0 < n; c0 += CH) {
            u32 ka[SPW], kb[SPW], ps[SPW];
            u16 rk[SPW];
            const u32 q0 = base + c0 + w * PW;
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                const u32 i = q0 + j * 64 + lane;
                const bool v = i < base + n;
                ka[j] = v ? sa[i] : 0u;
                kb[j] = v ? sb[i] : 0u;
                ps[j] = v ? (sp ? sp[i] : i) : 0u;
            }
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                const bool v = q0 + j * 64 + lane < base + n;
                const u32 d = ((p < 4 ? ka[j] : kb[j]) >> sh) & 255u;
                u64 m = __ballot(v);
#pragma unroll
                for (int bit = 0; bit < 8; ++bit) {
                    const u64 bb = __ballot((d >> bit) & 1u);
                    m &= ((d >> bit) & 1u) ? bb : ~bb;
                }
                const u32 r = __popcll(m & lt);
                const u32 pre = v ? wc[w][d] : 0u;
                rk[j] = (u16)(pre + r);
                if (v && r == 0) wc[w][d] = (u16)(pre + __popcll(m));
            }
            __syncthreads();
            if (tid < 256) {
                u32 acc = run[tid];
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    const u32 cnt = wc[q][tid];
                    wb[q][tid] = acc;
                    wc[q][tid] = 0;
                    acc += cnt;
                }
                run[tid] = acc;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                if (q0 + j * 64 + lane < base + n) {
                    const u32 d = ((p < 4 ? ka[j] : kb[j]) >> sh) & 255u;
                    const u32 dst = wb[w][d] + rk[j];
                    da[dst] = ka[j];
                    db[dst] = kb[j];
                    dp[dst] = ps[j];
                }
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------
// Variant G: the same sweep with DB-bit digits over the 60 code bits (bits SH..63 of the
// 64-bit key), P = ceil(60 / DB) passes, all P digit histograms from one pre-pass.
// ---------------------------------------------------------------------------------
template <int DB, int NW, int SPW>
__global__ __launch_bounds__(NW * 64) void k_sweepg(u32 N, const u32* KA0, const u32* KB0, u32* A1, u32* B1, u32* P1,
                                                   u32* A2, u32* B2, u32* P2) {
    constexpr u32 NT = NW * 64, CH = NT * SPW, PW = CH / NW, R = 1u << DB, P = (60 + DB - 1) / DB;
    __shared__ u32 hist[P][R];
    __shared__ u32 run[R];
    __shared__ u16 wc[NW][R];
    __shared__ u32 wb[NW][R];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 b = blockIdx.x;
    const u32 base = b * BS, n = min(BS, N - base);
    for (u32 i = tid; i < P * R; i += NT) (&hist[0][0])[i] = 0;
    for (u32 i = tid; i < NW * R; i += NT) (&wc[0][0])[i] = 0;
    __syncthreads();
    for (u32 i = tid; i < n; i += NT) {
        const u64 key = (u64)KB0[base + i] << 32 | KA0[base + i];
#pragma unroll
        for (u32 q = 0; q < P; ++q) atomicAdd(&hist[q][(key >> (SH + DB * q)) & (R - 1)], 1u);
    }
    __syncthreads();
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (u32 p = 0; p < P; ++p) {
        if (tid < 64) {
            constexpr u32 PER = R / 64;
            u32 v[PER], s = 0;
#pragma unroll
            for (u32 q = 0; q < PER; ++q) v[q] = hist[p][tid * PER + q], s += v[q];
            u32 inc = s;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 t = __shfl_up(inc, o);
                if ((int)lane >= o) inc += t;
            }
            u32 ex = inc - s;
#pragma unroll
            for (u32 q = 0; q < PER; ++q) run[tid * PER + q] = base + ex, ex += v[q];
        }
        __syncthreads();
        const u32 *sa, *sb, *sp;
        u32 *da, *db, *dp;
        if (p == 0) sa = KA0, sb = KB0, sp = nullptr;
        else if (p & 1) sa = A1, sb = B1, sp = P1;
        else sa = A2, sb = B2, sp = P2;
        if (p & 1) da = A2, db = B2, dp = P2;
        else da = A1, db = B1, dp = P1;
        const u32 sh = SH + DB * p;
        for (u32 c0 = 0; c0 < n; c0 += CH) {
            u32 ka[SPW], kb[SPW], ps[SPW];
            u16 rk[SPW];
            const u32 q0 = base + c0 + w * PW;
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                const u32 i = q0 + j * 64 + lane;
                const bool v = i < base + n;
                ka[j] = v ? sa[i] : 0u;
                kb[j] = v ? sb[i] : 0u;
                ps[j] = v ? (sp ? sp[i] : i) : 0u;
            }
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                const bool v = q0 + j * 64 + lane < base + n;
                const u32 d = (u32)((((u64)kb[j] << 32) | ka[j]) >> sh) & (R - 1);
                u64 m = __ballot(v);
#pragma unroll
                for (int bit = 0; bit < DB; ++bit) {
                    const u64 bb = __ballot((d >> bit) & 1u);
                    m &= ((d >> bit) & 1u) ? bb : ~bb;
                }
                const u32 r = __popcll(m & lt);
                const u32 pre = v ? wc[w][d] : 0u;
                rk[j] = (u16)(pre + r);
                if (v && r == 0) wc[w][d] = (u16)(pre + __popcll(m));
            }
            __syncthreads();
            for (u32 dd = tid; dd < R; dd += NT) {
                u32 acc = run[dd];
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    const u32 cnt = wc[q][dd];
                    wb[q][dd] = acc;
                    wc[q][dd] = 0;
                    acc += cnt;
                }
                run[dd] = acc;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                if (q0 + j * 64 + lane < base + n) {
                    const u32 d = (u32)((((u64)kb[j] << 32) | ka[j]) >> sh) & (R - 1);
                    const u32 dst = wb[w][d] + rk[j];
                    da[dst] = ka[j];
                    db[dst] = kb[j];
                    dp[dst] = ps[j];
                }
            }
        }
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: lsd_lab text.bin\n");
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    std::vector<u8> text;
    {
        fseek(f, 0, SEEK_END);
        long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        text.resize(n);
        if (fread(text.data(), 1, n, f) != (size_t)n) return 3;
        fclose(f);
    }
    const u32 N = (u32)text.size();
    const u32 nb = (N + BS - 1) / BS;
    u8 code[256];
    {
        bool pres[256] = {};
        for (u8 c : text) pres[c] = true;
        u32 r = 0;
        for (int c = 0; c < 256; ++c) code[c] = pres[c] ? r++ : 0;
        printf("N %u blocks %u sigma %u\n", N, nb, r);
    }
    u8 *d_text, *d_code;
    u32 *KA, *KB, *A1, *B1, *P1, *A2, *B2, *P2;
    CK(hipMalloc(&d_text, N + 64));
    CK(hipMalloc(&d_code, 256));
    for (u32** p : {&KA, &KB, &A1, &B1, &P1, &A2, &B2, &P2}) CK(hipMalloc(p, (size_t)N * 4 + 64));
    CK(hipMemcpy(d_text, text.data(), N, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_code, code, 256, hipMemcpyHostToDevice));
    k_keys<<<(N + 255) / 256, 256>>>(d_text, d_code, N, KA, KB);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        const int R = 5;
        for (int r = 0; r < R; ++r) {
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            sum += ms;
        }
        printf("%-28s best %.3f ms  avg %.3f ms  (%.2f GB/s at 24 B/elem/pass)\n", name, best, sum / R,
               (double)N * (8 * 24) / (best * 1e-3) / 1e9);
    };
    // host reference for the first and last block: stable sort of positions by the 64-bit key
    auto check = [&](const char* name, const u32* dA, const u32* dB, const u32* dP) {
        std::vector<u32> ka(N), kb(N), pp(N), ra(N), rb(N);
        CK(hipMemcpy(ka.data(), KA, (size_t)N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(kb.data(), KB, (size_t)N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ra.data(), dA, (size_t)N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(rb.data(), dB, (size_t)N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pp.data(), dP, (size_t)N * 4, hipMemcpyDeviceToHost));
        u64 bad = 0;
        for (u32 b : {0u, nb / 2, nb - 1}) {
            const u32 lo = b * BS, n = std::min(BS, N - lo);
            std::vector<u32> idx(n);
            std::iota(idx.begin(), idx.end(), lo);
            auto K = [&](u32 i) { return (u64)kb[i] << 32 | ka[i]; };
            std::stable_sort(idx.begin(), idx.end(), [&](u32 x, u32 y) { return K(x) < K(y); });
            for (u32 i = 0; i < n; ++i)
                if (pp[lo + i] != idx[i] || ra[lo + i] != ka[idx[i]] || rb[lo + i] != kb[idx[i]]) ++bad;
        }
        printf("%-28s check: %s (%llu mismatches)\n", name, bad ? "FAIL" : "ok", (unsigned long long)bad);
    };
    timeit("sweepg DB=10 NW=8 SPW=8", [&] { k_sweepg<10, 8, 8><<<nb, 512>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweepg DB=10 NW=8 SPW=8", A2, B2, P2);  // 6 passes: ends in set 2
    timeit("sweepg DB=10 NW=4 SPW=16", [&] { k_sweepg<10, 4, 16><<<nb, 256>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweepg DB=10 NW=4 SPW=16", A2, B2, P2);
    timeit("sweepg DB=8 NW=8 SPW=8", [&] { k_sweepg<8, 8, 8><<<nb, 512>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweepg DB=8 NW=8 SPW=8", A2, B2, P2);  // 8 passes
    timeit("sweep NW=8 SPW=8", [&] { k_sweep<8, 8><<<nb, 512>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweep NW=8 SPW=8", A2, B2, P2);
    timeit("sweep NW=16 SPW=4", [&] { k_sweep<16, 4><<<nb, 1024>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweep NW=16 SPW=4", A2, B2, P2);
    timeit("sweep NW=8 SPW=4", [&] { k_sweep<8, 4><<<nb, 512>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweep NW=8 SPW=4", A2, B2, P2);
    timeit("sweep NW=4 SPW=8", [&] { k_sweep<4, 8><<<nb, 256>>>(N, KA, KB, A1, B1, P1, A2, B2, P2); });
    check("sweep NW=4 SPW=8", A2, B2, P2);
    return 0;
}
