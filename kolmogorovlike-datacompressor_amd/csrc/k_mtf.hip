// Move-to-front over each block (replaces PY:460-468 mtf_encode, CPP:1159-1176).
//
// MTF is a sequential recency list.  The list state after a chunk of input is
//     (distinct symbols of the chunk, most recent first) ++ (previous state minus them),
// so the state entering every chunk is obtained by composing chunk summaries:
//   1. k_mtf_summary : one thread per chunk scans it backwards -> its recency list;
//   2. k_mtf_compose : one wave per block folds the summaries in order, writing the
//                      256-byte state at the start of every chunk (lane l holds entries
//                      4l..4l+3; stable compaction by ballot/popcount);
//   3. k_mtf_replay  : one thread per chunk replays MTF from its start state with the
//                      table in LDS (word-interleaved per thread -> no bank conflicts),
//                      zero-byte search 4 entries per compare.
#include "kolm_internal.h"

namespace kolm {

namespace {

struct ChunkGeom {
    Geom geo;
    u32 cpb;  // chunks per block
    __device__ inline bool range(u32 c, u32& lo, u32& hi) const {
        const u32 b = c / cpb;
        const u32 k = c - b * cpb;
        lo = geo.base(b) + k * MTF_CHUNK;
        const u32 e = geo.end(b);
        hi = min(lo + (u32)MTF_CHUNK, e);
        return lo < e;
    }
};

__global__ __launch_bounds__(256) void k_mtf_summary(ChunkGeom cg, const u8* in, u8* summary,
                                                     u16* scnt, u32 nchunks) {
    const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    u32 lo, hi;
    u16 cnt = 0;
    if (cg.range(c, lo, hi)) {
        u32 seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        u8* out = summary + (u64)c * 256;
        auto visit = [&](u32 b) {
            const u32 w = b >> 5, bit = 1u << (b & 31);
            u32 sw = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) sw = (k == (int)w) ? seen[k] : sw;
            if (!(sw & bit)) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k == (int)w) seen[k] |= bit;
                out[cnt++] = (u8)b;
            }
        };
        if (((lo | hi) & 15) == 0) {
            // 16-byte loads (threads are 1 KiB apart: byte loads thrash L1)
            for (u32 i = hi; i > lo; i -= 16) {
                const uint4 v = *reinterpret_cast<const uint4*>(in + i - 16);
                const u32 wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int q = 3; q >= 0; --q)
#pragma unroll
                    for (int j = 3; j >= 0; --j) visit((wv[q] >> (8 * j)) & 0xFF);
            }
        } else {
            for (u32 i = hi; i > lo; --i) visit(in[i - 1]);
        }
    }
    scnt[c] = cnt;
}

// one wave (64 threads) per block
__global__ __launch_bounds__(64) void k_mtf_compose(ChunkGeom cg, const u8* summary, const u16* scnt,
                                                    u8* states) {
    __shared__ u32 st[64];      // current state, 256 bytes
    __shared__ u8 nst[256];     // next state
    __shared__ u32 member[8];
    const u32 b = blockIdx.x, lane = threadIdx.x;
    st[lane] = (4 * lane) | ((4 * lane + 1) << 8) | ((4 * lane + 2) << 16) | ((4 * lane + 3) << 24);
    __syncthreads();
    const u64 lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (u32 k = 0; k < cg.cpb; ++k) {
        const u32 c = b * cg.cpb + k;
        u32 lo, hi;
        if (!cg.range(c, lo, hi)) break;
        // publish the state at chunk start
        reinterpret_cast<u32*>(states + (u64)c * 256)[lane] = st[lane];
        const u32 cnt = scnt[c];
        if (lane < 8) member[lane] = 0;
        __syncthreads();
        const u8* sm = summary + (u64)c * 256;
        u32 sv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 i = 4 * lane + j;
            sv[j] = i < cnt ? sm[i] : 0;
            if (i < cnt) atomicOr(&member[sv[j] >> 5], 1u << (sv[j] & 31));
        }
        __syncthreads();
        const u32 word = st[lane];
        u32 keep = 0;
        u8 e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            e[j] = (word >> (8 * j)) & 0xFF;
            const bool in_sum = (member[e[j] >> 5] >> (e[j] & 31)) & 1u;
            keep |= (in_sum ? 0u : 1u) << j;
        }
        // stable compaction: rank = kept entries before this lane + within lane
        const u32 nk = __popc(keep);
        // wave exclusive prefix of nk
        u32 incl = nk;
        for (u32 o = 1; o < 64; o <<= 1) {
            const u32 t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        u32 pos = cnt + incl - nk;
        (void)lt_mask;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 i = 4 * lane + j;
            if (i < cnt) nst[i] = (u8)sv[j];
            if ((keep >> j) & 1u) nst[pos++] = e[j];
        }
        __syncthreads();
        st[lane] = reinterpret_cast<const u32*>(nst)[lane];
        __syncthreads();
    }
}

constexpr int RT = 128;  // threads per workgroup in the replay kernel

__global__ __launch_bounds__(RT) void k_mtf_replay(ChunkGeom cg, const u8* in, const u8* states, u8* out,
                                                   u32 nchunks) {
    __shared__ u32 tab[64 * RT];  // word w of thread t at tab[w * RT + t]
    const u32 t = threadIdx.x;
    const u32 c = blockIdx.x * RT + t;
    if (c >= nchunks) return;
    u32 lo, hi;
    if (!cg.range(c, lo, hi)) return;
    const u32* s = reinterpret_cast<const u32*>(states + (u64)c * 256);
    for (int w = 0; w < 64; ++w) tab[w * RT + t] = s[w];
    auto step = [&](u32 b) -> u32 {
        const u32 bb = b * 0x01010101u;
        u32 w = 0, x, z;
        for (;;) {
            x = tab[w * RT + t];
            const u32 y = x ^ bb;
            z = (y - 0x01010101u) & ~y & 0x80808080u;
            if (z) break;
            ++w;
        }
        const u32 j = (__ffs(z) - 1) >> 3;  // byte index inside word w
        // move to front: shift entries [0, 4w+j) up by one, entry 0 = b
        u32 carry = b;
        for (u32 v = 0; v < w; ++v) {
            const u32 xv = tab[v * RT + t];
            tab[v * RT + t] = (xv << 8) | carry;
            carry = xv >> 24;
        }
        const u32 lowmask = j ? ((1u << (8 * j)) - 1) : 0u;
        const u32 highmask = j == 3 ? 0u : ~((1u << (8 * (j + 1))) - 1);
        tab[w * RT + t] = (x & highmask) | ((x & lowmask) << 8) | carry;
        return 4 * w + j;
    };
    if (((lo | hi) & 15) == 0) {
        // 16 bytes in / 16 bytes out per global access (threads are 1 KiB apart)
        for (u32 i = lo; i < hi; i += 16) {
            const uint4 v = *reinterpret_cast<const uint4*>(in + i);
            const u32 wv[4] = {v.x, v.y, v.z, v.w};
            u32 ov[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                u32 o = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) o |= step((wv[q] >> (8 * j)) & 0xFF) << (8 * j);
                ov[q] = o;
            }
            *reinterpret_cast<uint4*>(out + i) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
        }
    } else {
        for (u32 i = lo; i < hi; ++i) out[i] = (u8)step(in[i]);
    }
}

}  // namespace

void launch_mtf(const Geom& geo, const u8* in, u8* out, u8* summary, u16* summary_cnt, u8* states,
                hipStream_t s, KTimer* kt) {
    if (!geo.N) return;
    ChunkGeom cg{geo, (geo.bs + MTF_CHUNK - 1) / MTF_CHUNK};
    const u32 nchunks = cg.cpb * geo.nb;
    const u64 N = geo.N;
    {
        KScope k(kt, KT_MTF, "k_mtf_summary", N + (u64)nchunks * 256);
        k_mtf_summary<<<(nchunks + 255) / 256, 256, 0, s>>>(cg, in, summary, summary_cnt, nchunks);
    }
    {
        KScope k(kt, KT_MTF, "k_mtf_compose", (u64)nchunks * 512);
        k_mtf_compose<<<geo.nb, 64, 0, s>>>(cg, summary, summary_cnt, states);
    }
    {
        KScope k(kt, KT_MTF, "k_mtf_replay", 2 * N + (u64)nchunks * 256);
        k_mtf_replay<<<(nchunks + RT - 1) / RT, RT, 0, s>>>(cg, in, states, out, nchunks);
    }
}

}  // namespace kolm
