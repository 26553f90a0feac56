// Move-to-front over each block (replaces PY:460-468 mtf_encode, CPP:1159-1176).
//
// MTF is a sequential recency list.  The list state after a chunk of input is
//     (distinct symbols of the chunk, most recent first) ++ (previous state minus them),
// so the state entering every chunk is obtained by composing chunk summaries:
//   1. k_mtf_summary : one thread per chunk scans it backwards -> its recency list;
//   2. k_mtf_cp1..3  : the summaries composed in three levels (ranges of chunks by a wave
//                      each, the ranges of a block chained by one workgroup, the ranges
//                      re-walked), writing the 256-byte state at the start of every chunk
//                      (lane l holds entries 4l..4l+3; stable compaction by ballot/popcount);
//   3. k_mtf_replay  : one thread per chunk replays MTF from its start state with the
//                      table in LDS (word-interleaved per thread -> no bank conflicts),
//                      zero-byte search 4 entries per compare.
#include "kolm_internal.h"

namespace kolm {

namespace {

struct ChunkGeom {
    Geom geo;
    u32 cpb;  // chunks per block
    u32 csz;  // bytes per chunk (mtf_chunk_bytes: MTF_CHUNK, smaller for batches of few blocks)
    __device__ inline bool range(u32 c, u32& lo, u32& hi) const {
        const u32 b = c / cpb;
        const u32 k = c - b * cpb;
        lo = geo.base(b) + k * csz;
        const u32 e = geo.end(b);
        hi = min(lo + csz, e);
        return lo < e;
    }
};

constexpr u32 MTF_SLAB = 64;  // bytes per thread and round of the whole-workgroup paths

__global__ __launch_bounds__(256) void k_mtf_summary(ChunkGeom cg, const u8* in, u8* summary,
                                                     u16* scnt, u32 nchunks) {
    __shared__ u32 sl[256 * MTF_SLAB / 4];
    __shared__ u32 slo[256];
    const u32 t = threadIdx.x;
    const u32 c = blockIdx.x * blockDim.x + t;
    u32 lo = 0, hi = 0;
    const bool valid = c < nchunks && cg.range(c, lo, hi);
    u16 cnt = 0;
    // whole-workgroup path (every chunk a full aligned 1 KiB): the chunks are read backwards
    // 64 bytes at a time through LDS slabs that the workgroup loads as whole 64-byte lines
    // (per-thread 16-byte loads 1 KiB apart over-fetched ~4x, PMC)
    if (__syncthreads_and(valid && hi - lo == cg.csz && (lo & 15) == 0)) {
        u32 seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        u8* out = summary + (u64)c * 256;
        slo[t] = lo;
        __syncthreads();
        for (u32 r = cg.csz; r > 0; r -= MTF_SLAB) {
#pragma unroll
            for (u32 q = 0; q < MTF_SLAB / 16; ++q) {
                const u32 m = q * 256 + t, owner = m >> 2, part = m & 3;
                reinterpret_cast<uint4*>(sl)[m] =
                    *reinterpret_cast<const uint4*>(in + slo[owner] + r - MTF_SLAB + 16 * part);
            }
            __syncthreads();
            const u32* slab = sl + t * (MTF_SLAB / 4);
#pragma unroll
            for (int q = MTF_SLAB / 4 - 1; q >= 0; --q) {
                const u32 wv = slab[q];
#pragma unroll
                for (int j = 3; j >= 0; --j) {
                    const u32 b = (wv >> (8 * j)) & 0xFF, w = b >> 5, bit = 1u << (b & 31);
                    u32 sw = 0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) sw = (k == (int)w) ? seen[k] : sw;
                    if (!(sw & bit)) {
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if (k == (int)w) seen[k] |= bit;
                        out[cnt++] = (u8)b;
                    }
                }
            }
            __syncthreads();
        }
        scnt[c] = cnt;
        return;
    }
    if (!valid) {
        if (c < nchunks) scnt[c] = 0;
        return;
    }
    {
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

// One wave applies a recency summary (cnt symbols, most recent first) to a 256-entry
// state held as 64 words in LDS: state' = summary ++ (state minus the summary's symbols),
// a stable compaction by ballot counts.  All 64 lanes of the wave call it together.
__device__ inline void mtf_apply(u32* st, u8* nst, u32* member, const u8* sm, u32 cnt) {
    const u32 lane = threadIdx.x & 63;
    if (lane < 8) member[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    u32 sv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u32 i = 4 * lane + j;
        sv[j] = i < cnt ? sm[i] : 0;
        if (i < cnt) atomicOr(&member[sv[j] >> 5], 1u << (sv[j] & 31));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const u32 word = st[lane];
    u32 keep = 0;
    u8 e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        e[j] = (word >> (8 * j)) & 0xFF;
        const bool in_sum = (member[e[j] >> 5] >> (e[j] & 31)) & 1u;
        keep |= (in_sum ? 0u : 1u) << j;
    }
    const u32 nk = __popc(keep);
    u32 pos = cnt + wave_incl_scan(nk, OpAddU(), 0u) - nk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u32 i = 4 * lane + j;
        if (i < cnt) nst[i] = (u8)sv[j];
        if ((keep >> j) & 1u) nst[pos++] = e[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    st[lane] = reinterpret_cast<const u32*>(nst)[lane];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}


// The same composition in three launches and three levels, so the
// dependent mtf_apply chain of a block is ~55 steps instead of 2 * 64 + 16 (one gradient BMP
// block: 1024 chunks of 1 KiB).  A block's chunks form CP_R ranges of CP_S-range groups:
//   k_mtf_cp1: a wave per range composes its chunk summaries from the identity;
//   k_mtf_cp2: a workgroup per block, a wave per group: composes its ranges' summaries into
//              the group's, wave 0 chains the group summaries, each wave re-walks its ranges
//              and writes every range's entry state;
//   k_mtf_cp3: a wave per range re-walks its chunks from its entry state, writing the state at
//              every chunk start.
constexpr u32 CP_W = 16;          // waves per workgroup of cp1 / cp3
constexpr u32 CP_G = 8;           // groups per block (waves of cp2)
constexpr u32 CP_S = 16;          // ranges per group
constexpr u32 CP_R = CP_G * CP_S;  // ranges per block

__device__ inline u32 mtf_ident(u32 lane) {
    return (4 * lane) | ((4 * lane + 1) << 8) | ((4 * lane + 2) << 16) | ((4 * lane + 3) << 24);
}

// a range's chunks [k0, k1) of block b
__device__ inline void cp_range(const ChunkGeom& cg, u32 b, u32 r, u32& k0, u32& k1) {
    const u32 nch = (cg.geo.end(b) - cg.geo.base(b) + cg.csz - 1) / cg.csz;
    const u32 per = (nch + CP_R - 1) / CP_R;
    k0 = min(r * per, nch);
    k1 = min(k0 + per, nch);
}

__global__ __launch_bounds__(64 * CP_W) void k_mtf_cp1(ChunkGeom cg, const u8* summary, const u16* scnt, u32* rst,
                                                      u32* rdist) {
    __shared__ u32 st[CP_W][64];
    __shared__ u8 nst[CP_W][256];
    __shared__ u32 member[CP_W][8];
    __shared__ u32 uni[CP_W][8];
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u32 gr = blockIdx.x * CP_W + w, b = gr / CP_R, r = gr - b * CP_R;
    if (b >= cg.geo.nb) return;  // whole waves (wave-level sync only)
    u32 k0, k1;
    cp_range(cg, b, r, k0, k1);
    st[w][lane] = mtf_ident(lane);
    if (lane < 8) uni[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (u32 k = k0; k < k1; ++k) {
        const u32 c = b * cg.cpb + k;
        const u8* sm = summary + (u64)c * 256;
        const u32 cnt = scnt[c];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 i = 4 * lane + j;
            if (i < cnt) atomicOr(&uni[w][sm[i] >> 5], 1u << (sm[i] & 31));
        }
        mtf_apply(st[w], nst[w], member[w], sm, cnt);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    rst[(u64)gr * 64 + lane] = st[w][lane];
    if (lane == 0) {
        u32 d = 0;
        for (int q = 0; q < 8; ++q) d += __popc(uni[w][q]);
        rdist[gr] = d;
    }
}

__global__ __launch_bounds__(64 * CP_G) void k_mtf_cp2(const u32* rst, const u32* rdist, u32* rentry) {
    __shared__ u32 st[CP_G][64];
    __shared__ u8 nst[CP_G][256];
    __shared__ u32 member[CP_G][8];
    __shared__ u32 uni[CP_G][8];
    __shared__ u8 gsum[CP_G][256];
    __shared__ u32 gentry[CP_G][64];
    __shared__ u32 gdist[CP_G];
    const u32 lane = threadIdx.x & 63, g = threadIdx.x >> 6, b = blockIdx.x;
    const u64 r0 = (u64)b * CP_R + g * CP_S;
    // (a) the group's summary: its ranges' summaries composed from the identity
    st[g][lane] = mtf_ident(lane);
    if (lane < 8) uni[g][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (u32 v = 0; v < CP_S; ++v) {
        const u8* sm = reinterpret_cast<const u8*>(rst + (r0 + v) * 64);
        const u32 cnt = rdist[r0 + v];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 i = 4 * lane + j;
            if (i < cnt) atomicOr(&uni[g][sm[i] >> 5], 1u << (sm[i] & 31));
        }
        mtf_apply(st[g], nst[g], member[g], sm, cnt);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    reinterpret_cast<u32*>(gsum[g])[lane] = st[g][lane];
    if (lane == 0) {
        u32 d = 0;
        for (int q = 0; q < 8; ++q) d += __popc(uni[g][q]);
        gdist[g] = d;
    }
    __syncthreads();
    // (b) wave 0 chains the group summaries: gentry[g] = state entering group g
    if (g == 0) {
        st[0][lane] = mtf_ident(lane);
        __builtin_amdgcn_wave_barrier();
        for (u32 v = 0; v < CP_G; ++v) {
            gentry[v][lane] = st[0][lane];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (v + 1 < CP_G) mtf_apply(st[0], nst[0], member[0], gsum[v], gdist[v]);
        }
    }
    __syncthreads();
    // (c) each group re-walks its ranges from its entry state
    st[g][lane] = gentry[g][lane];
    __builtin_amdgcn_wave_barrier();
    for (u32 v = 0; v < CP_S; ++v) {
        rentry[(r0 + v) * 64 + lane] = st[g][lane];
        mtf_apply(st[g], nst[g], member[g], reinterpret_cast<const u8*>(rst + (r0 + v) * 64), rdist[r0 + v]);
    }
}

__global__ __launch_bounds__(64 * CP_W) void k_mtf_cp3(ChunkGeom cg, const u8* summary, const u16* scnt,
                                                      const u32* rentry, u8* states) {
    __shared__ u32 st[CP_W][64];
    __shared__ u8 nst[CP_W][256];
    __shared__ u32 member[CP_W][8];
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u32 gr = blockIdx.x * CP_W + w, b = gr / CP_R, r = gr - b * CP_R;
    if (b >= cg.geo.nb) return;
    u32 k0, k1;
    cp_range(cg, b, r, k0, k1);
    st[w][lane] = rentry[(u64)gr * 64 + lane];
    __builtin_amdgcn_wave_barrier();
    for (u32 k = k0; k < k1; ++k) {
        const u32 c = b * cg.cpb + k;
        reinterpret_cast<u32*>(states + (u64)c * 256)[lane] = st[w][lane];
        mtf_apply(st[w], nst[w], member[w], summary + (u64)c * 256, scnt[c]);
    }
}

constexpr int RT = 128;  // threads per workgroup in the replay kernel

// Rice-k bit lengths of the 5 BBWT candidates (PY:2028-2073: flags 0, bit-plane, nibble,
// bit reverse, Gray) accumulated while the MTF indices are produced (counter order of
// k_entropy.hip: 0 plain, 1 bit-plane, 2 nibble, 3 bit reverse, 4 Gray).
// Four bytes at a time (SWAR): the per-byte maps act on a whole word, v >> k on every byte
// is one shift and mask, and V_SAD_U8 sums the four bytes into the counter.
struct RiceAcc {
    u32 c[5] = {0, 0, 0, 0, 0};
    int k;
    u32 kk = 0, km = 0;  // shift and per-byte mask of v >> k (k >= 8: every byte shifts to 0)
    __device__ inline void init(int rk) {
        k = rk;
        kk = rk < 8 ? (u32)rk : 0u;
        km = rk < 8 ? (0xFFu >> rk) * 0x01010101u : 0u;
    }
    __device__ inline u32 rb(u32 v) const { return (v >> k) + 1 + k; }
    // sum over the 4 bytes x of x >> k, added to a
    __device__ inline u32 sum4(u32 w, u32 a) const { return __builtin_amdgcn_sad_u8((w >> kk) & km, 0u, a); }
    __device__ inline void add(u32 v) {
        c[0] += rb(v);
        c[2] += rb(((v & 0x0Fu) << 4) | (v >> 4));
        c[3] += rb(__brev(v) >> 24);
        c[4] += rb(v ^ (v >> 1));
    }
    // add() of the four bytes of o
    __device__ inline void add4(u32 o) {
        const u32 one = 4 * (1 + k);
        c[0] = sum4(o, c[0] + one);
        c[2] = sum4(((o & 0x0F0F0F0Fu) << 4) | ((o >> 4) & 0x0F0F0F0Fu), c[2] + one);  // nibble swap
        c[3] = sum4(__brev(o), c[3] + one);  // byte order reversed too: the sum does not see it
        c[4] = sum4(o ^ ((o >> 1) & 0x7F7F7F7Fu), c[4] + one);  // Gray
    }
    // one 8-byte bit-plane group (PY:1100-1120), bytes little-endian in lo / hi: plane b's
    // value has byte i's bit b at bit 7 - i.  With the bytes reversed (byte 7 - i at i) that is
    // the 8x8 bit-matrix transpose (byte r, bit c) -> (byte c, bit r), three delta swaps; the
    // order of the 8 plane values does not matter to the sum
    __device__ inline void group(u32 lo, u32 hi) {
        u64 x = ((u64)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
        u64 t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
        x ^= t ^ (t << 7);
        t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
        x ^= t ^ (t << 14);
        t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
        x ^= t ^ (t << 28);
        c[1] = sum4((u32)(x >> 32), sum4((u32)x, c[1] + 8 * (1 + k)));
    }
};

__global__ __launch_bounds__(RT) void k_mtf_replay(ChunkGeom cg, const u8* in, const u8* states, u8* out,
                                                   u32 nchunks, u64* bits, int rice_k) {
    __shared__ u32 tab[64 * RT];  // word w of thread t at tab[w * RT + t]
    const u32 t = threadIdx.x;
    const u32 c = blockIdx.x * RT + t;
    u32 lo = 0, hi = 0;
    const bool valid = c < nchunks && cg.range(c, lo, hi);  // (no early return: barriers below)
    // entries 0..7 (words 0, 1) live in registers: BBWT output is mostly short MTF indices,
    // which then cost no LDS round trip; words 2..63 stay in LDS
    u32 r0 = 0, r1 = 0;
    if (valid) {
        const u32* s = reinterpret_cast<const u32*>(states + (u64)c * 256);
        r0 = s[0];
        r1 = s[1];
        for (int w = 2; w < 64; ++w) tab[w * RT + t] = s[w];
    }
    auto haszero = [](u32 y) { return (y - 0x01010101u) & ~y & 0x80808080u; };
    // word x with its byte j moved to byte 0's side: bytes [0, j) shift up, byte 0 = in
    auto front = [](u32 x, u32 j, u32 in) {
        const u32 lowmask = j ? ((1u << (8 * j)) - 1) : 0u;
        const u32 highmask = j == 3 ? 0u : ~((1u << (8 * (j + 1))) - 1);
        return (x & highmask) | ((x & lowmask) << 8) | in;
    };
    auto step = [&](u32 b) -> u32 {
        const u32 bb = b * 0x01010101u;
        u32 z = haszero(r0 ^ bb);
        if (z) {
            const u32 j = (__ffs(z) - 1) >> 3;
            r0 = front(r0, j, b);
            return j;
        }
        const u32 c0 = r0 >> 24;
        z = haszero(r1 ^ bb);
        if (z) {
            const u32 j = (__ffs(z) - 1) >> 3;
            r0 = (r0 << 8) | b;
            r1 = front(r1, j, c0);
            return 4 + j;
        }
        u32 w = 2, x;
        for (;;) {
            x = tab[w * RT + t];
            z = haszero(x ^ bb);
            if (z) break;
            ++w;
        }
        const u32 j = (__ffs(z) - 1) >> 3;  // byte index inside word w
        // move to front: shift entries [0, 4w+j) up by one, entry 0 = b
        u32 carry = r1 >> 24;
        r1 = (r1 << 8) | c0;
        r0 = (r0 << 8) | b;
        for (u32 v = 2; v < w; ++v) {
            const u32 xv = tab[v * RT + t];
            tab[v * RT + t] = (xv << 8) | carry;
            carry = xv >> 24;
        }
        tab[w * RT + t] = front(x, j, carry);
        return 4 * w + j;
    };
    RiceAcc acc;
    acc.init(rice_k);
    if (!valid) return;
    if (((lo | hi) & 63) == 0) {
        // 64 bytes in / 64 bytes out per step as four back-to-back 16-byte accesses, so a
        // line is completed by consecutive instructions (threads are 1 KiB apart: one 16-byte
        // store per step left the lines' quarters to be merged across many steps — PMC:
        // ~4x the output bytes written); chunk starts are multiples of 1 KiB from the block
        // start, so 8-byte groups align
        for (u32 i = lo; i < hi; i += 64) {
            uint4 v[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) v[h] = *reinterpret_cast<const uint4*>(in + i + 16 * h);
            u32 ov[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const u32 wq = q % 4 == 0 ? v[q / 4].x : q % 4 == 1 ? v[q / 4].y : q % 4 == 2 ? v[q / 4].z : v[q / 4].w;
                u32 o = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) o |= step((wq >> (8 * j)) & 0xFF) << (8 * j);
                ov[q] = o;
                if (bits) acc.add4(o);
                if (bits && (q & 1)) acc.group(ov[q - 1], o);
            }
#pragma unroll
            for (int h = 0; h < 4; ++h)
                *reinterpret_cast<uint4*>(out + i + 16 * h) = make_uint4(ov[4 * h], ov[4 * h + 1], ov[4 * h + 2], ov[4 * h + 3]);
        }
    } else if (((lo | hi) & 15) == 0) {
        // 16 bytes in / 16 bytes out per global access
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
                if (bits) acc.add4(o);
            }
            *reinterpret_cast<uint4*>(out + i) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
            if (bits) {
                acc.group(ov[0], ov[1]);
                acc.group(ov[2], ov[3]);
            }
        }
    } else {
        u32 g[2] = {0, 0}, gi = 0;
        for (u32 i = lo; i < hi; ++i) {
            const u32 m = step(in[i]);
            out[i] = (u8)m;
            if (bits) {
                acc.add(m);
                g[gi >> 2] |= m << (8 * (gi & 3));
                if (++gi == 8) {
                    acc.group(g[0], g[1]);
                    g[0] = g[1] = 0;
                    gi = 0;
                }
            }
        }
        if (bits && gi) acc.group(g[0], g[1]);  // zero-padded last group of the block
    }
    if (bits) {
        u64* dst = bits + (u64)(c / cg.cpb) * 8;
#pragma unroll
        for (int q = 0; q < 5; ++q)
            if (acc.c[q]) atomicAdd((unsigned long long*)&dst[q], (unsigned long long)acc.c[q]);
    }
}

// Position-parallel replay for batches of few blocks: one wave per chunk, 64 bytes per step
// with one lane per byte, from the chunk's entry state S (k_mtf_cp3).  With Seen = the
// distinct symbols of the chunk before byte i (most recent first), MTF's list before i is
// Seen ++ (S minus Seen), so byte i = s gets
//   * if s occurred before in the chunk (last at p): the number of distinct symbols in (p, i);
//   * else: |Seen| + pos_S(s) - #{u in Seen : pos_S(u) < pos_S(s)}.
// Per step the lanes of each distinct symbol are found with one ballot per symbol (the
// symbol's class mask E); two passes over the classes give p, the window counts, |Seen| and
// the rank term; the state then moves to the step's recency summary ++ the rest (mtf_apply).
// No lane walks the list, so deep indices (images, audio: the gradient BMP's BBWT has most
// indices past 8) cost the same as shallow ones, and a 1 MiB block runs on 1024 waves
// instead of 8192 sequential 128-byte walks.
__global__ __launch_bounds__(256) void k_mtf_wave(ChunkGeom cg, const u8* in, const u8* states, u8* out,
                                                  u32 nchunks, u64* bits, int rice_k) {
    __shared__ u32 st[4][64];
    __shared__ u8 nst[4][256];
    __shared__ u32 member[4][8];
    __shared__ u8 inv[4][256];  // position of each symbol in the current state
    __shared__ u8 smy[4][64];   // the step's recency summary
    __shared__ __align__(8) u8 mb[4][64];  // the step's output bytes (bit-plane groups)
    const u32 w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const u32 c = blockIdx.x * 4 + w;
    u32 lo = 0, hi = 0;
    if (!(c < nchunks && cg.range(c, lo, hi))) return;  // whole waves (wave-level sync only)
    {
        const u32 word = reinterpret_cast<const u32*>(states + (u64)c * 256)[lane];
        st[w][lane] = word;
#pragma unroll
        for (int j = 0; j < 4; ++j) inv[w][(word >> (8 * j)) & 0xFF] = (u8)(4 * lane + j);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    RiceAcc acc;
    acc.init(rice_k);
    const u64 below = (1ull << lane) - 1ull;  // lanes before this one
    for (u32 p = lo; p < hi; p += 64) {
        const u32 i = p + lane;
        const bool v = i < hi;
        const u32 sym = v ? in[i] : 0u;
        const u64 vm = __ballot(v);
        const u32 mypos = inv[w][sym];
        // pass 1: this lane's class (lanes holding the same symbol)
        u64 rem = vm, mine = 0;
        while (rem) {
            const u32 k = (u32)__ffsll((long long)rem) - 1;
            const u32 sk = __builtin_amdgcn_readlane(sym, k);
            const u64 eq = __ballot(v && sym == sk);
            if (sym == sk) mine = eq;
            rem &= ~eq;
        }
        const u64 pm = mine & below;  // earlier lanes with my symbol
        const u32 prev = pm ? 63u - (u32)__clzll((long long)pm) : 0u;
        const u64 win = pm ? below & ~((2ull << prev) - 1ull) : 0ull;  // lanes in (prev, lane)
        // pass 2: distinct symbols in the window / before this lane, and their state ranks
        u32 cnt = 0, seen = 0, less = 0;
        rem = vm;
        while (rem) {
            const u32 k = (u32)__ffsll((long long)rem) - 1;  // the class's first lane
            const u32 sk = __builtin_amdgcn_readlane(sym, k);
            const u32 pk = __builtin_amdgcn_readlane(mypos, k);
            const u64 eq = __ballot(v && sym == sk);
            cnt += (eq & win) ? 1u : 0u;
            if (k < lane) {
                ++seen;
                less += pk < mypos ? 1u : 0u;
            }
            rem &= ~eq;
        }
        const u32 m = pm ? cnt : seen + mypos - less;
        if (v) out[i] = (u8)m;
        mb[w][lane] = v ? (u8)m : (u8)0;
        if (bits && v) acc.add(m);
        // recency summary of the step: last lanes of each symbol, most recent first
        const bool last = v && (mine >> lane) == 1ull;
        const u64 lm = __ballot(last);
        if (last) smy[w][__popcll(lm >> lane) - 1] = (u8)sym;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (bits && (lane & 7) == 0 && v) {
            const u32* g = reinterpret_cast<const u32*>(&mb[w][lane]);
            acc.group(g[0], g[1]);  // (a short last group reads the zeroed lanes)
        }
        mtf_apply(st[w], nst[w], member[w], smy[w], (u32)__popcll(lm));
        const u32 word = st[w][lane];
#pragma unroll
        for (int j = 0; j < 4; ++j) inv[w][(word >> (8 * j)) & 0xFF] = (u8)(4 * lane + j);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (bits) {
        u64* dst = bits + (u64)(c / cg.cpb) * 8;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const u32 sum = wave_reduce(acc.c[q], OpAddU(), 0u);
            if (lane == 0 && sum) atomicAdd((unsigned long long*)&dst[q], (unsigned long long)sum);
        }
    }
}

}  // namespace

// The position-parallel replay (k_mtf_wave, 1 KiB chunks) for batches of few blocks;
// KOLM_MTF_WAVE = 0 / 1 forces it off / on (read per call).
bool mtf_wave_mode(const Geom& geo) {
    const char* e = getenv("KOLM_MTF_WAVE");
    const int force = e ? atoi(e) : -1;
    return force >= 0 ? force != 0 : geo.nb < 64;
}

// Bytes per MTF chunk: MTF_CHUNK when the batch has chunks enough to fill the GPU; for
// batches of few blocks (BASELINE configs 2 and 5: 1 and 3 blocks) smaller chunks, down to
// 128 bytes, so the replay — one thread per chunk, a sequential walk — runs on up to 8x more
// threads (the compose then folds as many more summaries per block, in 8 waves: 32 blocks
// at 512 B measured compose 0.35 -> 0.70 ms for replay 0.48 -> 0.44 ms, so the halving
// stops at 16 K chunks; one gradient block at 128 B: 8.5 -> 6.0 ms per call).
u32 mtf_chunk_bytes(const Geom& geo) {
    static const u32 force = getenv("KOLM_MTF_CHUNK") ? (u32)atoi(getenv("KOLM_MTF_CHUNK")) : 0u;
    if (force >= 64 && force <= MTF_CHUNK && (force & (force - 1)) == 0) return force;
    u32 csz = MTF_CHUNK;
    if (mtf_wave_mode(geo)) return csz;
    while (csz > 128 && (u64)((geo.bs + csz - 1) / csz) * geo.nb < 16384) csz >>= 1;
    return csz;
}

// The three-launch compose (k_mtf_cp1..3) for every batch (one A/B call: config 2 1.90 -> 1.75
// ms, config 5 6.23 -> 6.09 ms, 256 MiB text MTF family 1.91 -> 1.76 ms against the round-4
// compose, one workgroup per block)
u64 mtf_cp_words(const Geom& geo) { return (u64)geo.nb * CP_R * 129; }

void launch_mtf(const Geom& geo, const u8* in, u8* out, u8* summary, u16* summary_cnt, u8* states,
                hipStream_t s, KTimer* kt, u64* bits, int rice_k, u32* cp_scratch) {
    if (!geo.N) return;
    const u32 csz = mtf_chunk_bytes(geo);
    ChunkGeom cg{geo, (geo.bs + csz - 1) / csz, csz};
    const u32 nchunks = cg.cpb * geo.nb;
    const u64 N = geo.N;
    {
        KScope k(kt, KT_MTF, "k_mtf_summary", N + (u64)nchunks * 256);
        k_mtf_summary<<<(nchunks + 255) / 256, 256, 0, s>>>(cg, in, summary, summary_cnt, nchunks);
    }
    {
        KScope k(kt, KT_MTF, "k_mtf_compose", (u64)nchunks * 512);
        {
            u32* rst = cp_scratch;                           // [nb * CP_R][64]
            u32* rentry = cp_scratch + (u64)geo.nb * CP_R * 64;  // [nb * CP_R][64]
            u32* rdist = rentry + (u64)geo.nb * CP_R * 64;        // [nb * CP_R]
            const u32 g13 = (geo.nb * CP_R + CP_W - 1) / CP_W;
            k_mtf_cp1<<<g13, 64 * CP_W, 0, s>>>(cg, summary, summary_cnt, rst, rdist);
            k_mtf_cp2<<<geo.nb, 64 * CP_G, 0, s>>>(rst, rdist, rentry);
            k_mtf_cp3<<<g13, 64 * CP_W, 0, s>>>(cg, summary, summary_cnt, rentry, states);
        }
    }
    if (mtf_wave_mode(geo)) {
        KScope k(kt, KT_MTF, "k_mtf_wave", 2 * N + (u64)nchunks * 256);
        k_mtf_wave<<<(nchunks + 3) / 4, 256, 0, s>>>(cg, in, states, out, nchunks, bits, rice_k);
    } else {
        KScope k(kt, KT_MTF, "k_mtf_replay", 2 * N + (u64)nchunks * 256);
        k_mtf_replay<<<(nchunks + RT - 1) / RT, RT, 0, s>>>(cg, in, states, out, nchunks, bits, rice_k);
    }
}

}  // namespace kolm
