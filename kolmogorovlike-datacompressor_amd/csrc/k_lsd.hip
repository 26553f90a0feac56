// Round 0 of the cyclic suffix sort (gfx950): every block's positions stably sorted by the
// first 4 characters of their rotation (4 LSD passes of 8 bits, 4096-element tiles:
// per-wave LDS histograms -> per-block scan over (digit, tile) -> stable scatter with wave
// ballot ranking), then group starts, ranks and the next round's segments (k_sort.hip).
// No host synchronisation: a fixed sequence of launches on the sort stream.
#include "kolm_internal.h"

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

namespace kolm {

namespace {

#ifndef KOLM_LSD_T
#define KOLM_LSD_T 4096
#endif
constexpr u32 LSD_T = KOLM_LSD_T;    // elements per tile
constexpr u32 LSD_PT = LSD_T / WG;   // 16 per thread
static_assert(LSD_PT % 4 == 0 && LSD_PT <= 32, "head masks hold 32 slots per thread");

struct LsdGeom {
    Geom geo;
    u32 tpb;  // tiles per block
    const u8* text;
    const u8* FEd;    // min(distance to the factor end, 255)
    Factors fac;      // Lyndon factor starts per block
    __device__ inline bool range(u32 t, u32& lo, u32& hi, u32& b) const {
        b = t / tpb;
        const u32 k = t - b * tpb;
        lo = geo.base(b) + k * LSD_T;
        const u32 e = geo.end(b);
        hi = min(lo + LSD_T, e);
        return lo < e;
    }
};

template <int P>
__device__ inline u32 digit(u32 key) {
    return (key >> (8 * P)) & 255u;
}

// the thread's 16 consecutive words X[i0 .. i0+15] (0 past hi): four 16-byte loads when
// aligned and whole (the 16 scalar loads per array were 48 read instructions per wave)
__device__ inline void load16(const u32* X, u32 i0, u32 hi, u32 (&v)[LSD_PT]) {
    if ((i0 & 3) == 0 && i0 + LSD_PT <= hi) {
        const uint4* p = reinterpret_cast<const uint4*>(X + i0);
#pragma unroll
        for (int q = 0; q < (int)LSD_PT / 4; ++q) {
            const uint4 t = p[q];
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (u32 e = 0; e < LSD_PT; ++e) v[e] = i0 + e < hi ? X[i0 + e] : 0u;
    }
}

// the same with non-temporal loads (streamed through, not kept in L2)
__device__ inline void load16nt(const u32* X, u32 i0, u32 hi, u32 (&v)[LSD_PT]) {
    if ((i0 & 3) == 0 && i0 + LSD_PT <= hi) {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* p = reinterpret_cast<const u32x4*>(X + i0);
#pragma unroll
        for (int q = 0; q < (int)LSD_PT / 4; ++q) {
            const u32x4 t = __builtin_nontemporal_load(p + q);
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (u32 e = 0; e < LSD_PT; ++e) v[e] = i0 + e < hi ? __builtin_nontemporal_load(X + i0 + e) : 0u;
    }
}

// where a pass reads its (key, position) pairs: keys by position (first pass) or pairs
// SRC_PK: one packed word per element, (digit 3 of the key) << 24 | position - block base (the
// first half's last pass reads what its previous pass wrote that way: 8 bytes less per element)
// SRC_REC: (key, position) as one u64 record per element (key in the low word)
enum Src { SRC_KP = 1, SRC_PAIR = 2, SRC_PK = 3, SRC_REC = 4 };
// what a pass writes: (key, position) pairs in two arrays, the packed word, or u64 records (one
// 8-byte store per element: half the write transactions of the two arrays' 4-byte stores,
// which a probe measured 1.5-1.8x faster on LSD run patterns, tools/scatter_probe.hip)
enum Out { OUT_PAIR = 0, OUT_PK = 1, OUT_REC = 2 };

// Per-(block, part) digit totals for k_lsd_scan2: a block's tiles form parts of 2^plt tiles.
struct ScanParts {
    u32* cur = nullptr;    // [nb * np * 256] this pass's totals (accumulated by the histogram)
    u32* other = nullptr;  // the other buffer: k_lsd_scan2 zeroes it for the pass after next
    u32 np = 0, plt = 0;
};
__device__ inline void add_part_total(const LsdGeom& g, const ScanParts& sp, u32 t, u32 v) {
    if (sp.cur && v) {
        const u32 b = t / g.tpb, k = t - b * g.tpb;
        atomicAdd(&sp.cur[((u64)b * sp.np + (k >> sp.plt)) * 256 + threadIdx.x], v);
    }
}

// Tile digit counts in LDS: 16 copies (4 per wave, by lane & 3) of 256 16-bit counters, two per
// dword.  The packed codes of text give a tile few distinct digit values, and one wave's
// same-address LDS atomics serialise: with one copy per wave, 60 % of the keys on one digit value
// ran a 1 GiB pass at 1.95 TB/s against 5.5 TB/s for spread digits (tools/bw_probe.hip); with 16
// copies, 4.6 TB/s.
struct TileCounts {
    u32 c[16][128];
    __device__ inline void clear() {
        for (u32 i = threadIdx.x; i < 16 * 128; i += WG) (&c[0][0])[i] = 0;
    }
    __device__ inline void add(u32 d) {
        atomicAdd(&c[((threadIdx.x >> 6) << 2) | (threadIdx.x & 3)][d >> 1], 1u << (16 * (d & 1)));
    }
    __device__ inline u32 total(u32 d) const {  // after a barrier
        u32 v = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) v += (c[i][d >> 1] >> (16 * (d & 1))) & 0xFFFFu;
        return v;
    }
};

template <int P, int SRC>
__global__ __launch_bounds__(WG) void k_lsd_hist(LsdGeom g, const u32* K, u32* hist, ScanParts sp) {
    __shared__ TileCounts h;
    const u32 tid = threadIdx.x;
    h.clear();
    __syncthreads();
    u32 lo, hi, b;
    if (g.range(xcd_tile(), lo, hi, b)) {
        const u32 i0 = lo + tid * LSD_PT;
        if (SRC == SRC_REC) {  // keys in the low words of the records
            if ((lo & 1) == 0 && hi - lo == LSD_T) {
                const uint4* p = reinterpret_cast<const uint4*>(K + 2 * (u64)lo);
                uint4 v[LSD_PT / 2];
#pragma unroll
                for (u32 q = 0; q < LSD_PT / 2; ++q) v[q] = p[q * WG + tid];
#pragma unroll
                for (u32 q = 0; q < LSD_PT / 2; ++q) {
                    h.add(digit<P>(v[q].x));
                    h.add(digit<P>(v[q].z));
                }
            } else {
                for (u32 i = i0; i < min(i0 + LSD_PT, hi); ++i) h.add(digit<P>(K[2 * (u64)i]));
            }
        } else if ((lo & 3) == 0 && hi - lo == LSD_T) {
            // a whole aligned tile: four 16-byte loads per thread, lane-contiguous (a wave
            // reads 1 KiB per instruction; the order of the keys is irrelevant here).  The
            // per-thread-contiguous form (lanes 64 B apart) ran at ~2 TB/s.
            const uint4* p = reinterpret_cast<const uint4*>(K + lo);
            uint4 v[LSD_PT / 4];
#pragma unroll
            for (u32 q = 0; q < LSD_PT / 4; ++q) v[q] = p[q * WG + tid];
#pragma unroll
            for (u32 q = 0; q < LSD_PT / 4; ++q) {
                h.add(digit<P>(v[q].x));
                h.add(digit<P>(v[q].y));
                h.add(digit<P>(v[q].z));
                h.add(digit<P>(v[q].w));
            }
        } else {
            for (u32 i = i0; i < min(i0 + LSD_PT, hi); ++i) h.add(digit<P>(K[i]));
        }
    }
    __syncthreads();
    const u32 v = h.total(tid);
    hist[(u64)xcd_tile() * 256 + tid] = v;
    add_part_total(g, sp, xcd_tile(), v);
}

// hist[t][d] -> absolute destination of the first element of digit d in tile t, one
// workgroup per (block, part of 2^plt tiles): the block's digit totals and the earlier parts'
// counts come from the per-part totals, so the sequential chain is one part long.  Zeroes its
// entries of the other totals buffer (the pass after next accumulates there).
__global__ __launch_bounds__(WG) void k_lsd_scan2(LsdGeom g, u32* hist, ScanParts sp) {
    __shared__ u32 sh[WG / 64];
    const u32 b = blockIdx.x / sp.np, part = blockIdx.x - b * sp.np, d = threadIdx.x, lane = d & 63, w = d >> 6;
    u32 tot = 0, pre = 0;
    for (u32 q = 0; q < sp.np; ++q) {
        const u32 c = sp.cur[((u64)b * sp.np + q) * 256 + d];
        tot += c;
        pre += q < part ? c : 0u;
    }
    const u32 incl = wave_incl_scan(tot, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = 0;
    for (u32 i = 0; i < w; ++i) carry += sh[i];
    u32 run = g.geo.base(b) + carry + incl - tot + pre;
    const u64 t0 = (u64)b * g.tpb;
    const u32 k0 = part << sp.plt, k1 = min(g.tpb, (part + 1) << sp.plt);
    constexpr u32 B = 16;
    for (u32 k = k0; k < k1; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < k1 ? hist[(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j)
            if (k + j < k1) {
                hist[(t0 + k + j) * 256 + d] = run;
                run += v[j];
            }
    }
    sp.other[((u64)b * sp.np + part) * 256 + d] = 0;
}

// hist[t][d] -> absolute destination of the first element of digit d in tile t.
__global__ __launch_bounds__(WG) void k_lsd_scan(LsdGeom g, u32* hist) {
    __shared__ u32 sh[WG / 64];
    const u32 b = blockIdx.x, d = threadIdx.x, lane = d & 63, w = d >> 6;
    const u64 t0 = (u64)b * g.tpb;
    constexpr u32 B = 16;
    u32 acc = 0;
    for (u32 k = 0; k < g.tpb; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < g.tpb ? hist[(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j) {
            if (k + j < g.tpb) hist[(t0 + k + j) * 256 + d] = acc;
            acc += v[j];
        }
    }
    // exclusive scan of the digit totals
    const u32 incl = wave_incl_scan(acc, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = 0;
    for (u32 i = 0; i < w; ++i) carry += sh[i];
    const u32 base = g.geo.base(b) + carry + incl - acc;
    for (u32 k = 0; k < g.tpb; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < g.tpb ? hist[(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j)
            if (k + j < g.tpb) hist[(t0 + k + j) * 256 + d] = v[j] + base;
    }
}

// The same scan with NP threads per digit (NP * 256-thread workgroup), each over 1 / NP of
// the block's tiles: the per-digit dependent chains are 1 / NP as long (the scan is
// latency-bound: one workgroup per block, 256 tiles of loads per thread).
template <u32 NP>
__global__ __launch_bounds__(NP * WG) void k_lsd_scanp(LsdGeom g, u32* hist) {
    static_assert(NP == 2 || NP == 4, "2 or 4 parts");
    __shared__ u32 pt[NP][256];
    __shared__ u32 sh[4];
    const u32 b = blockIdx.x, d = threadIdx.x & 255, q = threadIdx.x >> 8;
    const u64 t0 = (u64)b * g.tpb;
    const u32 per = (g.tpb + NP - 1) / NP, k0 = min(g.tpb, q * per), k1 = min(g.tpb, k0 + per);
    constexpr u32 B = 16;
    u32 acc = 0;
    for (u32 k = k0; k < k1; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < k1 ? hist[(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j) acc += v[j];
    }
    pt[q][d] = acc;
    __syncthreads();
    // digit totals -> exclusive scan over the 256 digits (waves 0..3), then each part's start
    u32 tot = 0, incl = 0;
    if (q == 0) {
        for (u32 i = 0; i < NP; ++i) tot += pt[i][d];
        incl = wave_incl_scan(tot, OpAddU(), 0u);
        if ((d & 63) == 63) sh[d >> 6] = incl;
    }
    __syncthreads();
    if (q == 0) {
        u32 carry = 0;
        for (u32 i = 0; i < (d >> 6); ++i) carry += sh[i];
        u32 run = g.geo.base(b) + carry + incl - tot;
        for (u32 i = 0; i < NP; ++i) {
            const u32 c = pt[i][d];
            pt[i][d] = run;
            run += c;
        }
    }
    __syncthreads();
    u32 run = pt[q][d];
    for (u32 k = k0; k < k1; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < k1 ? hist[(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j)
            if (k + j < k1) {
                hist[(t0 + k + j) * 256 + d] = run;
                run += v[j];
            }
    }
}


// Stable scatter of one tile by digit P with three barriers per tile (round 2 replaced a form
// with three per 256 elements): wave w owns the contiguous quarter [lo + 1024 w, lo + 1024 (w + 1)) of the tile (64
// elements per step, 16 steps, all held in registers).  Pass 1: every element's offset
// among its wave's equal digits (ballot match; the digit's leader advances the wave's LDS
// counter — a wave's LDS operations retire in order, so no barrier between steps).  Then
// per digit the waves' counts become bases (tile base + counts of the lower waves), and
// pass 2 writes every element to base + offset; (wave, step, lane) is tile order, so the
// scatter is stable.  SRC_KP reads the keys by position (positions implicit).  G: the pass
// writes Kg[position] as the key (the next digit set, gathered by position) instead of the
// key it sorted by — the last pass of the 8-character sort's first half.
// OUT: OUT_PK writes the packed word (digit 3 << 24 | position - block base), OUT_REC u64
// records at Kout, OUT_PAIR (key, position) to Kout / Pout
template <int P, int SRC, int G, int OUT = OUT_PAIR>
__global__ __launch_bounds__(WG) void k_lsd_scatter_w(LsdGeom g, const u32* Kin, const u32* Pin, u32* Kout,
                                                     u32* Pout, const u32* Kg, const u32* hist) {
    static_assert(SRC != SRC_PK || P == 3, "packed words hold digit 3 only");
    static_assert(OUT != OUT_PK || P == 2, "a packed word carries the next digit, 3");
    // few registers on purpose (keys and positions, offsets in LDS): the pass runs beside
    // the LZ77 parse, which holds 4 waves per SIMD, and a 108-VGPR version of this kernel
    // was starved for the parse's whole duration (one pass 1.7 -> 11 ms)
    __shared__ u32 wc[WG / 64][256];
    __shared__ u16 loc[LSD_T];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32 lo, hi, b;
    const u32 t = xcd_tile();
    if (!g.range(t, lo, hi, b)) return;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) wc[i][tid] = 0;
    const u32 tb = hist[(u64)t * 256 + tid];
    u32 key[LSD_PT], pos[LSD_PT];
    const u32 q0 = lo + w * (LSD_T / 4);
#pragma unroll
    for (u32 j = 0; j < LSD_PT; ++j) {
        const u32 i = q0 + j * 64 + lane;
        key[j] = 0;
        pos[j] = 0;
        if (i < hi) {
            if (SRC == SRC_REC) {
                const u64 r = reinterpret_cast<const u64*>(Kin)[i];
                key[j] = (u32)r;
                pos[j] = (u32)(r >> 32);
            } else {
                key[j] = Kin[i];
                pos[j] = SRC == SRC_KP ? i : SRC == SRC_PK ? g.geo.base(b) + (key[j] & 0xFFFFFFu) : Pin[i];
            }
        }
    }
    // G: the next key gathered by position up front (its latency under the ranking; at
    // write time it measured 2.5 -> 3.4 ms per step)
    u32 kg[G ? LSD_PT : 1];
    if (G) {
#pragma unroll
        for (u32 j = 0; j < LSD_PT; ++j) kg[j] = q0 + j * 64 + lane < hi ? Kg[pos[j]] : 0u;
    }
    __syncthreads();
    const u64 lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    u16* lw = loc + w * (LSD_T / 4) + lane;
#pragma unroll
    for (u32 j = 0; j < LSD_PT; ++j) {
        const bool valid = q0 + j * 64 + lane < hi;
        const u32 dg = digit<P>(key[j]);
        u64 m = __ballot(valid);
#pragma unroll
        for (u32 bit = 0; bit < 8; ++bit) {
            const u64 bal = __ballot((dg >> bit) & 1u);
            m &= ((dg >> bit) & 1u) ? bal : ~bal;
        }
        const u32 rank = __popcll(m & lt_mask);
        const u32 pre = valid ? wc[w][dg] : 0u;
        lw[j * 64] = (u16)(pre + rank);
        if (valid && rank == 0) wc[w][dg] = pre + (u32)__popcll(m);
    }
    __syncthreads();
    {
        u32 acc = tb;
#pragma unroll
        for (int q = 0; q < WG / 64; ++q) {
            const u32 c = wc[q][tid];
            wc[q][tid] = acc;
            acc += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (u32 j = 0; j < LSD_PT; ++j) {
        if (q0 + j * 64 + lane < hi) {
            const u32 dst = wc[w][digit<P>(key[j])] + lw[j * 64];
            if (OUT == OUT_PK) {
                Kout[dst] = (key[j] & 0xFF000000u) | (pos[j] - g.geo.base(b));
            } else if (OUT == OUT_REC) {
                reinterpret_cast<u64*>(Kout)[dst] = ((u64)pos[j] << 32) | (G ? kg[G ? j : 0] : key[j]);
            } else {
                Kout[dst] = G ? kg[G ? j : 0] : key[j];
                Pout[dst] = pos[j];
            }
        }
    }
}

__device__ inline u32 wave_max(u32 v) { return wave_reduce(v, OpMaxU(), 0u); }

// per block: exclusive max over its tiles (one workgroup per block)
__global__ __launch_bounds__(WG) void k_tiles_max_scan(const u32* in, u32* out, u32 tpb) {
    __shared__ u32 sh[WG / 64];
    __shared__ u32 edge;
    const u32 b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 carry = 0;
    for (u32 c0 = 0; c0 < tpb; c0 += WG) {
        const u32 k = c0 + threadIdx.x;
        const u32 v = k < tpb ? in[(u64)b * tpb + k] : 0u;
        const u32 incl = wave_incl_scan(v, OpMaxU(), 0u);
        const u32 ex = KOLM_DPP(0u, incl, DPP_WAVE_SHR1, 0xF);
        if (lane == 63) sh[w] = incl;
        __syncthreads();
        u32 wc = carry;
        for (u32 i = 0; i < w; ++i) wc = max(wc, sh[i]);
        if (k < tpb) out[(u64)b * tpb + k] = max(wc, ex);
        if (threadIdx.x == WG - 1) edge = max(wc, incl);
        __syncthreads();
        carry = edge;
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------------
// Round 0 of the cyclic suffix sort: after 4 LSD passes over the 4-character rotation
// keys (K sorted, SA = positions), slot g starts a group iff g is the block's first slot
// or K[g] != K[g-1].  Every position gets RK = its group's first slot (PY's (fi, i) tie
// rule is position order, kept by the stable passes); groups of >= 2 go to the next
// round; a block with more than one group has split.
// ---------------------------------------------------------------------------------
constexpr u32 BIG = 0xFFFFFFFFu;
constexpr u32 R0_WS = 12;             // position windows of the RK write (k_r0_rk below)
constexpr u32 R0_WIN = 1u << R0_WS;

__device__ inline u32 wave_min(u32 v) { return wave_reduce(v, OpMinU(), BIG); }

// Group heads of every tile: bit e of HF[t * WG + tid] = slot lo + 16 tid + e starts a group
// (the block's first slot, or its key differs from the previous slot's; with KA — the
// 8-character round 0, K = characters 0..3 — also when characters 4..7, KA[SA[slot]],
// differ).  tmax / tmin = the tile's last / first head.
__global__ __launch_bounds__(WG) void k_r0_tile_heads(LsdGeom g, const u32* K, const u32* SA, const u32* KA, u32* HF,
                                                      u32* tmax, u32* tmin, u32* BH) {
    __shared__ u32 s1[WG / 64], s2[WG / 64];
    __shared__ u32 bh[WG / 64][256];  // BH: per wave, slots of this tile per position window
    const u32 t = xcd_tile();
    const u32 w = threadIdx.x >> 6;
    if (BH) {
#pragma unroll
        for (int i = 0; i < WG / 64; ++i) bh[i][threadIdx.x] = 0;
        __syncthreads();
    }
    u32 lo, hi, b;
    u32 mx = 0, mn = BIG;
    if (g.range(t, lo, hi, b)) {
        const u32 base = g.geo.base(b);
        const u32 i0 = lo + threadIdx.x * LSD_PT;
        u32 hm = 0;
        if (i0 < hi) {
            u32 kv[LSD_PT], av[LSD_PT];
            load16(K, i0, hi, kv);
            u32 kprev = i0 > base ? K[i0 - 1] : 0u, aprev = 0;
            u32 sv[LSD_PT];
            if (BH || KA) load16(SA, i0, hi, sv);
            if (BH) {
#pragma unroll
                for (u32 e = 0; e < LSD_PT; ++e)
                    if (i0 + e < hi) atomicAdd(&bh[w][(sv[e] - base) >> R0_WS], 1u);
            }
            if (KA) {
#pragma unroll
                for (u32 e = 0; e < LSD_PT; ++e) av[e] = i0 + e < hi ? KA[sv[e]] : 0u;
                aprev = i0 > base ? KA[SA[i0 - 1]] : 0u;
            } else {
#pragma unroll
                for (u32 e = 0; e < LSD_PT; ++e) av[e] = 0;
            }
#pragma unroll
            for (u32 e = 0; e < LSD_PT; ++e) {
                const u32 i = i0 + e;
                if (i < hi && (i == base || kv[e] != kprev || av[e] != aprev)) {
                    hm |= 1u << e;
                    mx = max(mx, i);
                    mn = min(mn, i);
                }
                kprev = kv[e];
                aprev = av[e];
            }
        }
        HF[(u64)t * WG + threadIdx.x] = hm;
    }
    if (BH) {
        __syncthreads();
        BH[(u64)t * 256 + threadIdx.x] = bh[0][threadIdx.x] + bh[1][threadIdx.x] + bh[2][threadIdx.x] + bh[3][threadIdx.x];
    }
    mx = wave_max(mx);
    mn = wave_min(mn);
    if ((threadIdx.x & 63) == 0) {
        s1[threadIdx.x >> 6] = mx;
        s2[threadIdx.x >> 6] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        tmax[t] = max(max(s1[0], s1[1]), max(s1[2], s1[3]));
        tmin[t] = min(min(s2[0], s2[1]), min(s2[2], s2[3]));
    }
}

// RK without a random scatter (blocks of at most 1 MiB = 256 windows of 2^R0_WS
// positions): k_r0_tile_heads counts every tile's slots per position window (BH),
// k_lsd_scan turns the counts into each (tile, window)'s place in the window-major pair
// array, the final pass stages its tile's pairs (position in the window << 20 | rank in
// the block) grouped by window in LDS and writes every window's run with consecutive
// lanes, and k_r0_rk assembles each window's 16 KB of RK in LDS and writes it with
// whole-line stores.  Every global store is then part of a coalesced wave store: stores
// that meet a line only across instructions are not merged well (PMC, 256 MiB: the direct
// 4-byte scatter wrote 8.4x the RK bytes, unstaged pair runs of ~16 entries 2.7x).
// per block: exclusive suffix min over its tiles (one workgroup per block)
__global__ __launch_bounds__(WG) void k_r0_tiles_rscan(const u32* in, u32* out, u32 tpb) {
    __shared__ u32 sh[WG / 64];
    __shared__ u32 edge;
    const u32 b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 carry = BIG;
    const u32 nch = (tpb + WG - 1) / WG;
    for (u32 cc = 0; cc < nch; ++cc) {
        const u32 k = (nch - 1 - cc) * WG + threadIdx.x;
        const u32 v = k < tpb ? in[(u64)b * tpb + k] : BIG;
        const u32 incl = wave_incl_scan_rev(v, OpMinU(), BIG);
        const u32 ex = KOLM_DPP(BIG, incl, DPP_WAVE_SHL1, 0xF);
        if (lane == 0) sh[w] = incl;
        __syncthreads();
        u32 wc = carry;
        for (u32 i = w + 1; i < WG / 64; ++i) wc = min(wc, sh[i]);
        if (k < tpb) out[(u64)b * tpb + k] = min(wc, ex);
        if (threadIdx.x == 0) edge = min(wc, incl);
        __syncthreads();
        carry = edge;
        __syncthreads();
    }
}

// RK is scattered for the positions p with p - base in [plo, phi) only (several launches
// over disjoint position windows keep one XCD's concurrent scatters inside a part of the
// block's RK that its L2 holds, so partial lines combine before write-back); `segs`: this
// launch also writes the next-round segments and split flags; `xcd`: XCD-contiguous tiles.
// PP (null: scatter RK directly): the window-major packed pair array; BH its offsets
__global__ __launch_bounds__(WG) void k_r0_final(LsdGeom g, const u32* HF, const u32* SA, const u32* cmax,
                                                 const u32* cmin, u32* RK, Seg* next, u32* next_cnt,
                                                 u32* blk_split, u32 plo, u32 phi, u32 segs, u32 xcd, u32 nt,
                                                 const u32* BH, u32* PP) {
    __shared__ u32 sh[WG / 64], sh2[WG / 64], sh3[WG / 64], sh4[WG / 64];
    __shared__ u32 wbase, anysplit;
    __shared__ u32 wo[256];     // PP: per window, where this tile's pairs go in PP
    __shared__ u32 wc[256];     // PP: per window, this tile's pair count, then its staging offset
    __shared__ u32 stg[LSD_T];  // PP: the tile's pairs grouped by window
    __shared__ u8 sbin[LSD_T];  // PP: window of each staged pair
    u32 lo, hi, b;
    const u32 t = xcd ? xcd_tile() : blockIdx.x;
    if (!g.range(t, lo, hi, b)) return;
    const u32 base = g.geo.base(b), bend = g.geo.end(b);
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) anysplit = 0;
    if (PP) {
        wo[tid] = BH[(u64)t * 256 + tid];
        wc[tid] = 0;
    }
    const u32 i0 = lo + tid * LSD_PT;
    u32 sv[LSD_PT];
    if (nt)  // SA / HF streamed past L2, which keeps the RK lines being filled
        load16nt(SA, i0, hi, sv);
    else
        load16(SA, i0, hi, sv);
    const u32 hm = nt ? __builtin_nontemporal_load(HF + (u64)t * WG + tid) : HF[(u64)t * WG + tid];
    bool hd[LSD_PT];
    u32 lmax = 0, lmin = BIG;
#pragma unroll
    for (u32 e = 0; e < LSD_PT; ++e) {
        const u32 i = i0 + e;
        hd[e] = (hm >> e) & 1u;
        if (hd[e]) {
            lmax = max(lmax, i);
            lmin = min(lmin, i);
        }
    }
    // forward exclusive max (group start entering the thread), reverse exclusive min
    // (first head after the thread)
    const u32 fi = wave_incl_scan(lmax, OpMaxU(), 0u), ri = wave_incl_scan_rev(lmin, OpMinU(), BIG);
    const u32 fex = KOLM_DPP(0u, fi, DPP_WAVE_SHR1, 0xF), rex = KOLM_DPP(BIG, ri, DPP_WAVE_SHL1, 0xF);
    if (lane == 63) sh[w] = fi;
    if (lane == 0) sh2[w] = ri;
    __syncthreads();
    u32 run = max(cmax[t], fex);
    for (u32 q = 0; q < w; ++q) run = max(run, sh[q]);
    u32 nh = min(cmin[t], rex);
    for (u32 q = w + 1; q < WG / 64; ++q) nh = min(nh, sh2[q]);
    if (nh == BIG) nh = bend;
    // ranks
    bool split = false;
    u32 pk[LSD_PT], loc[LSD_PT];
#pragma unroll
    for (u32 e = 0; e < LSD_PT; ++e) {
        const u32 i = i0 + e;
        pk[e] = loc[e] = 0;
        if (i < hi) {
            if (hd[e]) {
                run = i;
                split |= i != base;
            }
            if (PP) {  // the window counts are ready: barrier above
                pk[e] = ((sv[e] - base) & (R0_WIN - 1)) << 20 | (run - base);
                loc[e] = atomicAdd(&wc[(sv[e] - base) >> R0_WS], 1u);
            } else if (sv[e] - base - plo < phi - plo) {
                RK[sv[e]] = run;
            }
        }
    }
    if (PP) {
        __syncthreads();
        const u32 c = wc[tid], inc = wave_incl_scan(c, OpAddU(), 0u);
        if (lane == 63) sh4[w] = inc;
        __syncthreads();
        u32 so = inc - c;
        for (u32 q = 0; q < w; ++q) so += sh4[q];
        wc[tid] = so;
        __syncthreads();
#pragma unroll
        for (u32 e = 0; e < LSD_PT; ++e)
            if (i0 + e < hi) {
                const u32 k = (sv[e] - base) >> R0_WS, q = wc[k] + loc[e];
                stg[q] = pk[e];
                sbin[q] = (u8)k;
            }
        __syncthreads();
        for (u32 q = tid; q < hi - lo; q += WG) {
            const u32 k = sbin[q];
            PP[wo[k] + q - wc[k]] = stg[q];
        }
    }
    if (!segs) return;
    // group lengths (backwards) and next-round segments, one global atomic per workgroup
    u32 len[LSD_PT];
    u32 nseg = 0;
#pragma unroll
    for (int e = LSD_PT - 1; e >= 0; --e) {
        const u32 i = i0 + e;
        len[e] = 0;
        if (hd[e]) {
            len[e] = nh - i;
            nh = i;
            nseg += len[e] >= 2;
        }
    }
    const u32 incl = wave_incl_scan(nseg, OpAddU(), 0u);
    if (lane == 63) sh3[w] = incl;
    if (split) anysplit = 1;
    __syncthreads();
    u32 off = incl - nseg;
    for (u32 q = 0; q < w; ++q) off += sh3[q];
    if (tid == WG - 1) {
        const u32 tot = off + nseg;
        wbase = tot ? atomicAdd(next_cnt, tot) : 0u;
        if (anysplit) blk_split[b] = 1;
    }
    __syncthreads();
    off += wbase;
#pragma unroll
    for (u32 e = 0; e < LSD_PT; ++e)
        if (len[e] >= 2) next[off++] = Seg{i0 + e, len[e]};
}

// RK of one position window from its pairs (exactly the window's positions), through LDS
__global__ __launch_bounds__(WG) void k_r0_rk(Geom geo, u32 nwin, const u32* PP, u32* RK) {
    __shared__ u32 win[R0_WIN];
    const u32 b = blockIdx.x / nwin, k = blockIdx.x - b * nwin;
    const u32 base = geo.base(b), e = geo.end(b);
    const u32 lo = base + k * R0_WIN;
    if (lo >= e) return;
    const u32 n = min(R0_WIN, e - lo);
    for (u32 d = threadIdx.x; d < n; d += WG) {
        const u32 v = PP[lo + d];
        win[v >> 20] = base + (v & 0xFFFFFu);
    }
    __syncthreads();
    if ((lo & 3) == 0 && (n & 1023) == 0) {
        uint4* dst = reinterpret_cast<uint4*>(RK + lo);
        const uint4* src = reinterpret_cast<const uint4*>(win);
        for (u32 i = threadIdx.x; i < n / 4; i += WG) dst[i] = src[i];
    } else {
        for (u32 i = threadIdx.x; i < n; i += WG) RK[lo + i] = win[i];
    }
}

// ---------------------------------------------------------------------------------
// Alphabet compaction.  Rotation comparisons inside a block depend only on the ORDER of
// its byte values, so every byte is replaced by its rank among the block's distinct bytes
// (code < sigma_b) and a round-0 key packs C = min(32, 64 / w) characters of w = the
// batch's max ceil(log2 sigma_b) bits each into 64 bits (enwik-style text: 50 distinct
// bytes -> w = 6, C = 10 characters in the same 8 LSD passes that held 8 raw bytes; bit
// planes: w = 1, C = 32 in 4 passes).  Fewer positions stay active after round 0
// (text: 60 % instead of 79 %) and the doubling rounds start at h = C.
// ---------------------------------------------------------------------------------
constexpr u32 AL_PER = 65536;  // bytes per workgroup of k_alpha_present

// pres[b * 8 + (c >> 5)] bit (c & 31): byte value c occurs in block b
__global__ __launch_bounds__(WG) void k_alpha_present(Geom geo, const u8* text, u32 parts, u32* pres) {
    __shared__ u32 f[256];
    f[threadIdx.x] = 0;
    __syncthreads();
    const u32 b = blockIdx.x / parts, part = blockIdx.x - b * parts;
    const u32 lo = geo.base(b) + part * AL_PER, hi = min(lo + AL_PER, geo.end(b));
    for (u32 i = lo + threadIdx.x; i < hi; i += WG) f[text[i]] = 1u;  // benign same-value races
    __syncthreads();
    const u64 m = __ballot(f[threadIdx.x] != 0);
    if ((threadIdx.x & 31) == 0) {
        const u32 word = (u32)(m >> (threadIdx.x & 32));
        if (word) atomicOr(&pres[(u64)b * 8 + (threadIdx.x >> 5)], word);
    }
}

// code[b * 256 + c] = rank of byte c among block b's byte values; wmax = max bits per code
__global__ __launch_bounds__(WG) void k_alpha_codes(const u32* pres, u8* code, u32* wmax) {
    __shared__ u32 pw[8];
    const u32 b = blockIdx.x, c = threadIdx.x;
    if (c < 8) pw[c] = pres[(u64)b * 8 + c];
    __syncthreads();
    u32 r = 0;
    for (u32 k = 0; k < (c >> 5); ++k) r += __popc(pw[k]);
    r += __popc(pw[c >> 5] & ((1u << (c & 31)) - 1u));
    code[(u64)b * 256 + c] = (u8)r;
    if (c == 255) {
        const u32 sigma = r + ((pw[7] >> 31) & 1u);
        const u32 w = sigma > 1 ? 32 - __clz(sigma - 1) : 1u;
        atomicMax(wmax, w);
    }
}

// Round-0 keys by position: KA = the low 32 bits, KB = the high bits of the packed codes of
// the first C rotation characters (first character most significant).  A workgroup owns
// one LSD tile (one block's positions): text [lo, hi + C) and the block's code table in
// LDS, 16 consecutive positions per thread with a rolling key (drop the oldest character,
// append the next); positions whose C characters wrap inside their Lyndon factor (FEd <
// C) are rebuilt from the factor record.
// hist0 (optional): the first LSD pass's per-tile digit counts (digit 0 of KA), so that
// pass needs no histogram kernel of its own.
// part (0 .. min(sh, w)): the top `part` of the sh padding bits below the C codes hold the top
// `part` bits of character C's code, so round 0 also splits positions tied on C characters by most of the next one;
// the doubling rounds still start from h = C (groups equal on C characters and the partial one
// refine consistently: doubling compares (group(p), group(p + h)), and group(p + h) orders
// character h fully)
__global__ __launch_bounds__(WG) void k_keypos_r0(LsdGeom g, const u8* code, u32 C, u32 w, u32 sh, u32* KA, u32* KB,
                                                  u32* hist0,
                                                  ScanParts sp = ScanParts{}, u32 part = 0) {
    __shared__ __align__(16) u8 tx[LSD_T + 64];
    __shared__ u8 cd[256];
    __shared__ TileCounts h0;
    u32 lo, hi, b;
    const u32 tile = xcd_tile();
    if (!g.range(tile, lo, hi, b)) {  // a tile past its block's end (the whole workgroup)
        if (hist0) hist0[(u64)tile * 256 + threadIdx.x] = 0;
        return;
    }
    if (hist0) h0.clear();
    const u32 N = (u32)g.geo.N;
    cd[threadIdx.x] = code[(u64)b * 256 + threadIdx.x];
    const u32 n = min(hi + C + (part ? 1u : 0u), N) - lo;
    if ((((uintptr_t)g.text + lo) & 3) == 0) {  // dword copies (a dword that starts before N is allocated)
        const u32* src = reinterpret_cast<const u32*>(g.text + lo);
        u32* dst = reinterpret_cast<u32*>(tx);
        for (u32 i = threadIdx.x; i < (n + 3) / 4; i += WG) dst[i] = src[i];
    } else {
        for (u32 i = threadIdx.x; i < n; i += WG) tx[i] = g.text[lo + i];
    }
    __syncthreads();
    const u32 i0 = threadIdx.x * LSD_PT;
    if (lo + i0 < hi) {  // (no return: every thread reaches the histogram's barrier)
    // the 16 distances to the factor end (one 16-byte load when aligned and whole)
    u8 fed[LSD_PT];
    if (((lo + i0) & 15) == 0 && lo + i0 + LSD_PT <= hi) {
#pragma unroll
        for (u32 q = 0; q < LSD_PT / 16; ++q) {
            const uint4 v = reinterpret_cast<const uint4*>(g.FEd + lo + i0)[q];
            const u32 wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (u32 e = 0; e < 16; ++e) fed[16 * q + e] = (u8)(wd[e >> 2] >> (8 * (e & 3)));
        }
    } else {
#pragma unroll
        for (u32 e = 0; e < LSD_PT; ++e) fed[e] = lo + i0 + e < hi ? g.FEd[lo + i0 + e] : (u8)255;
    }
    const u64 mask = C * w >= 64 ? ~0ull : ((1ull << (C * w)) - 1);
    u64 key = 0;
    for (u32 k = 0; k < C; ++k) key = (key << w) | (i0 + k < n ? cd[tx[i0 + k]] : 0u);
    u32 ka[LSD_PT], kb[LSD_PT];
    const u32 psh = w - part, plo = sh - part;  // the partial character: its code's top `part` bits, right below character C - 1
#pragma unroll
    for (u32 e = 0; e < LSD_PT; ++e) {
        const u32 x = i0 + e + C;
        const u32 nc = x < n ? cd[tx[x]] : 0u;
        const u64 kk = (key << sh) | (part ? (u64)(nc >> psh) << plo : 0ull);
        ka[e] = (u32)kk;
        kb[e] = (u32)(kk >> 32);
        key = ((key << w) | nc) & mask;
    }
    const u32 need = C + (part ? 1u : 0u);  // characters read per position
#pragma unroll
    for (u32 e = 0; e < LSD_PT; ++e) {
        const u32 p = lo + i0 + e;
        if (p < hi && fed[e] < need) {  // the characters wrap inside the factor
            u32 fs, m;
            g.fac.locate(g.geo, p, fs, m);
            u32 t = p - fs;
            u64 k2 = 0;
            for (u32 k = 0; k < C; ++k) {
                k2 = (k2 << w) | cd[g.text[fs + t]];
                if (++t == m) t = 0;
            }
            const u64 kk = (k2 << sh) | (part ? (u64)(cd[g.text[fs + t]] >> psh) << plo : 0ull);
            ka[e] = (u32)kk;
            kb[e] = (u32)(kk >> 32);
        }
    }
    const u32 p0 = lo + i0;
    if ((p0 & 3) == 0 && p0 + LSD_PT <= hi) {
#pragma unroll
        for (u32 q = 0; q < LSD_PT / 4; ++q) {
            reinterpret_cast<uint4*>(KA + p0)[q] = make_uint4(ka[4 * q], ka[4 * q + 1], ka[4 * q + 2], ka[4 * q + 3]);
            if (KB) reinterpret_cast<uint4*>(KB + p0)[q] = make_uint4(kb[4 * q], kb[4 * q + 1], kb[4 * q + 2], kb[4 * q + 3]);
        }
    } else {
        for (u32 e = 0; e < LSD_PT && p0 + e < hi; ++e) {
            KA[p0 + e] = ka[e];
            if (KB) KB[p0 + e] = kb[e];
        }
    }
    if (hist0) {
#pragma unroll
        for (u32 e = 0; e < LSD_PT; ++e)
            if (p0 + e < hi) h0.add(digit<0>(ka[e]));
    }
    }
    if (hist0) {
        __syncthreads();
        const u32 v = h0.total(threadIdx.x);
        hist0[(u64)tile * 256 + threadIdx.x] = v;
        add_part_total(g, sp, tile, v);
    }
}

template <int P, int SRC, int G, int OUT>
void lsd_pass(const LsdGeom& g, u32 nt, const u32* kin, const u32* pin, u32* kout, u32* pout, const u32* kg,
              u32* hist, bool counted, hipStream_t s, KTimer* kt, const ScanParts& sp) {
    static const std::string hn = "k_lsd_hist<" + std::to_string(P) + ", " + std::to_string(SRC) + ">";
    // the timer carries the launched name
    static const std::string sn = "k_lsd_scatter_w<" + std::to_string(P) + ", " + std::to_string(SRC) + ", " +
                                  std::to_string(G) + (OUT ? ", " + std::to_string(OUT) + ">" : std::string(">"));
    const u64 N = g.geo.N, H = (u64)nt * 1024;  // H: per-tile histogram bytes
    if (!counted) {  // counted: the producer of kin wrote the tile histograms
        KScope k(kt, KT_LSD, hn.c_str(), (SRC == SRC_REC ? 8 : 4) * N + H);
        k_lsd_hist<P, SRC><<<nt, WG, 0, s>>>(g, kin, hist, sp);
    }
    if (sp.cur) {
        KScope k(kt, KT_LSD, "k_lsd_scan2", 2 * H);
        k_lsd_scan2<<<g.geo.nb * sp.np, WG, 0, s>>>(g, hist, sp);
    } else {
        KScope k(kt, KT_LSD, "k_lsd_scan", 3 * H);
        // four threads per digit for batches of fewer than 64 blocks (a latency-bound workgroup
        // per block; on full batches the 1024-thread workgroups wait beside the LZ77 parse:
        // 256 MiB LSD 18.4 -> 19.2 ms with them).  KOLM_LSD_SCAN4 = 0 / 1 forces it.
        // KOLM_LSD_SCAN4 = 0 / 1 / 2: one / four / two threads per digit
        static const int s4e = getenv("KOLM_LSD_SCAN4") ? atoi(getenv("KOLM_LSD_SCAN4")) : -1;
        const int mode = s4e >= 0 ? s4e : (g.geo.nb < 64 ? 1 : 0);
        if (mode == 1)
            k_lsd_scanp<4><<<g.geo.nb, 4 * WG, 0, s>>>(g, hist);
        else if (mode == 2)
            k_lsd_scanp<2><<<g.geo.nb, 2 * WG, 0, s>>>(g, hist);
        else
            k_lsd_scan<<<g.geo.nb, WG, 0, s>>>(g, hist);
    }
    {
        // key + position in (the first pass reads the key by position only) and out; G: + the gather
        // bytes in: key (+ position unless implicit or packed); out: key + position, or the packed word
        const u64 in = (SRC == SRC_PAIR || SRC == SRC_REC) ? 8 : 4, outb = OUT == OUT_PK ? 4 : 8;
        KScope k(kt, KT_LSD, sn.c_str(), (in + outb) * N + (G ? 4 * N : 0) + H);
        // k_lsd_scatter_w (three barriers per tile; 256 MiB text, overlapped: 1.5-1.7 -> 0.9-1.0
        // ms per pass)
        k_lsd_scatter_w<P, SRC, G, OUT><<<nt, WG, 0, s>>>(g, kin, pin, kout, pout, kg, hist);
    }
}

// The eight passes of record mode (8-byte keys, both halves 4 passes): the first half KA
// (positions) -> records -> records -> packed words -> records with KB gathered; the second half
// records -> records -> records -> records -> (K2, SA) pairs for the group heads
void run_pass_rec(u32 idx, const LsdGeom& g, u32 nt, const u32* kin, u32* kout, u32* pout, const u32* kg,
                  u32* hist, hipStream_t s, KTimer* kt, const ScanParts& sp) {
    switch (idx) {
        case 0: return lsd_pass<0, SRC_KP, 0, OUT_REC>(g, nt, kin, nullptr, kout, nullptr, nullptr, hist, true, s, kt, sp);
        case 1: return lsd_pass<1, SRC_REC, 0, OUT_REC>(g, nt, kin, nullptr, kout, nullptr, nullptr, hist, false, s, kt, sp);
        case 2: return lsd_pass<2, SRC_REC, 0, OUT_PK>(g, nt, kin, nullptr, kout, nullptr, nullptr, hist, false, s, kt, sp);
        case 3: return lsd_pass<3, SRC_PK, 1, OUT_REC>(g, nt, kin, nullptr, kout, nullptr, kg, hist, false, s, kt, sp);
        case 4: return lsd_pass<0, SRC_REC, 0, OUT_REC>(g, nt, kin, nullptr, kout, nullptr, nullptr, hist, false, s, kt, sp);
        case 5: return lsd_pass<1, SRC_REC, 0, OUT_REC>(g, nt, kin, nullptr, kout, nullptr, nullptr, hist, false, s, kt, sp);
        case 6: return lsd_pass<2, SRC_REC, 0, OUT_REC>(g, nt, kin, nullptr, kout, nullptr, nullptr, hist, false, s, kt, sp);
        default: return lsd_pass<3, SRC_REC, 0, OUT_PAIR>(g, nt, kin, nullptr, kout, pout, nullptr, hist, false, s, kt, sp);
    }
}

using PassFn = void (*)(const LsdGeom&, u32, const u32*, const u32*, u32*, u32*, const u32*, u32*, bool, hipStream_t,
                        KTimer*, const ScanParts&);
template <int P>
constexpr PassFn pass_of(int src_kp, int gat) {
    return src_kp ? (gat ? lsd_pass<P, SRC_KP, 1, 0> : lsd_pass<P, SRC_KP, 0, 0>)
                  : (gat ? lsd_pass<P, SRC_PAIR, 1, 0> : lsd_pass<P, SRC_PAIR, 0, 0>);
}
// pk: 1 = this pass (P = 2, pairs in) writes packed words, 2 = this pass (P = 3, gather) reads them
void run_pass(int P, bool src_kp, bool gat, const LsdGeom& g, u32 nt, const u32* kin, const u32* pin, u32* kout,
              u32* pout, const u32* kg, u32* hist, bool counted, hipStream_t s, KTimer* kt, int pk,
              const ScanParts& sp) {
    if (pk == 1) return lsd_pass<2, SRC_PAIR, 0, OUT_PK>(g, nt, kin, pin, kout, pout, kg, hist, counted, s, kt, sp);
    if (pk == 2) return lsd_pass<3, SRC_PK, 1, OUT_PAIR>(g, nt, kin, pin, kout, pout, kg, hist, counted, s, kt, sp);
    const int a = src_kp ? 1 : 0, c = gat ? 1 : 0;
    const PassFn f = P == 0 ? pass_of<0>(a, c) : P == 1 ? pass_of<1>(a, c) : P == 2 ? pass_of<2>(a, c) : pass_of<3>(a, c);
    f(g, nt, kin, pin, kout, pout, kg, hist, counted, s, kt, sp);
}

}  // namespace

u32 lsd_tiles(const Geom& geo) { return (geo.bs + LSD_T - 1) / LSD_T * geo.nb; }

// Per-block code tables (alphabet compaction); returns the max code width w of the batch
// (one host round trip).  compact = false: identity codes, w = 8.
u32 launch_alpha(const Geom& geo, const u8* text, u32* pres, u8* code, u32* d_w, u32* h_w, bool compact,
                 hipStream_t s, KTimer* kt) {
    if (!geo.N) return 8;
    if (!compact) {
        std::vector<u8> id(256 * (size_t)geo.nb);
        for (size_t i = 0; i < id.size(); ++i) id[i] = (u8)i;
        KOLM_HIP_CHECK(hipMemcpyAsync(code, id.data(), id.size(), hipMemcpyHostToDevice, s));
        KOLM_HIP_CHECK(hipStreamSynchronize(s));
        return 8;
    }
    launch_alpha_async(geo, text, pres, code, d_w, h_w, s, kt);
    KOLM_HIP_CHECK(hipStreamSynchronize(s));
    return alpha_width(*h_w);
}

void launch_alpha_async(const Geom& geo, const u8* text, u32* pres, u8* code, u32* d_w, u32* h_w, hipStream_t s,
                        KTimer* kt, bool zeroed) {
    if (!geo.N) {
        if (h_w) *h_w = 8;
        return;
    }
    const u32 parts = (geo.bs + AL_PER - 1) / AL_PER;
    if (!zeroed) {  // (zeroed: the caller's k_zero_spans cleared pres and *d_w)
        KOLM_HIP_CHECK(hipMemsetAsync(pres, 0, sizeof(u32) * 8 * geo.nb, s));
        KOLM_HIP_CHECK(hipMemsetAsync(d_w, 0, sizeof(u32), s));
    }
    {
        KScope k(kt, KT_LSD, "k_alpha_present", geo.N);
        k_alpha_present<<<parts * geo.nb, WG, 0, s>>>(geo, text, parts, pres);
        k_alpha_codes<<<geo.nb, WG, 0, s>>>(pres, code, d_w);
    }
    if (h_w) KOLM_HIP_CHECK(hipMemcpyAsync(h_w, d_w, sizeof(u32), hipMemcpyDeviceToHost, s));
}

u32 alpha_width(u32 h_w) { return std::max<u32>(1, std::min<u32>(8, h_w)); }

// Round 0 of the cyclic sort: a stable sort of every block's positions by the packed codes
// of their first C rotation characters (k_keypos_r0: KA = low 32 bits -> RK, KB = high bits
// -> KP, by position).  LSD passes over the digits of KA (text order -> ... ), the last of
// them writing KB[SA] as the next key when KB has digits, then over the digits of KB; the
// passes alternate (K2, SA) / (K22, SA2) and end in (K2, SA).  A slot heads a group when K2
// differs from the previous slot's or (two halves) KA[SA[slot]] does: head masks (HF), then
// ranks and next-round segments.
void launch_round0(const Geom& geo, const R0Bufs& t, Seg* next, u32* next_cnt, u32* blk_split, hipStream_t s,
                   KTimer* kt) {
    if (!geo.N) return;
    LsdGeom g{geo, (geo.bs + LSD_T - 1) / LSD_T, t.text, t.FEd, t.fac};
    const u32 nt = g.tpb * geo.nb;
    const u64 N = geo.N;
    // D byte digits; the packed codes are left-aligned in them, so the 8 D - C w padding bits
    // fall into the first pass's digit (its few distinct values keep that scatter's runs long)
    const u32 bits = t.chars * t.w, D = (bits + 7) / 8, sh = 8 * D - bits;
    const u32 pa = std::min<u32>(4, D), pb = D - pa;
    u32* K[2] = {t.K2, t.K22};
    u32* S[2] = {t.SA, t.SA2};
    const u32 T = pa + pb;
    int o = (T & 1) ? 0 : 1;  // output pair of the first pass: the last one lands in (K2, SA)
    {
        // the padding bits carry the next character's top bits
        const u32 part = std::min(sh, t.w);
        // per-(block, part) totals for the one-part-long scans
        const bool parts = t.swc && g.tpb > 1;
        ScanParts sp[2];
        if (parts) {
            u32 plt = 0;
            while (((g.tpb + (1u << plt) - 1) >> plt) > 16) ++plt;
            const u32 np = (g.tpb + (1u << plt) - 1) >> plt;
            const u64 cw = (u64)geo.nb * np * 256;  // np <= 16: t.swc holds 2 * nb * 16 * 256 words
            sp[0] = ScanParts{t.swc, t.swc + cw, np, plt};
            sp[1] = ScanParts{t.swc + cw, t.swc, np, plt};
            KOLM_HIP_CHECK(hipMemsetAsync(t.swc, 0, sizeof(u32) * 2 * cw, s));
        }
        u32 pidx = 0;
        auto spp = [&]() -> const ScanParts& { return sp[parts ? (pidx & 1) : 0]; };
        {
            // text + FEd 2 (+ factor starts near factor ends), KA 4 (+ KB 4)
            KScope k(kt, KT_KEYGEN, "k_keypos_r0", N * (pb ? 10 : 6));
            k_keypos_r0<<<nt, WG, 0, s>>>(g, t.code, t.chars, t.w, sh, t.RK, pb ? t.KP : nullptr, t.hist, spp(),
                                          part);
        }
        // the first half's passes 2 -> 3 exchange one packed word per element (digit 3 and the
        // position inside the block) when a block position fits 24 bits
        const bool pack = pa == 4 && pb > 0 && geo.bs <= (1u << 24);
        // record mode for 8-byte keys: the pairs between passes as u64 records
        const bool rec = pack && pb == 4 && t.rec[0] && t.rec[1];
        if (rec) {
            u32* R2[2] = {reinterpret_cast<u32*>(t.rec[0]), reinterpret_cast<u32*>(t.rec[1])};
            // inputs / outputs per pass: KA -> R0 -> R1 -> K22 (packed) -> R0 -> R1 -> R0 -> R1 -> (K2, SA)
            const u32* in[8] = {t.RK, R2[0], R2[1], t.K22, R2[0], R2[1], R2[0], R2[1]};
            u32* out[8] = {R2[0], R2[1], t.K22, R2[0], R2[1], R2[0], R2[1], t.K2};
            for (u32 q = 0; q < 8; ++q, ++pidx)
                run_pass_rec(q, g, nt, in[q], out[q], q == 7 ? t.SA : nullptr, q == 3 ? t.KP : nullptr, t.hist, s, kt,
                             spp());
        }
        for (u32 q = 0; q < (rec ? 0u : pa); ++q) {
            const bool first = q == 0, gat = q + 1 == pa && pb > 0;
            const int pk = pack ? (q == 2 ? 1 : q == 3 ? 2 : 0) : 0;
            run_pass((int)q, first, gat, g, nt, first ? t.RK : K[o ^ 1], first ? nullptr : S[o ^ 1], K[o], S[o],
                     gat ? t.KP : nullptr, t.hist, first, s, kt, pk, spp());
            o ^= 1;
            ++pidx;
        }
        for (u32 q = 0; q < (rec ? 0u : pb); ++q) {
            run_pass((int)q, false, false, g, nt, K[o ^ 1], S[o ^ 1], K[o], S[o], nullptr, t.hist, false, s, kt, 0,
                     spp());
            o ^= 1;
            ++pidx;
        }
    }
    // RK through position windows (k_r0_rk) when every block has at most 256 of them, else
    // the direct scatter
    const bool win = geo.bs <= 256 * R0_WIN;
    {
        // K 4 (+ SA 4 + the KA gather 4) read, head masks written
        KScope k(kt, KT_LSD, "k_r0_tile_heads", (pb || win ? 12 : 4) * N);
        k_r0_tile_heads<<<nt, WG, 0, s>>>(g, t.K2, t.SA, pb ? t.RK : nullptr, t.HF, t.tmax, t.tmin,
                                          win ? t.hist : nullptr);
        k_tiles_max_scan<<<geo.nb, WG, 0, s>>>(t.tmax, t.cmax, g.tpb);
        k_r0_tiles_rscan<<<geo.nb, WG, 0, s>>>(t.tmin, t.cmin, g.tpb);
    }
    if (win) {
        const u32 nwin = (geo.bs + R0_WIN - 1) / R0_WIN;
        static const int s4e = getenv("KOLM_LSD_SCAN4") ? atoi(getenv("KOLM_LSD_SCAN4")) : -1;
        const int mode = s4e >= 0 ? s4e : (geo.nb < 64 ? 1 : 0);
        if (mode == 1)
            k_lsd_scanp<4><<<geo.nb, 4 * WG, 0, s>>>(g, t.hist);  // window counts -> pair offsets
        else if (mode == 2)
            k_lsd_scanp<2><<<geo.nb, 2 * WG, 0, s>>>(g, t.hist);
        else
            k_lsd_scan<<<geo.nb, WG, 0, s>>>(g, t.hist);
        {
            // SA 4 read, pairs 4 written (+ head masks, 8 B per new segment)
            KScope k(kt, KT_LSD, "k_r0_final", 8 * N);
            k_r0_final<<<nt, WG, 0, s>>>(g, t.HF, t.SA, t.cmax, t.cmin, t.RK, next, next_cnt, blk_split, 0, 0, 1, 1, 0,
                                         t.hist, t.K22);
        }
        {
            KScope k(kt, KT_LSD, "k_r0_rk", 8 * N);  // pairs 4 read, RK 4 written
            k_r0_rk<<<nwin * geo.nb, WG, 0, s>>>(geo, nwin, t.K22, t.RK);
        }
        return;
    }
    {
        // SA 4 read, RK 4 scattered (+ head masks, 8 B per new segment)
        KScope k(kt, KT_LSD, "k_r0_final", 8 * N);
        // two position windows per block on XCD-contiguous tiles (256 MiB text 3.24 -> 2.42 ms per
        // step against one window)
        constexpr u32 parts = 2, xcd = 1, ntl = 0;
        const u32 step = (geo.bs + parts - 1) / parts;
        for (u32 q = 0; q < parts; ++q)
            k_r0_final<<<nt, WG, 0, s>>>(g, t.HF, t.SA, t.cmax, t.cmin, t.RK, next, next_cnt, blk_split, q * step,
                                         q + 1 == parts ? 0xFFFFFFFFu : (q + 1) * step, q == 0, xcd, ntl, nullptr,
                                         nullptr);
    }
}

}  // namespace kolm
