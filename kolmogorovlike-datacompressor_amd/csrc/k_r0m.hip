// Round 0 of the cyclic suffix sort as MSD radix partitions + LDS bucket sorts (gfx950).
//
// Round 0 orders every block's positions by the first C characters of their rotation (the
// packed alphabet codes, C w <= 64 bits, left-aligned in a 64-bit key), ties in position
// order (PY's (fi, i) rule, PY:362-378 / 379-423).  The LSD form (k_lsd.hip) streams all
// 64 key bits through 8 scatter passes whatever the data; text needs far fewer: after the
// first one or two key bytes most positions sit in buckets small enough to finish inside
// one workgroup's LDS.  So:
//   level 0     per block: counts of the top key byte per 4096-position tile (fused into the
//               key kernel), a per-block scan, and a stable scatter of (key, position) into
//               bucket order;
//   level l>=1  the same over the buckets still too large for LDS (segments with their own
//               tile lists), one key byte further; a bucket whose key bits are exhausted is
//               a tie group and is final as it stands;
//   finish      every final bucket sorted in LDS by its remaining key bits (a bucket's
//               elements arrive in position order, so the sort word is (key << consumed) |
//               index and ties keep position order), then SA, RK (= group start slot), the
//               next round's tie groups and the block split flags, exactly as the LSD
//               form's k_r0_final writes them.
// 256 MiB of text: ~2.3 scatter passes of 24 B per element instead of eight of 16-20 B.
#include "kolm_internal.h"

#include <algorithm>
#include <cstring>
#include <type_traits>
#include <cstdlib>
#include <string>
#include <vector>

namespace kolm {

namespace {

constexpr u32 MT = 4096;        // elements per MSD tile (one 256-thread workgroup, 16 per thread)
constexpr u32 MPT = MT / WG;
constexpr u32 NCLS = 11;        // final classes: 0 small ties / singletons, 1 big ties, 2 + (C - 5): LDS sorts
constexpr u32 TIE_SMALL = 256;  // tie groups up to this length: one thread each
constexpr u32 CMIN = 5, CMAX = 13;  // LDS sort sub-arrays of 2^C slots (32 .. 8192 elements)

// counters (zeroed per round 0): per level parity next-segment / next-tile counts, final class
// counts
enum : int { RC_SEG = 0, RC_TILE = 2, RC_CLS = 4, RC_N = 16 };
static_assert(RC_CLS + NCLS <= RC_N && NCLS == R0M_NCLS, "counter slots / class count");

struct Fin {  // a final bucket: slots [start, start + len), sorted `lvl` key bytes deep
    u32 start;
    u32 len;
    u32 lvl;  // key bytes consumed (>= 1); its data lies in buffer (lvl - 1) & 1
};

struct R0M {
    Geom geo;
    u32 tpb;        // level 0: LSD tiles per block (k_keypos_r0's histogram rows)
    u32 kbits;      // key bits C w (left-aligned in 64)
    const u32* KH0; // level 0 input: key words by position
    const u32* KL0;
    u32* KH[2];     // level outputs (ping-pong): key high / low words and positions by slot
    u32* KL[2];
    u32* PS[2];
    u32* SA;        // out
    u32* RK;        // out
    u32* blk_split;
    Seg* next;      // out: next round's groups of >= 2
    u32* next_cnt;
    Fin* fin[NCLS];
    u32* cnt;       // RC_*
    LSeg* segs[2];  // per level parity
    LTile* tiles[2];
    // level 0 from the text (k_r0m_hist0 / k_r0m_scatter0t): keys computed, not loaded
    const u8* text;
    const u8* FEd;   // min(distance to the factor end, 255)
    Factors fac;
    const u8* code;  // [nb * 256] per-block alphabet codes
    u32 C, w;        // characters per key, bits per code
};

// level-0 tile t: block positions [lo, hi) (false: a tile past its block's end)
__device__ inline bool tile0(const R0M& r, u32 t, u32& lo, u32& hi, u32& b) {
    b = t / r.tpb;
    lo = r.geo.base(b) + (t - b * r.tpb) * MT;
    hi = min(lo + MT, r.geo.end(b));
    return lo < hi;
}

// the tile's text [lo, hi + C) and the block's code table into LDS
__device__ inline void stage0(const R0M& r, u32 lo, u32 hi, u32 b, u8* tx, u8* cd) {
    cd[threadIdx.x] = r.code[(u64)b * 256 + threadIdx.x];
    const u32 n = min(hi + r.C, (u32)r.geo.N) - lo;
    if ((((uintptr_t)r.text + lo) & 3) == 0) {  // a dword that starts before N is allocated
        const u32* src = reinterpret_cast<const u32*>(r.text + lo);
        u32* dst = reinterpret_cast<u32*>(tx);
        for (u32 i = threadIdx.x; i < (n + 3) / 4; i += WG) dst[i] = src[i];
    } else {
        for (u32 i = threadIdx.x; i < n; i += WG) tx[i] = r.text[lo + i];
    }
}

// the left-aligned 64-bit key of position p: its first C rotation characters (as
// k_keypos_r0: straight from the staged text unless they wrap inside p's Lyndon factor)
__device__ inline u64 key0(const R0M& r, const u8* tx, const u8* cd, u32 lo, u32 p, u32 fed) {
    u64 key = 0;
    if (fed >= r.C) {
        const u8* t = tx + (p - lo);
        for (u32 k = 0; k < r.C; ++k) key = (key << r.w) | cd[t[k]];
    } else {
        u32 fs, m;
        r.fac.locate(r.geo, p, fs, m);
        u32 t = p - fs;
        for (u32 k = 0; k < r.C; ++k) {
            key = (key << r.w) | cd[r.text[fs + t]];
            if (++t == m) t = 0;
        }
    }
    return key << (64 - r.kbits);
}

// exclusive scan over a workgroup of nw waves (REV: from the last thread down)
template <bool REV, class Op>
__device__ inline u32 wg_scan_x(u32 v, Op op, u32 ident, u32* sh, u32 nw) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u32 incl = REV ? wave_incl_scan_rev(v, op, ident) : wave_incl_scan(v, op, ident);
    const u32 ex = REV ? KOLM_DPP(ident, incl, DPP_WAVE_SHL1, 0xF) : KOLM_DPP(ident, incl, DPP_WAVE_SHR1, 0xF);
    if (REV ? lane == 0 : lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = ident;
    if (!REV) {
        for (u32 i = 0; i < w; ++i) carry = op(carry, sh[i]);
    } else {
        for (u32 i = w + 1; i < nw; ++i) carry = op(carry, sh[i]);
    }
    __syncthreads();
    return op(carry, ex);
}

__device__ inline u32 digit_of(u32 kh, u32 kl, u32 lvl) {  // key byte `lvl` (0 = top)
    return lvl < 4 ? (kh >> (24 - 8 * lvl)) & 255u : (kl >> (56 - 8 * lvl)) & 255u;
}

// a bucket of `len` elements whose first lvl key bytes are known: final when its key bits are
// exhausted (a tie group) or it fits an LDS sort whose words hold (remaining key, index)
__device__ inline int final_class(u32 len, u32 lvl, u32 kbits) {
    if (8 * lvl >= kbits || len == 1) return len <= TIE_SMALL ? 0 : 1;
    const u32 F = 64 - kbits + 8 * lvl;  // zero bits below the remaining key in (key << 8 lvl)
    const u32 lim = F >= CMAX ? (1u << CMAX) : (1u << F);
    if (len > lim) return -1;
    const u32 c = 32 - __clz(len - 1);  // sub-array of 2^c >= len slots
    return 2 + (int)(max(c, CMIN) - CMIN);
}

// ---------------------------------------------------------------------------------------
// level 0 straight from the text: per-tile counts of the top key byte (rolling keys over 16
// consecutive positions per thread), then the stable scatter with the keys recomputed —
// no keys by position are written or read
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_r0m_hist0(R0M r, u32* hist) {
    __shared__ __align__(16) u8 tx[MT + 64];
    __shared__ u8 cd[256];
    __shared__ u32 h[WG / 64][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
    const u32 t = xcd_tile();
    u32 lo, hi, b;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) h[i][tid] = 0;
    if (!tile0(r, t, lo, hi, b)) {
        hist[(u64)t * 256 + tid] = 0;
        return;
    }
    stage0(r, lo, hi, b, tx, cd);
    __syncthreads();
    const u32 i0 = tid * MPT, n = min(hi + r.C, (u32)r.geo.N) - lo;
    if (lo + i0 < hi) {
        const u64 mask = r.kbits >= 64 ? ~0ull : ((1ull << r.kbits) - 1);
        u64 key = 0;
        for (u32 k = 0; k < r.C; ++k) key = (key << r.w) | (i0 + k < n ? cd[tx[i0 + k]] : 0u);
        for (u32 e = 0; e < MPT && lo + i0 + e < hi; ++e) {
            const u32 p = lo + i0 + e;
            const u32 fed = r.FEd[p];
            const u64 k64 = fed >= r.C ? key << (64 - r.kbits) : key0(r, tx, cd, lo, p, fed);
            atomicAdd(&h[w][(u32)(k64 >> 56)], 1u);
            const u32 x = i0 + e + r.C;
            key = ((key << r.w) | (x < n ? cd[tx[x]] : 0u)) & mask;
        }
    }
    __syncthreads();
    hist[(u64)t * 256 + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

__global__ __launch_bounds__(WG) void k_r0m_scatter0t(R0M r, const u32* hist) {
    __shared__ __align__(16) u8 tx[MT + 64];
    __shared__ u8 cd[256];
    __shared__ u32 wc[WG / 64][256];
    __shared__ u16 loc[MT];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 t = xcd_tile();
    u32 lo, hi, b;
    if (!tile0(r, t, lo, hi, b)) return;
    stage0(r, lo, hi, b, tx, cd);
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) wc[i][tid] = 0;
    const u32 tb = hist[(u64)t * 256 + tid];
    const u32 q0 = lo + w * (MT / 4);
    u8 fed[MPT];
#pragma unroll
    for (u32 j = 0; j < MPT; ++j) {
        const u32 i = q0 + j * 64 + lane;
        fed[j] = i < hi ? r.FEd[i] : (u8)255;
    }
    __syncthreads();
    u64 key[MPT];
#pragma unroll
    for (u32 j = 0; j < MPT; ++j) {
        const u32 i = q0 + j * 64 + lane;
        key[j] = i < hi ? key0(r, tx, cd, lo, i, fed[j]) : 0ull;
    }
    const u64 lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    u16* lw = loc + w * (MT / 4) + lane;
#pragma unroll
    for (u32 j = 0; j < MPT; ++j) {
        const bool valid = q0 + j * 64 + lane < hi;
        const u32 dg = (u32)(key[j] >> 56);
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
    for (u32 j = 0; j < MPT; ++j) {
        const u32 i = q0 + j * 64 + lane;
        if (i < hi) {
            const u32 o = wc[w][(u32)(key[j] >> 56)] + lw[j * 64];
            r.KH[0][o] = (u32)(key[j] >> 32);
            r.KL[0][o] = (u32)key[j];
            r.PS[0][o] = i;
        }
    }
}

// ---------------------------------------------------------------------------------------
// level l >= 1: per-tile counts of key byte l
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_r0m_hist(R0M r, u32 lvl, const u32* ntiles_dev, u32* hist) {
    __shared__ u32 h[WG / 64][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
    const LTile* tiles = r.tiles[lvl & 1];
    const LSeg* segs = r.segs[lvl & 1];
    const u32 t = xcd_tile();
    if (t >= *ntiles_dev) return;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) h[i][tid] = 0;
    __syncthreads();
    const LTile tl = tiles[t];
    const LSeg sg = segs[tl.seg];
    const u32 lo = sg.start + tl.k * MT, hi = min(lo + MT, sg.start + sg.len);
    const u32* K = lvl < 4 ? r.KH[(lvl - 1) & 1] : r.KL[(lvl - 1) & 1];
    const u32 sh = lvl < 4 ? 24 - 8 * lvl : 56 - 8 * lvl;
    u32 v[MPT];  // all 16 loads in flight before the LDS atomics
#pragma unroll
    for (u32 j = 0; j < MPT; ++j) v[j] = lo + j * WG + tid < hi ? K[lo + j * WG + tid] : 0u;
#pragma unroll
    for (u32 j = 0; j < MPT; ++j)
        if (lo + j * WG + tid < hi) atomicAdd(&h[w][(v[j] >> sh) & 255u], 1u);
    __syncthreads();
    hist[(u64)t * 256 + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

// ---------------------------------------------------------------------------------------
// per segment (level 0: per block): digit totals, bucket starts, per-(tile, digit) scatter
// offsets (in place in hist), and the buckets' fate: final (class lists) or the next level
// ---------------------------------------------------------------------------------------
template <int L0>
__global__ __launch_bounds__(WG) void k_r0m_scan(R0M r, u32 lvl, const u32* nseg_dev, u32* hist) {
    __shared__ u32 sh[WG / 64];
    __shared__ u32 lcnt[NCLS + 1], lbase[NCLS + 1], ltile, ltb, nz;
    const u32 d = threadIdx.x, lane = d & 63, w = d >> 6;
    u32 start, t0, nt, b;
    if (L0) {
        b = blockIdx.x;
        start = r.geo.base(b);
        t0 = b * r.tpb;
        nt = r.tpb;
    } else {
        if (blockIdx.x >= *nseg_dev) return;
        const LSeg sg = r.segs[lvl & 1][blockIdx.x];
        start = sg.start;
        t0 = sg.tile_base;
        nt = sg.ntiles;
        b = r.geo.block_of(start);
    }
    if (d <= NCLS) lcnt[d] = 0;
    if (d == 0) {
        ltile = 0;
        nz = 0;
    }
    constexpr u32 B = 16;
    u32 acc = 0;
    for (u32 k = 0; k < nt; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < nt ? hist[(u64)(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j) {
            if (k + j < nt) hist[(u64)(t0 + k + j) * 256 + d] = acc;
            acc += v[j];
        }
    }
    const u32 incl = wave_incl_scan(acc, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = 0;
    for (u32 i = 0; i < w; ++i) carry += sh[i];
    const u32 bstart = start + carry + incl - acc;  // this digit's bucket
    for (u32 k = 0; k < nt; k += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = k + j < nt ? hist[(u64)(t0 + k + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j)
            if (k + j < nt) hist[(u64)(t0 + k + j) * 256 + d] = v[j] + bstart;
    }
    // the buckets' fate (this level consumes key byte lvl: lvl + 1 bytes are known after it)
    int cls = acc ? final_class(acc, lvl + 1, r.kbits) : -2;
    const u32 ntn = cls == -1 ? (acc + MT - 1) / MT : 0u;
    u32 slot = 0, tslot = 0;
    if (acc) atomicAdd(&nz, 1u);
    if (cls >= 0) slot = atomicAdd(&lcnt[cls], 1u);
    if (cls == -1) {
        slot = atomicAdd(&lcnt[NCLS], 1u);
        tslot = atomicAdd(&ltile, ntn);
    }
    __syncthreads();
    if (d < NCLS && lcnt[d]) lbase[d] = atomicAdd(&r.cnt[RC_CLS + d], lcnt[d]);
    if (d == NCLS && lcnt[NCLS]) lbase[NCLS] = atomicAdd(&r.cnt[RC_SEG + ((lvl + 1) & 1)], lcnt[NCLS]);
    if (d == NCLS + 1 && ltile) ltb = atomicAdd(&r.cnt[RC_TILE + ((lvl + 1) & 1)], ltile);
    if (d == NCLS + 2 && nz > 1) r.blk_split[b] = 1;  // two or more groups in the block
    __syncthreads();
    if (cls >= 0) {
        r.fin[cls][lbase[cls] + slot] = Fin{bstart, acc, lvl + 1};
    } else if (cls == -1) {
        const u32 si = lbase[NCLS] + slot, tb = ltb + tslot;
        r.segs[(lvl + 1) & 1][si] = LSeg{bstart, acc, tb, ntn};
        for (u32 k = 0; k < ntn; ++k) r.tiles[(lvl + 1) & 1][tb + k] = LTile{si, k};
    }
}

// ---------------------------------------------------------------------------------------
// stable scatter of one tile by key byte lvl (k_lsd_scatter_w's form: wave w owns the tile's
// quarter [1024 w, 1024 (w + 1)), ballot ranking, per-wave digit counters, bases per
// (digit, wave)); level 0 reads the keys by position (positions implicit)
// ---------------------------------------------------------------------------------------
template <int L0>
__global__ __launch_bounds__(WG) void k_r0m_scatter(R0M r, u32 lvl, const u32* ntiles_dev, const u32* hist) {
    __shared__ u32 wc[WG / 64][256];
    __shared__ u16 loc[MT];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 t = xcd_tile();
    u32 lo, hi;
    if (L0) {
        const u32 b = t / r.tpb, k = t - b * r.tpb;
        lo = r.geo.base(b) + k * MT;
        hi = min(lo + MT, r.geo.end(b));
        if (lo >= hi) return;
    } else {
        if (t >= *ntiles_dev) return;
        const LTile tl = r.tiles[lvl & 1][t];
        const LSeg sg = r.segs[lvl & 1][tl.seg];
        lo = sg.start + tl.k * MT;
        hi = min(lo + MT, sg.start + sg.len);
    }
    const u32 src = (lvl - 1) & 1, dst = lvl & 1;
    const u32* KHi = L0 ? r.KH0 : r.KH[src];
    const u32* KLi = L0 ? r.KL0 : r.KL[src];
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) wc[i][tid] = 0;
    const u32 tb = hist[(u64)t * 256 + tid];
    u32 kh[MPT], kl[MPT], ps[MPT];
    const u32 q0 = lo + w * (MT / 4);
#pragma unroll
    for (u32 j = 0; j < MPT; ++j) {
        const u32 i = q0 + j * 64 + lane;
        kh[j] = kl[j] = ps[j] = 0;
        if (i < hi) {
            kh[j] = KHi[i];
            kl[j] = KLi[i];
            ps[j] = L0 ? i : r.PS[src][i];
        }
    }
    __syncthreads();
    const u64 lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    u16* lw = loc + w * (MT / 4) + lane;
#pragma unroll
    for (u32 j = 0; j < MPT; ++j) {
        const bool valid = q0 + j * 64 + lane < hi;
        const u32 dg = digit_of(kh[j], kl[j], lvl);
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
    for (u32 j = 0; j < MPT; ++j) {
        if (q0 + j * 64 + lane < hi) {
            const u32 o = wc[w][digit_of(kh[j], kl[j], lvl)] + lw[j * 64];
            r.KH[dst][o] = kh[j];
            r.KL[dst][o] = kl[j];
            r.PS[dst][o] = ps[j];
        }
    }
}

// ---------------------------------------------------------------------------------------
// final buckets
// ---------------------------------------------------------------------------------------
// tie groups (key bits exhausted) and singletons up to TIE_SMALL elements: one thread each;
// the elements are in position order already
__global__ __launch_bounds__(WG) void k_r0m_ties(R0M r) {
    __shared__ u32 sh[WG / 64], wtot;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 i = xcd_tile() * WG + tid;
    const u32 n = r.cnt[RC_CLS + 0];
    Fin f{0, 0, 1};
    if (i < n) f = r.fin[0][i];
    const u32 nseg = f.len >= 2 ? 1u : 0u;
    const u32 incl = wave_incl_scan(nseg, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 off = incl - nseg;
    for (u32 q = 0; q < w; ++q) off += sh[q];
    if (tid == WG - 1) {
        const u32 tot = off + nseg;
        wtot = tot ? atomicAdd(r.next_cnt, tot) : 0u;
    }
    __syncthreads();
    if (!f.len) return;
    const u32* P = r.PS[(f.lvl - 1) & 1];
    for (u32 k = 0; k < f.len; ++k) {
        const u32 p = P[f.start + k];
        r.SA[f.start + k] = p;
        r.RK[p] = f.start;
    }
    if (nseg) r.next[wtot + off] = Seg{f.start, f.len};
}

// long tie groups: one workgroup each
__global__ __launch_bounds__(WG) void k_r0m_ties_big(R0M r) {
    if (blockIdx.x >= r.cnt[RC_CLS + 1]) return;
    const Fin f = r.fin[1][blockIdx.x];
    const u32* P = r.PS[(f.lvl - 1) & 1];
    for (u32 k = threadIdx.x; k < f.len; k += WG) {
        const u32 p = P[f.start + k];
        r.SA[f.start + k] = p;
        r.RK[p] = f.start;
    }
    if (threadIdx.x == 0) r.next[atomicAdd(r.next_cnt, 1u)] = Seg{f.start, f.len};
}

// Final buckets of one size class C (len <= 2^C), T / 2^C of them per workgroup of NT = T / 8
// threads, each in a sub-array of 2^C slots padded with ~0: words (key << 8 lvl) | index
// sorted by a bitonic network (distances >= 8 through LDS, < 8 in registers; every sub-array
// ascending).  The index is the input order = position order, so equal remaining keys keep
// position order.  Then heads -> SA, RK, the next round's groups, split flags.
template <int J>
__device__ inline void bit_reg_stage(u64 (&r)[8], u32 tid, u32 k, u32 S) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (e & J) continue;
        const u32 i = 8 * tid + e;
        const bool up = (k == S) || ((i & k) == 0);
        const u64 x = r[e], y = r[e + J];
        const bool sw = (x > y) == up;
        r[e] = sw ? y : x;
        r[e + J] = sw ? x : y;
    }
}
__device__ inline u32 BKI(u32 i) { return i + (i >> 6); }  // one pad word per 64: 8-runs hit distinct banks

template <u32 C, u32 NT>
__global__ __launch_bounds__(NT) void k_r0m_bsort(R0M r) {
    constexpr u32 T = 8 * NT, S = 1u << C, SPT = T / S, NWV = NT / 64;
    constexpr u32 cls = 2 + C - CMIN;
    constexpr u64 NONEK = ~0ull;
    __shared__ u64 sk[T + T / 64];
    __shared__ Fin fs[SPT];
    __shared__ u8 sF[SPT], ssplit[SPT];
    __shared__ u32 sh[NWV], wtot;
    const u32 tid = threadIdx.x;
    const u32 first = xcd_tile() * SPT, count = r.cnt[RC_CLS + cls];
    if (first >= count) return;
    const u32 nthis = min(SPT, count - first);
    for (u32 i = tid; i < SPT; i += NT) {
        const Fin f = i < nthis ? r.fin[cls][first + i] : Fin{0, 0, 1};
        fs[i] = f;
        sF[i] = (u8)min(64u - r.kbits + 8 * f.lvl, 63u);
        ssplit[i] = 0;
    }
    __syncthreads();
#pragma unroll
    for (u32 j = 0; j < 8; ++j) {
        const u32 slot = j * NT + tid;
        const u32 si = slot >> C, k = slot & (S - 1);
        u64 wv = NONEK;
        if (si < nthis && k < fs[si].len) {
            const Fin f = fs[si];
            const u32 b = (f.lvl - 1) & 1, g = f.start + k;
            wv = ((((u64)r.KH[b][g] << 32) | r.KL[b][g]) << (8 * f.lvl)) | k;
        }
        sk[BKI(slot)] = wv;
    }
    __syncthreads();
    u64 w[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = sk[BKI(8 * tid + e)];
    for (u32 k = 2; k <= S; k <<= 1) {
        if (k > 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) sk[BKI(8 * tid + e)] = w[e];
            __syncthreads();
            for (u32 j = k >> 1; j >= 8; j >>= 1) {
                const u32 lj = 31 - __clz(j);
#pragma unroll
                for (u32 q0 = 0; q0 < 4; ++q0) {  // T / 2 compare-exchanges, 4 per thread
                    const u32 q = q0 * NT + tid;
                    const u32 i = ((q >> lj) << (lj + 1)) | (q & (j - 1));
                    const u32 l = i + j;
                    const bool up = (k == S) || ((i & k) == 0);
                    const u64 x = sk[BKI(i)], y = sk[BKI(l)];
                    if ((x > y) == up) {
                        sk[BKI(i)] = y;
                        sk[BKI(l)] = x;
                    }
                }
                __syncthreads();
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = sk[BKI(8 * tid + e)];
            __syncthreads();
        }
        if (k >= 8) bit_reg_stage<4>(w, tid, k, S);
        if (k >= 4) bit_reg_stage<2>(w, tid, k, S);
        bit_reg_stage<1>(w, tid, k, S);
    }
    // heads: slot 0 of a sub-array, or the remaining key differs from the previous slot's
    sk[BKI(8 * tid + 7)] = w[7];
    __syncthreads();
    u64 prev = tid ? sk[BKI(8 * tid - 1)] : 0;
    bool valid[8], head[8], stop[8];
    u32 agg = 0, loc[8], sagg = T;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const u32 i = 8 * tid + e, si = i >> C, kk = i & (S - 1);
        const u32 F = sF[si];
        valid[e] = si < nthis && kk < fs[si].len;
        head[e] = valid[e] && (kk == 0 || (w[e] >> F) != (prev >> F));
        stop[e] = kk == 0 || head[e] || !valid[e];
        if (head[e] && kk != 0) ssplit[si] = 1;
        prev = w[e];
        if (head[e]) agg = i;
        loc[e] = agg;
        if (stop[e] && i < sagg) sagg = i;
    }
    // run start: max-scan of head indices; run end: the next stop (reverse min-scan)
    const u32 carry = wg_scan_x<false>(agg, OpMaxU(), 0u, sh, NWV);
    const u32 scarry = wg_scan_x<true>(sagg, OpMinU(), T, sh, NWV);
    u32 nxt[8], run_min = scarry;
#pragma unroll
    for (int e = 7; e >= 0; --e) {
        nxt[e] = run_min;
        if (stop[e]) run_min = 8 * tid + e;
    }
    u32 nnew = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) nnew += (head[e] && nxt[e] - (8 * tid + e) >= 2) ? 1u : 0u;
    const u32 my_off = wg_scan_x<false>(nnew, OpAddU(), 0u, sh, NWV);
    if (tid == NT - 1) {
        const u32 tot = my_off + nnew;
        wtot = tot ? atomicAdd(r.next_cnt, tot) : 0u;
    }
    __syncthreads();
    u32 wpos = wtot + my_off;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (!valid[e]) continue;
        const u32 i = 8 * tid + e, si = i >> C, kk = i & (S - 1);
        const Fin f = fs[si];
        const u32 rs = max(loc[e], carry) - (si << C);  // run start inside the sub-array
        const u32 p = r.PS[(f.lvl - 1) & 1][f.start + (u32)(w[e] & ((1ull << sF[si]) - 1))];
        r.SA[f.start + kk] = p;
        r.RK[p] = f.start + rs;
        if (head[e]) {
            const u32 len = nxt[e] - i;
            if (len >= 2) r.next[wpos++] = Seg{f.start + kk, len};
        }
    }
    __syncthreads();
    if (tid < nthis && ssplit[tid]) r.blk_split[r.geo.block_of(fs[tid].start)] = 1;
}

// One final bucket (len <= NT * PT) per workgroup: a stable LSD radix sort in registers + LDS.
// The words (key << 8 lvl) | index stay in registers, element i = (wave, step, lane) order;
// per varying key byte: ballot-match ranking per 64-element step against the wave's own
// digit counters (a wave's LDS operations retire in order: no barrier between steps), bases
// per (digit, wave), one scatter into LDS and a reload.  Bytes that hold only index bits, or
// do not vary in the bucket, are skipped (the input order is position order).  Then the same
// epilogue as the bitonic form: heads -> SA, RK, next-round groups, split flags.
template <u32 NT, u32 PT>
__global__ __launch_bounds__(NT) void k_r0m_rsort(R0M r, u32 cls, u32 dbg) {
    constexpr u32 NWV = NT / 64, CAP = NT * PT, WSPAN = 64 * PT;
    __shared__ u64 buf[CAP];
    __shared__ u32 wc[NWV][256];
    __shared__ u32 red[NWV][2], sh[NWV], wtot, vlo, vhi, anysplit;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 fi = xcd_tile();
    if (fi >= r.cnt[RC_CLS + cls]) return;
    const Fin f = r.fin[cls][fi];
    const u32 n = f.len, s0 = f.start, bsel = (f.lvl - 1) & 1, shl = 8 * f.lvl;
    const u32 F = 64 - r.kbits + shl;
    const u32* KH = r.KH[bsel];
    const u32* KL = r.KL[bsel];
    const u64 w0 = (((u64)KH[s0] << 32) | KL[s0]) << shl;
    u64 x[PT], var = 0;
#pragma unroll
    for (u32 sp = 0; sp < PT; ++sp) {
        const u32 i = w * WSPAN + sp * 64 + lane;
        x[sp] = ~0ull;
        if (i < n) {
            const u64 k = (((u64)KH[s0 + i] << 32) | KL[s0 + i]) << shl;
            x[sp] = k | i;
            var |= k ^ w0;
        }
    }
    {
        u32 a = (u32)var, b = (u32)(var >> 32);
        for (int o = 32; o; o >>= 1) {
            a |= __shfl_xor(a, o);
            b |= __shfl_xor(b, o);
        }
        if (lane == 0) {
            red[w][0] = a;
            red[w][1] = b;
        }
    }
    if (tid == 0) anysplit = 0;
    __syncthreads();
    if (tid == 0) {
        u32 a = 0, b = 0;
        for (u32 q = 0; q < NWV; ++q) {
            a |= red[q][0];
            b |= red[q][1];
        }
        vlo = a;
        vhi = b;
    }
    __syncthreads();
    const u64 vm = ((u64)vhi << 32) | vlo;
    const u64 lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (u32 byte = F / 8; byte < 8; ++byte) {
        if (((vm >> (8 * byte)) & 255u) == 0 || (dbg & 2)) continue;  // dbg 2: timing only, no passes
        const u32 shift = 8 * byte;
#pragma unroll
        for (u32 q = 0; q < 4; ++q) wc[w][q * 64 + lane] = 0;
        u32 loc[PT];
#pragma unroll
        for (u32 sp = 0; sp < PT; ++sp) {
            const bool v = w * WSPAN + sp * 64 + lane < n;
            const u32 dg = (u32)(x[sp] >> shift) & 255u;
            u64 m = __ballot(v);
#pragma unroll
            for (u32 bit = 0; bit < 8; ++bit) {
                const u64 bal = __ballot((dg >> bit) & 1u);
                m &= ((dg >> bit) & 1u) ? bal : ~bal;
            }
            const u32 rank = __popcll(m & lt_mask);
            const u32 pre = v ? wc[w][dg] : 0u;
            loc[sp] = pre + rank;
            if (v && rank == 0) wc[w][dg] = pre + (u32)__popcll(m);
        }
        if (NWV > 1) __syncthreads();
        // bases per (digit, wave): digits ascending, waves in order
        if (NWV == 1) {
            u32 c[4], t4 = 0;
#pragma unroll
            for (u32 q = 0; q < 4; ++q) {
                c[q] = wc[0][4 * lane + q];
                t4 += c[q];
            }
            u32 ex = wave_incl_scan(t4, OpAddU(), 0u) - t4;
#pragma unroll
            for (u32 q = 0; q < 4; ++q) {
                wc[0][4 * lane + q] = ex;
                ex += c[q];
            }
        } else {
            u32 tot = 0;
            if (tid < 256)
                for (u32 q = 0; q < NWV; ++q) tot += wc[q][tid];
            const u32 ex = wg_scan_x<false>(tot, OpAddU(), 0u, sh, NWV);
            if (tid < 256) {
                u32 acc = ex;
                for (u32 q = 0; q < NWV; ++q) {
                    const u32 c = wc[q][tid];
                    wc[q][tid] = acc;
                    acc += c;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (u32 sp = 0; sp < PT; ++sp)
            if (w * WSPAN + sp * 64 + lane < n) buf[wc[w][(u32)(x[sp] >> shift) & 255u] + loc[sp]] = x[sp];
        __syncthreads();
#pragma unroll
        for (u32 sp = 0; sp < PT; ++sp) {
            const u32 i = w * WSPAN + sp * 64 + lane;
            x[sp] = i < n ? buf[i] : ~0ull;
        }
        if (NWV > 1) __syncthreads();
    }
    // epilogue: thread tid takes the sorted slots PT tid .. PT tid + PT - 1
#pragma unroll
    for (u32 sp = 0; sp < PT; ++sp) buf[w * WSPAN + sp * 64 + lane] = x[sp];
    __syncthreads();
    const u64 imask = (1ull << F) - 1;
    u64 y[PT];
    bool hd[PT];
    u32 lmax = 0, lmin = 0xFFFFFFFFu;
    u64 prev = tid ? buf[PT * tid - 1] : 0;
#pragma unroll
    for (u32 e = 0; e < PT; ++e) {
        const u32 i = PT * tid + e;
        y[e] = buf[i];
        hd[e] = i < n && (i == 0 || (y[e] >> F) != (prev >> F));
        prev = y[e];
        if (hd[e]) {
            lmax = max(lmax, i);
            lmin = min(lmin, i);
        }
    }
    const u32 carry = wg_scan_x<false>(lmax, OpMaxU(), 0u, sh, NWV);
    const u32 scarry = wg_scan_x<true>(lmin, OpMinU(), 0xFFFFFFFFu, sh, NWV);
    u32 run = carry, nh = scarry == 0xFFFFFFFFu ? n : scarry;
    bool split = false;
    const u32* PS = r.PS[bsel];
#pragma unroll
    for (u32 e = 0; e < PT; ++e) {
        const u32 i = PT * tid + e;
        if (i < n) {
            if (hd[e]) {
                run = i;
                split |= i != 0;
            }
            const u32 p = PS[s0 + (u32)(y[e] & imask)];
            r.SA[s0 + i] = p;
            if (!(dbg & 1)) r.RK[p] = s0 + run;  // dbg 1: timing only, no RK scatter
        }
    }
    u32 len[PT], nseg = 0;
#pragma unroll
    for (int e = (int)PT - 1; e >= 0; --e) {
        const u32 i = PT * tid + e;
        len[e] = 0;
        if (hd[e]) {
            len[e] = nh - i;
            nh = i;
            nseg += len[e] >= 2;
        }
    }
    const u32 off0 = wg_scan_x<false>(nseg, OpAddU(), 0u, sh, NWV);
    if (split) anysplit = 1;
    if (tid == NT - 1) {
        const u32 tot = off0 + nseg;
        wtot = tot ? atomicAdd(r.next_cnt, tot) : 0u;
    }
    __syncthreads();
    u32 off = wtot + off0;
#pragma unroll
    for (u32 e = 0; e < PT; ++e)
        if (len[e] >= 2) r.next[off++] = Seg{s0 + PT * tid + e, len[e]};
    if (tid == 0 && anysplit) r.blk_split[r.geo.block_of(s0)] = 1;
}

}  // namespace

void launch_r0_keys64(const Geom& geo, const R0Bufs& t, u32* KL, u32* KH, u32* hist, hipStream_t s, KTimer* kt);

// Buffers: level 0 reads the keys by position from t.RK (low words) / t.KP (high words);
// levels write (KH, KL, PS) to A = (K2, K22, SA2) and B = (KP, x[0], x[1]) alternately (KP is
// free once level 0 has read it); SA and RK are written by the finishing kernels only.
u32 launch_round0_msd(const Geom& geo, const R0Bufs& t, Seg* next, u32* next_cnt, u32* blk_split, R0MBufs& mb,
                      hipStream_t s, KTimer* kt, u32* h_cnt) {
    if (!geo.N) return 0;
    const u32 tpb = (geo.bs + MT - 1) / MT;
    const u32 nt0 = tpb * geo.nb;
    const u64 N = geo.N;
    R0M r{};
    r.geo = geo;
    r.tpb = tpb;
    r.kbits = t.chars * t.w;
    r.KH0 = t.KP;
    r.KL0 = t.RK;
    r.KH[0] = t.K2;
    r.KL[0] = t.K22;
    r.PS[0] = t.SA2;
    r.KH[1] = t.KP;
    r.KL[1] = mb.x0;
    r.PS[1] = mb.x1;
    r.SA = t.SA;
    r.RK = t.RK;
    r.blk_split = blk_split;
    r.next = next;
    r.next_cnt = next_cnt;
    for (u32 c = 0; c < NCLS; ++c) r.fin[c] = reinterpret_cast<Fin*>(mb.fin[c]);
    r.cnt = mb.cnt;
    r.text = t.text;
    r.FEd = t.FEd;
    r.fac = t.fac;
    r.code = t.code;
    r.C = t.chars;
    r.w = t.w;
    for (int k = 0; k < 2; ++k) {
        r.segs[k] = mb.segs[k];
        r.tiles[k] = mb.tiles[k];
    }
    KOLM_HIP_CHECK(hipMemsetAsync(mb.cnt, 0, sizeof(u32) * RC_N, s));
    // level 0 from the text (KOLM_R0M_TEXT=0: keys by position from k_keypos_r0, then loaded)
    const char* te = getenv("KOLM_R0M_TEXT");
    const bool from_text = !(te && atoi(te) == 0);
    if (from_text) {
        KScope k(kt, KT_LSD, "k_r0m_hist0", N * 2 + (u64)nt0 * 1024);  // text 1 + FEd 1
        k_r0m_hist0<<<nt0, WG, 0, s>>>(r, mb.hist);
    } else {
        launch_r0_keys64(geo, t, t.RK, t.KP, mb.hist, s, kt);
    }
    {
        KScope k(kt, KT_LSD, "k_r0m_scan<0>", (u64)nt0 * 1024 * 3);
        k_r0m_scan<1><<<geo.nb, WG, 0, s>>>(r, 0, nullptr, mb.hist);
    }
    if (from_text) {
        // text 1 + FEd 1 in, keys + position 12 out
        KScope k(kt, KT_LSD, "k_r0m_scatter0t", N * 14 + (u64)nt0 * 1024);
        k_r0m_scatter0t<<<nt0, WG, 0, s>>>(r, mb.hist);
    } else {
        KScope k(kt, KT_LSD, "k_r0m_scatter<0>", N * 20 + (u64)nt0 * 1024);  // keys 8 in, keys + position 12 out
        k_r0m_scatter<1><<<nt0, WG, 0, s>>>(r, 0, nullptr, mb.hist);
    }
    u32 levels = 1;
    for (u32 lvl = 1; lvl < 8; ++lvl) {
        KOLM_HIP_CHECK(hipMemcpyAsync(h_cnt, mb.cnt, sizeof(u32) * RC_N, hipMemcpyDeviceToHost, s));
        KOLM_HIP_CHECK(hipStreamSynchronize(s));
        const u32 nseg = h_cnt[RC_SEG + (lvl & 1)], ntl = h_cnt[RC_TILE + (lvl & 1)];
        if (!nseg) break;
        // the next level's counters start from zero (this level's are read above)
        KOLM_HIP_CHECK(hipMemsetAsync(mb.cnt + RC_SEG + ((lvl + 1) & 1), 0, sizeof(u32), s));
        KOLM_HIP_CHECK(hipMemsetAsync(mb.cnt + RC_TILE + ((lvl + 1) & 1), 0, sizeof(u32), s));
        const u32* dseg = mb.cnt + RC_SEG + (lvl & 1);
        const u32* dtile = mb.cnt + RC_TILE + (lvl & 1);
        {
            KScope k(kt, KT_LSD, "k_r0m_hist", (u64)ntl * (MT * 4 + 1024));
            k_r0m_hist<<<ntl, WG, 0, s>>>(r, lvl, dtile, mb.hist);
        }
        {
            KScope k(kt, KT_LSD, "k_r0m_scan<1>", (u64)ntl * 1024 * 3);
            k_r0m_scan<0><<<nseg, WG, 0, s>>>(r, lvl, dseg, mb.hist);
        }
        {
            KScope k(kt, KT_LSD, "k_r0m_scatter<1>", (u64)ntl * (MT * 24 + 1024));
            k_r0m_scatter<0><<<ntl, WG, 0, s>>>(r, lvl, dtile, mb.hist);
        }
        ++levels;
    }
    KOLM_HIP_CHECK(hipMemcpyAsync(h_cnt, mb.cnt, sizeof(u32) * RC_N, hipMemcpyDeviceToHost, s));
    KOLM_HIP_CHECK(hipStreamSynchronize(s));
    const u32* nc = h_cnt + RC_CLS;
    if (nc[0]) {
        KScope k(kt, KT_LSD, "k_r0m_ties", (u64)nc[0] * 12);
        k_r0m_ties<<<(nc[0] + WG - 1) / WG, WG, 0, s>>>(r);
    }
    if (nc[1]) {
        KScope k(kt, KT_LSD, "k_r0m_ties_big", (u64)nc[1] * TIE_SMALL * 12);
        k_r0m_ties_big<<<nc[1], WG, 0, s>>>(r);
    }
    // per element: key 8 in, SA 4 + RK 4 out, position 4 gathered inside the bucket
    auto bs_launch = [&](auto cval, auto ntval) {
        constexpr u32 C = decltype(cval)::value, NT = decltype(ntval)::value;
        constexpr u32 SPT = 8 * NT >> C;
        const u32 n = nc[2 + C - CMIN];
        if (!n) return;
        static const std::string nm = "k_r0m_bsort<" + std::to_string(C) + ", " + std::to_string(NT) + ">";
        KScope k(kt, KT_LSD, nm.c_str(), (u64)n * (1u << C) * 20);
        k_r0m_bsort<C, NT><<<(n + SPT - 1) / SPT, NT, 0, s>>>(r);
    };
    // one bucket per workgroup, stable radix in registers + LDS (default), or packed bitonic
    // sub-arrays (KOLM_R0M_SORT=bitonic, A/B)
    const char* se = getenv("KOLM_R0M_SORT");
    if (se && !strcmp(se, "bitonic")) {
        bs_launch(std::integral_constant<u32, 5>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 6>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 7>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 8>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 9>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 10>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 11>{}, std::integral_constant<u32, 256>{});
        bs_launch(std::integral_constant<u32, 12>{}, std::integral_constant<u32, 512>{});
        bs_launch(std::integral_constant<u32, 13>{}, std::integral_constant<u32, 1024>{});
    } else {
        const u32 dbg = getenv("KOLM_R0M_DBG") ? (u32)atoi(getenv("KOLM_R0M_DBG")) : 0u;  // timing experiments only
        auto rs_launch = [&](u32 C, auto ntval, auto ptval) {
            constexpr u32 NT = decltype(ntval)::value, PT = decltype(ptval)::value;
            const u32 n = nc[2 + C - CMIN];
            if (!n) return;
            static const std::string nm = "k_r0m_rsort<" + std::to_string(NT) + ", " + std::to_string(PT) + ">";
            KScope k(kt, KT_LSD, nm.c_str(), (u64)n * (1u << C) * 20);
            k_r0m_rsort<NT, PT><<<n, NT, 0, s>>>(r, 2 + C - CMIN, dbg);
        };
        using std::integral_constant;
        rs_launch(5, integral_constant<u32, 64>{}, integral_constant<u32, 1>{});
        rs_launch(6, integral_constant<u32, 64>{}, integral_constant<u32, 1>{});
        rs_launch(7, integral_constant<u32, 64>{}, integral_constant<u32, 4>{});
        rs_launch(8, integral_constant<u32, 64>{}, integral_constant<u32, 4>{});
        rs_launch(9, integral_constant<u32, 64>{}, integral_constant<u32, 16>{});
        rs_launch(10, integral_constant<u32, 64>{}, integral_constant<u32, 16>{});
        rs_launch(11, integral_constant<u32, 256>{}, integral_constant<u32, 16>{});
        rs_launch(12, integral_constant<u32, 256>{}, integral_constant<u32, 16>{});
        rs_launch(13, integral_constant<u32, 512>{}, integral_constant<u32, 16>{});
    }
    return levels;
}

u32 r0m_tiles(const Geom& geo) { return (geo.bs + MT - 1) / MT * geo.nb; }

// list capacities: a class-c bucket holds more than the previous class's bound (len 1 and
// tie groups up to TIE_SMALL: class 0; a non-final bucket holds more than 256 elements, since
// the LDS index bits F >= 8 at every level)
u64 r0m_fin_cap(u64 N, u32 nb, int cls) {
    // class 2 + (C - 5) holds buckets of more than 2^(C-1) elements (class 2: at least 2)
    const u64 lo = cls == 0 ? 1 : cls == 1 ? TIE_SMALL + 1 : cls == 2 ? 2 : (1ull << (cls + CMIN - 3)) + 1;
    return N / lo + nb + 16;
}
u64 r0m_seg_cap(u64 N, u32 nb) { return N / 257 + nb + 16; }
u64 r0m_tile_cap(u64 N, u32 nb, u32 bs) {
    return std::max<u64>((u64)((bs + MT - 1) / MT) * nb, N / MT + r0m_seg_cap(N, nb)) + 16;
}

}  // namespace kolm
