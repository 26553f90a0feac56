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
#include <cstdlib>
#include <string>
#include <vector>

namespace kolm {

namespace {

constexpr u32 MT = 4096;        // elements per MSD tile (one 256-thread workgroup, 16 per thread)
constexpr u32 MPT = MT / WG;
constexpr u32 NCLS = 6;         // final classes: 0 small ties / singletons, 1 big ties, 2..5 LDS sorts
constexpr u32 TIE_SMALL = 256;  // tie groups up to this length: one thread each
// LDS sort capacity per class: 2: 64, 3: 512, 4: 2048, 5: 8192 elements

// counters (zeroed per round 0): per level parity next-segment / next-tile counts, final class
// counts
enum : int { RC_SEG = 0, RC_TILE = 2, RC_CLS = 4, RC_N = 16 };

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
};

__device__ inline u32 digit_of(u32 kh, u32 kl, u32 lvl) {  // key byte `lvl` (0 = top)
    return lvl < 4 ? (kh >> (24 - 8 * lvl)) & 255u : (kl >> (56 - 8 * lvl)) & 255u;
}

// a bucket of `len` elements whose first lvl key bytes are known: final when its key bits are
// exhausted (a tie group) or it fits an LDS sort whose words hold (remaining key, index)
__device__ inline int final_class(u32 len, u32 lvl, u32 kbits) {
    if (8 * lvl >= kbits || len == 1) return len <= TIE_SMALL ? 0 : 1;
    const u32 F = 64 - kbits + 8 * lvl;  // zero bits below the remaining key in (key << 8 lvl)
    const u32 lim = F >= 13 ? 8192u : (1u << F);
    if (len > lim) return -1;
    return len <= 64 ? 2 : len <= 512 ? 3 : len <= 2048 ? 4 : 5;
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
    for (u32 i = lo + tid; i < hi; i += WG) atomicAdd(&h[w][(K[i] >> sh) & 255u], 1u);
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

// One final bucket of at most CAP elements per workgroup of NT threads: words (key << 8 lvl)
// | index sorted by a stable LSD radix over the bytes that hold remaining key bits and vary
// in this bucket (the index is the input order = position order, so equal remaining keys
// keep position order); then heads -> SA, RK, next-round groups, split flag.
template <u32 NT, u32 CAP>
__global__ __launch_bounds__(NT) void k_r0m_bsort(R0M r, u32 cls) {
    constexpr u32 NWV = NT / 64;
    constexpr u32 E = CAP / NT;  // sorted elements per thread in the epilogue
    __shared__ u64 wb[2][CAP];
    __shared__ u32 wc[NWV][256];
    __shared__ u16 loc[CAP];
    __shared__ u32 red[NWV][2], sh1[NWV], sh2[NWV], sh3[NWV];
    __shared__ u32 vlo, vhi, wbase, anysplit;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 fi = xcd_tile();
    if (fi >= r.cnt[RC_CLS + cls]) return;
    const Fin f = r.fin[cls][fi];
    const u32 n = f.len, s0 = f.start, buf = (f.lvl - 1) & 1, shl = 8 * f.lvl;
    const u32 F = 64 - r.kbits + shl;  // free low bits of the word (>= 13 or > log2 n)
    const u32* KH = r.KH[buf];
    const u32* KL = r.KL[buf];
    const u32* PS = r.PS[buf];
    // load the words; OR of (word ^ first word) = the bits that vary in this bucket
    const u64 w0 = (((u64)KH[s0] << 32) | KL[s0]) << shl;
    u64 var = 0;
    for (u32 i = tid; i < n; i += NT) {
        const u64 k = (((u64)KH[s0 + i] << 32) | KL[s0 + i]) << shl;
        wb[0][i] = k | i;
        var |= k ^ w0;
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
    // wave w's contiguous range of the bucket, in steps of 64
    const u32 per = ((n + NWV - 1) / NWV + 63) & ~63u;
    const u32 r0 = min(n, w * per), r1 = min(n, r0 + per);
    u32 cur = 0;
    for (u32 byte = F / 8; byte < 8; ++byte) {
        if (((vm >> (8 * byte)) & 255u) == 0) continue;  // constant in this bucket
        const u32 shift = 8 * byte;
        for (u32 q = lane; q < 256; q += 64) wc[w][q] = 0;
        // pass 1: offset among the wave's equal digits (the wave's LDS ops retire in order)
        for (u32 i0 = r0; i0 < r1; i0 += 64) {
            const u32 i = i0 + lane;
            const bool v = i < r1;
            const u32 dg = v ? (u32)(wb[cur][i] >> shift) & 255u : 0u;
            u64 m = __ballot(v);
#pragma unroll
            for (u32 bit = 0; bit < 8; ++bit) {
                const u64 bal = __ballot((dg >> bit) & 1u);
                m &= ((dg >> bit) & 1u) ? bal : ~bal;
            }
            const u32 rank = __popcll(m & lt_mask);
            const u32 pre = v ? wc[w][dg] : 0u;
            if (v) loc[i] = (u16)(pre + rank);
            if (v && rank == 0) wc[w][dg] = pre + (u32)__popcll(m);
        }
        __syncthreads();
        // bases per (digit, wave): digits ascending, waves in order
        if (tid < 64) {
            u32 t4[4], tt = 0;
#pragma unroll
            for (u32 k = 0; k < 4; ++k) {
                t4[k] = 0;
                for (u32 q = 0; q < NWV; ++q) t4[k] += wc[q][4 * tid + k];
                tt += t4[k];
            }
            u32 ex = wave_incl_scan(tt, OpAddU(), 0u) - tt;
#pragma unroll
            for (u32 k = 0; k < 4; ++k) {
                for (u32 q = 0; q < NWV; ++q) {
                    const u32 c = wc[q][4 * tid + k];
                    wc[q][4 * tid + k] = ex;
                    ex += c;
                }
            }
        }
        __syncthreads();
        for (u32 i = r0 + lane; i < r1; i += 64) {
            const u64 x = wb[cur][i];
            wb[cur ^ 1][wc[w][(u32)(x >> shift) & 255u] + loc[i]] = x;
        }
        __syncthreads();
        cur ^= 1;
    }
    // epilogue: thread tid holds sorted slots E tid .. E tid + E - 1
    const u64 imask = (1ull << F) - 1;
    u64 x[E];
    bool hd[E];
    u32 lmax = 0, lmin = 0xFFFFFFFFu;
    u64 prev = tid ? wb[cur][E * tid - 1] : 0;
#pragma unroll
    for (u32 e = 0; e < E; ++e) {
        const u32 i = E * tid + e;
        x[e] = i < n ? wb[cur][i] : 0;
        hd[e] = i < n && (i == 0 || (x[e] >> F) != (prev >> F));
        prev = x[e];
        if (hd[e]) {
            lmax = max(lmax, i);
            lmin = min(lmin, i);
        }
    }
    // group start entering each thread (forward exclusive max), next head after it (reverse)
    const u32 fiw = wave_incl_scan(lmax, OpMaxU(), 0u), riw = wave_incl_scan_rev(lmin, OpMinU(), 0xFFFFFFFFu);
    const u32 fex = KOLM_DPP(0u, fiw, DPP_WAVE_SHR1, 0xF), rex = KOLM_DPP(0xFFFFFFFFu, riw, DPP_WAVE_SHL1, 0xF);
    if (lane == 63) sh1[w] = fiw;
    if (lane == 0) sh2[w] = riw;
    __syncthreads();
    u32 run = fex;
    for (u32 q = 0; q < w; ++q) run = max(run, sh1[q]);
    u32 nh = rex;
    for (u32 q = w + 1; q < NWV; ++q) nh = min(nh, sh2[q]);
    if (nh == 0xFFFFFFFFu) nh = n;
    bool split = false;
#pragma unroll
    for (u32 e = 0; e < E; ++e) {
        const u32 i = E * tid + e;
        if (i < n) {
            if (hd[e]) {
                run = i;
                split |= i != 0;
            }
            const u32 p = PS[s0 + (u32)(x[e] & imask)];
            r.SA[s0 + i] = p;
            r.RK[p] = s0 + run;
        }
    }
    u32 len[E], nseg = 0;
#pragma unroll
    for (int e = (int)E - 1; e >= 0; --e) {
        const u32 i = E * tid + e;
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
    if (tid == NT - 1) {
        const u32 tot = off + nseg;
        wbase = tot ? atomicAdd(r.next_cnt, tot) : 0u;
        if (anysplit) r.blk_split[r.geo.block_of(s0)] = 1;
    }
    __syncthreads();
    off += wbase;
#pragma unroll
    for (u32 e = 0; e < E; ++e)
        if (len[e] >= 2) r.next[off++] = Seg{s0 + E * tid + e, len[e]};
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
    for (int k = 0; k < 2; ++k) {
        r.segs[k] = mb.segs[k];
        r.tiles[k] = mb.tiles[k];
    }
    KOLM_HIP_CHECK(hipMemsetAsync(mb.cnt, 0, sizeof(u32) * RC_N, s));
    launch_r0_keys64(geo, t, t.RK, t.KP, mb.hist, s, kt);
    {
        KScope k(kt, KT_LSD, "k_r0m_scan<0>", (u64)nt0 * 1024 * 3);
        k_r0m_scan<1><<<geo.nb, WG, 0, s>>>(r, 0, nullptr, mb.hist);
    }
    {
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
    // per element: key 8 + position 4 in, SA 4 + RK 4 out
    if (nc[2]) {
        KScope k(kt, KT_LSD, "k_r0m_bsort<64, 64>", (u64)nc[2] * 64 * 20);
        k_r0m_bsort<64, 64><<<nc[2], 64, 0, s>>>(r, 2);
    }
    if (nc[3]) {
        KScope k(kt, KT_LSD, "k_r0m_bsort<64, 512>", (u64)nc[3] * 512 * 20);
        k_r0m_bsort<64, 512><<<nc[3], 64, 0, s>>>(r, 3);
    }
    if (nc[4]) {
        KScope k(kt, KT_LSD, "k_r0m_bsort<256, 2048>", (u64)nc[4] * 2048 * 20);
        k_r0m_bsort<256, 2048><<<nc[4], 256, 0, s>>>(r, 4);
    }
    if (nc[5]) {
        KScope k(kt, KT_LSD, "k_r0m_bsort<512, 8192>", (u64)nc[5] * 8192 * 20);
        k_r0m_bsort<512, 8192><<<nc[5], 512, 0, s>>>(r, 5);
    }
    return levels;
}

u32 r0m_tiles(const Geom& geo) { return (geo.bs + MT - 1) / MT * geo.nb; }

// list capacities: a class-c bucket holds more than the previous class's bound (len 1 and
// tie groups up to TIE_SMALL: class 0; a non-final bucket holds more than 256 elements, since
// the LDS index bits F >= 8 at every level)
u64 r0m_fin_cap(u64 N, u32 nb, int cls) {
    static const u64 lo[NCLS] = {1, TIE_SMALL + 1, 2, 65, 513, 2049};
    return N / lo[cls] + nb + 16;
}
u64 r0m_seg_cap(u64 N, u32 nb) { return N / 257 + nb + 16; }
u64 r0m_tile_cap(u64 N, u32 nb, u32 bs) {
    return std::max<u64>((u64)((bs + MT - 1) / MT) * nb, N / MT + r0m_seg_cap(N, nb)) + 16;
}

}  // namespace kolm
