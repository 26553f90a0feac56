// LZ77 (replaces PY:1686-1763 _lz77_match_len_overlap + encode_lz77, CPP:2268-2377).
//
// Reference semantics: greedy parse; at position pos the window is the previous
// min(pos, 4096) bytes of the block; every distance d in [1, min(pos,4096)] is tried in
// ascending order and the match length is the overlapping LCP of block[pos:] and
// block[pos-d:] (unbounded); a strictly longer match wins (ties -> smallest d);
// best >= 3 emits [1][ULEB len][ULEB dist], otherwise [0][byte].
//
// GPU formulation (bit-exact), three kernels:
//   * k_lz_local: one workgroup per 4 KiB "home" of a block.  Any match >= 3 starts with
//     an equal 3-gram, so p's candidates are the earlier positions of its 3-gram inside
//     [p - 4096, p).  The workgroup copies the window [home - 4096 - lead-in, home end)
//     to LDS, buckets its positions by a 10-bit 3-gram hash with one stable counting-sort
//     pass in LDS, and parses the home with 16 speculative chains (16 lanes = 16
//     candidates at a time, nearest first; max length, ties -> nearest);
//   * k_lz_stitch_l: per block, the TRUE path over the chunk summaries: a chunk whose
//     first recorded token is the true entry is taken whole; otherwise exact tokens by a
//     brute-force window search until the true path lands on a recorded token (greedy
//     parses re-synchronise within a few tokens; the lead-in makes that happen before
//     the chunk start: 54 off-path tokens per 56 M on 256 MiB of text);
//   * k_lz_emit: one thread per token slot writes its bytes at its final offset.
#include <algorithm>
#include <cstdlib>

#include "kolm_internal.h"

namespace kolm {

namespace {

__device__ inline u32 uleb_len(u32 v) {
    u32 n = 1;
    while (v >= 128) {
        v >>= 7;
        ++n;
    }
    return n;
}

__device__ inline u32 tok_bytes(u32 len, u32 dist) { return len ? 1 + uleb_len(len) + uleb_len(dist) : 2; }

// Text accessor: an LDS copy of [lo, hi) with global memory outside it.
struct LText {
    const u8* g;
    const u8* l;
    u32 lo, hi;
    __device__ inline u8 operator[](u32 x) const { return (x - lo < hi - lo) ? l[x - lo] : g[x]; }
};

// Exact LCP(p, q) >= start, wave-cooperative (64 lanes x 4 bytes per step); maxl bounds it.
template <class T>
__device__ u32 wave_lcp(const T& t, u32 p, u32 q, u32 start, u32 maxl) {
    const u32 lane = threadIdx.x & 63;
    u32 l = start;
    for (;;) {
        u32 mism = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 o = l + j * 64 + lane;
            const bool bad = (o >= maxl) || (t[p + o] != t[q + o]);
            const u64 bal = __ballot(bad);
            if (bal && mism == 0xFFFFFFFFu) mism = l + j * 64 + (__ffsll((long long)bal) - 1);
        }
        if (mism != 0xFFFFFFFFu) return mism;
        l += 256;
    }
}

// 8 bytes at window offset x (any alignment) from three aligned LDS dwords, little-endian.
__device__ inline u64 lds8(const u8* l, u32 x) {
    const u32* w = reinterpret_cast<const u32*>(l) + (x >> 2);
    const u32 sh = x & 3;
    const u32 w0 = w[0], w1 = w[1], w2 = w[2];
    return ((u64)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// 8 bytes of the text at x (little-endian) through an LText: the LDS copy when they lie in
// it, else three aligned global dwords (bytes at or past `end` read as 0; a dword that
// starts before `end` is allocated)
__device__ inline u64 text8(const LText& t, u32 x, u32 end) {
    if (x - t.lo < t.hi - t.lo && x + 8 <= t.hi) return lds8(t.l, x - t.lo);
    if (x + 12 <= end) {
        const u32* w = reinterpret_cast<const u32*>(t.g) + (x >> 2);
        const u32 sh = x & 3;
        const u32 w0 = w[0], w1 = w[1], w2 = w[2];
        return ((u64)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    u64 v = 0;
    for (u32 k = 0; k < 8; ++k)
        if (x + k < end) v |= (u64)t[x + k] << (8 * k);
    return v;
}

// 8 bytes of global text at x (little-endian) from three aligned dwords; x + 12 <= end
__device__ inline u64 glob8(const u8* g, u32 x) {
    const u32* w = reinterpret_cast<const u32*>(g) + (x >> 2);
    const u32 sh = x & 3;
    const u32 w0 = w[0], w1 = w[1], w2 = w[2];
    return ((u64)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// wave_lcp for long extensions in the stitch (matches of periodic data run to hundreds of
// KB): 8 bytes per lane, 512 per wave step; where both sides lie in global memory well
// before `end`, four steps per round trip (loads issued unconditionally, compared after)
__device__ u32 wave_lcp8(const LText& t, u32 p, u32 q, u32 start, u32 maxl, u32 end) {
    const u32 lane = threadIdx.x & 63;
    constexpr u32 U = 4;
    u32 l = start;
    for (;;) {
        const u32 hi = max(p, q) + l + 512 * U;  // furthest byte this round trip may touch
        if (min(p, q) + l >= t.hi && hi + 12 <= end && l + 512 * U <= maxl) {
            u64 d[U];
#pragma unroll
            for (u32 s = 0; s < U; ++s) {
                const u32 o = l + 512 * s + 8 * lane;
                d[s] = glob8(t.g, p + o) ^ glob8(t.g, q + o);
            }
#pragma unroll
            for (u32 s = 0; s < U; ++s) {
                const u64 bal = __ballot(d[s] != 0);
                if (bal) {
                    const u32 j = (u32)__ffsll((long long)bal) - 1;
                    const u32 k = (u32)(__ffsll((long long)d[s]) - 1) >> 3;
                    return l + 512 * s + 8 * j + (u32)__builtin_amdgcn_readlane((int)k, (int)j);
                }
            }
            l += 512 * U;
            continue;
        }
        const u32 o = l + 8 * lane;
        u32 k = 8;  // first mismatching byte of this lane's 8 (8: none)
        if (o >= maxl) {
            k = 0;
        } else {
            const u64 d = text8(t, p + o, end) ^ text8(t, q + o, end);
            if (d) k = (u32)(__ffsll((long long)d) - 1) >> 3;
            k = min(k, maxl - o);
        }
        const u64 bal = __ballot(k < 8);
        if (bal) {
            const u32 j = (u32)__ffsll((long long)bal) - 1;
            return l + 8 * j + (u32)__builtin_amdgcn_readlane((int)k, (int)j);
        }
        l += 512;
    }
}

constexpr u32 LZL_HB = 10;
constexpr u32 LZL_NBK = 1u << LZL_HB;

// =====================================================================================
// Workgroup-local 3-gram index and speculative parse.
//
// A workgroup owns the LZL_HOME home positions [hs, he) of one block.  Every candidate of
// a home position p lies in [p - 4096, p), so the window W = [hs - 4096 - LZL_LEAD, he)
// (clipped to the block) holds them all.  The workgroup copies W's text into LDS, sorts
// W's 3-gram positions by (hash of the 3-gram, position) with one stable counting-sort pass
// in LDS (u16 window offsets; no global traffic), and keeps the slot of every home position
// (islot) and a bucket-head bitmap: p's candidates are the slots islot(p)-1, islot(p)-2, ...
// down to p's bucket start, in ascending distance, every load an LDS load.
//
// The home is parsed by 16 speculative chains (16 lanes each, 4 per wave) over 256-byte
// chunks.  A chain starts LZL_LEAD bytes before its chunk (a lead-in whose tokens are not
// recorded) so that its path has usually re-synchronised with the true greedy path by the
// chunk start.  Matches are compared (exactly, in LDS) up to LZL_CAPX bytes past the chunk
// end; a token that reaches that cap ends the chunk with its length unresolved (LZ_UNRES).
//
// k_lz_stitch_l then walks each block's true path over the chunk summaries (64 chunks
// per wave load): a chunk whose first recorded token starts at the true entry is taken
// as it is; otherwise the true path is followed token by token with an exact brute-force
// search of the 4096-byte window (LDS copy) until it lands on a recorded token; an
// unresolved last token on the path is recomputed exactly.
// =====================================================================================
// Geometry of one k_lz_local variant: HOME positions per workgroup, LPC lanes per chain (the
// candidates a chain compares per batch); 256 threads either way (4 waves, 64 / LPC chains each).
// IDX: how the workgroup gets its window's 3-gram index (LzIdx below).
template <u32 HOME, u32 LPC, u32 IDX>
struct LzlGeom {
    static constexpr u32 NW = HOME + LZ_WINDOW + (IDX ? 0u : (u32)LZL_LEAD);  // window positions indexed
    static constexpr u32 TXT = NW + LZL_CAPX + 32;          // text window + alignment + compare slack
    static constexpr u32 ISL = HOME + LZL_LEAD;             // islot entries [hs - LEAD, he)
    static constexpr u32 NCHAIN = HOME / LZL_CHUNK;
    static constexpr u32 CPW = 64 / LPC;                    // chains per wave
    static constexpr u32 NWV = NCHAIN / CPW;                // waves per workgroup
    static constexpr u32 NT = 64 * NWV;                     // threads per workgroup
    static constexpr u32 PER = (NW + NT - 1) / NT;          // window elements per lane in the sort
    static constexpr u32 PER2 = (ISL + NT - 1) / NT;        // islot positions per lane (tile index)
    static constexpr u32 cmax(u32 a, u32 b) { return a > b ? a : b; }
    // B: islot (u16 slots in form 0, u8 ranks in form 2) and, before it, the sort's histograms
    // (form 0) or the two tiles' bucket counts (form 2)
    static constexpr u32 BBYTES = IDX == 0 ? cmax(2 * ISL, NWV * LZL_NBK * 2) : cmax(ISL, 2 * 2 * LZL_NBK);
    static constexpr u32 CST = IDX == 2 ? LZL_NBK + 8 : 1;  // form 2: bucket starts, kept for the parse
    static_assert(NCHAIN % CPW == 0, "whole waves of 64 / LPC chains");
    static_assert(NW < (1u << 14), "window offsets in 14 bits (the winner key)");
    static_assert(IDX == 0 || NT * 4 == LZL_NBK, "tile-index forms: 4 buckets per thread in the start scan");
};

// LDS text without bounds checks (every access is inside the loaded window by construction)
struct WinText {
    const u8* l;
    u32 tlo;
    __device__ inline u8 operator[](u32 x) const { return l[x - tlo]; }
};

// LZL_HB-bit hash of the 3-gram at window offset x: the LDS index buckets the window's
// positions by hash (ascending position inside a bucket); a candidate whose 3-gram differs
// is rejected by the first byte compare, so other 3-grams sharing the bucket only cost
// lanes (about 4096 / 2^LZL_HB of them per token).
__device__ inline u32 hash3(const u8* t, u32 x) {
    const u32 k = ((u32)t[x] << 16) | ((u32)t[x + 1] << 8) | t[x + 2];
    return (k * 0x9E3779B1u) >> (32 - LZL_HB);
}


// Stable counting sort of the nw window positions by hash into A (one pass).  Wave w owns
// the contiguous position range [w*Q, (w+1)*Q): per-wave bucket counts (LDS atomics),
// bucket-major / wave-minor offsets, then each wave places its positions 64 at a time in
// order (ballot match-any ranking over the LZL_HB hash bits; the leader advances the
// wave's bucket offset — a wave's LDS operations retire in program order, so no barrier
// is needed between its steps).
// hist: [4][LZL_NBK] 16-bit counters / offsets (window positions < 2^16; a count is added
// to its dword with the half's shift, plain 16-bit stores otherwise)
template <u32 PER, u32 NWV = 4>
__device__ void lzl_bucket(const u8* t, u16* A, u32 nw, u16* hist, u32* sh) {
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr u32 NT = 64 * NWV;
    constexpr u32 R = (LZL_NBK + NT - 1) / NT;  // buckets per thread in the scan
    const u32 Q = (nw + NWV - 1) / NWV;
    const u32 b0 = min(w * Q, nw), b1 = min(b0 + Q, nw);
    u32 hv[PER];
#pragma unroll
    for (u32 k = 0; k < PER; ++k) {
        const u32 e = b0 + k * 64 + lane;
        hv[k] = e < b1 ? hash3(t, e) : 0u;
    }
    for (u32 i = tid; i < NWV * LZL_NBK / 2; i += NT) reinterpret_cast<u32*>(hist)[i] = 0;
    __syncthreads();
#pragma unroll
    for (u32 k = 0; k < PER; ++k)
        if (b0 + k * 64 + lane < b1)
            atomicAdd(reinterpret_cast<u32*>(hist) + ((w * LZL_NBK + hv[k]) >> 1), 1u << (16 * (hv[k] & 1)));
    __syncthreads();
    {
        u32 h[NWV][R], tot = 0;
#pragma unroll
        for (u32 r = 0; r < R; ++r)
#pragma unroll
            for (u32 q = 0; q < NWV; ++q) {
                h[q][r] = tid * R + r < LZL_NBK ? hist[q * LZL_NBK + tid * R + r] : 0u;
                tot += h[q][r];
            }
        const u32 incl = wave_incl_scan(tot, OpAddU(), 0u);
        if (lane == 63) sh[w] = incl;
        __syncthreads();
        u32 ex = incl - tot;
        for (u32 i = 0; i < w; ++i) ex += sh[i];
#pragma unroll
        for (u32 r = 0; r < R; ++r)
#pragma unroll
            for (u32 q = 0; q < NWV; ++q) {
                if (tid * R + r < LZL_NBK) hist[q * LZL_NBK + tid * R + r] = (u16)ex;
                ex += h[q][r];
            }
    }
    __syncthreads();
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
    for (u32 k = 0; k < PER; ++k) {
        if (b0 + k * 64 >= b1) break;  // wave-uniform
        const u32 e = b0 + k * 64 + lane;
        const bool valid = e < b1;
        const u32 dg = hv[k];
        u64 m = __ballot(valid);
#pragma unroll
        for (u32 bit = 0; bit < LZL_HB; ++bit) {
            const u64 bal = __ballot((dg >> bit) & 1u);
            m &= ((dg >> bit) & 1u) ? bal : ~bal;
        }
        const u32 rank = (u32)__popcll(m & lt);
        const u32 o = valid ? hist[w * LZL_NBK + dg] : 0u;
        if (valid) A[o + rank] = (u16)e;
        if (valid && rank == 0) hist[w * LZL_NBK + dg] = (u16)(o + (u32)__popcll(m));
    }
    __syncthreads();
}

// The window's index from a per-tile one (form 2 of k_lz_local).  Every position of a
// block is ranked once, inside its 4 KiB tile, instead of once in each of the two windows that
// hold it: k_lz_tiles (one workgroup per tile, the stable counting-sort pass of lzl_bucket over
// the tile alone) writes rank[x], x's rank among the tile's positions of the same hash in
// position order, and the tile's 1024 bucket counts.  A home's window is its own tile t and
// tile t - 1, whose bucket lists concatenated per hash (t - 1 first) are the window's bucket
// lists in position order, so x's slot in the window index is
//     start(h) + rank[x]                 (x in tile t - 1)
//     start(h) + cnt_{t-1}(h) + rank[x]  (x in tile t)
// with start(h) the exclusive scan of cnt_{t-1} + cnt_t: the workgroup places every window
// position with one coalesced load and one LDS store, no ranking.  (The lead-in positions of
// the home's first chain lie in tile t - 1; their own candidates before hs - 4096 are left out,
// which a lead-in may do: the stitch checks where it lands.)
__global__ __launch_bounds__(256) void k_lz_tiles(LzArgs z, u32 hpb) {
    constexpr u32 NT = 256, NWV = 4, PER = LZL_HOME / NT;
    __shared__ __align__(16) u8 txt[LZL_HOME + 16];
    __shared__ __align__(16) u16 hist[NWV * LZL_NBK];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 b = blockIdx.x / hpb, h = blockIdx.x - b * hpb;
    const u32 base = z.geo.base(b), end = z.geo.end(b);
    const u32 ts = base + h * LZL_HOME;
    if (ts >= end) return;
    const u32 te = min(ts + (u32)LZL_HOME, end);
    const u32 lim3 = end - base >= 3 ? end - 2 : base;
    const u32 top = min(te, lim3);
    const u32 n = top > ts ? top - ts : 0u;
    const u32 tlo = ts & ~3u, thi = min(end, te + 2);
    if (((uintptr_t)z.text & 3) == 0) {
        const u32* src = reinterpret_cast<const u32*>(z.text + tlo);
        u32* dst = reinterpret_cast<u32*>(txt);
        const u32 nd = (thi - tlo) / 4;
        for (u32 i = tid; i < nd; i += NT) dst[i] = src[i];
        if (tid < ((thi - tlo) & 3u)) txt[4 * nd + tid] = z.text[tlo + 4 * nd + tid];
    } else {
        for (u32 i = tid; i < thi - tlo; i += NT) txt[i] = z.text[tlo + i];
    }
    for (u32 i = tid; i < NWV * LZL_NBK / 2; i += NT) reinterpret_cast<u32*>(hist)[i] = 0;
    __syncthreads();
    const u8* tt = txt + (ts - tlo);
    const u32 Q = (n + NWV - 1) / NWV;
    const u32 b0 = min(w * Q, n), b1 = min(b0 + Q, n);
    u32 hv[PER];
#pragma unroll
    for (u32 k = 0; k < PER; ++k) {
        const u32 e = min(b0 + k * 64 + lane, LZL_HOME - 1);
        hv[k] = hash3(tt, e);
    }
#pragma unroll
    for (u32 k = 0; k < PER; ++k)
        if (b0 + k * 64 + lane < b1)
            atomicAdd(reinterpret_cast<u32*>(hist) + ((w * LZL_NBK + hv[k]) >> 1), 1u << (16 * (hv[k] & 1)));
    __syncthreads();
    // per bucket: the waves' exclusive offsets (wave order = position order) and the tile's count
    for (u32 d = tid; d < LZL_NBK; d += NT) {
        u32 run = 0;
#pragma unroll
        for (u32 q = 0; q < NWV; ++q) {
            const u32 cq = hist[q * LZL_NBK + d];
            hist[q * LZL_NBK + d] = (u16)run;
            run += cq;
        }
        z.tcnt[(u64)blockIdx.x * LZL_NBK + d] = (u16)run;
    }
    __syncthreads();
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
    for (u32 k = 0; k < PER; ++k) {
        if (b0 + k * 64 >= b1) break;  // wave-uniform
        const u32 e = b0 + k * 64 + lane;
        const bool valid = e < b1;
        const u32 dg = hv[k];
        u64 m = __ballot(valid);
#pragma unroll
        for (u32 bit = 0; bit < LZL_HB; ++bit) {
            const u64 bal = __ballot((dg >> bit) & 1u);
            m &= ((dg >> bit) & 1u) ? bal : ~bal;
        }
        const u32 rank = (u32)__popcll(m & lt);
        const u32 o = valid ? hist[w * LZL_NBK + dg] : 0u;
        if (valid) z.rank[ts + e] = (u16)(o + rank);
        if (valid && rank == 0) hist[w * LZL_NBK + dg] = (u16)(o + (u32)__popcll(m));
    }
}

// the lanes of this lane's chain (LPC consecutive lanes)
template <u32 LPC>
__device__ inline u64 grp_mask(u32 lane) { return ((1ull << LPC) - 1ull) << (lane & (64 - LPC)); }

// max over the LPC (16 or 8) lanes of this lane's chain, in every lane of it: quad butterflies,
// then row rotates (16) or the half-row mirror (8)
template <u32 LPC>
__device__ inline u32 grp_max(u32 v) {
    static_assert(LPC == 16 || LPC == 8, "chains of 16 or 8 lanes");
    v = max(v, KOLM_DPP(0u, v, 0xB1, 0xF));   // quad_perm [1,0,3,2]
    v = max(v, KOLM_DPP(0u, v, 0x4E, 0xF));   // quad_perm [2,3,0,1]
    if (LPC == 16) {
        v = max(v, KOLM_DPP(0u, v, 0x124, 0xF));  // row_ror:4
        v = max(v, KOLM_DPP(0u, v, 0x128, 0xF));  // row_ror:8
    } else {
        v = max(v, KOLM_DPP(0u, v, 0x141, 0xF));  // row_half_mirror
    }
    return v;
}

// ULEB128 byte count of v (PY:111-124), branch-free
__device__ inline u32 uleb_n(u32 v) {
    return 1u + (v >= (1u << 7)) + (v >= (1u << 14)) + (v >= (1u << 21)) + (v >= (1u << 28));
}

// =====================================================================================
// k_lz_local's chains advance independently (round 6).  Before, the four chains of a wave
// stepped their tokens together: a token step lasts as many candidate batches as the chain with the most
// candidates needs (2.4 batches per step against 1.5 per token on text), and every step
// pays the token setup once more.  Here one loop trip runs one candidate batch for every
// chain with a token in progress, then finishes the tokens whose walk ended in that batch
// and sets up those chains' next tokens, so a chain never waits for another chain's
// candidates.  The bucket heads are flags in the index itself (bit 15 of A: the first slot
// of a hash bucket), so a walk ends at the first flagged slot or at the first candidate
// out of the 4096-byte window, with no bitmap scan per token.
// =====================================================================================
constexpr u32 LZC_HEAD = 0x8000u;   // A[slot] flag: first slot of its hash bucket

// Window index forms (IDX): 0 = the workgroup sorts its whole window in LDS (lzl_bucket);
// 2 = placed from the tile index (k_lz_tiles), islot as u8 ranks inside the bucket plus the
// window's bucket starts (31 KB of LDS instead of 33: five workgroups per CU); a rank of 255 or
// more is found by a binary search of the bucket.  (Form 1, the tile index with u16 islot slots at
// four workgroups per CU, measured between the two and was removed.)
template <u32 HOME, u32 LPC, u32 IDX>
__global__ __launch_bounds__(64 * (HOME / LZL_CHUNK) / (64 / LPC)) void k_lz_local(LzArgs z, u32 hpb, u32 lead) {
    using G = LzlGeom<HOME, LPC, IDX>;
    __shared__ __align__(16) u8 txt[G::TXT];
    __shared__ __align__(16) u16 A[G::NW];
    constexpr u32 NT = G::NT;
    // islot of [ilo, he); before it the sort's histograms (form 0) or the tiles' counts (1, 2)
    __shared__ __align__(16) u8 B[G::BBYTES];
    __shared__ __align__(16) u16 cst[G::CST];
    __shared__ u32 sh[G::NWV];
    u16* hist = reinterpret_cast<u16*>(B);

    static_assert(G::NW <= 0x3FFFu + 1u, "window offsets below the head flag");
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 b = blockIdx.x / hpb, h = blockIdx.x - b * hpb;
    const u32 base = z.geo.base(b), end = z.geo.end(b);
    const u32 hs = base + h * HOME;
    if (hs >= end) return;
    const u32 he = min(hs + HOME, end);
    constexpr u32 WSPAN = IDX ? (u32)LZ_WINDOW : (u32)(LZ_WINDOW + LZL_LEAD);
    const u32 lo = hs - base >= WSPAN ? hs - WSPAN : base;
    const u32 ilo = hs - base > (u32)LZL_LEAD ? hs - LZL_LEAD : base;
    const u32 hi = min(end, he + (u32)LZL_CAPX);
    const u32 tlo = lo & ~3u;
    u64 t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    if (z.prof) t0 = wall_clock64();
    {
        const u32 n = hi - tlo;
        if (((uintptr_t)z.text & 3) == 0) {
            const u32* src = reinterpret_cast<const u32*>(z.text + tlo);
            u32* dst = reinterpret_cast<u32*>(txt);
            for (u32 i = tid; i < n / 4; i += NT) dst[i] = src[i];
            for (u32 i = (n & ~3u) + tid; i < n; i += NT) txt[i] = z.text[tlo + i];
        } else {
            for (u32 i = tid; i < n; i += NT) txt[i] = z.text[tlo + i];
        }
    }
    const u32 lim3 = end - base >= 3 ? end - 2 : base;
    const u32 top = min(he, lim3);
    const u32 nw = top > lo ? top - lo : 0u;
    const u8* tw = txt + (lo - tlo);
    u16* isl = reinterpret_cast<u16*>(B);  // forms 0, 1
    u8* r8 = B;                            // form 2
    if constexpr (IDX == 0) {
        __syncthreads();
        if (z.prof) t1 = wall_clock64();
        if (nw) {
            lzl_bucket<G::PER, G::NWV>(tw, A, nw, hist, sh);
            // flag the first slot of every non-empty bucket (the last wave's offsets are the bucket ends)
            for (u32 d = tid; d < LZL_NBK; d += NT) {
                const u32 e = hist[(G::NWV - 1) * LZL_NBK + d], st = d ? hist[(G::NWV - 1) * LZL_NBK + d - 1] : 0u;
                if (e > st) A[st] = (u16)(A[st] | LZC_HEAD);
            }
            __syncthreads();  // the islot writes below overwrite the histograms
        }
        for (u32 j = tid; j < nw; j += NT) {
            const u32 x = A[j] & 0x7FFFu;
            if (lo + x >= ilo) isl[lo + x - ilo] = (u16)j;
        }
        if (z.prof) t2 = wall_clock64();
    } else {
        // the two tiles' bucket counts (tile t - 1 absent for a block's first home)
        u16* c0 = reinterpret_cast<u16*>(B);
        u16* c1 = c0 + LZL_NBK;
        u16* cs = cst;
        {
            const u32* s1 = reinterpret_cast<const u32*>(z.tcnt + (u64)blockIdx.x * LZL_NBK);
            const u32* s0 = s1 - LZL_NBK / 2;
            for (u32 i = tid; i < LZL_NBK / 2; i += NT) {
                reinterpret_cast<u32*>(c1)[i] = s1[i];
                reinterpret_cast<u32*>(c0)[i] = h ? s0[i] : 0u;
            }
        }
        __syncthreads();
        if (z.prof) t1 = wall_clock64();
        {
            // window bucket starts: exclusive scan of cnt_{t-1} + cnt_t, 4 buckets per thread
            u32 v[4], tot = 0;
#pragma unroll
            for (u32 i = 0; i < 4; ++i) {
                v[i] = (u32)c0[4 * tid + i] + c1[4 * tid + i];
                tot += v[i];
            }
            const u32 incl = wave_incl_scan(tot, OpAddU(), 0u);
            if (lane == 63) sh[w] = incl;
            __syncthreads();
            u32 ex = incl - tot;
            for (u32 i = 0; i < w; ++i) ex += sh[i];
#pragma unroll
            for (u32 i = 0; i < 4; ++i) {
                cs[4 * tid + i] = (u16)ex;
                ex += v[i];
            }
            if (tid == NT - 1) cs[LZL_NBK] = (u16)ex;
        }
        __syncthreads();
        // tile t - 1's positions below the islot range: slot = start(h) + rank
        const u32 p1 = min(ilo, top);
        for (u32 x0 = lo; x0 < p1; x0 += NT * 4) {
            u32 r[4];
#pragma unroll
            for (u32 i = 0; i < 4; ++i) {
                const u32 x = x0 + i * NT + tid;
                r[i] = x < p1 ? (u32)z.rank[x] : 0u;
            }
#pragma unroll
            for (u32 i = 0; i < 4; ++i) {
                const u32 x = x0 + i * NT + tid;
                if (x < p1) A[cs[hash3(tw, x - lo)] + r[i]] = (u16)((x - lo) | (r[i] ? 0u : LZC_HEAD));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // [ilo, top): the lead-in (tile t - 1) and the home (tile t, after tile t - 1's entries);
        // the islot values wait in registers (packed) until the counts are no longer read
        constexpr u32 KB = 4;  // u8 ranks per keep word
        u32 keep[(G::PER2 + KB - 1) / KB] = {};
#pragma unroll
        for (u32 i0 = 0; i0 < G::PER2; i0 += 4) {
            u32 r[4];
#pragma unroll
            for (u32 i = i0; i < i0 + 4 && i < G::PER2; ++i) {
                const u32 x = ilo + i * NT + tid;
                r[i - i0] = x < top ? (u32)z.rank[x] : 0u;
            }
#pragma unroll
            for (u32 i = i0; i < i0 + 4 && i < G::PER2; ++i) {
                const u32 x = ilo + i * NT + tid;
                if (x < top) {
                    const u32 hh = hash3(tw, x - lo);
                    const u32 rr = r[i - i0] + (x >= hs ? (u32)c0[hh] : 0u);
                    A[cs[hh] + rr] = (u16)((x - lo) | (rr ? 0u : LZC_HEAD));
                    keep[i / KB] |= min(rr, 255u) << ((32 / KB) * (i % KB));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (z.prof) t2 = wall_clock64();
        __syncthreads();  // islot overwrites the counts
#pragma unroll
        for (u32 i = 0; i < G::PER2; ++i) {
            const u32 x = ilo + i * NT + tid;
            const u32 v = (keep[i / KB] >> ((32 / KB) * (i % KB))) & 0xFFu;
            if (x < top) {
                r8[x - ilo] = (u8)v;
            }
        }
    }
    __syncthreads();
    if (z.prof) t3 = wall_clock64();

    const u32 hl = lane & (LPC - 1);
    const u64 GM = grp_mask<LPC>(lane);
    const u32 gb = lane & (64 - LPC);                     // the chain's first lane
    const u64 below = ((1ull << hl) - 1ull) << gb;        // lanes of the chain before this one
    const u32 cid = w * G::CPW + lane / LPC;
    const u32 s = hs + cid * LZL_CHUNK;
    const bool has = s < end;
    const u32 e = has ? min(s + (u32)LZL_CHUNK, end) : 0u;
    const u32 c = b * z.cpb + h * G::NCHAIN + cid;
    const u32 lend = has ? min(end, e + (u32)LZL_CAPX) : 0u;
    const WinText T{txt, tlo};
    u32 p = has ? ((cid == 0 && hs == base) ? s : s - lead) : 0u;
    bool alive = has && p < e;
    u32 k = 0, qa = 0, best = 0, bd = 0, lim = 0, capl = 0;
    bool qok = false;  // qa holds the entry of this lane's slot (false: below slot 0)
    u64 pv = 0, pv1 = 0;  // p's first 16 bytes
    u32 ntok = 0, off = 0, nlong = 0, nbuf = 0, nbatch = 0;
    u32 bpos = 0, blen = 0, bdist = 0, boff = 0;
    bool un = false;
    // a token's setup: p's slot in the index, its first 8 bytes and the first batch's entry
    auto setup = [&]() {
        best = 0;
        bd = 0;
        lim = lend - p;
        capl = min((u32)LZ_CAP, lim);
        pv = lds8(txt, p - tlo);
        pv1 = lds8(txt, p - tlo + 8);
        if constexpr (IDX == 0) {
            k = p + (u32)LZ_MIN <= end ? (u32)isl[p - ilo] : 0u;
        } else if (p + (u32)LZ_MIN <= end) {
            const u32 hh = (__builtin_bswap32((u32)pv) >> 8) * 0x9E3779B1u >> (32 - LZL_HB);
            const u32 rr = r8[p - ilo];
            k = (u32)cst[hh] + rr;
            if (rr == 255u) {  // rank >= 255: binary search of the bucket for p's own slot
                u32 a0 = k, a1 = cst[hh + 1];
                const u32 tx = p - lo;
                while (a0 < a1) {
                    const u32 m = (a0 + a1) >> 1;
                    if ((A[m] & 0x3FFFu) < tx) a0 = m + 1; else a1 = m;
                }
                k = a0;
            }
        } else {
            k = 0;
        }
        qok = k > hl;
        qa = A[qok ? k - 1 - hl : 0u];
    };
    if (alive) setup();
    while (__ballot(alive)) {
        ++nbatch;
        // one candidate batch per chain: slot k-1-hl (ascending distance); the walk stops at the
        // bucket's first slot (flagged, itself a candidate) or before the first slot out of the
        // window (or below slot 0)
        const u32 q = lo + (qa & 0x3FFFu);
        const u32 qr = q - tlo;
        // the candidate's first 16 bytes, loaded for every lane (an entry past the walk's end
        // still lies in the window): one LDS round trip decides almost every candidate (on text
        // 13 % of the same-3-gram candidates share 8 bytes with p, ~0.3 % share 16)
        const u32* cw = reinterpret_cast<const u32*>(txt) + (qr >> 2);
        const u32 c0 = cw[0], c1 = cw[1], c2 = cw[2], c3 = cw[3], c4 = cw[4];
        // the next batch's entries, in the same LDS round trip (loaded unconditionally from a
        // clamped slot: no branch splits the loads)
        const bool qnok = k > LPC + hl;
        const u32 qn = A[qnok ? k - LPC - 1 - hl : 0u];
        const u32 sh = qr & 3;
        const u64 cv = ((u64)__builtin_amdgcn_alignbyte(c2, c1, sh) << 32) | __builtin_amdgcn_alignbyte(c1, c0, sh);
        const u64 cv1 = ((u64)__builtin_amdgcn_alignbyte(c4, c3, sh) << 32) | __builtin_amdgcn_alignbyte(c3, c2, sh);
        const bool bad = !qok || p - q > (u32)LZ_WINDOW;
        const u64 sm = __ballot(alive && (bad || (qa & LZC_HEAD))) & GM;
        const bool valid = alive && !bad && !(sm & below);
        const u64 d0 = pv ^ cv, d1 = pv1 ^ cv1;
        // the same 3-gram (not only the same hash): length from the first differing byte of 16
        u32 l = (valid && (d0 & 0xFFFFFFull) == 0)
                    ? (d0 ? (u32)(__ffsll((long long)d0) - 1) >> 3
                          : d1 ? 8u + ((u32)(__ffsll((long long)d1) - 1) >> 3) : 16u)
                    : 0u;
        if (l == 16 && capl > 16 && (best < 16 || (best < lim && T[p + best] == T[q + best]))) {
            // 16 equal bytes (rare): a strictly longer match must also match at `best`
            const u32 pr = p - tlo;
#pragma unroll
            for (int kk = 2; kk < LZ_CAP / 8; ++kk) {
                if (l >= capl) break;
                const u64 d = lds8(txt, pr + 8 * kk) ^ lds8(txt, qr + 8 * kk);
                if (d) {
                    l += (u32)(__ffsll((long long)d) - 1) >> 3;
                    break;
                }
                l += 8;
            }
        }
        l = min(l, capl);
        u64 longm = __ballot(valid && l >= capl && capl < lim);
        while (longm) {
            const u32 j = (u32)__ffsll((long long)longm) - 1;
            const u32 pj = __builtin_amdgcn_readlane(p, j), qj = __builtin_amdgcn_readlane(q, j);
            const u32 cj = __builtin_amdgcn_readlane(capl, j), mj = __builtin_amdgcn_readlane(lim, j);
            const u32 lj = wave_lcp(T, pj, qj, cj, mj);
            if (lane == j) l = lj;
            longm &= longm - 1;
            ++nlong;
        }
        const u32 key = grp_max<LPC>(valid && l >= (u32)LZ_MIN ? (l << 14) | (q - lo) : 0u);
        if ((key >> 14) > best) {
            best = key >> 14;
            bd = p - (lo + (key & 0x3FFFu));
        }
        qa = qn;
        qok = qnok;
        k = k > LPC ? k - LPC : 0u;
        // (round 6: lead-in tokens cut after their first candidate batch left 100x more chunks off
        // the true path — the stitch's serial fix-ups took the LZ77 stream 31 -> 51 ms per step)
        const bool fin = alive && (sm != 0 || best >= lim);
        if (__ballot(fin)) {
            if (fin) {
                const u32 len = best >= (u32)LZ_MIN ? best : 0u;
                const u32 dist = len ? bd : 0u;
                un = un || (len && best >= lim && lim < end - p);
                if (p >= s) {
                    if (hl == nbuf) {
                        bpos = p;
                        blen = len;
                        bdist = dist;
                        boff = off;
                    }
                    if (++nbuf == LPC) {
                        const u32 slot = s + ntok + 1 - LPC + hl;
                        z.tok_pos[slot] = bpos;
                        z.tok_len[slot] = blen;
                        z.tok_dist[slot] = bdist;
                        z.tok_off[slot] = boff;
                        nbuf = 0;
                    }
                    ++ntok;
                    off += len ? 1u + uleb_n(len) + uleb_n(dist) : 2u;
                }
                p += len ? len : 1u;
                alive = p < e;
                if (alive) setup();  // the next token's loads issue before the loop turns
            }
        }
    }
    if (has && hl < nbuf) {
        const u32 slot = s + ntok - nbuf + hl;
        z.tok_pos[slot] = bpos;
        z.tok_len[slot] = blen;
        z.tok_dist[slot] = bdist;
        z.tok_off[slot] = boff;
    }
    if (has && hl == 0) {
        z.c_ntok[c] = ntok;
        z.c_exit[c] = p | (un ? LZ_UNRES : 0u);
        z.c_bytes[c] = off;
    }
    nlong = wave_reduce(nlong, OpAddU(), 0u);
    if (lane == 0 && nlong) atomicAdd(z.nlong, nlong);
    if (z.prof) {
        if (lane == 0) {
            atomicAdd(z.prof + 4, (u64)nbatch);
            atomicAdd(z.prof + 5, (u64)nbatch);
        }
        __syncthreads();
        if (tid == 0) {
            const u64 t4 = wall_clock64();
            atomicAdd(z.prof + 0, t1 - t0);
            atomicAdd(z.prof + 1, t2 - t1);
            atomicAdd(z.prof + 2, t3 - t2);
            atomicAdd(z.prof + 3, t4 - t3);
            atomicAdd(z.prof + 6, (u64)1);
        }
    }
}

// Exact longest match at q (PY:1686-1708 semantics: ascending distance, strictly longer
// wins, unbounded length) by brute force over the window, from an LDS copy of the text
// [wlo, whi) refreshed when q's window is not inside it.  One wave.
constexpr u32 BF_WIN = LZ_WINDOW + 1024;
// batches of few blocks (BASELINE config 5): a 62 KiB window, so the re-searches of periodic
// data — candidate checks at q + best and the samples below best, best ~2 KB on the checker
// BMP — read LDS instead of global memory (one stitch wave per block, nothing else to share
// the CU with)
// (62 KiB: with the fingerprint array beside it, a 64 KiB window makes this ROCm's gfx950
// backend emit an invalid V_CMP on src_shared_base — "Operand has incorrect register class")
constexpr u32 BF_WIN_BIG = 62 * 1024;

// Fingerprint filter of the big-window searches.  A distance can only beat `best` if its
// match covers [q, q + best]; the sampled byte checks below let through thousands of
// candidates of periodic text (the checker BMP: runs of 48 equal bytes, period 96) that
// match for hundreds of bytes and then fail, each one extended by the wave.  With prefix
// fingerprints H(i) = sum_{hlo <= j < i} t[j] B^(j - hlo) (mod 2^64, B odd) over
// [q - dmax, q + dmax] in LDS, (H(x + L) - H(x)) B^(q - x) == H(q + L) - H(q) is necessary
// for t[x, x + L) == t[q, q + L): a candidate that fails it is rejected exactly, one that
// passes is still extended byte-exactly, so a collision costs time, never the result.
constexpr u32 HF_N = 2 * LZ_WINDOW + 1;  // H(hlo .. hlo + 2 * dmax)
constexpr u64 HF_B = 0x9E3779B97F4A7C15ull;

__device__ inline u64 hf_pow(u64 b, u32 e) {
    u64 r = 1;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}

// hh[k] = H(hlo + k) for k in [0, n]; one wave: per-lane partial sums over contiguous
// ranges, an exclusive scan of the scaled partials, then the prefix values.
__device__ void hf_build(const LText& t, u64* hh, u32 hlo, u32 n) {
    const u32 lane = threadIdx.x & 63;
    const u32 per = (n + 63) / 64;
    const u32 k0 = min(n, lane * per), k1 = min(n, k0 + per);
    u64 sum = 0;
    for (u32 k = k1; k > k0; --k) sum = sum * HF_B + t[hlo + k - 1];  // Horner
    const u64 w = hf_pow(HF_B, k0);
    u64 g = sum * w;  // lane's contribution to H, scaled to hlo
    // exclusive scan over the wave
    u64 inc = g;
    for (u32 o = 1; o < 64; o <<= 1) {
        const u64 v = __shfl_up(inc, o);
        if (lane >= o) inc += v;
    }
    u64 h = inc - g, pw = w;
    for (u32 k = k0; k < k1; ++k) {
        hh[k] = h;
        h += (u64)t[hlo + k] * pw;
        pw *= HF_B;
    }
    if (k1 == n && k0 < k1) hh[n] = h;
    if (n == 0 && lane == 0) hh[0] = 0;
    __syncthreads();
}

// d0s > 0 (an unresolved token of k_lz_local): every distance below d0s matches fewer than
// l0s bytes and d0s at least l0s (the local parse's capped answer), so the search starts
// from d0s's exact length and only tries the distances past it.
template <u32 WIN>
__device__ void bf_match(const LzArgs& z, u8* win, u32& wlo, u32& whi, u32 q, u32 base, u32 end, u32& out_len,
                         u32& out_dist, u32& nlong, u32 d0s = 0, u32 l0s = 0) {
    constexpr bool HF = WIN > BF_WIN;  // fingerprint filter
    __shared__ u64 hh[HF ? HF_N + 1 : 1];
    const u32 lane = threadIdx.x & 63;
    out_len = 0;
    out_dist = 0;
    if (q + (u32)LZ_MIN > end) return;
    const u32 dmax = min(q - base, (u32)LZ_WINDOW);
    if (!dmax) return;
    const u32 need = q - dmax;
    if (!(wlo <= need && wlo <= whi && (q + 256 <= whi || whi == end))) {
        const u64 tr0 = z.prof ? wall_clock64() : 0;
        wlo = need;
        const u32 tlo = need & ~3u;
        whi = min(end, tlo + WIN);
        const u32 n = whi - tlo;
        __syncthreads();
        if (((uintptr_t)z.text & 15) == 0 && WIN > BF_WIN) {  // 16-byte copies (tlo is 4-aligned)
            const u32 h = (16 - (tlo & 15)) & 15;  // bytes before the first 16-byte source boundary
            for (u32 i = lane; i < min(h, n); i += 64) win[i] = z.text[tlo + i];
            const uint4* src = reinterpret_cast<const uint4*>(z.text + tlo + h);
            for (u32 i = lane; i < (n - min(h, n)) / 16; i += 64) {
                const uint4 v = src[i];
                u32* d = reinterpret_cast<u32*>(win + h + 16 * i);  // 4-byte aligned (h and tlo are)
                d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
            }
            for (u32 i = h + ((n - min(h, n)) & ~15u) + lane; i < n; i += 64) win[i] = z.text[tlo + i];
        } else if (((uintptr_t)z.text & 3) == 0) {
            // 4 dwords per lane in flight before their LDS stores (one wave copies ~5 KB: the
            // one-dword loop waited a round trip per dword, ~13 us per window)
            const u32* src = reinterpret_cast<const u32*>(z.text + tlo);
            u32* dst = reinterpret_cast<u32*>(win);
            const u32 nd = n / 4;
            u32 i = lane;
            for (; i + 192 < nd; i += 256) {
                const u32 v0 = src[i], v1 = src[i + 64], v2 = src[i + 128], v3 = src[i + 192];
                dst[i] = v0, dst[i + 64] = v1, dst[i + 128] = v2, dst[i + 192] = v3;
            }
            for (; i < nd; i += 64) dst[i] = src[i];
            for (u32 i = (n & ~3u) + lane; i < n; i += 64) win[i] = z.text[tlo + i];
        } else {
            for (u32 i = lane; i < n; i += 64) win[i] = z.text[tlo + i];
        }
        __syncthreads();
        if (z.prof && lane == 0) {
            atomicAdd(z.prof + 24, wall_clock64() - tr0);
            atomicAdd(z.prof + 26, (u64)1);
        }
    }
    const LText t{z.text, win, wlo & ~3u, whi};
    const u32 maxl = end - q;
    const u32 capl = min((u32)LZ_CAP, maxl);
    // 8-byte candidate compares in the 5 KB-window form (the 62 KiB form keeps byte compares:
    // with them ROCm's gfx950 backend emits an invalid V_CMP on src_shared_base there)
    constexpr bool V8 = !HF;
    // 8 bytes at y (little-endian; 0 past the block end): the LDS window when they lie in it
    const u32 wl = wlo & ~3u, wh = whi;
    auto tx8 = [&](u32 y) -> u64 {
        if (y >= wl && y + 8 <= wh) return lds8(win, y - wl);
        if (y + 12 <= end) return glob8(z.text, y);
        u64 v = 0;
        for (u32 k = 0; k < 8; ++k)
            if (y + k < end) v |= (u64)z.text[y + k] << (8 * k);
        return v;
    };
    const u64 qv = V8 ? tx8(q) : 0ull;  // q's first 8 bytes
    const u8 c0 = t[q], c1 = t[q + 1], c2 = t[q + 2];
    u32 best = 0, bd = 0;
    const u32 hlo = q - dmax, hn = min(end, q + dmax) - hlo;  // fingerprints over [hlo, hlo + hn]
    bool hbuilt = false;
    const u64 blane = HF ? hf_pow(HF_B, lane) : 0, b64 = HF ? hf_pow(HF_B, 64) : 0;
    u32 hd0 = 0;   // distance whose power hbd0 holds
    u64 hbd0 = 1;
    if (d0s) {
        const u64 tl0 = z.prof ? wall_clock64() : 0;
        best = wave_lcp8(t, q, q - d0s, l0s, maxl, end);
        bd = d0s;
        ++nlong;
        if (z.prof && lane == 0) {
            atomicAdd(z.prof + 14, wall_clock64() - tl0);
            atomicAdd(z.prof + 15, (u64)best);
        }
    }
    // No distance d > bd with d - gcd(d, bd) <= best beats the match at bd (Fine and Wilf: a
    // strictly longer match at d would give t[q - bd, q + best) the periods d and bd, hence
    // period gcd(d, bd), and then the byte at q + best would match at bd too).  So the scan
    // starts past best + 1 (gcd >= 1) once a match is known, skips the multiples of bd up to best + bd, and ends
    // once best + 1 >= dmax.
    const u64 tlp0 = z.prof ? wall_clock64() : 0;
    for (u32 d0 = bd ? max(d0s + 1, best + 2) : d0s + 1; d0 <= dmax && best < maxl && best + 1 < dmax;
         d0 = bd ? max(d0 + 64, best + 2) : d0 + 64) {
        const u32 d = d0 + lane;
        const u32 x = q - d;
        // fingerprint mode: a lane passes iff t[x, x + best] fingerprints equal to t[q, q + best]
        // (which covers the 3-gram, the byte at best and the Fine-Wilf exclusions); a passing
        // lane is then extended from 0 by the wave, so a collision cannot change the result
        const bool hfm = HF && best > 2 * LZ_CAP;
        bool ok;
        u32 l = 0;
        u64 dx = 0;  // (non-fingerprint mode) x's first 8 bytes ^ q's
        if (hfm) {
            // inside the loop best + 1 < dmax, so x + best + 1 <= q + best + 1 <= hlo + hn
            if (!hbuilt) {
                const u64 th0 = z.prof ? wall_clock64() : 0;
                hf_build(t, hh, hlo, hn);
                hbuilt = true;
                if (z.prof && lane == 0) atomicAdd(z.prof + 23, wall_clock64() - th0);
            }
            if (d0 != hd0) {
                hbd0 = d0 == hd0 + 64 ? hbd0 * b64 : hf_pow(HF_B, d0);
                hd0 = d0;
            }
            const u32 L = best + 1;
            const u64 hq = hh[q + L - hlo] - hh[q - hlo];
            ok = d <= dmax && (hh[x + L - hlo] - hh[x - hlo]) * (hbd0 * blane) == hq;
            if (ok) l = capl;
        } else {
            ok = d <= dmax;
            if (V8) {
                if (ok) {
                    dx = tx8(x) ^ qv;  // x + 8 <= q + 8: inside the window or the block
                    ok = (dx & 0xFFFFFFull) == 0;  // the same 3-gram
                }
            } else {
                ok = ok && t[x] == c0 && t[x + 1] == c1 && t[x + 2] == c2;
            }
            if (ok && bd && d <= best + bd) ok = d % bd != 0;
            if (ok && best) ok = best < maxl && t[x + best] == t[q + best];
        }
        if (!hfm && ok && best > 2 * LZ_CAP) {
            // a longer match agrees everywhere below best: 8 spread samples reject most
            // candidates of periodic text that run out earlier (each would be an
            // extension over KB of text)
#pragma unroll
            for (u32 k = 1; k <= 8; ++k) {
                const u32 y = (u32)(((u64)best * k) / 9);
                ok = ok && t[x + y] == t[q + y];
            }
        }
        if (ok && !hfm && !V8) {
            l = LZ_MIN;
            while (l < capl && t[x + l] == t[q + l]) ++l;
        } else if (ok && !hfm) {
            // exact length up to capl, 8 bytes per step (x + l < q + l <= end: bytes read past
            // the block end only lie beyond capl, which clamps them)
            if (dx) {
                l = (u32)(__ffsll((long long)dx) - 1) >> 3;
            } else {
                l = 8;
                while (l < capl) {
                    const u64 dl = tx8(x + l) ^ tx8(q + l);
                    if (dl) {
                        l += (u32)(__ffsll((long long)dl) - 1) >> 3;
                        break;
                    }
                    l += 8;
                }
            }
            l = min(l, capl);
        }
        // capped candidates in ascending distance, each extended by the whole wave unless it
        // cannot be strictly longer than the longest one so far (`bb`): that needs a match at
        // bb (periodic text otherwise extends every multiple of its period to the same end)
        u64 longm = __ballot(ok && l >= capl && capl < maxl);
        const u64 okm = z.prof ? __ballot(ok) : 0;
        if (z.prof && d0s && lane == 0) {
            atomicAdd(z.prof + 16, (u64)1);
            atomicAdd(z.prof + 17, (u64)__popcll(okm));
            atomicAdd(z.prof + 18, (u64)__popcll(longm));
        }
        u32 bb = best;
        while (longm) {
            const u32 j = (u32)__ffsll((long long)longm) - 1;
            const u32 xj = __builtin_amdgcn_readlane(x, j);
            if (bb > capl && (bb >= maxl || t[xj + bb] != t[q + bb])) {
                if (lane == j) l = capl;  // LCP <= bb: an earlier candidate or `best` wins
            } else {
                const u64 te0 = z.prof ? wall_clock64() : 0;
                const u32 lj = wave_lcp8(t, q, xj, hfm ? 0u : capl, maxl, end);
                if (z.prof && d0s && lane == 0) {
                    atomicAdd(z.prof + 19, (u64)1);
                    atomicAdd(z.prof + 20, (u64)(lj - capl));
                    atomicAdd(z.prof + 21, wall_clock64() - te0);
                    atomicAdd(z.prof + 22, (u64)(lj > bb));
                }
                if (lane == j) l = lj;
                bb = max(bb, lj);
                ++nlong;
            }
            longm &= longm - 1;
        }
        const u32 lv = ok ? l : 0u;
        const u32 lm = wave_reduce(lv, OpMaxU(), 0u);
        if (lm > best) {
            const u64 eq = __ballot(lv == lm);
            best = lm;
            bd = d0 + (u32)__ffsll((long long)eq) - 1;
        }
        if (best >= maxl || best + 1 >= dmax) break;
    }
    if (z.prof && d0s && lane == 0) atomicAdd(z.prof + 25, wall_clock64() - tlp0);
    if (best >= (u32)LZ_MIN) {
        out_len = best;
        out_dist = bd;
    }
}

// Per block (one wave): the true path over the chunk summaries of k_lz_local.  WIN: the
// brute-force searches' LDS text window (BF_WIN, or BF_WIN_BIG for batches of few blocks).
template <u32 WIN>
__global__ __launch_bounds__(64) void k_lz_stitch_l(LzArgs z) {
    __shared__ __align__(16) u8 win[WIN + 16];
    const u64 tst = z.prof ? wall_clock64() : 0;
    const u32 b = blockIdx.x, lane = threadIdx.x;
    const u32 base = z.geo.base(b), bend = z.geo.end(b);
    const u32 CH = 1u << z.cshift;
    const u32 nck = (bend - base + CH - 1) >> z.cshift;
    u32 wlo = 1, whi = 0;  // no window loaded
    u32 entry = base, boff = 0, ntot = 0, fi = 0, nlong = 0, nfix_all = 0;
    for (u32 kb = 0; kb < nck; kb += 64) {
        const u32 k = kb + lane;
        const bool have = k < nck;
        const u32 c = b * z.cpb + k;
        const u32 sl = base + (k << z.cshift);
        const u32 nt_l = have ? z.c_ntok[c] : 0u;
        const u32 ex_l = have ? z.c_exit[c] : 0u;
        const u32 by_l = have ? z.c_bytes[c] : 0u;
        const u32 fp_l = (have && nt_l) ? z.tok_pos[sl] : NONE;
        u32 o_first = 0, o_fix0 = 0, o_nfix = 0, o_fixb = 0, o_off = 0;
        const u32 kn = min(64u, nck - kb);
        const u32 ex_prev = (u32)__shfl_up((int)ex_l, 1);  // the previous chunk's exit (lanes >= 1)
        for (u32 j = 0; j < kn; ++j) {
            // Runs of chunks taken whole, lane-parallel: chunk l is taken whole when its first
            // recorded token starts at its entry and its last token is resolved; inside a run the
            // entry of chunk l is chunk l-1's exit, so a ballot finds the run and a scan gives
            // every chunk's output offset (one serial step per chunk before: ~0.9 ms per batch)
            if (z.stitch_runs) {
                const u32 pred = lane == j ? entry : ex_prev;
                const bool ok = lane >= j && lane < kn && !(ex_l & LZ_UNRES) && fp_l == pred;
                const u64 bad = ~__ballot(ok) & (~0ull << j);
                const u32 jn = min(kn, bad ? (u32)__ffsll((long long)bad) - 1 : 64u);
                if (jn > j) {
                    const bool inrun = lane >= j && lane < jn;
                    const u32 bv = inrun ? by_l : 0u;
                    const u32 incl = wave_incl_scan(bv, OpAddU(), 0u);
                    const u32 nv = wave_reduce(inrun ? nt_l : 0u, OpAddU(), 0u);
                    if (inrun) {
                        o_first = 0;
                        o_fix0 = base + fi;
                        o_nfix = 0;
                        o_fixb = 0;
                        o_off = boff + incl - bv;
                    }
                    boff += (u32)__builtin_amdgcn_readlane((int)incl, 63);
                    ntot += nv;
                    entry = (u32)__builtin_amdgcn_readlane((int)ex_l, (int)(jn - 1));
                    j = jn;
                    if (j >= kn) break;
                }
            }
            const u32 s = base + ((kb + j) << z.cshift);
            const u32 e = min(s + CH, bend);
            const u32 nt = __builtin_amdgcn_readlane(nt_l, j), ex = __builtin_amdgcn_readlane(ex_l, j);
            const u32 by = __builtin_amdgcn_readlane(by_l, j), fp = __builtin_amdgcn_readlane(fp_l, j);
            const u32 fix0 = base + fi;
            u32 first, nfix = 0, fixb = 0, spec = 0, next;
            if (entry >= e) {
                first = nt;
                next = entry;
            } else if (fp == entry && !(ex & LZ_UNRES)) {
                first = 0;
                spec = by;
                next = ex;
            } else {
                if (z.prof && lane == 0) atomicAdd(z.prof + 13, (u64)1);
                u32 q = entry, jt = 0;
                bool conv = false;
                while (q < e) {
                    // first recorded token at or after q (tokens ascend; jt only grows)
                    u32 tq = NONE;
                    for (;;) {
                        const u32 i = jt + lane;
                        const u32 tp = i < nt ? z.tok_pos[s + i] : NONE;
                        const u64 ge = __ballot(tp >= q);
                        if (ge) {
                            const u32 f = (u32)__ffsll((long long)ge) - 1;
                            jt += f;
                            tq = (u32)__shfl((int)tp, (int)f);
                            break;
                        }
                        jt += 64;
                    }
                    if (jt < nt && tq == q) {
                        conv = true;
                        break;
                    }
                    u32 len, dist;
                    const u64 tb0 = z.prof ? wall_clock64() : 0;
                    bf_match<WIN>(z, win, wlo, whi, q, base, bend, len, dist, nlong);
                    if (z.prof && lane == 0) {
                        atomicAdd(z.prof + 8, (u64)1);
                        atomicAdd(z.prof + 9, wall_clock64() - tb0);
                    }
                    if (lane == 0) {
                        z.fix_pos[base + fi] = q;
                        z.fix_len[base + fi] = len;
                        z.fix_dist[base + fi] = dist;
                        z.fix_off[base + fi] = boff + fixb;
                    }
                    ++fi;
                    ++nfix;
                    fixb += tok_bytes(len, dist);
                    q += len ? len : 1;
                }
                if (conv) {
                    first = jt;
                    spec = by - z.tok_off[s + jt];
                    next = ex & ~LZ_UNRES;
                    if (ex & LZ_UNRES) {
                        // the last recorded token reached the speculative cap: exact length
                        const u32 li = s + nt - 1;
                        const u32 pp = z.tok_pos[li], ol = z.tok_len[li], od = z.tok_dist[li];
                        u32 nl, nd;
                        const u64 tb0 = z.prof ? wall_clock64() : 0;
                        bf_match<WIN>(z, win, wlo, whi, pp, base, bend, nl, nd, nlong, od, ol);
                        if (z.prof && lane == 0) {
                            atomicAdd(z.prof + 10, (u64)1);
                            atomicAdd(z.prof + 11, wall_clock64() - tb0);
                        }
                        spec = spec + tok_bytes(nl, nd) - tok_bytes(ol, od);
                        if (lane == 0) {
                            z.tok_len[li] = nl;
                            z.tok_dist[li] = nd;
                        }
                        next = pp + (nl ? nl : 1u);
                    }
                } else {
                    first = nt;
                    next = q;
                }
                nfix_all += nfix;
            }
            if (lane == j) {
                o_first = first;
                o_fix0 = fix0;
                o_nfix = nfix;
                o_fixb = fixb;
                o_off = boff;
            }
            boff += fixb + spec;
            ntot += nfix + (nt - first);
            entry = next;
        }
        if (have) {
            z.c_first[c] = o_first;
            z.c_fix0[c] = o_fix0;
            z.c_nfix[c] = o_nfix;
            z.c_fixbytes[c] = o_fixb;
            z.c_off[c] = o_off;
        }
    }
    if (z.prof && lane == 0) atomicMax((unsigned long long*)(z.prof + 12), (unsigned long long)(wall_clock64() - tst));
    if (lane == 0) {
        z.lz_size[b] = boff;
        z.ntok[b] = ntot;
        z.b_nfix[b] = fi;
        if (nlong) atomicAdd(z.nlong, nlong);
        if (nfix_all && z.nfix) atomicAdd(z.nfix, nfix_all);
    }
}

__device__ inline u32 put_uleb(u8* d, u32 v) {
    u32 n = 0;
    for (;;) {
        const u32 byte = v & 0x7F;
        v >>= 7;
        if (v) {
            d[n++] = (u8)(byte | 0x80);
        } else {
            d[n++] = (u8)byte;
            return n;
        }
    }
}

__device__ inline void write_token(u8* d, const u8* text, u32 pos, u32 len, u32 dist) {
    if (len == 0) {
        d[0] = 0;
        d[1] = text[pos];
    } else {
        d[0] = 1;
        const u32 n1 = put_uleb(d + 1, len);
        put_uleb(d + 1 + n1, dist);
    }
}

// One thread per token slot g: speculative token (slot in its chunk) and fix-up token.
__global__ __launch_bounds__(256) void k_lz_emit(LzArgs z, const u32* method, const u64* off, u8* arena,
                                                 int force_all) {
    const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= z.geo.N) return;
    const u32 b = z.geo.block_of(g);
    if (!force_all && method[b] != 7u) return;
    const u32 base = z.geo.base(b);
    u8* dst = arena + off[b];
    const u32 k = (g - base) >> z.cshift;
    const u32 c = b * z.cpb + k;
    const u32 s = base + (k << z.cshift);
    const u32 i = g - s;
    const u32 first = z.c_first[c];
    if (i >= first && i < z.c_ntok[c]) {
        const u32 o = z.c_off[c] + z.c_fixbytes[c] + (z.tok_off[g] - z.tok_off[s + first]);
        write_token(dst + o, z.text, z.tok_pos[g], z.tok_len[g], z.tok_dist[g]);
    }
    if (g - base < z.b_nfix[b]) write_token(dst + z.fix_off[g], z.text, z.fix_pos[g], z.fix_len[g], z.fix_dist[g]);
}

}  // namespace

const char* lz_spec_name() { return "k_lz_local"; }

u32 lz_chunk_shift() { return 8u; }  // 256-byte chunks

int lz_index_form(u32 nb) {
    // Batches of 64 blocks or more: form 0.  There the parse is hidden beside the sort stream
    // (it ends ~4 ms before it), so the index work inside it costs the step nothing, while the
    // tile index is one more kernel whose time lands on the sort stream: k_lz_tiles takes ~0.4
    // ms alone but ~2 ms beside Lyndon or round 0 and slows what it meets (the Lyndon merge 0.27
    // -> 0.94 ms, the first round-0 pass 0.97 -> 1.73 ms), so form 2 measured 34.1-34.4 ms per
    // step against 33.2-33.4 for form 0 in every placement (round 6, profiles/r06/ab_lz_idx_*).
    // Smaller batches: form 2 (config 4's 32-block shard 6.25-6.28 -> 5.92-5.94 ms).
    // KOLM_LZ_IDX overrides (read per call: tests).
    if (getenv("KOLM_LZ_IDX")) return atoi(getenv("KOLM_LZ_IDX"));
    return nb < 64 ? 2 : 0;
}

static void launch_lz_tiles(const LzArgs& z, hipStream_t s, KTimer* kt) {
    if (!z.geo.nb || lz_index_form(z.geo.nb) == 0) return;
    const u32 hpb = (z.geo.bs + LZL_HOME - 1) / LZL_HOME;
    // text 1 B + rank 2 B per position + 2 KiB of counts per tile
    KScope k(kt, KT_LZPARSE, "k_lz_tiles", z.geo.N * 3 + (u64)z.geo.nb * hpb * 2048);
    k_lz_tiles<<<z.geo.nb * hpb, 256, 0, s>>>(z, hpb);
}

void launch_lz_parse(const LzArgs& z, hipStream_t s, KTimer* kt) {
    if (!z.geo.nb) return;
    // 4 KiB homes, 16 chains of 16 lanes (4 workgroups per CU, LDS-limited).  Measured and
    // removed: 8 KiB homes parsed by 32 chains of 8 lanes (round 5: 2 waves per SIMD no longer hide
    // the chains' LDS latency, step 35.7 -> 39.9 ms), 5 KiB homes in 5-wave workgroups (round 6:
    // step 33.4 -> 36.7 ms beside the sort stream) and a chain per lane over 64-byte chunks with
    // hash chains in LDS (round 6: 512 chains per CU, but 64 independent chains per wave take
    // every branch in every trip — 81 K VALU per wave — k_lz_local alone 8.4 -> 15.6 ms)
    constexpr u32 home = 4096u;
    static_assert(home == (u32)LZL_HOME, "tile index and homes share the 4 KiB geometry");
    const u32 hpb = (z.geo.bs + home - 1) / home;
    const int idx = lz_index_form(z.geo.nb);
    launch_lz_tiles(z, s, kt);
    {
        // lead-in bytes parsed before each chain's chunk (at most LZL_LEAD, the window's margin):
        // 48 since the stitch's fix-up searches got cheaper (round 5, two A/B calls, profiles/r05/
        // ab_lz_lead_*: 33.67-33.76 ms per step at 48 and 56 against 33.84-34.30 at 64; 32 and 40
        // measured 34.09-34.44 and 34.18).  KOLM_LZ_LEAD overrides.
        static const u32 lead =
            getenv("KOLM_LZ_LEAD") ? std::min<u32>(atoi(getenv("KOLM_LZ_LEAD")), LZL_LEAD) : 48u;
        // (round 6: the parse capped at 3 workgroups per CU by extra LDS measured 33.3 -> 34.2-34.3 ms
        // per step with form 0, 34.1 -> 33.9-34.0 with form 2)
        constexpr u32 pad = 0;
        KScope k(kt, KT_LZPARSE, "k_lz_local", z.geo.N * 2);
        if (idx == 0)
            k_lz_local<home, 16, 0><<<z.geo.nb * hpb, LzlGeom<home, 16, 0>::NT, pad, s>>>(z, hpb, lead);
        else
            k_lz_local<home, 16, 2><<<z.geo.nb * hpb, LzlGeom<home, 16, 2>::NT, pad, s>>>(z, hpb, lead);
    }
    {
        KScope k(kt, KT_LZPARSE, "k_lz_stitch", (u64)z.cpb * z.geo.nb * 16);
        // KOLM_LZ_BIGWIN = 0 / 1 forces the window; default: 62 KiB (+ fingerprints) below 64 blocks
        const int bw = getenv("KOLM_LZ_BIGWIN") ? atoi(getenv("KOLM_LZ_BIGWIN")) : -1;  // read per call (tests)
        if (bw == 1 || (bw < 0 && z.geo.nb < 64))
            k_lz_stitch_l<BF_WIN_BIG><<<z.geo.nb, 64, 0, s>>>(z);
        else
            k_lz_stitch_l<BF_WIN><<<z.geo.nb, 64, 0, s>>>(z);
    }
}

void launch_lz_emit(const LzArgs& z, const u32* method, const u64* off, u8* arena, hipStream_t s) {
    if (!z.geo.N) return;
    k_lz_emit<<<(u32)((z.geo.N + 255) / 256), 256, 0, s>>>(z, method, off, arena, method == nullptr ? 1 : 0);
}

}  // namespace kolm
