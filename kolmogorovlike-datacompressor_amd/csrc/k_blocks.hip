// Per-block scans: Lyndon factorisation from the linear suffix order, BBWT gather.
//
// Lyndon factorisation (replaces Duval, PY:326-349 / CPP:902-933): position p starts a
// Lyndon factor of its block iff its suffix is smaller than every suffix starting
// before it inside the block, i.e. ISA[p] < min(ISA[base..p)) — left-to-right minima of
// the inverse suffix array (the factors are the non-increasing Lyndon words, and the
// last factor is the minimal suffix).  Computed as a tiled per-block prefix-min scan.
// Then every position gets its factor's start FS and length FL (prefix-max of starts,
// suffix-min of the next start).
//
// BBWT gather (PY:417: out.append(w[(i - 1) % m])): out[r] = text[prev(SA[r])] where
// prev steps back cyclically inside the factor.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "kolm_internal.h"

namespace kolm {

namespace {

constexpr u32 BIG = 0xFFFFFFFFu;

struct TileGeom {
    Geom geo;
    u32 tpb;  // tiles per block
    __device__ inline bool range(u32 t, u32& lo, u32& hi, u32& b) const {
        b = t / tpb;
        const u32 k = t - b * tpb;
        lo = geo.base(b) + k * TILE;
        const u32 e = geo.end(b);
        hi = min(lo + (u32)TILE, e);
        return lo < e;
    }
};

__device__ inline u32 wave_reduce_min(u32 v) { return wave_reduce(v, OpMinU(), BIG); }
__device__ inline u32 wave_reduce_max(u32 v) { return wave_reduce(v, OpMaxU(), 0u); }

// exclusive scan across the workgroup (min or max, forward or reverse); DPP within waves
template <bool REV, bool MAX>
__device__ inline u32 wg_excl(u32 v, u32 ident, u32* sh) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 incl, ex;
    if (MAX) {
        incl = REV ? wave_incl_scan_rev(v, OpMaxU(), ident) : wave_incl_scan(v, OpMaxU(), ident);
    } else {
        incl = REV ? wave_incl_scan_rev(v, OpMinU(), ident) : wave_incl_scan(v, OpMinU(), ident);
    }
    ex = REV ? KOLM_DPP(ident, incl, DPP_WAVE_SHL1, 0xF) : KOLM_DPP(ident, incl, DPP_WAVE_SHR1, 0xF);
    if (REV ? lane == 0 : lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = ident;
    if (!REV) {
        for (u32 i = 0; i < w; ++i) carry = MAX ? max(carry, sh[i]) : min(carry, sh[i]);
    } else {
        for (u32 i = w + 1; i < WG / 64; ++i) carry = MAX ? max(carry, sh[i]) : min(carry, sh[i]);
    }
    __syncthreads();
    return MAX ? max(carry, ex) : min(carry, ex);
}

// Phase B: per block, exclusive scan over the block's tiles (one workgroup per block).
template <bool REV, bool MAX>
__global__ __launch_bounds__(WG) void k_tiles_scan(const u32* in, u32* out, u32 tpb, u32 ident) {
    __shared__ u32 sh[WG / 64];
    const u32 b = blockIdx.x;
    u32 carry = ident;
    const u32 nch = (tpb + WG - 1) / WG;
    for (u32 c = 0; c < nch; ++c) {
        const u32 cc = REV ? nch - 1 - c : c;
        const u32 k = cc * WG + threadIdx.x;
        const u32 v = k < tpb ? in[b * tpb + k] : ident;
        const u32 ex = wg_excl<REV, MAX>(v, ident, sh);
        const u32 r = MAX ? max(carry, ex) : min(carry, ex);
        if (k < tpb) out[b * tpb + k] = r;
        // chunk total
        u32 tot = MAX ? max(ex, v) : min(ex, v);  // inclusive at this thread
        __shared__ u32 edge;
        if (REV ? threadIdx.x == 0 : threadIdx.x == WG - 1) edge = tot;
        __syncthreads();
        carry = MAX ? max(carry, edge) : min(carry, edge);
        __syncthreads();
    }
}

// Phase A': per-tile first factor start.
__global__ __launch_bounds__(WG) void k_tile_starts(TileGeom tg, const u8* flag, u32* tmin) {
    __shared__ u32 sh[WG / 64];
    u32 lo, hi, b;
    const bool ok = tg.range(blockIdx.x, lo, hi, b);
    u32 mn = BIG;
    if (ok) {
        const u32 i0 = lo + threadIdx.x * PER_THREAD;
        if ((i0 & 7) == 0 && i0 + PER_THREAD <= hi) {
            const u64 f8 = *reinterpret_cast<const u64*>(flag + i0);  // 8 flags (0/1 bytes)
            if (f8) mn = i0 + ((u32)__ffsll((long long)f8) - 1) / 8;
        } else {
            for (u32 i = i0; i < min(i0 + PER_THREAD, hi); ++i)
                if (flag[i]) mn = min(mn, i);
        }
    }
    mn = wave_reduce_min(mn);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) tmin[blockIdx.x] = min(min(sh[0], sh[1]), min(sh[2], sh[3]));
}

// Phase C': FEd[p] = min(distance from p to its factor's end (next start or block end), 255).
__global__ __launch_bounds__(WG) void k_fed(TileGeom tg, const u8* flag, const u32* cmin, u8* FEd) {
    __shared__ u32 sh[WG / 64];
    u32 lo, hi, b;
    if (!tg.range(blockIdx.x, lo, hi, b)) return;
    const u32 bend = tg.geo.end(b);
    const u32 i0 = lo + threadIdx.x * PER_THREAD;
    const bool full = (i0 & 7) == 0 && i0 + PER_THREAD <= hi;  // 8-byte flag load and store
    u64 fl8 = 0;
    if (full) fl8 = *reinterpret_cast<const u64*>(flag + i0);
    bool f[PER_THREAD];
    u32 lmin = BIG;
#pragma unroll
    for (int e = 0; e < PER_THREAD; ++e) {
        const u32 i = i0 + e;
        f[e] = full ? ((fl8 >> (8 * e)) & 0xFF) != 0 : (i < hi && flag[i]);
        if (f[e]) lmin = min(lmin, i);
    }
    u32 fe = min(cmin[blockIdx.x], wg_excl<true, false>(lmin, BIG, sh));
    u64 fed8 = 0;
#pragma unroll
    for (int e = PER_THREAD - 1; e >= 0; --e) {
        const u32 i = i0 + e;
        const u32 end = fe == BIG ? bend : fe;
        const u32 d = min(end - i, 255u);
        fed8 |= (u64)d << (8 * e);
        if (!full && i < hi) FEd[i] = (u8)d;
        if (f[e]) fe = i0 + e;
    }
    if (full) *reinterpret_cast<u64*>(FEd + i0) = fed8;
}

// ---------------------------------------------------------------------------------
// Parallel Duval (restates PY:326-349 exactly) in two levels.
//   k_duval_span: one workgroup per 8 KiB span of a block (duval_span_bytes), staged in LDS.
//     Every thread runs Duval on its DUVAL_CH-byte chunk, then the chunk factorizations
//     are merged pairwise up a binary tree (6 levels) inside LDS; factor starts are kept
//     as a bitmap.  Merge rule (concatenation of two factorizations): for Lyndon words
//     x < y, xy is Lyndon, so pushing the right part's factors on the stack of the left
//     part's factors and merging while stack[-2] < stack[-1] gives the (unique) Lyndon
//     factorization of the concatenation; once a right factor is pushed without merging,
//     the remaining right factors (non-increasing) cannot merge either.
//   k_duval_merge: one wave per block merges the span factorizations left to right with
//     the same rule (comparisons read the text from global memory).
// ---------------------------------------------------------------------------------
constexpr u32 DUVAL_CH = 128;                 // bytes per thread
constexpr u32 DUVAL_PAD = 4;                  // LDS pad per chunk (bank spread)
constexpr u32 DUVAL_WAVE_W = 4096;            // tree levels merged by whole waves (from this width on)
constexpr u32 DUVAL_PF = 64;                  // factors per span with a cached 32-byte prefix

__device__ inline u32 lds_addr(u32 q) { return q + (q / DUVAL_CH) * DUVAL_PAD; }

// bytes q .. q+3 of the staged span (span-local positions, little-endian): two aligned
// LDS dwords of the logical word stream (a chunk's 128 bytes are whole words, the pad
// between chunks is skipped by lds_addr) and a byte funnel shift
__device__ inline u32 lds_word(const u8* t, u32 q) {
    const u32* d = reinterpret_cast<const u32*>(t);
    const u32 k = q & ~3u;
    return __builtin_amdgcn_alignbyte(d[lds_addr(k + 4) >> 2], d[lds_addr(k) >> 2], q & 3);
}

// x = t[x0, x1) < y = t[x1, y1) (span-local positions, proper prefix smaller); 4 bytes per
// step (factors of text share long prefixes: repeated words)
__device__ inline bool span_less(const u8* t, u32 x0, u32 x1, u32 y1) {
    const u32 la = x1 - x0, lb = y1 - x1, m = min(la, lb);
    u32 i = 0;
    for (; i + 4 <= m; i += 4) {
        const u32 a = lds_word(t, x0 + i), b = lds_word(t, x1 + i);
        if (a != b) {
            const u32 sh = (u32)(__ffs(a ^ b) - 1) & ~7u;  // the first differing byte
            return ((a >> sh) & 255u) < ((b >> sh) & 255u);
        }
    }
    for (; i < m; ++i) {
        const u8 a = t[lds_addr(x0 + i)], b = t[lds_addr(x1 + i)];
        if (a != b) return a < b;
    }
    return la < lb;
}

// The same comparison by the G lanes of this lane's aligned group (G = 2 .. 64, a power of
// two; the group's lanes are converged and agree on every argument): 4 G bytes per step, the
// first differing word found by a ballot over the group.  Reads up to 7 bytes past y1 inside
// the staged array (padded); bytes at or past m are masked.
__device__ inline bool span_less_grp(const u8* t, u32 x0, u32 x1, u32 y1, u32 G) {
    const u32 la = x1 - x0, lb = y1 - x1, m = min(la, lb);
    const u32 lane = threadIdx.x & 63, gl = lane & (G - 1);
    const u64 gm = (G >= 64 ? ~0ull : ((1ull << G) - 1ull)) << (lane & ~(G - 1) & 63u);
    for (u32 o = 0; o < m; o += 4 * G) {
        const u32 i = o + 4 * gl;
        u32 a = 0, b = 0, x = 0;
        if (i < m) {
            a = lds_word(t, x0 + i);
            b = lds_word(t, x1 + i);
            x = a ^ b;
            if (m - i < 4) x &= (1u << (8 * (m - i))) - 1u;
        }
        const u64 bal = __ballot(x != 0) & gm;
        if (bal) {
            u32 r = 0;
            if (x) {
                const u32 sh = (u32)(__ffs(x) - 1) & ~7u;  // the first differing byte
                r = ((a >> sh) & 255u) < ((b >> sh) & 255u) ? 1u : 0u;
            }
            return __shfl((int)r, (int)(__ffsll((unsigned long long)bal) - 1)) != 0;
        }
    }
    return la < lb;
}

// the same comparison by a whole wave, 64 bytes per step (uniform result)
__device__ inline bool span_less_wave(const u8* t, u32 x0, u32 x1, u32 y1, u32 lane) {
    const u32 la = x1 - x0, lb = y1 - x1, m = min(la, lb);
    for (u32 o = 0; o < m; o += 64) {
        const u32 i = o + lane;
        const bool diff = i < m && t[lds_addr(x0 + i)] != t[lds_addr(x1 + i)];
        const u64 bal = __ballot(diff);
        if (bal) {
            const u32 d = o + (u32)__ffsll((unsigned long long)bal) - 1;
            return t[lds_addr(x0 + d)] < t[lds_addr(x1 + d)];
        }
    }
    return la < lb;
}

// Two-level bitmap of factor starts: bm (1 bit per position) + sm (1 bit per non-zero bm
// word), so a search across a long factor costs O(len / 1024) instead of O(len / 32).
// largest set bit position <= q (a set bit at or below q must exist)
__device__ inline u32 bm_prev(const u32* bm, const u32* sm, u32 q) {
    u32 w = q >> 5;
    u32 v = bm[w] & (0xFFFFFFFFu >> (31 - (q & 31)));
    if (!v) {
        // previous non-zero word below w
        u32 sw = w >> 5;
        u32 sv = (w & 31) ? (sm[sw] & (0xFFFFFFFFu >> (32 - (w & 31)))) : 0u;
        while (!sv) sv = sm[--sw];
        w = (sw << 5) + 31 - __clz(sv);
        v = bm[w];
    }
    return (w << 5) + 31 - __clz(v);
}
// smallest set bit position >= q, or hi
__device__ inline u32 bm_next(const u32* bm, const u32* sm, u32 q, u32 hi) {
    if (q >= hi) return hi;
    u32 w = q >> 5;
    u32 v = bm[w] & (0xFFFFFFFFu << (q & 31));
    if (!v) {
        const u32 wl = (hi + 31) >> 5;  // words that may hold bits < hi
        const u32 swl = (wl + 31) >> 5;
        u32 sw = (w + 1) >> 5;
        if (sw >= swl) return hi;
        u32 sv = ((w + 1) & 31) ? (sm[sw] & (0xFFFFFFFFu << ((w + 1) & 31))) : sm[sw];
        while (!sv) {
            if (++sw >= swl) return hi;
            sv = sm[sw];
        }
        w = (sw << 5) + __ffs(sv) - 1;
        if (w >= wl) return hi;
        v = bm[w];
    }
    const u32 r = (w << 5) + __ffs(v) - 1;
    return r < hi ? r : hi;
}

// prof (debug, KOLM_DUVAL_PROF): wall-clock ticks per phase summed over workgroups
__device__ inline void dprof(u64* prof, u32 k, u64& last) {
    if (prof && threadIdx.x == 0) {
        const u64 now = wall_clock64();
        atomicAdd((unsigned long long*)&prof[k], (unsigned long long)(now - last));
        atomicMax((unsigned long long*)&prof[24 + k], (unsigned long long)(now - last));  // slowest workgroup
        last = now;
    }
}
// NT threads (of DUVAL_CH bytes each) per span: 64 (8 KiB spans, the default: duval_span_bytes)
// or 256 (32 KiB)
template <u32 NT>
__global__ __launch_bounds__(NT) void k_duval_span(Geom geo, u32 spb, const u8* s, u32* fstart, uint4* fpre,
                                                   u32* nfac, u64* prof, u32 wave_w, u32 grp) {
    constexpr u32 SPAN = DUVAL_CH * NT;
    u64 tlast = prof ? wall_clock64() : 0;
    __shared__ __align__(16) u8 t[SPAN + NT * DUVAL_PAD + 16];  // + 16: lds_word's reads past the end
    __shared__ u32 bm[SPAN / 32];
    __shared__ u32 sm[(SPAN + 1023) / 1024];
    __shared__ u32 sh[NT / 64];
    const u32 sp = blockIdx.x, tid = threadIdx.x;
    const u32 b = sp / spb, k = sp - b * spb;
    const u32 lo = geo.base(b) + k * SPAN;
    const u32 e = geo.end(b), e_blk = e;
    if (lo >= e) {
        if (tid == 0) nfac[sp] = 0;
        return;
    }
    const u32 n = min(SPAN, e - lo);
    // stage the span (16-byte loads when aligned and whole)
    if (n == SPAN && (lo & 15) == 0) {
        const uint4* src = reinterpret_cast<const uint4*>(s + lo);
        for (u32 i = tid; i < SPAN / 16; i += NT) {
            const uint4 v = src[i];
            u32* d = reinterpret_cast<u32*>(&t[lds_addr(i * 16)]);  // 4-byte aligned, inside one chunk
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    } else {
        for (u32 i = tid; i < n; i += NT) t[lds_addr(i)] = s[lo + i];
    }
    for (u32 i = tid; i < SPAN / 32; i += NT) bm[i] = 0;
    __syncthreads();
    dprof(prof, 0, tlast);
    // Duval on the thread's chunk; factor starts -> bitmap (bits of one chunk are 4 words
    // owned by this thread only).  One flat loop: every trip advances the lane's own state
    // machine by exactly one step — a comparison (scan phase) or one factor emitted (emit
    // phase) — so the lanes of a wave stay in step instead of serialising the nested
    // loops' data-dependent trip counts.
    {
        const u32 clo = tid * DUVAL_CH, chi = min(clo + DUVAL_CH, n);
        u32 i = clo, j = clo + 1, kk = clo, p = 1;
        bool emit = false;
        u32 w0 = 0, w1 = 0, w2 = 0, w3 = 0;  // the chunk's 128 start bits
        static_assert(DUVAL_CH == 128, "four bitmap words per chunk");
        while (i < chi) {
            if (!emit) {
                bool stop = j >= chi;
                if (!stop) {
                    const u8 a = t[lds_addr(kk)], bb = t[lds_addr(j)];
                    stop = a > bb;
                    if (!stop) {
                        kk = (a < bb) ? i : kk + 1;
                        ++j;
                    }
                }
                if (stop) {
                    emit = true;
                    p = j - kk;
                }
            } else {
                const u32 li = i - clo, bit = 1u << (li & 31), wq = li >> 5;
                w0 |= wq == 0 ? bit : 0u;
                w1 |= wq == 1 ? bit : 0u;
                w2 |= wq == 2 ? bit : 0u;
                w3 |= wq == 3 ? bit : 0u;
                i += p;
                if (i > kk) {  // the run of equal factors is out: scan from the next start
                    emit = false;
                    kk = i;
                    j = i + 1;
                }
            }
        }
        bm[clo / 32] = w0;
        bm[clo / 32 + 1] = w1;
        bm[clo / 32 + 2] = w2;
        bm[clo / 32 + 3] = w3;
    }
    __syncthreads();
    dprof(prof, 1, tlast);
    if (tid < (SPAN + 1023) / 1024) {
        u32 v = 0;
        for (u32 q = 0; q < 32 && tid * 32 + q < SPAN / 32; ++q) v |= (bm[tid * 32 + q] != 0) << q;
        sm[tid] = v;
    }
    __syncthreads();
    // tree merge of adjacent factorizations: a thread per merge on the low levels, a wave
    // per merge (64-lane factor comparisons) from wave_w up, where few merges remain
    // and adjacent factors of text share long prefixes
    for (u32 w = DUVAL_CH; w < SPAN; w <<= 1) {
        if (grp) {
            // a group of G = w / 64 lanes per merge (NT / G groups = the level's SPAN / 2w merges;
            // G capped at one wave): the merges of a level run in parallel as in the thread form
            // and every factor comparison reads 4 G bytes per step
            const u32 G = min(64u, w / 64);
            const u32 a0 = (tid / G) * 2 * w, m = a0 + w;
            if (m < n) {
                const u32 hi = min(m + w, n);
                u32 r = m;
                while (r < hi) {
                    const u32 re = bm_next(bm, sm, r + 1, hi);
                    u32 ts = r;
                    bool merged = false;
                    while (ts > a0) {
                        const u32 ps = bm_prev(bm, sm, ts - 1);
                        if (!span_less_grp(t, ps, ts, re, G)) break;
                        // the group's lanes write the same value: each then reads its own write
                        const u32 nw = bm[ts >> 5] & ~(1u << (ts & 31));
                        bm[ts >> 5] = nw;
                        if (!nw) atomicAnd(&sm[ts >> 10], ~(1u << ((ts >> 5) & 31)));
                        ts = ps;
                        merged = true;
                    }
                    if (!merged) break;
                    r = re;
                }
            }
            __syncthreads();
            dprof(prof, 2 + (31 - __clz(w)) - 7, tlast);
            continue;
        }
        if (w >= wave_w) {
            const u32 lane = tid & 63, wv = tid >> 6;
            for (u32 a0 = wv * 2 * w; a0 + w < n; a0 += 2 * w * (NT / 64)) {
                const u32 m = a0 + w, hi = min(m + w, n);
                u32 r = m;
                while (r < hi) {
                    const u32 re = bm_next(bm, sm, r + 1, hi);
                    u32 ts = r;
                    bool merged = false;
                    while (ts > a0) {
                        const u32 ps = bm_prev(bm, sm, ts - 1);
                        if (!span_less_wave(t, ps, ts, re, lane)) break;
                        // every lane writes the same value: each then reads its own write
                        const u32 nw = bm[ts >> 5] & ~(1u << (ts & 31));
                        bm[ts >> 5] = nw;
                        if (!nw) atomicAnd(&sm[ts >> 10], ~(1u << ((ts >> 5) & 31)));
                        ts = ps;
                        merged = true;
                    }
                    if (!merged) break;
                    r = re;
                }
            }
            __syncthreads();
            dprof(prof, 2 + (31 - __clz(w)) - 7, tlast);
            continue;
        }
        // one merge per thread (a flat state-machine form of this loop, one step per trip,
        // measured 2.5x slower per level: the three masked paths every trip cost more than
        // the divergence they remove)
        const u32 a0 = tid * 2 * w, m = a0 + w;
        if (m < n) {
            const u32 hi = min(m + w, n);
            u32 r = m;
            while (r < hi) {
                const u32 re = bm_next(bm, sm, r + 1, hi);
                u32 ts = r;
                bool merged = false;
                while (ts > a0) {
                    const u32 ps = bm_prev(bm, sm, ts - 1);
                    if (!span_less(t, ps, ts, re)) break;
                    const u32 nw = bm[ts >> 5] & ~(1u << (ts & 31));
                    bm[ts >> 5] = nw;
                    if (!nw) atomicAnd(&sm[ts >> 10], ~(1u << ((ts >> 5) & 31)));
                    ts = ps;
                    merged = true;
                }
                if (!merged) break;
                r = re;
            }
        }
        __syncthreads();
        dprof(prof, 2 + (31 - __clz(w)) - 7, tlast);  // levels w = 128 .. 16384 -> 2 .. 9
    }
    // compact the factor starts of the span into fstart[lo ...]
    u32 cnt = 0;
    for (u32 q = 0; q < DUVAL_CH / 32; ++q) cnt += __popc(bm[tid * (DUVAL_CH / 32) + q]);
    u32 o = 0;
    {
        // exclusive scan over the NT threads
        const u32 lane = tid & 63, wv = tid >> 6;
        u32 incl = cnt;
        for (u32 d = 1; d < 64; d <<= 1) {
            const u32 x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        if (lane == 63) sh[wv] = incl;
        __syncthreads();
        u32 carry = 0;
        for (u32 i = 0; i < wv; ++i) carry += sh[i];
        o = carry + incl - cnt;
        if (tid == NT - 1) nfac[sp] = carry + incl;
    }
    for (u32 q = 0; q < DUVAL_CH / 32; ++q) {
        u32 v = bm[tid * (DUVAL_CH / 32) + q];
        while (v) {
            const u32 bit = __ffs(v) - 1;
            v &= v - 1;
            const u32 x = tid * DUVAL_CH + q * 32 + bit;  // span-local start
            if (o < DUVAL_PF) {
                // its first 32 bytes, big-endian words (k_duval_merge compares these first)
                u32 w[8];
#pragma unroll
                for (u32 k = 0; k < 8; ++k) {
                    u32 v4 = 0;
#pragma unroll
                    for (u32 e = 0; e < 4; ++e) {
                        const u32 y = x + 4 * k + e;
                        const u8 ch = y < n ? t[lds_addr(y)] : (lo + y < e_blk ? s[lo + y] : (u8)0);
                        v4 = (v4 << 8) | ch;
                    }
                    w[k] = v4;
                }
                fpre[((u64)sp * DUVAL_PF + o) * 2] = make_uint4(w[0], w[1], w[2], w[3]);
                fpre[((u64)sp * DUVAL_PF + o) * 2 + 1] = make_uint4(w[4], w[5], w[6], w[7]);
            }
            fstart[lo + o++] = lo + x;
        }
    }
    __syncthreads();
    dprof(prof, 10, tlast);
}

// 8 bytes at s + x (any alignment) from three aligned dwords, little-endian
__device__ inline u64 load8u(const u8* s, u32 x) {
    const uintptr_t a = (uintptr_t)(s + x);
    const u32* w = reinterpret_cast<const u32*>(a & ~(uintptr_t)3);
    const u32 sh = (u32)(a & 3);
    const u32 w0 = w[0], w1 = w[1], w2 = w[2];
    return ((u64)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// One round trip of U 512-byte steps of lyn_less at offset o: the first differing offset,
// or ~0u when all U * 512 bytes agree.
template <u32 U>
__device__ inline u32 lyn_trip(const u8* s, u32 a0, u32 a1, u32 o, u32 lane) {
    u64 d[U];
#pragma unroll
    for (u32 k = 0; k < U; ++k) {
        const u32 t = o + 512 * k + 8 * lane;
        d[k] = load8u(s, a0 + t) ^ load8u(s, a1 + t);
    }
#pragma unroll
    for (u32 k = 0; k < U; ++k) {
        const u64 bal = __ballot(d[k] != 0);
        if (bal) {
            const u32 j = (u32)__ffsll((long long)bal) - 1;
            const u32 dj = (u32)__ffsll((long long)d[k]) - 1;
            return o + 512 * k + 8 * j + (u32)__builtin_amdgcn_readlane((int)dj, (int)j) / 8;
        }
    }
    return ~0u;
}

// x = s[a0, a1) < y = s[a1, b1) lexicographically (proper prefix smaller); wave-uniform.
// 8 bytes per lane per step (512 per wave) while the loads stay inside s[0, N).  The bytes
// from o0 on are compared (the first o0 are known equal).  lcp / exact: where it stopped —
// the text's LCP of a0 and a1 is lcp (exact) or at least lcp (no difference below min(la, lb)).
__device__ bool lyn_less(const u8* s, u32 a0, u32 a1, u32 b1, u32 N, u32* nsteps, u32 o0, u32& lcp, bool& exact) {
    const u32 lane = threadIdx.x & 63;
    const u32 la = a1 - a0, lb = b1 - a1, m = min(la, lb);
    u32 o = o0;
    // long common prefixes (periodic data: factors agree on KB): four 512-byte steps per
    // round trip while they lie wholly inside both factors and s[0, N) (larger trips measured
    // slower: a single wave is bound by its own load issue, not by the latency)
    while (o + 2048 <= m && (u64)a1 + o + 2048 + 12 <= N) {
        if (nsteps) *nsteps += 4;
        const u32 dpos = lyn_trip<4>(s, a0, a1, o, lane);
        if (dpos != ~0u) {
            lcp = dpos;
            exact = true;
            return s[a0 + dpos] < s[a1 + dpos];
        }
        o += 2048;
    }
    for (; o < m; o += 512) {
        if (nsteps) ++*nsteps;
        const u32 t = o + 8 * lane;
        u32 dpos = 0xFFFFFFFFu;
        if ((u64)a1 + o + 512 + 12 <= N) {
            if (t < m) {
                u64 d = load8u(s, a0 + t) ^ load8u(s, a1 + t);
                if (t + 8 > m) d &= (1ull << (8 * (m - t))) - 1ull;
                if (d) dpos = t + (u32)(__ffsll((long long)d) - 1) / 8;
            }
        } else {
            for (u32 e = 0; e < 8; ++e) {
                const u32 tt = t + e;
                if (tt < m && s[a0 + tt] != s[a1 + tt]) {
                    dpos = tt;
                    break;
                }
            }
        }
        const u64 bal = __ballot(dpos != 0xFFFFFFFFu);
        if (bal) {
            const u32 d = __builtin_amdgcn_readlane(dpos, __ffsll((long long)bal) - 1);
            lcp = d;
            exact = true;
            return s[a0 + d] < s[a1 + d];
        }
    }
    lcp = m;
    exact = false;
    return la < lb;
}

constexpr u32 MERGE_LDS = 8192;  // factor stack entries kept in LDS (more: the global stack)
constexpr u32 PRE_LDS = 512;     // stack entries with their 32-byte prefix in LDS

struct Pre {  // a factor's first 32 bytes as big-endian words
    uint4 a, b;
};

// Order of x, y on their first min(m, 32) bytes: -1, 1, or 0 (equal so far).
__device__ inline int pre_cmp(const Pre& x, const Pre& y, u32 m) {
    const u32 xs[8] = {x.a.x, x.a.y, x.a.z, x.a.w, x.b.x, x.b.y, x.b.z, x.b.w};
    const u32 ys[8] = {y.a.x, y.a.y, y.a.z, y.a.w, y.b.x, y.b.y, y.b.z, y.b.w};
    const u32 mm = min(m, 32u);
#pragma unroll
    for (u32 k = 0; k < 8; ++k) {
        if (4 * k >= mm) break;
        const u32 valid = mm - 4 * k;
        const u32 mask = valid >= 4 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (8 * valid));
        const u32 a = xs[k] & mask, b = ys[k] & mask;
        if (a != b) return a < b ? -1 : 1;
    }
    return 0;
}

// The first 32 bytes of the text at x as a Pre (bytes at or past e read as 0: the layout
// k_duval_span writes to fpre)
__device__ inline Pre text_pre(const u8* s, u32 x, u32 e) {
    u32 w[8];
    if (x + 48 <= e) {
#pragma unroll
        for (u32 k = 0; k < 4; ++k) {
            const u64 v = load8u(s, x + 8 * k);
            w[2 * k] = __builtin_bswap32((u32)v);
            w[2 * k + 1] = __builtin_bswap32((u32)(v >> 32));
        }
    } else {
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            u32 v4 = 0;
            for (u32 b = 0; b < 4; ++b) {
                const u32 y = x + 4 * k + b;
                v4 = (v4 << 8) | (y < e ? s[y] : 0u);
            }
            w[k] = v4;
        }
    }
    return Pre{make_uint4(w[0], w[1], w[2], w[3]), make_uint4(w[4], w[5], w[6], w[7])};
}

__device__ inline u32 rdl(u32 v, u32 l) { return (u32)__builtin_amdgcn_readlane((int)v, l); }
__device__ inline Pre rdl(const Pre& p, u32 l) {
    return Pre{make_uint4(rdl(p.a.x, l), rdl(p.a.y, l), rdl(p.a.z, l), rdl(p.a.w, l)),
               make_uint4(rdl(p.b.x, l), rdl(p.b.y, l), rdl(p.b.z, l), rdl(p.b.w, l))};
}

// One wave per block merges the span factorisations left to right (stack rule of
// k_duval_span).  A span's factor starts and 32-byte prefixes arrive 64 at a time, one per
// lane (the first DUVAL_PF from fpre, the later ones read from the text by their lanes, so
// spans of many factors — audio, images — do not pay a dependent global round trip per
// factor); the two stack entries under comparison are held in registers (the
// one below them is re-read from LDS only after a merge) and every entry keeps its
// prefix in LDS, so nearly all comparisons are decided in registers.  Only factors that
// agree on 32 bytes compare the text in global memory: the chain of ~800 dependent
// comparisons per 1 MiB text block cost ~0.7 us of load latency each.
__global__ __launch_bounds__(64) void k_duval_merge(Geom geo, u32 cpb, u32 span, const u8* s, const u32* fstart,
                                                    const uint4* fpre, const u32* nfac, u32* stack, u32* fcount,
                                                    u8* flag, u64* prof) {
    __shared__ u32 lstk[MERGE_LDS];
    __shared__ Pre lpre[PRE_LDS];
    __shared__ u32 lok[PRE_LDS];
    const u64 t0 = prof ? wall_clock64() : 0;
    u32 ncmp = 0, nstep = 0, npush = 0, nmerge = 0, nlyn = 0, nb_try = 0, nb_lim = 0, nb_hit = 0;
    // the last two text comparisons: pair (mxs, mys), LCP mL (exact: mex, then x < y is mlt)
    u32 mxs[2] = {~0u, ~0u}, mys[2] = {~0u, ~0u}, mL[2] = {0, 0};
    bool mex[2] = {false, false}, mlt[2] = {false, false};
    int mold = 0;  // the slot to replace
    u64 tlyn = 0;
    const u32 b = blockIdx.x, lane = threadIdx.x;
    const u32 base = geo.base(b), end = geo.end(b);
    // the stack never holds more entries than the span factorisations together: in LDS
    // when they fit (text: a few dozen), else in global memory (e.g. a run: n factors)
    u32 tot = 0;
    for (u32 k = lane; k < cpb; k += 64)
        if (base + k * span < end) tot += nfac[b * cpb + k];
    tot = wave_reduce(tot, OpAddU(), 0u);
    // written by lane 0, re-read uniformly: volatile keeps the reads off the scalar cache
    volatile u32* stk = tot <= MERGE_LDS ? lstk : stack + base;
    u32 sp = 0;
    // the stack's top entry (valid when sp > 0): start, prefix, prefix valid
    u32 top = 0, tok = 0;
    Pre tpre{};
    for (u32 k = 0; k < cpb; ++k) {
        const u32 c = b * cpb + k;
        const u32 lo = base + k * span;
        if (lo >= end) break;
        const u32 hi = min(lo + span, end);
        const u32 nf = nfac[c];
        // factors g0 .. g0 + 63 of the span: start, next start (or hi), prefix — one per lane
        static_assert(DUVAL_PF == 64, "group 0 of the span comes from fpre");
        u32 g0 = 0;
        u32 vst = lane < nf ? fstart[lo + lane] : hi;
        u32 vnx = lane + 1 < nf ? fstart[lo + lane + 1] : hi;
        Pre vpr{};
        if (lane < nf) {
            vpr.a = fpre[((u64)c * DUVAL_PF + lane) * 2];
            vpr.b = fpre[((u64)c * DUVAL_PF + lane) * 2 + 1];
        }
        u32 t = 0;
        while (t < nf) {
            if (t - g0 >= 64) {
                g0 += 64;
                const u32 gi = g0 + lane;
                vst = gi < nf ? fstart[lo + gi] : hi;
                vnx = gi + 1 < nf ? fstart[lo + gi + 1] : hi;
                if (gi < nf) vpr = text_pre(s, vst, end);
            }
            // Batch absorption: while the top T keeps absorbing the span's factors (T' = T f_t
            // ... f_(i-1) < f_i; audio and images merge thousands of span factors into a few),
            // the decisions for a whole group come from one lane-parallel prefix comparison
            // against T's prefix (T' starts with T).  Valid while nothing below T can merge
            // into T': the entry below differs from T within T's first bytes and is larger.
            // When the entry below, x, shares T's first bytes (periodic data: the checker BMP's
            // factors), T' = T f_t ... stays no larger than x while it is a prefix of x or
            // first differs from x downwards: the text LCP of x and T (memoised, extended to
            // the group's reach) bounds how far T' may grow (xlim) without x absorbing it.
            if (sp >= 1 && tok) {
                bool safe = sp == 1;
                u32 xlim = 0;
                const u32 lT = rdl(vst, t - g0) - top;  // |T'| before factor t
                if (sp >= 2 && sp - 2 < PRE_LDS && lok[sp - 2]) {
                    const u32 bst = stk[sp - 2], lx = top - bst;
                    const int cb = pre_cmp(lpre[sp - 2], tpre, min(lx, lT));
                    safe = cb > 0;
                    if (cb == 0 && min(lx, lT) > 32) {
                        ++nb_try;
                        const u32 last = min(63u, nf - 1 - g0);
                        const u32 need = min(lx, rdl(vnx, last) - top);  // the group's reach
                        const int hit = bst == mxs[0] && top == mys[0] ? 0 : bst == mxs[1] && top == mys[1] ? 1 : -1;
                        u32 L;
                        bool ex;
                        if (hit >= 0 && (mex[hit] || mL[hit] >= need)) {
                            L = mL[hit];
                            ex = mex[hit];
                        } else {
                            const u32 o0 = max(32u, hit >= 0 ? mL[hit] : 0u);
                            (void)lyn_less(s, bst, top, top + need, (u32)geo.N, prof ? &nstep : nullptr, min(o0, need),
                                           L, ex);
                            const int sl = hit >= 0 ? hit : mold;
                            mxs[sl] = bst;
                            mys[sl] = top;
                            mL[sl] = L;
                            mex[sl] = ex;
                            mlt[sl] = ex && L < need ? s[bst + L] < s[top + L] : false;
                            mold = 1 - sl;
                        }
                        if (ex && L < need) {
                            // x and T' first differ at L (for every T' reaching past L)
                            if (s[bst + L] > s[top + L]) safe = L < lx;  // x stays larger
                            else xlim = min(L, lx - 1);
                        } else {
                            xlim = min(L, lx - 1);  // T' a prefix of x up to L
                        }
                    }
                }
                if (safe || xlim) {
                    nb_lim += xlim ? 1u : 0u;
                    const u32 l0 = t - g0;
                    bool ok = false;
                    if (lane >= l0 && g0 + lane < nf) {
                        const u32 la = vst - top, lb = vnx - vst, m = min(la, lb);
                        const int cr = pre_cmp(tpre, vpr, m);
                        bool dec = cr != 0 || m <= 32;
                        bool lt = cr < 0 || (cr == 0 && m <= 32 && la < lb);
                        if (!dec && m <= 512) {
                            // T' and f agree on 32 bytes (periodic data): the lane compares
                            // the rest itself, 8 bytes per step (the text has 64 bytes of slack)
                            dec = true;
                            lt = la < lb;
                            for (u32 o = 32; o < m; o += 8) {
                                u64 d = load8u(s, top + o) ^ load8u(s, vst + o);
                                if (o + 8 > m) d &= (1ull << (8 * (m - o))) - 1ull;
                                if (d) {
                                    const u32 k8 = (u32)(__ffsll((long long)d) - 1) >> 3;
                                    lt = s[top + o + k8] < s[vst + o + k8];
                                    break;
                                }
                            }
                        }
                        ok = dec && lt && (safe || vnx - top <= xlim);
                    }
                    const u64 okm = __ballot(ok) >> l0;
                    const u32 k = okm == ~0ull ? 64u : (u32)__ffsll((long long)~okm) - 1;
                    if (k) {
                        ++nb_hit;
                        t += k;
                        npush += k;
                        nmerge += k;
                        continue;
                    }
                }
            }
            const u32 cached = 1u;
            const u32 r = rdl(vst, t - g0);
            const u32 frontier = rdl(vnx, t - g0);
            const Pre rp = rdl(vpr, t - g0);
            if (lane == 0) {
                stk[sp] = r;
                if (sp < PRE_LDS) {
                    lok[sp] = cached;
                    lpre[sp] = rp;
                }
            }
            ++sp;
            ++npush;
            // y = the top (r, or what r merged into), x = the entry below it
            u32 ys = r, yok = cached;
            Pre yp = rp;
            u32 xs = top, xok = tok;
            Pre xp = tpre;
            bool merged = false;
            while (sp >= 2) {
                ++ncmp;
                const u32 la = ys - xs, lb = frontier - ys, m = min(la, lb);
                bool less;
                int cr = 0;
                if (xok && yok) cr = pre_cmp(xp, yp, m);
                if (cr)
                    less = cr < 0;
                else if (xok && yok && m <= 32)
                    less = la < lb;
                else {
                    // memo of the last two text comparisons (pairs alternate: the checker
                    // BMP's merges re-compare one long factor against a growing one between
                    // short comparisons): a known pair resumes past its known-equal bytes, or
                    // is decided by its exact LCP
                    const int hit = xs == mxs[0] && ys == mys[0] ? 0 : xs == mxs[1] && ys == mys[1] ? 1 : -1;
                    if (hit >= 0 && mex[hit]) {
                        less = mL[hit] < m ? mlt[hit] : la < lb;
                    } else {
                        const u32 o0 = max(xok && yok ? 32u : 0u, hit >= 0 ? min(mL[hit], m) : 0u);
                        const u64 tl = prof ? wall_clock64() : 0;
                        u32 L;
                        bool ex;
                        less = lyn_less(s, xs, ys, frontier, (u32)geo.N, prof ? &nstep : nullptr, o0, L, ex);
                        const int sl = hit >= 0 ? hit : mold;
                        mxs[sl] = xs;
                        mys[sl] = ys;
                        mL[sl] = L;
                        mex[sl] = ex;
                        mlt[sl] = less;
                        if (prof) {
                            ++nlyn;
                            tlyn += wall_clock64() - tl;
                        }
                    }
                    mold = hit >= 0 ? 1 - hit : 1 - mold;  // the slot not used now is replaced next
                }
                if (!less) break;
                ++nmerge;
                --sp;  // x absorbs y: the merged factor keeps x's start and prefix
                ys = xs;
                yok = xok;
                yp = xp;
                merged = true;
                if (sp >= 2) {
                    __builtin_amdgcn_s_waitcnt(0);
                    xs = stk[sp - 2];
                    xok = sp - 2 < PRE_LDS ? lok[sp - 2] : 0u;
                    if (xok) xp = lpre[sp - 2];
                }
            }
            top = ys;
            tok = yok;
            tpre = yp;
            ++t;
            if (!merged) break;
        }
        // remaining right factors cannot merge: append in bulk (prefixes of the entries that
        // land in the LDS prefix cache read from the text, lane-parallel)
        for (u32 o = t; o < nf; o += 64) {
            const u32 idx = o + lane;
            if (idx < nf) {
                const u32 d = sp + (idx - t);
                const u32 sv = fstart[lo + idx];
                stk[d] = sv;
                if (d < PRE_LDS) {
                    lok[d] = 1u;
                    lpre[d] = text_pre(s, sv, end);
                }
            }
        }
        if (t < nf) {
            sp += nf - t;
            top = fstart[lo + nf - 1];  // the new top
            tok = 1u;
            tpre = text_pre(s, top, end);
        }
        __builtin_amdgcn_s_waitcnt(0);
    }
    // the block's factor starts: flags, and the sorted list at stack + base (in place when
    // the stack spilled to global memory)
    for (u32 i = lane; i < sp; i += 64) {
        const u32 v = stk[i];
        flag[v] = 1;
        if (tot <= MERGE_LDS) stack[base + i] = v;
    }
    if (lane == 0) fcount[b] = sp;
    if (prof && lane == 0) {
        atomicAdd((unsigned long long*)&prof[11], (unsigned long long)(wall_clock64() - t0));
        atomicMax((unsigned long long*)&prof[12], (unsigned long long)(wall_clock64() - t0));
        atomicAdd((unsigned long long*)&prof[13], (unsigned long long)ncmp);
        atomicAdd((unsigned long long*)&prof[14], (unsigned long long)nstep);
        atomicAdd((unsigned long long*)&prof[15], (unsigned long long)tot);
        atomicAdd((unsigned long long*)&prof[16], (unsigned long long)npush);
        atomicAdd((unsigned long long*)&prof[17], (unsigned long long)nmerge);
        atomicAdd((unsigned long long*)&prof[18], (unsigned long long)nlyn);
        atomicAdd((unsigned long long*)&prof[19], (unsigned long long)tlyn);
        atomicAdd((unsigned long long*)&prof[20], (unsigned long long)sp);
        atomicAdd((unsigned long long*)&prof[21], (unsigned long long)nb_try);
        atomicAdd((unsigned long long*)&prof[22], (unsigned long long)nb_lim);
        atomicAdd((unsigned long long*)&prof[23], (unsigned long long)nb_hit);
    }
}

// prevc[p] = the character preceding p cyclically inside its factor (streaming pass), so
// the BBWT gather needs one random byte per slot instead of a factor lookup + a byte.
__global__ void k_prevc1(Geom geo, const u8* text, const u8* flag, Factors fac, u8* prevc) {
    for (u32 p = blockIdx.x * blockDim.x + threadIdx.x; p < geo.N; p += gridDim.x * blockDim.x) {
        u32 src = p - 1;
        if (flag[p]) {  // factor start: its predecessor is the factor's last byte
            u32 fs, m;
            fac.locate(geo, p, fs, m);
            src = fs + m - 1;
        }
        prevc[p] = text[src];
    }
}

// 16 positions per thread: flags and output as 16-byte words, text bytes p-1 .. p+14 from
// aligned words (text 16-byte aligned; the launcher checks).  A factor start's end is the
// next flag inside the 16 (every block's first position is flagged, so a flag past the
// block's end is that end) or, past them, a search of the block's factor starts.
__global__ __launch_bounds__(256) void k_prevc(Geom geo, const u8* text, const u8* flag, Factors fac, u8* prevc) {
    const u32 p0 = (blockIdx.x * 256 + threadIdx.x) * 16;
    const u32 N = (u32)geo.N;
    if (p0 >= N) return;
    if (p0 + 16 > N || p0 < 4) {
        for (u32 p = p0; p < min(p0 + 16, N); ++p) {
            u32 src = p - 1;
            if (flag[p]) {
                u32 fs, m;
                fac.locate(geo, p, fs, m);
                src = fs + m - 1;
            }
            prevc[p] = text[src];
        }
        return;
    }
    const uint4 fv = *reinterpret_cast<const uint4*>(flag + p0);
    const u32 fw[4] = {fv.x, fv.y, fv.z, fv.w};
    u32 fm = 0;  // bit e: position p0+e starts a factor
#pragma unroll
    for (int e = 0; e < 16; ++e) fm |= ((fw[e >> 2] >> (8 * (e & 3))) & 1u) << e;
    const u32* tw = reinterpret_cast<const u32*>(text + p0) - 1;  // bytes p0-4 .. p0+15
    u32 w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = tw[i];
    u32 o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        // byte p0+e-1 = byte (e+3) of the 20-byte window starting at p0-4
        u32 c = (w[(e + 3) >> 2] >> (8 * ((e + 3) & 3))) & 0xFF;
        if ((fm >> e) & 1u) {  // factor start: the factor's last byte
            const u32 rest = fm >> (e + 1);
            u32 last;
            if (rest) {
                last = p0 + e + __builtin_ctz(rest);  // next start - 1
            } else {
                u32 fs, m;
                fac.locate(geo, p0 + e, fs, m);
                last = fs + m - 1;
            }
            c = text[last];
        }
        o[e >> 2] |= c << (8 * (e & 3));
    }
    *reinterpret_cast<uint4*>(prevc + p0) = make_uint4(o[0], o[1], o[2], o[3]);
}

// 4096 slots per workgroup, XCD-remapped so a block's slots (and its 1 MiB of prevc)
// stay on one XCD's L2
__global__ __launch_bounds__(256) void k_bbwt_gather(Geom geo, const u32* SA, const u8* prevc, u8* out) {
    const u32 g0 = xcd_tile() * 4096u;
#pragma unroll
    for (u32 j = 0; j < 16; ++j) {
        const u32 g = g0 + j * 256 + threadIdx.x;
        if (g < geo.N) out[g] = prevc[SA[g]];
    }
}

// Early BBWT gather (bbwt_early_round): the slots outside the still-active segments of a
// doubling round hold their final SA entries — later rounds only reorder slots inside those
// segments — so their BBWT bytes can be gathered while the last rounds run.  BM: one bit per
// slot, set for the slots of the active segments (one thread per segment; words inside a
// segment are written whole, the partial end words by atomic OR).
__global__ __launch_bounds__(256) void k_mark_active(const Seg* cur, const u32* ncur, u32 bound, u64* bm) {
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    if (i >= min(bound, *ncur)) return;
    const Seg sg = cur[i];
    if (!sg.len) return;
    const u32 a = sg.start, e = sg.start + sg.len;  // [a, e)
    const u32 wa = a >> 6, we = (e - 1) >> 6;
    const u64 ma = ~0ull << (a & 63), me = ~0ull >> (63 - ((e - 1) & 63));
    if (wa == we) {
        atomicOr((unsigned long long*)&bm[wa], (unsigned long long)(ma & me));
        return;
    }
    atomicOr((unsigned long long*)&bm[wa], (unsigned long long)ma);
    for (u32 w = wa + 1; w < we; ++w) bm[w] = ~0ull;
    atomicOr((unsigned long long*)&bm[we], (unsigned long long)me);
}

// k_bbwt_gather for the slots whose BM bit is set only: 16 consecutive slots per thread, one
// 16-bit piece of the mask each (most are zero: a few percent of the slots stay active)
__global__ __launch_bounds__(256) void k_bbwt_gather_m(Geom geo, const u32* SA, const u8* prevc, u8* out,
                                                       const u64* bm) {
    const u32 g0 = xcd_tile() * 4096u + 16u * threadIdx.x;
    if (g0 >= geo.N) return;
    u32 m = (u32)(bm[g0 >> 6] >> (g0 & 63)) & 0xFFFFu;
    while (m) {
        const u32 g = g0 + (u32)__ffs(m) - 1;
        if (g < geo.N) out[g] = prevc[SA[g]];
        m &= m - 1;
    }
}

}  // namespace

// The doubling round after whose classification the early BBWT gather starts.  Round 3 (text:
// ~0.2 % of the slots still active): one A/B call, two runs each (profiles/r05/ab_early_gather_*):
// the sort stream ends 0.4 ms sooner (ms_sa 32.2 -> 31.8 ms); config 4's shard 6.26 / 6.41 ->
// 6.20 / 6.23 ms.  Round 2 (~9 % active) costs more than it saves (35.0 ms: its gather competes
// with round 2's sorts and the parse).
u32 bbwt_early_round() { return 3u; }

void launch_mark_active(const Seg* cur, const u32* ncur_dev, u32 bound, u64* bm, hipStream_t s) {
    if (bound) k_mark_active<<<(bound + 255) / 256, 256, 0, s>>>(cur, ncur_dev, bound, bm);
}
void launch_bbwt_gather_masked(const Geom& geo, const u32* SA, const u8* prevc, u8* out, const u64* bm,
                               hipStream_t s) {
    if (!geo.N) return;
    k_bbwt_gather_m<<<(u32)((geo.N + 4095) / 4096), 256, 0, s>>>(geo, SA, prevc, out, bm);
}

// KOLM_DUVAL_PROF=1 (debug): per-phase wall-clock of k_duval_span and k_duval_merge
u64* dprof_buf() {
    static u64* prof = nullptr;
    static const bool dp = getenv("KOLM_DUVAL_PROF") && atoi(getenv("KOLM_DUVAL_PROF"));
    if (dp && !prof) {
        KOLM_HIP_CHECK(hipMalloc(&prof, 40 * sizeof(u64)));
        KOLM_HIP_CHECK(hipMemset(prof, 0, 40 * sizeof(u64)));
    }
    return prof;
}

// Lyndon factorisation of every block (parallel Duval + merge) -> factor-start lists,
// flags and FEd.
// Bytes per Duval span: 8 KiB (64-thread workgroups) for every batch: the span pass's tree
// levels are latency-bound per workgroup, and the merge absorbs the extra span factorisations
// in batches.  Against 32 KiB spans: config 5 span 1.82 -> 1.19 ms, merge 0.18 -> 0.41 ms, 8.82 ->
// 8.54 ms per call; 256 MiB text (two alternating A/B runs): Lyndon family 4.37 -> 3.94 ms, step
// 37.08 -> 36.58 ms.  Every tree level merges with lane groups (span_less_grp; a thread per merge
// measured slower, round 5), whole waves from level DUVAL_WAVE_W.
u32 duval_span_bytes(const Geom& geo) {
    (void)geo;
    return DUVAL_CH * 64;
}

void launch_lyndon(const Geom& geo, const u8* text, u8* flag, u8* FEd, u32* fstart, uint4* fpre, u32* nfac,
                   u32* stack, u32* fcount, u32* tile_tmp, hipStream_t s, KTimer* kt) {
    if (!geo.N) return;
    TileGeom tg{geo, (geo.bs + TILE - 1) / TILE};
    const u32 nt = tg.tpb * geo.nb;
    u32* A = tile_tmp;        // [nt]
    u32* B = tile_tmp + nt;   // [nt]
    const u32 span = duval_span_bytes(geo);
    const u32 cpb = (geo.bs + span - 1) / span;
    const u32 nch = cpb * geo.nb;
    const u64 N = geo.N;
    KOLM_HIP_CHECK(hipMemsetAsync(flag, 0, geo.N, s));
    {
        KScope k(kt, KT_LYNDON, "k_duval_span", N);  // text once (+ 4 B per factor start)
        k_duval_span<64><<<nch, 64, 0, s>>>(geo, cpb, text, fstart, fpre, nfac, dprof_buf(), DUVAL_WAVE_W, 1u);
    }
    {
        KScope k(kt, KT_LYNDON, "k_duval_merge", (u64)nch * 8);
        k_duval_merge<<<geo.nb, 64, 0, s>>>(geo, cpb, span, text, fstart, fpre, nfac, stack, fcount, flag,
                                             dprof_buf());
    }
    if (u64* prof = dprof_buf()) {
        u64 h[40];
        KOLM_HIP_CHECK(hipStreamSynchronize(s));
        KOLM_HIP_CHECK(hipMemcpy(h, prof, sizeof h, hipMemcpyDeviceToHost));
        KOLM_HIP_CHECK(hipMemset(prof, 0, 40 * sizeof(u64)));
        fprintf(stderr, "[kolm] duval_span us per workgroup (mean/max):");
        for (int k = 0; k < 11; ++k) fprintf(stderr, " %d:%.1f/%.1f", k, (double)h[k] / nch / 100.0, (double)h[24 + k] / 100.0);
        fprintf(stderr, " | merge us per block mean %.1f max %.1f, compares/block %.1f, 512-B steps/block %.1f, "
                "span factors/block %.1f\n", (double)h[11] / geo.nb / 100.0, (double)h[12] / 100.0,
                (double)h[13] / geo.nb, (double)h[14] / geo.nb, (double)h[15] / geo.nb);
        fprintf(stderr, "[kolm] merge per block: pushes %.1f merges %.1f text compares %.1f (%.1f us), final factors %.1f; "
                "batch: LCP-bounded tries %.1f, bounded %.1f, batches taken %.1f\n",
                (double)h[16] / geo.nb, (double)h[17] / geo.nb, (double)h[18] / geo.nb, (double)h[19] / geo.nb / 100.0,
                (double)h[20] / geo.nb, (double)h[21] / geo.nb, (double)h[22] / geo.nb, (double)h[23] / geo.nb);
    }
    {
        KScope k(kt, KT_LYNDON, "k_tile_starts", N);
        k_tile_starts<<<nt, WG, 0, s>>>(tg, flag, A);
        k_tiles_scan<true, false><<<geo.nb, WG, 0, s>>>(A, B, tg.tpb, BIG);
    }
    {
        KScope k(kt, KT_LYNDON, "k_fed", 2 * N);  // flag 1 + FEd 1
        k_fed<<<nt, WG, 0, s>>>(tg, flag, B, FEd);
    }
}

void launch_prevc(const Geom& geo, const u8* text, const u8* flag, Factors fac, u8* prevc, hipStream_t s) {
    if (!geo.N) return;
    const u32 grid = (u32)std::min<u64>((geo.N + 255) / 256, 65535);
    if (((uintptr_t)text & 15) == 0)
        k_prevc<<<(u32)((geo.N + 4095) / 4096), 256, 0, s>>>(geo, text, flag, fac, prevc);
    else  // caller's device buffer not 16-byte aligned
        k_prevc1<<<grid, 256, 0, s>>>(geo, text, flag, fac, prevc);
}

void launch_bbwt_gather(const Geom& geo, const u32* SA, const u8* prevc, u8* out, hipStream_t s) {
    if (!geo.N) return;
    k_bbwt_gather<<<(u32)((geo.N + 4095) / 4096), 256, 0, s>>>(geo, SA, prevc, out);
}

}  // namespace kolm
