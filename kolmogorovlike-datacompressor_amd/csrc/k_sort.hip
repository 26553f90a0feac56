// Suffix sorting for the BBWT (gfx950): segmented prefix doubling over a batch of blocks.
//
// Replaces the reference's per-factor comparison-sort prefix doubling + k-way heap merge
// (PY:351-423, CPP:939-1093).  Two passes use these kernels:
//   * linear  — suffix order of each block (sentinel < every byte), used for the Lyndon
//               factorisation (factor starts = left-to-right minima of the inverse SA,
//               replacing Duval PY:326-349) and for the LZ77 3-gram chains;
//   * cyclic  — omega-order of all rotations of all Lyndon factors of a block
//               (succ(p) = next position inside p's factor, cyclically).  A stable sort
//               of positions by that order with ties in position order IS the BBWT
//               order of PY's heap merge (ties (fi, i) = position order, PY:408-409).
//
// State per position: SA (positions in current order), RK (rank = SA index of the start
// of the position's group), K2 (sort key of the current round, per SA slot).  Each round
// refines every unsorted group ("segment") by the key of this round:
//   round 0:  packed leading characters (linear: 3 x 9-bit chars with 0 = end;
//             cyclic: 4 chars of the rotation)
//   round r:  RK[succ^h(p)] with h = h0 * 2^(r-1)  (prefix doubling).
// Segments are processed by size: len <= TILE in one workgroup (LDS bitonic sort of
// (key, position), which yields position order among equal keys), longer ones by stable
// 8-bit MSD radix passes (LDS histograms, per-segment tile scan, stable scatter) until
// their buckets fit a tile.  A group splitting or not is tracked per block: in cyclic
// mode a block whose groups did not split in a doubling round can never split again
// (E_2h == E_h => fixed point) and is retired.  See DESIGN.md §4.
#include "kolm_internal.h"

namespace kolm {

void geom_init(Geom& g, u64 N, u32 bs) {
    g.N = N;
    g.bs = bs;
    g.nb = bs ? (u32)((N + bs - 1) / bs) : 0;
    u32 s = 0;
    while ((1ull << s) < bs) ++s;
    g.shift = 32 + s;
    g.magic = ((1ull << g.shift) / bs) + 1;
}

// ------------------------------------------------------------------------------------
// block-wide scans (256 threads = 4 waves of 64)
// ------------------------------------------------------------------------------------
struct OpMax {
    __device__ u32 operator()(u32 a, u32 b) const { return a > b ? a : b; }
};
struct OpMin {
    __device__ u32 operator()(u32 a, u32 b) const { return a < b ? a : b; }
};
struct OpAdd {
    __device__ u32 operator()(u32 a, u32 b) const { return a + b; }
};

// Exclusive scan over the threads of the workgroup (REV: from the last thread down).
template <bool REV, class Op, u32 NW = WG / 64>
__device__ inline u32 wg_excl_scan(u32 v, Op op, u32 ident, u32* sh /*[NW]*/) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u32 incl = REV ? wave_incl_scan_rev(v, op, ident) : wave_incl_scan(v, op, ident);
    const u32 ex = REV ? KOLM_DPP(ident, incl, DPP_WAVE_SHL1, 0xF) : KOLM_DPP(ident, incl, DPP_WAVE_SHR1, 0xF);
    if (REV ? lane == 0 : lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = ident;
    if (!REV) {
        for (u32 i = 0; i < w; ++i) carry = op(carry, sh[i]);
    } else {
        for (u32 i = w + 1; i < NW; ++i) carry = op(carry, sh[i]);
    }
    __syncthreads();
    return op(carry, ex);
}

__device__ inline int size_class(u32 len) { return len <= 1 ? 0 : 32 - __clz(len - 1); }

// ------------------------------------------------------------------------------------
// keys
// ------------------------------------------------------------------------------------
__device__ inline u32 cyc_succ(const SortArgs& a, u32 p, u32 h) {
    u32 fs, m;
    a.fac.locate(a.geo, p, fs, m);
    u32 hm = h < m ? h : h % m;
    u32 t = (p - fs) + hm;
    if (t >= m) t -= m;
    return fs + t;
}

// characters off .. off+3 of the rotation starting at p (cyclic inside p's Lyndon factor),
// the first most significant
__device__ inline u32 cyc_chars(const SortArgs& a, u32 p, u32 off) {
    if (a.FEd[p] > off + 3) {  // the 4 characters do not wrap
        const u8* t = a.text + p + off;
        return ((u32)t[0] << 24) | ((u32)t[1] << 16) | ((u32)t[2] << 8) | t[3];
    }
    u32 fs, m;
    a.fac.locate(a.geo, p, fs, m);
    u32 t = (p - fs) + off % m, k = 0;
    if (t >= m) t -= m;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        k = (k << 8) | a.text[fs + t];
        if (++t == m) t = 0;
    }
    return k;
}

__device__ inline u32 make_key(const SortArgs& a, u32 p, u32 base, u32 end) {
    if (a.KP) return a.KP[p];
    if (a.initial) {
        if (!a.cyclic) {
            u32 c0 = (u32)a.text[p] + 1;
            u32 c1 = p + 1 < end ? (u32)a.text[p + 1] + 1 : 0;
            u32 c2 = p + 2 < end ? (u32)a.text[p + 2] + 1 : 0;
            return (c0 << 18) | (c1 << 9) | c2;
        }
        return cyc_chars(a, p, 0);
    }
    if (!a.cyclic) {
        const u32 q = p + a.h;
        return q < end ? a.RK[q] - base + 1 : 0;
    }
    if (a.h < a.FEd[p]) return a.RK[p + a.h] - base;  // no wrap: no factor lookup
    return a.RK[cyc_succ(a, p, a.h)] - base;
}

// Keys of every position in position order: the factor record and RK[succ^h(p)] are read
// (nearly) sequentially here, so the per-slot key generation needs a single random gather.
__global__ __launch_bounds__(256) void k_keypos(SortArgs a, u32* KP) {
    a.KP = nullptr;
    for (u32 p = blockIdx.x * blockDim.x + threadIdx.x; p < a.geo.N; p += gridDim.x * blockDim.x) {
        const u32 b = a.geo.block_of(p);
        KP[p] = make_key(a, p, a.geo.base(b), a.geo.end(b));
        if (a.initial && a.KA) a.KA[p] = cyc_chars(a, p, 4);
    }
}

// Cyclic keys by position, 16 consecutive positions per thread with 16-byte loads/stores
// (the grid-stride form above keeps one load per thread in flight).  Positions whose
// rotation wraps inside the next h (round 0: 4) characters take the factor-record path.
__global__ __launch_bounds__(256) void k_keypos_cyc(SortArgs a, u32* KP) {
    a.KP = nullptr;
    const u32 p0 = (blockIdx.x * 256 + threadIdx.x) * 16;
    const u32 N = (u32)a.geo.N;
    if (p0 >= N) return;
    if (p0 + 16 > N) {  // ragged end of the batch
        for (u32 p = p0; p < N; ++p) {
            const u32 b = a.geo.block_of(p);
            KP[p] = make_key(a, p, a.geo.base(b), a.geo.end(b));
            if (a.initial && a.KA) a.KA[p] = cyc_chars(a, p, 4);
        }
        return;
    }
    const uint4 dv = *reinterpret_cast<const uint4*>(a.FEd + p0);
    const u32 dw[4] = {dv.x, dv.y, dv.z, dv.w};
    u32 key[16], ka[16];
    if (a.initial) {
        // bytes p0 .. p0+23 cover the 8-character windows of the 16 positions
        const u32* tw = reinterpret_cast<const u32*>(a.text + p0);
        u32 w[6];
#pragma unroll
        // a word that starts before N is inside the allocation (4-byte granular); bytes
        // past N only feed positions that take the factor-record path (FEd <= 3 / 7)
        for (int i = 0; i < 6; ++i) w[i] = (p0 + 4 * i < N) ? tw[i] : 0u;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const u32 lo = w[e >> 2], mid = w[(e >> 2) + 1], hi = w[(e >> 2) + 2];
            key[e] = __builtin_bswap32(__builtin_amdgcn_alignbyte(mid, lo, e & 3));  // bytes p..p+3, first most significant
            ka[e] = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, mid, e & 3));   // bytes p+4..p+7
        }
    } else {
        if (p0 + a.h + 16 <= N) {
            const uint4* rk = reinterpret_cast<const uint4*>(a.RK + p0 + a.h);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint4 r = rk[i];
                key[4 * i] = r.x;
                key[4 * i + 1] = r.y;
                key[4 * i + 2] = r.z;
                key[4 * i + 3] = r.w;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) key[e] = p0 + e + a.h < N ? a.RK[p0 + e + a.h] : 0u;
        }
    }
    const u32 b0 = a.geo.block_of(p0), base0 = a.geo.base(b0), end0 = a.geo.end(b0);
    const u32 need = a.initial ? 3u : a.h;  // fast path iff need < FEd[p]
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const u32 p = p0 + e;
        const u32 d = (dw[e >> 2] >> (8 * (e & 3))) & 0xFF;
        if (need < d && p < end0) {
            if (!a.initial) key[e] -= base0;
        } else {
            const u32 b = a.geo.block_of(p);
            key[e] = make_key(a, p, a.geo.base(b), a.geo.end(b));
        }
    }
    uint4* out = reinterpret_cast<uint4*>(KP + p0);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = make_uint4(key[4 * i], key[4 * i + 1], key[4 * i + 2], key[4 * i + 3]);
    if (a.initial && a.KA) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const u32 d = (dw[e >> 2] >> (8 * (e & 3))) & 0xFF;
            if (d <= 7) ka[e] = cyc_chars(a, p0 + e, 4);
        }
        uint4* oa = reinterpret_cast<uint4*>(a.KA + p0);
#pragma unroll
        for (int i = 0; i < 4; ++i) oa[i] = make_uint4(ka[4 * i], ka[4 * i + 1], ka[4 * i + 2], ka[4 * i + 3]);
    }
}

// ------------------------------------------------------------------------------------
// setup kernels
// ------------------------------------------------------------------------------------
__global__ void k_iota(u32* SA, u32 N) {
    for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) SA[i] = i;
}

__global__ void k_block_segs(Seg* segs, Geom geo) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < geo.nb) segs[b] = Seg{geo.base(b), geo.end(b) - geo.base(b)};
}

// Persistent two-pass classification (list order is irrelevant: every segment is refined
// independently).  A bounded grid of workgroups strides over the segment list: pass 1
// counts per class (wave-level aggregation into LDS), then ONE global atomic per class
// per workgroup reserves its ranges, pass 2 re-reads its segments and writes them.
// (One atomic per class per 256 segments serialised on a handful of hot counter words:
// 4.3 -> 0.9 ms per step.)
__device__ inline int seg_class(const SortArgs& a, const Seg* cur, u32 ncur, u32 i, Seg& s) {
    s = Seg{0, 0};
    if (i >= ncur) return -1;
    s = cur[i];
    if (a.cyclic && a.blk_done[a.geo.block_of(s.start)]) return -1;
    return s.len > (u32)TILE ? NCLASS : size_class(s.len);
}

// MODE 0: all segments placed by per-workgroup reservations (list order arbitrary).
// MODE 1: counts as MODE 0 plus per-(class, bin) counts; only the large segments are written.
// MODE 2: small segments placed at their bin's offset (after k_bin_scan).
// ncur_dev (when set): the list's length as the previous round left it in device memory, so
// the host does not wait for the round's end to launch the next one (the grid covers a bound)
template <int MODE>
__global__ __launch_bounds__(256) void k_classify(const Seg* cur, u32 ncur_in, const u32* ncur_dev, SortArgs a,
                                                  Lists L, Level lv, Bins bn) {
    const u32 ncur = ncur_dev ? *ncur_dev : ncur_in;
    __shared__ u32 lcnt[NCLASS + 1], lbase[NCLASS + 1], lel[NCLASS + 1], lcur[NCLASS + 1];
    __shared__ u32 lact, ltiles, ltb;
    const u32 tid = threadIdx.x, lane = tid & 63;
    if (tid <= NCLASS) {
        lcnt[tid] = 0;
        lel[tid] = 0;
        lcur[tid] = 0;
    }
    if (tid == 0) {
        lact = 0;
        ltiles = 0;
    }
    __syncthreads();
    // each workgroup walks one contiguous share of the list (concurrent workgroups then work
    // in different regions of it, so the per-(class, bin) atomics of MODE 1 / 2 do not pile on
    // the same few counters)
    const u32 per = ((ncur + gridDim.x * 256 - 1) / (gridDim.x * 256)) * 256;
    const u32 wbeg = a.cls_chunk ? min(blockIdx.x * per, ncur) : blockIdx.x * 256;
    const u32 wend = a.cls_chunk ? min(wbeg + per, ncur) : ncur;
    const u32 stride = a.cls_chunk ? 256u : gridDim.x * 256;
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (MODE == 2) {
        for (u32 i0 = wbeg; i0 < wend; i0 += stride) {
            Seg s;
            const int c = seg_class(a, cur, wend, i0 + tid, s);
            const u32 key = (c >= 0 && c < NCLASS) ? (u32)c * CLS_NBIN + (s.start >> bn.bsh) : ~0u;
            u64 pend = __ballot(key != ~0u);
            u32 dst = 0;
            while (pend) {
                const u32 f = (u32)__ffsll((long long)pend) - 1;
                const u32 kk = __builtin_amdgcn_readlane(key, f);
                const u64 m = __ballot(key == kk);
                u32 base = 0;
                if (lane == f) base = bn.cnt[kk] + atomicAdd(&bn.fill[kk], (u32)__popcll(m));
                base = __builtin_amdgcn_readlane(base, f);
                if (key == kk) dst = base + (u32)__popcll(m & lt);
                pend &= ~m;
            }
            if (key != ~0u) L.cls[c][dst] = Seg{s.start, s.len | SEG_FIRST};
        }
        return;
    }
    // pass 1: counts
    for (u32 i0 = wbeg; i0 < wend; i0 += stride) {
        Seg s;
        const int c = seg_class(a, cur, wend, i0 + tid, s);
        if (MODE == 1) {
            const u32 key = (c >= 0 && c < NCLASS) ? (u32)c * CLS_NBIN + (s.start >> bn.bsh) : ~0u;
            u64 bp = __ballot(key != ~0u);
            while (bp) {
                const u32 f = (u32)__ffsll((long long)bp) - 1;
                const u32 kk = __builtin_amdgcn_readlane(key, f);
                const u64 m = __ballot(key == kk);
                if (lane == f) atomicAdd(&bn.cnt[kk], (u32)__popcll(m));
                bp &= ~m;
            }
        }
        u64 pend = __ballot(c >= 0);
        u32 nt = c == NCLASS ? (s.len + TILE - 1) / TILE : 0u;
        nt = wave_reduce(nt, OpAddU(), 0u);
        if (lane == 0 && nt) atomicAdd(&ltiles, nt);
        if (nt) {  // the longest large segment (the host picks the medium sort or the MSD levels)
            const u32 lm = wave_reduce(c == NCLASS ? (s.len & SEG_LEN) : 0u, OpMaxU(), 0u);
            if (lane == 0) atomicMax(L.lmax, lm);
        }
        while (pend) {
            const u32 f = (u32)__ffsll((long long)pend) - 1;
            const int cc = __builtin_amdgcn_readlane(c, f);
            const u64 m = __ballot(c == cc);
            const u32 v = wave_reduce(c == cc ? s.len : 0u, OpAddU(), 0u);
            if (lane == f) {
                atomicAdd(&lcnt[cc], (u32)__popcll(m));
                atomicAdd(&lel[cc], v);
                atomicAdd(&lact, v);
            }
            pend &= ~m;
        }
    }
    __syncthreads();
    if (tid < NCLASS && lcnt[tid]) {
        lbase[tid] = atomicAdd(&L.cls_cnt[tid], lcnt[tid]);
        atomicAdd(&L.cls_elems[tid], lel[tid]);
    }
    if (tid == NCLASS && lcnt[NCLASS]) {
        lbase[NCLASS] = atomicAdd(lv.nseg, lcnt[NCLASS]);
        atomicAdd(lv.nelem, lel[NCLASS]);
        ltb = atomicAdd(lv.ntiles, ltiles);
        ltiles = 0;
    }
    if (tid == NCLASS + 1 && lact) atomicAdd(&L.misc[0], lact);
    __syncthreads();
    if (MODE == 1 && lcnt[NCLASS] == 0) return;  // small segments are placed by MODE 2
    // pass 2: writes
    for (u32 i0 = wbeg; i0 < wend; i0 += stride) {
        Seg s;
        const int c = seg_class(a, cur, wend, i0 + tid, s);
        u64 pend = __ballot(MODE == 1 ? c == NCLASS : c >= 0);
        u32 li = 0;
        while (pend) {
            const u32 f = (u32)__ffsll((long long)pend) - 1;
            const int cc = __builtin_amdgcn_readlane(c, f);
            const u64 m = __ballot(c == cc);
            u32 base = 0;
            if (lane == f) base = atomicAdd(&lcur[cc], (u32)__popcll(m));
            base = __builtin_amdgcn_readlane(base, f);
            if (c == cc) li = base + (u32)__popcll(m & lt);
            pend &= ~m;
        }
        if (c == NCLASS) {
            const u32 nt = (s.len + TILE - 1) / TILE;
            const u32 si = lbase[NCLASS] + li;
            const u32 tb = ltb + atomicAdd(&ltiles, nt);
            lv.segs[si] = LSeg{s.start, s.len | SEG_FIRST, tb, nt};
            for (u32 k = 0; k < nt; ++k) lv.tiles[tb + k] = LTile{si, k};
        } else if (MODE == 0 && c >= 0) {
            L.cls[c][lbase[c] + li] = Seg{s.start, s.len | SEG_FIRST};
        }
    }
}

// per class: exclusive scan of the bin counts -> class-local bin offsets (one workgroup per class)
__global__ __launch_bounds__(256) void k_bin_scan(Bins bn) {
    constexpr u32 R = CLS_NBIN / 256;
    __shared__ u32 sh[4];
    u32* c = bn.cnt + blockIdx.x * CLS_NBIN;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32 v[R], tot = 0;
#pragma unroll
    for (u32 r = 0; r < R; ++r) {
        v[r] = c[tid * R + r];
        tot += v[r];
    }
    const u32 incl = wave_incl_scan(tot, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 ex = incl - tot;
    for (u32 i = 0; i < w; ++i) ex += sh[i];
#pragma unroll
    for (u32 r = 0; r < R; ++r) {
        c[tid * R + r] = ex;
        ex += v[r];
    }
}

// ------------------------------------------------------------------------------------
// key generation
// ------------------------------------------------------------------------------------
// One launch for every class of the round (KgClasses): workgroup t belongs to the class whose
// workgroup range [wg0[c], wg0[c + 1]) holds it (one launch per class before: ~8 short grids per
// round, each with its own ramp-up and drain)
__device__ __attribute__((always_inline)) inline void keygen_small_body(const Seg* segs, u32 count, int c, const SortArgs& a, u32 tile) {
    const u32 spt = TILE >> c;
    const u32 first = tile * spt;
    const u32 mask = (1u << c) - 1;
    if (a.KP) {
        // dense rounds: K2[g] = KP[SA[g]].  All loads staged before the first store (the
        // stores may alias the loads for the compiler, which otherwise serialises every
        // element's segment -> SA -> KP chain)
        u32 g[PER_THREAD], v[PER_THREAD];
#pragma unroll
        for (int j = 0; j < PER_THREAD; ++j) {
            const u32 slot = j * WG + threadIdx.x;
            const u32 si = first + (slot >> c);
            g[j] = ~0u;
            if (si < count) {
                const Seg s = segs[si];
                const u32 k = slot & mask;
                if (k < (s.len & SEG_LEN)) g[j] = s.start + k;
            }
        }
#pragma unroll
        for (int j = 0; j < PER_THREAD; ++j) v[j] = g[j] != ~0u ? a.SA[g[j]] : 0u;
#pragma unroll
        for (int j = 0; j < PER_THREAD; ++j) v[j] = g[j] != ~0u ? a.KP[v[j]] : 0u;
#pragma unroll
        for (int j = 0; j < PER_THREAD; ++j)
            if (g[j] != ~0u) a.K2[g[j]] = v[j];
        return;
    }
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
        const u32 slot = j * WG + threadIdx.x;
        const u32 si = first + (slot >> c);
        const u32 k = slot & mask;
        if (si >= count) continue;
        const Seg s = segs[si];
        if (k >= (s.len & SEG_LEN)) continue;
        const u32 g = s.start + k;
        const u32 b = a.geo.block_of(s.start);
        a.K2[g] = make_key(a, a.SA[g], a.geo.base(b), a.geo.end(b));
    }
}

__global__ __launch_bounds__(WG) void k_keygen_small(KgClasses kc, SortArgs a) {
    const u32 t = blockIdx.x;
    int c = 1;
    while (c + 1 < NCLASS && kc.wg0[c + 1] <= t) ++c;
    // XCD-contiguous tiles inside the class (each class's list is in position order: one XCD's
    // workgroups then gather RK / KP from one part of each block)
    const u32 w = t - kc.wg0[c], G = kc.wg0[c + 1] - kc.wg0[c];
    keygen_small_body(kc.segs[c], kc.count[c], c, a, a.xcd ? xcd_map(w, G) : w);
}

__global__ __launch_bounds__(WG) void k_keygen_large(const LTile* tiles, const LSeg* segs, SortArgs a) {
    const LTile t = tiles[blockIdx.x];
    const LSeg s = segs[t.seg];
    const u32 base = s.start + t.k * TILE;
    const u32 cnt = min((u32)TILE, s.start + (s.len & SEG_LEN) - base);
    const u32 b = a.geo.block_of(s.start);
    const u32 bb = a.geo.base(b), be = a.geo.end(b);
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
        const u32 e = j * WG + threadIdx.x;
        if (e < cnt) a.K2[base + e] = make_key(a, a.SA[base + e], bb, be);
    }
}

// ------------------------------------------------------------------------------------
// MSD radix passes for segments longer than a tile
// ------------------------------------------------------------------------------------
// MSD kernels: ndev (when set) is the level's tile / segment count in device memory and
// the grid a bound on it (levels after the first are launched without a host round trip)
__global__ __launch_bounds__(WG) void k_msd_hist(const LTile* tiles, const LSeg* segs, SortArgs a,
                                                 u32 shift, u32 mask, u32* hist, const u32* ndev) {
    if (ndev && blockIdx.x >= *ndev) return;
    if (a.med && (segs[tiles[blockIdx.x].seg].len & SEG_LEN) <= MED_T) return;  // sorted by the medium form
    __shared__ u32 h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const LTile t = tiles[blockIdx.x];
    const LSeg s = segs[t.seg];
    const u32 base = s.start + t.k * TILE;
    const u32 cnt = min((u32)TILE, s.start + (s.len & SEG_LEN) - base);
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
        const u32 e = j * WG + threadIdx.x;
        if (e < cnt) atomicAdd(&h[(a.K2[base + e] >> shift) & mask], 1u);
    }
    __syncthreads();
    hist[(u64)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// One workgroup per segment: per-digit running offsets over the segment's tiles, bucket
// starts, and classification of the buckets (small -> class list, large -> next level,
// large after the last digit -> equal-key run).
__global__ __launch_bounds__(WG) void k_msd_scan(const LSeg* segs, SortArgs a, u32* hist, int last_level,
                                                 Lists L, Level nx, const u32* ndev) {
    if (ndev && blockIdx.x >= *ndev) return;
    if (a.med && (segs[blockIdx.x].len & SEG_LEN) <= MED_T) return;
    __shared__ u32 sh[WG / 64];
    const LSeg s = segs[blockIdx.x];
    const u32 d = threadIdx.x;
    // pass 1: per-digit totals (16 independent loads in flight per thread)
    constexpr u32 B = 16;
    const u32 t0 = s.tile_base, t1 = s.tile_base + s.ntiles;
    u32 run = 0;
    for (u32 t = t0; t < t1; t += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = t + j < t1 ? hist[(u64)(t + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j) run += v[j];
    }
    const u32 bstart = wg_excl_scan<false>(run, OpAdd(), 0u, sh);
    const u32 abs0 = s.start + bstart;
    // pass 2: absolute scatter base of every (tile, digit)
    u32 acc = abs0;
    for (u32 t = t0; t < t1; t += B) {
        u32 v[B];
#pragma unroll
        for (u32 j = 0; j < B; ++j) v[j] = t + j < t1 ? hist[(u64)(t + j) * 256 + d] : 0u;
#pragma unroll
        for (u32 j = 0; j < B; ++j) {
            if (t + j < t1) hist[(u64)(t + j) * 256 + d] = acc;
            acc += v[j];
        }
    }
    const int nonzero = __syncthreads_count(run > 0);
    if (nonzero > 1 && d == 0) a.blk_split[a.geo.block_of(s.start)] = 1;
    // classify the buckets; appends aggregated per workgroup (LDS counters, one global
    // atomic per list) — per-bucket global atomics on a dozen hot counters serialise
    __shared__ u32 lcnt[NCLASS + 2], lel[NCLASS + 2], lbase[NCLASS + 2], ltiles, ltb;
    if (d < NCLASS + 2) {
        lcnt[d] = 0;
        lel[d] = 0;
    }
    if (d == 0) ltiles = 0;
    __syncthreads();
    // the first non-empty bucket of a FIRST segment starts at its round group's start
    const Seg sub{abs0, run | (((s.len & SEG_FIRST) && bstart == 0) ? SEG_FIRST : 0u)};
    int kind = -1;  // 0..NCLASS-1 class, NCLASS next level, NCLASS+1 equal run
    u32 li = 0, lt = 0, nt = 0;
    if (run > 0) {
        kind = run <= (u32)TILE ? size_class(run) : (!last_level ? NCLASS : NCLASS + 1);
        li = atomicAdd(&lcnt[kind], 1u);
        atomicAdd(&lel[kind], run);
        if (kind == NCLASS) {
            nt = (run + TILE - 1) / TILE;
            lt = atomicAdd(&ltiles, nt);
        }
    }
    __syncthreads();
    if (d < NCLASS && lcnt[d]) {
        lbase[d] = atomicAdd(&L.cls_cnt[d], lcnt[d]);
        atomicAdd(&L.cls_elems[d], lel[d]);
    }
    if (d == NCLASS && lcnt[d]) {
        lbase[d] = atomicAdd(nx.nseg, lcnt[d]);
        atomicAdd(nx.nelem, lel[d]);
        ltb = atomicAdd(nx.ntiles, ltiles);
    }
    if (d == NCLASS + 1 && lcnt[d]) lbase[d] = atomicAdd(L.eq_cnt, lcnt[d]);
    __syncthreads();
    if (kind < 0) return;
    if (kind < NCLASS) {
        L.cls[kind][lbase[kind] + li] = sub;
    } else if (kind == NCLASS) {
        const u32 si = lbase[NCLASS] + li;
        const u32 tb = ltb + lt;
        nx.segs[si] = LSeg{sub.start, sub.len, tb, nt};
        for (u32 k = 0; k < nt; ++k) nx.tiles[tb + k] = LTile{si, k};
    } else {
        L.eq[lbase[NCLASS + 1] + li] = sub;
    }
}

// Stable scatter of one tile by digit: element order inside the tile is e = j*WG + tid,
// each wave ranks its 64 elements per digit with ballots; per-wave digit counts are
// combined through LDS in (j, wave) order, so equal digits keep their tile order.
__global__ __launch_bounds__(WG) void k_msd_scatter(const LTile* tiles, const LSeg* segs, SortArgs a,
                                                    u32 shift, u32 width, const u32* hist, const u32* ndev) {
    if (ndev && blockIdx.x >= *ndev) return;
    if (a.med && (segs[tiles[blockIdx.x].seg].len & SEG_LEN) <= MED_T) return;
    __shared__ u32 wcnt[WG / 64][256];
    __shared__ u32 running[256];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const LTile t = tiles[blockIdx.x];
    const LSeg s = segs[t.seg];
    const u32 base = s.start + t.k * TILE;
    const u32 cnt = min((u32)TILE, s.start + (s.len & SEG_LEN) - base);
    const u32 mask = (1u << width) - 1;
    running[tid] = hist[(u64)blockIdx.x * 256 + tid];
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) wcnt[i][tid] = 0;
    __syncthreads();
    const u64 lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int j = 0; j < PER_THREAD; ++j) {
        const u32 e = j * WG + tid;
        const bool valid = e < cnt;
        u32 sa = 0, key = 0, dg = 0;
        if (valid) {
            sa = a.SA[base + e];
            key = a.K2[base + e];
            dg = (key >> shift) & mask;
        }
        u64 m = __ballot(valid);
        for (u32 bit = 0; bit < width; ++bit) {
            const u64 bal = __ballot((dg >> bit) & 1u);
            m &= ((dg >> bit) & 1u) ? bal : ~bal;
        }
        const u32 rank = __popcll(m & lt_mask);
        const bool leader = valid && rank == 0;
        if (leader) wcnt[w][dg] = __popcll(m);
        __syncthreads();
        if (valid) {
            u32 pre = running[dg];
            for (u32 i = 0; i < w; ++i) pre += wcnt[i][dg];
            const u32 dst = pre + rank;
            a.SA2[dst] = sa;
            a.K22[dst] = key;
        }
        __syncthreads();
        u32 add = 0;
#pragma unroll
        for (int i = 0; i < WG / 64; ++i) {
            add += wcnt[i][tid];
            wcnt[i][tid] = 0;
        }
        running[tid] += add;
        __syncthreads();
    }
}

__global__ __launch_bounds__(WG) void k_copy_back(const LTile* tiles, const LSeg* segs, SortArgs a,
                                                  const u32* ndev) {
    if (ndev && blockIdx.x >= *ndev) return;
    if (a.med && (segs[tiles[blockIdx.x].seg].len & SEG_LEN) <= MED_T) return;
    const LTile t = tiles[blockIdx.x];
    const LSeg s = segs[t.seg];
    const u32 base = s.start + t.k * TILE;
    const u32 cnt = min((u32)TILE, s.start + (s.len & SEG_LEN) - base);
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
        const u32 e = j * WG + threadIdx.x;
        if (e < cnt) {
            a.SA[base + e] = a.SA2[base + e];
            a.K2[base + e] = a.K22[base + e];
        }
    }
}

// ------------------------------------------------------------------------------------
// small segments: one tile = TILE/2^C segments, each padded to 2^C slots, sorted by
// (key, position) with a bitonic network (distances >= 8 through LDS, < 8 in registers),
// then split into runs of equal key: new groups.
// ------------------------------------------------------------------------------------
// Sort words: u64 = (key << 32 | position); u32 = (key << C | index in the segment) when
// key and index fit 32 bits (keys < 2^kbits, elements of a segment are in position order,
// so index order is position order) — half the LDS traffic and registers.
template <int J, class KT>
__device__ inline void reg_stage(KT (&r)[8], u32 tid, u32 k, u32 S) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (e & J) continue;
        const u32 i = 8 * tid + e;
        const bool up = (k == S) || ((i & k) == 0);
        const KT x = r[e], y = r[e + J];
        const bool sw = (x > y) == up;
        r[e] = sw ? y : x;
        r[e + J] = sw ? x : y;
    }
}

__device__ inline u32 SKI(u32 i) { return i + (i >> 6); }

// Shared tail of the small and medium sorts: r[8] = this thread's sorted words 8 tid .. 8 tid + 7
// of sub-arrays of S slots (KT: (key << C | index) with sa_l, or (key << 32 | position));
// runs of equal key -> RK of their heads, SA where a sub-array split, new groups of >= 2
// elements to the next round, split flags.
template <int C, class KT, u32 T, u32 NT>
__device__ inline void sort_epilogue(KT (&r)[8], const Seg* ss, u8* ssplit, const u32* sa_l, u32* sh, u32* last_hi,
                                     const SortArgs& a, const Lists& L) {
    constexpr u32 NWV = NT / 64;
    constexpr u32 S = 1u << C;
    constexpr bool W32 = sizeof(KT) == 4;
    constexpr KT NONEK = ~(KT)0;
    const u32 tid = threadIdx.x;
    constexpr u32 HS = W32 ? C : 32;  // key = word >> HS
    // runs of equal key inside each sub-array
    last_hi[tid] = (u32)(r[7] >> HS);
    __syncthreads();
    bool valid[8], head[8], stop[8];
    u32 prev_hi = tid ? last_hi[tid - 1] : 0;
    bool prev_valid = tid ? true : false;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const u32 i = 8 * tid + e;
        const u32 kk = i & (S - 1);
        valid[e] = r[e] != NONEK;
        const u32 hi = (u32)(r[e] >> HS);
        head[e] = valid[e] && (kk == 0 || hi != prev_hi);
        stop[e] = kk == 0 || head[e] || !valid[e];
        if (head[e] && kk != 0) ssplit[i >> C] = 1;
        prev_hi = hi;
        (void)prev_valid;
    }
    // run start: inclusive max-scan of head indices
    u32 loc[8];
    u32 agg = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (head[e]) agg = 8 * tid + e;
        loc[e] = agg;
    }
    const u32 carry = wg_excl_scan<false, OpMax, NWV>(agg, OpMax(), 0u, sh);
    u32 start_idx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) start_idx[e] = loc[e] > carry ? loc[e] : carry;
    // run end: exclusive suffix min of stop indices
    u32 sagg = T;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        if (stop[e] && (u32)(8 * tid + e) < sagg) sagg = 8 * tid + e;
    const u32 scarry = wg_excl_scan<true, OpMin, NWV>(sagg, OpMin(), (u32)T, sh);
    u32 nxt[8];
    u32 run_min = scarry;
#pragma unroll
    for (int e = 7; e >= 0; --e) {
        nxt[e] = run_min;
        if (stop[e]) run_min = 8 * tid + e;
    }
    // new groups of >= 2 elements go to the next round (one global atomic per workgroup)
    u32 nnew = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) nnew += (valid[e] && head[e] && nxt[e] - (8 * tid + e) >= 2) ? 1u : 0u;
    const u32 my_off = wg_excl_scan<false, OpAdd, NWV>(nnew, OpAdd(), 0u, sh);
    if (tid == NT - 1) last_hi[0] = my_off + nnew;  // reuse LDS: workgroup total
    __syncthreads();
    const u32 total_new = last_hi[0];
    __syncthreads();
    if (tid == 0) last_hi[1] = total_new ? atomicAdd(L.next_cnt, total_new) : 0u;
    __syncthreads();
    u32 wpos = last_hi[1] + my_off;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (!valid[e]) continue;
        const u32 i = 8 * tid + e;
        const u32 si = i >> C, kk = i & (S - 1);
        const Seg sg = ss[si];
        u32 pos;
        if constexpr (W32)
            pos = sa_l[(si << C) + ((u32)r[e] & (S - 1))];
        else
            pos = (u32)r[e];
        const u32 rs = start_idx[e] - (si << C);  // run start inside the segment
        // an unsplit segment keeps its order (ties are in position order already); the
        // first run of a FIRST segment keeps its rank (except in round 0: RK undefined)
        if (ssplit[si]) a.SA[sg.start + kk] = pos;
        if (a.initial || rs != 0 || !(sg.len & SEG_FIRST)) a.RK[pos] = sg.start + rs;
        if (head[e]) {
            const u32 len = nxt[e] - i;
            if (len >= 2) L.next[wpos++] = Seg{sg.start + kk, len};
            if (kk > 0) a.blk_split[a.geo.block_of(sg.start)] = 1;
        }
    }
}

// The small sort of class C for the workgroup's tile `tile` of the class list, on LDS arrays its
// kernel provides (k_small_sort: one class per launch; k_small_sort_all: classes 5..11 of one
// round in one launch, arrays sized for the smallest class).
template <int C, class KT, u32 T, u32 NT>
__device__ __attribute__((always_inline)) inline void small_sort_body(const Seg* segs, u32 count, SortArgs a, Lists L,
                                                                     u32 tile, KT* sk, u32* sa_l, Seg* ss, u32* sh,
                                                                     u32* last_hi, u8* ssplit) {
    static_assert(T == 8 * NT, "8 elements per thread");
    constexpr u32 PT = T / NT;
    constexpr u32 S = 1u << C;
    constexpr u32 SPT = T / S;
    constexpr bool W32 = sizeof(KT) == 4;
    constexpr KT NONEK = ~(KT)0;
    const u32 tid = threadIdx.x;
    const u32 first = tile * SPT;
    const u32 nthis = min(SPT, count - first);
    for (u32 i = tid; i < SPT; i += NT) {
        ss[i] = i < nthis ? segs[first + i] : Seg{0, 0};
        ssplit[i] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (int)PT; ++j) {
        const u32 slot = j * NT + tid;
        const u32 si = slot >> C, k = slot & (S - 1);
        KT key = NONEK;
        if (si < nthis && k < (ss[si].len & SEG_LEN)) {
            const u32 g = ss[si].start + k;
            // (gathering KP[SA[g]] here instead of in k_keygen_small measured slower: the
            // dependent gather is exposed at the sort's LDS-limited occupancy)
            const u32 p = a.SA[g];
            const u32 kv = a.K2[g];
            if constexpr (W32) {
                key = (kv << C) | k;
                sa_l[slot] = p;
            } else {
                key = ((u64)kv << 32) | p;
            }
        }
        sk[SKI(slot)] = key;
    }
    __syncthreads();
    KT r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = sk[SKI(8 * tid + e)];
    for (u32 k = 2; k <= S; k <<= 1) {
        if (k > 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) sk[SKI(8 * tid + e)] = r[e];
            __syncthreads();
            for (u32 j = k >> 1; j >= 8; j >>= 1) {
                const u32 lj = 31 - __clz(j);
#pragma unroll
                for (int q0 = 0; q0 < (int)(T / 2 / NT); ++q0) {
                    const u32 q = q0 * NT + tid;
                    const u32 i = ((q >> lj) << (lj + 1)) | (q & (j - 1));
                    const u32 l = i + j;
                    const bool up = (k == S) || ((i & k) == 0);
                    const KT x = sk[SKI(i)], y = sk[SKI(l)];
                    if ((x > y) == up) {
                        sk[SKI(i)] = y;
                        sk[SKI(l)] = x;
                    }
                }
                __syncthreads();
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] = sk[SKI(8 * tid + e)];
            __syncthreads();
        }
        if (k >= 8) reg_stage<4>(r, tid, k, S);
        if (k >= 4) reg_stage<2>(r, tid, k, S);
        reg_stage<1>(r, tid, k, S);
    }
    sort_epilogue<C, KT, T, NT>(r, ss, ssplit, sa_l, sh, last_hi, a, L);
}

template <int C, class KT, u32 T = TILE, u32 NT = WG>
__global__ __launch_bounds__(NT) void k_small_sort(const Seg* segs, u32 count, SortArgs a, Lists L) {
    constexpr u32 SPT = T >> C;
    constexpr bool W32 = sizeof(KT) == 4;
    // one pad word per 64: the per-thread 8-element runs (8*tid + e) hit 64 distinct banks
    __shared__ KT sk[T + T / 64];
    __shared__ u32 sa_l[W32 ? T : 1];
    __shared__ Seg ss[SPT];
    __shared__ u32 sh[NT / 64];
    __shared__ u32 last_hi[NT];
    __shared__ u8 ssplit[SPT];  // sub-array split by this round's key
    small_sort_body<C, KT, T, NT>(segs, count, a, L, a.xcd ? xcd_tile() : blockIdx.x, sk, sa_l, ss, sh, last_hi,
                                  ssplit);
}

// classes 5..11 of a round in one launch (every class sorts TILE elements per workgroup in the
// same LDS arrays; the per-segment arrays are sized for class 5); workgroup t belongs to the class
// whose range [wg0[c], wg0[c + 1]) holds it, tiles XCD-contiguous inside each class
template <class KT>
__global__ __launch_bounds__(WG) void k_small_sort_all(SsClasses sc, SortArgs a, Lists L) {
    constexpr u32 T = TILE, NT = WG, SPT = T >> 5;
    constexpr bool W32 = sizeof(KT) == 4;
    __shared__ KT sk[T + T / 64];
    __shared__ u32 sa_l[W32 ? T : 1];
    __shared__ Seg ss[SPT];
    __shared__ u32 sh[NT / 64];
    __shared__ u32 last_hi[NT];
    __shared__ u8 ssplit[SPT];
    const u32 t = blockIdx.x;
    int c = 5;
    while (c < 11 && sc.wg0[c + 1] <= t) ++c;
    const u32 w = t - sc.wg0[c], G = sc.wg0[c + 1] - sc.wg0[c];
    const u32 tile = a.xcd ? xcd_map(w, G) : w;
    switch (c) {
#define KOLM_SS_CASE(K) \
    case K: small_sort_body<K, KT, T, NT>(sc.segs[K], sc.count[K], a, L, tile, sk, sa_l, ss, sh, last_hi, ssplit); break;
        KOLM_SS_CASE(5) KOLM_SS_CASE(6) KOLM_SS_CASE(7) KOLM_SS_CASE(8) KOLM_SS_CASE(9) KOLM_SS_CASE(10)
        default: small_sort_body<11, KT, T, NT>(sc.segs[11], sc.count[11], a, L, tile, sk, sa_l, ss, sh, last_hi, ssplit); break;
#undef KOLM_SS_CASE
    }
}

// Medium sort (batches of few blocks): one 1024-thread workgroup sorts one large group of
// TILE < len <= MED_T elements of an MSD level list by its key (K2), in place of the level's
// hist / scan / scatter / copy launches.  Stable LSD radix over 8-bit digits in LDS: keys and
// 16-bit element indices ping-pong between two buffers; per 1024-element chunk each wave ranks
// its lanes per digit with 8 ballots (as k_msd_scatter), the waves' digit counts combine in
// chunk / wave order, so equal keys keep their index (= position) order.  The sorted words
// (key << 32 | position) then go through the small sorts' epilogue.
constexpr u32 MED_NT = MED_T / 8;  // 1024 threads
__global__ __launch_bounds__(MED_NT) void k_med_sort(const LSeg* msegs, const u32* mcount, SortArgs a, Lists L) {
    constexpr u32 NWV = MED_NT / 64;
    __shared__ u32 kb[2][MED_T];
    __shared__ u16 ib[2][MED_T];
    __shared__ u32 wcnt[NWV][256];
    __shared__ u32 base[256];
    __shared__ u32 running[256];
    __shared__ Seg ss[1];
    __shared__ u8 ssplit[1];
    __shared__ u32 sh[NWV];
    __shared__ u32 last_hi[MED_NT];
    // ~118 KiB of LDS: one workgroup per CU, gfx950's 160 KiB LDS only (a 64 KiB part fails here)
    static_assert(sizeof(kb) + sizeof(ib) + sizeof(wcnt) + sizeof(base) + sizeof(running) + sizeof(last_hi) +
                      sizeof(sh) <= 160 * 1024 && sizeof(kb) + sizeof(ib) + sizeof(wcnt) > 64 * 1024,
                  "k_med_sort is sized for the 160 KiB LDS of gfx950");
    if (blockIdx.x >= *mcount) return;
    const LSeg ls = msegs[blockIdx.x];
    const u32 n = ls.len & SEG_LEN;
    if (n > MED_T) return;  // left to the MSD levels
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) {
        ss[0] = Seg{ls.start, ls.len};
        ssplit[0] = 0;
    }
    for (u32 i = tid; i < n; i += MED_NT) {
        kb[0][i] = a.K2[ls.start + i];
        ib[0][i] = (u16)i;
    }
    const u64 lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    u32 cur = 0;
    for (u32 shift = 0; shift < a.key_bits; shift += 8, cur ^= 1) {
        const u32 width = min(8u, a.key_bits - shift), dmask = (1u << width) - 1;
        if (tid < 256) {
            base[tid] = 0;
            running[tid] = 0;
        }
        for (u32 i = tid; i < NWV * 256; i += MED_NT) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        // digit totals without LDS atomics (a group's keys often share their digits: 8192
        // atomics on one counter serialise): per wave and chunk, one add per distinct digit
        for (u32 c0 = 0; c0 < n; c0 += MED_NT) {
            const u32 i = c0 + tid;
            const bool v = i < n;
            const u32 dg = v ? (kb[cur][i] >> shift) & dmask : 0u;
            u64 m = __ballot(v);
            for (u32 bit = 0; bit < width; ++bit) {
                const u64 bal = __ballot((dg >> bit) & 1u);
                m &= ((dg >> bit) & 1u) ? bal : ~bal;
            }
            if (v && __popcll(m & lt_mask) == 0) wcnt[w][dg] += __popcll(m);
        }
        __syncthreads();
        if (tid < 256) {
            u32 t = 0;
            for (u32 q = 0; q < NWV; ++q) {
                t += wcnt[q][tid];
                wcnt[q][tid] = 0;
            }
            base[tid] = t;
        }
        __syncthreads();
        if (tid < 64) {  // exclusive scan of the 256 digit counts by wave 0 (4 per lane)
            const u32 c0 = base[4 * tid], c1 = base[4 * tid + 1], c2 = base[4 * tid + 2], c3 = base[4 * tid + 3];
            const u32 t4 = c0 + c1 + c2 + c3;
            const u32 ex = wave_incl_scan(t4, OpAddU(), 0u) - t4;
            base[4 * tid] = ex;
            base[4 * tid + 1] = ex + c0;
            base[4 * tid + 2] = ex + c0 + c1;
            base[4 * tid + 3] = ex + c0 + c1 + c2;
        }
        __syncthreads();
        for (u32 c0 = 0; c0 < n; c0 += MED_NT) {
            const u32 i = c0 + tid;
            const bool v = i < n;
            u32 key = 0, idx = 0, dg = 0;
            if (v) {
                key = kb[cur][i];
                idx = ib[cur][i];
                dg = (key >> shift) & dmask;
            }
            u64 m = __ballot(v);
            for (u32 bit = 0; bit < width; ++bit) {
                const u64 bal = __ballot((dg >> bit) & 1u);
                m &= ((dg >> bit) & 1u) ? bal : ~bal;
            }
            const u32 rank = __popcll(m & lt_mask);
            if (v && rank == 0) wcnt[w][dg] = __popcll(m);
            __syncthreads();
            if (v) {
                u32 pre = base[dg] + running[dg];
                for (u32 q = 0; q < w; ++q) pre += wcnt[q][dg];
                kb[cur ^ 1][pre + rank] = key;
                ib[cur ^ 1][pre + rank] = (u16)idx;
            }
            __syncthreads();
            if (tid < 256) {
                u32 add = 0;
                for (u32 q = 0; q < NWV; ++q) {
                    add += wcnt[q][tid];
                    wcnt[q][tid] = 0;
                }
                running[tid] += add;
            }
            __syncthreads();
        }
    }
    // this thread's sorted words 8 tid .. 8 tid + 7: (key << 32 | position)
    u64 r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const u32 i = 8 * tid + e;
        r[e] = i < n ? ((u64)kb[cur][i] << 32) | a.SA[ls.start + ib[cur][i]] : ~0ull;
    }
    __syncthreads();
    sort_epilogue<13, u64, MED_T, MED_NT>(r, ss, ssplit, nullptr, sh, last_hi, a, L);
}

// Tiny segments (class C <= TINY_C, at most 16 elements): one thread per segment, the
// (key << 32 | position) words sorted by a bitonic network in registers (ties in position
// order), runs -> new groups.  In dense rounds the key is gathered here from KP (no K2
// round trip, no LDS: full occupancy hides the gather); otherwise K2 from k_keygen_small.
// Same write rules as k_small_sort (SA only if split, RK skipped for a FIRST run).
template <int C>
__global__ __launch_bounds__(256) void k_tiny_sort(const Seg* segs, u32 count, SortArgs a, Lists L) {
    constexpr u32 S = 1u << C;
    __shared__ u32 sh[WG / 64], wtot;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 i = (a.xcd ? xcd_tile() : blockIdx.x) * WG + tid;
    Seg sg{0, 0};
    u32 len = 0;
    if (i < count) {
        sg = segs[i];
        len = sg.len & SEG_LEN;
    }
    u64 v[S];
#pragma unroll
    for (u32 e = 0; e < S; ++e) {
        v[e] = ~0ull;
        if (e < len) {
            const u32 g = sg.start + e;
            const u32 p = a.SA[g];
            const u32 kv = a.KP ? a.KP[p] : a.K2[g];
            v[e] = ((u64)kv << 32) | p;
        }
    }
#pragma unroll
    for (u32 k = 2; k <= S; k <<= 1)
#pragma unroll
        for (u32 j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (u32 e = 0; e < S; ++e) {
                const u32 l = e ^ j;
                if (l > e) {
                    const bool up = (e & k) == 0;
                    const u64 x = v[e], y = v[l];
                    if ((x > y) == up) {
                        v[e] = y;
                        v[l] = x;
                    }
                }
            }
    // runs
    bool split = false;
    u32 nnew = 0;
    {
        u32 prev = 0;
#pragma unroll
        for (u32 e = 0; e < S; ++e) {
            if (e < len) {
                const u32 kv = (u32)(v[e] >> 32);
                if (e > 0 && kv != prev) split = true;
                prev = kv;
            }
        }
    }
    {
        u32 rs = 0;
#pragma unroll
        for (u32 e = 0; e < S; ++e) {
            if (e < len) {
                if (e > 0 && (u32)(v[e] >> 32) != (u32)(v[e - 1] >> 32)) {
                    nnew += (e - rs >= 2) ? 1u : 0u;
                    rs = e;
                }
            }
        }
        if (len && len - rs >= 2) ++nnew;
    }
    // one global atomic per workgroup for the new segments
    const u32 incl = wave_incl_scan(nnew, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 off = incl - nnew;
    for (u32 q = 0; q < w; ++q) off += sh[q];
    if (tid == WG - 1) {
        const u32 tot = off + nnew;
        wtot = tot ? atomicAdd(L.next_cnt, tot) : 0u;
    }
    __syncthreads();
    off += wtot;
    if (!len) return;
    const bool first = (sg.len & SEG_FIRST) != 0;
    u32 rs = 0;
#pragma unroll
    for (u32 e = 0; e < S; ++e) {
        if (e < len) {
            const u32 kv = (u32)(v[e] >> 32), pos = (u32)v[e];
            if (e > 0 && kv != (u32)(v[e - 1] >> 32)) {
                if (e - rs >= 2) L.next[off++] = Seg{sg.start + rs, e - rs};
                rs = e;
            }
            if (split) a.SA[sg.start + e] = pos;
            if (a.initial || rs != 0 || !first) a.RK[pos] = sg.start + rs;
        }
    }
    if (len - rs >= 2) L.next[off++] = Seg{sg.start + rs, len - rs};
    if (split) a.blk_split[a.geo.block_of(sg.start)] = 1;
}

__global__ void k_single(const Seg* segs, u32 count, SortArgs a) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) {
        const Seg s = segs[i];
        if (a.initial || !(s.len & SEG_FIRST)) {
            const u32 p = a.SA[s.start];
            a.RK[p] = s.start;
        }
    }
}

// gridDim.y workgroups share one run (periodic data: runs of 10^5-10^6 equal keys)
__global__ __launch_bounds__(WG) void k_finalize_eq(const Seg* eq, SortArgs a, Lists L) {
    const Seg s = eq[blockIdx.x];
    const u32 len = s.len & SEG_LEN;
    // a FIRST run keeps its group's rank after round 0
    if (a.initial || !(s.len & SEG_FIRST)) {
        for (u32 i = blockIdx.y * WG + threadIdx.x; i < len; i += gridDim.y * WG) {
            const u32 p = a.SA[s.start + i];
            a.RK[p] = s.start;
        }
    }
    if (blockIdx.y == 0 && threadIdx.x == 0) L.next[atomicAdd(L.next_cnt, 1u)] = Seg{s.start, len};
}

// done[b] = 1 + the round in which block b stopped splitting (0 while it still splits);
// last[b] = 1 + the last round in which one of block b's groups split
__global__ void k_update_done(u32* done, u32* last, const u32* split, u32 nb, u32 round) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    if (split[b]) last[b] = round + 1;
    else if (!done[b]) done[b] = round + 1;
}

// sum over blocks of the rounds each block needed: round 0 through the last round that split
// one of its groups (at least 1).  A function of the block alone — the rounds a batch runs to
// confirm convergence, or runs for its other blocks, are not counted
__global__ void k_rounds_sum(const u32* last, u32 nb, unsigned long long* out) {
    u64 acc = 0;
    for (u32 b = threadIdx.x; b < nb; b += blockDim.x) acc += max(last[b], 1u);
    for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static inline u32 cdiv(u64 a, u64 b) { return (u32)((a + b - 1) / b); }

void launch_iota(u32* SA, u64 N, hipStream_t s) {
    if (!N) return;
    k_iota<<<std::min<u32>(cdiv(N, 256), 65535u), 256, 0, s>>>(SA, (u32)N);
}
void launch_block_segs(Seg* segs, const Geom& geo, hipStream_t s) {
    if (geo.nb) k_block_segs<<<cdiv(geo.nb, 256), 256, 0, s>>>(segs, geo);
}
__global__ void k_zero_spans(ZeroSpans z) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < 6; ++k) {
        if (i < z.n[k]) {
            if (k == 3 && z.done) {  // the previous round's k_update_done, fused
                if (z.p[3][i]) z.last[i] = z.round + 1;
                else if (!z.done[i]) z.done[i] = z.round + 1;
            }
            z.p[k][i] = 0;
            return;
        }
        i -= z.n[k];
    }
}
void launch_zero_spans(const ZeroSpans& z, hipStream_t s) {
    u64 tot = 0;
    for (int k = 0; k < 6; ++k) tot += z.p[k] ? z.n[k] : 0;
    if (tot) k_zero_spans<<<cdiv(tot, 256), 256, 0, s>>>(z);
}
__global__ void k_pack_spans(PackSpans ps, u32* dst) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < 6; ++k) {
        if (i < ps.n[k]) {
            dst[ps.o[k] + i] = ps.p[k][i];
            return;
        }
        i -= ps.n[k];
    }
}
void launch_pack_spans(const PackSpans& ps, u32* dst, hipStream_t s) {
    u64 tot = 0;
    for (int k = 0; k < 6; ++k) tot += ps.n[k];
    if (tot) k_pack_spans<<<cdiv(tot, 256), 256, 0, s>>>(ps, dst);
}
void launch_classify_bins(const Seg* cur, u32 ncur, const u32* ncur_dev, const SortArgs& a, const Lists& L,
                          const Level& lv0, const Bins& bn, hipStream_t s, bool bins_zeroed) {
    if (!ncur) return;
    const u32 grid = std::min<u32>(cdiv(ncur, 256), 2048u);
    if (!bins_zeroed) {
        KOLM_HIP_CHECK(hipMemsetAsync(bn.cnt, 0, sizeof(u32) * NCLASS * CLS_NBIN, s));
        KOLM_HIP_CHECK(hipMemsetAsync(bn.fill, 0, sizeof(u32) * NCLASS * CLS_NBIN, s));
    }
    k_classify<1><<<grid, 256, 0, s>>>(cur, ncur, ncur_dev, a, L, lv0, bn);
    k_bin_scan<<<NCLASS, 256, 0, s>>>(bn);
    k_classify<2><<<grid, 256, 0, s>>>(cur, ncur, ncur_dev, a, L, lv0, bn);
}
void launch_keypos(const SortArgs& a, u32* KP, hipStream_t s) {
    if (!a.geo.N) return;
    if (a.cyclic && a.FEd && ((uintptr_t)a.text & 15) == 0) {
        k_keypos_cyc<<<cdiv(a.geo.N, 4096), 256, 0, s>>>(a, KP);
        return;
    }
    const u32 grid = (u32)std::min<u64>((a.geo.N + 255) / 256, 8192);
    k_keypos<<<grid, 256, 0, s>>>(a, KP);
}

void launch_keygen_small(KgClasses kc, const SortArgs& a, hipStream_t s) {
    u32 n = 0;
    for (int c = 1; c < NCLASS; ++c) {
        kc.wg0[c] = n;
        n += kc.count[c] ? cdiv(kc.count[c], TILE >> c) : 0u;
    }
    kc.wg0[0] = 0;
    kc.wg0[NCLASS] = n;
    if (n) k_keygen_small<<<n, WG, 0, s>>>(kc, a);
}
void launch_keygen_large(const LTile* tiles, u32 ntiles, const LSeg* segs, const SortArgs& a,
                         hipStream_t s) {
    if (ntiles) k_keygen_large<<<ntiles, WG, 0, s>>>(tiles, segs, a);
}
void launch_msd_hist(const LTile* tiles, u32 ntiles, const u32* ndev, const LSeg* segs, const SortArgs& a,
                     u32 shift, u32 width, u32* hist, hipStream_t s) {
    if (ntiles) k_msd_hist<<<ntiles, WG, 0, s>>>(tiles, segs, a, shift, (1u << width) - 1, hist, ndev);
}
void launch_msd_scan(const LSeg* segs, u32 nseg, const u32* ndev, const SortArgs& a, u32 width, u32* hist,
                     bool last_level, const Lists& L, const Level& next, hipStream_t s) {
    (void)width;
    if (nseg) k_msd_scan<<<nseg, WG, 0, s>>>(segs, a, hist, last_level ? 1 : 0, L, next, ndev);
}
void launch_msd_scatter(const LTile* tiles, u32 ntiles, const u32* ndev, const LSeg* segs, const SortArgs& a,
                        u32 shift, u32 width, const u32* hist, hipStream_t s) {
    if (ntiles) k_msd_scatter<<<ntiles, WG, 0, s>>>(tiles, segs, a, shift, width, hist, ndev);
}
void launch_copy_back(const LTile* tiles, u32 ntiles, const u32* ndev, const LSeg* segs, const SortArgs& a,
                      hipStream_t s) {
    if (ntiles) k_copy_back<<<ntiles, WG, 0, s>>>(tiles, segs, a, ndev);
}

template <int C>
static void small_sort_c(const Seg* segs, u32 count, const SortArgs& a, const Lists& L, hipStream_t s) {
    if (a.key_bits + C <= 31)
        k_small_sort<C, u32><<<cdiv(count, TILE >> C), WG, 0, s>>>(segs, count, a, L);
    else
        k_small_sort<C, u64><<<cdiv(count, TILE >> C), WG, 0, s>>>(segs, count, a, L);
}

void launch_tiny_sort(int c, const Seg* segs, u32 count, const SortArgs& a, const Lists& L, hipStream_t s) {
    if (!count) return;
    switch (c) {
        case 1: k_tiny_sort<1><<<cdiv(count, WG), WG, 0, s>>>(segs, count, a, L); break;
        case 2: k_tiny_sort<2><<<cdiv(count, WG), WG, 0, s>>>(segs, count, a, L); break;
        case 3: k_tiny_sort<3><<<cdiv(count, WG), WG, 0, s>>>(segs, count, a, L); break;
        case 4: k_tiny_sort<4><<<cdiv(count, WG), WG, 0, s>>>(segs, count, a, L); break;
        case 5: k_tiny_sort<5><<<cdiv(count, WG), WG, 0, s>>>(segs, count, a, L); break;
        default: break;
    }
}

void launch_small_sort(int c, const Seg* segs, u32 count, const SortArgs& a, const Lists& L,
                       hipStream_t s) {
    if (!count) return;
    switch (c) {
        case 0: k_single<<<cdiv(count, 256), 256, 0, s>>>(segs, count, a); break;
        case 1: small_sort_c<1>(segs, count, a, L, s); break;
        case 2: small_sort_c<2>(segs, count, a, L, s); break;
        case 3: small_sort_c<3>(segs, count, a, L, s); break;
        case 4: small_sort_c<4>(segs, count, a, L, s); break;
        case 5: small_sort_c<5>(segs, count, a, L, s); break;
        case 6: small_sort_c<6>(segs, count, a, L, s); break;
        case 7: small_sort_c<7>(segs, count, a, L, s); break;
        case 8: small_sort_c<8>(segs, count, a, L, s); break;
        case 9: small_sort_c<9>(segs, count, a, L, s); break;
        case 10: small_sort_c<10>(segs, count, a, L, s); break;
        case 11: small_sort_c<11>(segs, count, a, L, s); break;
        default: break;
    }
}
// Up to 6 u32 spans into coherent host memory (hdst[o[k] + j] = p[k][j]), then each wave's
// sequence word: lane 0's system-scope release store waits for the wave's earlier stores and
// makes them visible to the host first, so the host reads the spans once every wave's word
// holds `seq` (no blit, no stream query).
__global__ __launch_bounds__(256) void k_spans_to_host(PackSpans ps, u32* hdst, u32* hseq, u32 seq) {
    for (int k = 0; k < 6; ++k)
        for (u32 j = threadIdx.x; j < ps.n[k]; j += blockDim.x)
            __hip_atomic_store(hdst + ps.o[k] + j, ps.p[k][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((threadIdx.x & 63) == 0)
        __hip_atomic_store(hseq + (threadIdx.x >> 6), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
u32 launch_spans_to_host(const PackSpans& ps, u32* hdst, u32* hseq, u32 seq, hipStream_t s) {
    u32 tot = 0;
    for (int k = 0; k < 6; ++k) tot += ps.p[k] ? ps.n[k] : 0;
    const u32 waves = std::max<u32>(1, std::min<u32>(4, (tot + 255) / 256));
    PackSpans q = ps;
    for (int k = 0; k < 6; ++k)
        if (!q.p[k]) q.n[k] = 0;
    k_spans_to_host<<<1, 64 * waves, 0, s>>>(q, hdst, hseq, seq);
    return waves;
}
void launch_small_sorts(SsClasses sc, bool w32, const SortArgs& a, const Lists& L, hipStream_t s) {
    u32 n = 0;
    for (int c = 5; c <= 11; ++c) {
        sc.wg0[c] = n;
        n += sc.count[c] ? cdiv(sc.count[c], TILE >> c) : 0u;
    }
    sc.wg0[12] = n;
    if (!n) return;
    if (w32)
        k_small_sort_all<u32><<<n, WG, 0, s>>>(sc, a, L);
    else
        k_small_sort_all<u64><<<n, WG, 0, s>>>(sc, a, L);
}
void launch_med_sort(const LSeg* segs, u32 nseg, const u32* ndev, const SortArgs& a, const Lists& L,
                     hipStream_t s) {
    if (!nseg || !a.med) return;
    k_med_sort<<<nseg, MED_NT, 0, s>>>(segs, ndev, a, L);
}
void launch_finalize_eq(const Seg* eq, u32 count, const SortArgs& a, const Lists& L, hipStream_t s) {
    if (count) k_finalize_eq<<<dim3(count, 32), WG, 0, s>>>(eq, a, L);
}
void launch_rounds_sum(const u32* blk_last, u32 nb, u64* out, hipStream_t s) {
    KOLM_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(u64), s));
    k_rounds_sum<<<1, 256, 0, s>>>(blk_last, nb, reinterpret_cast<unsigned long long*>(out));
}

void launch_update_done(u32* blk_done, u32* blk_last, const u32* blk_split, u32 nb, u32 round, hipStream_t s) {
    if (nb) k_update_done<<<cdiv(nb, 256), 256, 0, s>>>(blk_done, blk_last, blk_split, nb, round);
}

// ------------------------------------------------------------------------------------
// variable (content-defined) block geometry
// ------------------------------------------------------------------------------------
// vmap[k] = the block holding position k << vshift (last b with vb[b] <= k << vshift)
__global__ void k_vmap(const u32* vb, u32 nb, u32* vmap, u32 ngran, u32 vshift) {
    const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ngran) return;
    const u32 g = k << vshift;
    u32 lo = 0, hi = nb;
    while (hi - lo > 1) {
        const u32 m = (lo + hi) >> 1;
        if (vb[m] <= g) lo = m; else hi = m;
    }
    vmap[k] = lo;
}

// granule 2^vshift <= the shortest block: block_of walks at most one boundary per lookup
u32 geom_var_shift(const u32* hb, u32 nb) {
    u32 mn = 0xFFFFFFFFu;
    for (u32 b = 0; b < nb; ++b) mn = std::min(mn, hb[b + 1] - hb[b]);
    u32 s = 0;
    while (s < 16 && (2u << s) <= mn) ++s;
    return s;
}

void geom_init_var(Geom& g, const u32* hb, u32 nb, u32* d_vb, u32* d_vmap, u32 vshift, hipStream_t s) {
    g = Geom{};
    g.N = hb[nb];
    g.nb = nb;
    u32 mx = 1;
    for (u32 b = 0; b < nb; ++b) mx = std::max(mx, hb[b + 1] - hb[b]);
    g.bs = mx;
    g.magic = 0;
    g.shift = 0;
    g.vb = d_vb;
    g.hvb = hb;
    g.vmap = d_vmap;
    g.vshift = vshift;
    KOLM_HIP_CHECK(hipMemcpyAsync(d_vb, hb, sizeof(u32) * ((u64)nb + 1), hipMemcpyHostToDevice, s));
    const u32 ngran = g.N ? (u32)((g.N - 1) >> vshift) + 1 : 0u;
    if (ngran) k_vmap<<<cdiv(ngran, 256), 256, 0, s>>>(d_vb, nb, d_vmap, ngran, vshift);
    KOLM_HIP_CHECK(hipStreamSynchronize(s));  // hb is pageable caller memory
}

}  // namespace kolm
