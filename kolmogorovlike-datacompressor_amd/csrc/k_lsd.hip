// Round 0 of the cyclic suffix sort (gfx950): every block's positions stably sorted by the
// first 4 characters of their rotation (4 LSD passes of 8 bits, 4096-element tiles:
// per-wave LDS histograms -> per-block scan over (digit, tile) -> stable scatter with wave
// ballot ranking), then group starts, ranks and the next round's segments (k_sort.hip).
// No host synchronisation: a fixed sequence of launches on the sort stream.
#include "kolm_internal.h"

#include <string>

namespace kolm {

namespace {

constexpr u32 LSD_T = 4096;          // elements per tile
constexpr u32 LSD_PT = LSD_T / WG;     // 16 per thread

struct LsdGeom {
    Geom geo;
    u32 tpb;  // tiles per block
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

// where a pass reads its (key, position) pairs: keys by position (first pass) or pairs
enum Src { SRC_KP = 1, SRC_PAIR = 2 };

template <int P, int SRC>
__global__ __launch_bounds__(WG) void k_lsd_hist(LsdGeom g, const u32* K, u32* hist) {
    __shared__ u32 h[WG / 64][256];
    const u32 tid = threadIdx.x, w = tid >> 6;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) h[i][tid] = 0;
    __syncthreads();
    u32 lo, hi, b;
    if (g.range(xcd_tile(), lo, hi, b)) {
        // 16 consecutive keys per thread, four 16-byte loads when aligned (order is irrelevant)
        const u32 i0 = lo + tid * LSD_PT;
        if ((i0 & 3) == 0 && i0 + LSD_PT <= hi) {
            const uint4* p = reinterpret_cast<const uint4*>(K + i0);
            uint4 v[LSD_PT / 4];
#pragma unroll
            for (u32 q = 0; q < LSD_PT / 4; ++q) v[q] = p[q];
#pragma unroll
            for (u32 q = 0; q < LSD_PT / 4; ++q) {
                atomicAdd(&h[w][digit<P>(v[q].x)], 1u);
                atomicAdd(&h[w][digit<P>(v[q].y)], 1u);
                atomicAdd(&h[w][digit<P>(v[q].z)], 1u);
                atomicAdd(&h[w][digit<P>(v[q].w)], 1u);
            }
        } else {
            for (u32 i = i0; i < min(i0 + LSD_PT, hi); ++i) atomicAdd(&h[w][digit<P>(K[i])], 1u);
        }
    }
    __syncthreads();
    hist[(u64)xcd_tile() * 256 + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
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

// Stable scatter of one tile by digit P: element order e = j*WG + tid; each wave ranks
// its 64 elements per digit with ballots, per-wave counts are combined in (j, wave)
// order.  SRC_KP reads the keys by position (positions implicit).
// G: the pass writes Kg[position] as the key (the next digit set, gathered by position)
// instead of the key it sorted by — the last pass of the 8-character sort's first half.
template <int P, int SRC, int G>
__global__ __launch_bounds__(WG) void k_lsd_scatter(LsdGeom g, const u32* Kin, const u32* Pin,
                                                   u32* Kout, u32* Pout, const u32* Kg, const u32* hist) {
    __shared__ u32 wcnt[WG / 64][256];
    __shared__ u32 running[256];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32 lo, hi, b;
    if (!g.range(xcd_tile(), lo, hi, b)) return;
    running[tid] = hist[(u64)xcd_tile() * 256 + tid];
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) wcnt[i][tid] = 0;
    __syncthreads();
    const u64 lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (u32 j = 0; j < LSD_PT; ++j) {
        const u32 i = lo + j * WG + tid;
        const bool valid = i < hi;
        u32 key = 0, pos = 0, dg = 0;
        if (valid) {
            if (SRC == SRC_KP) {
                key = Kin[i];
                pos = i;
            } else {
                key = Kin[i];
                pos = Pin[i];
            }
            dg = digit<P>(key);
        }
        u64 m = __ballot(valid);
#pragma unroll
        for (u32 bit = 0; bit < 8; ++bit) {
            const u64 bal = __ballot((dg >> bit) & 1u);
            m &= ((dg >> bit) & 1u) ? bal : ~bal;
        }
        const u32 rank = __popcll(m & lt_mask);
        if (valid && rank == 0) wcnt[w][dg] = __popcll(m);
        __syncthreads();
        if (valid) {
            u32 pre = running[dg];
            for (u32 q = 0; q < w; ++q) pre += wcnt[q][dg];
            const u32 dst = pre + rank;
            Kout[dst] = G ? Kg[pos] : key;
            Pout[dst] = pos;
        }
        __syncthreads();
        u32 add = 0;
#pragma unroll
        for (int q = 0; q < WG / 64; ++q) {
            add += wcnt[q][tid];
            wcnt[q][tid] = 0;
        }
        running[tid] += add;
        __syncthreads();
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

// ---------------------------------------------------------------------------------
// Round 0 of the cyclic suffix sort: after 4 LSD passes over the 4-character rotation
// keys (K sorted, SA = positions), slot g starts a group iff g is the block's first slot
// or K[g] != K[g-1].  Every position gets RK = its group's first slot (PY's (fi, i) tie
// rule is position order, kept by the stable passes); groups of >= 2 go to the next
// round; a block with more than one group has split.
// ---------------------------------------------------------------------------------
constexpr u32 BIG = 0xFFFFFFFFu;

__device__ inline u32 wave_min(u32 v) { return wave_reduce(v, OpMinU(), BIG); }

// Group heads of every tile: bit e of HF[t * WG + tid] = slot lo + 16 tid + e starts a group
// (the block's first slot, or its key differs from the previous slot's; with KA — the
// 8-character round 0, K = characters 0..3 — also when characters 4..7, KA[SA[slot]],
// differ).  tmax / tmin = the tile's last / first head.
__global__ __launch_bounds__(WG) void k_r0_tile_heads(LsdGeom g, const u32* K, const u32* SA, const u32* KA, u32* HF,
                                                      u32* tmax, u32* tmin) {
    __shared__ u32 s1[WG / 64], s2[WG / 64];
    const u32 t = xcd_tile();
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
            if (KA) {
                u32 sv[LSD_PT];
                load16(SA, i0, hi, sv);
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

__global__ __launch_bounds__(WG) void k_r0_final(LsdGeom g, const u32* HF, const u32* SA, const u32* cmax,
                                                 const u32* cmin, u32* RK, Seg* next, u32* next_cnt,
                                                 u32* blk_split) {
    __shared__ u32 sh[WG / 64], sh2[WG / 64], sh3[WG / 64];
    __shared__ u32 wbase, anysplit;
    u32 lo, hi, b;
    if (!g.range(blockIdx.x, lo, hi, b)) return;
    const u32 base = g.geo.base(b), bend = g.geo.end(b);
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) anysplit = 0;
    const u32 i0 = lo + tid * LSD_PT;
    u32 sv[LSD_PT];
    load16(SA, i0, hi, sv);
    const u32 hm = HF[(u64)blockIdx.x * WG + tid];
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
    u32 run = max(cmax[blockIdx.x], fex);
    for (u32 q = 0; q < w; ++q) run = max(run, sh[q]);
    u32 nh = min(cmin[blockIdx.x], rex);
    for (u32 q = w + 1; q < WG / 64; ++q) nh = min(nh, sh2[q]);
    if (nh == BIG) nh = bend;
    // ranks
    bool split = false;
#pragma unroll
    for (u32 e = 0; e < LSD_PT; ++e) {
        const u32 i = i0 + e;
        if (i < hi) {
            if (hd[e]) {
                run = i;
                split |= i != base;
            }
            RK[sv[e]] = run;
        }
    }
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

template <int P, int SRC, int G>
void lsd_pass(const LsdGeom& g, u32 nt, const u32* kin, const u32* pin, u32* kout, u32* pout, const u32* kg,
              u32* hist, hipStream_t s, KTimer* kt) {
    static const std::string hn = "k_lsd_hist<" + std::to_string(P) + ", " + std::to_string(SRC) + ">";
    static const std::string sn =
        "k_lsd_scatter<" + std::to_string(P) + ", " + std::to_string(SRC) + ", " + std::to_string(G) + ">";
    const u64 N = g.geo.N, H = (u64)nt * 1024;  // H: per-tile histogram bytes
    {
        KScope k(kt, KT_LSD, hn.c_str(), 4 * N + H);
        k_lsd_hist<P, SRC><<<nt, WG, 0, s>>>(g, kin, hist);
    }
    {
        KScope k(kt, KT_LSD, "k_lsd_scan", 3 * H);
        k_lsd_scan<<<g.geo.nb, WG, 0, s>>>(g, hist);
    }
    {
        // key + position in (the first pass reads the key by position only) and out; G: + the gather
        KScope k(kt, KT_LSD, sn.c_str(), (SRC == SRC_KP ? 12 : 16) * N + (G ? 4 * N : 0) + H);
        k_lsd_scatter<P, SRC, G><<<nt, WG, 0, s>>>(g, kin, pin, kout, pout, kg, hist);
    }
}

}  // namespace

u32 lsd_tiles(const Geom& geo) { return (geo.bs + LSD_T - 1) / LSD_T * geo.nb; }

// Round 0 of the cyclic sort: a stable sort of every block's positions by the first 4 or 8
// rotation characters (KP = characters 0..3 by position; 8 characters: RK holds characters
// 4..7 by position on entry).  4 characters: (KP, p) -> (K2, SA) -> (K22, SA2) -> (KP, RK) ->
// (K2, SA).  8 characters: 4 passes over characters 4..7 (RK, p) -> (K22, SA2) -> (K2, SA)
// -> (K22, SA2) -> (K2 = KP[SA], SA), then 4 over characters 0..3 ending in (K2, SA).  Then
// group heads (HF), ranks and next-round segments.
void launch_round0(const Geom& geo, const R0Bufs& t, Seg* next, u32* next_cnt, u32* blk_split, hipStream_t s,
                   KTimer* kt) {
    if (!geo.N) return;
    LsdGeom g{geo, (geo.bs + LSD_T - 1) / LSD_T};
    const u32 nt = g.tpb * geo.nb;
    const u64 N = geo.N;
    const bool c8 = t.chars == 8;
    if (!c8) {
        lsd_pass<0, SRC_KP, 0>(g, nt, t.KP, nullptr, t.K2, t.SA, nullptr, t.hist, s, kt);
        lsd_pass<1, SRC_PAIR, 0>(g, nt, t.K2, t.SA, t.K22, t.SA2, nullptr, t.hist, s, kt);
        lsd_pass<2, SRC_PAIR, 0>(g, nt, t.K22, t.SA2, t.KP, t.RK, nullptr, t.hist, s, kt);
        lsd_pass<3, SRC_PAIR, 0>(g, nt, t.KP, t.RK, t.K2, t.SA, nullptr, t.hist, s, kt);
    } else {
        lsd_pass<0, SRC_KP, 0>(g, nt, t.RK, nullptr, t.K22, t.SA2, nullptr, t.hist, s, kt);
        lsd_pass<1, SRC_PAIR, 0>(g, nt, t.K22, t.SA2, t.K2, t.SA, nullptr, t.hist, s, kt);
        lsd_pass<2, SRC_PAIR, 0>(g, nt, t.K2, t.SA, t.K22, t.SA2, nullptr, t.hist, s, kt);
        lsd_pass<3, SRC_PAIR, 1>(g, nt, t.K22, t.SA2, t.K2, t.SA, t.KP, t.hist, s, kt);
        lsd_pass<0, SRC_PAIR, 0>(g, nt, t.K2, t.SA, t.K22, t.SA2, nullptr, t.hist, s, kt);
        lsd_pass<1, SRC_PAIR, 0>(g, nt, t.K22, t.SA2, t.K2, t.SA, nullptr, t.hist, s, kt);
        lsd_pass<2, SRC_PAIR, 0>(g, nt, t.K2, t.SA, t.K22, t.SA2, nullptr, t.hist, s, kt);
        lsd_pass<3, SRC_PAIR, 0>(g, nt, t.K22, t.SA2, t.K2, t.SA, nullptr, t.hist, s, kt);
    }
    {
        // K 4 (+ SA 4 + the KA gather 4) read, head masks written
        KScope k(kt, KT_LSD, "k_r0_tile_heads", (c8 ? 12 : 4) * N);
        k_r0_tile_heads<<<nt, WG, 0, s>>>(g, t.K2, t.SA, c8 ? t.RK : nullptr, t.HF, t.tmax, t.tmin);
        k_tiles_max_scan<<<geo.nb, WG, 0, s>>>(t.tmax, t.cmax, g.tpb);
        k_r0_tiles_rscan<<<geo.nb, WG, 0, s>>>(t.tmin, t.cmin, g.tpb);
    }
    {
        // SA 4 read, RK 4 scattered (+ head masks, 8 B per new segment)
        KScope k(kt, KT_LSD, "k_r0_final", 8 * N);
        k_r0_final<<<nt, WG, 0, s>>>(g, t.HF, t.SA, t.cmax, t.cmin, t.RK, next, next_cnt, blk_split);
    }
}

}  // namespace kolm
