// FastCDC content-defined chunking (PY:140-309 cdc_fast_boundaries_strict) on gfx950.
//
// The reference rolls fp' = (fp << 1) + GEAR[byte] (mod 2^32) from each chunk's min-size
// point (PY:270-271) and cuts after the first position whose fp has its low k_s bits clear
// before the normal size (MaskS, PY:274-281) or its low k_l bits clear after it (MaskL,
// PY:283-291), else at the local maximum (PY:293-295).  Bit i of fp depends only on the
// last i+1 rolled bytes, so at any position 32 or more bytes past the roll's start every
// mask test (k <= 20 bits) equals the same test on the unclipped window hash
//     H(p) = sum_{j<32} GEAR[d[p-j]] << j   (mod 2^32).
// The chunk chain is a function of the chunk start alone, which makes it parallel:
//   1. k_cdc_flags   H(p) for every position, one thread per 64 positions (a 96-byte
//                    roll), into two bitmaps: S (MaskS clear) and L (MaskL clear).
//   2. k_cdc_spec    one wave per segment runs the chain speculatively from the segment
//                    start as if a chunk started there: the first 64 positions past a
//                    chunk's min point get their clipped roll exactly (one lane each), the
//                    rest come from the bitmaps (64 words per wave step, ballot for the
//                    first hit).  Cuts -> bitmap C; the first cut past the segment -> exit.
//   3. k_cdc_stitch  one wave walks the segments in order with the TRUE entry: an entry
//                    that is the segment start or a speculative cut joins the speculative
//                    chain (same start, same chain); otherwise the true chain runs from the
//                    entry until it meets a speculative cut (fix-up cuts -> bitmap F).
//                    Content-defined cuts re-synchronise within a chunk or two.
//   4. k_cdc_count / k_cdc_scan / k_cdc_emit: true cuts = F | (C from each segment's join
//                    point on); per-workgroup popcounts, one exclusive scan, positions in
//                    ascending order.
// The orphan-tail merge (PY:300-306) is applied by the host to the returned list.
// Bound: the flags pass streams the input once (1 B/position + 2 bits out); the chain
// passes touch a few bitmap words per chunk.
#include <algorithm>
#include <numeric>

#include "kolm_internal.h"

namespace kolm {

namespace {

constexpr u32 CDC_NONE = 0xFFFFFFFFu;

struct CdcArgs {
    const u8* d;
    u32 n, mn, av, mx;
    u32 ms, ml;            // MaskS / MaskL (PY:238-240)
    const u32* gear;       // [256] PY's GEAR table
    u64 *WS, *WL, *C, *F;  // [nw] bitmaps, bit p & 63 of word p >> 6
    u32* exitp;            // [nseg] first speculative cut at or past the segment end
    u32* join;             // [nseg] position where the true chain joins the speculative one
    u32* wgcnt;            // [nwg] true cuts per 256-word group -> exclusive offsets
    u32* cuts;             // out: true cut positions, ascending
    u32* total;            // out: number of true cuts
    u32 seg, nseg, nw;
    int vec;               // d is 16-byte aligned
};

__device__ inline void load_gear(const u32* g, u32* lg) {
    for (u32 i = threadIdx.x; i < 256; i += blockDim.x) lg[i] = g[i];
    __syncthreads();
}

__device__ inline bool bit_at(const u64* B, u32 p) { return (B[p >> 6] >> (p & 63)) & 1ull; }

__device__ inline void set_bit(u64* B, u32 p) {
    atomicOr(reinterpret_cast<unsigned long long*>(&B[p >> 6]), 1ull << (p & 63));
}

__device__ inline u64 shfl64(u64 v, u32 src) {
    const u32 lo = (u32)__shfl((int)(u32)v, (int)src), hi = (u32)__shfl((int)(u32)(v >> 32), (int)src);
    return ((u64)hi << 32) | lo;
}

// 1. window hashes of 64 positions per thread -> S / L bitmap words
__global__ __launch_bounds__(256) void k_cdc_flags(CdcArgs a) {
    __shared__ u32 G[256];
    load_gear(a.gear, G);
    const u32 w = blockIdx.x * 256 + threadIdx.x;
    if (w >= a.nw) return;
    const u32 p0 = w << 6;
    u64 s = 0, l = 0;
    u32 h = 0;
    if (a.vec && p0 >= 32 && p0 + 64 <= a.n) {
        // bytes p0-32 .. p0+63 as six 16-byte loads; the 32 leading bytes fill the window
        const uint4* src = reinterpret_cast<const uint4*>(a.d + p0 - 32);
        u32 wv[24];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint4 v = src[k];
            wv[4 * k] = v.x;
            wv[4 * k + 1] = v.y;
            wv[4 * k + 2] = v.z;
            wv[4 * k + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) h = (h << 1) + G[(wv[i >> 2] >> (8 * (i & 3))) & 0xFF];
#pragma unroll
        for (int e = 0; e < 64; ++e) {
            h = (h << 1) + G[(wv[8 + (e >> 2)] >> (8 * (e & 3))) & 0xFF];
            s |= (u64)((h & a.ms) == 0) << e;
            l |= (u64)((h & a.ml) == 0) << e;
        }
    } else {
        for (u32 i = p0 >= 32 ? p0 - 32 : 0; i < p0; ++i) h = (h << 1) + G[a.d[i]];
        const u32 e1 = min(p0 + 64, a.n);
        for (u32 p = p0; p < e1; ++p) {
            h = (h << 1) + G[a.d[p]];
            s |= (u64)((h & a.ms) == 0) << (p - p0);
            l |= (u64)((h & a.ml) == 0) << (p - p0);
        }
    }
    a.WS[w] = s;
    a.WL[w] = l;
}

// End of the chunk that starts at s: one iteration of PY:247-298, wave-uniform result.
__device__ u32 cdc_next(const CdcArgs& a, const u32* G, u32 s) {
    const u32 lane = threadIdx.x & 63;
    const u32 rem = a.n - s;
    if (rem <= a.mn) return a.n;  // PY:251-256
    const u32 lmax = min(rem, a.mx);
    const u32 emin = s + a.mn, enorm = s + min(a.av, lmax), elim = s + lmax;
    {
        // positions emin .. emin+63: the roll restarted at emin (fp = 0), exactly
        const u32 p = emin + lane;
        bool hit = false;
        if (p < elim) {
            u32 h = 0;
            for (u32 j = p - emin >= 32 ? p - 31 : emin; j <= p; ++j) h = (h << 1) + G[a.d[j]];
            hit = (h & (p < enorm ? a.ms : a.ml)) == 0;
        }
        const u64 m = __ballot(hit);
        if (m) return emin + (u32)__ffsll((unsigned long long)m);  // cut after that position
    }
    // later positions: window hashes, 64 bitmap words (4096 positions) per step
    for (u32 w0 = (emin + 64) >> 6, q = emin + 64; q < elim; w0 += 64, q = w0 << 6) {
        const u32 w = w0 + lane, wp = w << 6;
        u64 bits = 0;
        if (wp < elim) {
            u64 valid = ~0ull;
            if (wp < q) valid <<= (q - wp);
            if (elim - wp < 64) valid &= (1ull << (elim - wp)) - 1ull;
            const u64 useS = enorm <= wp ? 0ull : enorm - wp >= 64 ? ~0ull : (1ull << (enorm - wp)) - 1ull;
            bits = ((a.WS[w] & useS) | (a.WL[w] & ~useS)) & valid;
        }
        const u64 m = __ballot(bits != 0);
        if (m) {
            const u32 L = (u32)__ffsll((unsigned long long)m) - 1;
            const u64 bb = shfl64(bits, L);
            return ((w0 + L) << 6) + (u32)__ffsll((unsigned long long)bb);
        }
    }
    return elim;
}

// 2. speculative chain per segment (4 waves per workgroup, one segment each)
__global__ __launch_bounds__(256) void k_cdc_spec(CdcArgs a) {
    __shared__ u32 G[256];
    load_gear(a.gear, G);
    const u32 k = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= a.nseg) return;
    const u32 lane = threadIdx.x & 63;
    const u32 S1 = min((k + 1) * a.seg, a.n);
    u32 s = k * a.seg;
    for (;;) {
        const u32 c = cdc_next(a, G, s);
        if (c >= S1) {
            if (lane == 0) a.exitp[k] = c;
            break;
        }
        if (lane == 0) set_bit(a.C, c);
        s = c;
    }
}

// 3. the true chain over the segments (one wave)
__global__ __launch_bounds__(64) void k_cdc_stitch(CdcArgs a) {
    __shared__ u32 G[256];
    load_gear(a.gear, G);
    const u32 lane = threadIdx.x;
    u32 e = 0;  // start of the chunk being entered
    for (u32 k = 0; k < a.nseg; ++k) {
        const u32 S0 = k * a.seg, S1 = min(S0 + a.seg, a.n);
        u32 jn = CDC_NONE;
        if (e < S1) {
            u32 s = e, nx = 0;
            bool joined = s == S0 || bit_at(a.C, s);
            while (!joined) {
                const u32 c = cdc_next(a, G, s);
                if (c >= S1) {
                    nx = c;
                    break;
                }
                if (lane == 0) set_bit(a.F, c);
                s = c;
                joined = bit_at(a.C, c);
            }
            if (joined) {
                jn = s;
                e = a.exitp[k];
            } else {
                e = nx;
            }
            if (lane == 0 && e < a.n) set_bit(a.F, e);
        }
        if (lane == 0) a.join[k] = jn;
    }
}

// true cuts of bitmap word w: fix-up cuts, and speculative cuts at or after the join point
__device__ inline u64 true_word(const CdcArgs& a, u32 w) {
    const u32 wp = w << 6;
    const u32 jn = a.join[wp / a.seg];
    u64 c = 0;
    if (jn != CDC_NONE) {
        c = a.C[w];
        if (jn > wp) c = jn - wp >= 64 ? 0ull : c & (~0ull << (jn - wp));
    }
    return c | a.F[w];
}

// 4. per-group counts, one exclusive scan, positions
__global__ __launch_bounds__(256) void k_cdc_count(CdcArgs a) {
    __shared__ u32 sh[WG / 64];
    const u32 w = blockIdx.x * 256 + threadIdx.x;
    const u32 v = w < a.nw ? (u32)__popcll(true_word(a, w)) : 0u;
    const u32 t = wave_reduce(v, OpAddU(), 0u);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) a.wgcnt[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(256) void k_cdc_scan(u32* cnt, u32 nwg, u32* total) {
    __shared__ u32 sh[WG / 64];
    __shared__ u32 carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (u32 c0 = 0; c0 < nwg; c0 += 256) {
        const u32 i = c0 + threadIdx.x;
        const u32 v = i < nwg ? cnt[i] : 0u;
        const u32 incl = wave_incl_scan(v, OpAddU(), 0u);
        if (lane == 63) sh[wv] = incl;
        __syncthreads();
        u32 pre = carry;
        for (u32 q = 0; q < wv; ++q) pre += sh[q];
        if (i < nwg) cnt[i] = pre + incl - v;
        __syncthreads();
        if (threadIdx.x == 255) carry = pre + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void k_cdc_emit(CdcArgs a) {
    __shared__ u32 sh[WG / 64];
    const u32 w = blockIdx.x * 256 + threadIdx.x;
    const u64 tw = w < a.nw ? true_word(a, w) : 0ull;
    const u32 v = (u32)__popcll(tw);
    const u32 incl = wave_incl_scan(v, OpAddU(), 0u);
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 63) sh[wv] = incl;
    __syncthreads();
    u32 o = a.wgcnt[blockIdx.x] + incl - v;
    for (u32 q = 0; q < wv; ++q) o += sh[q];
    u64 x = tw;
    while (x) {
        const u32 bit = (u32)__ffsll((unsigned long long)x) - 1;
        x &= x - 1;
        a.cuts[o++] = (w << 6) + bit;
    }
}

}  // namespace

// Segment length: about 32 average chunks, a multiple of 64 (bitmap words never straddle
// two segments) and, when that stays small, of max_size: PY's GEAR entries are all odd
// (PY:164), so every fingerprint is odd, no mask test passes and the reference cuts every
// chunk at max_size -- with segments a multiple of it, each segment start is a true cut
// and the stitch joins at once instead of walking the chain.
u32 cdc_segment(u32 avg, u32 mx) {
    const u64 target = std::min<u64>(std::max<u64>(4096, 32ull * avg), 1ull << 22);
    const u64 l = (u64)mx / std::gcd<u64>(mx, 64) * 64;  // lcm(max_size, 64)
    if (l <= (1ull << 22)) return (u32)((target + l - 1) / l * l);
    u64 s = 4096;
    while (s < target && s < (1ull << 22)) s <<= 1;
    return (u32)s;
}

void launch_cdc(const CdcParams& p, const CdcBufs& b, hipStream_t s, KTimer* kt) {
    if (!p.n) return;
    CdcArgs a{};
    a.d = p.d;
    a.n = p.n;
    a.mn = p.mn;
    a.av = p.av;
    a.mx = p.mx;
    a.ms = p.ms;
    a.ml = p.ml;
    a.gear = b.gear;
    a.WS = b.WS;
    a.WL = b.WL;
    a.C = b.C;
    a.F = b.F;
    a.exitp = b.exitp;
    a.join = b.join;
    a.wgcnt = b.wgcnt;
    a.cuts = b.cuts;
    a.total = b.total;
    a.nw = (p.n + 63) / 64;
    a.seg = cdc_segment(p.av, p.mx);
    a.nseg = (p.n + a.seg - 1) / a.seg;
    a.vec = ((uintptr_t)p.d & 15) == 0;
    const u32 nwg = (a.nw + 255) / 256;
    KOLM_HIP_CHECK(hipMemsetAsync(b.C, 0, sizeof(u64) * a.nw, s));
    KOLM_HIP_CHECK(hipMemsetAsync(b.F, 0, sizeof(u64) * a.nw, s));
    {
        KScope k(kt, KT_CDC, "k_cdc_flags", (u64)p.n + (u64)a.nw * 16);  // text once + two bitmaps
        k_cdc_flags<<<nwg, 256, 0, s>>>(a);
    }
    {
        KScope k(kt, KT_CDC, "k_cdc_spec", (u64)a.nseg * 64);
        k_cdc_spec<<<(a.nseg + 3) / 4, 256, 0, s>>>(a);
    }
    {
        KScope k(kt, KT_CDC, "k_cdc_stitch", (u64)a.nseg * 16);
        k_cdc_stitch<<<1, 64, 0, s>>>(a);
    }
    {
        KScope k(kt, KT_CDC, "k_cdc_cuts", (u64)a.nw * 32);  // C + F read twice
        k_cdc_count<<<nwg, 256, 0, s>>>(a);
        k_cdc_scan<<<1, 256, 0, s>>>(b.wgcnt, nwg, b.total);
        k_cdc_emit<<<nwg, 256, 0, s>>>(a);
    }
}

}  // namespace kolm
