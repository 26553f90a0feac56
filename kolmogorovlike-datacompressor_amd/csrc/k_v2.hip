// Candidate 10, v2_new: encode_new_pipeline PY:1498-1576 (gfx950).
//
// As shipped, the reference calls circuit_map_automaton_forward with parallel=True and
// raises NameError (os / ProcessPoolExecutor are never imported, PY:1037-1043), so PY
// never emits id 10 and the default candidate mask leaves it out.  With
// KOLM_M_V2NEW in the mask the pipeline's defined result is computed — the automaton
// evaluated serially (PY:1033-1035), SURVEY §8f row 3 — and is bit-exact against PY's own
// encode_new_pipeline run that way (tests/golden/v2new.npz).
//
//   1. k_v2_hist     per 4 KiB tile, the byte histograms of the 13 automaton candidates
//                    (identity, delta-k k=1..4, 4 Gray variants, nibble interleave,
//                    majority-of-3, morpho close/open — PY:664-900; every model is
//                    out[i] = raw[i] ^ predictor(raw[i-1..i-4])), in LDS, flushed per block
//   2. k_v2_select   per block: H0 of each candidate (PY:631-643: bins summed in index order
//                    in double) folded in PY's `kinds` order by _pick_better (PY:936-950)
//   3. k_v2_planes   the winner's mapped bytes split into 8 MSB-first bit-planes (PY:1137)
//                    laid out as 8 consecutive "plane blocks" per block (block b, plane j =
//                    [8*base(b) + j*len(b), +len(b)))
//   4. (kolm_api.cpp) Lyndon + cyclic sort + gather of every plane block: the BBWT of each
//                    binary plane (PY:1539), by the same batched pipeline as candidates 2..6
//   5. k_v2_runs     per plane block (one workgroup): runs of the BBWT output (rle_binary
//                    PY:1177) and the Rice bit count of the run lengths for k = 0..15
//                    (_choose_best_rice PY:1489: first minimal byte size)
//   6. k_v2_size     per block: raw vs encoded per plane (raw <= rice + 1 -> raw), slim header
//                    size (PY:1558-1576) -> the candidate's payload size for the MDL
//   7. emission      header bytes; raw planes packed MSB-first (PY:1191); encoded planes'
//                    runs Rice-coded at bit offsets from a per-plane scan of the code lengths
#include <cmath>

#include "kolm_internal.h"

namespace kolm {

namespace {

constexpr u32 V2T = 4096;   // positions per histogram tile
constexpr u32 V2C = 13;     // automaton candidates
constexpr u32 RWG = 1024;   // threads of a per-plane-block workgroup
constexpr u32 RPER = 8;     // positions per thread per step in those workgroups

// (model code, param) of the candidates in PY's `kinds` order (PY:1024-1030)
__constant__ u8 kV2Kind[V2C][2] = {{0, 0}, {1, 1}, {1, 2}, {1, 3}, {1, 4}, {2, 0}, {2, 1},
                                   {2, 2}, {2, 3}, {3, 0}, {4, 0}, {5, 0}, {5, 1}};

__device__ inline u8 gray8(u32 v) { return (u8)(v ^ (v >> 1)); }
__device__ inline u8 dil1(u32 x) { return (u8)((((x << 1) & 0xFE) | x) | (((x >> 1) & 0x7F) | x)); }
__device__ inline u8 ero1(u32 x) { return (u8)(~dil1((u8)~x) & 0xFF); }

// predictor of the byte at block offset rel from the raw bytes before it (r1 = raw[rel-1], ...)
__device__ inline u8 v2_pred(u32 code, u32 param, u32 rel, u8 r1, u8 r2, u8 r3, u8 r4) {
    switch (code) {
        case 1: {  // Delta-k PY:664-690
            if (rel < param) return 0;
            return param == 1 ? r1 : param == 2 ? r2 : param == 3 ? r3 : r4;
        }
        case 2: {  // Gray family PY:698-752
            if (rel == 0) return 0;
            if (rel == 1) return r1;
            const u32 v = param & 3;
            return gray8(v == 0 ? r1 : v == 1 ? r2 : v == 2 ? (u32)(r1 ^ r2) : (u32)(r1 | r2));
        }
        case 3: {  // Nibble-MUX interleave PY:780-826: mux(select, cross, run) = cross
            if (rel == 0) return 0;
            if (rel == 1) return r1;
            const u8 cross = (u8)((r1 & 0xF0) | (r2 & 0x0F));
            const u8 hi_eq = ((r1 ^ r2) & 0xF0) ? 0x00 : 0xF0, lo_eq = ((r1 ^ r2) & 0x0F) ? 0x00 : 0x0F;
            const u8 sel = (u8)((((u8)~hi_eq) & 0xF0) | (((u8)~lo_eq) & 0x0F));
            return (u8)((cross & sel) | (r1 & (u8)~sel));
        }
        case 4:  // Majority-of-3 PY:828-866
            if (rel == 0) return 0;
            if (rel < 3) return r1;
            return (u8)((r1 & r2) | (r1 & r3) | (r2 & r3));
        case 5: {  // Morpho-Predict PY:868-900
            if (rel == 0) return 0;
            const u8 m = (param & 1) == 0 ? ero1(dil1(r1)) : dil1(ero1(r1));
            const u8 e = (u8)(dil1(r1) ^ ero1(r1));
            return (u8)((m & e) | (r1 & (u8)~e));
        }
        default:
            return 0;
    }
}

struct Near {
    u8 x, r1, r2, r3, r4;
};
__device__ inline Near near_bytes(const u8* text, u32 p, u32 rel) {
    Near v;
    v.x = text[p];
    v.r1 = rel >= 1 ? text[p - 1] : 0;
    v.r2 = rel >= 2 ? text[p - 2] : 0;
    v.r3 = rel >= 3 ? text[p - 3] : 0;
    v.r4 = rel >= 4 ? text[p - 4] : 0;
    return v;
}

__global__ __launch_bounds__(256) void k_v2_hist(Geom geo, const u8* text, u32 tpb, u32* hist) {
    __shared__ u32 h[V2C][256];
    for (u32 i = threadIdx.x; i < V2C * 256; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    const u32 b = blockIdx.x / tpb, k = blockIdx.x - b * tpb;
    const u32 base = geo.base(b), end = geo.end(b);
    const u32 lo = base + k * V2T, hi = min(lo + V2T, end);
    for (u32 p = lo + threadIdx.x; p < hi; p += 256) {
        const u32 rel = p - base;
        const Near v = near_bytes(text, p, rel);
#pragma unroll
        for (u32 c = 0; c < V2C; ++c)
            atomicAdd(&h[c][(u8)(v.x ^ v2_pred(kV2Kind[c][0], kV2Kind[c][1], rel, v.r1, v.r2, v.r3, v.r4))], 1u);
    }
    __syncthreads();
    if (lo >= hi) return;
    u32* hb = hist + (u64)b * V2C * 256;
    for (u32 i = threadIdx.x; i < V2C * 256; i += 256)
        if ((&h[0][0])[i]) atomicAdd(hb + i, (&h[0][0])[i]);
}

// Per block: H0 of the 13 candidates (PY:631-643 order: bins 0..255, H -= p*log2(p)) and
// the _pick_better fold (PY:936-950, 1005-1011).  sel[b] = code | param << 8.
__global__ __launch_bounds__(256) void k_v2_select(Geom geo, const u32* hist, u32* sel) {
    __shared__ double term[V2C][256];
    const u32 b = blockIdx.x, t = threadIdx.x;
    const double n = (double)(geo.end(b) - geo.base(b));
    const u32* hb = hist + (u64)b * V2C * 256;
    for (u32 c = 0; c < V2C; ++c) {
        const u32 f = hb[c * 256 + t];
        double v = 0.0;
        if (f) {
            const double p = (double)f / n;
            v = p * log2(p);
        }
        term[c][t] = v;
    }
    __syncthreads();
    if (t != 0) return;
    u32 code = 0, param = 0;
    double bh = 0.0;
    for (u32 c = 0; c < V2C; ++c) {
        double H = 0.0;
        for (u32 v = 0; v < 256; ++v)
            if (hb[c * 256 + v]) H -= term[c][v];
        const u32 cc = kV2Kind[c][0], cp = kV2Kind[c][1];
        bool take = c == 0;
        if (!take) {
            if (H < bh - 1e-12) take = true;
            else if (fabs(H - bh) <= 1e-12 && (cc < code || (cc == code && cp < param))) take = true;
        }
        if (take) {
            bh = H;
            code = cc;
            param = cp;
        }
    }
    sel[b] = code | (param << 8);
}

// mapped byte -> 8 plane bytes (0/1) at [8*base + j*len + rel]
__global__ __launch_bounds__(256) void k_v2_planes(Geom geo, const u8* text, const u32* sel, u8* U) {
    const u32 p = blockIdx.x * 256 + threadIdx.x;
    if (p >= geo.N) return;
    const u32 b = geo.block_of(p), base = geo.base(b), len = geo.end(b) - base, rel = p - base;
    const u32 s = sel[b];
    const Near v = near_bytes(text, p, rel);
    const u8 m = (u8)(v.x ^ v2_pred(s & 0xFF, s >> 8, rel, v.r1, v.r2, v.r3, v.r4));
    u8* o = U + 8ull * base + rel;
#pragma unroll
    for (u32 j = 0; j < 8; ++j) o[(u64)j * len] = (m >> (7 - j)) & 1;
}

__device__ inline u64 wg_sum64(u64 v, u64* sh) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    u64 t = 0;
    for (u32 i = 0; i < blockDim.x / 64; ++i) t += sh[i];
    return t;
}

// Runs of one plane block's BBWT output, walked in order by one workgroup: a run ends at
// every run start after the first (and at the plane end); F(len) is called per run by the
// thread that owns the run's end.  prev = the previous run start, from a workgroup max-scan
// of each thread's last start plus the carry of the previous step.
template <class F>
__device__ void v2_walk_runs(const u8* L, u32 n, u32* sh, u32* carry_s, F&& f) {
    const u32 t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) *carry_s = 0;
    __syncthreads();
    for (u32 c0 = 0; c0 < n; c0 += RWG * RPER) {
        const u32 i0 = c0 + t * RPER;
        u8 v[RPER + 1];
        v[0] = (i0 >= 1 && i0 - 1 < n) ? L[i0 - 1] : 0;
#pragma unroll
        for (u32 e = 0; e < RPER; ++e) v[e + 1] = i0 + e < n ? L[i0 + e] : 0;
        u32 last = 0;  // last run start inside my positions (0: none; position 0 is handled by carry)
#pragma unroll
        for (u32 e = 0; e < RPER; ++e) {
            const u32 i = i0 + e;
            if (i < n && i > 0 && v[e + 1] != v[e]) last = i;
        }
        const u32 incl = wave_incl_scan(last, OpMaxU(), 0u);
        const u32 ex = KOLM_DPP(0u, incl, DPP_WAVE_SHR1, 0xF);
        if (lane == 63) sh[w] = incl;
        __syncthreads();
        u32 prev = max(*carry_s, ex);
        for (u32 i = 0; i < w; ++i) prev = max(prev, sh[i]);
        u32 top = *carry_s;
        for (u32 i = 0; i < RWG / 64; ++i) top = max(top, sh[i]);
#pragma unroll
        for (u32 e = 0; e < RPER; ++e) {
            const u32 i = i0 + e;
            if (i < n && i > 0 && v[e + 1] != v[e]) {
                f(prev, i - prev);
                prev = i;
            }
        }
        __syncthreads();
        if (t == 0) *carry_s = top;
        __syncthreads();
    }
    if (t == 0 && n) f(*carry_s, n - *carry_s);  // the last run
}

// per plane block q (one workgroup): Rice bits of the runs for k = 0..15, first bit
__global__ __launch_bounds__(RWG) void k_v2_runs(const u32* pb, const u8* L, u64* rbits, u32* b1) {
    __shared__ u32 sh[RWG / 64];
    __shared__ u64 sh64[RWG / 64];
    __shared__ u32 carry;
    const u32 q = blockIdx.x, s = pb[q], n = pb[q + 1] - s;
    const u8* Lq = L + s;
    u64 acc[16];
#pragma unroll
    for (u32 k = 0; k < 16; ++k) acc[k] = 0;
    v2_walk_runs(Lq, n, sh, &carry, [&](u32, u32 r) {
#pragma unroll
        for (u32 k = 0; k < 16; ++k) acc[k] += (u64)(r >> k) + 1 + k;
    });
#pragma unroll
    for (u32 k = 0; k < 16; ++k) {
        const u64 tot = wg_sum64(acc[k], sh64);
        if (threadIdx.x == 0) rbits[(u64)q * 16 + k] = tot;
    }
    if (threadIdx.x == 0) b1[q] = n ? Lq[0] & 1 : 0;
}

// per block: plane decisions, header, payload size.  meta[b] (V2_META words):
//   [0] code | param << 8 | raw_mask << 16 | b1_mask << 24, [1] k of the 8 planes (4 bits
//   each), [2] header bytes, [3..10] plane chunk bytes
__global__ void k_v2_size(Geom geo, const u32* sel, const u64* rbits, const u32* b1, u32* meta, u32* size) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= geo.nb) return;
    const u32 n = geo.end(b) - geo.base(b);
    const u32 s = sel[b], param = s >> 8;
    const u32 plen = param == 0 ? 0 : param <= 0xFF ? 1 : param <= 0xFFFF ? 2 : param <= 0xFFFFFF ? 3 : 4;
    const u32 raw = (n + 7) / 8;
    u32 raw_mask = 0, b1_mask = 0, ks = 0, nenc = 0, tot = 0;
    u32* m = meta + (u64)b * V2_META;
    for (u32 j = 0; j < 8; ++j) {
        const u32 q = 8 * b + j;
        u32 bk = 0;
        u64 bb = ~0ull;
        for (u32 k = 0; k < 16; ++k) {
            const u64 by = (rbits[(u64)q * 16 + k] + 7) / 8;
            if (by < bb) {
                bb = by;
                bk = k;
            }
        }
        u32 chunk;
        if ((u64)raw <= bb + 1) {
            raw_mask |= 1u << j;
            chunk = raw;
        } else {
            if (b1[q] & 1) b1_mask |= 1u << j;
            ks |= bk << (4 * j);
            ++nenc;
            chunk = (u32)bb;
        }
        m[3 + j] = chunk;
        tot += chunk;
    }
    const u32 hdr = 1 + plen + 2 + nenc;
    m[0] = (s & 0xFF) | ((param & 0xFF) << 8) | (raw_mask << 16) | (b1_mask << 24);
    m[1] = ks;
    m[2] = hdr;
    size[b] = n ? hdr + tot : 0;
}

__global__ void k_v2_emit_header(Geom geo, const u32* meta, const u32* method, const u64* off, u8* arena,
                                 int force_all) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= geo.nb || (!force_all && method[b] != 10u) || geo.end(b) == geo.base(b)) return;
    const u32* m = meta + (u64)b * V2_META;
    const u32 code = m[0] & 0xFF, param = (m[0] >> 8) & 0xFF, raw_mask = (m[0] >> 16) & 0xFF;
    const u32 b1_mask = m[0] >> 24, plen = param ? 1u : 0u;
    u8* o = arena + off[b];
    u32 k = 0;
    o[k++] = (u8)((code << 5) | plen);
    if (plen) o[k++] = (u8)param;
    o[k++] = (u8)raw_mask;
    o[k++] = (u8)b1_mask;
    for (u32 j = 0; j < 8; ++j)
        if (!((raw_mask >> j) & 1)) o[k++] = (u8)((m[1] >> (4 * j)) & 0xF);
}

__device__ inline u64 v2_chunk_off(const u32* m, u32 j) {
    u64 o = m[2];
    for (u32 i = 0; i < j; ++i) o += m[3 + i];
    return o;
}

// raw planes: one thread per output byte (PY:1191-1195, MSB first); tpq tiles per plane block
__global__ __launch_bounds__(256) void k_v2_emit_raw(Geom geo, const u32* meta, const u32* method, const u64* off,
                                                     const u8* U, u8* arena, int force_all, u32 tpq) {
    const u32 q = blockIdx.x / tpq, b = q >> 3, j = q & 7;
    if (!force_all && method[b] != 10u) return;
    const u32* m = meta + (u64)b * V2_META;
    if (!((m[0] >> 16) >> j & 1)) return;
    const u32 base = geo.base(b), n = geo.end(b) - base;
    const u32 t = (blockIdx.x - q * tpq) * 256 + threadIdx.x;
    if (t >= (n + 7) / 8) return;
    const u8* u = U + 8ull * base + (u64)j * n;
    u32 v = 0;
#pragma unroll
    for (u32 i = 0; i < 8; ++i) v |= (8 * t + i < n ? (u32)(u[8 * t + i] & 1) : 0u) << (7 - i);
    arena[off[b] + v2_chunk_off(m, j) + t] = (u8)v;
}

// set bits [g, g + cnt) of the MSB-first bit string at byte address base (zeroed beforehand)
__device__ inline void set_bits(u8* base, u64 g, u32 cnt) {
    while (cnt) {
        const uintptr_t a = (uintptr_t)(base + (g >> 3));
        u32* word = reinterpret_cast<u32*>(a & ~(uintptr_t)3);
        // bits of this byte: MSB-first inside the byte, bytes little-endian inside the word
        const u32 bit = (u32)(g & 7), take = min(cnt, 8 - bit);
        const u32 byte_mask = ((0xFFu >> bit) & ~(0xFFu >> (bit + take))) & 0xFF;
        atomicOr(word, byte_mask << (8 * (a & 3)));
        g += take;
        cnt -= take;
    }
}

// encoded planes (one workgroup per plane block): run code lengths (q + 1 + k) -> bit
// offsets by a workgroup scan over the runs in order (+ carry), then unary + k bits
__global__ __launch_bounds__(RWG) void k_v2_emit_rice(Geom geo, const u32* pb, const u32* meta, const u32* method,
                                                      const u64* off, const u8* L, u8* arena, int force_all) {
    __shared__ u32 sh[RWG / 64];
    __shared__ u64 sh64[RWG / 64];
    __shared__ u32 carry;
    __shared__ u64 bcarry;
    const u32 q = blockIdx.x, b = q >> 3, j = q & 7;
    if (!force_all && method[b] != 10u) return;
    const u32* m = meta + (u64)b * V2_META;
    if ((m[0] >> 16) >> j & 1) return;  // raw plane
    const u32 k = (m[1] >> (4 * j)) & 0xF;
    const u32 s = pb[q], n = pb[q + 1] - s;
    u8* dst = arena + off[b] + v2_chunk_off(m, j);
    const u32 t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) bcarry = 0;
    // pass over the runs in steps; every step: my runs' code lengths -> exclusive prefix
    const u8* Lq = L + s;
    if (t == 0) carry = 0;
    __syncthreads();
    for (u32 c0 = 0; c0 < n; c0 += RWG * RPER) {
        const u32 i0 = c0 + t * RPER;
        u8 v[RPER + 1];
        v[0] = (i0 >= 1 && i0 - 1 < n) ? Lq[i0 - 1] : 0;
#pragma unroll
        for (u32 e = 0; e < RPER; ++e) v[e + 1] = i0 + e < n ? Lq[i0 + e] : 0;
        u32 last = 0;
#pragma unroll
        for (u32 e = 0; e < RPER; ++e) {
            const u32 i = i0 + e;
            if (i < n && i > 0 && v[e + 1] != v[e]) last = i;
        }
        const u32 incl = wave_incl_scan(last, OpMaxU(), 0u);
        const u32 ex = KOLM_DPP(0u, incl, DPP_WAVE_SHR1, 0xF);
        if (lane == 63) sh[w] = incl;
        __syncthreads();
        u32 prev = max(carry, ex);
        for (u32 i = 0; i < w; ++i) prev = max(prev, sh[i]);
        u32 top = carry;
        for (u32 i = 0; i < RWG / 64; ++i) top = max(top, sh[i]);
        // my runs (those ending at my run starts) and their total code length
        u32 rl[RPER];
        u64 mybits = 0;
        {
            u32 pv = prev;
#pragma unroll
            for (u32 e = 0; e < RPER; ++e) {
                const u32 i = i0 + e;
                rl[e] = 0;
                if (i < n && i > 0 && v[e + 1] != v[e]) {
                    rl[e] = i - pv;
                    pv = i;
                    mybits += (u64)(rl[e] >> k) + 1 + k;
                }
            }
        }
        // exclusive scan of mybits over the workgroup (u64)
        u64 x = mybits;
        for (int o = 1; o < 64; o <<= 1) {
            const u64 y = __shfl_up(x, o);
            if (lane >= (u32)o) x += y;
        }
        __syncthreads();
        if (lane == 63) sh64[w] = x;
        __syncthreads();
        u64 g = bcarry + x - mybits;
        for (u32 i = 0; i < w; ++i) g += sh64[i];
        u64 stepbits = 0;
        for (u32 i = 0; i < RWG / 64; ++i) stepbits += sh64[i];
#pragma unroll
        for (u32 e = 0; e < RPER; ++e) {
            if (!rl[e]) continue;
            const u32 r = rl[e], qv = r >> k;
            set_bits(dst, g, qv);  // unary q ones, then the 0 (already zero)
            g += qv + 1;
            for (u32 i = 0; i < k; ++i)
                if ((r >> (k - 1 - i)) & 1) set_bits(dst, g + i, 1);
            g += k;
        }
        __syncthreads();
        if (t == 0) {
            carry = top;
            bcarry += stepbits;
        }
        __syncthreads();
    }
    if (t == 0 && n) {  // the last run
        const u32 r = n - carry, qv = r >> k;
        u64 g = bcarry;
        set_bits(dst, g, qv);
        g += qv + 1;
        for (u32 i = 0; i < k; ++i)
            if ((r >> (k - 1 - i)) & 1) set_bits(dst, g + i, 1);
    }
}

}  // namespace

void launch_v2_sizes(const Geom& geo, const u8* text, u32* hist, u32* sel, u8* U, hipStream_t s, KTimer* kt) {
    if (!geo.nb) return;
    KOLM_HIP_CHECK(hipMemsetAsync(hist, 0, sizeof(u32) * V2C * 256 * geo.nb, s));
    const u32 tpb = (geo.bs + V2T - 1) / V2T;
    {
        KScope k(kt, KT_SIZES, "k_v2_hist", geo.N * 5);
        k_v2_hist<<<geo.nb * tpb, 256, 0, s>>>(geo, text, tpb, hist);
    }
    {
        KScope k(kt, KT_SIZES, "k_v2_select", (u64)geo.nb * V2C * 1024);
        k_v2_select<<<geo.nb, 256, 0, s>>>(geo, hist, sel);
    }
    {
        KScope k(kt, KT_SIZES, "k_v2_planes", geo.N * 13);
        k_v2_planes<<<(u32)((geo.N + 255) / 256), 256, 0, s>>>(geo, text, sel, U);
    }
}

void launch_v2_runs(u32 nplanes, const u32* d_pb, const u8* L, u64* rbits, u32* b1, hipStream_t s, KTimer* kt,
                    u64 bytes) {
    if (!nplanes) return;
    KScope k(kt, KT_SIZES, "k_v2_runs", bytes);
    k_v2_runs<<<nplanes, RWG, 0, s>>>(d_pb, L, rbits, b1);
}

void launch_v2_size(const Geom& geo, const u32* sel, const u64* rbits, const u32* b1, u32* meta, u32* size,
                    hipStream_t s) {
    if (geo.nb) k_v2_size<<<(geo.nb + 255) / 256, 256, 0, s>>>(geo, sel, rbits, b1, meta, size);
}

void launch_v2_emit(const Geom& geo, const u32* d_pb, const u32* meta, const u32* method, const u64* off,
                    const u8* U, const u8* L, u8* arena, hipStream_t s) {
    if (!geo.nb) return;
    const int all = method == nullptr ? 1 : 0;
    k_v2_emit_header<<<(geo.nb + 255) / 256, 256, 0, s>>>(geo, meta, method, off, arena, all);
    const u32 tpq = (geo.bs + 8 * 256 - 1) / (8 * 256);
    k_v2_emit_raw<<<8 * geo.nb * tpq, 256, 0, s>>>(geo, meta, method, off, U, arena, all, tpq);
    k_v2_emit_rice<<<8 * geo.nb, RWG, 0, s>>>(geo, d_pb, meta, method, off, L, arena, all);
}

}  // namespace kolm
