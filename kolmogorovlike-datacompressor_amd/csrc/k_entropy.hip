// Candidate sizes, MDL argmin and payload emission for the simple / entropy models.
//
//   * raw  (PY:2098)         size n
//   * xor  (PY:2105-2111)    ULEB((b - prev) & 0xFF): size n + #{delta >= 128}
//   * lfsr (PY:1984-2003)    ULEB((b - s_i) & 0xFF), s_i = LFSR^i(1), taps 0x96, period 255
//   * bbwt family (PY:2028-2073, candidates 2..6 = flags 0, 1, 4, 8, 16): Rice k=2 of the
//     MTF of the BBWT, optionally after bit-plane interleave (8-byte groups, zero padded,
//     PY:1100-1120), nibble swap, bit reverse or Gray code (PY:1650-1662).
// The 5 Rice sizes are counted by the MTF replay as it produces the indices (k_mtf.hip),
// xor / lfsr from one text pass on the index stream; only the MDL winner (PY:2350-2369: smallest payload, ties -> lowest id) is emitted.
// Rice emission is a two-pass scan: per-tile bit counts -> per-block exclusive scan over
// tiles -> each thread writes its symbols' bits (MSB-first, PY:1231-1254) into an LDS
// big-endian word buffer, flushed with plain stores (interior words) and atomicOr
// (the two edge words shared with neighbouring tiles).
#include "kolm_internal.h"

namespace kolm {

__constant__ u8 c_lfsr[256];

namespace {

struct TileG {
    Geom geo;
    u32 tpb;
    __device__ inline bool range(u32 t, u32& lo, u32& hi, u32& b) const {
        b = t / tpb;
        const u32 k = t - b * tpb;
        lo = geo.base(b) + k * TILE;
        const u32 e = geo.end(b);
        hi = min(lo + (u32)TILE, e);
        return lo < e;
    }
};

__device__ inline u32 bitrev8(u32 v) { return __brev(v) >> 24; }

__device__ inline u32 variant_sym(u32 v, int flag) {
    switch (flag) {
        case 4: return ((v & 0x0F) << 4) | ((v & 0xF0) >> 4);
        case 8: return bitrev8(v);
        case 16: return v ^ (v >> 1);
        default: return v;
    }
}

// transpose an 8-byte group: out byte `bit` collects bit (7-bit) of every input byte
__device__ inline void bitplane8(const u32 (&in)[8], u32 (&out)[8]) {
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        u32 v = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) v |= ((in[i] >> (7 - bit)) & 1u) << (7 - i);
        out[bit] = v;
    }
}

__device__ inline u32 rice_bits(u32 v, int k) { return (v >> k) + 1 + k; }

template <class T>
__device__ inline T wg_sum(T v, T* sh) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    T r = 0;
    for (int i = 0; i < (int)(blockDim.x / 64); ++i) r += sh[i];
    __syncthreads();
    return r;
}

__device__ inline u32 wg_excl_add(u32 v, u32* sh) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 incl = v;
    for (u32 o = 1; o < 64; o <<= 1) {
        const u32 t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 carry = 0;
    for (u32 i = 0; i < w; ++i) carry += sh[i];
    __syncthreads();
    return carry + incl - v;
}

// counters per block in `bits`: 0 b0, 1 bp, 2 nib, 3 br, 4 gray (added by the MTF replay,
// k_mtf.hip), 5 xor extra, 6 lfsr extra (k_cheap_sizes)
// xor / lfsr_pred counters only (5, 6): 16 text bytes per thread (one 16-byte load when
// aligned), LFSR table in LDS (per-lane indices would serialise on the constant cache)
constexpr u32 CHEAP_T = 4096;  // bytes per workgroup
__global__ __launch_bounds__(WG) void k_cheap_sizes(Geom geo, u32 tpb, const u8* text, u64* bits) {
    __shared__ u64 sh[WG / 64];
    __shared__ u8 lf[256];
    lf[threadIdx.x] = c_lfsr[threadIdx.x];
    __syncthreads();
    const u32 b = blockIdx.x / tpb, k = blockIdx.x - b * tpb;
    const u32 base = geo.base(b), e = geo.end(b);
    const u32 g0 = base + k * CHEAP_T + threadIdx.x * 16;
    u32 c5 = 0, c6 = 0;
    if (g0 < e) {
        u32 t[16];
        const u32 m = min(16u, e - g0);
        if (m == 16 && ((uintptr_t)(text + g0) & 15) == 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(text + g0);
            const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = (w[q >> 2] >> (8 * (q & 3))) & 0xFFu;
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = (u32)q < m ? text[g0 + q] : 0u;
        }
        u32 prev = (g0 == base) ? 0u : (u32)text[g0 - 1];
        u32 ph = (g0 - base) % 255u;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if ((u32)q < m) {
                c5 += ((t[q] - prev) & 0xFFu) >= 128u;
                c6 += ((t[q] - (u32)lf[ph]) & 0xFFu) >= 128u;
                prev = t[q];
                ph = ph == 254u ? 0u : ph + 1;
            }
        }
    }
    const u64 t5 = wg_sum<u64>(c5, sh), t6 = wg_sum<u64>(c6, sh);
    if (threadIdx.x == 0) {
        if (t5) atomicAdd((unsigned long long*)&bits[(u64)b * 8 + 5], (unsigned long long)t5);
        if (t6) atomicAdd((unsigned long long*)&bits[(u64)b * 8 + 6], (unsigned long long)t6);
    }
}

__global__ void k_mdl(Geom geo, const u64* bits, const u32* lz_size, const u32* rp_result, const u32* v2_size,
                      u32* sizes, u32* method, const int32_t* force, u32 mask, u64* wsize) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= geo.nb) return;
    const u32 n = geo.end(b) - geo.base(b);
    const u64* c = bits + (u64)b * 8;
    u64 sz[NCAND];
    sz[0] = n;
    sz[1] = n + c[5];
    sz[2] = (c[0] + 7) / 8;
    sz[3] = (c[1] + 7) / 8;
    sz[4] = (c[2] + 7) / 8;
    sz[5] = (c[3] + 7) / 8;
    sz[6] = (c[4] + 7) / 8;
    sz[7] = lz_size ? lz_size[b] : 0xFFFFFFFFull;
    sz[8] = n + c[6];
    sz[9] = rp_result ? rp_result[(u64)b * RP_RS_N + RP_RS_SIZE] : 0xFFFFFFFFull;
    sz[10] = v2_size ? v2_size[b] : 0xFFFFFFFFull;
    u32 best = 0;
    u64 bsz = ~0ull;
    for (u32 m = 0; m < NCAND; ++m) {
        const bool en = (mask >> m) & 1u;
        sizes[(u64)b * NCAND + m] = en ? (u32)sz[m] : 0xFFFFFFFFu;
        if (en && sz[m] < bsz) {
            bsz = sz[m];
            best = m;
        }
    }
    if (bsz == ~0ull) best = 0;  // PY:2362-2364 all candidates failed -> raw
    if (force && force[b] >= 0) best = (u32)force[b];
    method[b] = best;
    wsize[b] = sz[best];
}

// exclusive scan of per-block winner sizes -> payload offsets (single workgroup)
__global__ __launch_bounds__(WG) void k_offsets(const u64* wsize, u32 nb, u64* off, u64 cap, u32* status) {
    __shared__ u64 sh[WG / 64];
    __shared__ u64 carry_s;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (u32 c0 = 0; c0 < nb; c0 += WG) {
        const u32 b = c0 + threadIdx.x;
        const u64 v = b < nb ? wsize[b] : 0;
        const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        u64 incl = v;
        for (u32 o = 1; o < 64; o <<= 1) {
            const u64 t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        if (lane == 63) sh[w] = incl;
        __syncthreads();
        u64 pre = carry_s;
        for (u32 i = 0; i < w; ++i) pre += sh[i];
        if (b < nb) off[b] = pre + incl - v;
        __syncthreads();
        if (threadIdx.x == WG - 1) carry_s = pre + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        off[nb] = carry_s;
        if (carry_s > cap) *status = 1;
    }
}

// ---------------- simple models: raw copy, xor / lfsr ULEB streams ----------------
__device__ inline u32 simple_delta(int m, const u8* text, u32 i, u32 base) {
    const u32 bt = text[i];
    if (m == 1) return (bt - (i == base ? 0u : (u32)text[i - 1])) & 0xFFu;
    return (bt - (u32)c_lfsr[(i - base) % 255u]) & 0xFFu;
}

// per-tile byte counts of the chosen simple stream (xor/lfsr) -> tsum
__global__ __launch_bounds__(WG) void k_simple_count(TileG tg, const u8* text, const u32* method, u32* tsum) {
    __shared__ u32 sh[WG / 64];
    u32 lo, hi, b;
    const bool ok = tg.range(blockIdx.x, lo, hi, b);
    const int m = ok ? (int)method[b] : -1;
    u32 cnt = 0;
    if (m == 1 || m == 8) {
        const u32 base = tg.geo.base(b);
        for (u32 i = lo + threadIdx.x; i < hi; i += WG) cnt += 1 + (simple_delta(m, text, i, base) >= 128u);
    }
    cnt = wg_sum<u32>(cnt, sh);
    if (threadIdx.x == 0) tsum[blockIdx.x] = cnt;
}

__global__ __launch_bounds__(WG) void k_tiles_excl_add(const u32* in, u32* out, u32 tpb) {
    __shared__ u32 sh[WG / 64];
    __shared__ u32 edge;
    const u32 b = blockIdx.x;
    u32 carry = 0;
    for (u32 c0 = 0; c0 < tpb; c0 += WG) {
        const u32 k = c0 + threadIdx.x;
        const u32 v = k < tpb ? in[(u64)b * tpb + k] : 0;
        const u32 ex = wg_excl_add(v, sh);
        if (k < tpb) out[(u64)b * tpb + k] = carry + ex;
        if (threadIdx.x == WG - 1) edge = ex + v;
        __syncthreads();
        carry += edge;
        __syncthreads();
    }
}

__global__ __launch_bounds__(WG) void k_emit_simple(TileG tg, const u8* text, const u32* method,
                                                    const u64* off, const u32* toff, u8* arena) {
    __shared__ u32 sh[WG / 64];
    u32 lo, hi, b;
    if (!tg.range(blockIdx.x, lo, hi, b)) return;
    const int m = (int)method[b];
    if (m != 0 && m != 1 && m != 8) return;
    const u32 base = tg.geo.base(b);
    u8* dst = arena + off[b];
    if (m == 0) {
        for (u32 i = lo + threadIdx.x; i < hi; i += WG) dst[i - base] = text[i];
        return;
    }
    // thread handles PER_THREAD consecutive bytes
    const u32 i0 = lo + threadIdx.x * PER_THREAD;
    u32 d[PER_THREAD];
    u32 cnt = 0;
#pragma unroll
    for (int e = 0; e < PER_THREAD; ++e) {
        d[e] = (i0 + e < hi) ? simple_delta(m, text, i0 + e, base) : 0;
        cnt += (i0 + e < hi) ? 1 + (d[e] >= 128u) : 0;
    }
    u32 o = toff[blockIdx.x] + wg_excl_add(cnt, sh);
#pragma unroll
    for (int e = 0; e < PER_THREAD; ++e) {
        if (i0 + e >= hi) break;
        if (d[e] < 128u) {
            dst[o++] = (u8)d[e];
        } else {
            dst[o++] = (u8)((d[e] & 0x7F) | 0x80);
            dst[o++] = (u8)(d[e] >> 7);
        }
    }
}

// ---------------- Rice emission ----------------
// flag per block (-1 = not a Rice block): from method 2..6 -> {0, 1, 4, 8, 16}
__device__ inline int rice_flag_of(u32 m) {
    switch (m) {
        case 2: return 0;
        case 3: return 1;
        case 4: return 4;
        case 5: return 8;
        case 6: return 16;
        default: return -1;
    }
}

// symbols of thread's 8-group for the variant; returns count
__device__ inline int group_syms(const u8* seq, u32 g0, u32 hi, int flag, u32 (&sym)[8]) {
    u32 v[8];
    int nvalid = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const bool ok = g0 + e < hi;
        v[e] = ok ? seq[g0 + e] : 0;
        nvalid += ok;
    }
    if (!nvalid) return 0;
    if (flag == 1) {
        bitplane8(v, sym);
        return 8;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sym[e] = variant_sym(v[e], flag);
    return nvalid;
}

__global__ __launch_bounds__(WG) void k_rice_count(TileG tg, const u8* seq, const u32* method, int force_flag,
                                                   int k, u32* tsum) {
    __shared__ u32 sh[WG / 64];
    u32 lo, hi, b;
    const bool ok = tg.range(blockIdx.x, lo, hi, b);
    const int flag = !ok ? -1 : (method == nullptr ? force_flag : rice_flag_of(method[b]));
    u32 cnt = 0;
    if (flag >= 0) {
        u32 sym[8];
        const int ns = group_syms(seq, lo + threadIdx.x * 8, hi, flag, sym);
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (e < ns) cnt += rice_bits(sym[e], k);
    }
    cnt = wg_sum<u32>(cnt, sh);
    if (threadIdx.x == 0) tsum[blockIdx.x] = cnt;
}

__device__ inline void put_bits(u32* buf, u32 pos, u32 v, u32 len) {
    // BE-word bit writer: bit `pos` is bit (31 - pos%32) of word pos/32
    if (!len) return;
    const u32 w = pos >> 5, o = pos & 31;
    if (o + len <= 32) {
        atomicOr(&buf[w], v << (32 - o - len));
    } else {
        const u32 l1 = 32 - o, l2 = len - l1;
        atomicOr(&buf[w], v >> l2);
        atomicOr(&buf[w + 1], v << (32 - l2));
    }
}

__global__ __launch_bounds__(WG) void k_rice_emit(TileG tg, const u8* seq, const u32* method, int force_flag,
                                                  int k, const u64* off, const u32* toff, u8* arena,
                                                  u32 lds_words) {
    extern __shared__ __attribute__((aligned(16))) u32 lds[];
    __shared__ u32 sh[WG / 64];
    u32 lo, hi, b;
    if (!tg.range(blockIdx.x, lo, hi, b)) return;
    const int flag = method == nullptr ? force_flag : rice_flag_of(method[b]);
    if (flag < 0) return;
    u32 sym[8];
    const int ns = group_syms(seq, lo + threadIdx.x * 8, hi, flag, sym);
    u32 cnt = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        if (e < ns) cnt += rice_bits(sym[e], k);
    const u32 my = wg_excl_add(cnt, sh);
    const u64 gstart = off[b] * 8 + toff[blockIdx.x];  // tile start bit (global)
    const u32 lead = (u32)(gstart & 31);               // bit offset inside first word
    const u64 w0 = gstart >> 5;
    // total bits of the tile; only the words the tile's code reaches are cleared (a few hundred
    // of the lds_words sized for the worst case)
    __shared__ u32 tot;
    if (threadIdx.x == WG - 1) tot = my + cnt;
    __syncthreads();
    const u32 nclr = min(lds_words, ((lead + tot + 31) >> 5) + 3);
    for (u32 i = threadIdx.x; i < nclr; i += WG) lds[i] = 0;
    __syncthreads();
    u32 pos = lead + my;
    if (cnt <= 64) {
        // the thread's whole code (usually a few dozen bits) assembled in one register and
        // OR-ed into at most three LDS words, instead of one atomic per symbol
        u64 acc = 0;
        for (int e = 0; e < ns; ++e) {
            const u32 s = sym[e], q = s >> k, len = q + 1 + k;  // q < 64 here
            const u64 code = (((q ? ~0ull >> (64 - q) : 0ull)) << (1 + k)) | (s & ((1u << k) - 1));
            acc = len >= 64 ? code : (acc << len) | code;
        }
        if (cnt) {
            const u64 v = acc << (64 - cnt);  // left-aligned
            const u32 w = pos >> 5, o = pos & 31, h32 = (u32)(v >> 32), l32 = (u32)v;
            const u32 x0 = h32 >> o, x1 = (o ? h32 << (32 - o) : 0u) | (l32 >> o), x2 = o ? l32 << (32 - o) : 0u;
            if (x0) atomicOr(&lds[w], x0);
            if (x1) atomicOr(&lds[w + 1], x1);
            if (x2) atomicOr(&lds[w + 2], x2);
        }
        pos += cnt;
    } else
    for (int e = 0; e < ns; ++e) {
        const u32 s = sym[e];
        u32 q = s >> k;
        const u32 r = s & ((1u << k) - 1);
        // unary: q ones then a zero, then k bits of r
        while (q >= 32) {
            put_bits(lds, pos, 0xFFFFFFFFu, 32);
            pos += 32;
            q -= 32;
        }
        if (q + 1 + k <= 32) {
            const u32 val = (((1u << q) - 1u) << (1 + k)) | r;
            put_bits(lds, pos, val, q + 1 + k);
            pos += q + 1 + k;
        } else {
            put_bits(lds, pos, (1u << q) - 1u, q);
            pos += q;
            put_bits(lds, pos, r, 1 + k);
            pos += 1 + k;
        }
    }
    __syncthreads();
    const u32 nwords = (lead + tot + 31) >> 5;
    u32* a32 = reinterpret_cast<u32*>(arena);
    for (u32 i = threadIdx.x; i < nwords; i += WG) {
        const u32 v = __builtin_bswap32(lds[i]);
        if (i == 0 || i == nwords - 1) {
            if (v) atomicOr(&a32[w0 + i], v);
        } else {
            a32[w0 + i] = v;
        }
    }
}

}  // namespace

static inline u32 cdiv32(u64 a, u64 b) { return (u32)((a + b - 1) / b); }

static void lfsr_init_once() {
    static bool done[64] = {};
    int dev = 0;
    KOLM_HIP_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64 || done[dev]) return;
    u8 tab[256];
    u32 s = 1;
    for (int i = 0; i < 256; ++i) {
        tab[i] = (u8)s;
        u32 fb = 0;
        for (int bit = 0; bit < 8; ++bit)
            if ((0x96 >> bit) & 1) fb ^= (s >> bit) & 1;
        s = ((s << 1) & 0xFF) | fb;
    }
    KOLM_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_lfsr), tab, 256));
    done[dev] = true;
}

void launch_cheap_sizes(const EmitArgs& e, hipStream_t s) {
    lfsr_init_once();
    if (!e.geo.N) return;
    const u32 tpb = cdiv32(e.geo.bs, CHEAP_T);
    k_cheap_sizes<<<tpb * e.geo.nb, WG, 0, s>>>(e.geo, tpb, e.text, e.bits);
}

void launch_mdl(const EmitArgs& e, const u32* lz_sizes, const u32* rp_result, const u32* v2_size, u32* status,
                hipStream_t s) {
    if (!e.geo.nb) return;
    u64* wsize = reinterpret_cast<u64*>(e.tile_tmp2);  // nb u64 scratch
    k_mdl<<<cdiv32(e.geo.nb, 256), 256, 0, s>>>(e.geo, e.bits, lz_sizes, rp_result, v2_size, e.sizes, e.method, e.force,
                                                e.cand_mask, wsize);
    k_offsets<<<1, WG, 0, s>>>(wsize, e.geo.nb, e.off, e.arena_cap, status);
}

void launch_emit_simple(const EmitArgs& e, hipStream_t s) {
    lfsr_init_once();
    if (!e.geo.N) return;
    TileG tg{e.geo, cdiv32(e.geo.bs, TILE)};
    const u32 nt = tg.tpb * e.geo.nb;
    k_simple_count<<<nt, WG, 0, s>>>(tg, e.text, e.method, e.tile_tmp);
    k_tiles_excl_add<<<e.geo.nb, WG, 0, s>>>(e.tile_tmp, e.tile_tmp + nt, tg.tpb);
    k_emit_simple<<<nt, WG, 0, s>>>(tg, e.text, e.method, e.off, e.tile_tmp + nt, e.arena);
}

static void rice_emit_common(const Geom& geo, const u8* seq, const u32* method, int force_flag, int k,
                             const u64* off, u8* arena, u32* tile_tmp, hipStream_t s) {
    TileG tg{geo, cdiv32(geo.bs, TILE)};
    const u32 nt = tg.tpb * geo.nb;
    k_rice_count<<<nt, WG, 0, s>>>(tg, seq, method, force_flag, k, tile_tmp);
    k_tiles_excl_add<<<geo.nb, WG, 0, s>>>(tile_tmp, tile_tmp + nt, tg.tpb);
    const u32 maxbits = TILE * ((255u >> k) + 1 + k) + 64;
    const u32 words = (maxbits + 31) / 32 + 2;
    if (words * 4 > 65536)
        KOLM_HIP_CHECK(hipFuncSetAttribute((const void*)k_rice_emit, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(words * 4)));
    k_rice_emit<<<nt, WG, words * 4, s>>>(tg, seq, method, force_flag, k, off, tile_tmp + nt, arena, words);
}

void launch_emit_rice(const EmitArgs& e, hipStream_t s) {
    if (!e.geo.N) return;
    rice_emit_common(e.geo, e.mtf, e.method, -1, e.rice_k, e.off, e.arena, e.tile_tmp, s);
}

// Rice of a plain byte sequence (kolm_rice_encode): one block, flag 0.  out must be zeroed;
// *out_size receives the byte size.
__global__ void k_rice_total(const u32* toff, const u32* tsum, u32 nt, u32* out_size) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const u64 bits = (u64)toff[nt - 1] + tsum[nt - 1];
        *out_size = (u32)((bits + 7) / 8);
    }
}

void launch_rice_only(const Geom& geo, const u8* in, int k, u8* out, u32* tile_tmp, u32* tile_tmp2,
                      u32* out_size, hipStream_t s) {
    if (!geo.N) return;
    // offsets: single block at byte 0 (tile_tmp2 holds a zero u64)
    KOLM_HIP_CHECK(hipMemsetAsync(tile_tmp2, 0, sizeof(u64), s));
    rice_emit_common(geo, in, nullptr, 0, k, reinterpret_cast<const u64*>(tile_tmp2), out, tile_tmp, s);
    TileG tg{geo, cdiv32(geo.bs, TILE)};
    const u32 nt = tg.tpb * geo.nb;
    k_rice_total<<<1, 64, 0, s>>>(tile_tmp + nt, tile_tmp, nt, out_size);
}

}  // namespace kolm
