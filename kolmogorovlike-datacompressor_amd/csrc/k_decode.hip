// Block decoders on gfx950 (decode side of the candidate registry, PY:2194-2207): every
// block is independent, so a batch decodes one workgroup per block; inside a block the
// reference's sequential loops are restated in parallel form:
//   raw  (PY:2101)        copy.
//   xor  (PY:2113-2122)   ULEB values < 256 (1 or 2 bytes): a byte starts a value iff the
//   lfsr (PY:2005-2019)   previous byte is < 128 -> start flags + workgroup scan give each
//                         value's index; xor = running sum mod 256 (scan), lfsr = value +
//                         LFSR state of the position (PY:1984-2003 table, taps 0x96, seed 1).
//   lz77 (PY:1765-1812)   one thread per block parses the token stream (byte-aligned, the
//                         only sequential part) into token records; the workgroup then
//                         labels every output position with its token (max-scan of token
//                         starts), sets src[o] = literal byte | LIT or o - dist, and resolves
//                         copy chains (overlapping ones included) by pointer jumping:
//                         src[o] <- src[src[o]] until every position names a literal.
// Errors (malformed payloads: lengths, distances, flags) set a per-block status word and
// never read or write outside the block's payload / output range.
#include "kolm_internal.h"

namespace kolm {

namespace {

constexpr u32 LIT = 0x80000000u;  // src[o] of a literal: LIT | byte

__device__ inline u32 wg_excl_sum(u32 v, u32* sh, u32* total) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u32 incl = wave_incl_scan(v, OpAddU(), 0u);
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    u32 pre = 0, tot = 0;
    for (u32 i = 0; i < blockDim.x / 64; ++i) {
        const u32 x = sh[i];
        pre += i < w ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return pre + incl - v;
}

// ---------------------------------------------------------------- raw
__global__ __launch_bounds__(256) void k_dec_raw(DecArgs a) {
    const u32 b = a.list[blockIdx.x];
    const u64 p0 = a.poff[b], plen = a.poff[b + 1] - p0;
    const u32 o0 = a.obase[b], n = a.obase[b + 1] - o0;
    if (plen != n) {
        if (threadIdx.x == 0) a.status[b] = DEC_ELEN;
        return;
    }
    for (u32 i = threadIdx.x; i < n; i += 256) a.out[o0 + i] = a.pay[p0 + i];
}

// ---------------------------------------------------------------- xor / lfsr
// 8 payload bytes per thread per step, 2048 per workgroup step, carries across steps.
template <bool LFSR>
__global__ __launch_bounds__(256) void k_dec_uleb(DecArgs a) {
    __shared__ u32 sh[4];
    __shared__ u8 lfsr[256];
    const u32 b = a.list[blockIdx.x], tid = threadIdx.x;
    const u64 p0 = a.poff[b];
    const u32 plen = (u32)(a.poff[b + 1] - p0);
    const u32 o0 = a.obase[b], n = a.obase[b + 1] - o0;
    const u8* pay = a.pay + p0;
    if (LFSR && tid == 0) {  // PY:1984-2003 state sequence, period 255
        u32 s = 1;
        for (u32 i = 0; i < 255; ++i) {
            lfsr[i] = (u8)s;
            const u32 fb = __popc(s & 0x96u) & 1u;
            s = ((s << 1) & 0xFFu) | fb;
        }
    }
    __syncthreads();
    u32 vcount = 0;  // values before this step
    u32 run = 0;     // xor: running sum (mod 256) before this step
    bool bad = false;
    for (u32 s0 = 0; s0 < plen; s0 += 2048) {
        const u32 j0 = s0 + tid * 8;
        u32 v[8];
        u32 nv = 0, sum = 0;
#pragma unroll
        for (u32 e = 0; e < 8; ++e) {
            const u32 j = j0 + e;
            v[e] = 0xFFFFFFFFu;
            if (j < plen && (j == 0 || pay[j - 1] < 128)) {
                u32 x = pay[j] & 0x7Fu;
                if (pay[j] & 0x80u) {
                    if (j + 1 >= plen || pay[j + 1] >= 2) bad = true;  // values are < 256
                    else x |= (u32)pay[j + 1] << 7;
                }
                v[e] = x;
                ++nv;
                sum += x;
            }
        }
        u32 tot_v = 0, tot_s = 0;
        const u32 vi0 = vcount + wg_excl_sum(nv, sh, &tot_v);
        const u32 sp = run + wg_excl_sum(sum, sh, &tot_s);
        u32 vi = vi0, acc = sp;
#pragma unroll
        for (u32 e = 0; e < 8; ++e) {
            if (v[e] == 0xFFFFFFFFu) continue;
            if (vi < n) {
                if (LFSR) {
                    a.out[o0 + vi] = (u8)((v[e] + lfsr[vi % 255u]) & 0xFFu);
                } else {
                    acc += v[e];
                    a.out[o0 + vi] = (u8)(acc & 0xFFu);
                }
            }
            ++vi;
        }
        vcount += tot_v;
        run += tot_s;
    }
    if (__syncthreads_or(bad) && tid == 0) a.status[b] = DEC_EFORMAT;
    if (tid == 0 && vcount != n) a.status[b] = DEC_ELEN;
}

// ---------------------------------------------------------------- lz77
__device__ inline bool uleb_get(const u8* p, u32 plen, u32& j, u32& v) {
    v = 0;
    for (u32 sh = 0; sh < 35; sh += 7) {
        if (j >= plen) return false;
        const u32 b = p[j++];
        v |= (b & 0x7Fu) << sh;
        if (!(b & 0x80u)) return true;
    }
    return false;
}

// One thread per block: token records (output start, length, literal byte | LIT or distance)
// in the token slots [obase, obase + ntok) of the block; validation as PY:1765-1812.
__global__ __launch_bounds__(64) void k_dec_lz_parse(DecArgs a, u32* tpos, u32* tval, u32* ntok) {
    const u32 li = blockIdx.x * 64 + threadIdx.x;
    if (li >= a.nlist) return;
    const u32 b = a.list[li];
    const u64 p0 = a.poff[b];
    const u32 plen = (u32)(a.poff[b + 1] - p0);
    const u32 o0 = a.obase[b], n = a.obase[b + 1] - o0;
    const u8* p = a.pay + p0;
    u32 j = 0, o = 0, t = 0, err = DEC_OK;
    while (j < plen && o < n) {
        const u32 flag = p[j++];
        if (flag == 0) {
            if (j >= plen) {
                err = DEC_EFORMAT;
                break;
            }
            tpos[o0 + t] = o;
            tval[o0 + t] = LIT | p[j++];
            ++t;
            ++o;
        } else if (flag == 1) {
            u32 len, dist;
            if (!uleb_get(p, plen, j, len) || !uleb_get(p, plen, j, dist) || dist == 0 || dist > min(o, 4096u)) {
                err = DEC_EFORMAT;
                break;
            }
            tpos[o0 + t] = o;
            tval[o0 + t] = dist;
            ++t;
            o += min(len, n - o);  // PY truncates the last copy at orig_len
        } else {
            err = DEC_EFORMAT;
            break;
        }
    }
    if (err == DEC_OK && o != n) err = DEC_ELEN;
    ntok[b] = err == DEC_OK ? t : 0u;
    if (err != DEC_OK) a.status[b] = err;
}

// One workgroup per block: token of every output position (max-scan of starts), source
// positions, pointer jumping, bytes.  src / mark live in the block's output range of the
// two scratch arrays.
__global__ __launch_bounds__(1024) void k_dec_lz_resolve(DecArgs a, const u32* tpos, const u32* tval,
                                                         const u32* ntok, u32* mark, u32* src) {
    __shared__ u32 sh[16];
    __shared__ u32 changed;
    const u32 b = a.list[blockIdx.x], tid = threadIdx.x;
    const u32 o0 = a.obase[b], n = a.obase[b + 1] - o0;
    const u32 nt = ntok[b];
    if (a.status[b] != DEC_OK || n == 0) return;
    for (u32 o = tid; o < n; o += 1024) mark[o0 + o] = 0;
    __syncthreads();
    for (u32 t = tid; t < nt; t += 1024) mark[o0 + tpos[o0 + t]] = t + 1;
    __syncthreads();
    // contiguous position range per thread: running max of token marks, carried across threads
    const u32 per = (n + 1023) / 1024, lo = min(tid * per, n), hi = min(lo + per, n);
    u32 m = 0;
    for (u32 o = lo; o < hi; ++o) m = max(m, mark[o0 + o]);
    u32 carry;
    {
        const u32 lane = tid & 63, w = tid >> 6;
        const u32 incl = wave_incl_scan(m, OpMaxU(), 0u);
        if (lane == 63) sh[w] = incl;
        __syncthreads();
        carry = KOLM_DPP(0u, incl, DPP_WAVE_SHR1, 0xF);
        for (u32 i = 0; i < w; ++i) carry = max(carry, sh[i]);
    }
    u32 run = carry;
    for (u32 o = lo; o < hi; ++o) {
        run = max(run, mark[o0 + o]);
        const u32 v = tval[o0 + run - 1];
        src[o0 + o] = (v & LIT) ? v : o - v;  // copies read the output dist bytes back
    }
    __syncthreads();
    // pointer jumping (in place: a read sees an old or a new source, both valid ancestors)
    for (;;) {
        if (tid == 0) changed = 0;
        __syncthreads();
        u32 ch = 0;
        for (u32 o = tid; o < n; o += 1024) {
            const u32 s = src[o0 + o];
            if (!(s & LIT)) {
                src[o0 + o] = src[o0 + s];
                ch = 1;
            }
        }
        if (ch) changed = 1;
        __syncthreads();
        if (!changed) break;
        __syncthreads();
    }
    for (u32 o = tid; o < n; o += 1024) a.out[o0 + o] = (u8)src[o0 + o];
}

// ---------------------------------------------------------------- BBWT / MTF / Rice (ids 2..6)
// PY:2075-2089 decode_bbwt_mtf_rice: Rice k=2 values -> inverse bitwise map -> MTF decode
// -> inverse BBWT.
__device__ inline u32 bw_flags(u32 m) { return m == 3 ? 1u : m == 4 ? 4u : m == 5 ? 8u : m == 6 ? 16u : 0u; }

__device__ inline u32 inv_map(u32 x, u32 flags) {
    if (flags == 16) {  // gray decode (PY:1664-1669)
        x ^= x >> 1;
        x ^= x >> 2;
        x ^= x >> 4;
    } else if (flags == 8) {
        x = __brev(x) >> 24;
    } else if (flags == 4) {
        x = ((x & 0x0Fu) << 4) | (x >> 4);
    }
    return x;
}

// 64 stream bits from bit g (MSB-first bytes, zero past plen)
__device__ inline u64 bits64(const u8* p, u32 plen, u32 g) {
    const u32 B = g >> 3, s = g & 7;
    u64 w = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) w = (w << 8) | (B + i < plen ? p[B + i] : 0u);
    if (s) w = (w << s) | ((B + 8 < plen ? p[B + 8] : 0u) >> (8 - s));
    return w;
}

// Rice-k=2 phase at a word boundary: a codeword starts here (S), inside a unary run (U),
// or 2 / 1 remainder bits pending.  walk() runs one 64-bit word from a phase.
enum : u32 { RS_S = 0, RS_U = 1, RS_R2 = 2, RS_R1 = 3 };

template <class F>
__device__ inline u32 rice_walk(u64 w, u32 nvalid, u32 st, u32& starts, F&& on_start) {
    u32 pos = 0;
    while (pos < nvalid) {
        if (st == RS_R2) {
            ++pos;
            st = RS_R1;
            continue;
        }
        if (st == RS_R1) {
            ++pos;
            st = RS_S;
            continue;
        }
        if (st == RS_S) {
            on_start(pos);
            ++starts;
        }
        const u32 z = (u32)__clzll((long long)~(w << pos));  // ones from pos (<= 64 - pos)
        if (pos + z >= nvalid) {
            pos = nvalid;
            st = RS_U;
        } else {
            pos += z + 1;
            st = RS_R2;
        }
    }
    return st;
}

// 64 stream bits from bit g: two aligned 8-byte loads inside the payload (bytes near its
// end one at a time, zero past plen)
__device__ inline u64 bits64f(const u8* p, u32 plen, u32 g) {
    const u32 B = g >> 3, s = g & 7;
    if (B + 16 <= plen) {
        const uintptr_t ad = (uintptr_t)(p + B);
        const u64* q = reinterpret_cast<const u64*>(ad & ~(uintptr_t)7);
        const u32 sh = (u32)(ad & 7) * 8;
        const u64 lo = q[0], hi = q[1];
        const u64 be = __builtin_bswap64(sh ? (lo >> sh) | (hi << (64 - sh)) : lo);
        if (!s) return be;
        return (be << s) | ((u32)((hi >> sh) & 0xFFu) >> (8 - s));
    }
    return bits64(p, plen, g);
}

struct RiceBlk {
    u32 b, plen, nbits, nw, o0, n, flags, L, wb;
    const u8* p;
};
__device__ inline RiceBlk rice_blk(const BwArgs& a, u32 li) {
    RiceBlk k;
    k.b = a.d.list[li];
    const u64 p0 = a.d.poff[k.b];
    k.plen = (u32)(a.d.poff[k.b + 1] - p0);
    k.p = a.d.pay + p0;
    k.nbits = k.plen * 8;
    k.nw = (k.nbits + 63) / 64;
    k.o0 = a.d.obase[k.b];
    k.n = a.d.obase[k.b + 1] - k.o0;
    k.flags = bw_flags(a.meth[k.b]);
    k.L = (k.flags & 1) ? 8 * ((k.n + 7) / 8) : k.n;
    k.wb = a.wbase[li];
    return k;
}

// Rice parse, three grid-wide steps over the 64-bit words of every payload:
// (A) each word's phase function: exit phase + codeword starts for each entry phase
__global__ __launch_bounds__(256) void k_rice_phase(BwArgs a) {
    const RiceBlk k = rice_blk(a, blockIdx.y);
    const u32 wi = blockIdx.x * 256 + threadIdx.x;
    if (wi >= k.nw) return;
    const u64 w = bits64f(k.p, k.plen, wi * 64);
    const u32 nv = min(64u, k.nbits - wi * 64);
    u32 f = 0;
#pragma unroll
    for (u32 e = 0; e < 4; ++e) {
        u32 cnt = 0;  // <= 22 starts per word
        const u32 ex = rice_walk(w, nv, e, cnt, [](u32) {});
        f |= (ex | (cnt << 2)) << (8 * e);
    }
    a.fw[k.wb + wi] = f;
}

// (B) per block: compose the functions over per-thread word ranges, chain the ranges,
// then every word's entry phase and first value index; too few values -> malformed
constexpr u32 DRC = 1024;
__global__ __launch_bounds__(DRC) void k_rice_chain(BwArgs a) {
    __shared__ u32 fex[DRC][4], fcnt[DRC][4], entry[DRC], sbase[DRC];
    __shared__ u32 total;
    const RiceBlk k = rice_blk(a, blockIdx.x);
    const u32 tid = threadIdx.x;
    const u32 per = (k.nw + DRC - 1) / DRC, w0 = min(tid * per, k.nw), w1 = min(w0 + per, k.nw);
    const u32* fw = a.fw + k.wb;
    u32 st[4] = {0, 1, 2, 3}, cnt[4] = {0, 0, 0, 0};
    for (u32 wi = w0; wi < w1; ++wi) {
        const u32 f = fw[wi];
#pragma unroll
        for (u32 e = 0; e < 4; ++e) {
            const u32 by = f >> (8 * st[e]);
            cnt[e] += (by >> 2) & 63u;
            st[e] = by & 3u;
        }
    }
#pragma unroll
    for (u32 e = 0; e < 4; ++e) {
        fex[tid][e] = st[e];
        fcnt[tid][e] = cnt[e];
    }
    __syncthreads();
    if (tid == 0) {
        u32 s = RS_S, base = 0;
        for (u32 t = 0; t < DRC; ++t) {
            entry[t] = s;
            sbase[t] = base;
            base += fcnt[t][s];
            s = fex[t][s];
        }
        total = base;
    }
    __syncthreads();
    if (total < k.L) {
        if (tid == 0) a.d.status[k.b] = DEC_EFORMAT;
        return;
    }
    u32 s = entry[tid], base = sbase[tid];
    for (u32 wi = w0; wi < w1; ++wi) {
        a.es[k.wb + wi] = (u8)s;
        a.vbw[k.wb + wi] = base;
        const u32 by = fw[wi] >> (8 * s);
        base += (by >> 2) & 63u;
        s = by & 3u;
    }
}

// (C) each word from its entry phase: the values of the codewords starting in it
// (index < L), inverse bitwise map, written at their index
__global__ __launch_bounds__(256) void k_rice_vals(BwArgs a) {
    const RiceBlk k = rice_blk(a, blockIdx.y);
    const u32 wi = blockIdx.x * 256 + threadIdx.x;
    if (wi >= k.nw || a.d.status[k.b] != DEC_OK) return;
    const u32 vb0 = a.vbw[k.wb + wi];
    if (vb0 >= k.L) return;
    u8* dst = (k.flags & 1) ? a.vals + a.vbase[k.b] : a.mi + k.o0;
    const u64 w = bits64f(k.p, k.plen, wi * 64);
    const u32 nv = min(64u, k.nbits - wi * 64);
    u32 cnt = 0;
    bool bad = false;
    rice_walk(w, nv, a.es[k.wb + wi], cnt, [&](u32 pos) {
        const u32 vi = vb0 + cnt;
        if (vi >= k.L) return;
        const u32 g = wi * 64 + pos;
        const u64 v = pos ? bits64f(k.p, k.plen, g) : w;
        const u32 q = (u32)__clzll((long long)~v);
        if (q > 63 || g + q + 2 >= k.nbits) {  // unary run past the stream, or a value > 255
            bad = true;
            return;
        }
        u32 r;
        if (q <= 61) {  // both remainder bits inside v
            r = (u32)(v >> (61 - q)) & 3u;
        } else {
            const u32 r0 = (k.p[(g + q + 1) >> 3] >> (7 - ((g + q + 1) & 7))) & 1u;
            const u32 r1 = (k.p[(g + q + 2) >> 3] >> (7 - ((g + q + 2) & 7))) & 1u;
            r = (r0 << 1) | r1;
        }
        const u32 val = (q << 2) | r;
        if (val > 255) {
            bad = true;
            return;
        }
        dst[vi] = (u8)inv_map(val, k.flags);
    });
    if (bad) a.d.status[k.b] = DEC_EFORMAT;
}

// (D) bit-plane blocks (id 3): deinterleave (PY:1122-1134); the 8x8 bit transpose is an
// involution
__global__ __launch_bounds__(256) void k_rice_bitplane(BwArgs a) {
    const RiceBlk k = rice_blk(a, blockIdx.y);
    const u32 gi = blockIdx.x * 256 + threadIdx.x;
    if (!(k.flags & 1) || gi >= k.L / 8 || a.d.status[k.b] != DEC_OK) return;
    const u8* src = a.vals + a.vbase[k.b];
    u32 in[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) in[i] = src[8 * gi + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u32 v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) v |= ((in[j] >> (7 - i)) & 1u) << (7 - j);
        if (8 * gi + i < k.n) a.mi[k.o0 + 8 * gi + i] = (u8)v;
    }
}

// MTF decode.  One "move the entry at position idx to the front" step on a 256-entry table
// held as 64 words per thread (tab[w * RT + t]); returns the entry.
constexpr int DRT = 128;
// word x with its byte j moved out: bytes [0, j) shift up one, `in` enters byte 0
__device__ inline u32 mtf_front(u32 x, u32 j, u32 in) {
    const u32 lowmask = j ? ((1u << (8 * j)) - 1) : 0u;
    const u32 highmask = j == 3 ? 0u : ~((1u << (8 * (j + 1))) - 1);
    return (x & highmask) | ((x & lowmask) << 8) | in;
}
// Pop entry idx to the front.  Entries 0..7 (words 0, 1) are held in registers r0, r1 (MTF
// indices of BBWT output are mostly small: no LDS round trip); words 2..63 are in LDS.
__device__ inline u32 mtf_pop_front(u32* tab, u32 t, u32 idx, u32& r0, u32& r1) {
    if (idx < 4) {
        const u32 b = (r0 >> (8 * idx)) & 0xFFu;
        r0 = mtf_front(r0, idx, b);
        return b;
    }
    const u32 c0 = r0 >> 24;
    if (idx < 8) {
        const u32 j = idx - 4, b = (r1 >> (8 * j)) & 0xFFu;
        r0 = (r0 << 8) | b;
        r1 = mtf_front(r1, j, c0);
        return b;
    }
    const u32 w = idx >> 2, j = idx & 3;
    const u32 x = tab[w * DRT + t];
    const u32 b = (x >> (8 * j)) & 0xFFu;
    u32 carry = r1 >> 24;
    r1 = (r1 << 8) | c0;
    r0 = (r0 << 8) | b;
    for (u32 v = 2; v < w; ++v) {
        const u32 xv = tab[v * DRT + t];
        tab[v * DRT + t] = (xv << 8) | carry;
        carry = xv >> 24;
    }
    tab[w * DRT + t] = mtf_front(x, j, carry);
    return b;
}

__device__ inline bool dec_chunk(const BwArgs& a, u32 c, u32& b, u32& lo, u32& hi) {
    const u32 li = c / a.cpb, k = c - li * a.cpb;
    if (li >= a.d.nlist) return false;
    b = a.d.list[li];
    const u32 o0 = a.d.obase[b], n = a.d.obase[b + 1] - o0;
    lo = o0 + k * MTF_CHUNK;
    hi = min(lo + (u32)MTF_CHUNK, o0 + n);
    return lo < o0 + n && a.d.status[b] == DEC_OK;
}

// chunk summary: the table reached from the identity (a permutation of positions)
__global__ __launch_bounds__(DRT) void k_dec_mtf_summary(BwArgs a, u32 nch) {
    __shared__ u32 tab[64 * DRT];
    const u32 t = threadIdx.x, c = blockIdx.x * DRT + t;
    u32 b, lo, hi;
    if (c >= nch || !dec_chunk(a, c, b, lo, hi)) return;
    for (u32 w = 2; w < 64; ++w) tab[w * DRT + t] = (4 * w) | ((4 * w + 1) << 8) | ((4 * w + 2) << 16) | ((4 * w + 3) << 24);
    u32 r0 = 0x03020100u, r1 = 0x07060504u;
    for (u32 i = lo; i < hi; ++i) mtf_pop_front(tab, t, a.mi[i], r0, r1);
    u32* out = reinterpret_cast<u32*>(a.summ + (u64)c * 256);
    out[0] = r0;
    out[1] = r1;
    for (u32 w = 2; w < 64; ++w) out[w] = tab[w * DRT + t];
}

// per block: entry state of every chunk; state' = state o summary
__global__ __launch_bounds__(256) void k_dec_mtf_compose(BwArgs a) {
    __shared__ u8 S[2][256];
    const u32 li = blockIdx.x, j = threadIdx.x;
    const u32 b = a.d.list[li];
    const u32 n = a.d.obase[b + 1] - a.d.obase[b];
    if (a.d.status[b] != DEC_OK) return;
    const u32 nk = (n + MTF_CHUNK - 1) / MTF_CHUNK;
    S[0][j] = (u8)j;
    __syncthreads();
    for (u32 k = 0; k < nk; ++k) {
        const u32 c = li * a.cpb + k;
        const u32 cur = k & 1;
        a.states[(u64)c * 256 + j] = S[cur][j];
        S[cur ^ 1][j] = S[cur][a.summ[(u64)c * 256 + j]];
        __syncthreads();
    }
}

__global__ __launch_bounds__(DRT) void k_dec_mtf_replay(BwArgs a, u32 nch) {
    __shared__ u32 tab[64 * DRT];
    const u32 t = threadIdx.x, c = blockIdx.x * DRT + t;
    u32 b, lo, hi;
    if (c >= nch || !dec_chunk(a, c, b, lo, hi)) return;
    const u32* s = reinterpret_cast<const u32*>(a.states + (u64)c * 256);
    u32 r0 = s[0], r1 = s[1];
    for (u32 w = 2; w < 64; ++w) tab[w * DRT + t] = s[w];
    for (u32 i = lo; i < hi; ++i) a.bw[i] = (u8)mtf_pop_front(tab, t, a.mi[i], r0, r1);
}

// Inverse BBWT (PY:425-454), grid-wide.  PI = stable counting sort of the BBWT string L
// (F-slot x -> L index); every cycle of PI is one Lyndon factor, read from its minimum
// slot m as L[PI(m)], L[PI^2(m)], ..., L[m], and the factors appear in descending order
// of m.  Cycle minima and distances come from a
// ruling set instead of pointer jumping over all n elements (n log n random gathers):
//   * splitters = slots that are multiples of S = 1 << sshift; one thread per splitter
//     walks PI to the next splitter, tagging every slot with (segment, offset);
//   * cycles that hold no splitter (e.g. the n one-slot cycles of a run) are settled by
//     their own elements: a slot walks until it meets a smaller slot or returns (minimum);
//   * the splitter graph (<= BWI_NODES per block) is solved in LDS by one workgroup:
//     min doubling, then list ranking cut at the segment holding the cycle minimum.
constexpr u32 FREE = 0x80000000u;  // segment tag of a slot on a splitter-free cycle (| its minimum)

struct BwiBlock {
    u32 b, o0, n;
    bool ok;
};
__device__ inline BwiBlock bwi_block(const BwArgs& a, u32 li) {
    BwiBlock r;
    r.b = a.d.list[li];
    r.o0 = a.d.obase[r.b];
    r.n = a.d.obase[r.b + 1] - r.o0;
    r.ok = a.d.status[r.b] == DEC_OK;
    return r;
}

// (1) byte histogram per BWI_TILE tile
__global__ __launch_bounds__(256) void k_bwi_hist(BwArgs a) {
    __shared__ u32 h[256];
    const BwiBlock k = bwi_block(a, blockIdx.y);
    const u32 lo = blockIdx.x * BWI_TILE;
    h[threadIdx.x] = 0;
    __syncthreads();
    if (k.ok && lo < k.n) {
        const u32 hi = min(lo + BWI_TILE, k.n);
        const u8* L = a.bw + k.o0;
        for (u32 i = lo + threadIdx.x; i < hi; i += 256) atomicAdd(&h[L[i]], 1u);
    }
    __syncthreads();
    a.th[((u64)blockIdx.y * a.tpb + blockIdx.x) * 256 + threadIdx.x] = h[threadIdx.x];
}

// (2) per block: slot of each tile's first byte value d = digit base + earlier tiles
__global__ __launch_bounds__(256) void k_bwi_scan(BwArgs a) {
    __shared__ u32 ws[4];
    const BwiBlock k = bwi_block(a, blockIdx.x);
    if (!k.ok || k.n == 0) return;
    const u32 d = threadIdx.x, nt = (k.n + BWI_TILE - 1) / BWI_TILE;
    u32* th = a.th + (u64)blockIdx.x * a.tpb * 256;
    u32 acc = 0;
    for (u32 t = 0; t < nt; ++t) {
        const u32 c = th[t * 256 + d];
        th[t * 256 + d] = acc;
        acc += c;
    }
    const u32 incl = wave_incl_scan(acc, OpAddU(), 0u);
    if ((d & 63) == 63) ws[d >> 6] = incl;
    __syncthreads();
    u32 base = incl - acc;
    for (u32 q = 0; q < (d >> 6); ++q) base += ws[q];
    for (u32 t = 0; t < nt; ++t) th[t * 256 + d] += base;
}

// (3) stable scatter PI[slot] = i (ballot ranking per wave, LDS counts across waves);
// also resets SO (unvisited) and D (cycle lengths) of the tile
__global__ __launch_bounds__(1024) void k_bwi_scatter(BwArgs a) {
    __shared__ u32 running[256];
    __shared__ u32 wcnt[16][256];
    const BwiBlock k = bwi_block(a, blockIdx.y);
    const u32 lo = blockIdx.x * BWI_TILE;
    if (!k.ok || lo >= k.n) return;
    const u32 hi = min(lo + BWI_TILE, k.n);
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32* th = a.th + ((u64)blockIdx.y * a.tpb + blockIdx.x) * 256;
    if (tid < 256) running[tid] = th[tid];
    for (u32 i = tid; i < 16 * 256; i += 1024) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const u8* L = a.bw + k.o0;
    u32* PI = a.X[0] + k.o0;
    u64* SO = a.so + k.o0;
    u32* D = a.X[3] + k.o0;
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (u32 s0 = lo; s0 < hi; s0 += 1024) {
        const u32 i = s0 + tid;
        const bool valid = i < hi;
        const u32 d = valid ? L[i] : 0u;
        if (valid) {
            SO[i] = NONE;
            D[i] = 0;
        }
        u64 m = __ballot(valid);
#pragma unroll
        for (u32 bit = 0; bit < 8; ++bit) {
            const u64 bal = __ballot((d >> bit) & 1u);
            m &= ((d >> bit) & 1u) ? bal : ~bal;
        }
        const u32 rank = __popcll(m & lt);
        if (valid && rank == 0) wcnt[wv][d] = __popcll(m);
        __syncthreads();
        if (valid) {
            u32 pre = running[d];
            for (u32 q = 0; q < wv; ++q) pre += wcnt[q][d];
            PI[pre + rank] = i;
        }
        __syncthreads();
        if (tid < 256) {
            u32 add = 0;
            for (u32 q = 0; q < 16; ++q) {
                add += wcnt[q][tid];
                wcnt[q][tid] = 0;
            }
            running[tid] += add;
        }
        __syncthreads();
    }
}

// node arrays of list entry li: next splitter node, segment length, segment minimum,
// cycle minimum, rank (distance from the cycle's anchor splitter)
__device__ inline u32* bwi_nodes(const BwArgs& a, u32 arr, u32 li) {
    return a.nd + ((u64)arr * a.d.nlist + li) * a.nnmax;
}

// (4) one thread per splitter: walk to the next splitter
__global__ __launch_bounds__(256) void k_bwi_walk(BwArgs a) {
    const BwiBlock k = bwi_block(a, blockIdx.y);
    const u32 j = blockIdx.x * 256 + threadIdx.x;
    const u32 x0 = j << a.sshift;
    if (!k.ok || x0 >= k.n) return;
    const u32 msk = (1u << a.sshift) - 1;
    const u32* PI = a.X[0] + k.o0;
    u64* SO = a.so + k.o0;
    u32 y = x0, len = 0, smin = x0;
    do {
        SO[y] = (u64)j | ((u64)len << 32);
        smin = min(smin, y);
        ++len;
        y = PI[y];
    } while (y & msk);
    bwi_nodes(a, 0, blockIdx.y)[j] = y >> a.sshift;
    bwi_nodes(a, 1, blockIdx.y)[j] = len;
    bwi_nodes(a, 2, blockIdx.y)[j] = smin;
}

// (5) one thread per slot on a splitter-free cycle: is it the cycle minimum?  The
// minimum then tags its cycle with (FREE | minimum, distance) and stores the length.
__global__ __launch_bounds__(256) void k_bwi_free(BwArgs a) {
    const BwiBlock k = bwi_block(a, blockIdx.y);
    const u32 x = blockIdx.x * 256 + threadIdx.x;
    if (!k.ok || x >= k.n) return;
    u64* SO = a.so + k.o0;
    if ((u32)SO[x] != NONE) return;
    const u32* PI = a.X[0] + k.o0;
    u32 z = PI[x], t = 1;
    while (z > x) {
        z = PI[z];
        ++t;
    }
    if (z != x) return;
    a.X[3][k.o0 + x] = t;
    u32 y = x, d = 0;
    do {
        SO[y] = (u64)(FREE | x) | ((u64)d << 32);
        ++d;
        y = PI[y];
    } while (y != x);
}

// (6) per block, the splitter graph in LDS: cycle minimum by min doubling, then the
// distance of every splitter from its cycle's anchor (the splitter whose segment holds
// the minimum) by list ranking with the link into the anchor cut
constexpr u32 BWI_NPT = BWI_NODES / 1024;
__global__ __launch_bounds__(1024) void k_bwi_nodes(BwArgs a) {
    __shared__ u32 J[BWI_NODES], V[BWI_NODES];
    const BwiBlock k = bwi_block(a, blockIdx.x);
    if (!k.ok || k.n == 0) return;
    const u32 nn = (k.n + (1u << a.sshift) - 1) >> a.sshift, tid = threadIdx.x;
    const u32* NX = bwi_nodes(a, 0, blockIdx.x);
    const u32* NL = bwi_nodes(a, 1, blockIdx.x);
    const u32* NS = bwi_nodes(a, 2, blockIdx.x);
    u32* NM = bwi_nodes(a, 3, blockIdx.x);
    u32* NP = bwi_nodes(a, 4, blockIdx.x);
    const u64* SO = a.so + k.o0;
    u32 R = 0;
    while ((1u << R) < nn) ++R;
    for (u32 j = tid; j < nn; j += 1024) {
        J[j] = NX[j];
        V[j] = NS[j];
    }
    __syncthreads();
    u32 rj[BWI_NPT], rv[BWI_NPT];
    for (u32 r = 0; r < R; ++r) {
#pragma unroll
        for (u32 q = 0; q < BWI_NPT; ++q) {
            const u32 j = tid + q * 1024;
            if (j < nn) {
                const u32 y = J[j];
                rv[q] = min(V[j], V[y]);
                rj[q] = J[y];
            }
        }
        __syncthreads();
#pragma unroll
        for (u32 q = 0; q < BWI_NPT; ++q) {
            const u32 j = tid + q * 1024;
            if (j < nn) {
                V[j] = rv[q];
                J[j] = rj[q];
            }
        }
        __syncthreads();
    }
    u32 anc[BWI_NPT], cm[BWI_NPT];
#pragma unroll
    for (u32 q = 0; q < BWI_NPT; ++q) {
        const u32 j = tid + q * 1024;
        if (j < nn) {
            cm[q] = V[j];
            anc[q] = (u32)SO[cm[q]];
            NM[j] = cm[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (u32 q = 0; q < BWI_NPT; ++q) {
        const u32 j = tid + q * 1024;
        if (j < nn) {
            const u32 y = NX[j];
            J[j] = y == anc[q] ? NONE : y;
            V[j] = NL[j];
        }
    }
    __syncthreads();
    for (u32 r = 0; r < R; ++r) {
#pragma unroll
        for (u32 q = 0; q < BWI_NPT; ++q) {
            const u32 j = tid + q * 1024;
            if (j < nn) {
                const u32 y = J[j];
                rv[q] = V[j] + (y != NONE ? V[y] : 0u);
                rj[q] = y != NONE ? J[y] : NONE;
            }
        }
        __syncthreads();
#pragma unroll
        for (u32 q = 0; q < BWI_NPT; ++q) {
            const u32 j = tid + q * 1024;
            if (j < nn) {
                V[j] = rv[q];
                J[j] = rj[q];
            }
        }
        __syncthreads();
    }
    // V[j] = slots from splitter j forward to the anchor's splitter (the whole cycle for the anchor)
#pragma unroll
    for (u32 q = 0; q < BWI_NPT; ++q) {
        const u32 j = tid + q * 1024;
        if (j < nn) {
            const u32 len = V[anc[q]];
            NP[j] = j == anc[q] ? 0u : len - V[j];
            if (j == anc[q]) a.X[3][k.o0 + cm[q]] = len;
        }
    }
}

// (7) per block: OFF[m] = sum of the cycle lengths D[m'] over minima m' > m (the factors
// are emitted in descending order of their minimum slot); 16 slots per thread
__global__ __launch_bounds__(1024) void k_bwi_offsets(BwArgs a) {
    __shared__ u32 sh[16];
    __shared__ u32 carry_s;
    const BwiBlock k = bwi_block(a, blockIdx.x);
    if (!k.ok || k.n == 0) return;
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32* D = a.X[3] + k.o0;
    u32* OFF = a.X[4] + k.o0;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (u32 r0 = 0; r0 < k.n; r0 += 16 * 1024) {
        // reversed index r -> slot n-1-r; thread covers r in [r0 + 16 tid, +16)
        const u32 rb = r0 + 16 * tid;
        u32 v[16], sum = 0;
#pragma unroll
        for (u32 q = 0; q < 16; ++q) {
            const u32 r = rb + q;
            v[q] = r < k.n ? D[k.n - 1 - r] : 0u;
            sum += v[q];
        }
        const u32 incl = wave_incl_scan(sum, OpAddU(), 0u);
        if (lane == 63) sh[wv] = incl;
        __syncthreads();
        u32 pre = carry_s + incl - sum;
        for (u32 q = 0; q < wv; ++q) pre += sh[q];
#pragma unroll
        for (u32 q = 0; q < 16; ++q) {
            const u32 r = rb + q;
            if (v[q]) OFF[k.n - 1 - r] = pre;
            pre += v[q];
        }
        __syncthreads();
        if (tid == 1023) carry_s = pre;
        __syncthreads();
    }
}

// (8) one thread per slot x = PI^t(m) of the cycle with minimum m:
// out[OFF[m] + (t - 1 mod D[m])] = L[x]
__global__ __launch_bounds__(256) void k_bwi_emit(BwArgs a) {
    const BwiBlock k = bwi_block(a, blockIdx.y);
    const u32 x = blockIdx.x * 256 + threadIdx.x;
    if (!k.ok || x >= k.n) return;
    const u64* SO = a.so + k.o0;
    const u64 so = SO[x];
    const u32 s = (u32)so, o = (u32)(so >> 32);
    u32 m, t, dm;
    if (s & FREE) {
        m = s & ~FREE;
        t = o;
        dm = a.X[3][k.o0 + m];
    } else {
        m = bwi_nodes(a, 3, blockIdx.y)[s];
        dm = a.X[3][k.o0 + m];
        t = bwi_nodes(a, 4, blockIdx.y)[s] + o + dm - (u32)(SO[m] >> 32);
        if (t >= dm) t -= dm;
    }
    const u32 idx = a.X[4][k.o0 + m] + (t ? t - 1 : dm - 1);
    a.d.out[k.o0 + idx] = a.bw[k.o0 + x];
}

// ---------------------------------------------------------------- Re-Pair (id 9)
// PY:1913-1978 repair_decompress: "RP" ULEB(256) ULEB(nrules) nrules x (ULEB a, ULEB b)
// ULEB(seq_len) seq_len x ULEB(sym); rule r defines symbol 256 + r; the output is the
// expansion of the final sequence.  Device: (1) every ULEB value of the stream by start
// flags + scan; (2) per block the rule lengths (in rule order: the encoder's rules only
// reference earlier symbols; a hand-made grammar with forward references takes a
// depth-first pass instead, and only a USED rule that does not resolve is an error, as
// in PY) and the final sequence's output offsets; (3) breadth-first expansion: (symbol, offset) entries split into their
// two children until only terminals remain (work = grammar tree nodes, depth iterations).
constexpr u32 RP_INVALID = 0xFFFFFFFFu;
constexpr u32 RP_INPROG = 0xFFFFFFFFu;  // rule length marks of k_rp_rules' general pass
constexpr u32 RP_BADLEN = 0xFFFFFFFEu;

__global__ __launch_bounds__(256) void k_rp_values(DecArgs a, u32* vals, u32* nval) {
    __shared__ u32 sh[4];
    const u32 b = a.list[blockIdx.x], tid = threadIdx.x;
    const u64 p0 = a.poff[b];
    const u32 plen = (u32)(a.poff[b + 1] - p0);
    const u8* pay = a.pay + p0;
    u32* V = vals + p0;
    if (plen < 2 || pay[0] != 'R' || pay[1] != 'P') {
        if (tid == 0) a.status[b] = DEC_EFORMAT;
        return;
    }
    u32 vcount = 0;
    for (u32 s0 = 2; s0 < plen; s0 += 2048) {
        const u32 j0 = s0 + tid * 8;
        u32 v[8];
        u32 nv = 0;
#pragma unroll
        for (u32 e = 0; e < 8; ++e) {
            const u32 j = j0 + e;
            v[e] = RP_INVALID;
            if (j < plen && (j == 2 || pay[j - 1] < 128)) {
                u32 x = 0, q = j;
                bool ok = false;
                for (u32 shf = 0; shf < 35 && q < plen; shf += 7) {
                    const u32 by = pay[q++];
                    if (shf == 28 && (by & 0x70u)) break;  // >= 2^32
                    x |= (by & 0x7Fu) << shf;
                    if (!(by & 0x80u)) {
                        ok = true;
                        break;
                    }
                }
                v[e] = ok && x != RP_INVALID ? x : RP_INVALID - 1;  // truncated / oversized -> marker
                ++nv;
            }
        }
        u32 tot = 0;
        u32 vi = vcount + wg_excl_sum(nv, sh, &tot);
#pragma unroll
        for (u32 e = 0; e < 8; ++e)
            if (v[e] != RP_INVALID) V[vi++] = v[e];
        vcount += tot;
    }
    if (tid == 0) nval[b] = vcount;
}

constexpr u32 RP_LDS_RULES = 32768;  // rule lengths kept in LDS (longer grammars: global)
constexpr u32 RP_CH = 2048;          // rules staged per chunk

// One workgroup per block: header checks, rule lengths (sequential in rule order, lengths
// in LDS, saturated above n), final-sequence offsets by a workgroup scan, first BFS level.
__global__ __launch_bounds__(1024) void k_rp_rules(DecArgs a, const u32* vals, const u32* nval, u32* rlen,
                                                   u64* ea, u32* ecount) {
    __shared__ u32 L[RP_LDS_RULES];
    __shared__ uint2 ch[RP_CH];
    __shared__ u32 sh[16];
    __shared__ u32 s_bad, s_carry;
    const u32 b = a.list[blockIdx.x], tid = threadIdx.x;
    if (a.status[b] != DEC_OK) return;
    const u64 p0 = a.poff[b];
    const u32* V = vals + p0;
    u32* RL = rlen + p0;
    const u32 nv = nval[b];
    const u32 o0 = a.obase[b], n = a.obase[b + 1] - o0;
    const u32 cap = n + 1;  // saturation: any expansion longer than the block is an error
    // header: 256, nrules, 2 nrules symbols, seq_len, seq_len symbols
    bool bad = nv < 3 || V[0] != 256u;
    const u32 nr = bad ? 0u : V[1];
    bad = bad || nr > (nv - 3) / 2;
    const u32 sl = bad ? 0u : V[2 + 2 * nr];
    bad = bad || sl > nv - 3 - 2 * nr || sl > n;
    if (bad) {
        if (tid == 0) a.status[b] = DEC_EFORMAT;
        return;
    }
    if (tid == 0) s_bad = NONE;
    __syncthreads();
    // rule lengths, in rule order (the encoder's rules only reference earlier symbols)
    for (u32 c0 = 0; c0 < nr && s_bad == NONE; c0 += RP_CH) {
        const u32 m = min(RP_CH, nr - c0);
        for (u32 i = tid; i < m; i += 1024) ch[i] = make_uint2(V[2 + 2 * (c0 + i)], V[3 + 2 * (c0 + i)]);
        __syncthreads();
        if (tid == 0) {
            for (u32 i = 0; i < m; ++i) {
                const u32 r = c0 + i, x = ch[i].x, y = ch[i].y;
                if (x >= 256 + r || y >= 256 + r) {  // forward / self reference: general pass below
                    s_bad = r;
                    break;
                }
                const u32 lx = x < 256 ? 1u : (x - 256 < RP_LDS_RULES ? L[x - 256] : RL[x - 256]);
                const u32 ly = y < 256 ? 1u : (y - 256 < RP_LDS_RULES ? L[y - 256] : RL[y - 256]);
                const u32 l = min(lx + ly, cap);
                if (r < RP_LDS_RULES)
                    L[r] = l;
                else
                    RL[r] = l;
            }
        }
        __syncthreads();
    }
    __syncthreads();
    if (s_bad != NONE) {
        // A hand-made grammar may reference later rules; PY (PY:1945-1970) accepts it as
        // long as every symbol it expands resolves, and never looks at unused rules.
        // Rules from r0 on get their lengths by an iterative depth-first pass (thread 0,
        // explicit stack in RL[nr, 2nr): 2nr + 3 <= values <= payload bytes).  Marks:
        // 0 unknown, RP_INPROG on the stack (a child on the stack = a cycle), RP_BADLEN for
        // a rule that does not resolve (cycle / undefined symbol): an error only if used.
        const u32 r0 = s_bad;
        for (u32 r = r0 + tid; r < nr; r += 1024) {
            if (r < RP_LDS_RULES)
                L[r] = 0;
            else
                RL[r] = 0;
        }
        __syncthreads();
        if (tid == 0) {
            auto get = [&](u32 s) -> u32 {
                return s < 256 ? 1u : s - 256 >= nr ? RP_BADLEN : s - 256 < RP_LDS_RULES ? L[s - 256] : RL[s - 256];
            };
            auto put = [&](u32 r, u32 v) {
                if (r < RP_LDS_RULES)
                    L[r] = v;
                else
                    RL[r] = v;
            };
            u32* stk = RL + nr;
            for (u32 r = r0; r < nr; ++r) {
                if (get(256 + r)) continue;
                u32 sp = 0;
                stk[sp++] = r;
                put(r, RP_INPROG);
                while (sp) {
                    const u32 t = stk[sp - 1], x = V[2 + 2 * t], y = V[3 + 2 * t];
                    const u32 lx = get(x), ly = get(y);
                    if (!lx || !ly) {
                        const u32 c = (!lx ? x : y) - 256;
                        put(c, RP_INPROG);
                        stk[sp++] = c;
                        continue;
                    }
                    put(t, lx >= RP_BADLEN || ly >= RP_BADLEN ? RP_BADLEN : min(lx + ly, cap));
                    --sp;
                }
            }
        }
        __syncthreads();
    }
    for (u32 r = tid; r < min(nr, RP_LDS_RULES); r += 1024) RL[r] = L[r];
    // final sequence: lengths, offsets, first level of entries
    const u32* S = V + 3 + 2 * nr;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    bool sbad = false;
    for (u32 j0 = 0; j0 < sl; j0 += 1024) {
        const u32 j = j0 + tid;
        u32 sym = 0, l = 0;
        if (j < sl) {
            sym = S[j];
            if (sym >= 256 + nr) {
                sbad = true;
            } else {
                l = sym < 256 ? 1u : (sym - 256 < RP_LDS_RULES ? L[sym - 256] : RL[sym - 256]);
                if (l >= RP_BADLEN) {  // an unresolvable rule (cycle / undefined symbol) is used
                    sbad = true;
                    l = 0;
                }
            }
        }
        u32 tot = 0;
        const u32 off = s_carry + wg_excl_sum(l, sh, &tot);
        if (j < sl && off + l <= n) ea[o0 + j] = (u64)sym | ((u64)off << 32);
        if (j < sl && off + l > n) sbad = true;
        __syncthreads();
        if (tid == 0) s_carry = min(s_carry + tot, cap);  // totals past n are errors
        __syncthreads();
    }
    const bool anyb = __syncthreads_or(sbad);
    if (tid == 0) {
        if (anyb || s_carry != n) a.status[b] = anyb && s_carry <= n ? DEC_EFORMAT : DEC_ELEN;
        ecount[blockIdx.x] = sl;
    }
}

// Breadth-first expansion, one workgroup per block: terminals write their byte, rule
// entries append their two children (wave-aggregated LDS counter), until none remain.
__global__ __launch_bounds__(1024) void k_rp_expand(DecArgs a, const u32* vals, const u32* rlen, u64* ea, u64* eb,
                                                    const u32* ecount) {
    __shared__ u32 s_next;
    const u32 b = a.list[blockIdx.x], tid = threadIdx.x, lane = tid & 63;
    if (a.status[b] != DEC_OK) return;
    const u64 p0 = a.poff[b];
    const u32* V = vals + p0;
    const u32* RL = rlen + p0;
    const u32 o0 = a.obase[b];
    u8* out = a.out + o0;
    u64* A = ea + o0;
    u64* B = eb + o0;
    u32 cnt = ecount[blockIdx.x];
    while (cnt) {
        if (tid == 0) s_next = 0;
        __syncthreads();
        for (u32 i0 = 0; i0 < cnt; i0 += 1024) {
            const u32 i = i0 + tid;
            const bool valid = i < cnt;
            u64 e = valid ? A[i] : 0ull;
            const u32 sym = (u32)e, off = (u32)(e >> 32);
            const bool nt = valid && sym >= 256;
            if (valid && !nt) out[off] = (u8)sym;
            u32 x = 0, y = 0, lx = 0;
            if (nt) {
                const u32 r = sym - 256;
                x = V[2 + 2 * r];
                y = V[3 + 2 * r];
                lx = x < 256 ? 1u : RL[x - 256];
            }
            const u64 m = __ballot(nt);
            u32 base = 0;
            if (m) {
                const u32 leader = __ffsll((long long)m) - 1;
                if (lane == leader) base = atomicAdd(&s_next, 2u * (u32)__popcll(m));
                base = __shfl(base, leader);
            }
            if (nt) {
                const u32 k = base + 2u * (u32)__popcll(m & ((1ull << lane) - 1ull));
                B[k] = (u64)x | ((u64)off << 32);
                B[k + 1] = (u64)y | ((u64)(off + lx) << 32);
            }
        }
        __syncthreads();
        cnt = s_next;
        u64* t = A;
        A = B;
        B = t;
        __syncthreads();
    }
}

}  // namespace

void launch_dec_bw(const BwArgs& a, hipStream_t s) {
    if (!a.d.nlist) return;
    const u32 nch = a.d.nlist * a.cpb;
    const u32 wg = (a.wmax + 255) / 256;
    k_rice_phase<<<dim3(wg, a.d.nlist), 256, 0, s>>>(a);
    k_rice_chain<<<a.d.nlist, DRC, 0, s>>>(a);
    k_rice_vals<<<dim3(wg, a.d.nlist), 256, 0, s>>>(a);
    k_rice_bitplane<<<dim3((a.tpb * BWI_TILE / 8 + 255) / 256, a.d.nlist), 256, 0, s>>>(a);
    k_dec_mtf_summary<<<(nch + DRT - 1) / DRT, DRT, 0, s>>>(a, nch);
    k_dec_mtf_compose<<<a.d.nlist, 256, 0, s>>>(a);
    k_dec_mtf_replay<<<(nch + DRT - 1) / DRT, DRT, 0, s>>>(a, nch);
    const u32 nl = a.d.nlist;
    const u32 mx = a.tpb * BWI_TILE;  // >= the longest block
    k_bwi_hist<<<dim3(a.tpb, nl), 256, 0, s>>>(a);
    k_bwi_scan<<<nl, 256, 0, s>>>(a);
    k_bwi_scatter<<<dim3(a.tpb, nl), 1024, 0, s>>>(a);
    k_bwi_walk<<<dim3((a.nnmax + 255) / 256, nl), 256, 0, s>>>(a);
    k_bwi_free<<<dim3((mx + 255) / 256, nl), 256, 0, s>>>(a);
    k_bwi_nodes<<<nl, 1024, 0, s>>>(a);
    k_bwi_offsets<<<nl, 1024, 0, s>>>(a);
    k_bwi_emit<<<dim3((mx + 255) / 256, nl), 256, 0, s>>>(a);
}

void launch_dec_raw(const DecArgs& a, hipStream_t s) {
    if (a.nlist) k_dec_raw<<<a.nlist, 256, 0, s>>>(a);
}

void launch_dec_uleb(const DecArgs& a, bool lfsr, hipStream_t s) {
    if (!a.nlist) return;
    if (lfsr)
        k_dec_uleb<true><<<a.nlist, 256, 0, s>>>(a);
    else
        k_dec_uleb<false><<<a.nlist, 256, 0, s>>>(a);
}

void launch_dec_repair(const DecArgs& a, u32* vals, u32* nval, u32* ecount, u32* rlen, u64* ea, u64* eb,
                       hipStream_t s) {
    if (!a.nlist) return;
    k_rp_values<<<a.nlist, 256, 0, s>>>(a, vals, nval);
    k_rp_rules<<<a.nlist, 1024, 0, s>>>(a, vals, nval, rlen, ea, ecount);
    k_rp_expand<<<a.nlist, 1024, 0, s>>>(a, vals, rlen, ea, eb, ecount);
}

void launch_dec_lz77(const DecArgs& a, u32* tpos, u32* tval, u32* ntok, u32* mark, u32* src, hipStream_t s) {
    if (!a.nlist) return;
    k_dec_lz_parse<<<(a.nlist + 63) / 64, 64, 0, s>>>(a, tpos, tval, ntok);
    k_dec_lz_resolve<<<a.nlist, 1024, 0, s>>>(a, tpos, tval, ntok, mark, src);
}

}  // namespace kolm
