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

__device__ inline u64 word_at(const u8* p, u32 plen, u32 wi) { return bits64(p, plen, wi * 64); }

// One workgroup per block: per-thread word ranges -> phase functions -> sequential phase
// chain over the 256 ranges -> values at every codeword start (index < L), inverse map,
// bit-plane transpose for id 3.  Output: MTF indices at obase.
__global__ __launch_bounds__(256) void k_dec_rice(BwArgs a) {
    __shared__ u32 fex[256][4], fcnt[256][4], entry[256], sbase[256];
    __shared__ u32 total;
    const u32 b = a.d.list[blockIdx.x], tid = threadIdx.x;
    const u64 p0 = a.d.poff[b];
    const u32 plen = (u32)(a.d.poff[b + 1] - p0);
    const u32 o0 = a.d.obase[b], n = a.d.obase[b + 1] - o0;
    const u32 flags = bw_flags(a.meth[b]);
    const u32 L = (flags & 1) ? 8 * ((n + 7) / 8) : n;
    const u8* p = a.d.pay + p0;
    const u32 nbits = plen * 8, nw = (nbits + 63) / 64;
    const u32 per = (nw + 255) / 256, w0 = min(tid * per, nw), w1 = min(w0 + per, nw);
    // phase function of the thread's words for each entry phase
    for (u32 e = 0; e < 4; ++e) {
        u32 st = e, cnt = 0;
        for (u32 wi = w0; wi < w1; ++wi)
            st = rice_walk(word_at(p, plen, wi), min(64u, nbits - wi * 64), st, cnt, [](u32) {});
        fex[tid][e] = st;
        fcnt[tid][e] = cnt;
    }
    __syncthreads();
    if (tid == 0) {
        u32 st = RS_S, base = 0;
        for (u32 t = 0; t < 256; ++t) {
            entry[t] = st;
            sbase[t] = base;
            base += fcnt[t][st];
            st = fex[t][st];
        }
        total = base;
    }
    __syncthreads();
    bool bad = total < L;
    u8* dst = (flags & 1) ? a.vals + a.vbase[b] : a.mi + o0;
    {
        u32 st = entry[tid], cnt = 0;
        const u32 vb0 = sbase[tid];
        for (u32 wi = w0; wi < w1; ++wi) {
            st = rice_walk(word_at(p, plen, wi), min(64u, nbits - wi * 64), st, cnt, [&](u32 pos) {
                const u32 vi = vb0 + cnt;
                if (vi >= L) return;
                const u32 g = wi * 64 + pos;
                const u64 v = bits64(p, plen, g);
                const u32 q = (u32)__clzll((long long)~v);
                if (q > 63 || g + q + 2 >= nbits) {
                    bad = true;
                    return;
                }
                const u32 r0 = (p[(g + q + 1) >> 3] >> (7 - ((g + q + 1) & 7))) & 1u;
                const u32 r1 = (p[(g + q + 2) >> 3] >> (7 - ((g + q + 2) & 7))) & 1u;
                const u32 val = (q << 2) | (r0 << 1) | r1;
                if (val > 255) {
                    bad = true;
                    return;
                }
                dst[vi] = (u8)inv_map(val, flags);
            });
        }
    }
    if (__syncthreads_or(bad)) {
        if (tid == 0) a.d.status[b] = DEC_EFORMAT;
        return;
    }
    if (flags & 1) {  // bit-plane deinterleave (PY:1122-1134): the 8x8 bit transpose is an involution
        for (u32 gi = tid; gi < L / 8; gi += 256) {
            u32 in[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) in[i] = dst[8 * gi + i];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                u32 v = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) v |= ((in[j] >> (7 - i)) & 1u) << (7 - j);
                if (8 * gi + i < n) a.mi[o0 + 8 * gi + i] = (u8)v;
            }
        }
    }
}

// MTF decode.  One "move the entry at position idx to the front" step on a 256-entry table
// held as 64 words per thread (tab[w * RT + t]); returns the entry.
constexpr int DRT = 128;
__device__ inline u32 mtf_pop_front(u32* tab, u32 t, u32 idx) {
    const u32 w = idx >> 2, j = idx & 3;
    const u32 x = tab[w * DRT + t];
    const u32 b = (x >> (8 * j)) & 0xFFu;
    u32 carry = b;
    for (u32 v = 0; v < w; ++v) {
        const u32 xv = tab[v * DRT + t];
        tab[v * DRT + t] = (xv << 8) | carry;
        carry = xv >> 24;
    }
    const u32 lowmask = j ? ((1u << (8 * j)) - 1) : 0u;
    const u32 highmask = j == 3 ? 0u : ~((1u << (8 * (j + 1))) - 1);
    tab[w * DRT + t] = (x & highmask) | ((x & lowmask) << 8) | carry;
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
    for (u32 w = 0; w < 64; ++w) tab[w * DRT + t] = (4 * w) | ((4 * w + 1) << 8) | ((4 * w + 2) << 16) | ((4 * w + 3) << 24);
    for (u32 i = lo; i < hi; ++i) mtf_pop_front(tab, t, a.mi[i]);
    u32* out = reinterpret_cast<u32*>(a.summ + (u64)c * 256);
    for (u32 w = 0; w < 64; ++w) out[w] = tab[w * DRT + t];
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
    for (u32 w = 0; w < 64; ++w) tab[w * DRT + t] = s[w];
    for (u32 i = lo; i < hi; ++i) a.bw[i] = (u8)mtf_pop_front(tab, t, a.mi[i]);
}

// Inverse BBWT (PY:425-454), one workgroup per block.  pi = stable sort of positions by
// byte; every cycle of pi is one factor, read from its minimum c as L[pi(c)], L[pi^2(c)],
// ..., L[c]; factors are emitted by decreasing minimum.  Here: cycle minima by doubling
// (m <- min(m, m[P]), P <- P[P]), the steps s(x) from x to its minimum by list ranking,
// cycle lengths d(c) = s(pi(c)) + 1, factor offsets by a reverse scan over the minima, and
// x = pi^k(c) with k = d(c) - s(x) lands at offset(c) + k - 1.
__global__ __launch_bounds__(1024) void k_dec_bwi(BwArgs a) {
    __shared__ u32 hist[256], running[256];
    __shared__ u32 wcnt[16][256];
    __shared__ u32 sh[16];
    __shared__ u32 carry_s;
    const u32 b = a.d.list[blockIdx.x], tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32 o0 = a.d.obase[b], n = a.d.obase[b + 1] - o0;
    if (a.d.status[b] != DEC_OK || n == 0) return;
    const u8* L = a.bw + o0;
    u32 *PI = a.X[0] + o0, *P0 = a.X[1] + o0, *P1 = a.X[2] + o0, *M0 = a.X[3] + o0, *M1 = a.X[4] + o0;
    u32 *N0 = a.X[5] + o0, *N1 = a.X[6] + o0, *W0 = a.X[7] + o0;
    // (a) stable counting sort by byte
    for (u32 i = tid; i < 256; i += 1024) hist[i] = 0;
    __syncthreads();
    for (u32 i = tid; i < n; i += 1024) atomicAdd(&hist[L[i]], 1u);
    __syncthreads();
    if (tid == 0) {
        u32 acc = 0;
        for (u32 d = 0; d < 256; ++d) {
            running[d] = acc;
            acc += hist[d];
        }
    }
    for (u32 i = tid; i < 16 * 256; i += 1024) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (u32 t0 = 0; t0 < n; t0 += 1024) {
        const u32 i = t0 + tid;
        const bool valid = i < n;
        const u32 d = valid ? L[i] : 0u;
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
    // (b) cycle minima: ceil(log2 n) doubling rounds cover every cycle
    u32 R = 0;
    while ((1u << R) < n) ++R;
    for (u32 x = tid; x < n; x += 1024) {
        const u32 y = PI[x];
        P0[x] = y;
        M0[x] = min(x, y);
    }
    __syncthreads();
    for (u32 r = 0; r < R; ++r) {
        for (u32 x = tid; x < n; x += 1024) {
            const u32 y = P0[x];
            M1[x] = min(M0[x], M0[y]);
            P1[x] = P0[y];
        }
        __syncthreads();
        u32* t = P0; P0 = P1; P1 = t;
        t = M0; M0 = M1; M1 = t;
    }
    // (c) steps to the cycle minimum by list ranking (x -> pi(x) unless x is the minimum)
    u32* Wa = W0;
    u32* Wb = P1;  // free now
    for (u32 x = tid; x < n; x += 1024) {
        const bool head = M0[x] == x;
        N0[x] = head ? NONE : PI[x];
        Wa[x] = head ? 0u : 1u;
    }
    __syncthreads();
    for (u32 r = 0; r < R; ++r) {
        for (u32 x = tid; x < n; x += 1024) {
            const u32 y = N0[x];
            Wb[x] = Wa[x] + (y != NONE ? Wa[y] : 0u);
            N1[x] = y != NONE ? N0[y] : NONE;
        }
        __syncthreads();
        u32* t = N0; N0 = N1; N1 = t;
        t = Wa; Wa = Wb; Wb = t;
    }
    // (d) cycle lengths at the minima, offsets by a reverse exclusive scan over positions
    u32* D = P0;    // d(c) at minima
    u32* OFF = N0;  // offset(c) at minima
    for (u32 x = tid; x < n; x += 1024)
        if (M0[x] == x) D[x] = Wa[PI[x]] + 1;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (u32 t1 = n; t1 > 0;) {
        const u32 t0 = t1 > 1024 ? t1 - 1024 : 0;
        const u32 x = t1 - 1 - tid;  // descending within the tile
        const bool valid = tid < t1 - t0;
        const u32 v = (valid && M0[x] == x) ? D[x] : 0u;
        const u32 incl = wave_incl_scan(v, OpAddU(), 0u);
        if (lane == 63) sh[wv] = incl;
        __syncthreads();
        u32 pre = carry_s;
        for (u32 q = 0; q < wv; ++q) pre += sh[q];
        if (valid && M0[x] == x) OFF[x] = pre + incl - v;
        __syncthreads();
        if (tid == 1023) carry_s = pre + incl;
        __syncthreads();
        t1 = t0;
    }
    // (e) emit
    for (u32 x = tid; x < n; x += 1024) {
        const u32 c = M0[x];
        const u32 k = D[c] - Wa[x];
        a.d.out[o0 + OFF[c] + k - 1] = L[x];
    }
}

}  // namespace

void launch_dec_bw(const BwArgs& a, hipStream_t s) {
    if (!a.d.nlist) return;
    const u32 nch = a.d.nlist * a.cpb;
    k_dec_rice<<<a.d.nlist, 256, 0, s>>>(a);
    k_dec_mtf_summary<<<(nch + DRT - 1) / DRT, DRT, 0, s>>>(a, nch);
    k_dec_mtf_compose<<<a.d.nlist, 256, 0, s>>>(a);
    k_dec_mtf_replay<<<(nch + DRT - 1) / DRT, DRT, 0, s>>>(a, nch);
    k_dec_bwi<<<a.d.nlist, 1024, 0, s>>>(a);
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

void launch_dec_lz77(const DecArgs& a, u32* tpos, u32* tval, u32* ntok, u32* mark, u32* src, hipStream_t s) {
    if (!a.nlist) return;
    k_dec_lz_parse<<<(a.nlist + 63) / 64, 64, 0, s>>>(a, tpos, tval, ntok);
    k_dec_lz_resolve<<<a.nlist, 1024, 0, s>>>(a, tpos, tval, ntok, mark, src);
}

}  // namespace kolm
