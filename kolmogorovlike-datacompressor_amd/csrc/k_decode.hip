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

}  // namespace

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
