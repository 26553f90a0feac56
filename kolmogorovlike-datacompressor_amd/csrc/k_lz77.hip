// LZ77 (replaces PY:1686-1763 _lz77_match_len_overlap + encode_lz77, CPP:2268-2377).
//
// Reference semantics: greedy parse; at position pos the window is the previous
// min(pos, 4096) bytes of the block; every distance d in [1, min(pos,4096)] is tried in
// ascending order and the match length is the overlapping LCP of block[pos:] and
// block[pos-d:] (unbounded); a strictly longer match wins (ties -> smallest d);
// best >= 3 emits [1][ULEB len][ULEB dist], otherwise [0][byte].
//
// GPU formulation (bit-exact):
//   * any match >= 3 starts with an equal 3-gram, so the candidates are exactly the
//     previous occurrences of p's 3-gram inside the window: the chain prev3[] read off
//     the linear suffix array right after its 3-character round (k_sort.hip k_prev3),
//     walked from the nearest (= ascending distance);
//   * k_lz_match: for every position, the best match capped at LZ_CAP bytes (exact when
//     shorter than the cap; the chain walk stops once the cap is reached);
//   * k_lz_parse: one wave per block walks the greedy path, 64 positions per window
//     (Lc/Dc loaded by the 64 lanes, path resolved with uniform readlane steps).  A
//     position whose capped length hit LZ_CAP ("long") is resolved exactly on the spot:
//     the wave walks the whole chain and extends each candidate that can still beat the
//     current best with 64-lane byte compares;
//   * k_lz_emit: one thread per token writes its bytes at the token's offset.
#include "kolm_internal.h"

namespace kolm {

namespace {

__global__ __launch_bounds__(256) void k_lz_match(LzArgs z) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= z.geo.N) return;
    const u32 b = z.geo.block_of(p);
    const u32 end = z.geo.end(b);
    const u8* t = z.text;
    u32 best = 0, bd = 0;
    if (p + (u32)LZ_MIN <= end) {
        const u32 maxl = min((u32)LZ_CAP, end - p);
        u32 q = z.prev3[p];
        while (q != NONE && p - q <= (u32)LZ_WINDOW) {
            u32 l = LZ_MIN;
            while (l < maxl && t[p + l] == t[q + l]) ++l;
            if (l > best) {
                best = l;
                bd = p - q;
                if (l >= maxl) break;
            }
            q = z.prev3[q];
        }
    }
    z.Lc[p] = (u8)best;
    z.Dc[p] = (u16)bd;
}

__device__ inline u32 uleb_len(u32 v) {
    u32 n = 1;
    while (v >= 128) {
        v >>= 7;
        ++n;
    }
    return n;
}

// Exact longest match at p (wave-cooperative; all lanes call with identical arguments).
__device__ void exact_match(const u8* t, const u32* prev3, u32 p, u32 end, u32& out_len, u32& out_dist) {
    const u32 lane = threadIdx.x & 63;
    u32 best = 0, bd = 0;
    const u32 maxl = end - p;
    u32 q = prev3[p];
    while (q != NONE && p - q <= (u32)LZ_WINDOW) {
        bool cand = true;
        if (best >= maxl) break;  // nothing can be longer
        if (best > 0) cand = t[p + best] == t[q + best];  // must extend past best
        if (cand) {
            // LCP(p, q), 64 lanes x 4 bytes per step
            u32 l = 0;
            for (;;) {
                u32 mism = 0xFFFFFFFFu;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const u32 o = l + j * 64 + lane;
                    const bool bad = (o >= maxl) || (t[p + o] != t[q + o]);
                    const u64 bal = __ballot(bad);
                    if (bal && mism == 0xFFFFFFFFu) mism = l + j * 64 + (__ffsll((long long)bal) - 1);
                }
                if (mism != 0xFFFFFFFFu) {
                    l = mism;
                    break;
                }
                l += 256;
            }
            if (l > best) {
                best = l;
                bd = p - q;
            }
        }
        q = prev3[q];
    }
    out_len = best;
    out_dist = bd;
}

// one wave per block
__global__ __launch_bounds__(64) void k_lz_parse(LzArgs z) {
    const u32 b = blockIdx.x;
    const u32 lane = threadIdx.x;
    const u32 base = z.geo.base(b), end = z.geo.end(b);
    u32 pos = base;
    u32 ntok = 0, off = 0, nlong = 0;
    u32* tp = z.tok_pos + base;
    u32* tl = z.tok_len + base;
    u32* td = z.tok_dist + base;
    u32* to = z.tok_off + base;
    while (pos < end) {
        const u32 P = pos + lane;
        const u32 Lw = P < end ? (u32)z.Lc[P] : 0u;
        const u32 Dw = P < end ? (u32)z.Dc[P] : 0u;
        u32 cur = 0;
        while (cur < 64 && pos + cur < end) {
            const u32 Lv = __builtin_amdgcn_readlane(Lw, cur);
            u32 len, dist;
            if (Lv >= (u32)LZ_CAP) {
                exact_match(z.text, z.prev3, pos + cur, end, len, dist);
                ++nlong;
            } else {
                len = Lv;
                dist = __builtin_amdgcn_readlane(Dw, cur);
            }
            if (lane == 0) {
                tp[ntok] = pos + cur;
                to[ntok] = off;
                if (len >= (u32)LZ_MIN) {
                    tl[ntok] = len;
                    td[ntok] = dist;
                } else {
                    tl[ntok] = 0;
                    td[ntok] = 0;
                }
            }
            ++ntok;
            if (len >= (u32)LZ_MIN) {
                off += 1 + uleb_len(len) + uleb_len(dist);
                cur += len;
            } else {
                off += 2;
                cur += 1;
            }
        }
        pos += cur;
    }
    if (lane == 0) {
        z.ntok[b] = ntok;
        z.lz_size[b] = off;
        if (nlong) atomicAdd(z.nlong, nlong);
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

__global__ __launch_bounds__(256) void k_lz_emit(LzArgs z, const u32* method, const u64* off, u8* arena,
                                                 int force_all) {
    const u32 b = blockIdx.y;
    if (!force_all && method[b] != 7u) return;
    const u32 nt = z.ntok[b];
    const u32 base = z.geo.base(b);
    u8* dst = arena + off[b];
    for (u32 t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
        const u32 o = z.tok_off[base + t];
        const u32 len = z.tok_len[base + t];
        u8* d = dst + o;
        if (len == 0) {
            d[0] = 0;
            d[1] = z.text[z.tok_pos[base + t]];
        } else {
            d[0] = 1;
            const u32 n1 = put_uleb(d + 1, len);
            put_uleb(d + 1 + n1, z.tok_dist[base + t]);
        }
    }
}

}  // namespace

void launch_lz_match(const LzArgs& z, hipStream_t s) {
    if (!z.geo.N) return;
    k_lz_match<<<(u32)((z.geo.N + 255) / 256), 256, 0, s>>>(z);
}

void launch_lz_parse(const LzArgs& z, hipStream_t s) {
    if (!z.geo.nb) return;
    k_lz_parse<<<z.geo.nb, 64, 0, s>>>(z);
}

void launch_lz_emit(const LzArgs& z, const u32* method, const u64* off, u8* arena, hipStream_t s) {
    if (!z.geo.nb) return;
    dim3 grid(64, z.geo.nb);
    k_lz_emit<<<grid, 256, 0, s>>>(z, method, off, arena, method == nullptr ? 1 : 0);
}

}  // namespace kolm
