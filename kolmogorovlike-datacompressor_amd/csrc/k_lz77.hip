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
//   * the greedy parse is made parallel by speculation: k_lz_spec parses every
//     LZ_CHUNK-byte chunk with its own wave starting at the chunk start (64-position
//     windows of Lc/Dc loaded by the lanes and prefetched one window ahead, tokens
//     buffered in lanes and stored 64 at a time).  k_lz_stitch then walks, per block,
//     the TRUE path from the real entry of each chunk only until it lands on a position
//     of that chunk's speculative path (from there both parses are identical because a
//     token depends on its position only); greedy parses re-synchronise within a few
//     tokens.  A position whose capped length hit LZ_CAP ("long") is resolved exactly on
//     the spot (whole chain, candidates extended with 64-lane byte compares);
//   * k_lz_emit: one thread per token slot writes its bytes at its final offset.
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

__device__ inline u32 tok_bytes(u32 len, u32 dist) { return len ? 1 + uleb_len(len) + uleb_len(dist) : 2; }

// Exact longest match at p (wave-cooperative; all lanes call with identical arguments).
__device__ void exact_match(const u8* t, const u32* prev3, u32 p, u32 end, u32& out_len, u32& out_dist) {
    const u32 lane = threadIdx.x & 63;
    u32 best = 0, bd = 0;
    const u32 maxl = end - p;
    u32 q = prev3[p];
    while (q != NONE && p - q <= (u32)LZ_WINDOW) {
        if (best >= maxl) break;  // nothing can be longer
        bool cand = true;
        if (best > 0) cand = t[p + best] == t[q + best];  // must extend past best
        if (cand) {
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

// token at q from its (capped) match record; len 0 = literal
__device__ inline void token_at(const LzArgs& z, u32 q, u32 end, u32 Lv, u32 Dv, u32& len, u32& dist, u32& nlong) {
    if (Lv >= (u32)LZ_CAP) {
        exact_match(z.text, z.prev3, q, end, len, dist);
        ++nlong;
    } else {
        len = Lv;
        dist = Dv;
    }
    if (len < (u32)LZ_MIN) {
        len = 0;
        dist = 0;
    }
}

// Speculative parse of one chunk per wave (4 waves per workgroup).
__global__ __launch_bounds__(256) void k_lz_spec(LzArgs z, u32 nchunks) {
    const u32 lane = threadIdx.x & 63;
    const u32 c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nchunks) return;
    const u32 b = c / z.cpb, k = c - b * z.cpb;
    const u32 bend = z.geo.end(b);
    const u32 s = z.geo.base(b) + k * LZ_CHUNK;
    if (s >= bend) {
        if (lane == 0) {
            z.c_ntok[c] = 0;
            z.c_exit[c] = s;
            z.c_bytes[c] = 0;
        }
        return;
    }
    const u32 e = min(s + (u32)LZ_CHUNK, bend);
    u32 wbase = s;
    u32 P = wbase + lane;
    u32 Lw = P < bend ? (u32)z.Lc[P] : 0u, Dw = P < bend ? (u32)z.Dc[P] : 0u;
    P += 64;
    u32 Ln = P < bend ? (u32)z.Lc[P] : 0u, Dn = P < bend ? (u32)z.Dc[P] : 0u;
    u32 q = s, ntok = 0, off = 0, nlong = 0, nbuf = 0;
    u32 bpos = 0, blen = 0, bdist = 0, boff = 0;
    while (q < e) {
        if (q >= wbase + 64) {
            if (q < wbase + 128) {
                Lw = Ln;
                Dw = Dn;
                wbase += 64;
            } else {
                wbase = q;
                const u32 P0 = wbase + lane;
                Lw = P0 < bend ? (u32)z.Lc[P0] : 0u;
                Dw = P0 < bend ? (u32)z.Dc[P0] : 0u;
            }
            const u32 P1 = wbase + 64 + lane;
            Ln = P1 < bend ? (u32)z.Lc[P1] : 0u;
            Dn = P1 < bend ? (u32)z.Dc[P1] : 0u;
        }
        const u32 cur = q - wbase;
        const u32 Lv = __builtin_amdgcn_readlane(Lw, cur);
        const u32 Dv = __builtin_amdgcn_readlane(Dw, cur);
        u32 len, dist;
        token_at(z, q, bend, Lv, Dv, len, dist, nlong);
        if (lane == nbuf) {
            bpos = q;
            blen = len;
            bdist = dist;
            boff = off;
        }
        if (++nbuf == 64) {
            const u32 slot = s + ntok + 1 - 64 + lane;
            z.tok_pos[slot] = bpos;
            z.tok_len[slot] = blen;
            z.tok_dist[slot] = bdist;
            z.tok_off[slot] = boff;
            nbuf = 0;
        }
        ++ntok;
        off += tok_bytes(len, dist);
        q += len ? len : 1;
    }
    if (lane < nbuf) {
        const u32 slot = s + ntok - nbuf + lane;
        z.tok_pos[slot] = bpos;
        z.tok_len[slot] = blen;
        z.tok_dist[slot] = bdist;
        z.tok_off[slot] = boff;
    }
    if (lane == 0) {
        z.c_ntok[c] = ntok;
        z.c_exit[c] = q;
        z.c_bytes[c] = off;
        if (nlong) atomicAdd(z.nlong, nlong);
    }
}

// Per block (one wave): real chunk entries, fix-up tokens, chunk output offsets, size.
__global__ __launch_bounds__(64) void k_lz_stitch(LzArgs z) {
    const u32 b = blockIdx.x;
    const u32 lane = threadIdx.x;
    const u32 base = z.geo.base(b), bend = z.geo.end(b);
    u32 entry = base, boff = 0, ntot = 0, fi = 0, nlong = 0;
    for (u32 k = 0; k < z.cpb; ++k) {
        const u32 c = b * z.cpb + k;
        const u32 s = base + k * LZ_CHUNK;
        if (s >= bend) break;
        const u32 e = min(s + (u32)LZ_CHUNK, bend);
        const u32 nt = z.c_ntok[c];
        u32 first, nfix = 0, fixbytes = 0, next;
        const u32 fix0 = base + fi;
        if (entry == s) {
            first = 0;
            next = z.c_exit[c];
        } else if (entry >= e) {
            first = nt;
            next = entry;
        } else {
            u32 q = entry, j = 0;
            bool conv = false;
            while (q < e) {
                while (j < nt && z.tok_pos[s + j] < q) ++j;
                if (j < nt && z.tok_pos[s + j] == q) {
                    conv = true;
                    break;
                }
                u32 len, dist;
                token_at(z, q, bend, z.Lc[q], z.Dc[q], len, dist, nlong);
                if (lane == 0) {
                    z.fix_pos[base + fi] = q;
                    z.fix_len[base + fi] = len;
                    z.fix_dist[base + fi] = dist;
                    z.fix_off[base + fi] = boff + fixbytes;
                }
                ++fi;
                ++nfix;
                fixbytes += tok_bytes(len, dist);
                q += len ? len : 1;
            }
            first = conv ? j : nt;
            next = conv ? z.c_exit[c] : q;
        }
        const u32 spec_bytes = first < nt ? z.c_bytes[c] - z.tok_off[s + first] : 0u;
        if (lane == 0) {
            z.c_first[c] = first;
            z.c_fix0[c] = fix0;
            z.c_nfix[c] = nfix;
            z.c_fixbytes[c] = fixbytes;
            z.c_off[c] = boff;
        }
        boff += fixbytes + spec_bytes;
        ntot += nfix + (nt - first);
        entry = next;
    }
    if (lane == 0) {
        z.lz_size[b] = boff;
        z.ntok[b] = ntot;
        z.b_nfix[b] = fi;
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

__device__ inline void write_token(u8* d, const u8* text, u32 pos, u32 len, u32 dist) {
    if (len == 0) {
        d[0] = 0;
        d[1] = text[pos];
    } else {
        d[0] = 1;
        const u32 n1 = put_uleb(d + 1, len);
        put_uleb(d + 1 + n1, dist);
    }
}

// One thread per token slot g: speculative token (slot in its chunk) and fix-up token.
__global__ __launch_bounds__(256) void k_lz_emit(LzArgs z, const u32* method, const u64* off, u8* arena,
                                                 int force_all) {
    const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= z.geo.N) return;
    const u32 b = z.geo.block_of(g);
    if (!force_all && method[b] != 7u) return;
    const u32 base = z.geo.base(b);
    u8* dst = arena + off[b];
    const u32 k = (g - base) / LZ_CHUNK;
    const u32 c = b * z.cpb + k;
    const u32 s = base + k * LZ_CHUNK;
    const u32 i = g - s;
    const u32 first = z.c_first[c];
    if (i >= first && i < z.c_ntok[c]) {
        const u32 o = z.c_off[c] + z.c_fixbytes[c] + (z.tok_off[g] - z.tok_off[s + first]);
        write_token(dst + o, z.text, z.tok_pos[g], z.tok_len[g], z.tok_dist[g]);
    }
    if (g - base < z.b_nfix[b]) write_token(dst + z.fix_off[g], z.text, z.fix_pos[g], z.fix_len[g], z.fix_dist[g]);
}

}  // namespace

void launch_lz_match(const LzArgs& z, hipStream_t s) {
    if (!z.geo.N) return;
    k_lz_match<<<(u32)((z.geo.N + 255) / 256), 256, 0, s>>>(z);
}

void launch_lz_parse(const LzArgs& z, hipStream_t s) {
    if (!z.geo.nb) return;
    const u32 nchunks = z.cpb * z.geo.nb;
    k_lz_spec<<<(nchunks + 3) / 4, 256, 0, s>>>(z, nchunks);
    k_lz_stitch<<<z.geo.nb, 64, 0, s>>>(z);
}

void launch_lz_emit(const LzArgs& z, const u32* method, const u64* off, u8* arena, hipStream_t s) {
    if (!z.geo.N) return;
    k_lz_emit<<<(u32)((z.geo.N + 255) / 256), 256, 0, s>>>(z, method, off, arena, method == nullptr ? 1 : 0);
}

}  // namespace kolm
