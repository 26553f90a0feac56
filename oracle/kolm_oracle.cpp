// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the
// product path (kolmogorovlike-datacompressor_amd/).  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may use it, as the checker / CPU baseline.
//
// A faithful CPU restatement of the reference's block-transform hot path,
// kolm_final_researched_v2-2.py ("PY"), with the SAME algorithms as the reference
// (comparison-sort prefix doubling per Lyndon factor, k-way heap merge under the
// omega-order, list MTF, bit-serial Rice, exhaustive 4096-window LZ77, O(n*rules)
// Re-Pair), so that it doubles as the "reference CPU path" baseline.
// Every function cites the PY lines it restates.  Parity is pinned by
// tests/golden/ (fixtures produced by importing PY itself) and by the known-answer
// FNV-1a-64 hashes of SURVEY.md §8c (tests/test_oracle.py).
//
// C ABI (ctypes): all outputs caller-allocated; functions return the number of bytes
// written, or -1 when the capacity is too small.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

using u8 = uint8_t;
using Bytes = std::vector<u8>;

// PY:111-124 uleb128_encode
inline void uleb(Bytes& out, uint64_t v) {
    for (;;) {
        u8 b = v & 0x7F;
        v >>= 7;
        if (v) {
            out.push_back(b | 0x80);
        } else {
            out.push_back(b);
            return;
        }
    }
}

// PY:326-349 duval_lyndon
std::vector<std::pair<int64_t, int64_t>> duval(const u8* s, int64_t n) {
    std::vector<std::pair<int64_t, int64_t>> out;
    int64_t i = 0;
    while (i < n) {
        int64_t j = i + 1, k = i;
        while (j < n && s[k] <= s[j]) {
            if (s[k] < s[j]) k = i; else ++k;
            ++j;
        }
        int64_t p = j - k;
        while (i <= k) {
            out.emplace_back(i, i + p);
            i += p;
        }
    }
    return out;
}

// PY:362-378 sa_prefix_doubling (comparison sort of (rank[i], rank[i+k] or -1))
std::vector<int64_t> sa_prefix_doubling(const Bytes& t) {
    const int64_t n = (int64_t)t.size();
    std::vector<int64_t> rank(t.begin(), t.end()), tmp(n), idx(n);
    for (int64_t i = 0; i < n; ++i) idx[i] = i;
    int64_t k = 1;
    for (;;) {
        auto key2 = [&](int64_t i) { return i + k < n ? rank[i + k] : (int64_t)-1; };
        std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
            if (rank[a] != rank[b]) return rank[a] < rank[b];
            return key2(a) < key2(b);
        });
        tmp[idx[0]] = 0;
        for (int64_t j = 1; j < n; ++j) {
            int64_t a = idx[j - 1], b = idx[j];
            bool lt = rank[a] < rank[b] || (rank[a] == rank[b] && key2(a) < key2(b));
            tmp[b] = tmp[a] + (lt ? 1 : 0);
        }
        std::swap(rank, tmp);
        if (rank[idx[n - 1]] == n - 1) break;
        k <<= 1;
    }
    return idx;
}

// PY:351-423 bbwt_forward (per-factor rotation sort + heap merge, ties (fi, i))
Bytes bbwt_forward(const u8* s, int64_t n) {
    Bytes out;
    if (n == 0) return out;
    auto facs = duval(s, n);
    struct Fac { const u8* w; int64_t m; std::vector<int64_t> order; };
    std::vector<Fac> F;
    F.reserve(facs.size());
    for (auto& ab : facs) {
        int64_t m = ab.second - ab.first;
        Bytes ww(2 * m);
        std::memcpy(ww.data(), s + ab.first, m);
        std::memcpy(ww.data() + m, s + ab.first, m);
        auto sa = sa_prefix_doubling(ww);
        Fac f{s + ab.first, m, {}};
        f.order.reserve(m);
        for (int64_t p : sa) if (p < m) f.order.push_back(p);
        F.push_back(std::move(f));
    }
    struct Node { int64_t fi, k; };
    // Node.__lt__ (PY:395-409): compare u[i:]+u[:i] vs v[j:]+v[:j] over m+n chars
    auto less = [&](const Node& a, const Node& b) {
        const Fac& A = F[a.fi];
        const Fac& B = F[b.fi];
        int64_t i = A.order[a.k], j = B.order[b.k];
        int64_t m = A.m, nn = B.m;
        int64_t ia = i, jb = j;
        for (int64_t p = 0; p < m + nn; ++p) {
            u8 cu = A.w[ia], cv = B.w[jb];
            if (cu != cv) return cu < cv;
            if (++ia == m) ia = 0;
            if (++jb == nn) jb = 0;
        }
        return a.fi != b.fi ? a.fi < b.fi : i < j;
    };
    auto gt = [&](const Node& a, const Node& b) { return less(b, a); };  // min-heap
    std::vector<Node> heap;
    for (int64_t fi = 0; fi < (int64_t)F.size(); ++fi)
        if (!F[fi].order.empty()) heap.push_back({fi, 0});
    std::make_heap(heap.begin(), heap.end(), gt);
    out.reserve(n);
    while (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end(), gt);
        Node nd = heap.back();
        heap.pop_back();
        const Fac& f = F[nd.fi];
        int64_t i = f.order[nd.k];
        out.push_back(f.w[(i - 1 + f.m) % f.m]);
        nd.k += 1;
        if (nd.k < (int64_t)f.order.size()) {
            heap.push_back(nd);
            std::push_heap(heap.begin(), heap.end(), gt);
        }
    }
    return out;
}

// PY:460-468 mtf_encode (list index/pop/insert)
Bytes mtf_encode(const u8* d, int64_t n) {
    u8 table[256];
    for (int i = 0; i < 256; ++i) table[i] = (u8)i;
    Bytes out(n);
    for (int64_t t = 0; t < n; ++t) {
        u8 b = d[t];
        int idx = 0;
        while (table[idx] != b) ++idx;
        out[t] = (u8)idx;
        std::memmove(table + 1, table, idx);
        table[0] = b;
    }
    return out;
}

// PY:1100-1120 bitplane_interleave (8-byte groups, zero padded)
Bytes bitplane_interleave(const Bytes& d) {
    Bytes out;
    out.reserve((d.size() + 7) / 8 * 8);
    for (size_t g = 0; g < d.size(); g += 8) {
        u8 blk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (size_t i = 0; i < 8 && g + i < d.size(); ++i) blk[i] = d[g + i];
        for (int bit = 0; bit < 8; ++bit) {
            u8 v = 0;
            for (int i = 0; i < 8; ++i) v |= ((blk[i] >> (7 - bit)) & 1) << (7 - i);
            out.push_back(v);
        }
    }
    return out;
}

// PY:1650-1662 nibble_swap / bit_reverse / gray_encode_bytes
u8 bitrev8(u8 b) {
    u8 r = 0;
    for (int i = 0; i < 8; ++i) r |= ((b >> i) & 1) << (7 - i);
    return r;
}

// PY:1231-1254 _BitWriter + PY:1413-1421 rice_encode
struct BitWriter {
    Bytes buf;
    u8 cur = 0;
    int bitpos = 0;
    void bit(int b) {
        cur |= (u8)((b & 1) << (7 - bitpos));
        if (++bitpos == 8) { buf.push_back(cur); cur = 0; bitpos = 0; }
    }
    void pad() { if (bitpos) { buf.push_back(cur); cur = 0; bitpos = 0; } }
};

Bytes rice_encode(const Bytes& seq, int k) {
    BitWriter bw;
    const uint64_t M = 1ull << k;
    for (u8 v : seq) {
        uint64_t q = k > 0 ? v / M : v, r = k > 0 ? v % M : 0;
        for (uint64_t i = 0; i < q; ++i) bw.bit(1);
        bw.bit(0);
        for (int i = k - 1; i >= 0; --i) bw.bit((r >> i) & 1);
    }
    bw.pad();
    return bw.buf;
}

// PY:2028-2073 encode_bbwt_mtf_rice (BBWT recomputed per call, as in the reference)
Bytes encode_bbwt_mtf_rice(const u8* blk, int64_t n, int flags, int k) {
    Bytes b = bbwt_forward(blk, n);
    Bytes seq = mtf_encode(b.data(), (int64_t)b.size());
    if (flags & 1) seq = bitplane_interleave(seq);
    if (flags & 2) {  // lfsr_whiten PY:480-498 (never selected by a candidate)
        u8 state = 1;
        for (auto& x : seq) {
            u8 o = x ^ state;
            int fb = 0;
            for (int bit = 0; bit < 8; ++bit) if ((0x96 >> bit) & 1) fb ^= (state >> bit) & 1;
            state = (u8)(((state << 1) & 0xFF) | fb);
            x = o;
        }
    }
    if (flags & 4) for (auto& x : seq) x = (u8)(((x & 0x0F) << 4) | ((x & 0xF0) >> 4));
    if (flags & 8) for (auto& x : seq) x = bitrev8(x);
    if (flags & 16) for (auto& x : seq) x = (u8)(x ^ (x >> 1));
    return rice_encode(seq, k);
}

// PY:1686-1763 encode_lz77 (exhaustive window search, ties -> smallest distance)
Bytes encode_lz77(const u8* blk, int64_t n) {
    const int64_t WINDOW_MAX = 4096, MIN_MATCH = 3;
    Bytes out;
    int64_t pos = 0;
    while (pos < n) {
        int64_t best_len = 0, best_dist = 0;
        int64_t maxw = std::min(pos, WINDOW_MAX);
        for (int64_t dist = 1; dist <= maxw; ++dist) {
            int64_t m = 0;  // _lz77_match_len_overlap: block[pos+m] vs block[pos+m-dist]
            while (pos + m < n && blk[pos + m - dist] == blk[pos + m]) ++m;
            if (m > best_len) { best_len = m; best_dist = dist; }
        }
        if (best_len >= MIN_MATCH) {
            out.push_back(1);
            uleb(out, (uint64_t)best_len);
            uleb(out, (uint64_t)best_dist);
            pos += best_len;
        } else {
            out.push_back(0);
            out.push_back(blk[pos]);
            pos += 1;
        }
    }
    return out;
}

// PY:2105-2111 encode_xor
Bytes encode_xor(const u8* blk, int64_t n) {
    Bytes out;
    u8 prev = 0;
    for (int64_t i = 0; i < n; ++i) { uleb(out, (u8)(blk[i] - prev)); prev = blk[i]; }
    return out;
}

// PY:1984-2003 encode_lfsr_predict
Bytes encode_lfsr(const u8* blk, int64_t n) {
    Bytes out;
    u8 state = 1;
    for (int64_t i = 0; i < n; ++i) {
        uleb(out, (u8)(blk[i] - state));
        int fb = 0;
        for (int bit = 0; bit < 8; ++bit) if ((0x96 >> bit) & 1) fb ^= (state >> bit) & 1;
        state = (u8)(((state << 1) & 0xFF) | fb);
    }
    return out;
}

// PY:1817-1911 repair_compress (full recount each round, as in the reference)
Bytes repair_compress(const u8* blk, int64_t n) {
    Bytes out{'R', 'P'};
    std::vector<int64_t> seq(blk, blk + n);
    std::vector<std::pair<int64_t, int64_t>> rules;
    int64_t next_sym = 256;
    while (seq.size() >= 2) {
        std::map<std::pair<int64_t, int64_t>, int64_t> freq;  // ordered: ties -> smallest pair
        for (size_t i = 0; i + 1 < seq.size(); ++i) freq[{seq[i], seq[i + 1]}]++;
        std::pair<int64_t, int64_t> best{-1, -1};
        int64_t best_f = 1;
        for (auto& kv : freq)
            if (kv.second > best_f) { best = kv.first; best_f = kv.second; }
        if (best.first < 0 || best_f < 2) break;
        std::vector<int64_t> ns;
        ns.reserve(seq.size());
        int64_t replaced = 0;
        for (size_t i = 0; i < seq.size();) {
            if (i + 1 < seq.size() && seq[i] == best.first && seq[i + 1] == best.second) {
                ns.push_back(next_sym); i += 2; ++replaced;
            } else {
                ns.push_back(seq[i]); i += 1;
            }
        }
        if (replaced < 2) break;
        rules.push_back(best);
        seq.swap(ns);
        ++next_sym;
    }
    uleb(out, 256);
    uleb(out, rules.size());
    for (auto& r : rules) { uleb(out, (uint64_t)r.first); uleb(out, (uint64_t)r.second); }
    uleb(out, seq.size());
    for (int64_t s : seq) uleb(out, (uint64_t)s);
    return out;
}

int64_t emit(const Bytes& b, uint8_t* out, int64_t cap) {
    if ((int64_t)b.size() > cap) return -1;
    if (!b.empty()) std::memcpy(out, b.data(), b.size());
    return (int64_t)b.size();
}

}  // namespace

extern "C" {

int64_t oracle_duval(const uint8_t* s, int64_t n, int64_t* starts, int64_t cap) {
    auto f = duval(s, n);
    if ((int64_t)f.size() > cap) return -1;
    for (size_t i = 0; i < f.size(); ++i) starts[i] = f[i].first;
    return (int64_t)f.size();
}

int64_t oracle_bbwt(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    return emit(bbwt_forward(s, n), out, cap);
}

int64_t oracle_mtf(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    return emit(mtf_encode(s, n), out, cap);
}

int64_t oracle_rice(const uint8_t* s, int64_t n, int k, uint8_t* out, int64_t cap) {
    return emit(rice_encode(Bytes(s, s + n), k), out, cap);
}

int64_t oracle_bbwt_mtf_rice(const uint8_t* s, int64_t n, int flags, int k, uint8_t* out, int64_t cap) {
    return emit(encode_bbwt_mtf_rice(s, n, flags, k), out, cap);
}

int64_t oracle_lz77(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    return emit(encode_lz77(s, n), out, cap);
}

int64_t oracle_xor(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    return emit(encode_xor(s, n), out, cap);
}

int64_t oracle_lfsr(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    return emit(encode_lfsr(s, n), out, cap);
}

int64_t oracle_repair(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    return emit(repair_compress(s, n), out, cap);
}

// Candidate payload of method id `mid` (PY:2152-2178 order, ids 0..9).
int64_t oracle_candidate(int mid, const uint8_t* s, int64_t n, uint8_t* out, int64_t cap) {
    static const int bbwt_flags[5] = {0, 1, 4, 8, 16};
    switch (mid) {
        case 0: return emit(Bytes(s, s + n), out, cap);
        case 1: return oracle_xor(s, n, out, cap);
        case 2: case 3: case 4: case 5: case 6:
            return oracle_bbwt_mtf_rice(s, n, bbwt_flags[mid - 2], 2, out, cap);
        case 7: return oracle_lz77(s, n, out, cap);
        case 8: return oracle_lfsr(s, n, out, cap);
        case 9: return oracle_repair(s, n, out, cap);
        default: return -2;  // v2_new (10) raises in PY
    }
}

}  // extern "C"
