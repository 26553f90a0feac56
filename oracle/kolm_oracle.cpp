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
#include <cmath>
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

// ---------------------------------------------------------------------------------
// v2_new (candidate 10): encode_new_pipeline PY:1498-1576 with the automaton evaluated
// serially (circuit_map_automaton_forward(parallel=False), PY:1013-1054; as shipped, PY
// calls it with parallel=True and raises NameError, SURVEY §0.3, so PY itself never
// emits id 10 — this is the pipeline's defined result).
// ---------------------------------------------------------------------------------
// gates on bytes (PY:550-626): xor/or/not reduce to the plain bit operations
inline u8 gray8(u8 v) { return (u8)(v ^ (v >> 1)); }                       // PY:596
inline u8 maj3(u8 a, u8 b, u8 c) { return (u8)((a & b) | (a & c) | (b & c)); }  // PY:599-604
inline u8 mux8(u8 m, u8 a, u8 b) { return (u8)((a & m) | (b & (u8)~m)); }       // PY:592-594
inline u8 dilate1(u8 x) { return (u8)((((x << 1) & 0xFE) | x) | (((x >> 1) & 0x7F) | x)); }  // PY:608-615
inline u8 erode1(u8 x) { return (u8)(~dilate1((u8)~x) & 0xFF); }                 // PY:617-618
inline u8 edge1(u8 x) { return (u8)(dilate1(x) ^ erode1(x)); }                   // PY:626-627
inline u8 nib_hi_eq(u8 a, u8 b) { return ((a ^ b) & 0xF0) ? 0x00 : 0xF0; }      // PY:754-767
inline u8 nib_lo_eq(u8 a, u8 b) { return ((a ^ b) & 0x0F) ? 0x00 : 0x0F; }      // PY:769-778

// predictor of byte i from the raw bytes before it (every model is out[i] = raw[i] ^ pred)
inline u8 v2_pred(int code, int param, const u8* r, int64_t i) {
    switch (code) {
        case 1:  // Delta-k PY:664-690
            return i < param ? 0 : r[i - param];
        case 2: {  // Gray family PY:698-752
            if (i == 0) return 0;
            if (i == 1) return r[0];
            const u8 p1 = r[i - 1], p2 = r[i - 2];
            switch (param & 3) {
                case 0: return gray8(p1);
                case 1: return gray8(p2);
                case 2: return gray8((u8)(p1 ^ p2));
                default: return gray8((u8)(p1 | p2));
            }
        }
        case 3: {  // Nibble-MUX interleave PY:780-826
            if (i == 0) return 0;
            if (i == 1) return r[0];
            const u8 a = r[i - 1], b = r[i - 2];
            const u8 cross = (u8)((a & 0xF0) | (b & 0x0F));
            const u8 sel = (u8)((((u8)~nib_hi_eq(a, b)) & 0xF0) | (((u8)~nib_lo_eq(a, b)) & 0x0F));
            return mux8(sel, cross, a);
        }
        case 4:  // Majority-of-3 PY:828-866
            if (i == 0) return 0;
            if (i < 3) return r[i - 1];
            return maj3(r[i - 1], r[i - 2], r[i - 3]);
        case 5: {  // Morpho-Predict PY:868-900 (param 0: close1, 1: open1)
            if (i == 0) return 0;
            const u8 d = r[i - 1];
            const u8 m = (param & 1) == 0 ? erode1(dilate1(d)) : dilate1(erode1(d));
            return mux8(edge1(d), m, d);
        }
        default:
            return 0;
    }
}

Bytes v2_forward(const u8* r, int64_t n, int code, int param) {
    Bytes out(n);
    for (int64_t i = 0; i < n; ++i) out[i] = (u8)(r[i] ^ v2_pred(code, param, r, i));
    return out;
}

// PY:631-643 zero_order_entropy_bits_per_byte (same summation order, C log2 as CPython)
double h0_bits(const Bytes& d) {
    if (d.empty()) return 0.0;
    int64_t f[256] = {0};
    for (u8 v : d) f[v]++;
    const double n = (double)d.size();
    double H = 0.0;
    for (int i = 0; i < 256; ++i)
        if (f[i]) {
            const double p = (double)f[i] / n;
            H -= p * std::log2(p);
        }
    return H;
}

// PY:1013-1054 (parallel=False) + PY:936-1011: candidates in `kinds` order, folded by
// _pick_better (H0 lower by more than 1e-12 wins; within 1e-12 the smaller (code, param))
void v2_automaton(const u8* r, int64_t n, int& code, int& param, Bytes& mapped) {
    static const int K[13][2] = {{0, 0}, {1, 1}, {1, 2}, {1, 3}, {1, 4}, {2, 0}, {2, 1},
                                 {2, 2}, {2, 3}, {3, 0}, {4, 0}, {5, 0}, {5, 1}};
    double bh = 0;
    for (int c = 0; c < 13; ++c) {
        Bytes y = v2_forward(r, n, K[c][0], K[c][1]);
        if (K[c][0] == 0) y.assign(r, r + n);
        const double h = h0_bits(y);
        bool take = c == 0;
        if (!take) {
            if (h < bh - 1e-12) take = true;
            else if (std::fabs(h - bh) <= 1e-12 &&
                     (K[c][0] < code || (K[c][0] == code && K[c][1] < param))) take = true;
        }
        if (take) { bh = h; code = K[c][0]; param = K[c][1]; mapped.swap(y); }
    }
}

// PY:1413-1421 rice_encode over arbitrary non-negative integers
Bytes rice_encode_u(const std::vector<uint64_t>& seq, int k) {
    BitWriter bw;
    for (uint64_t v : seq) {
        const uint64_t q = v >> k, r = v & ((1ull << k) - 1);
        for (uint64_t i = 0; i < q; ++i) bw.bit(1);
        bw.bit(0);
        for (int i = k - 1; i >= 0; --i) bw.bit((int)((r >> i) & 1));
    }
    bw.pad();
    return bw.buf;
}

Bytes encode_new_pipeline(const u8* blk, int64_t n) {
    if (n == 0) return Bytes();
    int code = 0, param = 0;
    Bytes mapped;
    v2_automaton(blk, n, code, param, mapped);
    const uint32_t mp = (uint32_t)param;
    const int plen = mp == 0 ? 0 : mp <= 0xFF ? 1 : mp <= 0xFFFF ? 2 : mp <= 0xFFFFFF ? 3 : 4;
    int raw_mask = 0, b1_mask = 0;
    std::vector<int> ks;
    Bytes payload;
    for (int j = 0; j < 8; ++j) {
        Bytes U(n);
        for (int64_t t = 0; t < n; ++t) U[t] = (mapped[t] >> (7 - j)) & 1;  // PY:1137-1155
        Bytes raw((n + 7) / 8, 0);                                           // PY:1191-1195
        for (int64_t t = 0; t < n; ++t) if (U[t]) raw[t >> 3] |= (u8)(1 << (7 - (t & 7)));
        Bytes L = bbwt_forward(U.data(), n);
        std::vector<uint64_t> runs;                                          // PY:1177-1183
        uint64_t cur = 1;
        for (int64_t i = 1; i < n; ++i) {
            if (L[i] == L[i - 1]) ++cur;
            else { runs.push_back(cur); cur = 1; }
        }
        runs.push_back(cur);
        int bk = 0;
        Bytes best;
        for (int k = 0; k < 16; ++k) {                                       // PY:1489-1496
            Bytes b = rice_encode_u(runs, k);
            if (k == 0 || b.size() < best.size()) { bk = k; best.swap(b); }
        }
        if (raw.size() <= best.size() + 1) {
            raw_mask |= 1 << j;
            payload.insert(payload.end(), raw.begin(), raw.end());
        } else {
            if (L[0] & 1) b1_mask |= 1 << j;
            ks.push_back(bk & 0xFF);
            payload.insert(payload.end(), best.begin(), best.end());
        }
    }
    Bytes out;
    out.push_back((u8)(((code & 7) << 5) | (plen & 7)));
    for (int i = 0; i < plen; ++i) out.push_back((u8)((mp >> (8 * i)) & 0xFF));
    out.push_back((u8)raw_mask);
    out.push_back((u8)b1_mask);
    for (int k : ks) out.push_back((u8)k);
    out.insert(out.end(), payload.begin(), payload.end());
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

// v2_new automaton choice: (code, param) of the winning transform, and its H0
int64_t oracle_v2_automaton(const uint8_t* s, int64_t n, int32_t* code_param, double* h0) {
    int code = 0, param = 0;
    Bytes mapped;
    v2_automaton(s, n, code, param, mapped);
    code_param[0] = code;
    code_param[1] = param;
    if (h0) *h0 = h0_bits(mapped);
    return 0;
}

// Candidate payload of method id `mid` (PY:2152-2178 order, ids 0..10).
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
        case 10: return emit(encode_new_pipeline(s, n), out, cap);  // serial automaton (see above)
        default: return -2;
    }
}

}  // extern "C"
