// kolm_toc.cpp — the KOLR container's header and table of contents, host side (C ABI:
// kolm_toc_write / kolm_toc_read, include/kolm.h).  No device code: the container is a
// few hundred bytes of metadata per batch, written once after the per-block MDL winners
// are known (PY = final_researched/kolm_final_researched_v2-2.py).
//
// Byte format (PY:2332-2445 fixed mode, PY:2213-2326 CDC mode, PY:2451-2550 reader):
//   "KOLR" | u32le mode<<31 | size | u32le total_len | u16le nblocks
//   ULEB hdr_len | ULEB toc_bits | ULEB payload_bytes
//   hdr:  ULEB n_runs, ULEB K, K x (ULEB method, ULEB code_len) ordered by (code_len,
//         method), ULEB k_runs, then FIXED: ULEB len(last block) / CDC: ULEB k_lens
//   bits (MSB first): canonical prefix code of each run's method id; Rice(k_runs) of the
//         run lengths; CDC: Rice(k_lens) of zigzag(len - avg); Elias-Fano of the payload
//         end offsets (the low bits of every offset first, then the unary high part).
//
// The prefix-code lengths follow the reference's construction, whose only subtle part
// is how equal-weight entries are ordered: the reference pops its entries from Python's
// heapq (CPython Lib/heapq.py, the pinned interpreter 3.10: heapify = _siftup from the
// last parent down, heappop = move the last leaf to the root + _siftup, heappush =
// append + _siftdown, where _siftup walks the smaller child down to a leaf and then sifts
// back up), ordering entries by (weight, method id) with merged entries ranked as id -1
// (PY:1267-1276).  Merged entries of equal weight compare equal, so which of them leaves
// the heap first depends on the heap's array layout: this file keeps the same array-heap
// discipline (HeapQ below) so those ties resolve identically.  Depths come from the
// parent links of the finished merge tree.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kolm.h"
#include "kolm_internal.h"

using kolm::set_err;
using kolm::u32;
using kolm::u64;
using kolm::u8;

namespace {

// ---- byte / bit output ---------------------------------------------------------------
void put_uleb(std::vector<u8>& o, u64 v) {
    do {
        u8 b = v & 0x7F;
        v >>= 7;
        o.push_back(v ? (u8)(b | 0x80) : b);
    } while (v);
}

struct BitOut {
    std::vector<u8> bytes;
    u64 nbits = 0;
    void bit(u32 b) {
        if ((nbits & 7) == 0) bytes.push_back(0);
        if (b) bytes.back() |= (u8)(0x80u >> (nbits & 7));
        ++nbits;
    }
    void field(u64 v, u32 k) {  // k bits of v, most significant first
        for (u32 i = k; i-- > 0;) bit((u32)(v >> i) & 1u);
    }
    void rice(u64 v, u32 k) {  // unary (v >> k) ones, a zero, then the k low bits
        for (u64 q = v >> k; q; --q) bit(1);
        bit(0);
        field(v & ((1ull << k) - 1), k);
    }
};

u64 rice_cost(const std::vector<u64>& v, u32 k) {
    u64 bits = 0;
    for (u64 x : v) bits += (x >> k) + 1 + k;
    return bits;
}

// smallest k in 0..7 with the fewest bits (PY:2399-2404: strict '<' from k = 0)
u32 best_rice_k(const std::vector<u64>& v) {
    u32 best = 0;
    u64 bb = ~0ull;
    for (u32 k = 0; k < 8; ++k) {
        const u64 b = rice_cost(v, k);
        if (b < bb) bb = b, best = k;
    }
    return best;
}

// Elias-Fano low-bit width: floor(log2(U / n)) when U / n > 1 (PY:1352-1357 takes the
// float log2 of an integer quotient < 2^32, which this integer form equals exactly)
u32 ef_low_bits(u64 U, u64 n) {
    if (n == 0 || U <= 1) return 0;
    const u64 q = U / n;
    if (q <= 1) return 0;
    return 63 - (u32)__builtin_clzll(q);
}

u64 zigzag(int64_t x) { return x >= 0 ? (u64)x << 1 : (((u64)(-x)) << 1) - 1; }
int64_t unzigzag(u64 z) { return (z & 1) ? -(int64_t)((z + 1) >> 1) : (int64_t)(z >> 1); }

// ---- the merge heap --------------------------------------------------------------------
struct HeapQ {
    struct Ent {
        u64 w;
        int64_t id;  // method id of a leaf, -1 for a merged entry
    };
    std::vector<Ent> ent;  // all entries ever created (leaves first)
    std::vector<int> a;    // the heap array (indices into ent)
    bool lt(int x, int y) const {
        const Ent &p = ent[x], &q = ent[y];
        return p.w != q.w ? p.w < q.w : p.id < q.id;
    }
    void sift_toward_root(size_t lo, size_t pos) {
        const int item = a[pos];
        while (pos > lo) {
            const size_t up = (pos - 1) >> 1;
            if (!lt(item, a[up])) break;
            a[pos] = a[up];
            pos = up;
        }
        a[pos] = item;
    }
    void sift_to_leaf(size_t pos) {
        const size_t n = a.size(), lo = pos;
        const int item = a[pos];
        for (size_t ch = 2 * pos + 1; ch < n; ch = 2 * pos + 1) {
            if (ch + 1 < n && !lt(a[ch], a[ch + 1])) ++ch;
            a[pos] = a[ch];
            pos = ch;
        }
        a[pos] = item;
        sift_toward_root(lo, pos);
    }
    void build() {
        for (size_t i = a.size() / 2; i-- > 0;) sift_to_leaf(i);
    }
    int pop() {
        const int last = a.back();
        a.pop_back();
        if (a.empty()) return last;
        const int top = a[0];
        a[0] = last;
        sift_to_leaf(0);
        return top;
    }
    void push(int e) {
        a.push_back(e);
        sift_toward_root(0, a.size() - 1);
    }
};

struct Code {
    u64 sym;
    u32 len;
    u64 bits;
};

// prefix-code lengths for the run symbols, leaves in first-appearance order (PY's
// Counter insertion order), weights = run counts per symbol (PY:1278-1300, 2385-2388)
std::vector<Code> code_lengths(const std::vector<u64>& syms_in_order, const std::vector<u64>& counts) {
    const size_t k = syms_in_order.size();
    std::vector<Code> out;
    if (k == 0) return out;
    if (k == 1) return {Code{syms_in_order[0], 1, 0}};
    HeapQ h;
    std::vector<int> parent;
    for (size_t i = 0; i < k; ++i) {
        h.ent.push_back({std::max<u64>(1, counts[i]), (int64_t)syms_in_order[i]});
        h.a.push_back((int)i);
        parent.push_back(-1);
    }
    h.build();
    while (h.a.size() > 1) {
        const int x = h.pop(), y = h.pop();
        const int m = (int)h.ent.size();
        h.ent.push_back({h.ent[x].w + h.ent[y].w, -1});
        parent.push_back(-1);
        parent[x] = parent[y] = m;
        h.push(m);
    }
    for (size_t i = 0; i < k; ++i) {
        u32 d = 0;
        for (int p = parent[i]; p >= 0; p = parent[p]) ++d;
        out.push_back(Code{syms_in_order[i], std::max<u32>(1, d), 0});
    }
    return out;
}

// canonical numbering in (length, symbol) order (PY:1302-1311)
void canonical(std::vector<Code>& c) {
    std::sort(c.begin(), c.end(), [](const Code& x, const Code& y) {
        return x.len != y.len ? x.len < y.len : x.sym < y.sym;
    });
    u64 code = 0;
    u32 prev = 0;
    for (Code& e : c) {
        if (e.len != prev) code <<= (e.len - prev), prev = e.len;
        e.bits = code++;
    }
}

// ---- byte / bit input -----------------------------------------------------------------
struct Fail {
    std::string msg;
};

struct ByteIn {
    const u8* p;
    u64 n, pos = 0;
    u64 uleb() {
        u64 v = 0;
        for (u32 sh = 0;; sh += 7) {
            if (pos >= n) throw Fail{"Truncated ULEB128"};
            const u8 b = p[pos++];
            if (sh >= 64 || (sh == 63 && (b & 0x7E))) throw Fail{"ULEB128 value out of range"};
            v |= (u64)(b & 0x7F) << sh;
            if (!(b & 0x80)) return v;
        }
    }
};

struct BitIn {
    const u8* p;
    u64 nbytes, at = 0;
    u32 bit() {
        if ((at >> 3) >= nbytes) throw Fail{"BitReader: out of data"};
        const u32 v = (p[at >> 3] >> (7 - (at & 7))) & 1u;
        ++at;
        return v;
    }
    u64 field(u32 k) {
        u64 v = 0;
        while (k--) v = (v << 1) | bit();
        return v;
    }
    u64 rice(u32 k) {
        u64 q = 0;
        while (bit()) ++q;
        return (q << k) | field(k);
    }
};

}  // namespace

extern "C" {

int kolm_toc_write(int mode, uint32_t size_field, uint64_t total_len, uint32_t nblocks, const uint32_t* methods,
                   const uint32_t* orig_lens, const uint64_t* payload_lens, uint8_t* out, uint64_t cap,
                   uint64_t* out_len) {
    if ((mode != 0 && mode != 1) || size_field > 0x7FFFFFFFu || !out_len ||
        (nblocks && (!methods || !orig_lens || !payload_lens))) {
        set_err("kolm_toc_write: bad argument");
        return KOLM_EARG;
    }
    if (total_len > 0xFFFFFFFFull || nblocks > 0xFFFFu) {  // PY: struct.pack '<I' / '<H'
        set_err(nblocks > 0xFFFFu ? "'H' format requires 0 <= number <= 65535"
                                  : "'I' format requires 0 <= number <= 4294967295");
        return KOLM_ERANGE;
    }
    // runs of equal method ids and their symbols' first-appearance order
    std::vector<u64> run_sym, run_len, order, count;
    for (u32 i = 0; i < nblocks; ++i) {
        if (i && methods[i] == run_sym.back()) {
            ++run_len.back();
            continue;
        }
        run_sym.push_back(methods[i]);
        run_len.push_back(1);
        size_t j = 0;
        while (j < order.size() && order[j] != methods[i]) ++j;
        if (j == order.size()) order.push_back(methods[i]), count.push_back(0);
        ++count[j];
    }
    std::vector<Code> codes = code_lengths(order, count);
    canonical(codes);
    const u32 k_runs = best_rice_k(run_len);
    std::vector<u64> deltas;
    u32 k_lens = 0;
    if (mode == 1) {
        for (u32 i = 0; i < nblocks; ++i) deltas.push_back(zigzag((int64_t)orig_lens[i] - (int64_t)size_field));
        k_lens = best_rice_k(deltas);
    }
    std::vector<u8> hdr;
    put_uleb(hdr, run_sym.size());
    put_uleb(hdr, codes.size());
    for (const Code& c : codes) put_uleb(hdr, c.sym), put_uleb(hdr, c.len);
    put_uleb(hdr, k_runs);
    put_uleb(hdr, mode == 0 ? (nblocks ? orig_lens[nblocks - 1] : 0) : k_lens);

    BitOut bo;
    for (u64 s : run_sym)
        for (const Code& c : codes)
            if (c.sym == s) {
                bo.field(c.bits, c.len);
                break;
            }
    for (u64 r : run_len) bo.rice(r, k_runs);
    for (u64 d : deltas) bo.rice(d, k_lens);
    u64 U = 0;
    for (u32 i = 0; i < nblocks; ++i) U += payload_lens[i];
    const u32 l = ef_low_bits(U, nblocks);
    u64 end = 0;
    for (u32 i = 0; i < nblocks; ++i) end += payload_lens[i], bo.field(end & ((1ull << l) - 1), l);
    // high part: m + n bits, a one at (end_i >> l) + i for every block
    const u64 m = (U + ((1ull << l) - 1)) >> l;
    u64 next = 0;
    end = 0;
    for (u32 i = 0; i < nblocks; ++i) {
        end += payload_lens[i];
        const u64 one = (end >> l) + i;
        for (; next < one; ++next) bo.bit(0);
        bo.bit(1);
        ++next;
    }
    for (; next < m + nblocks; ++next) bo.bit(0);

    std::vector<u8> o;
    o.insert(o.end(), {'K', 'O', 'L', 'R'});
    const u32 packed = ((u32)mode << 31) | size_field;
    for (int i = 0; i < 4; ++i) o.push_back((u8)(packed >> (8 * i)));
    for (int i = 0; i < 4; ++i) o.push_back((u8)(total_len >> (8 * i)));
    o.push_back((u8)nblocks);
    o.push_back((u8)(nblocks >> 8));
    put_uleb(o, hdr.size());
    put_uleb(o, bo.nbits);
    put_uleb(o, U);
    o.insert(o.end(), hdr.begin(), hdr.end());
    o.insert(o.end(), bo.bytes.begin(), bo.bytes.end());
    *out_len = o.size();
    if (!out) return KOLM_OK;
    if (cap < o.size()) {
        set_err("kolm_toc_write: output capacity too small");
        return KOLM_ECAP;
    }
    std::memcpy(out, o.data(), o.size());
    return KOLM_OK;
}

int kolm_toc_read(const uint8_t* buf, uint64_t n, uint32_t* fields, uint64_t* payload_start, uint32_t* methods,
                  uint32_t* orig_lens, uint64_t* payload_off, uint32_t cap) {
    if ((!buf && n) || !fields || !payload_start) {
        set_err("kolm_toc_read: bad argument");
        return KOLM_EARG;
    }
    try {
        if (n < 4 || std::memcmp(buf, "KOLR", 4) != 0) throw Fail{"Invalid magic"};
        if (n < 14) throw Fail{"Truncated container header"};
        auto le = [&](u64 at, int k) {
            u64 v = 0;
            for (int i = 0; i < k; ++i) v |= (u64)buf[at + i] << (8 * i);
            return v;
        };
        const u32 packed = (u32)le(4, 4);
        const u32 mode = packed >> 31, size_field = packed & 0x7FFFFFFFu, total_len = (u32)le(8, 4);
        const u32 nb = (u32)le(12, 2);
        fields[0] = mode, fields[1] = size_field, fields[2] = total_len, fields[3] = nb;
        ByteIn bi{buf, n, 14};
        const u64 hdr_len = bi.uleb(), toc_bits = bi.uleb(), U = bi.uleb();
        if (hdr_len > n - bi.pos) throw Fail{"Truncated TOC header"};
        ByteIn hd{buf + bi.pos, hdr_len};
        const u64 bits_at = bi.pos + hdr_len;
        const u64 bit_bytes = (toc_bits + 7) / 8;
        if (toc_bits > 8 * (n - bits_at) || bit_bytes > n - bits_at) throw Fail{"Truncated TOC bits"};
        const u64 pay_at = bits_at + bit_bytes;
        *payload_start = pay_at;
        if (cap < nb) {
            set_err("kolm_toc_read: arrays hold fewer entries than the block count");
            return KOLM_ECAP;
        }
        const u64 n_runs = hd.uleb(), K = hd.uleb();
        // PY keeps the code lengths as read, of any size, and numbers the codes with Python
        // integers (PY:1302-1311, 1318-1329).  Lengths here are u64 and the code values are
        // never formed: decoding tracks d = (bits read so far) - (first code of that length),
        // below.  A repeated symbol keeps its last length (dict semantics).
        struct LCode {
            u64 sym, len;
        };
        std::vector<LCode> codes;
        std::unordered_map<u64, size_t> at;
        for (u64 i = 0; i < K; ++i) {
            const u64 sym = hd.uleb(), len = hd.uleb();
            const auto it = at.find(sym);
            if (it != at.end()) {
                codes[it->second].len = len;
            } else {
                at.emplace(sym, codes.size());
                codes.push_back(LCode{sym, len});
            }
        }
        const u64 k_runs = hd.uleb();
        const u64 tail = hd.uleb();  // FIXED: last block's length; CDC: k of the length deltas
        if (k_runs > 63 || (mode == 1 && tail > 63)) throw Fail{"Rice parameter out of range"};
        // canonical order (length, symbol), as PY's numbering walks it
        std::sort(codes.begin(), codes.end(), [](const LCode& x, const LCode& y) {
            return x.len != y.len ? x.len < y.len : x.sym < y.sym;
        });
        // lengths present: (L, count, index of the first code of length L); length-0 symbols
        // take code numbers too (PY's counter runs over them) but never decode (PY reads from
        // length 1 on)
        struct Lvl {
            u64 len, cnt, idx;
        };
        std::vector<Lvl> lv;
        for (size_t i = 0; i < codes.size(); ++i) {
            if (lv.empty() || lv.back().len != codes[i].len) lv.push_back(Lvl{codes[i].len, 0, i});
            ++lv.back().cnt;
        }
        const u64 maxlen = lv.empty() ? 0 : lv.back().len;
        // PY numbers length L's codes nc_L .. nc_L + cnt_L - 1 with nc_(L+1) = 2 (nc_L + cnt_L)
        // (over every L, cnt_L = 0 where no code has length L).  After reading L bits, value v_L,
        // d_L = v_L - nc_L obeys d_(L+1) = 2 (d_L - cnt_L) + bit and a symbol decodes at the first
        // L with 0 <= d_L < cnt_L.  Once d_L < 0 it stays negative; once d_L >= 2^40 (> 2 cnt_L)
        // it only grows: no later length can match, and PY reads on to maxlen and fails.
        BitIn br{buf + bits_at, bit_bytes};
        std::vector<u64> syms;
        const int64_t DBIG = (int64_t)1 << 40;
        for (u64 r = 0; r < n_runs; ++r) {
            int64_t d = 0;
            u64 cntL = 0;  // cnt of the previous length
            size_t li = 0;
            bool hit = false;
            if (!lv.empty() && lv[0].len == 0) cntL = lv[0].cnt, li = 1;  // length 0 precedes length 1
            for (u64 L = 1; L <= maxlen; ++L) {
                d = 2 * (d - (int64_t)cntL) + (int64_t)br.bit();
                cntL = 0;
                if (li < lv.size() && lv[li].len == L) {
                    cntL = lv[li].cnt;
                    if (d >= 0 && (u64)d < cntL) {
                        syms.push_back(codes[lv[li].idx + (u64)d].sym);
                        hit = true;
                        break;
                    }
                    ++li;
                }
                if (d < 0 || d >= DBIG) {
                    // PY reads the rest of maxlen bits, then fails (or runs out of bits first)
                    const u64 left = maxlen - L;
                    if (left > 8 * (bit_bytes - (br.at >> 3))) throw Fail{"BitReader: out of data"};
                    break;
                }
            }
            if (!hit) throw Fail{"Huffman decode failed"};
        }
        u64 filled = 0;
        for (u64 r = 0; r < n_runs; ++r) {
            const u64 len = br.rice((u32)k_runs);
            if (len > nb - filled) throw Fail{"Method id RLE expands to wrong size"};
            if (syms[r] > 0xFFFFFFFFull) throw Fail{"Unknown method_id " + std::to_string(syms[r])};
            for (u64 j = 0; j < len; ++j) methods[filled++] = (u32)syms[r];
        }
        if (filled != nb) throw Fail{"Method id RLE expands to wrong size"};
        for (u32 i = 0; i < nb; ++i) {
            if (mode == 0) {
                orig_lens[i] = i + 1 < nb ? size_field : (u32)tail;
            } else {
                const int64_t v = (int64_t)size_field + unzigzag(br.rice((u32)tail));
                if (v < 0 || v > 0xFFFFFFFFll) throw Fail{"block length out of range"};
                orig_lens[i] = (u32)v;
            }
        }
        const u32 l = ef_low_bits(U, nb);
        payload_off[0] = 0;
        for (u32 i = 0; i < nb; ++i) payload_off[i + 1] = br.field(l);
        const u64 m = (U + ((1ull << l) - 1)) >> l;
        u32 ones = 0;
        for (u64 idx = 0; idx < m + nb && ones < nb; ++idx)
            if (br.bit()) {
                payload_off[ones + 1] |= (idx - ones) << l;
                ++ones;
            }
        if (ones < nb) throw Fail{"Elias-Fano positions truncated"};
        if (nb && payload_off[nb] != U) throw Fail{"Payload EF sum mismatch"};
        for (u32 i = 0; i < nb; ++i)
            if (payload_off[i + 1] < payload_off[i]) throw Fail{"payload ends decrease"};
        if (U > n - pay_at) throw Fail{"Truncated payload area"};
        if (pay_at + U != n) throw Fail{"Extra trailing " + std::to_string(n - pay_at - U) + " bytes after container end"};
        return KOLM_OK;
    } catch (const Fail& f) {
        set_err(f.msg);
        return KOLM_EFORMAT;
    } catch (const std::bad_alloc&) {
        set_err("host allocation failed");
        return KOLM_EHIP;
    }
}

}  // extern "C"
