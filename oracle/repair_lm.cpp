// ORACLE — TEST INFRASTRUCTURE ONLY (see kolm_oracle.cpp header).  Never linked into or
// called from the product path.
//
// Exact Re-Pair of the reference (PY:1817-1911 repair_compress) in O(n log n) instead of
// PY's O(n * rules) full recount, so that 1 MiB blocks can be checked in seconds.  The
// selection and replacement rules are the reference's, restated incrementally
// (Larsson & Moffat style pair records with occurrence lists):
//   * freq(a,b) = number of (overlapping) adjacent positions holding a,b   (PY:1817-1822)
//   * chosen pair = max freq, ties -> lexicographically smallest (a,b)     (PY:1868-1876)
//   * stop when freq < 2                                                   (PY:1875-1876)
//   * replacement left to right, non-overlapping                           (PY:1824-1839)
//   * stop (rule not added) when that replaces fewer than 2 occurrences    (PY:1879-1882)
// Counts are kept exact (the count of every pair equals a full recount of the current
// sequence), and a lazy max-heap keyed (freq, -a, -b) replaces the per-round scan.
// tests/test_oracle.py checks it byte for byte against the O(n*rules) restatement and
// against PY's own goldens.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <queue>
#include <unordered_map>
#include <vector>

namespace {

struct Pair {
    int32_t a, b;
    int64_t cnt;
    int32_t head;  // first occurrence position (list through onext/oprev), -1 if none
};

struct HeapEnt {
    int64_t cnt;
    int32_t a, b;
    bool operator<(const HeapEnt& o) const {  // max cnt first, then smallest (a,b)
        if (cnt != o.cnt) return cnt < o.cnt;
        if (a != o.a) return a > o.a;
        return b > o.b;
    }
};

inline void uleb(std::vector<uint8_t>& out, uint64_t v) {
    for (;;) {
        uint8_t b = v & 0x7F;
        v >>= 7;
        if (v) out.push_back(b | 0x80);
        else { out.push_back(b); return; }
    }
}

struct RePair {
    int32_t n;
    std::vector<int32_t> sym, nxt, prv, onext, oprev, opair;
    std::vector<Pair> pairs;
    std::unordered_map<uint64_t, int32_t> index;
    std::priority_queue<HeapEnt> heap;
    std::vector<int32_t> touched;
    std::vector<uint8_t> is_touched;

    static uint64_t key(int32_t a, int32_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

    int32_t pair_id(int32_t a, int32_t b) {
        auto it = index.find(key(a, b));
        if (it != index.end()) return it->second;
        int32_t id = (int32_t)pairs.size();
        pairs.push_back({a, b, 0, -1});
        is_touched.push_back(0);
        index.emplace(key(a, b), id);
        return id;
    }
    void touch(int32_t id) {
        if (!is_touched[id]) { is_touched[id] = 1; touched.push_back(id); }
    }
    void add_occ(int32_t pos) {  // pair starting at live position pos (nxt[pos] live)
        int32_t id = pair_id(sym[pos], sym[nxt[pos]]);
        Pair& p = pairs[id];
        opair[pos] = id;
        oprev[pos] = -1;
        onext[pos] = p.head;
        if (p.head >= 0) oprev[p.head] = pos;
        p.head = pos;
        p.cnt++;
        touch(id);
    }
    void del_occ(int32_t pos) {
        int32_t id = opair[pos];
        if (id < 0) return;
        Pair& p = pairs[id];
        if (oprev[pos] >= 0) onext[oprev[pos]] = onext[pos]; else p.head = onext[pos];
        if (onext[pos] >= 0) oprev[onext[pos]] = oprev[pos];
        opair[pos] = -1;
        p.cnt--;
        touch(id);
    }
    void flush_touched() {
        for (int32_t id : touched) {
            is_touched[id] = 0;
            if (pairs[id].cnt >= 2) heap.push({pairs[id].cnt, pairs[id].a, pairs[id].b});
        }
        touched.clear();
    }

    // returns the grammar; stats (optional): per-round frequency of the chosen pair
    void run(const uint8_t* s, int32_t len, std::vector<std::pair<int32_t, int32_t>>& rules,
             std::vector<int32_t>& final_seq, std::vector<int64_t>* round_freq) {
        n = len;
        sym.assign(s, s + n);
        nxt.resize(n); prv.resize(n); onext.assign(n, -1); oprev.assign(n, -1); opair.assign(n, -1);
        for (int32_t i = 0; i < n; ++i) { nxt[i] = i + 1 < n ? i + 1 : -1; prv[i] = i - 1; }
        for (int32_t i = n - 2; i >= 0; --i) add_occ(i);  // heads end in ascending order
        flush_touched();
        int32_t next_sym = 256;
        std::vector<int32_t> occ;
        while (!heap.empty()) {
            HeapEnt top = heap.top();
            heap.pop();
            auto it = index.find(key(top.a, top.b));
            if (it == index.end() || pairs[it->second].cnt != top.cnt) continue;  // stale
            const int32_t id = it->second;
            const int32_t a = top.a, b = top.b;
            occ.clear();
            for (int32_t q = pairs[id].head; q >= 0; q = onext[q]) occ.push_back(q);
            std::sort(occ.begin(), occ.end());
            int64_t replaced = 0;
            {
                int32_t last_del = -1;
                for (int32_t i : occ) {
                    if (i == last_del) continue;
                    ++replaced;
                    last_del = nxt[i];
                }
            }
            if (replaced < 2) break;  // PY:1879-1882
            if (round_freq) round_freq->push_back(top.cnt);
            const int32_t X = next_sym++;
            rules.push_back({a, b});
            for (int32_t i : occ) {
                if (opair[i] != id) continue;  // consumed by an earlier replacement this round
                const int32_t j = nxt[i];
                const int32_t p = prv[i], q = nxt[j];
                if (p >= 0) del_occ(p);
                if (q >= 0) del_occ(j);
                del_occ(i);
                sym[i] = X;
                nxt[i] = q;
                if (q >= 0) prv[q] = i;
                sym[j] = -1;
                if (p >= 0) add_occ(p);
                if (q >= 0) add_occ(i);
            }
            flush_touched();
        }
        final_seq.clear();
        for (int32_t i = 0; i >= 0 && n > 0; i = nxt[i]) final_seq.push_back(sym[i]);
    }
};

}  // namespace

extern "C" {

// Re-Pair payload (PY:1889-1903 serialisation); returns bytes written or -1 (capacity).
// stats (optional, 4 x int64): nrules, final_len, rounds with freq 2, max freq.
int64_t oracle_repair_fast(const uint8_t* s, int64_t n, uint8_t* out, int64_t cap, int64_t* stats) {
    std::vector<uint8_t> o{'R', 'P'};
    uleb(o, 256);
    std::vector<std::pair<int32_t, int32_t>> rules;
    std::vector<int32_t> seq;
    std::vector<int64_t> rf;
    if (n > 0) {
        RePair rp;
        rp.run(s, (int32_t)n, rules, seq, stats ? &rf : nullptr);
    }
    uleb(o, rules.size());
    for (auto& r : rules) { uleb(o, (uint32_t)r.first); uleb(o, (uint32_t)r.second); }
    uleb(o, seq.size());
    for (int32_t v : seq) uleb(o, (uint32_t)v);
    if (stats) {
        stats[0] = (int64_t)rules.size();
        stats[1] = (int64_t)seq.size();
        stats[2] = std::count(rf.begin(), rf.end(), 2);
        stats[3] = rf.empty() ? 0 : *std::max_element(rf.begin(), rf.end());
    }
    if ((int64_t)o.size() > cap) return -1;
    std::memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

}  // extern "C"
