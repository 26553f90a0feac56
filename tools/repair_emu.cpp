// TEST INFRASTRUCTURE ONLY — host emulation of the device Re-Pair (repair_core.h).
// Runs the kernel's phases thread by thread (NT virtual threads, a barrier = the end of a
// loop over threads), so the batch logic can be checked against the oracle on the CPU.
// Never loaded by the product (kolm/ only loads libkolm_hip.so).  Built by
// tests/test_repair_emu.py:  g++ -O2 -shared -fPIC tools/repair_emu.cpp -o <tmp>.so
#define RP_HD
#include "../kolmogorovlike-datacompressor_amd/csrc/repair_core.h"

#include <cstring>
#include <memory>
#include <vector>

using namespace kolm::rp;

namespace {

struct HostExec {
    // order[]: the order in which the virtual threads run a phase (identity, or a
    // permutation per phase when shuffling — exposes phases that depend on thread order)
    u32 order[NT];
    u64 seed = 0;
    template <class F>
    void par(F f) {
        if (seed) {
            for (u32 t = NT - 1; t > 0; --t) {
                seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17;
                const u32 r = (u32)(seed % (t + 1));
                const u32 x = order[t]; order[t] = order[r]; order[r] = x;
            }
        }
        for (u32 t = 0; t < NT; ++t) f(order[t]);
    }
    void scan(u32* a, u32* total) {
        u32 acc = 0;
        for (u32 t = 0; t < NT; ++t) {
            const u32 v = a[t];
            a[t] = acc;
            acc += v;
        }
        *total = acc;
    }
    void scan2(u32* a, u32* b, u32* ta, u32* tb) {
        scan(a, ta);
        scan(b, tb);
    }
    u32 add(u32* p, u32 v) { const u32 o = *p; *p = o + v; return o; }
    u32 sub(u32* p, u32 v) { const u32 o = *p; *p = o - v; return o; }
    u32 min(u32* p, u32 v) { const u32 o = *p; if (v < o) *p = v; return o; }
    u32 max(u32* p, u32 v) { const u32 o = *p; if (v > o) *p = v; return o; }
    u64 cas64(u64* p, u64 cmp, u64 v) { const u64 o = *p; if (o == cmp) *p = v; return o; }
    u32 cas32(u32* p, u32 cmp, u32 v) { const u32 o = *p; if (o == cmp) *p = v; return o; }
    void add_agg(u32* p, bool act, bool) { if (act) ++*p; }
    void sub_agg(u32* p, bool act, bool) { if (act) --*p; }
    u32 slot_agg(u32* p, bool act, bool) { return act ? (*p)++ : 0; }
    u32 leader(u64, bool, bool) { return 0; }
    bool is_leader(u32) const { return true; }
    u32 from_leader(u32 v, u32) const { return v; }
    void mark(u32) {}
    void begin(u32) {}
    void record(const u32 (&f)[8]);
    u32 append(u32* n, bool pred) { return pred ? (*n)++ : NIL; }
};

u64 g_stats[8];  // sums of the batch records: iterations, M, T, nocc, hused, nlate, aa, tot
void HostExec::record(const u32 (&f)[8]) {
    g_stats[0] += 1;
    for (u32 k = 1; k < 8; ++k) g_stats[k] += f[k];
}

}  // namespace

extern "C" void repair_emu_stats(uint64_t* out) {
    for (int k = 0; k < 8; ++k) { out[k] = g_stats[k]; g_stats[k] = 0; }
}

extern "C" int64_t repair_emu(const uint8_t* text, int64_t n64, uint8_t* out, int64_t cap, uint32_t* result,
                              uint64_t shuffle_seed) {
    const u32 n = (u32)n64;
    Block B{};
    const u64 bytes = workspace_layout(nullptr, n, B);
    std::vector<u64> ws(bytes / 8 + 1, 0xA5A5A5A5A5A5A5A5ull);  // garbage: the kernel initialises what it reads
    workspace_layout(reinterpret_cast<char*>(ws.data()), n, B);
    B.text = text;
    B.n = n;
    B.out = out;
    B.out_cap = (u64)cap;
    B.result = result;
    std::unique_ptr<Shared> sh(new Shared);
    HostExec ex;
    for (u32 t = 0; t < NT; ++t) ex.order[t] = t;
    ex.seed = shuffle_seed;
    repair_block(ex, B, *sh);
    if (result[RS_ERR] != RE_OK) return -(int64_t)result[RS_ERR];
    return result[RS_SIZE];
}
