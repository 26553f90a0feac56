// Exact Re-Pair of one block by one workgroup (candidate 9, PY:1817-1911 repair_compress).
//
// Included by k_repair.hip (the device kernel, Exec = one HIP workgroup of NT threads)
// and by tools/repair_emu.cpp (a host emulation that runs the same phases thread by
// thread; test infrastructure for the batch logic only, never part of the product).
// The includer defines RP_HD (function qualifiers) and provides the Exec policy:
//   ex.par(f)            f(tid) for every tid in [0, NT), then a workgroup barrier
//   ex.scan(a, &total)   in-place exclusive scan of a[0..NT) (LDS), total written by all
//   ex.scan2(a, b, &ta, &tb)  two such scans sharing their barriers
//   ex.add/sub/min/max/cas  atomics (u32; cas64 on u64)
//   ex.append(&n, pred)  index n++ for the threads with pred (wave-aggregated on the device), else NIL
//   ex.add_agg/sub_agg(p, act)  *p += / -= 1 for the threads with act; ex.slot_agg(p, act) the
//                        same returning the old value (a unique slot); on the device the lanes of
//                        a wave that hit the same word combine into one atomic
//   ex.leader(key, act), ex.is_leader(ld), ex.from_leader(v, ld)  one representative thread per
//                        distinct key (device: per wave; host: every thread represents itself)
//   ex.mark(id)          profiling hook: time since the previous mark goes to the previous id
//
// Reference semantics (PY:1817-1911), restated exactly:
//   freq(a,b) = number of overlapping adjacent positions holding (a,b); each round picks
//   the max freq, ties -> lexicographically smallest (a,b); stop when freq < 2; replace
//   left to right without overlap; stop (no rule) when that replaces fewer than 2.
//
// Device formulation (Larsson-Moffat style incremental counts, batched rounds):
//   * live positions form a doubly linked list (nxt/prv); opair[p] = id of the pair that
//     starts at live position p; cnt[id] is kept equal to a full recount at all times;
//     every pair id owns a region of occpos (positions where it was created — it is only
//     ever created once), validated lazily by opair[p] == id.
//   * the maximum count never increases (old pairs only lose occurrences; a new pair has
//     at most as many occurrences as the rule that created it), so rounds run by LEVEL f:
//     the pairs with count f, sorted by (a,b), are the next rounds in order, except that a
//     round can (i) lower the count of a later pair whose occurrences touch its own, and
//     (ii) create a pair (x, X) with count f that sorts before later ones.
//   * a BATCH is the longest prefix of the next W level pairs whose rounds commute with
//     the rounds before them: no occurrence of a member (chosen or not) overlaps an earlier
//     member's chosen occurrence span {i, nxt} (that would change the member's count), no
//     earlier member creates (x, X_k) with count f and x < a of the member (x = the left
//     symbol as of the member's turn), and no earlier member stops the run.  All rounds of
//     a batch then execute in parallel with symbols X_k = next + k, which is the
//     sequential result bit for bit.  Occurrences of two members that merely touch are
//     joined: the left one makes the pair (X_left, X_right) once, the right one makes no
//     left pair (the net effect of the two rounds in either order).  Overlapping runs of
//     (a,a) are resolved by pointer jumping (greedy left-to-right pairing = even distance
//     from the run start).
#pragma once
#include <stdint.h>

namespace kolm {
namespace rp {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;

// KOLM_RP_NT / KOLM_RP_RK: compile-time A/B knobs (tools/rp_variants.sh)
#ifndef KOLM_RP_NT
#define KOLM_RP_NT 1024
#endif
constexpr u32 NT = KOLM_RP_NT;    // threads of the block's workgroup (NT divides 2048).  At 1024 the
                                  // kernel holds 128 VGPRs x 4 waves per SIMD (the whole register file),
                                  // so no other stream's kernel runs on a CU beside it; 512 (170 VGPRs,
                                  // 2 waves) leaves registers, but its 94 KB of LDS still keeps the
                                  // 38-50 KB LDS kernels of the hot path off the CU (measured r3)
constexpr u32 W = 512;            // max rounds (members) per batch (<= NT: one window of NT entries)
constexpr u32 CAPR = 1u << 16;    // occurrence-region entries per batch beyond its first member
constexpr u32 SORT_LDS = 4096;    // level lists up to this size are sorted in LDS
constexpr u32 QLIM = 32768;       // level cache: a scan of all pairs picks flow so that Q holds <= QLIM pairs,
constexpr u32 TLIM = 2048;        //   a pass over Q picks ftop so that T holds <= TLIM pairs
constexpr u32 NIL = 0xFFFFFFFFu;
constexpr u32 DEAD = 0xFFFFFFFFu;
constexpr u64 EMPTY = ~0ull;
constexpr u32 BMAX = 1u << 21;    // mark tags ((BMAX - b) * W + member) << 1 | s, b = batch - tbase < BMAX
                                  // (the marks are reset and tbase moved when b reaches BMAX - 1)
constexpr u32 NBASE = 65536;      // ids of the byte pairs: (a << 8) | b
constexpr u32 MAX_N = 1u << 22;   // block length limit of the device Re-Pair
#ifndef KOLM_RP_RK
#define KOLM_RP_RK 4
#endif
constexpr u32 RK = KOLM_RP_RK;    // occurrences per thread per step in the occurrence loops
constexpr u32 AGG_MIN = 2048;     // batches with at least this many occurrences aggregate atomics
constexpr u32 WIN_MIN = 32;       // smallest adaptive window (members per batch)
#ifndef KOLM_RP_MCAP
#define KOLM_RP_MCAP(T) (2 * (T) + 16)  // window after a batch cut at T (A/B knob)
#endif
constexpr u32 MMAP = 1024;        // member map (pair id -> member index) slots, in sval[0 .. 2 MMAP)

enum : u32 { RS_SIZE = 0, RS_RULES, RS_FINAL, RS_BATCHES, RS_ERR, RS_LEVELS, RS_N };
// profile sections (ex.mark(id): time since the previous mark is charged to the previous id)
enum : u32 { P_INIT = 0, P_LVSCAN, P_LVSORT, P_WINDOW, P_GATHER, P_CHAINS, P_SELECT, P_APPLY_A, P_APPLY_B, P_LATE,
             P_SER, P_APPLY_A2, P_N };
enum : u32 { RE_OK = 0, RE_CAP = 1, RE_LOOP = 2, RE_LEN = 3 };

// Per position, one 16-byte record: the live sequence.  Every field an occurrence needs
// from a neighbour (its symbol, its links, the pair that starts there) is one vector load.
//   nxt/prv  the live doubly linked list
//   sym      symbol (DEAD once merged into its left neighbour)
//   opair    id of the pair starting here (NIL: none)
// The per-batch marks live beside it in mark[] (one word per position):
//   mark = min over the chosen occurrences covering the position of
//          ((BMAX - batch) * W + member) << 1 | (1 for the span's second position)
// so an earlier member's span (conflict), the same member's second position (left
// neighbour replaced too) and the same member's start (right neighbour replaced too) are
// all read from one word.  oidx[] (occurrence index by position) is used by (a,a) runs only.
struct alignas(16) Node {
    u32 nxt, prv, sym, opair;
};

// Per-block workspace (all device pointers).  Sizes for a block of length n:
//   n:      nd (16 B each), mark, oidx;  opos omem od0 od1 ot0 ot1 oidl oidr oj op oq
//           ox oy opj opp onp (occurrence neighbourhoods, by occurrence index)
//   3n+16:  occpos          PC = NBASE + 2n + 16: cnt poff plen pkey, lists (3 x key+id)
//   HS = pow2 >= n + 64:     hkey hval hcnt;  n + 16: husd;  n/2 + 16: rules
struct Block {
    const u8* text;
    u32 n;
    Node* nd;  // per position: the live sequence
    u32 *mark, *oidx;
    u32 *opos, *omem, *od0, *od1, *ot0, *ot1, *oidl, *oidr, *oj, *op, *oq;
    u32 *ox, *oy, *opj, *opp, *onp;
    u32* occpos;
    u32 *cnt, *poff, *plen;
    u64* pkey;
    u64 *lkA, *lkB, *lkL;
    u32 *liA, *liB, *liL;
    u64* hkey;
    u32 *hval, *hcnt;
    u32 hmask;
    u32* husd;
    u64* rules;
    u64 *qa, *qb, *ta, *tb;  // level cache tiers Q, T (PC entries each): (count when last read) << 32 | pair id
    u8* out;
    u64 out_cap;
    u32* result;  // RS_N words
};

struct Shared {
    u32 m_id[W], m_a[W], m_b[W], m_lpos[W], m_roff[W], m_rlen[W], m_pre[W + 1], m_repl[W], m_lmin[W], m_lmax[W];
    u32 scan[NT];
    u32 scan2[NT];
    u32 wtot[NT / 64], wtot2[NT / 64];
    u64 st_key[NT];             // window staging by level entry: key, id, region length / offset
    u32 st_id[NT], st_len[NT], st_off[NT];
    u32 irank[4 * NT];          // init: slot << 16 | rank of each position of a chunk
    u32 chg[3];
    u64 skey[SORT_LDS];
    u32 sval[SORT_LDS];
    u32 f, lp, lsize, M, V, T, tot, nocc, npairs, next_sym, nrules, pool, batch, hused, nlate;
    u32 t1, t2, ts, any_aa, cut, maxc, err, total, levels, tbase;
    u32 flow, qn, qn2, qvalid;  // level cache: Q = every pair with count >= flow
    u32 ftop, tn, tn2, tvalid, maxt, thr;  //   T = every pair of Q with count >= ftop
    u32 mcap;                   // adaptive window: members gathered per batch (<= W)
    u32 cslot[SORT_LDS];        // per LDS key slot: occurrences of the new pair, then the region fill counter
    u32 spoff[SORT_LDS];        //   and its region offset
};

// Carve a block's workspace out of `base` (nullptr: size query).  Returns the bytes
// used; every array is 256-byte aligned.  out/out_cap/result/text/n are set by the caller.
RP_HD inline u64 workspace_layout(char* base, u32 n, Block& B) {
    u64 off = 0;
    auto take = [&](u64 bytes) -> char* {
        char* p = base ? base + off : nullptr;
        off += (bytes + 255) & ~(u64)255;
        return p;
    };
    const u64 N = (u64)n + 16, PC = NBASE + 2ull * n + 16;
    u32 HS = 64;
    while (HS < n + 64) HS <<= 1;
    B.nd = (Node*)take(N * sizeof(Node));
    u32** n32[] = {&B.mark, &B.oidx, &B.opos, &B.omem, &B.od0, &B.od1, &B.ot0, &B.ot1, &B.oidl, &B.oidr,
                   &B.oj, &B.op, &B.oq, &B.ox, &B.oy, &B.opj, &B.opp, &B.onp, &B.husd};
    for (u32** p : n32) *p = (u32*)take(N * 4);
    B.occpos = (u32*)take(3 * N * 4);
    B.cnt = (u32*)take(PC * 4);
    B.poff = (u32*)take(PC * 4);
    B.plen = (u32*)take(PC * 4);
    B.pkey = (u64*)take(PC * 8);
    B.lkA = (u64*)take(PC * 8);
    B.lkB = (u64*)take(PC * 8);
    B.lkL = (u64*)take(PC * 8);
    B.liA = (u32*)take(PC * 4);
    B.liB = (u32*)take(PC * 4);
    B.liL = (u32*)take(PC * 4);
    B.hkey = (u64*)take((u64)HS * 8);
    B.hval = (u32*)take((u64)HS * 4);
    B.hcnt = (u32*)take((u64)HS * 4);
    B.hmask = HS - 1;
    B.rules = (u64*)take((N / 2 + 16) * 8);
    B.qa = (u64*)take(PC * 8);
    B.qb = (u64*)take(PC * 8);
    B.ta = (u64*)take(PC * 8);
    B.tb = (u64*)take(PC * 8);
    return off;
}

RP_HD inline u64 pkey_of(u32 a, u32 b) { return ((u64)a << 32) | b; }
RP_HD inline u32 umin(u32 a, u32 b) { return a < b ? a : b; }
RP_HD inline u32 umax(u32 a, u32 b) { return a > b ? a : b; }

RP_HD inline u32 hslot(u64 k, u32 mask) {
    k ^= k >> 31;
    k *= 0x9E3779B97F4A7C15ull;
    k ^= k >> 29;
    return (u32)k & mask;
}

RP_HD inline u32 uleb_len(u32 v) { return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5; }

RP_HD inline u32 uleb_put(u8* o, u32 v) {
    u32 k = 0;
    for (;;) {
        const u8 b = v & 0x7F;
        v >>= 7;
        if (v) {
            o[k++] = b | 0x80;
        } else {
            o[k++] = b;
            return k;
        }
    }
}

// The batch's table of new pair keys.  Every new pair contains a symbol created by this
// batch, so no earlier batch can hold its key: the table only deduplicates within the
// batch.  Small batches use the workgroup's LDS (the sort buffers, idle between the
// window and the late merge); large ones the block's global table (cleared via husd).
struct HTab {
    u64* k;
    u32* v;
    u32 mask;
    bool glob;
};

// Insert key into the batch's hash table; returns its slot.  The thread whose CAS wins
// allocates the pair id (read back from v[slot] after the next barrier).
template <class E>
RP_HD inline u32 hash_insert(E& ex, const Block& B, Shared& sh, const HTab& h, u64 key) {
    u32 s = hslot(key, h.mask);
    for (;;) {
        const u64 cur = h.k[s];
        if (cur == key) return s;
        if (cur == EMPTY) {
            const u64 old = ex.cas64(&h.k[s], EMPTY, key);
            if (old == EMPTY) {
                const u32 u = ex.add(&sh.hused, 1u);
                const u32 id = sh.npairs + u;
                if (h.glob) B.husd[u] = s;
                h.v[s] = id;
                B.pkey[id] = key;
                B.cnt[id] = 0;
                B.plen[id] = 0;
                return s;
            }
            if (old == key) return s;
        }
        s = (s + 1) & h.mask;
    }
}

// hash_insert by one representative thread per distinct key (device: per wave); every
// thread with act gets the key's slot.
template <class E>
RP_HD inline u32 hash_insert_wave(E& ex, const Block& B, Shared& sh, const HTab& h, u64 key, bool act, bool agg) {
    const u32 ld = ex.leader(key, act, agg);
    u32 s = 0;
    if (act && ex.is_leader(ld)) s = hash_insert(ex, B, sh, h, key);
    return ex.from_leader(s, ld);
}

// The slot of key in the batch's key table: the LDS table first (the thread whose CAS
// claims a slot allocates the pair id, as hash_insert does), the block's global table for a
// key whose LDS probe run exceeds HPROBE (table nearly full; rare: the big batches of text
// create a few dozen keys).  A key is never in both: a probe run that finds only other
// keys stays that way (slots are never freed within a batch), so every thread with that
// key goes global.  Global slots are returned with GSLOT set.
constexpr u32 HPROBE = 128;
constexpr u32 GSLOT = 0x80000000u;
template <class E>
RP_HD inline u32 hash_claim(E& ex, const Block& B, Shared& sh, u64 key) {
    u32 s = hslot(key, SORT_LDS - 1);
    for (u32 k = 0; k < HPROBE; ++k) {
        const u64 cur = sh.skey[s];
        if (cur == key) return s;
        if (cur == EMPTY) {
            const u64 old = ex.cas64(&sh.skey[s], EMPTY, key);
            if (old == EMPTY) {
                const u32 u = ex.add(&sh.hused, 1u);
                const u32 id = sh.npairs + u;
                B.husd[u] = NIL;
                sh.sval[s] = id;
                B.pkey[id] = key;
                B.cnt[id] = 0;
                B.plen[id] = 0;
                return s;
            }
            if (old == key) return s;
        }
        s = (s + 1) & (SORT_LDS - 1);
    }
    const HTab g{B.hkey, B.hval, B.hmask, true};
    return hash_insert(ex, B, sh, g, key) | GSLOT;
}

// Init-time pair table: slot of a 16-bit byte-pair code (IC positions per chunk into ICT
// slots; text holds ~1000-1500 distinct pairs per chunk).  NIL after IPROBE probes (random
// bytes nearly fill the table): the caller then counts / places that position directly.
constexpr u32 IC = 4 * NT;
constexpr u32 ICT = 4096;
constexpr u32 IPROBE = 64;
static_assert(ICT <= SORT_LDS && IC <= 4096, "init table (keys in sval, counts / bases in skey)");
template <class E>
RP_HD inline u32 ictab_slot(E& ex, u32* keys, u32 code) {
    u32 s = (code * 0x9E3779B1u) >> 20;
    for (u32 k = 0; k < IPROBE; ++k, s = (s + 1) & (ICT - 1)) {
        const u32 cur = keys[s];
        if (cur == code) return s;
        if (cur == NIL) {
            const u32 old = ex.cas32(&keys[s], NIL, code);
            if (old == NIL || old == code) return s;
        }
    }
    return NIL;
}

// hash_claim + one occurrence counted for the key (LDS slot counter, or the global slot's)
template <class E>
RP_HD inline u32 hash_count(E& ex, const Block& B, Shared& sh, u64 key) {
    const u32 s = hash_claim(ex, B, sh, key);
    if (s & GSLOT)
        ex.add(&B.hcnt[s & ~GSLOT], 1u);
    else
        ex.add(&sh.cslot[s], 1u);
    return s;
}

// The window's member map (LDS, open addressing over sval[0 .. MMAP) keys and
// sval[MMAP .. 2 MMAP) member indices): which pair ids are members of this batch.
RP_HD inline u32 mslot(u32 id) { return (id * 0x9E3779B1u) >> 22; }  // 10 bits = MMAP slots
template <class E>
RP_HD inline void member_put(E& ex, Shared& sh, u32 id, u32 r) {
    u32 s = mslot(id);
    while (ex.cas32(&sh.sval[s], NIL, id) != NIL) s = (s + 1) & (MMAP - 1);
    sh.sval[MMAP + s] = r;
}
RP_HD inline u32 member_of(const Shared& sh, u32 id) {
    if (id == NIL) return NIL;
    for (u32 s = mslot(id);; s = (s + 1) & (MMAP - 1)) {
        const u32 k = sh.sval[s];
        if (k == id) return sh.sval[MMAP + s];
        if (k == NIL) return NIL;
    }
}

// Sort key/id[0..n) ascending by key (keys unique); tk/ti is scratch of the same size.
// Result is left in k/i.
template <class E>
RP_HD inline void sort_list(E& ex, Shared& sh, u64* k, u32* id, u64* tk, u32* ti, u32 n) {
    // 1. runs of SORT_LDS sorted in LDS (bitonic)
    for (u32 base = 0; base < n; base += SORT_LDS) {
        const u32 len = n - base < SORT_LDS ? n - base : SORT_LDS;
        if (len <= NT) {
            // rank sort: two barriers; each key's rank = number of smaller keys (broadcast LDS reads)
            ex.par([&](u32 t) {
                if (t < len) {
                    sh.skey[t] = k[base + t];
                    sh.sval[t] = id[base + t];
                }
            });
            ex.par([&](u32 t) {
                if (t < len) {
                    const u64 key = sh.skey[t];
                    u32 r = 0;
                    for (u32 e = 0; e < len; ++e) r += sh.skey[e] < key ? 1u : 0u;
                    k[base + r] = key;
                    id[base + r] = sh.sval[t];
                }
            });
            continue;
        }
        u32 S = 2;
        while (S < len) S <<= 1;
        ex.par([&](u32 t) {
            for (u32 e = t; e < S; e += NT) {
                sh.skey[e] = e < len ? k[base + e] : EMPTY;
                sh.sval[e] = e < len ? id[base + e] : NIL;
            }
        });
        for (u32 kk = 2; kk <= S; kk <<= 1) {
            for (u32 j = kk >> 1; j > 0; j >>= 1) {
                ex.par([&](u32 t) {
                    for (u32 e = t; e < S; e += NT) {
                        const u32 l = e ^ j;
                        if (l > e) {
                            const bool asc = (e & kk) == 0;
                            const u64 x = sh.skey[e], y = sh.skey[l];
                            if (asc ? x > y : x < y) {
                                sh.skey[e] = y;
                                sh.skey[l] = x;
                                const u32 v = sh.sval[e];
                                sh.sval[e] = sh.sval[l];
                                sh.sval[l] = v;
                            }
                        }
                    }
                });
            }
        }
        ex.par([&](u32 t) {
            for (u32 e = t; e < len; e += NT) {
                k[base + e] = sh.skey[e];
                id[base + e] = sh.sval[e];
            }
        });
    }
    // 2. merge passes (merge path by binary search; keys are unique)
    u64* ka = k;
    u32* ia = id;
    u64* kb = tk;
    u32* ib = ti;
    for (u32 run = SORT_LDS; run < n; run <<= 1) {
        ex.par([&](u32 t) {
            for (u32 e = t; e < n; e += NT) {
                const u32 pairbase = e / (2 * run) * (2 * run);
                const u32 mid = pairbase + run < n ? pairbase + run : n;
                const u32 end = pairbase + 2 * run < n ? pairbase + 2 * run : n;
                const u64 key = ka[e];
                u32 lo, hi;
                if (e < mid) {
                    lo = mid;
                    hi = end;
                } else {
                    lo = pairbase;
                    hi = mid;
                }
                const u32 s0 = lo;
                while (lo < hi) {
                    const u32 m = (lo + hi) >> 1;
                    if (ka[m] < key) lo = m + 1; else hi = m;
                }
                const u32 rank = lo - s0;
                const u32 dst = e < mid ? e + rank : pairbase + (e - mid) + rank;
                kb[dst] = key;
                ib[dst] = ia[e];
            }
        });
        u64* tkk = ka; ka = kb; kb = tkk;
        u32* tii = ia; ia = ib; ib = tii;
    }
    if (ka != k) {
        ex.par([&](u32 t) {
            for (u32 e = t; e < n; e += NT) {
                k[e] = ka[e];
                id[e] = ia[e];
            }
        });
    }
}

// always_inline: as a called function its register budget and the call ABI spill to scratch
template <class E>
RP_HD __attribute__((always_inline)) inline void repair_block(E& ex, const Block& B, Shared& sh) {
    const u32 n = B.n;
    const u32 HS = B.hmask + 1;
    ex.mark(P_INIT);
    // init-time LDS pair table (ICT slots: keys in sval, counts / chunk bases in skey)
    u32* ictk = sh.sval;
    u32* ictc = reinterpret_cast<u32*>(sh.skey);
    u32* ictb = reinterpret_cast<u32*>(sh.skey) + ICT;
    // ---------------- init: linked list, byte-pair counts and regions ----------------
    ex.par([&](u32 t) {
        for (u32 i = t; i < NBASE; i += NT) {
            B.cnt[i] = 0;
            B.plen[i] = 0;
            B.pkey[i] = pkey_of(i >> 8, i & 255);
        }
        for (u32 i = t; i < HS; i += NT) {
            B.hkey[i] = EMPTY;
            B.hcnt[i] = 0;
        }
        if (t == 0) {
            sh.pool = 0; sh.npairs = NBASE; sh.next_sym = 256; sh.nrules = 0; sh.batch = 0;
            sh.lp = 0; sh.lsize = 0; sh.f = 0; sh.hused = 0; sh.nlate = 0; sh.err = RE_OK; sh.levels = 0;
            sh.qvalid = 0; sh.qn = 0; sh.flow = NIL; sh.mcap = W; sh.tbase = 0;
            sh.tvalid = 0; sh.tn = 0; sh.ftop = NIL;
        }
    });
    ex.par([&](u32 t) {
        for (u32 i = t; i < n; i += NT) {
            const bool last = i + 1 >= n;
            B.nd[i] = Node{last ? NIL : i + 1, i ? i - 1 : NIL, B.text[i], last ? NIL : ((u32)B.text[i] << 8) | B.text[i + 1]};
            B.mark[i] = NIL;
        }
        for (u32 s = t; s < ICT; s += NT) ictk[s] = NIL;
        for (u32 s = t; s < ICT; s += NT) ictc[s] = 0;
    });
    // byte-pair counts: every chunk of IC positions is counted in an LDS table first, then
    // one global atomic per distinct pair of the chunk (a global atomic per position is
    // throughput-bound at the L2 when every CU runs a block)
    for (u32 c0 = 0; c0 + 1 < n; c0 += IC) {
        ex.par([&](u32 t) {
#pragma unroll
            for (u32 k = 0; k < IC / NT; ++k) {
                const u32 i = c0 + k * NT + t;
                if (i + 1 < n) {
                    const u32 code = ((u32)B.text[i] << 8) | B.text[i + 1], sl = ictab_slot(ex, ictk, code);
                    ex.add(sl != NIL ? &ictc[sl] : &B.cnt[code], 1u);
                }
            }
        });
        ex.par([&](u32 t) {
            for (u32 s = t; s < ICT; s += NT) {
                const u32 code = ictk[s];
                if (code != NIL) {
                    ex.add(&B.cnt[code], ictc[s]);
                    ictk[s] = NIL;
                    ictc[s] = 0;
                }
            }
        });
    }
    ex.par([&](u32 t) {
        for (u32 c = t; c < NBASE; c += NT)
            if (B.cnt[c]) B.poff[c] = ex.add(&sh.pool, B.cnt[c]);
    });
    // occurrence regions: per chunk, each position's rank among its pair's positions in the
    // chunk (LDS), one returning global atomic per distinct pair for the chunk's base
    for (u32 c0 = 0; c0 + 1 < n; c0 += IC) {
        ex.par([&](u32 t) {
#pragma unroll
            for (u32 k = 0; k < IC / NT; ++k) {
                const u32 i = c0 + k * NT + t;
                if (i + 1 < n) {
                    const u32 code = ((u32)B.text[i] << 8) | B.text[i + 1], sl = ictab_slot(ex, ictk, code);
                    if (sl != NIL) {
                        sh.irank[k * NT + t] = sl << 16 | ex.add(&ictc[sl], 1u);
                    } else {
                        B.occpos[B.poff[code] + ex.add(&B.plen[code], 1u)] = i;
                        sh.irank[k * NT + t] = NIL;
                    }
                }
            }
        });
        ex.par([&](u32 t) {
            for (u32 s = t; s < ICT; s += NT) {
                const u32 code = ictk[s];
                if (code != NIL) ictb[s] = B.poff[code] + ex.add(&B.plen[code], ictc[s]);
            }
        });
        ex.par([&](u32 t) {
#pragma unroll
            for (u32 k = 0; k < IC / NT; ++k) {
                const u32 i = c0 + k * NT + t;
                if (i + 1 < n) {
                    const u32 v = sh.irank[k * NT + t];
                    if (v != NIL) B.occpos[ictb[v >> 16] + (v & 0xFFFFu)] = i;
                }
            }
            for (u32 s = t; s < ICT; s += NT) {  // ictb is read above, ictk / ictc no more
                ictk[s] = NIL;
                ictc[s] = 0;
            }
        });
    }
    ex.mark(P_INIT);
    u64* lk = B.lkA;
    u32* li = B.liA;
    u64* tk = B.lkB;
    u32* ti = B.liB;
    u64* qa = B.qa;  // level cache Q (and its compaction target)
    u64* qb = B.qb;
    u64* ta = B.ta;  // level cache T (and its compaction target)
    u64* tb = B.tb;
    u32 guard = 0;
    // ---------------- batches ----------------
    for (;;) {
        ex.begin(guard);
        if (++guard > 4 * n + 64) {  // unreachable: every batch retires >= 1 round or 1 level entry
            ex.par([&](u32 t) { if (t == 0) sh.err = RE_LOOP; });
            break;
        }
        if (sh.lp >= sh.lsize) {
            ex.mark(P_LVSCAN);
            // new level: f = max count; the level list = pairs with count f, sorted.  Counts
            // never rise except at creation, so a cache of every pair whose count is >= a
            // threshold, plus the pairs created since with a count >= it (apply 3), holds the
            // global maximum while its own maximum is >= the threshold.  Two tiers: Q = the
            // pairs with count >= flow (<= QLIM when taken from a scan of all pairs), T = the
            // pairs of Q with count >= ftop (<= TLIM when taken from Q).  A level reads T only;
            // T is retaken from Q when its maximum falls below ftop, Q from all pairs when its
            // maximum falls below flow.
            bool done = false;
            u32* hist = reinterpret_cast<u32*>(sh.skey);  // 2048 count bins (LDS, idle here)
            // sh.thr = the smallest bin >= lo whose suffix count is <= lim, at most the highest
            // non-empty bin (every pair of the top bin is taken); NIL when no count is >= lo
            auto pick = [&](u32 lo, u32 lim) {
                // suffix sums over the bins, top down: thread t holds the HB bins
                // 2047 - HB*t - k, k < HB (descending)
                constexpr u32 HB = 2048 / NT;
                ex.par([&](u32 t) {
                    u32 v = 0;
                    for (u32 k = 0; k < HB; ++k) v += hist[2047 - HB * t - k];
                    sh.scan[t] = v;
                    if (t == 0) { sh.thr = NIL; sh.maxc = 0; }
                });
                ex.scan(sh.scan, &sh.total);
                ex.par([&](u32 t) {
                    u32 run = sh.scan[t], cand = NIL;
                    bool top = false;
                    for (u32 k = 0; k < HB; ++k) {
                        const u32 bin = 2047 - HB * t - k;
                        run += hist[bin];  // #(count >= bin)
                        if (bin >= lo && run <= lim) cand = bin;
                        if (bin >= lo && hist[bin] && !top) {  // the highest non-empty bin
                            ex.max(&sh.maxc, bin);
                            top = true;
                        }
                    }
                    if (cand != NIL) ex.min(&sh.thr, cand);
                });
                ex.par([&](u32 t) {
                    if (t == 0) {
                        if (sh.maxc == 0) sh.thr = NIL;
                        else if (sh.thr == NIL || sh.thr > sh.maxc) sh.thr = sh.maxc;
                    }
                });
            };
            for (;;) {
                if (!sh.qvalid) {
                    ex.par([&](u32 t) {
                        for (u32 i = t; i < 2048; i += NT) hist[i] = 0;
                        if (t == 0) sh.qn = 0;
                    });
                    ex.par([&](u32 t) {
                        const u32 np = sh.npairs;
                        for (u32 i0 = 0; i0 < np; i0 += 4 * NT) {
                            u32 v[4];
#pragma unroll
                            for (u32 k = 0; k < 4; ++k) v[k] = i0 + k * NT + t < np ? B.cnt[i0 + k * NT + t] : 0u;
#pragma unroll
                            for (u32 k = 0; k < 4; ++k)
                                if (v[k] >= 2) ex.add(&hist[v[k] < 2047 ? v[k] : 2047u], 1u);
                        }
                    });
                    pick(2, QLIM);
                    if (sh.thr == NIL) {  // no pair occurs twice
                        done = true;
                        break;
                    }
                    ex.par([&](u32 t) {
                        const u32 np = sh.npairs, fl = sh.thr;
                        for (u32 i0 = 0; i0 < np; i0 += RK * NT) {
                            u32 c[RK];
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) c[k] = i0 + k * NT + t < np ? B.cnt[i0 + k * NT + t] : 0u;
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) {
                                const u32 id = i0 + k * NT + t;
                                const bool keep = id < np && c[k] >= fl;
                                const u32 slot = ex.append(&sh.qn, keep);
                                if (keep) qa[slot] = ((u64)c[k] << 32) | id;
                            }
                        }
                        if (t == 0) { sh.flow = fl; sh.qvalid = 1; sh.tvalid = 0; }
                    });
                }
                if (!sh.tvalid) {
                    // Q by current counts: drop the entries below flow, histogram of the rest,
                    // then T = the entries >= ftop (their counts are current: no second load)
                    ex.par([&](u32 t) {
                        for (u32 i = t; i < 2048; i += NT) hist[i] = 0;
                        if (t == 0) { sh.qn2 = 0; sh.tn = 0; sh.maxt = 0; }
                    });
                    ex.par([&](u32 t) {
                        const u32 qn = sh.qn, fl = sh.flow;
                        for (u32 e0 = 0; e0 < qn; e0 += RK * NT) {
                            u32 id[RK], c[RK];
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) id[k] = e0 + k * NT + t < qn ? (u32)qa[e0 + k * NT + t] : 0u;
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) c[k] = e0 + k * NT + t < qn ? B.cnt[id[k]] : 0u;
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) {
                                const bool keep = e0 + k * NT + t < qn && c[k] >= fl;
                                const u32 slot = ex.append(&sh.qn2, keep);
                                if (keep) {
                                    qb[slot] = ((u64)c[k] << 32) | id[k];
                                    ex.add(&hist[c[k] < 2047 ? c[k] : 2047u], 1u);
                                }
                            }
                        }
                    });
                    {
                        u64* x = qa; qa = qb; qb = x;
                    }
                    ex.par([&](u32 t) { if (t == 0) sh.qn = sh.qn2; });
                    if (sh.qn == 0) {  // every count of Q fell below flow
                        if (sh.flow <= 2) {  // every count is below 2: no further rule (PY:1879)
                            done = true;
                            break;
                        }
                        ex.par([&](u32 t) { if (t == 0) sh.qvalid = 0; });
                        continue;
                    }
                    pick(sh.flow, TLIM);
                    ex.par([&](u32 t) {
                        const u32 qn = sh.qn, ft = sh.thr;
                        u32 m = 0;
                        for (u32 e0 = 0; e0 < qn; e0 += RK * NT) {
                            u64 q[RK];
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) q[k] = e0 + k * NT + t < qn ? qa[e0 + k * NT + t] : 0ull;
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) {
                                const u32 c = (u32)(q[k] >> 32);
                                const bool keep = e0 + k * NT + t < qn && c >= ft;
                                const u32 slot = ex.append(&sh.tn, keep);
                                if (keep) {
                                    ta[slot] = q[k];
                                    m = c > m ? c : m;
                                }
                            }
                        }
                        if (m) ex.max(&sh.maxt, m);
                        if (t == 0) { sh.ftop = ft; sh.tvalid = 1; }
                    });
                    break;
                }
                // drop the entries of T below ftop, and the maximum of the rest
                ex.par([&](u32 t) {
                    for (u32 i = t; i < 2048; i += NT) hist[i] = 0;
                    if (t == 0) { sh.maxt = 0; sh.tn2 = 0; }
                });
                ex.par([&](u32 t) {
                    // current counts (they only fall between levels); the survivors keep
                    // theirs, so the level list below needs no second count load
                    u32 m = 0;
                    const u32 tn = sh.tn, fl = sh.ftop;
                    for (u32 e0 = 0; e0 < tn; e0 += RK * NT) {
                        u32 id[RK], c[RK];
#pragma unroll
                        for (u32 k = 0; k < RK; ++k) id[k] = e0 + k * NT + t < tn ? (u32)ta[e0 + k * NT + t] : 0u;
#pragma unroll
                        for (u32 k = 0; k < RK; ++k) c[k] = e0 + k * NT + t < tn ? B.cnt[id[k]] : 0u;
#pragma unroll
                        for (u32 k = 0; k < RK; ++k) {
                            const bool keep = e0 + k * NT + t < tn && c[k] >= fl;
                            const u32 slot = ex.append(&sh.tn2, keep);
                            if (keep) {
                                tb[slot] = ((u64)c[k] << 32) | id[k];
                                m = c[k] > m ? c[k] : m;
                                ex.add(&hist[c[k] < 2047 ? c[k] : 2047u], 1u);
                            }
                        }
                    }
                    if (m) ex.max(&sh.maxt, m);
                });
                {
                    u64* x = ta; ta = tb; tb = x;
                }
                ex.par([&](u32 t) { if (t == 0) sh.tn = sh.tn2; });
                if (sh.maxt >= sh.ftop && sh.tn > 2 * TLIM) {
                    // T grew with created pairs: raise ftop (the dropped entries stay in Q)
                    pick(sh.ftop, TLIM);
                    ex.par([&](u32 t) { if (t == 0) sh.tn2 = 0; });
                    ex.par([&](u32 t) {
                        const u32 tn = sh.tn, ft = sh.thr;
                        for (u32 e0 = 0; e0 < tn; e0 += RK * NT) {
                            u64 q[RK];
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) q[k] = e0 + k * NT + t < tn ? ta[e0 + k * NT + t] : 0ull;
#pragma unroll
                            for (u32 k = 0; k < RK; ++k) {
                                const bool keep = e0 + k * NT + t < tn && (u32)(q[k] >> 32) >= ft;
                                const u32 slot = ex.append(&sh.tn2, keep);
                                if (keep) tb[slot] = q[k];
                            }
                        }
                    });
                    {
                        u64* x = ta; ta = tb; tb = x;
                    }
                    ex.par([&](u32 t) { if (t == 0) { sh.tn = sh.tn2; sh.ftop = sh.thr; } });
                }
                if (sh.maxt >= sh.ftop) break;
                ex.par([&](u32 t) { if (t == 0) sh.tvalid = 0; });
            }
            if (done) break;
            ex.par([&](u32 t) {
                if (t == 0) { sh.f = sh.maxt; sh.lsize = 0; sh.lp = 0; sh.levels++; sh.mcap = W; }
            });
            ex.par([&](u32 t) {
                // T was just filtered / taken: its entries carry their current counts
                const u32 tn = sh.tn, fl = sh.f;
                for (u32 e0 = 0; e0 < tn; e0 += RK * NT) {
                    u64 q[RK];
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) q[k] = e0 + k * NT + t < tn ? ta[e0 + k * NT + t] : 0ull;
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) {
                        const bool hit = e0 + k * NT + t < tn && (u32)(q[k] >> 32) == fl;
                        const u32 slot = ex.append(&sh.lsize, hit);
                        if (hit) {
                            lk[slot] = B.pkey[(u32)q[k]];
                            li[slot] = (u32)q[k];
                        }
                    }
                }
            });
            ex.mark(P_LVSORT);
            sort_list(ex, sh, lk, li, tk, ti, sh.lsize);
        }
        ex.mark(P_WINDOW);
        if (sh.batch - sh.tbase >= BMAX - 1) {  // mark tags exhausted (> 2M batches): start over
            ex.par([&](u32 t) {
                for (u32 i = t; i < n; i += NT) B.mark[i] = NIL;
            });
            ex.par([&](u32 t) { if (t == 0) sh.tbase = sh.batch; });
        }
        const u32 f = sh.f;
        const u32 otag0 = (BMAX - (sh.batch - sh.tbase)) * W;
        // this batch's marks of member m: start (m2s(m)) / second position (m2s(m) | 1)
        auto m2s = [&](u32 m) { return (otag0 + m) << 1; };
        const u32 X0 = sh.next_sym;
        // ---- window: the next valid level entries (count still f), in list order; each
        //      entry's key, region and validity are read at once, the members (valid entries
        //      ranked by one scan, their region prefix by a second sharing its barriers) are
        //      then placed from LDS ----
        ex.par([&](u32 t) {
            const u32 idx = sh.lp + t;
            const bool in = idx < sh.lsize;
            const u32 id = in ? li[idx] : 0u;
            const u64 key = in ? lk[idx] : 0ull;
            const u32 c = in ? B.cnt[id] : 0u, len = in ? B.plen[id] : 0u, off = in ? B.poff[id] : 0u;
            const bool valid = in && c == f;
            sh.scan[t] = valid ? 1u : 0u;
            sh.scan2[t] = valid ? len : 0u;
            sh.st_key[t] = key;
            sh.st_id[t] = id;
            sh.st_len[t] = len;
            sh.st_off[t] = off;
            for (u32 e = t; e < SORT_LDS; e += NT) sh.skey[e] = EMPTY;  // the LDS key table (HTab)
            for (u32 e = t; e < MMAP; e += NT) sh.sval[e] = NIL;        // the member map
            for (u32 e = t; e < SORT_LDS; e += NT) sh.cslot[e] = 0;
            if (t == 0) {
                sh.cut = NIL; sh.any_aa = 0; sh.nocc = 0; sh.t1 = NIL; sh.t2 = NIL; sh.ts = NIL;
                sh.hused = 0; sh.nlate = 0;
            }
        });
        ex.scan2(sh.scan, sh.scan2, &sh.V, &sh.total);
        if (sh.V == 0) {
            ex.par([&](u32 t) {
                if (t == 0) sh.lp = sh.lp + NT < sh.lsize ? sh.lp + NT : sh.lsize;
            });
            continue;
        }
        // members beyond T are gathered and scanned for nothing (re-gathered by the next
        // batch): the window follows the previous batch's T (doubling when it was not cut)
        const u32 Mw = umin(sh.V, umin(W, sh.mcap));
        ex.par([&](u32 t) {
            const u32 r = sh.scan[t];
            const bool valid = (t + 1 < NT ? sh.scan[t + 1] : sh.V) != r;  // this entry's flag
            if (valid && r <= W) sh.m_pre[r] = sh.scan2[t];  // region prefix over the members
            if (valid && r < W) {
                const u32 id = sh.st_id[t], len = sh.st_len[t];
                const u64 key = sh.st_key[t];
                const u32 a = (u32)(key >> 32), b = (u32)key;
                sh.m_id[r] = id;
                sh.m_a[r] = a;
                sh.m_b[r] = b;
                sh.m_lpos[r] = sh.lp + t;
                sh.m_roff[r] = sh.st_off[t];
                sh.m_rlen[r] = len;
                sh.m_repl[r] = 0;
                sh.m_lmin[r] = NIL;
                sh.m_lmax[r] = 0;
                if (a == b) sh.any_aa = 1;
                member_put(ex, sh, id, r);
                if (r > 0 && r < Mw && sh.scan2[t] + len > CAPR) ex.min(&sh.cut, r);
            }
        });
        const u32 M = sh.cut < Mw ? sh.cut : Mw;
        const u32 tot = M < sh.V ? sh.m_pre[M] : sh.total;
        const bool aa = sh.any_aa != 0;
        ex.mark(P_GATHER);
        // Occurrence loops below take RK occurrences per thread per step, their dependent
        // loads staged level by level (every load of a level issued before any is used): the
        // phases are latency-bound, so RK chains are in flight per thread instead of one.
        // Wave-aggregated atomics pay off only when a batch has many occurrences (few hot
        // words then take thousands of +-1); below AGG_MIN they cost more than they save.
        const bool agg_g = tot >= AGG_MIN;
        // ---- no (a,a) member: every live occurrence is replaced, so two members' chosen
        //      occurrences touch exactly where a neighbouring pair of one occurrence is
        //      another member's pair.  One pass gathers each occurrence with its neighbourhood
        //      and decides everything the select phase below does for (a,a) batches: a
        //      conflict between members m' and m (the pair at p, j or q of one is the other's)
        //      cuts the batch at max(m, m') — the pair at pp is the one at q of the occurrence
        //      at pp, which flags it —; q starts a chosen occurrence of the same member iff
        //      its pair is the member's (right neighbour replaced too); p is the second
        //      position of one iff the pair at pp is the member's, possible only when the
        //      symbol at p is the member's b (then pp is read). ----
        if (!aa) {
            ex.par([&](u32 t) {
                for (u32 e0 = 0; e0 < tot; e0 += RK * NT) {
                    u32 pos[RK], lo[RK], p[RK], j[RK], q[RK], x[RK], pj[RK], pp[RK], ppv[RK], y[RK], pq[RK], lpr[RK];
                    bool valid[RK];
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) {
                        const u32 e = e0 + k * NT + t;
                        u32 l = 0;
                        pos[k] = 0;
                        if (e < tot) {
                            u32 hi = M;  // member l: m_pre[l] <= e < m_pre[l+1]
                            while (hi - l > 1) {
                                const u32 md = (l + hi) >> 1;
                                if (sh.m_pre[md] <= e) l = md; else hi = md;
                            }
                            pos[k] = B.occpos[sh.m_roff[l] + (e - sh.m_pre[l])];
                        }
                        lo[k] = l;
                    }
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) {
                        const bool in = e0 + k * NT + t < tot;
                        const Node c = B.nd[in ? pos[k] : 0u];
                        valid[k] = in && c.opair == sh.m_id[lo[k]];
                        j[k] = c.nxt;
                        p[k] = valid[k] ? c.prv : NIL;
                    }
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) {
                        const Node cj = B.nd[valid[k] ? j[k] : 0u];
                        const Node cp = B.nd[p[k] != NIL ? p[k] : 0u];
                        q[k] = valid[k] ? cj.nxt : NIL;
                        pj[k] = cj.opair;
                        x[k] = cp.sym;
                        pp[k] = p[k] != NIL ? cp.opair : NIL;
                        ppv[k] = cp.prv;
                    }
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) {
                        const Node cq = B.nd[q[k] != NIL ? q[k] : 0u];
                        y[k] = cq.sym;
                        pq[k] = q[k] != NIL ? cq.opair : NIL;
                        lpr[k] = p[k] != NIL && ppv[k] != NIL ? B.nd[ppv[k]].opair : NIL;  // pair ending at p
                    }
#pragma unroll
                    for (u32 k = 0; k < RK; ++k) {
                        const u32 o = ex.append(&sh.nocc, valid[k]);
                        if (valid[k]) {
                            const u32 m = lo[k];
                            // overlaps: the pair at p or at j is another member's
                            const u32 c1 = member_of(sh, pp[k]), c2 = q[k] != NIL ? member_of(sh, pj[k]) : NIL;
                            u32 cut = NIL;
                            if (c1 != NIL) cut = umax(m, c1);
                            if (c2 != NIL) cut = umin(cut, umax(m, c2));
                            if (cut != NIL) ex.min(&sh.t1, cut);
                            // neighbours: the member whose occurrence ends at p (lm) / starts at q (rm)
                            const u32 lm = member_of(sh, lpr[k]), rm = q[k] != NIL ? member_of(sh, pq[k]) : NIL;
                            // left symbol when m runs: p's (an earlier or the same member makes it new)
                            const u32 xl = (p[k] != NIL && !(lm != NIL && lm <= m)) ? x[k] : NIL;
                            ex.min(&sh.m_lmin[m], xl);
                            ex.max(&sh.m_lmax[m], xl);
                            B.opos[o] = pos[k];
                            B.omem[o] = m;
                            B.oj[o] = j[k];
                            B.op[o] = p[k];
                            B.oq[o] = q[k];
                            B.onp[o] = ppv[k];
                            B.ox[o] = x[k];
                            B.oy[o] = y[k];
                            B.oidl[o] = lm;
                            B.oidr[o] = rm;
                            B.opj[o] = pj[k];
                            B.opp[o] = pp[k];
                        }
                        ex.add_agg(&sh.m_repl[lo[k]], valid[k], agg_g);
                    }
                }
            });
        }
        // ---- (a,a) batches: gather the members' live occurrences with their neighbourhoods
        //      (the links and symbols do not change before apply 2); runs, marks and the
        //      select phase follow ----
        if (aa) ex.par([&](u32 t) {
            for (u32 e0 = 0; e0 < tot; e0 += RK * NT) {
                u32 pos[RK], lo[RK], p[RK], j[RK], q[RK], o[RK];
                bool valid[RK];
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const u32 e = e0 + k * NT + t;
                    u32 l = 0;
                    pos[k] = 0;
                    if (e < tot) {
                        u32 hi = M;  // member l: m_pre[l] <= e < m_pre[l+1]
                        while (hi - l > 1) {
                            const u32 md = (l + hi) >> 1;
                            if (sh.m_pre[md] <= e) l = md; else hi = md;
                        }
                        pos[k] = B.occpos[sh.m_roff[l] + (e - sh.m_pre[l])];
                    }
                    lo[k] = l;
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const bool in = e0 + k * NT + t < tot;
                    const Node c = B.nd[in ? pos[k] : 0u];
                    valid[k] = in && c.opair == sh.m_id[lo[k]];
                    j[k] = c.nxt;
                    p[k] = valid[k] ? c.prv : NIL;
                }
                // each field is stored as soon as it arrives (fewer live registers)
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    o[k] = ex.append(&sh.nocc, valid[k]);
                    if (valid[k]) {
                        B.opos[o[k]] = pos[k];
                        B.omem[o[k]] = lo[k];
                        B.oj[o[k]] = j[k];
                        B.op[o[k]] = p[k];
                    }
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const Node cj = B.nd[valid[k] ? j[k] : 0u];
                    const Node cp = B.nd[p[k] != NIL ? p[k] : 0u];
                    q[k] = cj.nxt;
                    if (valid[k]) {
                        B.oq[o[k]] = cj.nxt;
                        B.opj[o[k]] = cj.opair;
                        B.ox[o[k]] = cp.sym;
                        B.opp[o[k]] = cp.opair;
                        B.onp[o[k]] = cp.prv;
                    }
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const u32 y = B.nd[valid[k] && q[k] != NIL ? q[k] : 0u].sym;
                    if (valid[k]) {
                        B.oy[o[k]] = y;
                        B.oidx[pos[k]] = o[k];
                    }
                }
            }
        });
        const u32 nocc = sh.nocc;
        const bool agg = nocc >= AGG_MIN;
        ex.mark(P_CHAINS);
        // ---- runs of (a,a): distance from the run start by pointer jumping; greedy
        //      left-to-right pairing replaces the occurrences at even distance ----
        u32* dist = B.od0;
        if (aa) {
            ex.par([&](u32 t) {
                for (u32 o = t; o < nocc; o += NT) {
                    const u32 m = B.omem[o];
                    u32 pp = NIL;
                    if (sh.m_a[m] == sh.m_b[m]) {
                        const u32 p = B.op[o];  // the pair at p (gathered): the same (a,a)?
                        if (p != NIL && B.opp[o] == sh.m_id[m]) pp = B.oidx[p];
                    }
                    B.ot0[o] = pp;
                    B.od0[o] = pp != NIL ? 1u : 0u;
                }
            });
            u32 *d0 = B.od0, *d1 = B.od1, *p0 = B.ot0, *p1 = B.ot1;
            // three rotating flags: iteration k sets chg[k%3] and clears chg[(k+1)%3], which
            // was last read two iterations ago (a barrier in between)
            ex.par([&](u32 t) { if (t == 0) { sh.chg[0] = 0; sh.chg[1] = 0; sh.chg[2] = 0; } });
            for (u32 it = 0;; ++it) {
                const u32 c = it % 3;
                ex.par([&](u32 t) {
                    if (t == 0) sh.chg[(c + 1) % 3] = 0;
                    bool any = false;
                    for (u32 o = t; o < nocc; o += NT) {
                        const u32 p = p0[o];
                        if (p != NIL) {
                            d1[o] = d0[o] + d0[p];
                            p1[o] = p0[p];
                            any = true;
                        } else {
                            d1[o] = d0[o];
                            p1[o] = NIL;
                        }
                    }
                    if (any) ex.max(&sh.chg[c], 1u);
                });
                u32* x = d0; d0 = d1; d1 = x;
                x = p0; p0 = p1; p1 = x;
                if (!sh.chg[c]) break;
            }
            dist = d0;
            // chosen occurrences: tags, replacement counts, span owners
            ex.par([&](u32 t) {
                for (u32 o = t; o < nocc; o += NT) {
                    const bool ch = !(dist[o] & 1u);
                    const u32 m = B.omem[o];
                    if (ch) {
                        ex.min(&B.mark[B.opos[o]], m2s(m));
                        ex.min(&B.mark[B.oj[o]], m2s(m) | 1u);
                    }
                    ex.add_agg(&sh.m_repl[m], ch, agg);
                }
            });
        }
        ex.mark(P_SELECT);
        // ---- (a,a) batches: overlaps (i or j in an earlier member's span), the neighbouring
        //      chosen occurrences, left-neighbour uniformity; one mark word per position ----
        if (aa) ex.par([&](u32 t) {
            for (u32 o0 = t; o0 < nocc; o0 += RK * NT) {
                bool act[RK], in[RK];
                u32 m[RK], i[RK], p[RK], j[RK], q[RK], wi[RK], wj[RK], wp[RK], wq[RK];
                // mark of an earlier member of this batch (either position of its span)
                auto early = [&](u32 w, u32 mm) { return w >= m2s(0) && w < m2s(mm); };
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const u32 o = o0 + k * NT;
                    in[k] = o < nocc;
                    act[k] = in[k] && !(dist[o] & 1u);  // chosen
                    m[k] = in[k] ? B.omem[o] : 0u;
                    i[k] = in[k] ? B.opos[o] : 0u;
                    j[k] = in[k] ? B.oj[o] : 0u;
                    p[k] = act[k] ? B.op[o] : NIL;
                    q[k] = act[k] ? B.oq[o] : NIL;
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    wi[k] = in[k] ? B.mark[i[k]] : NIL;
                    wj[k] = in[k] ? B.mark[j[k]] : NIL;
                    wp[k] = p[k] != NIL ? B.mark[p[k]] : NIL;
                    wq[k] = q[k] != NIL ? B.mark[q[k]] : NIL;
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    // an occurrence of the member in an earlier member's span (chosen or not:
                    // the unchosen ones of a run count too) changes its count
                    if (in[k] && (early(wi[k], m[k]) || early(wj[k], m[k]))) ex.min(&sh.t1, m[k]);
                    if (!act[k]) continue;
                    const u32 o = o0 + k * NT;
                    // neighbours (resolved against T in apply 1): p the second position of a
                    // chosen occurrence (lm), q the start of one (rm) — this batch's marks only
                    auto cur = [&](u32 w) { return w >= m2s(0) && w < m2s(M); };
                    const u32 lm = p[k] != NIL && cur(wp[k]) && (wp[k] & 1u) ? (wp[k] >> 1) - otag0 : NIL;
                    const u32 rm = q[k] != NIL && cur(wq[k]) && !(wq[k] & 1u) ? (wq[k] >> 1) - otag0 : NIL;
                    const u32 x = (p[k] != NIL && !(lm != NIL && lm <= m[k])) ? B.ox[o] : NIL;
                    ex.min(&sh.m_lmin[m[k]], x);
                    ex.max(&sh.m_lmax[m[k]], x);
                    B.oidl[o] = lm;
                    B.oidr[o] = rm;
                }
            }
        });
        ex.par([&](u32 t) {
            for (u32 m = t; m < M; m += NT) {
                if (sh.m_repl[m] < 2) ex.min(&sh.ts, m);
                // (x, X_m) with count f sorts before every later member with a > x
                if (sh.m_lmin[m] == sh.m_lmax[m] && sh.m_lmin[m] != NIL && sh.m_repl[m] == f) {
                    const u32 x = sh.m_lmin[m];
                    u32 lo = m + 1, hi = M;
                    while (lo < hi) {
                        const u32 md = (lo + hi) >> 1;
                        if (sh.m_a[md] > x) hi = md; else lo = md + 1;
                    }
                    if (lo < M) ex.min(&sh.t2, lo);
                }
            }
        });
        u32 T = M;
        T = sh.t1 < T ? sh.t1 : T;
        T = sh.t2 < T ? sh.t2 : T;
        T = sh.ts < T ? sh.ts : T;
        const bool stop = sh.ts != NIL && sh.ts < sh.t1 && sh.ts < sh.t2;
        if (T == 0) break;  // the next round replaces < 2 occurrences (PY:1879-1882)
        ex.mark(P_APPLY_A);
        // ---- apply 1: destroy the old pair occurrences; claim the new pair keys (the claiming
        //      thread allocates the id) and count their occurrences per key slot (slots kept in
        //      ox (left) / opj (right)); j and q's link of the rewritten sequence (i and p's pair
        //      in apply 4, where the ids are read) ----
        ex.par([&](u32 t) {
            for (u32 o0 = t; o0 < nocc; o0 += RK * NT) {
                bool act[RK], rcf[RK];
                u32 m[RK], p[RK], q[RK], xl[RK], yr[RK], pj[RK], pp[RK];
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const u32 o = o0 + k * NT;
                    act[k] = o < nocc && !(aa && (dist[o] & 1u));
                    m[k] = act[k] ? B.omem[o] : 0u;
                    act[k] = act[k] && m[k] < T;
                    p[k] = act[k] ? B.op[o] : NIL;
                    q[k] = act[k] ? B.oq[o] : NIL;
                    if (act[k]) {
                        // the occurrences that end at p / start at q are replaced too when their
                        // members run in this batch: p then belongs to the left one (which makes
                        // the joint pair (X_lm, X_m) as its right pair), q's symbol becomes X_rm
                        const u32 lm = B.oidl[o], rm = B.oidr[o];
                        const bool lc = lm != NIL && lm < T;
                        rcf[k] = rm != NIL && rm < T;
                        const u32 pv = p[k];
                        if (lc) p[k] = NIL;
                        B.op[o] = p[k];
                        B.onp[o] = lc ? B.onp[o] : pv;  // i's new left neighbour: pp or p
                        xl[k] = B.ox[o];
                        yr[k] = rcf[k] ? X0 + rm : B.oy[o];
                    } else {
                        rcf[k] = false;
                        xl[k] = yr[k] = 0u;
                    }
                    pj[k] = q[k] != NIL ? B.opj[o] : 0u;  // pairs at j and p (gathered)
                    pp[k] = p[k] != NIL ? B.opp[o] : 0u;
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    // the member's own pair loses m_repl[m] occurrences: subtracted once in apply 3
                    const bool hq = q[k] != NIL, hp = p[k] != NIL;
                    ex.sub_agg(&B.cnt[pj[k]], hq, agg);
                    ex.sub_agg(&B.cnt[pp[k]], hp, agg);
                    const u32 X = X0 + m[k];
                    const u32 o = o0 + k * NT;
                    if (hq) B.opj[o] = hash_count(ex, B, sh, pkey_of(X, yr[k]));
                    if (hp) B.ox[o] = hash_count(ex, B, sh, pkey_of(xl[k], X));
                }
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    if (!act[k]) continue;
                    const u32 o = o0 + k * NT;
                    // j is written whole (i in apply 4, with its pair id); q's link only when q
                    // does not start a chosen occurrence itself (that one writes its own record)
                    B.nd[B.oj[o]] = Node{NIL, NIL, DEAD, NIL};
                    if (q[k] != NIL && !rcf[k]) B.nd[q[k]].prv = B.opos[o];
                }
            }
        });
        ex.mark(P_APPLY_B);
        // ---- apply 3: regions of the new pairs (LDS-table keys by slot, global-table keys by
        //      id); count-f pairs join the level late ----
        ex.par([&](u32 t) {
            const u32 np = sh.npairs;
            auto region = [&](u32 id, u32 c) {
                const u32 po = ex.add(&sh.pool, c);
                B.poff[id] = po;
                B.cnt[id] = c;
                if (c == f) {
                    const u32 k = ex.add(&sh.nlate, 1u);
                    B.lkL[k] = B.pkey[id];
                    B.liL[k] = id;
                }
                if (c >= sh.flow) qa[ex.add(&sh.qn, 1u)] = ((u64)c << 32) | id;  // keeps Q complete (level cache)
                if (c >= sh.ftop) ta[ex.add(&sh.tn, 1u)] = ((u64)c << 32) | id;  // and T
                return po;
            };
            for (u32 s = t; s < SORT_LDS; s += NT)
                if (sh.skey[s] != EMPTY) {
                    const u32 id = sh.sval[s], c = sh.cslot[s];
                    B.plen[id] = c;  // apply 4 fills the c slots of the region by the LDS counter
                    sh.spoff[s] = region(id, c);
                    sh.cslot[s] = 0;  // now the region's fill counter
                }
            for (u32 u = t; u < sh.hused; u += NT)
                if (B.husd[u] != NIL) {
                    const u32 g = B.husd[u], c = B.hcnt[g];
                    B.hcnt[g] = 0;
                    B.plen[np + u] = 0;  // apply 4 fills by global atomics
                    region(np + u, c);
                }
            for (u32 m = t; m < T; m += NT) {
                B.rules[sh.nrules + m] = pkey_of(sh.m_a[m], sh.m_b[m]);
                ex.sub(&B.cnt[sh.m_id[m]], sh.m_repl[m]);  // its replaced occurrences (apply 1)
            }
        });
        // ---- apply 4: occurrence positions of the new pairs; i's record, p's pair ----
        ex.par([&](u32 t) {
            for (u32 o0 = t; o0 < nocc; o0 += RK * NT) {
                bool act[RK];
                u32 p[RK], q[RK], i[RK], sr[RK], sl[RK], m[RK];
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    const u32 o = o0 + k * NT;
                    act[k] = o < nocc && !(aa && (dist[o] & 1u));
                    m[k] = act[k] ? B.omem[o] : 0u;
                    act[k] = act[k] && m[k] < T;
                    q[k] = act[k] ? B.oq[o] : NIL;
                    p[k] = act[k] ? B.op[o] : NIL;
                    i[k] = act[k] ? B.opos[o] : 0u;
                    sr[k] = q[k] != NIL ? B.opj[o] : 0u;
                    sl[k] = p[k] != NIL ? B.ox[o] : 0u;
                }
                // the new pair's id and this occurrence's place in its region
                auto place = [&](u32 slot, u32 pos) {
                    u32 id, at;
                    if (slot & GSLOT) {
                        id = B.hval[slot & ~GSLOT];
                        at = B.poff[id] + ex.add(&B.plen[id], 1u);
                    } else {
                        id = sh.sval[slot];
                        at = sh.spoff[slot] + ex.add(&sh.cslot[slot], 1u);
                    }
                    B.occpos[at] = pos;
                    return id;
                };
#pragma unroll
                for (u32 k = 0; k < RK; ++k) {
                    if (!act[k]) continue;
                    const u32 o = o0 + k * NT;
                    const u32 idr = q[k] != NIL ? place(sr[k], i[k]) : NIL;
                    B.nd[i[k]] = Node{q[k], B.onp[o], X0 + m[k], idr};  // one 16-byte store
                    if (p[k] != NIL) B.nd[p[k]].opair = place(sl[k], p[k]);
                }
            }
            for (u32 u = t; u < sh.hused; u += NT)  // clear the keys that went to the global table
                if (B.husd[u] != NIL) B.hkey[B.husd[u]] = EMPTY;
            if (t == 0) {
                sh.lp = sh.m_lpos[T - 1] + 1;
                sh.next_sym += T;
                sh.nrules += T;
                sh.npairs += sh.hused;
                sh.batch += 1;
                sh.mcap = T < M ? umax(WIN_MIN, umin(W, KOLM_RP_MCAP(T))) : umin(W, 2 * M);
            }
        });
        {
            const u32 fr[8] = {f, M, T, nocc, sh.hused, sh.nlate, aa ? 1u : 0u, tot};
            ex.record(fr);
        }
        ex.mark(P_LATE);
        if (sh.nlate) {
            // new pairs with count f join the level list at their key position.  When they all
            // start with a new symbol (X_m, y) they sort after every entry of the list (whose
            // symbols all predate this batch): append; otherwise merge.
            const u32 nl = sh.nlate;
            sort_list(ex, sh, B.lkL, B.liL, tk, ti, nl);
            if ((u32)(B.lkL[0] >> 32) >= X0) {
                ex.par([&](u32 t) {
                    const u32 base = sh.lsize;
                    for (u32 e = t; e < nl; e += NT) {
                        lk[base + e] = B.lkL[e];
                        li[base + e] = B.liL[e];
                    }
                });
                ex.par([&](u32 t) {
                    if (t == 0) {
                        sh.lsize += nl;
                        sh.nlate = 0;
                    }
                });
                if (stop) break;
                continue;
            }
            const u32 r0 = sh.lp, rn = sh.lsize - sh.lp;
            ex.par([&](u32 t) {
                for (u32 e = t; e < rn + nl; e += NT) {
                    u64 key;
                    u32 idv, lo, hi, base;
                    const u64* other;
                    if (e < rn) {
                        key = lk[r0 + e];
                        idv = li[r0 + e];
                        other = B.lkL;
                        lo = 0;
                        hi = nl;
                        base = e;
                    } else {
                        key = B.lkL[e - rn];
                        idv = B.liL[e - rn];
                        other = lk + r0;
                        lo = 0;
                        hi = rn;
                        base = e - rn;
                    }
                    while (lo < hi) {
                        const u32 md = (lo + hi) >> 1;
                        if (other[md] < key) lo = md + 1; else hi = md;
                    }
                    tk[base + lo] = key;
                    ti[base + lo] = idv;
                }
                if (t == 0) {
                    sh.lsize = rn + nl;
                    sh.lp = 0;
                    sh.nlate = 0;
                }
            });
            u64* xk = lk; lk = tk; tk = xk;
            u32* xi = li; li = ti; ti = xi;
        }
        if (stop) break;
        if (sh.next_sym - 256 > n) {  // impossible for a correct run (each rule removes >= 2 symbols)
            ex.par([&](u32 t) { if (t == 0) sh.err = RE_LOOP; });
            break;
        }
    }
    ex.mark(P_SER);
    // ---------------- serialise (PY:1889-1903): RP, 256, nrules, rules, len, seq ----------------
    const u32 R = sh.nrules;
    // final sequence length and ULEB bytes of the live symbols, per contiguous thread range
    const u32 cp = (n + NT - 1) / NT;
    ex.par([&](u32 t) {
        u32 bytes = 0, live = 0;
        const u32 e = (t + 1) * cp < n ? (t + 1) * cp : n;
        for (u32 i = t * cp; i < e; ++i)
            if (B.nd[i].sym != DEAD) {
                bytes += uleb_len(B.nd[i].sym);
                ++live;
            }
        sh.scan[t] = bytes;
        sh.scan2[t] = live;
    });
    ex.scan(sh.scan, &sh.total);
    const u32 seq_bytes = sh.total;
    ex.par([&](u32 t) {
        const u32 v = sh.scan[t];
        sh.scan[t] = sh.scan2[t];
        sh.scan2[t] = v;  // byte offset of thread t's symbols
    });
    ex.scan(sh.scan, &sh.total);
    const u32 L = sh.total;
    const u32 cr = (R + NT - 1) / NT;
    ex.par([&](u32 t) {
        u32 bytes = 0;
        const u32 e = (t + 1) * cr < R ? (t + 1) * cr : R;
        for (u32 r = t * cr; r < e; ++r) bytes += uleb_len((u32)(B.rules[r] >> 32)) + uleb_len((u32)B.rules[r]);
        sh.scan[t] = bytes;
    });
    ex.scan(sh.scan, &sh.total);
    const u32 rule_bytes = sh.total;
    const u32 head = 2 + 2 + uleb_len(R);
    const u64 size = (u64)head + rule_bytes + uleb_len(L) + seq_bytes;
    const bool fits = size <= B.out_cap && sh.err == RE_OK;
    if (fits) {
        ex.par([&](u32 t) {
            if (t == 0) {
                u8* o = B.out;
                o[0] = 'R';
                o[1] = 'P';
                u32 k = 2 + uleb_put(o + 2, 256);
                uleb_put(o + k, R);
                uleb_put(o + head + rule_bytes, L);
            }
            {
                u8* o = B.out + head + sh.scan[t];
                const u32 e = (t + 1) * cr < R ? (t + 1) * cr : R;
                for (u32 r = t * cr; r < e; ++r) {
                    o += uleb_put(o, (u32)(B.rules[r] >> 32));
                    o += uleb_put(o, (u32)B.rules[r]);
                }
            }
            {
                u8* o = B.out + head + rule_bytes + uleb_len(L) + sh.scan2[t];
                const u32 e = (t + 1) * cp < n ? (t + 1) * cp : n;
                for (u32 i = t * cp; i < e; ++i)
                    if (B.nd[i].sym != DEAD) o += uleb_put(o, B.nd[i].sym);
            }
        });
    }
    ex.par([&](u32 t) {
        if (t == 0) {
            B.result[RS_SIZE] = (u32)size;
            B.result[RS_RULES] = R;
            B.result[RS_FINAL] = L;
            B.result[RS_BATCHES] = sh.batch;
            B.result[RS_ERR] = sh.err != RE_OK ? sh.err : (fits ? RE_OK : RE_CAP);
            B.result[RS_LEVELS] = sh.levels;
        }
    });
}

}  // namespace rp
}  // namespace kolm
