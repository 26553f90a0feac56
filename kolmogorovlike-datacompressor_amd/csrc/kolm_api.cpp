// libkolm_hip.so — host orchestration + C ABI (include/kolm.h).
//
// One kolm_ctx per device owns a HIP stream and grow-only device scratch.  A batch runs
//   cheap sizes -> linear suffix sort (+ 3-gram chains) -> Lyndon factors -> cyclic
//   suffix sort -> BBWT gather -> MTF -> Rice sizes (5 variants) -> LZ77 match/parse ->
//   MDL argmin -> payload emission
// entirely on the device; the host only reads small per-round counters (to size the
// next launches) and the per-block results.  See DESIGN.md §2-§6.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <sys/mman.h>  // madvise (kolm_result_copy)
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kolm.h"
#include "kolm_internal.h"

using namespace kolm;

namespace kolm {
thread_local std::string g_err;  // kolm_last_error(); also set by kolm_toc.cpp
void set_err(const std::string& s) { g_err = s; }
}  // namespace kolm

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

// Host-side copy workers for the pinned staging buffers: a host buffer of the caller
// (pageable) is copied into pinned memory by several threads at once, so the DMA engine
// sees pinned memory and the host side keeps up with PCIe (one thread's memcpy does not).
class CopyPool {
  public:
    explicit CopyPool(unsigned n) {
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // dst[0, n) = src[0, n), split over the workers and the calling thread
    void copy(void* dst, const void* src, size_t n) {
        const size_t parts = th_.size() + 1, piece = ((n + parts - 1) / parts + 4095) & ~(size_t)4095;
        std::vector<Job> jobs;
        for (size_t o = piece; o < n; o += piece)
            jobs.push_back({(char*)dst + o, (const char*)src + o, std::min(piece, n - o)});
        {
            std::lock_guard<std::mutex> g(mu_);
            for (auto& j : jobs) q_.push_back(j);
            pending_ += jobs.size();
        }
        cv_.notify_all();
        std::memcpy(dst, src, std::min(piece, n));
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [this] { return pending_ == 0; });
    }

  private:
    struct Job {
        char* d;
        const char* s;
        size_t n;
    };
    void loop() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                j = q_.back();
                q_.pop_back();
            }
            std::memcpy(j.d, j.s, j.n);
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::vector<Job> q_;
    size_t pending_ = 0;
    bool stop_ = false;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
};

// counter slots in the device counter array
enum : int {
    C_CLS = 0,       // 12 slots
    C_NEXT = 12,
    C_EQ = 13,
    C_ACTIVE = 14,
    C_ALPHA = 15,    // round 0: max code width of the batch
    C_L0SEG = 16,
    C_L0TILE = 17,
    C_L1SEG = 18,
    C_L1TILE = 19,
    C_STATUS = 20,
    C_NLONG = 21,
    C_RICE = 22,
    C_NFIX = 23,     // LZ77 stitch fix-up tokens (statistics)
    C_CLSE = 24,     // 12 slots: elements per small class
    C_L0ELEM = 36,
    C_L1ELEM = 37,
    C_LMAX = 38,     // the round's longest large segment
    C_CDC = 40,      // FastCDC cut count
    C_N = 48,
    H_RSUM = C_N,    // host mirror only (2 words): summed per-block cyclic rounds
    H_ALPHA = C_N + 4,  // host mirror only: the batch's code width from the early alphabet pass
    H_N = C_N + 16
};

}  // namespace

struct kolm_ctx;
namespace {
// Records a HIP event pair around the launches in its scope (timing enabled only).
struct TScope {
    kolm_ctx* c;
    int fam;
    const char* name;  // kernel symbol (as rocprof shows it, namespaces stripped)
    u64 bytes;
    hipEvent_t a = nullptr;
    TScope(kolm_ctx* c_, int fam_, const char* name_, u64 bytes_);
    ~TScope() noexcept(false);
};
}  // namespace

struct kolm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // main stream
    hipStream_t aux = nullptr;     // second stream: Lyndon + cyclic sort chain runs beside LZ77
    hipStream_t active = nullptr;  // stream used by launches / TScope / sync()
    hipStream_t rp = nullptr;      // third stream: Re-Pair (candidate 9), one workgroup per block
    bool serial = false;           // every launch of a batch on one stream (kolm_ctx_set_serial; KOLM_SERIAL=1)
    // pinned host staging: an upload ring (input chunks) and the result buffer of
    // kolm_compress_fixed (container bytes, valid until the next call on this context)
    static constexpr int NSTAGE = 4;
    u8* stage[NSTAGE] = {};
    hipEvent_t stage_ev[NSTAGE] = {};
    u8* h_res = nullptr;
    size_t h_res_cap = 0, h_res_len = 0, h_res_off = 0;  // the container is h_res[off, off + len)
    hipStream_t up = nullptr, dl = nullptr;  // kolm_compress_fixed: upload / download streams
    hipEvent_t up_ev = nullptr;
    std::unique_ptr<CopyPool> pool;
    hipEvent_t evj[4] = {};        // join events
    hipEvent_t evr[2] = {};        // Re-Pair start / done
    hipEvent_t evg[2] = {};        // early BBWT gather: slots marked / gathered
    hipEvent_t eva = nullptr;      // the early alphabet pass's width copied to the host
    std::mutex mu;
    std::map<std::string, DevBuf> bufs;
    u32* h_cnt = nullptr;  // pinned mirror of the counters
    // fine-grained (coherent) host words small device results are stored into by k_spans_to_host
    // (read_spans below): RT_WORDS result words, then one sequence word per wave
    u32* h_rt = nullptr;
    u32* d_rt = nullptr;  // the same buffer as the device addresses it
    u32 rt_seq = 0;
    // pinned landing buffer of a batch's packed small results (one device-to-host copy per
    // host round trip instead of one per array: each copy is a blit launch of ~15-25 us)
    u32* h_tail = nullptr;
    size_t h_tail_cap = 0;
    u32* tail_host(size_t words) {
        if (words > h_tail_cap) {
            if (h_tail) KOLM_HIP_CHECK(hipHostFree(h_tail));
            h_tail = nullptr;
            h_tail_cap = 0;
            const size_t cap = std::max<size_t>(words + (words >> 2), 4096);
            KOLM_HIP_CHECK(hipHostMalloc((void**)&h_tail, cap * sizeof(u32), hipHostMallocDefault));
            h_tail_cap = cap;
        }
        return h_tail;
    }
    hipEvent_t ev[8] = {};
    // per-launch timing of kernel families (kolm_ctx_set_timing)
    bool timing = false;
    std::vector<hipEvent_t> evpool;
    size_t evused = 0;
    struct Pend {
        int fam;
        const char* name;
        hipEvent_t a, b;
        u64 bytes;
        int strm;  // 0 index stream, 1 sort stream, 2 Re-Pair stream
    };
    int strm_of(hipStream_t s) const { return s == aux ? 1 : s == rp ? 2 : 0; }
    std::vector<Pend> pend;
    struct Acc {
        double ms = 0;
        u64 launches = 0, bytes = 0;
        int fam = 0;   // KOLM_KT_* family of the kernel
        int strm = 0;  // stream of its last launch (Pend::strm)
    };
    std::map<std::string, Acc> kacc;  // per kernel, accumulated while timing is enabled
    // KTimer for multi-kernel launchers: events on the active stream, nested scopes allowed
    struct Hook : KTimer {
        kolm_ctx* c = nullptr;
        struct Open {
            int fam;
            const char* name;
            u64 bytes;
            hipEvent_t a;
        };
        std::vector<Open> open;
        void begin(int fam, const char* name, u64 bytes) override {
            hipEvent_t a = c->ev_take();
            KOLM_HIP_CHECK(hipEventRecord(a, c->active));
            open.push_back({fam, name, bytes, a});
        }
        void end() override {
            Open o = open.back();
            open.pop_back();
            hipEvent_t b = c->ev_take();
            KOLM_HIP_CHECK(hipEventRecord(b, c->active));
            c->pend.push_back({o.fam, o.name, o.a, b, o.bytes, c->strm_of(c->active)});
        }
    } hook;
    KTimer* kt() {
        hook.c = this;
        return timing ? &hook : nullptr;
    }
    hipEvent_t ev_take() {
        if (evused == evpool.size()) {
            hipEvent_t e;
            KOLM_HIP_CHECK(hipEventCreate(&e));
            evpool.push_back(e);
        }
        return evpool[evused++];
    }
    void timing_reset() {
        pend.clear();
        evused = 0;
    }
    void timing_collect(kolm_stats* st) {
        for (auto& p : pend) {
            float ms = 0;
            KOLM_HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
            st->kt[p.fam].ms += ms;
            st->kt[p.fam].launches += 1;
            st->kt[p.fam].bytes += p.bytes;
            Acc& a = kacc[p.name];
            a.fam = p.fam;
            a.strm = p.strm;
            a.ms += ms;
            a.launches += 1;
            a.bytes += p.bytes;
        }
        timing_reset();
    }

    void* raw(const char* name, size_t bytes) {
        DevBuf& b = bufs[name];
        if (bytes == 0) bytes = 16;
        if (b.cap < bytes) {
            if (b.p) KOLM_HIP_CHECK(hipFree(b.p));
            b.p = nullptr;
            const size_t cap = (bytes + 255) & ~(size_t)255;
            KOLM_HIP_CHECK(hipMalloc(&b.p, cap));
            b.cap = cap;
        }
        return b.p;
    }
    template <class T>
    T* get(const char* name, size_t count) {
        return static_cast<T*>(raw(name, count * sizeof(T)));
    }
    u64 bytes_held(const char* name) const {
        const auto it = bufs.find(name);
        return it == bufs.end() ? 0 : it->second.cap;
    }
    // Small device results back to the host (the doubling rounds' counters, the batch's
    // offsets / winners / sizes): k_spans_to_host stores the spans into coherent host memory
    // and then each wave's sequence word (system-scope release), and the host spins on those
    // words — no blit dispatch and no stream query between the last kernel and the host's next
    // launch.  A stream error, or a finished stream without the words, ends the wait with an
    // error.  Returns the spans' words (h_rt[o[k] + j]).
    static constexpr u32 RT_WORDS = 16384;  // h_rt: RT_WORDS result words, then 4 sequence words
    const u32* read_spans(const kolm::PackSpans& ps, hipStream_t s) {
        const u32 seq = ++rt_seq;
        const u32 waves = kolm::launch_spans_to_host(ps, d_rt, d_rt + RT_WORDS, seq, s);
        volatile u32* f = h_rt + RT_WORDS;
        for (u32 w = 0, it = 1; w < waves; ++it) {
            if (f[w] == seq) {
                ++w;
                continue;
            }
            if (it % 1024 == 0) {
                const hipError_t e = hipStreamQuery(s);
                if (e != hipErrorNotReady) {
                    KOLM_HIP_CHECK(e);
                    if (f[w] != seq)
                        throw kolm::HipError(hipErrorUnknown, "result words not seen after the stream finished", __LINE__);
                }
            }
            __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return h_rt;
    }
    static bool fits_rt(const kolm::PackSpans& ps) {
        u64 end = 0;
        for (int k = 0; k < 6; ++k)
            if (ps.p[k]) end = std::max<u64>(end, (u64)ps.o[k] + ps.n[k]);
        return end <= RT_WORDS;
    }
    void read_counts(u32* h, const u32* cnt, u32 n, hipStream_t s) {
        kolm::PackSpans ps{};
        ps.p[0] = cnt, ps.n[0] = n, ps.o[0] = 0;
        const volatile u32* r = read_spans(ps, s);
        for (u32 i = 0; i < n; ++i) h[i] = r[i];
    }
    // Host round trips (per-round counters) spin on the stream instead of sleeping in
    // hipStreamSynchronize: the sort stream idles for the host's wake-up otherwise.
    void sync() {
        static const bool block = getenv("KOLM_SYNC_BLOCK") && atoi(getenv("KOLM_SYNC_BLOCK"));
        if (block) {
            KOLM_HIP_CHECK(hipStreamSynchronize(active));
            return;
        }
        hipError_t e;
        while ((e = hipStreamQuery(active)) == hipErrorNotReady) {
        }
        KOLM_HIP_CHECK(e);
    }
};

namespace kolm {
int ctx_device(const kolm_ctx* c) { return c->device; }
}  // namespace kolm

namespace {

TScope::TScope(kolm_ctx* c_, int fam_, const char* name_, u64 bytes_) : c(c_), fam(fam_), name(name_), bytes(bytes_) {
    if (c->timing) {
        a = c->ev_take();
        KOLM_HIP_CHECK(hipEventRecord(a, c->active));
    }
}
TScope::~TScope() noexcept(false) {
    if (c->timing) {
        hipEvent_t b = c->ev_take();
        KOLM_HIP_CHECK(hipEventRecord(b, c->active));
        c->pend.push_back({fam, name, a, b, bytes, c->strm_of(c->active)});
    }
}

std::mutex g_mu;
kolm_ctx* g_default = nullptr;
std::vector<kolm_ctx*> g_multi;  // per-device contexts of kolm_encode_blocks_multi

u32 bitlen(u32 v) { return v ? 32 - __builtin_clz(v) : 0; }

// kernel symbols as rocprof shows them: [32-bit sort words][class]
const char* const kSmallSortName[2][NCLASS] = {
    {"k_single", "k_small_sort<1, unsigned long>", "k_small_sort<2, unsigned long>",
     "k_small_sort<3, unsigned long>", "k_small_sort<4, unsigned long>", "k_small_sort<5, unsigned long>",
     "k_small_sort<6, unsigned long>", "k_small_sort<7, unsigned long>", "k_small_sort<8, unsigned long>",
     "k_small_sort<9, unsigned long>", "k_small_sort<10, unsigned long>", "k_small_sort<11, unsigned long>"},
    {"k_single", "k_small_sort<1, unsigned int>", "k_small_sort<2, unsigned int>", "k_small_sort<3, unsigned int>",
     "k_small_sort<4, unsigned int>", "k_small_sort<5, unsigned int>", "k_small_sort<6, unsigned int>",
     "k_small_sort<7, unsigned int>", "k_small_sort<8, unsigned int>", "k_small_sort<9, unsigned int>",
     "k_small_sort<10, unsigned int>", "k_small_sort<11, unsigned int>"}};

struct SortOut {
    u32 rounds = 0;
    u64 active = 0;
    u32 r0_chars = 0;  // cyclic: rotation characters of round 0
};

// Segmented prefix-doubling suffix sort of every block of the batch (k_sort.hip).
// after_round0 (optional) runs on the host right after round 0 is enqueued (cyclic pass),
// before the pass waits for its counts: encode_batch hooks the LZ77 launch there.
// at_round (optional) runs on the host once round r's segment list `cur` is classified (its
// device count at ncur_dev, at most `bound`), before the round's sorts are enqueued.
using RoundHook = std::function<void(u32 round, const Seg* cur, u32 bound, const u32* ncur_dev)>;
// alpha_ready (optional): the batch's code tables were built by launch_alpha_async before Lyndon
// (on another stream, the width in h_cnt[H_ALPHA] once the event completes), so round 0 starts
// without a host round trip of its own
SortOut sort_pass(kolm_ctx* c, const Geom& geo, const u8* text, bool cyclic, Factors fac, const u8* FEd,
                  const std::function<void()>& after_round0 = {}, const RoundHook& at_round = {},
                  hipEvent_t alpha_ready = nullptr) {
    hipStream_t s = c->active;
    const u64 N = geo.N;
    SortOut out;
    SortArgs a{};
    a.geo = geo;
    a.text = text;
    a.SA = c->get<u32>("SA", N);
    a.RK = c->get<u32>("RK", N);
    a.K2 = c->get<u32>("K2", N);
    a.SA2 = c->get<u32>("SA2", N);
    a.K22 = c->get<u32>("K22", N);
    a.fac = fac;
    a.FEd = FEd;
    a.blk_split = c->get<u32>("blk_split", geo.nb);
    u32* blk_done = c->get<u32>("blk_done", geo.nb);
    a.blk_done = blk_done;
    u32* blk_last = c->get<u32>("blk_last", geo.nb);
    a.cyclic = cyclic ? 1 : 0;
    // large groups of at most MED_T elements: one-workgroup LDS sort instead of the MSD levels
    // (KOLM_MED_SORT=0: every large group through the MSD levels)
    // (batches of fewer than 64 blocks: its ~118 KiB of LDS — one workgroup per CU, needs the
    // 160 KiB LDS of gfx950 — would wait for the LZ77 parse's workgroups on a full batch, whose
    // large groups are few anyway — 256 MiB text: 41.8 vs 37.5 ms per step with it)
    static const int med = getenv("KOLM_MED_SORT") ? atoi(getenv("KOLM_MED_SORT")) : -1;
    a.med = (med > 0 || (med < 0 && geo.nb < 64)) ? 1u : 0u;
    a.cls_chunk = 1u;  // k_classify: one contiguous list share per workgroup (1.36 -> 1.29 ms per step)

    u32* cnt = c->get<u32>("counters", C_N);
    Lists L{};
    for (int k = 0; k < NCLASS; ++k) {
        const u64 cap = (k == 0 ? N : N / ((1ull << (k - 1)) + 1)) + 16;
        char nm[16];
        snprintf(nm, sizeof nm, "cls%d", k);
        L.cls[k] = c->get<Seg>(nm, cap);
    }
    L.cls_cnt = cnt + C_CLS;
    // the next list's length, double-buffered in device memory: round r appends to slot
    // r & 1 while its classify reads slot (r - 1) & 1, so the host launches round r + 1
    // without waiting for round r's count (the classify grid covers a bound instead)
    u32* ncnt = c->get<u32>("next_cnt2", 2);
    const u32* ncur_dev = nullptr;
    L.eq_cnt = cnt + C_EQ;
    L.misc = cnt + C_ACTIVE;
    L.cls_elems = cnt + C_CLSE;
    L.lmax = cnt + C_LMAX;
    L.eq = c->get<Seg>("eq", N / TILE + 16);
    const u64 seg_cap = N / 2 + geo.nb + 16;
    Seg* segA = c->get<Seg>("segA", seg_cap);
    Seg* segB = c->get<Seg>("segB", seg_cap);
    const u64 lseg_cap = N / TILE + 16;
    const u64 ltile_cap = 2 * (N / TILE) + 16;
    Level lv[2];
    lv[0] = Level{c->get<LSeg>("lseg0", lseg_cap), cnt + C_L0SEG, c->get<LTile>("ltile0", ltile_cap), cnt + C_L0TILE,
                  cnt + C_L0ELEM};
    lv[1] = Level{c->get<LSeg>("lseg1", lseg_cap), cnt + C_L1SEG, c->get<LTile>("ltile1", ltile_cap), cnt + C_L1TILE,
                  cnt + C_L1ELEM};
    u32* hist = c->get<u32>("hist", ltile_cap * 256);

    if (!cyclic) {
        launch_iota(a.SA, N, s);
        launch_block_segs(segA, geo, s);
    }
    KOLM_HIP_CHECK(hipMemsetAsync(blk_done, 0, sizeof(u32) * geo.nb, s));
    if (cyclic) KOLM_HIP_CHECK(hipMemsetAsync(blk_last, 0, sizeof(u32) * geo.nb, s));
    Seg* cur = segA;
    Seg* nxt = segB;
    u32 ncur = geo.nb;
    // cyclic: round 0 sorts by C rotation characters (alphabet-compacted codes, launch_alpha),
    // the doubling rounds continue at h = C
    u32 h0 = cyclic ? 8 : 3;
    const u32 kb_rank = bitlen(geo.bs) ? bitlen(geo.bs) : 1;
    u32* h = c->h_cnt;
    static const bool dbg = getenv("KOLM_DEBUG_ROUNDS") != nullptr;
    // KOLM_DEBUG_ROUNDS: per-round class counts and wall time (the round ends at a host sync)
    auto t_round = std::chrono::steady_clock::now();
    auto round_done = [&](u32 r) {
        if (!dbg) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[kolm] %s round %u: %.3f ms\n", cyclic ? "cyc" : "lin", r,
                std::chrono::duration<double, std::milli>(now - t_round).count());
        t_round = now;
    };
    // classes 1..tiny_c: one thread per segment (k_tiny_sort); larger: LDS sorts.  Class 5
    // (17-32 elements) goes to the LDS sort: k_tiny_sort<5> holds 32 64-bit words in 144
    // VGPRs and was starved beside the LZ77 parse (1.0 ms alone, 3.0 overlapped; step 45.7
    // -> 44.0 ms); class 4 to the LDS sort as well measured 41.8-41.9 -> 42.0-42.1 ms
    constexpr int tiny_c = 4;
    // the end-of-round k_update_done (cyclic) runs inside the next round's k_zero_spans, which
    // zeroes the split flags it reads (one launch less per round)
    int pend_done = -1;
    for (u32 round = 0; round < 64 && ncur; ++round) {
        a.initial = round == 0 ? 1 : 0;
        a.h = round == 0 ? 0u : (h0 << (round - 1));
        // round 0: packed characters (cyclic 32 bits, linear 27); later: ranks (+1 linear)
        a.key_bits = a.initial ? (cyclic ? 32u : 27u) : bitlen(cyclic ? geo.bs - 1 : geo.bs);
        L.next = nxt;
        L.next_cnt = ncnt + (round & 1);
        // the round's counters, split flags and (position-ordered lists) classify bins in one
        // launch: hipMemsetAsync fills are ~4.5 us kernels each on the sort stream (config 5:
        // 151 per batch, 0.68 ms)
        const bool zero_bins = !(round == 0 && cyclic);
        {
            ZeroSpans z{};
            z.p[0] = L.next_cnt;
            z.n[0] = 1;
            z.p[1] = cnt;
            z.n[1] = C_STATUS;
            z.p[2] = cnt + C_CLSE;
            z.n[2] = C_N - C_CLSE;
            z.p[3] = a.blk_split;
            z.n[3] = (u32)geo.nb;
            if (pend_done >= 0) {  // the previous round's done / last update rides on this launch
                z.done = blk_done;
                z.last = blk_last;
                z.round = (u32)pend_done;
                pend_done = -1;
            }
            if (round == 0 && cyclic && !alpha_ready) {
                // the alphabet pass's presence bits (its width word cnt[C_ALPHA] is in span 1)
                z.p[4] = c->get<u32>("r0pres", (u64)geo.nb * 8);
                z.n[4] = (u32)geo.nb * 8;
            }
            if (zero_bins) {
                z.p[4] = c->get<u32>("cls_bins", NCLASS * CLS_NBIN);
                z.n[4] = NCLASS * CLS_NBIN;
                z.p[5] = c->get<u32>("cls_fill", NCLASS * CLS_NBIN);
                z.n[5] = NCLASS * CLS_NBIN;
            }
            launch_zero_spans(z, s);
        }
        if (round == 0 && cyclic) {
            // round 0: stable LSD passes over the packed codes of the first C rotation
            // characters (alphabet-compacted codes), no host round trips but one
            const u64 nt = lsd_tiles(geo) + 1;
            u8* code = c->get<u8>("r0code", (u64)geo.nb * 256);
            u32 w;
            if (alpha_ready) {
                KOLM_HIP_CHECK(hipStreamWaitEvent(s, alpha_ready, 0));
                KOLM_HIP_CHECK(hipEventSynchronize(alpha_ready));
                w = alpha_width(h[H_ALPHA]);
            } else {
                // the width back through the counter flag (no fills, no blit, no blocking sync)
                launch_alpha_async(geo, text, c->get<u32>("r0pres", (u64)geo.nb * 8), code, cnt + C_ALPHA, nullptr,
                                   s, c->kt(), true);
                c->read_counts(h + C_ALPHA, cnt + C_ALPHA, 1, s);
                w = alpha_width(h[C_ALPHA]);
            }
            const u32 C = std::max<u32>(1, std::min<u32>(32, 64 / w));
            h0 = C;
            R0Bufs r{text, FEd, fac, code, C, w, c->get<u32>("KP", N), a.K2, a.SA, a.K22, a.SA2, a.RK,
                     c->get<u32>("r0hist", nt * 256), c->get<u32>("r0tmax", nt), c->get<u32>("r0tmin", nt),
                     c->get<u32>("r0cmax", nt), c->get<u32>("r0cmin", nt), c->get<u32>("r0hf", nt * WG),
                     c->get<u32>("r0swc", (u64)2 * geo.nb * 16 * 256)};
            r.rec[0] = c->get<u64>("r0rec0", N);
            r.rec[1] = c->get<u64>("r0rec1", N);
            out.r0_chars = C;
            if (dbg) fprintf(stderr, "[kolm] round 0: %u characters of %u bits\n", C, w);
            launch_round0(geo, r, nxt, L.next_cnt, a.blk_split, s, c->kt());
            out.active += N;
            out.rounds = 1;
            pend_done = 0;  // folded into the next round's k_zero_spans
            if (after_round0) {
                after_round0();
                c->active = s;
            }
            round_done(round);
            ncur = (u32)std::min<u64>(N / 2 + geo.nb, 0xFFFFFFFFu);  // bound: segments hold >= 2
            ncur_dev = L.next_cnt;
            std::swap(cur, nxt);
            continue;
        }
        {
            // position-ordered class lists
            TScope t(c, KOLM_KT_CLASSIFY, "k_classify", (u64)ncur * 24);
            const u32 nbits = bitlen((u32)(N - 1));
            const Bins bn{c->get<u32>("cls_bins", NCLASS * CLS_NBIN), c->get<u32>("cls_fill", NCLASS * CLS_NBIN),
                          nbits > 10 ? nbits - 10 : 0u};
            launch_classify_bins(cur, ncur, ncur_dev, a, L, lv[0], bn, s, zero_bins);
            a.xcd = 1;
        }
        c->read_counts(h, cnt, C_N, s);
        if (h[C_ACTIVE] == 0) break;
        out.active += h[C_ACTIVE];
        out.rounds = round + 1;
        if (dbg) {
            fprintf(stderr, "[kolm] round %u h=%u active=%u large: segs %u elems %u | class segs/elems:", round, a.h,
                    h[C_ACTIVE], h[C_L0SEG], h[C_L0ELEM]);
            for (int k = 0; k < NCLASS; ++k) fprintf(stderr, " %d:%u/%u", k, h[C_CLS + k], h[C_CLSE + k]);
            fprintf(stderr, "\n");
        }
        if (at_round) {
            at_round(round, cur, ncur, ncur_dev);
            c->active = s;
        }
        {
            // Dense rounds: keys by position first (sequential pass), then one gather per
            // slot; sparse rounds gather the key inputs per active slot directly.
            a.KP = nullptr;
            constexpr u64 ddiv = 8;  // dense when more than 1/8 of the positions are active
            if ((u64)h[C_ACTIVE] * ddiv > N) {
                u32* KP = c->get<u32>("KP", N);
                // cyclic: FEd 1 + RK 4 + KP 4 (factor starts only within h of a factor end); linear: RK 4 + KP 4
                TScope t(c, KOLM_KT_KEYGEN, "k_keypos", N * (cyclic ? 9 : 8));
                launch_keypos(a, KP, s);
                a.KP = KP;
            }
            // algorithmic bytes per element: SA read + key inputs + K2 write
            const u64 per = a.KP ? 12 : a.initial ? (cyclic ? 20 : 11) : (cyclic ? 20 : 12);
            KgClasses kc{};
            u64 kg_elems = 0;
            for (int k = 1; k < NCLASS; ++k) {
                kc.segs[k] = L.cls[k];
                if (!h[C_CLS + k]) continue;
                if (a.KP && k <= tiny_c) continue;  // k_tiny_sort gathers KP itself
                kc.count[k] = h[C_CLS + k];
                kg_elems += h[C_CLSE + k];
            }
            if (kg_elems) {
                TScope t(c, KOLM_KT_KEYGEN, "k_keygen_small", kg_elems * per);
                launch_keygen_small(kc, a, s);
            }
            if (h[C_L0TILE]) {
                TScope t(c, KOLM_KT_KEYGEN, "k_keygen_large", (u64)h[C_L0ELEM] * per);
                launch_keygen_large(lv[0].tiles, h[C_L0TILE], lv[0].segs, a, s);
            }
        }
        // MSD levels of the large segments, one per 8-bit digit down to the last, with no host
        // round trip between them: level 0's counts are known here, later levels read theirs
        // from device memory under bounds (a level's large buckets hold > TILE elements each
        // and at most the elements of level 0: nseg <= nelem / TILE, ntiles <= 2 nelem / TILE)
        const u32 nelem0 = h[C_L0ELEM], nseg0 = h[C_L0SEG], ntiles0 = h[C_L0TILE];
        u32 hi = a.initial ? (cyclic ? 32u : 27u) : kb_rank;
        int lvl = 0;
        if (a.med && nseg0 && h[C_LMAX] <= MED_T) {
            // every large group fits the medium sort: one launch, no MSD level (its runs go to
            // the next round's list directly, so the class counts stay as classify left them)
            TScope t(c, KOLM_KT_SMALLSORT, "k_small_sort<13> (medium)", (u64)nelem0 * 16);
            launch_med_sort(lv[0].segs, nseg0, lv[0].nseg, a, L, s);
            hi = 0;
        }
        for (; nseg0 && hi; ++lvl) {
            const u32 width = std::min<u32>(8, hi);
            const u32 shift = hi - width;
            const bool last = shift == 0;
            Level& lc = lv[lvl & 1];
            Level& ln = lv[(lvl + 1) & 1];
            const u32 nseg = lvl ? nelem0 / TILE + 1 : nseg0;
            const u32 ntiles = lvl ? 2 * (nelem0 / TILE) + 1 : ntiles0;
            const u32* dseg = lvl ? lc.nseg : nullptr;
            const u32* dtile = lvl ? lc.ntiles : nullptr;
            {
                // the next level's three counters in one launch (three fill kernels before)
                ZeroSpans zl{};
                zl.p[0] = ln.nseg, zl.n[0] = 1;
                zl.p[1] = ln.ntiles, zl.n[1] = 1;
                zl.p[2] = ln.nelem, zl.n[2] = 1;
                launch_zero_spans(zl, s);
            }
            if (a.med) {
                TScope t(c, KOLM_KT_SMALLSORT, "k_small_sort<13> (medium)", (u64)nelem0 * 16);
                launch_med_sort(lc.segs, nseg, lc.nseg, a, L, s);
            }
            {
                TScope t(c, KOLM_KT_MSD, "k_msd_hist", (u64)nelem0 * 4 + (u64)ntiles0 * 1024);
                launch_msd_hist(lc.tiles, ntiles, dtile, lc.segs, a, shift, width, hist, s);
            }
            {
                TScope t(c, KOLM_KT_MSD, "k_msd_scan", (u64)ntiles0 * 1024 * 3);
                launch_msd_scan(lc.segs, nseg, dseg, a, width, hist, last, L, ln, s);
            }
            {
                TScope t(c, KOLM_KT_MSD, "k_msd_scatter", (u64)nelem0 * 16 + (u64)ntiles0 * 1024);
                launch_msd_scatter(lc.tiles, ntiles, dtile, lc.segs, a, shift, width, hist, s);
            }
            {
                TScope t(c, KOLM_KT_MSD, "k_copy_back", (u64)nelem0 * 16);
                launch_copy_back(lc.tiles, ntiles, dtile, lc.segs, a, s);
            }
            hi = shift;
        }
        if (lvl) c->read_counts(h, cnt, C_N, s);  // the MSD levels appended segments to the class lists
        // per element: K2 + SA read, SA + RK write (16 B); per segment record 8 B.  (Round 6
        // measured and removed: the classes' sorts split over the sort stream and a second one —
        // 33.31-33.36 -> 33.58-33.59 ms per step, config 5 6.07 -> 6.27 ms.)
        // (Round 6 measured and removed: classes 1..4 in one launch — merged, the kernel holds the
        // largest class's registers, 38-60 VGPRs against 20-34 for classes 1-3 alone, and beside the
        // LZ77 parse that cost the 256 MiB step 33.1-33.3 -> 35.7-35.8 ms)
        for (int k = 0; k < NCLASS; ++k) {
            if (!h[C_CLS + k]) continue;
            if (k >= 1 && k <= tiny_c) {
                static const char* const tn[6] = {"",          "k_tiny_sort<1>", "k_tiny_sort<2>",
                                                  "k_tiny_sort<3>", "k_tiny_sort<4>", "k_tiny_sort<5>"};
                // SA + key (KP gather or K2) read, SA + RK write per element; 8 B per segment
                TScope t(c, KOLM_KT_SMALLSORT, tn[k], (u64)h[C_CLSE + k] * 16 + (u64)h[C_CLS + k] * 8);
                launch_tiny_sort(k, L.cls[k], h[C_CLS + k], a, L, s);
                continue;
            }
            if (k >= 5) continue;  // classes 5..11: below, one launch per sort-word width
            const int w32 = a.key_bits + k <= 31 ? 1 : 0;  // matches small_sort_c's choice
            TScope t(c, KOLM_KT_SMALLSORT, kSmallSortName[w32][k], (u64)h[C_CLSE + k] * 16 + (u64)h[C_CLS + k] * 8);
            launch_small_sort(k, L.cls[k], h[C_CLS + k], a, L, s);
        }
        for (int w32 = 1; w32 >= 0; --w32) {
            // classes 5..11 in one launch per sort-word width (k_small_sort_all; one launch per
            // class before: up to 7 short grids per round)
            SsClasses sc{};
            u64 els = 0, segs = 0;
            for (int k = 5; k < NCLASS; ++k) {
                sc.segs[k] = L.cls[k];
                if (!h[C_CLS + k] || (a.key_bits + k <= 31 ? 1 : 0) != w32) continue;
                sc.count[k] = h[C_CLS + k];
                els += h[C_CLSE + k];
                segs += h[C_CLS + k];
            }
            if (!segs) continue;
            TScope t(c, KOLM_KT_SMALLSORT, w32 ? "k_small_sort_all<u32>" : "k_small_sort_all<u64>", els * 16 + segs * 8);
            launch_small_sorts(sc, w32 != 0, a, L, s);
        }
        if (h[C_EQ]) {
            TScope t(c, KOLM_KT_SMALLSORT, "k_finalize_eq", (u64)h[C_EQ] * TILE * 8);
            launch_finalize_eq(L.eq, h[C_EQ], a, L, s);
        }
        if (cyclic) pend_done = (int)round;  // folded into the next round's k_zero_spans
        round_done(round);
        // the next list holds unresolved segments of >= 2 active elements each
        ncur = (u32)std::min<u64>(h[C_ACTIVE] / 2 + geo.nb, N / 2 + geo.nb);
        ncur_dev = L.next_cnt;
        std::swap(cur, nxt);
    }
    if (pend_done >= 0) launch_update_done(blk_done, blk_last, a.blk_split, geo.nb, (u32)pend_done, s);
    if (cyclic) launch_rounds_sum(blk_last, geo.nb, c->get<u64>("rsum", 1), s);
    return out;
}

struct Pipeline {
    kolm_ctx* c;
    Geom geo;
    const u8* text;
    kolm_stats st{};
    float t_sa = 0, t_lz = 0, t_ent = 0, t_emit = 0;

    // Lyndon factorisation of every block -> factor-start lists + FEd (on the active stream)
    void lyndon() {
        const u64 N = geo.N;
        const u64 ntiles = (u64)((geo.bs + TILE - 1) / TILE) * geo.nb + 16;
        const u64 nch = (geo.bs + duval_span_bytes(geo) - 1) / duval_span_bytes(geo) * (u64)geo.nb + 1;
        launch_lyndon(geo, text, c->get<u8>("flag", N), c->get<u8>("FEd", N),
                      c->get<u32>("lyn_fstart", N), c->get<uint4>("lyn_fpre", nch * 128),
                      c->get<u32>("lyn_nfac", nch), c->get<u32>("lyn_stack", N), c->get<u32>("lyn_fcount", geo.nb + 1), c->get<u32>("lyn_t1", 2 * ntiles + 16),
                      c->active, c->kt());
    }
    Factors factors() { return Factors{c->get<u32>("lyn_stack", geo.N), c->get<u32>("lyn_fcount", geo.nb + 1)}; }
    // omega-order of all rotations of the Lyndon factors + BBWT gather -> "bbwt"
    // cyclic predecessor byte of every position (needs the Lyndon factors only)
    hipEvent_t prevc_ready = nullptr;  // set when prevc() ran on another stream
    void prevc() {
        const u64 N = geo.N;
        TScope t(c, KOLM_KT_LYNDON, "k_prevc", N * 3);  // flag 1 + text 1 + prevc 1 (+ factor starts)
        launch_prevc(geo, text, c->get<u8>("flag", N), factors(), c->get<u8>("prevc", N), c->active);
    }
    // early_gather: the encode path allows the early BBWT gather on the third stream (idle:
    // no Re-Pair, prevc computed on another stream)
    bool early_gather = false;
    hipEvent_t alpha_ready = nullptr;  // set when the alphabet pass ran early (launch_alpha_async)
    u8* cyclic(const std::function<void()>& after_round0 = {}, u8* out = nullptr) {
        const u64 N = geo.N;
        if (!out) out = c->get<u8>("bbwt", N);
        u8* prevc = c->get<u8>("prevc", N);
        u32* SA = c->get<u32>("SA", N);
        // Early BBWT gather (bbwt_early_round() = R > 0): once doubling round R's segments are
        // classified, every slot outside them holds its final SA entry, so the third stream
        // gathers every slot's BBWT byte beside the remaining rounds (and the LZ77 parse), and
        // the slots of round R's segments — whose early bytes may be stale — are gathered
        // again after the last round
        const u32 er = early_gather && prevc_ready ? bbwt_early_round() : 0u;
        bool early = false;
        const RoundHook hook = [&](u32 round, const Seg* cur, u32 bound, const u32* ncur_dev) {
            if (early || round != er) return;
            hipStream_t s = c->active, x = c->rp;
            u64* bm = c->get<u64>("bbwt_bm", (N + 63) / 64);
            KOLM_HIP_CHECK(hipMemsetAsync(bm, 0, sizeof(u64) * ((N + 63) / 64), s));
            launch_mark_active(cur, ncur_dev, bound, bm, s);
            KOLM_HIP_CHECK(hipEventRecord(c->evg[0], s));
            KOLM_HIP_CHECK(hipStreamWaitEvent(x, c->evg[0], 0));
            KOLM_HIP_CHECK(hipStreamWaitEvent(x, prevc_ready, 0));
            c->active = x;
            {
                TScope t(c, KOLM_KT_LYNDON, "k_bbwt_gather (early)", N * 6);
                launch_bbwt_gather(geo, SA, prevc, out, x);
            }
            KOLM_HIP_CHECK(hipEventRecord(c->evg[1], x));
            c->active = s;
            early = true;
        };
        SortOut cyc = sort_pass(c, geo, text, true, factors(), c->get<u8>("FEd", N), after_round0,
                                er ? hook : RoundHook{}, alpha_ready);
        if (early) {
            KOLM_HIP_CHECK(hipStreamWaitEvent(c->active, c->evg[1], 0));
            TScope t(c, KOLM_KT_LYNDON, "k_bbwt_gather", N / 8 + N / 16);  // the mask + about 1/16 of the slots
            launch_bbwt_gather_masked(geo, SA, prevc, out, c->get<u64>("bbwt_bm", (N + 63) / 64), c->active);
        } else {
            if (prevc_ready)
                KOLM_HIP_CHECK(hipStreamWaitEvent(c->active, prevc_ready, 0));
            else
                this->prevc();
            TScope t(c, KOLM_KT_LYNDON, "k_bbwt_gather", N * 6);  // SA 4 + prevc 1 + out 1
            launch_bbwt_gather(geo, SA, prevc, out, c->active);
        }
        st.cyc_rounds = cyc.rounds;
        st.cyc_active = cyc.active;
        return out;
    }
    u8* bbwt() {
        lyndon();
        return cyclic();
    }

    u8* mtf(const u8* in, u64* bits = nullptr) {
        const u64 N = geo.N;
        const u32 csz = mtf_chunk_bytes(geo);
        const u64 nch = (u64)((geo.bs + csz - 1) / csz) * geo.nb + 1;
        u8* out = c->get<u8>("mtf", N);
        launch_mtf(geo, in, out, c->get<u8>("mtf_sum", nch * 256), c->get<u16>("mtf_cnt", nch),
                   c->get<u8>("mtf_states", nch * 256), c->active, c->kt(), bits, 2,
                   c->get<u32>("mtf_cp", mtf_cp_words(geo)));
        return out;
    }

    LzArgs lz_args() {
        const u64 N = geo.N;
        LzArgs z{};
        z.geo = geo;
        z.text = text;
        z.tok_pos = c->get<u32>("tok_pos", N);
        z.tok_len = c->get<u32>("tok_len", N);
        z.tok_dist = c->get<u32>("tok_dist", N);
        z.tok_off = c->get<u32>("tok_off", N);
        z.fix_pos = c->get<u32>("fix_pos", N);
        z.fix_len = c->get<u32>("fix_len", N);
        z.fix_dist = c->get<u32>("fix_dist", N);
        z.fix_off = c->get<u32>("fix_off", N);
        z.cshift = lz_chunk_shift();
        z.cpb = (geo.bs + (1u << z.cshift) - 1) >> z.cshift;
        const u64 nch = (u64)z.cpb * geo.nb + 1;
        z.c_ntok = c->get<u32>("c_ntok", nch);
        z.c_exit = c->get<u32>("c_exit", nch);
        z.c_bytes = c->get<u32>("c_bytes", nch);
        z.c_first = c->get<u32>("c_first", nch);
        z.c_fix0 = c->get<u32>("c_fix0", nch);
        z.c_nfix = c->get<u32>("c_nfix", nch);
        z.c_fixbytes = c->get<u32>("c_fixbytes", nch);
        z.c_off = c->get<u32>("c_off", nch);
        z.b_nfix = c->get<u32>("b_nfix", geo.nb);
        z.ntok = c->get<u32>("ntok", geo.nb);
        z.lz_size = c->get<u32>("lz_size", geo.nb);
        z.nlong = c->get<u32>("counters", C_N) + C_NLONG;
        z.nfix = c->get<u32>("counters", C_N) + C_NFIX;
        static const bool lz_prof = getenv("KOLM_LZ_PROF") && atoi(getenv("KOLM_LZ_PROF")) != 0;
        if (lz_prof) z.prof = c->get<u64>("lz_prof", 32);
        z.stitch_runs = 1u;
        z.rank = c->get<u16>("lz_rank", N + 16);
        z.tcnt = c->get<u16>("lz_tcnt", (u64)geo.nb * ((geo.bs + LZL_HOME - 1) / LZL_HOME) * 1024 + 16);
        return z;
    }

    void lz(const LzArgs& z) {
        KOLM_HIP_CHECK(hipMemsetAsync(z.nlong, 0, sizeof(u32), c->active));
        KOLM_HIP_CHECK(hipMemsetAsync(z.nfix, 0, sizeof(u32), c->active));
        if (z.prof) KOLM_HIP_CHECK(hipMemsetAsync(z.prof, 0, sizeof(u64) * 32, c->active));
        launch_lz_parse(z, c->active, c->kt());
    }
};

float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    KOLM_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int check_geom(u64 N, u32 bs) {
    if (N >= (1ull << 31)) {
        set_err("batch larger than 2^31-1 bytes");
        return KOLM_EARG;
    }
    if (bs == 0 || bs > (1u << 25)) {
        set_err("block size must be in [1, 32 MiB]");
        return KOLM_EARG;
    }
    return KOLM_OK;
}

// Content-defined blocks: hb[0] = 0, strictly increasing, total < 2^31, blocks <= 32 MiB.
int check_bounds(const u32* hb, u32 nb) {
    if (hb[0] != 0) {
        set_err("block bounds must start at 0");
        return KOLM_EARG;
    }
    for (u32 b = 0; b < nb; ++b)
        if (hb[b + 1] <= hb[b] || hb[b + 1] - hb[b] > (1u << 25)) {
            set_err("blocks must be non-empty, contiguous and at most 32 MiB");
            return KOLM_EARG;
        }
    if (hb[nb] >= (1u << 31)) {
        set_err("batch larger than 2^31-1 bytes");
        return KOLM_EARG;
    }
    return KOLM_OK;
}

// Candidate 10 (k_v2.hip): sizes of every block; U / L (planes and their BBWTs) stay
// resident for the emission.
struct V2State {
    u8* U = nullptr;    // [8N] bit planes, plane block (b, j) at 8*base(b) + j*len(b)
    u8* L = nullptr;    // [8N] their BBWTs
    u32* pb = nullptr;  // [8nb + 1] plane block bounds (device)
    u32* meta = nullptr;
    u32* size = nullptr;
};

bool v2_stage(kolm_ctx* c, const Geom& geo, const u8* d_text, hipStream_t s, V2State& v) {
    const u64 N = geo.N;
    const u32 nb = geo.nb;
    if (8 * N >= (1ull << 32)) {
        set_err("v2_new (candidate 10): batches up to 512 MiB");
        return false;
    }
    v.U = c->get<u8>("v2U", 8 * N + 64);
    v.L = c->get<u8>("v2L", 8 * N + 64);
    u32* sel = c->get<u32>("v2sel", nb);
    launch_v2_sizes(geo, d_text, c->get<u32>("v2hist", (u64)nb * 13 * 256), sel, v.U, s, c->kt());
    // plane block bounds
    std::vector<u32> hb(8 * (u64)nb + 1);
    for (u32 b = 0; b < nb; ++b) {
        const u32 base = geo.base(b), len = geo.end(b) - base;
        for (u32 j = 0; j < 8; ++j) hb[8 * (u64)b + j] = 8 * base + j * len;
    }
    hb[8 * (u64)nb] = (u32)(8 * N);
    v.pb = c->get<u32>("v2pb", 8 * (u64)nb + 1);
    KOLM_HIP_CHECK(hipMemcpyAsync(v.pb, hb.data(), sizeof(u32) * hb.size(), hipMemcpyHostToDevice, s));
    // BBWT of the planes in groups of blocks (< 2^28 plane positions per group)
    for (u32 b0 = 0; b0 < nb;) {
        u32 b1 = b0 + 1;
        while (b1 < nb && (u64)hb[8 * (u64)(b1 + 1)] - hb[8 * (u64)b0] <= (1ull << 28)) ++b1;
        const u32 nq = 8 * (b1 - b0);
        std::vector<u32> gb(nq + 1);
        for (u32 i = 0; i <= nq; ++i) gb[i] = hb[8 * (u64)b0 + i] - hb[8 * (u64)b0];
        Geom pg;
        const u32 vs = geom_var_shift(gb.data(), nq);
        geom_init_var(pg, gb.data(), nq, c->get<u32>("v2vb", (u64)nq + 1), c->get<u32>("v2vmap", (gb[nq] >> vs) + 2), vs, s);
        Pipeline P{c, pg, v.U + hb[8 * (u64)b0]};
        c->active = s;
        P.lyndon();
        P.cyclic({}, v.L + hb[8 * (u64)b0]);
        b0 = b1;
    }
    u64* rbits = c->get<u64>("v2rbits", 8 * (u64)nb * 16);
    u32* b1v = c->get<u32>("v2b1", 8 * (u64)nb);
    launch_v2_runs(8 * nb, v.pb, v.L, rbits, b1v, s, c->kt(), 8 * N);
    v.meta = c->get<u32>("v2meta", (u64)nb * V2_META);
    v.size = c->get<u32>("v2size", nb);
    launch_v2_size(geo, sel, rbits, b1v, v.meta, v.size, s);
    return true;
}

// Full batch: sizes of candidates 0..10, MDL, emission into d_arena.  Fixed blocks of bs
// bytes over [0, N), or (h_bounds != null) the nbv content-defined blocks
// [h_bounds[i], h_bounds[i+1]) (PY:2213 compress_blocks_cdc).
int encode_batch(kolm_ctx* c, const u8* d_text, u64 N, u32 bs, const u32* h_bounds, u32 nbv, u32 mask,
                 const int32_t* h_force, u8* d_arena, u64 arena_cap, u32* h_sizes, u32* h_method, u64* h_off,
                 kolm_stats* stats) {
    Geom geo;
    if (h_bounds) {
        if (int e = check_bounds(h_bounds, nbv)) return e;
        N = h_bounds[nbv];
        const u32 vs = geom_var_shift(h_bounds, nbv);
        geom_init_var(geo, h_bounds, nbv, c->get<u32>("vb", (u64)nbv + 1), c->get<u32>("vmap", (N >> vs) + 2), vs,
                      c->stream);
        bs = geo.bs;
    } else {
        if (int e = check_geom(N, bs)) return e;
        geom_init(geo, N, bs);
    }
    const u32 nb = geo.nb;
    if (nb == 0) {
        if (h_off) h_off[0] = 0;
        if (stats) *stats = kolm_stats{};
        return KOLM_OK;
    }
    // every argument check before the first launch: an error return never leaves work in flight
    if (((mask >> KOLM_M_V2NEW) & 1u) && 8 * N >= (1ull << 32)) {
        set_err("v2_new (candidate 10): batches up to 512 MiB");
        return KOLM_EARG;
    }
    if (((mask >> KOLM_M_REPAIR) & 1u) && bs > RP_MAX_N) {
        set_err("Re-Pair (candidate 9) supports blocks up to 4 MiB (KOLM_REPAIR_MAX_BLOCK)");
        return KOLM_EARG;
    }
    // Two streams: the index stream (main) runs the xor/lfsr size counters, the BBWT
    // predecessor bytes and the LZ77 parse (k_lz_local + stitch); the sort stream (aux,
    // higher priority: the critical path) runs the Lyndon factorisation, the cyclic sort,
    // BBWT, MTF and the Rice sizes, joins LZ77 and finishes MDL + emission.
    // KOLM_SERIAL=1 runs everything on one stream (profiling); KOLM_OVERLAP selects when
    // LZ77 starts: 0 (default) at once, 1 after the Lyndon factorisation, 2 after round 0 of
    // the cyclic sort.  With the 8-character round 0 (eight streaming LSD passes beside the
    // LDS-bound parse): 53.8-54.2 ms per 256 MiB for 0, 54.1-54.2 for 1, 55.4-56.2 for 2.
    const bool serial = c->serial;
    // (the MSD round 0's LDS bucket sorts need whole CUs: the parse starts after round 0 there)
    hipStream_t ms = c->stream, s = serial ? c->stream : c->aux;
    Pipeline P{c, geo, d_text};
    hipEvent_t* ev = c->ev;
    hipEvent_t* ej = c->evj;
    c->timing_reset();
    struct Restore {
        kolm_ctx* c;
        ~Restore() { c->active = c->stream; }
    } restore{c};
    // per-block size counters: xor / lfsr from the text on the index stream, the Rice
    // candidates from the MTF replay on the sort stream
    u64* d_bits = c->get<u64>("bits", (u64)nb * 8);
    KOLM_HIP_CHECK(hipMemsetAsync(d_bits, 0, sizeof(u64) * 8 * nb, ms));
    KOLM_HIP_CHECK(hipEventRecord(ev[0], ms));
    // Re-Pair (candidate 9): persistent workgroups (one per block) on their own stream,
    // launched first so they take their CUs while the sort / LZ77 chains queue beside them
    const bool want_rp = (mask >> KOLM_M_REPAIR) & 1u;
    RpArgs rpa{};
    if (want_rp) {
        rpa.geo = geo;
        rpa.text = d_text;
        rpa.ws_stride = repair_ws_bytes(bs);
        rpa.out_stride = 4ull * bs + 64;
        rpa.out = c->get<u8>("rp_out", (u64)nb * rpa.out_stride);
        rpa.result = c->get<u32>("rp_res", (u64)nb * RP_RS_N);
        static const bool rp_prof = getenv("KOLM_RP_PROF") && atoi(getenv("KOLM_RP_PROF")) != 0;
        if (rp_prof) {
            rpa.prof = c->get<u64>("rp_prof", (u64)nb * RP_P_N);
            KOLM_HIP_CHECK(hipMemsetAsync(rpa.prof, 0, sizeof(u64) * nb * RP_P_N, c->rp));
        }
        static const char* rp_trace = getenv("KOLM_RP_TRACE");
        if (rp_trace && *rp_trace) {
            rpa.trace = c->get<u32>("rp_trace", (u64)RP_TR_CAP * RP_TR_W);
            KOLM_HIP_CHECK(hipMemsetAsync(rpa.trace, 0, sizeof(u32) * RP_TR_CAP * RP_TR_W, c->rp));
        }
        // Blocks run in groups whose workspaces fit the budget (~258 MB per 1 MiB block);
        // a second group serialises behind the first, so the default budget is most of the
        // device memory still free (KOLM_RP_WS_GB overrides), not a fixed figure: 3/4 of
        // what is free (the workspace already held counts as free) after the rest of the
        // batch's scratch (about 96 B per position for the sort / LZ77 / emission arrays,
        // minus what this context already holds) is set aside.
        u64 budget;
        if (getenv("KOLM_RP_WS_GB")) {
            budget = (u64)(atof(getenv("KOLM_RP_WS_GB")) * (double)(1ull << 30));
        } else {
            size_t fr = 0, total = 0;
            KOLM_HIP_CHECK(hipMemGetInfo(&fr, &total));
            const u64 held_rp = c->bytes_held("rp_ws");
            u64 held_other = 0;
            for (const auto& kv : c->bufs)
                if (kv.first != "rp_ws") held_other += kv.second.cap;
            const u64 need_other = 96 * N > held_other ? 96 * N - held_other : 0;
            const u64 avail = fr + held_rp > need_other ? fr + held_rp - need_other : 0;
            budget = (u64)(avail * 0.75);
        }
        const u32 group = (u32)std::max<u64>(1, std::min<u64>(nb, budget / rpa.ws_stride));
        rpa.ws = c->get<char>("rp_ws", (u64)group * rpa.ws_stride);
        KOLM_HIP_CHECK(hipStreamWaitEvent(c->rp, ev[0], 0));
        KOLM_HIP_CHECK(hipEventRecord(c->evr[1], c->rp));
        c->active = c->rp;
        for (u32 b0 = 0; b0 < nb; b0 += group) {
            const u32 k = std::min(group, nb - b0);
            TScope t(c, KOLM_KT_REPAIR, "k_repair", (u64)(geo.end(b0 + k - 1) - geo.base(b0)) * 9);
            launch_repair(rpa, b0, k, c->rp);
        }
        KOLM_HIP_CHECK(hipEventRecord(c->evr[0], c->rp));
    }
    KOLM_HIP_CHECK(hipStreamWaitEvent(s, ev[0], 0));
    c->active = s;
    P.lyndon();
    KOLM_HIP_CHECK(hipEventRecord(ev[5], s));
    // Batches of fewer than 64 blocks: the xor / lfsr sizes and (below) the BBWT's predecessor
    // bytes go to the third stream when Re-Pair does not use it, so the LZ77 parse at the head of
    // the index stream starts at once instead of behind them (prevc waits for the Lyndon factors):
    // config 4's 32-block shard 6.30 -> 6.20-6.27 ms.  On full batches the early parse competes
    // with Lyndon and round 0 (256 MiB: 34.5 -> 35.2 ms), so they keep the index-stream order.
    // KOLM_SIDE_STREAM = 0 / 1 forces it.
    static const int side_env = getenv("KOLM_SIDE_STREAM") ? atoi(getenv("KOLM_SIDE_STREAM")) : -1;
    const bool side = (side_env >= 0 ? side_env != 0 : nb < 64) && !serial && !want_rp;
    hipStream_t xs = side ? c->rp : ms;
    // Round 0's alphabet (per-block code tables + the batch's code width, one host read) on the
    // side / index stream beside Lyndon instead of on the sort stream after it: the host reads the
    // width while Lyndon runs, and round 0 follows Lyndon without a round trip of its own
    if (nb < 64) {
        c->active = xs;
        launch_alpha_async(geo, d_text, c->get<u32>("r0pres", (u64)nb * 8), c->get<u8>("r0code", (u64)nb * 256),
                           c->get<u32>("r0w", 1), c->h_cnt + H_ALPHA, xs, c->kt());
        KOLM_HIP_CHECK(hipEventRecord(c->eva, xs));
        P.alpha_ready = c->eva;
    }
    const bool want_lz = (mask >> KOLM_M_LZ77) & 1u || (h_force != nullptr);
    LzArgs z = P.lz_args();
    // (k_lz_tiles, the tile index of the parse's forms 1 / 2, runs right before the parse: placed
    // ahead of the prevc wait or first on the index stream it measured no better)
    if (side) KOLM_HIP_CHECK(hipStreamWaitEvent(c->rp, ev[0], 0));
    c->active = xs;
    {
        EmitArgs ce{};
        ce.geo = geo;
        ce.text = d_text;
        ce.bits = d_bits;
        TScope t(c, KOLM_KT_SIZES, "k_cheap_sizes", N);
        launch_cheap_sizes(ce, xs);
    }
    // The BBWT gather's predecessor bytes on the index stream, off the sort chain — but
    // prevc waits for the Lyndon factors, and the LZ77 parse queued behind it on that stream
    // waits too.  Batches of under 16 blocks, where LZ77 (the stitch's one-wave-per-block
    // walk) is as long as the sort chain, run prevc inline on the sort stream (~15 us per
    // MiB) so the parse starts at once: BASELINE config 2 2.15 -> 1.90 ms, config 5 6.55 ->
    // 6.21 ms; config 4's 32-block shard measured 6.84 -> 7.30 ms that way (the parse then
    // competes with Lyndon and round 0 for CUs), so it keeps the index-stream form.
    // KOLM_PREVC_IDX = 0 / 1 forces it.
    const int prevc_idx = getenv("KOLM_PREVC_IDX") ? atoi(getenv("KOLM_PREVC_IDX")) : -1;  // read per call (tests)
    if (!serial && (prevc_idx >= 0 ? prevc_idx != 0 : nb >= 16)) {
        KOLM_HIP_CHECK(hipStreamWaitEvent(xs, ev[5], 0));
        P.prevc();
        KOLM_HIP_CHECK(hipEventRecord(ev[6], xs));
        P.prevc_ready = ev[6];
    }
    if (side) KOLM_HIP_CHECK(hipEventRecord(ev[7], xs));  // the sizes, joined before the MDL
    c->active = ms;
    KOLM_HIP_CHECK(hipEventRecord(ej[0], ms));
    auto launch_lz = [&] {
        c->active = ms;
        KOLM_HIP_CHECK(hipEventRecord(ej[2], ms));
        if (want_lz) P.lz(z);
        KOLM_HIP_CHECK(hipEventRecord(ej[1], ms));
    };
    u8* bw = nullptr;
    P.early_gather = !serial && !want_rp;  // the third stream is free for the early BBWT gather
    // The parse starts at once (behind prevc on full batches); started after Lyndon or after round
    // 0 it measured 0-0.4 / 1.5-2 ms slower (rounds 3-4) and 0.9-2.2 ms slower in round 6 (§4)
    launch_lz();
    c->active = s;
    bw = P.cyclic();
    P.early_gather = false;
    // per-block doubling rounds of the omega-order sort (R per block)
    KOLM_HIP_CHECK(hipMemcpyAsync(c->h_cnt + H_RSUM, c->get<u64>("rsum", 1), sizeof(u64), hipMemcpyDeviceToHost, s));
    KOLM_HIP_CHECK(hipEventRecord(ev[1], s));
    u8* mt = P.mtf(bw, d_bits);
    EmitArgs e{};
    e.geo = geo;
    e.text = d_text;
    e.mtf = mt;
    e.sizes = c->get<u32>("sizes", (u64)nb * KOLM_NCAND);
    e.bits = d_bits;
    e.method = c->get<u32>("method", nb);
    int32_t* d_force = nullptr;
    if (h_force) {
        d_force = c->get<int32_t>("force", nb);
        KOLM_HIP_CHECK(hipMemcpyAsync(d_force, h_force, sizeof(int32_t) * nb, hipMemcpyHostToDevice, s));
    }
    e.force = d_force;
    e.cand_mask = mask;
    e.off = c->get<u64>("off", nb + 1);
    e.arena = d_arena;
    e.arena_cap = arena_cap;
    const u64 ntiles = (u64)((geo.bs + TILE - 1) / TILE) * nb + 16;
    e.tile_tmp = c->get<u32>("tile_tmp", 2 * ntiles + 16);
    e.tile_tmp2 = c->get<u32>("tile_tmp2", 2 * ntiles + 2 * nb + 16);
    e.rice_k = 2;
    // candidate 10 (v2_new, opt-in): automaton + bit planes, the BBWT of every plane by the
    // same pipeline (groups of blocks whose 8 planes stay below 2^28 positions), runs and
    // Rice sizes; the plane BBWTs reuse the sort scratch (the blocks' own sort is done)
    const bool want_v2 = (mask >> KOLM_M_V2NEW) & 1u;
    V2State v2{};
    std::map<std::string, size_t> caps_before_v2;
    if (want_v2) {
        // the plane sorts reuse the sort scratch at up to 8x the batch's positions: the
        // buffers they grow are reallocated here, so the sort stream's own work on them
        // is drained first (the LZ77 / Re-Pair streams use none of them), and they are
        // released again once the batch is complete (hot-path batches keep their size)
        KOLM_HIP_CHECK(hipStreamSynchronize(s));
        for (const auto& kv : c->bufs) caps_before_v2[kv.first] = kv.second.cap;
        if (!v2_stage(c, geo, d_text, s, v2)) return KOLM_EARG;
    }
    KOLM_HIP_CHECK(hipEventRecord(ev[2], s));
    KOLM_HIP_CHECK(hipStreamWaitEvent(s, ej[1], 0));
    KOLM_HIP_CHECK(hipEventRecord(ev[3], s));
    u32* cnt = c->get<u32>("counters", C_N);
    KOLM_HIP_CHECK(hipMemsetAsync(cnt + C_STATUS, 0, sizeof(u32), s));
    if (want_rp) KOLM_HIP_CHECK(hipStreamWaitEvent(s, c->evr[0], 0));
    if (side) KOLM_HIP_CHECK(hipStreamWaitEvent(s, ev[7], 0));
    {
        TScope t(c, KOLM_KT_SIZES, "k_mdl+offsets", (u64)nb * 120);
        launch_mdl(e, want_lz ? z.lz_size : nullptr, want_rp ? rpa.result : nullptr, want_v2 ? v2.size : nullptr,
                   cnt + C_STATUS, s);
    }
    std::vector<u64> off(nb + 1);
    std::vector<u32> rpres(want_rp ? (u64)nb * RP_RS_N : 0), win(nb);
    {
        // offsets, winners, counters (and Re-Pair results) in one packed copy
        PackSpans ps{};
        const u32 w_off = 2 * (nb + 1), w_win = nb, w_rp = (u32)rpres.size();
        ps.p[0] = reinterpret_cast<const u32*>(e.off), ps.n[0] = w_off, ps.o[0] = 0;
        ps.p[1] = e.method, ps.n[1] = w_win, ps.o[1] = w_off;
        ps.p[2] = cnt, ps.n[2] = C_N, ps.o[2] = w_off + w_win;
        ps.p[3] = rpa.result, ps.n[3] = w_rp, ps.o[3] = w_off + w_win + C_N;
        const u32 words = w_off + w_win + C_N + w_rp;
        const u32* htail;
        if (kolm_ctx::fits_rt(ps)) {
            htail = c->read_spans(ps, s);  // straight into coherent host memory
        } else {
            u32* dtail = c->get<u32>("tail", words);
            u32* ht = c->tail_host(words);
            launch_pack_spans(ps, dtail, s);
            KOLM_HIP_CHECK(hipMemcpyAsync(ht, dtail, sizeof(u32) * words, hipMemcpyDeviceToHost, s));
            c->sync();
            htail = ht;
        }
        std::memcpy(off.data(), htail, sizeof(u64) * (nb + 1));
        std::memcpy(win.data(), htail + w_off, sizeof(u32) * nb);
        std::memcpy(c->h_cnt, htail + w_off + w_win, sizeof(u32) * C_N);
        if (w_rp) std::memcpy(rpres.data(), htail + w_off + w_win + C_N, sizeof(u32) * w_rp);
    }
    if (want_rp && rpa.prof) {
        // per-section wall-clock of the Re-Pair kernel (100 MHz ticks), summed over blocks
        std::vector<u64> pr((u64)nb * RP_P_N);
        KOLM_HIP_CHECK(hipMemcpy(pr.data(), rpa.prof, sizeof(u64) * pr.size(), hipMemcpyDeviceToHost));
        static const char* const nm[RP_P_N] = {"init", "lvscan", "lvsort", "window", "gather", "chains",
                                               "select", "applyA", "applyB", "late", "serialise", "applyA2"};
        fprintf(stderr, "[kolm] Re-Pair sections, ms per block (mean over %u blocks):", nb);
        for (u32 k = 0; k < RP_P_N; ++k) {
            u64 t = 0;
            for (u32 b = 0; b < nb; ++b) t += pr[(u64)b * RP_P_N + k];
            fprintf(stderr, " %s %.2f", nm[k], (double)t / nb / 1e5);
        }
        // spread of the per-block totals (the kernel lasts as long as its slowest block)
        std::vector<double> tb(nb, 0.0);
        for (u32 b = 0; b < nb; ++b)
            for (u32 k = 0; k < RP_P_N; ++k) tb[b] += (double)pr[(u64)b * RP_P_N + k] / 1e5;
        std::vector<double> so = tb;
        std::sort(so.begin(), so.end());
        if (nb) {
            u32 bmax = 0;
            for (u32 b = 0; b < nb; ++b) if (tb[b] > tb[bmax]) bmax = b;
            fprintf(stderr, " | block total ms min %.2f median %.2f max %.2f (block %u)", so[0], so[nb / 2], so[nb - 1], bmax);
        }
        fprintf(stderr, "\n");
    }
    if (want_rp && rpa.trace) {
        // per-batch records of block 0 (debug): raw u32 words, RP_TR_W per loop iteration
        std::vector<u32> tr((u64)RP_TR_CAP * RP_TR_W);
        KOLM_HIP_CHECK(hipMemcpy(tr.data(), rpa.trace, sizeof(u32) * tr.size(), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("KOLM_RP_TRACE"), "wb")) {
            fwrite(tr.data(), sizeof(u32), tr.size(), f);
            fclose(f);
        }
    }
    for (u32 b = 0; b < (want_rp ? nb : 0); ++b)
        if (rpres[(u64)b * RP_RS_N + RP_RS_ERR]) {
            char msg[128];
            snprintf(msg, sizeof msg, "Re-Pair internal error %u in block %u", rpres[(u64)b * RP_RS_N + RP_RS_ERR], b);
            set_err(msg);
            return KOLM_EHIP;
        }
    if (c->h_cnt[C_STATUS] || off[nb] + 4 > arena_cap) {
        set_err("payload arena too small");
        return KOLM_ECAP;
    }
    {
        // only the emitters of methods some block chose (the winners are on the host now)
        u32 used = 0;
        for (u32 m : win) used |= 1u << std::min<u32>(m, 31);
        TScope t(c, KOLM_KT_EMIT, "emit", N + 2 * off[nb]);
        KOLM_HIP_CHECK(hipMemsetAsync(d_arena, 0, (off[nb] + 8) & ~(u64)3, s));
        if (used & ((1u << KOLM_M_RAW) | (1u << KOLM_M_XOR) | (1u << KOLM_M_LFSR))) launch_emit_simple(e, s);
        if (used & (0x1Fu << KOLM_M_BBWT)) launch_emit_rice(e, s);
        if (want_lz && (used & (1u << KOLM_M_LZ77))) launch_lz_emit(z, e.method, e.off, d_arena, s);
        if (want_rp && (used & (1u << KOLM_M_REPAIR))) launch_rp_emit(rpa, e.method, e.off, d_arena, s);
        if (want_v2 && (used & (1u << KOLM_M_V2NEW))) launch_v2_emit(geo, v2.pb, v2.meta, e.method, e.off, v2.U, v2.L, d_arena, s);
    }
    KOLM_HIP_CHECK(hipEventRecord(ev[4], s));
    std::vector<u32> ntok(want_lz ? nb : 0);
    {
        // sizes, counters and LZ77 token counts in one packed copy (the winners are on the host)
        PackSpans ps{};
        const u32 w_sz = h_sizes ? nb * KOLM_NCAND : 0, w_nt = (u32)ntok.size();
        ps.p[0] = e.sizes, ps.n[0] = w_sz, ps.o[0] = 0;
        ps.p[1] = cnt, ps.n[1] = C_N, ps.o[1] = w_sz;
        ps.p[2] = z.ntok, ps.n[2] = w_nt, ps.o[2] = w_sz + C_N;
        const u32 words = w_sz + C_N + w_nt;
        const u32* htail;
        if (kolm_ctx::fits_rt(ps)) {
            htail = c->read_spans(ps, s);  // straight into coherent host memory
        } else {
            u32* dtail = c->get<u32>("tail", words);
            u32* ht = c->tail_host(words);
            launch_pack_spans(ps, dtail, s);
            KOLM_HIP_CHECK(hipMemcpyAsync(ht, dtail, sizeof(u32) * words, hipMemcpyDeviceToHost, s));
            c->sync();
            htail = ht;
        }
        if (h_sizes) std::memcpy(h_sizes, htail, sizeof(u32) * w_sz);
        if (h_method) std::memcpy(h_method, win.data(), sizeof(u32) * nb);
        std::memcpy(c->h_cnt, htail + w_sz, sizeof(u32) * C_N);
        if (w_nt) std::memcpy(ntok.data(), htail + w_sz + C_N, sizeof(u32) * w_nt);
    }
    if (want_v2) {
        KOLM_HIP_CHECK(hipDeviceSynchronize());
        for (auto& kv : c->bufs) {
            const auto it = caps_before_v2.find(kv.first);
            if (kv.second.p && (it == caps_before_v2.end() || kv.second.cap > it->second)) {
                KOLM_HIP_CHECK(hipFree(kv.second.p));
                kv.second = DevBuf{};
            }
        }
    }
    if (h_off) std::memcpy(h_off, off.data(), sizeof(u64) * (nb + 1));
    if (want_lz && z.prof) {
        u64 pr[32];
        KOLM_HIP_CHECK(hipMemcpy(pr, z.prof, sizeof pr, hipMemcpyDeviceToHost));
        const double nwg = pr[6] ? (double)pr[6] : 1.0;
        fprintf(stderr, "[kolm] k_lz_local us per workgroup: load %.2f sort %.2f index %.2f parse %.2f; "
                "wave token steps %.1f, candidate batches %.1f per wave (%llu workgroups)\n",
                pr[0] / nwg / 100.0, pr[1] / nwg / 100.0, pr[2] / nwg / 100.0, pr[3] / nwg / 100.0,
                pr[4] / nwg / 4.0, pr[5] / nwg / 4.0, (unsigned long long)pr[6]);
        fprintf(stderr, "[kolm] k_lz_stitch_l: %llu fix-up searches %.1f us, %llu unresolved re-searches %.1f us, "
                "%llu chunks walked token by token, max block %.1f us; re-search exact lengths: %.1f us, %llu bytes\n",
                (unsigned long long)pr[8], pr[9] / 100.0, (unsigned long long)pr[10], pr[11] / 100.0,
                (unsigned long long)pr[13], pr[12] / 100.0, pr[14] / 100.0, (unsigned long long)pr[15]);
        fprintf(stderr, "[kolm] re-search loop: %llu distance batches, %llu candidates, %llu capped, %llu extended "
                "(%llu longer) over %llu bytes in %.1f us\n", (unsigned long long)pr[16], (unsigned long long)pr[17],
                (unsigned long long)pr[18], (unsigned long long)pr[19], (unsigned long long)pr[22],
                (unsigned long long)pr[20], pr[21] / 100.0);
        fprintf(stderr, "[kolm] re-search phases: loop %.1f us, fingerprints %.1f us, %llu window loads %.1f us\n",
                pr[25] / 100.0, pr[23] / 100.0, (unsigned long long)pr[26], pr[24] / 100.0);
    }
    u64 tokens = 0;
    for (u32 v : ntok) tokens += v;
    if (stats) {
        kolm_stats& st = *stats;
        st = P.st;
        st.lz_tokens = tokens;
        c->timing_collect(&st);
        st.kt[KOLM_KT_LZPARSE].bytes += tokens * 16;
        if (c->timing && want_lz) c->kacc[lz_spec_name()].bytes += tokens * 16;  // token records
        st.lz_long = c->h_cnt[C_NLONG];
        st.lz_fix = c->h_cnt[C_NFIX];
        std::memcpy(&st.cyc_rounds_sum, c->h_cnt + H_RSUM, sizeof(u64));
        st.ms_sa = ev_ms(ev[0], ev[1]);
        st.ms_entropy = ev_ms(ev[1], ev[2]);
        st.ms_lz = ev_ms(ej[2], ej[1]);
        st.ms_emit = ev_ms(ev[3], ev[4]);
        st.ms_total = ev_ms(ev[0], ev[4]);
        if (want_rp) {
            st.ms_repair = ev_ms(c->evr[1], c->evr[0]);
            for (u32 b = 0; b < nb; ++b) {
                st.rp_rules += rpres[(u64)b * RP_RS_N + RP_RS_RULES];
                st.rp_batches += rpres[(u64)b * RP_RS_N + RP_RS_BATCHES];
                st.rp_final += rpres[(u64)b * RP_RS_N + RP_RS_FINAL];
            }
        }
    }
    return KOLM_OK;
}

template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const HipError& e) {
        char buf[256];
        snprintf(buf, sizeof buf, "HIP error %d (%s) at kolm_api line %d: %s", (int)e.err,
                 hipGetErrorString(e.err), e.line, e.what);
        set_err(buf);
        return KOLM_EHIP;
    } catch (const std::bad_alloc&) {
        set_err("host allocation failed");
        return KOLM_EHIP;
    }
}

int ctx_create(int device, kolm_ctx** out) {
    return guarded([&] {
        int n = 0;
        KOLM_HIP_CHECK(hipGetDeviceCount(&n));
        if (device < 0 || device >= n) {
            set_err("no such HIP device");
            return KOLM_EARG;
        }
        KOLM_HIP_CHECK(hipSetDevice(device));
        std::unique_ptr<kolm_ctx> c(new kolm_ctx);
        c->device = device;
        {
            // the sort chain (aux) is the critical path: give it the higher priority so its
            // workgroups dispatch ahead of the LZ77 stream (equal priorities and the LZ77 stream
            // higher measured slower, rounds 2-3)
            int lo = 0, hi = 0;
            KOLM_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            KOLM_HIP_CHECK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, lo));
            KOLM_HIP_CHECK(hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, hi));
        }
        KOLM_HIP_CHECK(hipStreamCreateWithFlags(&c->rp, hipStreamNonBlocking));
        c->active = c->stream;
        c->serial = getenv("KOLM_SERIAL") && atoi(getenv("KOLM_SERIAL")) != 0;
        for (auto& e : c->evj) KOLM_HIP_CHECK(hipEventCreate(&e));
        for (auto& e : c->evr) KOLM_HIP_CHECK(hipEventCreate(&e));
        for (auto& e : c->evg) KOLM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        KOLM_HIP_CHECK(hipEventCreateWithFlags(&c->eva, hipEventDisableTiming));
        KOLM_HIP_CHECK(hipHostMalloc((void**)&c->h_cnt, sizeof(u32) * H_N, hipHostMallocDefault));
        KOLM_HIP_CHECK(hipHostMalloc((void**)&c->h_rt, sizeof(u32) * (kolm_ctx::RT_WORDS + 64),
                                    hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(c->h_rt, 0, sizeof(u32) * (kolm_ctx::RT_WORDS + 64));
        KOLM_HIP_CHECK(hipHostGetDevicePointer((void**)&c->d_rt, c->h_rt, 0));
        for (auto& e : c->ev) KOLM_HIP_CHECK(hipEventCreate(&e));
        *out = c.release();
        return KOLM_OK;
    });
}

kolm_ctx* need_default() {
    std::lock_guard<std::mutex> g(g_mu);
    return g_default;
}

// Upload n host bytes to the context's "text" buffer (+64 bytes of zero padding).
u8* upload(kolm_ctx* c, const uint8_t* in, size_t n) {
    u8* d = c->get<u8>("text", n + 64);
    if (n) KOLM_HIP_CHECK(hipMemcpyAsync(d, in, n, hipMemcpyHostToDevice, c->stream));
    KOLM_HIP_CHECK(hipMemsetAsync(d + n, 0, 64, c->stream));
    return d;
}

// a += b for the statistics of consecutive batches of one call: counts and times add up,
// round counts take the maximum (first: a = b)
void stats_add(kolm_stats& a, const kolm_stats& b, bool first) {
    if (first) {
        a = b;
        return;
    }
    a.lin_rounds = std::max(a.lin_rounds, b.lin_rounds);
    a.cyc_rounds = std::max(a.cyc_rounds, b.cyc_rounds);
    a.lin_active += b.lin_active;
    a.cyc_active += b.cyc_active;
    a.cyc_rounds_sum += b.cyc_rounds_sum;
    a.lz_tokens += b.lz_tokens;
    a.lz_long += b.lz_long;
    a.lz_fix += b.lz_fix;
    a.ms_total += b.ms_total;
    a.ms_sa += b.ms_sa;
    a.ms_lz += b.ms_lz;
    a.ms_entropy += b.ms_entropy;
    a.ms_emit += b.ms_emit;
    a.ms_repair += b.ms_repair;
    a.rp_rules += b.rp_rules;
    a.rp_batches += b.rp_batches;
    a.rp_final += b.rp_final;
    for (int k = 0; k < KOLM_NKT; ++k) {
        a.kt[k].ms += b.kt[k].ms;
        a.kt[k].launches += b.kt[k].launches;
        a.kt[k].bytes += b.kt[k].bytes;
    }
}

constexpr size_t STAGE_BYTES = 32u << 20;

CopyPool& copy_pool(kolm_ctx* c) {
    if (!c->pool) {
        // hardware_concurrency() may be 0 (unknown): at least one worker, at most 7
        const unsigned hc = std::max(2u, std::thread::hardware_concurrency());
        c->pool.reset(new CopyPool(std::min(8u, hc) - 1));
    }
    return *c->pool;
}

// The same upload from pageable memory through a ring of pinned chunks: the copy workers
// fill chunk k + 1 while the DMA engine moves chunk k (hipMemcpy from pageable memory
// stages through the runtime's own buffers at about half the PCIe rate).
u8* upload_staged(kolm_ctx* c, const uint8_t* in, size_t n, u8* d = nullptr, hipStream_t st = nullptr) {
    if (!d) d = c->get<u8>("text", n + 64);
    if (!st) st = c->stream;
    CopyPool& pool = copy_pool(c);
    for (size_t o = 0, k = 0; o < n; o += STAGE_BYTES, ++k) {
        const int j = (int)(k % kolm_ctx::NSTAGE);
        if (!c->stage[j]) {
            KOLM_HIP_CHECK(hipHostMalloc((void**)&c->stage[j], STAGE_BYTES, hipHostMallocDefault));
            KOLM_HIP_CHECK(hipEventCreateWithFlags(&c->stage_ev[j], hipEventDisableTiming));
        } else {
            // the chunk's previous copy — of this call or of an earlier piece's call, whose
            // DMA may still be reading it — has left (normally long complete: no wait)
            KOLM_HIP_CHECK(hipEventSynchronize(c->stage_ev[j]));
        }
        const size_t len = std::min(STAGE_BYTES, n - o);
        pool.copy(c->stage[j], in + o, len);
        KOLM_HIP_CHECK(hipMemcpyAsync(d + o, c->stage[j], len, hipMemcpyHostToDevice, st));
        KOLM_HIP_CHECK(hipEventRecord(c->stage_ev[j], st));
    }
    KOLM_HIP_CHECK(hipMemsetAsync(d + n, 0, 64, st));
    return d;
}

}  // namespace

extern "C" {

const char* kolm_last_error(void) { return g_err.c_str(); }

int kolm_device_count(int* count) {
    if (!count) return KOLM_EARG;
    return guarded([&] {
        KOLM_HIP_CHECK(hipGetDeviceCount(count));
        return KOLM_OK;
    });
}

int kolm_ctx_create(int device, kolm_ctx** out) {
    if (!out) return KOLM_EARG;
    return ctx_create(device, out);
}

int kolm_ctx_destroy(kolm_ctx* c) {
    if (!c) return KOLM_EARG;
    return guarded([&] {
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->stream));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->aux));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->rp));
        for (auto& kv : c->bufs)
            if (kv.second.p) KOLM_HIP_CHECK(hipFree(kv.second.p));
        for (auto& e : c->ev) KOLM_HIP_CHECK(hipEventDestroy(e));
        for (auto& e : c->evj) KOLM_HIP_CHECK(hipEventDestroy(e));
        for (auto& e : c->evr) KOLM_HIP_CHECK(hipEventDestroy(e));
        for (auto& e : c->evg) KOLM_HIP_CHECK(hipEventDestroy(e));
        KOLM_HIP_CHECK(hipEventDestroy(c->eva));
        for (auto& e : c->evpool) KOLM_HIP_CHECK(hipEventDestroy(e));
        KOLM_HIP_CHECK(hipHostFree(c->h_cnt));
        if (c->h_rt) KOLM_HIP_CHECK(hipHostFree(c->h_rt));
        if (c->h_tail) KOLM_HIP_CHECK(hipHostFree(c->h_tail));
        for (int i = 0; i < kolm_ctx::NSTAGE; ++i) {
            if (c->stage[i]) KOLM_HIP_CHECK(hipHostFree(c->stage[i]));
            if (c->stage_ev[i]) KOLM_HIP_CHECK(hipEventDestroy(c->stage_ev[i]));
        }
        if (c->h_res) KOLM_HIP_CHECK(hipHostFree(c->h_res));
        if (c->up) KOLM_HIP_CHECK(hipStreamDestroy(c->up));
        if (c->dl) KOLM_HIP_CHECK(hipStreamDestroy(c->dl));
        if (c->up_ev) KOLM_HIP_CHECK(hipEventDestroy(c->up_ev));
        KOLM_HIP_CHECK(hipStreamDestroy(c->stream));
        KOLM_HIP_CHECK(hipStreamDestroy(c->aux));
        KOLM_HIP_CHECK(hipStreamDestroy(c->rp));
        delete c;
        return KOLM_OK;
    });
}

int kolm_init(int device) {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_default) return KOLM_OK;
    return ctx_create(device, &g_default);
}

int kolm_shutdown(void) {
    comm_shutdown();
    std::lock_guard<std::mutex> g(g_mu);
    int r = KOLM_OK;
    for (kolm_ctx*& c : g_multi)
        if (c) {
            const int e = kolm_ctx_destroy(c);
            if (e) r = e;
            c = nullptr;
        }
    g_multi.clear();
    if (!g_default) return r;
    const int e = kolm_ctx_destroy(g_default);
    g_default = nullptr;
    return e ? e : r;
}

int kolm_ctx_reserve(kolm_ctx* c, uint64_t total_bytes, uint32_t max_block) {
    (void)max_block;
    if (!c) return KOLM_EARG;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->get<u8>("text", total_bytes + 64);
        return KOLM_OK;
    });
}

int kolm_dev_alloc(kolm_ctx* c, uint64_t bytes, void** dptr) {
    if (!c || !dptr) return KOLM_EARG;
    return guarded([&] {
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        KOLM_HIP_CHECK(hipMalloc(dptr, bytes ? bytes : 16));
        return KOLM_OK;
    });
}

int kolm_dev_free(kolm_ctx* c, void* dptr) {
    if (!c) return KOLM_EARG;
    return guarded([&] {
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        KOLM_HIP_CHECK(hipFree(dptr));
        return KOLM_OK;
    });
}

int kolm_memcpy_h2d(kolm_ctx* c, void* dst, const void* src, uint64_t bytes) {
    if (!c) return KOLM_EARG;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (bytes) KOLM_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->stream));
        return KOLM_OK;
    });
}

int kolm_memcpy_d2h(kolm_ctx* c, void* dst, const void* src, uint64_t bytes) {
    if (!c) return KOLM_EARG;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (bytes) KOLM_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
        KOLM_HIP_CHECK(hipStreamSynchronize(c->stream));
        return KOLM_OK;
    });
}

int kolm_ctx_set_timing(kolm_ctx* c, int enable) {
    if (!c) return KOLM_EARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (enable && !c->timing) c->kacc.clear();
    c->timing = enable != 0;
    return KOLM_OK;
}

int kolm_ctx_set_serial(kolm_ctx* c, int serial) {
    if (!c) return KOLM_EARG;
    std::lock_guard<std::mutex> g(c->mu);
    c->serial = serial != 0;
    return KOLM_OK;
}

int kolm_ctx_kernel_times(kolm_ctx* c, char* buf, size_t cap, size_t* len) {
    if (!c) return KOLM_EARG;
    std::lock_guard<std::mutex> g(c->mu);
    std::string js = "{";
    bool first = true;
    for (auto& kv : c->kacc) {
        char tmp[320];
        static const char* const sn[3] = {"index", "sort", "repair"};
        snprintf(tmp, sizeof tmp,
                 "%s\"%s\": {\"ms\": %.6f, \"launches\": %llu, \"bytes\": %llu, \"family\": %d, \"stream\": \"%s\"}",
                 first ? "" : ", ", kv.first.c_str(), kv.second.ms, (unsigned long long)kv.second.launches,
                 (unsigned long long)kv.second.bytes, kv.second.fam, sn[kv.second.strm]);
        js += tmp;
        first = false;
    }
    js += "}";
    if (len) *len = js.size();
    if (!buf || cap < js.size() + 1) return buf ? KOLM_ECAP : KOLM_OK;
    std::memcpy(buf, js.c_str(), js.size() + 1);
    return KOLM_OK;
}

int kolm_ctx_sync(kolm_ctx* c) {
    if (!c) return KOLM_EARG;
    return guarded([&] {
        c->sync();
        return KOLM_OK;
    });
}

int kolm_encode_blocks_device(kolm_ctx* c, const uint8_t* d_data, uint64_t total, uint32_t block_size,
                              uint32_t cand_mask, const int32_t* force_method, uint8_t* d_arena,
                              uint64_t arena_cap, uint32_t* h_sizes, uint32_t* h_method, uint64_t* h_off,
                              kolm_stats* stats) {
    if (!c || (!d_data && total) || !d_arena) return KOLM_EARG;
    if ((cand_mask & KOLM_FULL_MASK) == 0) return KOLM_EARG;
    if (reinterpret_cast<uintptr_t>(d_arena) & 3) {
        set_err("device arena must be 4-byte aligned");
        return KOLM_EARG;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        return encode_batch(c, d_data, total, block_size, nullptr, 0, cand_mask & KOLM_FULL_MASK, force_method,
                            d_arena, arena_cap, h_sizes, h_method, h_off, stats);
    });
}

int kolm_encode_blocks(const uint8_t* data, const uint64_t* starts, const uint32_t* lens, uint32_t nblocks,
                       uint32_t cand_mask, const int32_t* force_method, uint32_t* sizes, uint32_t* method,
                       uint8_t* payload_arena, uint64_t arena_cap, uint64_t* payload_off, kolm_stats* stats) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if (nblocks && (!data || !starts || !lens)) return KOLM_EARG;
    if (!payload_off) return KOLM_EARG;
    if ((cand_mask & KOLM_FULL_MASK) == 0) return KOLM_EARG;
    // contiguous non-empty blocks; the fixed geometry when every block but a shorter last
    // one has lens[0] bytes, the variable one otherwise (content-defined chunks)
    uint64_t total = 0;
    const uint32_t bs = nblocks ? lens[0] : 1;
    bool fixed = true;
    for (uint32_t i = 0; i < nblocks; ++i) {
        if (lens[i] == 0 || starts[i] != starts[0] + total) {
            set_err("kolm_encode_blocks: blocks must be contiguous and non-empty");
            return KOLM_EARG;
        }
        if ((i + 1 < nblocks && lens[i] != bs) || lens[i] > bs) fixed = false;
        total += lens[i];
    }
    if (total >= (1ull << 31)) {
        set_err("batch larger than 2^31-1 bytes");
        return KOLM_EARG;
    }
    std::vector<u32> hb;
    if (!fixed) {
        hb.resize((size_t)nblocks + 1);
        hb[0] = 0;
        for (uint32_t i = 0; i < nblocks; ++i) hb[i + 1] = hb[i] + lens[i];
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (fixed)
            if (int e = check_geom(total, bs)) return e;
        u8* d = upload(c, data + (nblocks ? starts[0] : 0), total);
        const bool has_raw = (cand_mask & 1u) && force_method == nullptr;
        const u64 dcap = (has_raw ? total : 9 * total) + 64 * (u64)nblocks + 256;
        u8* arena = c->get<u8>("arena", dcap);
        std::vector<u64> off(nblocks + 1);
        int r = encode_batch(c, d, total, bs, fixed ? nullptr : hb.data(), nblocks, cand_mask & KOLM_FULL_MASK,
                             force_method, arena, dcap, sizes, method, off.data(), stats);
        if (r) return r;
        if (off[nblocks] > arena_cap) {
            set_err("payload_arena too small");
            return KOLM_ECAP;
        }
        if (off[nblocks]) {
            KOLM_HIP_CHECK(hipMemcpyAsync(payload_arena, arena, off[nblocks], hipMemcpyDeviceToHost, c->stream));
            c->sync();
        }
        std::memcpy(payload_off, off.data(), sizeof(u64) * (nblocks + 1));
        return KOLM_OK;
    });
}

int kolm_compress_fixed(const uint8_t* data, uint64_t n, uint32_t block_size, uint32_t cand_mask,
                        const uint8_t** out, uint64_t* out_len, kolm_stats* stats) {
    const auto th0 = std::chrono::steady_clock::now();
    kolm_ctx* c = need_default();
    if (!c) {
        set_err("kolm_init has not been called");
        return KOLM_ENOINIT;
    }
    if ((!data && n) || !out || !out_len || block_size == 0 || block_size > 0x7FFFFFFFu) {
        set_err("kolm_compress_fixed: bad argument (null buffer or block size outside [1, 2^31))");
        return KOLM_EARG;
    }
    if ((cand_mask & KOLM_FULL_MASK) == 0) {
        set_err("kolm_compress_fixed: the candidate mask selects no candidate of ids 0..10");
        return KOLM_EARG;
    }
    const u64 nb = (n + block_size - 1) / block_size;
    if (nb > 0xFFFFu || n > 0xFFFFFFFFull) {  // PY: struct.pack('<H' / '<I') raises
        set_err(nb > 0xFFFFu ? "'H' format requires 0 <= number <= 65535"
                             : "'I' format requires 0 <= number <= 4294967295");
        return KOLM_ERANGE;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        std::vector<u32> method(nb), lens(nb);
        std::vector<u64> plen(nb);
        for (u64 b = 0; b < nb; ++b) lens[b] = (u32)std::min<u64>(block_size, n - b * block_size);
        // Pieces of whole blocks, each one device batch: below the 2^31-position limit of a
        // batch (512 MiB with v2_new, whose 8 bit planes per byte share that index space;
        // KOLM_BATCH_BYTES lowers it — the tests run the multi-batch path that way), and
        // inputs of 128 MiB or more in two pieces so that the upload of piece k + 1 (a host
        // thread: pageable -> pinned staging -> DMA on the upload stream) and the download of
        // piece k - 1's payloads (download stream) run while piece k encodes.
        u64 lim = (cand_mask >> KOLM_M_V2NEW) & 1u ? (1ull << 29) - 1 : (1ull << 31) - 1;
        if (const char* e = getenv("KOLM_BATCH_BYTES")) lim = std::min<u64>(lim, std::max<u64>(1, strtoull(e, nullptr, 10)));
        static const u64 pipe_min = getenv("KOLM_PIPE_MIN") ? strtoull(getenv("KOLM_PIPE_MIN"), nullptr, 10) : (128ull << 20);
        const bool has_raw = (cand_mask & 1u) != 0;
        std::vector<std::pair<u64, u64>> pieces;  // (first block, blocks)
        {
            const u64 per = std::max<u64>(1, lim / block_size);
            for (u64 b0 = 0; b0 < nb; b0 += per) {
                const u64 k = std::min(per, nb - b0);
                const u64 len = std::min<u64>(n, (b0 + k) * block_size) - b0 * block_size;
                if (has_raw && len >= pipe_min && k >= 2) {
                    pieces.push_back({b0, k / 2});
                    pieces.push_back({b0 + k / 2, k - k / 2});
                } else {
                    pieces.push_back({b0, k});
                }
            }
        }
        const u64 np = pieces.size();
        auto piece_bytes = [&](u64 i, u64& lo) {
            lo = pieces[i].first * block_size;
            return std::min<u64>(n, (pieces[i].first + pieces[i].second) * block_size) - lo;
        };
        for (u64 i = 0; i < np; ++i) {
            u64 lo;
            if (int e = check_geom(piece_bytes(i, lo), block_size)) return e;
        }
        const u64 acap = (has_raw ? n : 9 * n) + 64 * nb + 256 * np;
        u8* arena = c->get<u8>("arena_c", acap);
        // the pinned result: the TOC goes in front of the payloads once every method is
        // known, so the payloads are downloaded behind room for the largest TOC (header and
        // code table, 4 bits per block of run symbol / run length in the worst case, the
        // Elias-Fano ends <= 2 + 33 bits per block).  Without raw among the candidates the
        // payload bound is 9n: then everything is downloaded after the last piece.
        const u64 head = 4096 + 16 * nb;
        const u64 need_max = head + (has_raw ? n + 64 * nb : 0) + 4096;
        if (has_raw && c->h_res_cap < need_max) {
            if (c->h_res) KOLM_HIP_CHECK(hipHostFree(c->h_res));
            c->h_res = nullptr;
            c->h_res_cap = 0;
            KOLM_HIP_CHECK(hipHostMalloc((void**)&c->h_res, need_max, hipHostMallocDefault));
            c->h_res_cap = need_max;
        }
        if (!c->up) {
            KOLM_HIP_CHECK(hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking));
            KOLM_HIP_CHECK(hipStreamCreateWithFlags(&c->dl, hipStreamNonBlocking));
            KOLM_HIP_CHECK(hipEventCreateWithFlags(&c->up_ev, hipEventDisableTiming));
        }
        u8* dtext[2] = {nullptr, nullptr};
        {
            u64 mx = 0, lo;
            for (u64 i = 0; i < np; ++i) mx = std::max(mx, piece_bytes(i, lo));
            dtext[0] = c->get<u8>("text", mx + 64);
            if (np > 1) dtext[1] = c->get<u8>("text_b", mx + 64);
        }
        // piece i's upload (on the calling thread for piece 0, a helper thread otherwise)
        auto upload = [&](u64 i) {
            u64 lo;
            const u64 len = piece_bytes(i, lo);
            KOLM_HIP_CHECK(hipSetDevice(c->device));
            upload_staged(c, data + lo, len, dtext[i & 1], c->up);
            KOLM_HIP_CHECK(hipEventRecord(c->up_ev, c->up));
        };
        struct Up {
            std::thread t;
            int rc = KOLM_OK;
            std::string err;
        } next;
        auto start_upload = [&](u64 i) {
            next.rc = KOLM_OK;
            next.t = std::thread([&, i] {
                next.rc = guarded([&] {
                    upload(i);
                    return KOLM_OK;
                });
                if (next.rc) next.err = g_err;
            });
        };
        auto join_upload = [&]() -> int {
            if (next.t.joinable()) next.t.join();
            if (next.rc) set_err(next.err);
            return next.rc;
        };
        struct JoinGuard {  // an early error return never leaves the helper running
            Up& u;
            ~JoinGuard() {
                if (u.t.joinable()) u.t.join();
            }
        } jg{next};
        // KOLM_HOST_PROF=1 (debug): wall-clock phases of the call on stderr
        static const bool hprof = getenv("KOLM_HOST_PROF") && atoi(getenv("KOLM_HOST_PROF"));
        auto hms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count(); };
        if (hprof) fprintf(stderr, "[kolm] host: setup %.2f ms\n", hms());
        upload(0);
        if (hprof) fprintf(stderr, "[kolm] host: piece 0 upload queued %.2f ms\n", hms());
        u64 pos = 0, dpos = head;
        std::vector<u64> apos(np), abytes(np);
        kolm_stats agg{};
        for (u64 i = 0; i < np; ++i) {
            u64 lo;
            const u64 len = piece_bytes(i, lo), b0 = pieces[i].first, k = pieces[i].second;
            if (i) {
                if (int e = join_upload()) return e;
            }
            // the encode (c->stream first) waits for this piece's upload
            KOLM_HIP_CHECK(hipStreamWaitEvent(c->stream, c->up_ev, 0));
            if (i + 1 < np) {
                // piece i + 1 goes up while piece i encodes; its buffer's previous user (piece
                // i - 1) is complete: encode_batch returns synchronised
                start_upload(i + 1);
            }
            std::vector<u64> o(k + 1);
            kolm_stats st{};
            int r = encode_batch(c, dtext[i & 1], len, block_size, nullptr, 0, cand_mask & KOLM_FULL_MASK, nullptr,
                                 arena + pos, acap - pos, nullptr, method.data() + b0, o.data(), &st);
            if (r) return r;
            if (hprof) fprintf(stderr, "[kolm] host: piece %llu encoded %.2f ms\n", (unsigned long long)i, hms());
            for (u64 j = 0; j < k; ++j) plen[b0 + j] = o[j + 1] - o[j];
            apos[i] = pos;
            abytes[i] = o[k];
            if (has_raw && o[k])  // this piece's payloads go down while the next one encodes
                KOLM_HIP_CHECK(hipMemcpyAsync(c->h_res + dpos, arena + pos, o[k], hipMemcpyDeviceToHost, c->dl));
            dpos += o[k];
            pos += o[k];
            pos = (pos + 3) & ~(u64)3;  // the next piece's arena is 4-byte aligned
            stats_add(agg, st, i == 0);
        }
        // the container: header + TOC (kolm_toc.cpp) right in front of the payloads
        u64 toc_len = 0;
        if (int e = kolm_toc_write(0, block_size, n, (u32)nb, method.data(), lens.data(), plen.data(), nullptr, 0,
                                   &toc_len))
            return e;
        u64 total_pay = 0;
        for (u64 b = 0; b < nb; ++b) total_pay += plen[b];
        const size_t need = toc_len + total_pay;
        u64 at = head - toc_len;
        if (!has_raw) {  // payload size known only now: allocate and download everything
            if (c->h_res_cap < need) {
                if (c->h_res) KOLM_HIP_CHECK(hipHostFree(c->h_res));
                c->h_res = nullptr;
                c->h_res_cap = 0;
                KOLM_HIP_CHECK(hipHostMalloc((void**)&c->h_res, need + (need >> 3) + 4096, hipHostMallocDefault));
                c->h_res_cap = need + (need >> 3) + 4096;
            }
            at = 0;
            u64 d = toc_len;
            for (u64 i = 0; i < np; ++i) {
                if (abytes[i])
                    KOLM_HIP_CHECK(hipMemcpyAsync(c->h_res + d, arena + apos[i], abytes[i], hipMemcpyDeviceToHost, c->dl));
                d += abytes[i];
            }
        } else if (toc_len > head) {
            set_err("kolm_compress_fixed: TOC larger than its reserved room");
            return KOLM_EHIP;
        }
        if (int e = kolm_toc_write(0, block_size, n, (u32)nb, method.data(), lens.data(), plen.data(), c->h_res + at,
                                   toc_len, &toc_len))
            return e;
        KOLM_HIP_CHECK(hipStreamSynchronize(c->dl));
        if (hprof) fprintf(stderr, "[kolm] host: payloads down, TOC written %.2f ms\n", hms());
        *out = c->h_res + at;
        *out_len = need;
        c->h_res_off = at;
        c->h_res_len = need;
        if (stats) *stats = agg;
        return KOLM_OK;
    });
}

int kolm_result_copy(uint8_t* dst, uint64_t n) {
    kolm_ctx* c = need_default();
    if (!c) {
        set_err("kolm_init has not been called");
        return KOLM_ENOINIT;
    }
    if (!dst && n) {
        set_err("kolm_result_copy: null destination");
        return KOLM_EARG;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        if (n > c->h_res_len) {
            set_err("kolm_result_copy: more bytes than the last container");
            return KOLM_ECAP;
        }
        // a large destination is fresh, untouched memory (the caller's new bytes object): ask
        // for transparent huge pages before the first touch, so the copy threads fault 2 MB
        // pages instead of 4 KB ones and the later free unmaps 50x fewer pages (108 MB
        // container: free 8.4 -> 0.4 ms, first-touch copy 2.5x faster; advisory, errors ignored)
        constexpr uintptr_t HP = 2u << 20;
        const uintptr_t a = (uintptr_t)dst, a0 = (a + HP - 1) & ~(HP - 1), a1 = (a + n) & ~(HP - 1);
        if (n >= (8u << 20) && a1 > a0) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
        if (n) copy_pool(c).copy(dst, c->h_res + c->h_res_off, n);
        return KOLM_OK;
    });
}

int kolm_encode_blocks_multi(int ngpu, const uint8_t* data, uint64_t total, uint32_t block_size,
                             uint32_t cand_mask, const int32_t* force_method, uint32_t* sizes, uint32_t* method,
                             uint8_t* payload_arena, uint64_t arena_cap, uint64_t* payload_off, kolm_stats* stats) {
    if (ngpu < 1 || (total && !data) || !payload_off || block_size == 0) return KOLM_EARG;
    if ((cand_mask & KOLM_FULL_MASK) == 0) return KOLM_EARG;
    // One call at a time from encode through the gather: each device's payloads wait in its
    // context's shared arena between the encode and the reassembly, so a concurrent call on
    // the same per-device contexts must not start until this one has copied them out
    // (kolm.h: calls are internally serialised).
    static std::mutex multi_mu;
    std::lock_guard<std::mutex> multi_lock(multi_mu);
    const u64 nb64 = (total + block_size - 1) / block_size;
    if (nb64 > 0xFFFFFFFFull) return KOLM_EARG;
    const u32 nb = (u32)nb64;
    int ndev = 0;
    if (int e = guarded([&] {
            KOLM_HIP_CHECK(hipGetDeviceCount(&ndev));
            return KOLM_OK;
        }))
        return e;
    if (ndev < 1) {
        set_err("no HIP device");
        return KOLM_ENOINIT;
    }
    const u32 G = (u32)std::max<u64>(1, std::min<u64>({(u64)ngpu, (u64)ndev, std::max<u64>(nb, 1)}));
    // contiguous shards of whole blocks (the last block may be short)
    std::vector<u32> b0(G + 1);
    for (u32 r = 0; r <= G; ++r) b0[r] = (u32)((u64)nb * r / G);
    // the shards' payloads stay in each device's arena until the reassembly below
    static const bool host_gather = getenv("KOLM_MULTI_GATHER") && !strcmp(getenv("KOLM_MULTI_GATHER"), "host");
    struct Part {
        int rc = KOLM_OK;
        std::string err;
        const u8* d_pay = nullptr;
        std::vector<u64> off;
        kolm_stats st{};
    };
    std::vector<Part> part(G);
    std::vector<u64> pbase(G + 1, 0);
    auto run = [&](u32 r) {
        Part& P = part[r];
        const u32 nbr = b0[r + 1] - b0[r];
        if (!nbr) {
            P.off.assign(1, 0);
            return;
        }
        const u64 lo = (u64)b0[r] * block_size, hi = std::min<u64>(total, (u64)b0[r + 1] * block_size);
        const u64 n = hi - lo;
        kolm_ctx* c = nullptr;
        {
            std::lock_guard<std::mutex> g(g_mu);
            if (g_multi.size() < G) g_multi.resize(G, nullptr);
            if (!g_multi[r] && (P.rc = ctx_create((int)r, &g_multi[r])) != KOLM_OK) {
                P.err = g_err;
                return;
            }
            c = g_multi[r];
        }
        P.rc = guarded([&] {
            std::lock_guard<std::mutex> g(c->mu);
            KOLM_HIP_CHECK(hipSetDevice(c->device));
            if (int e = check_geom(n, block_size)) return e;
            u8* d = upload(c, data + lo, n);
            const bool has_raw = (cand_mask & 1u) && force_method == nullptr;
            const u64 dcap = (has_raw ? n : 9 * n) + 64 * (u64)nbr + 256;
            u8* arena = c->get<u8>("arena", dcap);
            P.off.assign(nbr + 1, 0);
            int rc = encode_batch(c, d, n, block_size, nullptr, 0, cand_mask & KOLM_FULL_MASK,
                                  force_method ? force_method + b0[r] : nullptr, arena, dcap,
                                  sizes ? sizes + (u64)b0[r] * KOLM_NCAND : nullptr, method ? method + b0[r] : nullptr,
                                  P.off.data(), stats ? &P.st : nullptr);
            if (rc) return rc;
            P.d_pay = arena;
            return KOLM_OK;
        });
        if (P.rc) P.err = g_err;
    };
    // host reassembly (KOLM_MULTI_GATHER=host): every device copies its payloads into its
    // place in payload_arena (offsets known once every shard is encoded)
    auto download = [&](u32 r) {
        Part& P = part[r];
        const u64 nbytes = P.off.back();
        if (!nbytes || P.rc) return;
        kolm_ctx* c = g_multi[r];
        P.rc = guarded([&] {
            std::lock_guard<std::mutex> g(c->mu);
            KOLM_HIP_CHECK(hipSetDevice(c->device));
            KOLM_HIP_CHECK(hipMemcpyAsync(payload_arena + pbase[r], P.d_pay, nbytes, hipMemcpyDeviceToHost, c->stream));
            c->sync();
            return KOLM_OK;
        });
        if (P.rc) P.err = g_err;
    };
    auto each = [&](const std::function<void(u32)>& f) {
        std::vector<std::thread> th;
        for (u32 r = 1; r < G; ++r) th.emplace_back(f, r);
        f(0);
        for (auto& t : th) t.join();
        for (u32 r = 0; r < G; ++r)
            if (part[r].rc) {
                set_err(part[r].err);
                return part[r].rc;
            }
        return (int)KOLM_OK;
    };
    if (int e = each(run)) return e;
    for (u32 r = 0; r < G; ++r) pbase[r + 1] = pbase[r] + part[r].off.back();
    if (pbase[G] > arena_cap) {
        set_err("payload_arena too small");
        return KOLM_ECAP;
    }
    payload_off[0] = 0;
    for (u32 r = 0; r < G; ++r) {
        const u32 nbr = b0[r + 1] - b0[r];
        for (u32 i = 1; i <= nbr; ++i) payload_off[b0[r] + i] = pbase[r] + part[r].off[i];
    }
    if (pbase[G] == 0) {
        // no payload bytes (empty input): nothing to reassemble
    } else if (host_gather) {
        if (int e = each(download)) return e;
    } else {
        // RCCL: every device's payloads into device 0 over xGMI, one copy to the host
        std::vector<int> devs(G);
        std::vector<const u8*> dp(G);
        std::vector<u64> nbytes(G);
        for (u32 r = 0; r < G; ++r) {
            devs[r] = (int)r;
            dp[r] = part[r].d_pay;
            nbytes[r] = part[r].off.back();
        }
        std::unique_lock<std::mutex> g(g_mu);
        std::vector<std::unique_lock<std::mutex>> held;
        for (u32 r = 0; r < G; ++r) held.emplace_back(g_multi[r]->mu);
        g.unlock();
        if (int e = multi_rccl_gather(devs, dp, nbytes, payload_arena, arena_cap)) return e;
    }
    if (stats) {
        kolm_stats agg{};
        for (u32 r = 0; r < G; ++r) {
            const kolm_stats& s = part[r].st;
            agg.lin_rounds = std::max(agg.lin_rounds, s.lin_rounds);
            agg.cyc_rounds = std::max(agg.cyc_rounds, s.cyc_rounds);
            agg.lin_active += s.lin_active;
            agg.cyc_active += s.cyc_active;
            agg.cyc_rounds_sum += s.cyc_rounds_sum;
            agg.lz_tokens += s.lz_tokens;
            agg.lz_long += s.lz_long;
            agg.lz_fix += s.lz_fix;
            agg.ms_total = std::max(agg.ms_total, s.ms_total);
            agg.ms_sa = std::max(agg.ms_sa, s.ms_sa);
            agg.ms_lz = std::max(agg.ms_lz, s.ms_lz);
            agg.ms_entropy = std::max(agg.ms_entropy, s.ms_entropy);
            agg.ms_emit = std::max(agg.ms_emit, s.ms_emit);
            agg.ms_repair = std::max(agg.ms_repair, s.ms_repair);
            agg.rp_rules += s.rp_rules;
            agg.rp_batches += s.rp_batches;
            agg.rp_final += s.rp_final;
            for (int k = 0; k < KOLM_NKT; ++k) {
                agg.kt[k].ms += s.kt[k].ms;
                agg.kt[k].launches += s.kt[k].launches;
                agg.kt[k].bytes += s.kt[k].bytes;
            }
        }
        *stats = agg;
    }
    return KOLM_OK;
}

// FastCDC chunk starts of d_text[0, n) followed by n (PY:210-309): device kernels
// (k_cdc.hip) for the cuts, then the orphan-tail merge (PY:300-306).  Parameter errors
// carry PY's ValueError messages (PY:227-230).
static int cdc_bounds(kolm_ctx* c, const u8* d_text, u64 n, u32 mn, u32 av, u32 mx, bool merge,
                      std::vector<u32>& out) {
    out.clear();
    if (n == 0) return KOLM_OK;
    if (!(mn > 0 && mn <= av && av <= mx)) {
        set_err("Require 0 < min_size <= avg_size <= max_size");
        return KOLM_EARG;
    }
    if (av < 64) {
        set_err("avg_size too small; use >= 64");
        return KOLM_EARG;
    }
    if (n >= (1ull << 31)) {
        set_err("input larger than 2^31-1 bytes");
        return KOLM_EARG;
    }
    int k = 31 - __builtin_clz(av);  // bit_length(avg) - 1, clamped to [6, 20] (PY:172-185)
    k = k < 6 ? 6 : k > 20 ? 20 : k;
    const int ks = k + 2 <= 20 ? k + 2 : 20, kl = k > 2 ? k - 2 : 1;  // PY:235-236
    u32 gear[256];
    u32 x = 0x243F6A88u;  // PY:152-165 (xorshift32, entries | 1)
    for (int i = 0; i < 256; ++i) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        gear[i] = x | 1u;
    }
    u32* dg = c->get<u32>("cdc_gear", 256);
    KOLM_HIP_CHECK(hipMemcpyAsync(dg, gear, sizeof gear, hipMemcpyHostToDevice, c->stream));
    const u64 seg = cdc_segment(av, mx);
    const u64 nw = (n + 63) / 64, nseg = (n + seg - 1) / seg, nwg = (nw + 255) / 256;
    const u64 maxcuts = n / mn + 2;
    CdcParams p{d_text, (u32)n, mn, av, mx, (1u << ks) - 1u, (1u << kl) - 1u};
    CdcBufs b{dg,
              c->get<u64>("cdc_ws", nw),
              c->get<u64>("cdc_wl", nw),
              c->get<u64>("cdc_c", nw),
              c->get<u64>("cdc_f", nw),
              c->get<u32>("cdc_exit", nseg),
              c->get<u32>("cdc_join", nseg),
              c->get<u32>("cdc_wg", nwg),
              c->get<u32>("cdc_cuts", maxcuts),
              c->get<u32>("counters", C_N) + C_CDC};
    launch_cdc(p, b, c->stream, c->kt());
    KOLM_HIP_CHECK(hipMemcpyAsync(c->h_cnt + C_CDC, b.total, sizeof(u32), hipMemcpyDeviceToHost, c->stream));
    c->sync();
    const u32 total = c->h_cnt[C_CDC];
    if (total > maxcuts) {
        set_err("internal error: FastCDC cut count");
        return KOLM_EHIP;
    }
    out.resize((size_t)total + 2);
    out[0] = 0;
    if (total) KOLM_HIP_CHECK(hipMemcpy(out.data() + 1, b.cuts, sizeof(u32) * total, hipMemcpyDeviceToHost));
    out[total + 1] = (u32)n;
    if (merge && out.size() >= 3 && out[out.size() - 1] - out[out.size() - 2] < mn) out.erase(out.end() - 2);
    if (c->timing) {
        kolm_stats tmp{};
        c->timing_collect(&tmp);  // per-kernel totals (kolm_ctx_kernel_times)
    }
    return KOLM_OK;
}

int kolm_cdc_boundaries(const uint8_t* data, uint64_t n, uint32_t min_size, uint32_t avg_size, uint32_t max_size,
                        int merge_orphan_tail, uint64_t* starts, uint64_t cap, uint64_t* nchunks) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if ((n && (!data || !starts)) || !nchunks) return KOLM_EARG;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->timing_reset();
        const u8* d = (n && n < (1ull << 31)) ? upload(c, data, n) : nullptr;
        std::vector<u32> v;
        if (int e = cdc_bounds(c, d, n, min_size, avg_size, max_size, merge_orphan_tail != 0, v)) return e;
        *nchunks = v.empty() ? 0 : v.size() - 1;
        if (v.size() > cap) {
            set_err("starts capacity too small");
            return KOLM_ECAP;
        }
        for (size_t i = 0; i < v.size(); ++i) starts[i] = v[i];
        return KOLM_OK;
    });
}

int kolm_cdc_boundaries_device(kolm_ctx* c, const uint8_t* d_data, uint64_t n, uint32_t min_size, uint32_t avg_size,
                               uint32_t max_size, int merge_orphan_tail, uint32_t* h_starts, uint64_t cap,
                               uint64_t* nchunks) {
    if (!c || (n && (!d_data || !h_starts)) || !nchunks) return KOLM_EARG;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        c->timing_reset();
        std::vector<u32> v;
        if (int e = cdc_bounds(c, d_data, n, min_size, avg_size, max_size, merge_orphan_tail != 0, v)) return e;
        *nchunks = v.empty() ? 0 : v.size() - 1;
        if (v.size() > cap) {
            set_err("starts capacity too small");
            return KOLM_ECAP;
        }
        if (!v.empty()) std::memcpy(h_starts, v.data(), sizeof(u32) * v.size());
        return KOLM_OK;
    });
}

int kolm_encode_blocks_device_var(kolm_ctx* c, const uint8_t* d_data, const uint32_t* h_bounds, uint32_t nblocks,
                                  uint32_t cand_mask, const int32_t* force_method, uint8_t* d_arena,
                                  uint64_t arena_cap, uint32_t* h_sizes, uint32_t* h_method, uint64_t* h_off,
                                  kolm_stats* stats) {
    if (!c || !h_bounds || !d_arena || (nblocks && !d_data)) return KOLM_EARG;
    if ((cand_mask & KOLM_FULL_MASK) == 0) return KOLM_EARG;
    if (reinterpret_cast<uintptr_t>(d_arena) & 3) {
        set_err("device arena must be 4-byte aligned");
        return KOLM_EARG;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (nblocks == 0) {
            if (h_off) h_off[0] = 0;
            if (stats) *stats = kolm_stats{};
            return KOLM_OK;
        }
        return encode_batch(c, d_data, 0, 0, h_bounds, nblocks, cand_mask & KOLM_FULL_MASK, force_method, d_arena,
                            arena_cap, h_sizes, h_method, h_off, stats);
    });
}

// Checks a decode batch's method ids / offsets / lengths; total = decoded bytes.
static int check_decode(const uint64_t* payload_off, const uint32_t* methods, const uint32_t* orig_lens, u32 nb,
                        u64 out_cap, u64& total) {
    total = 0;
    for (u32 i = 0; i < nb; ++i) {
        if (methods[i] >= 32 || !((KOLM_DECODE_MASK >> methods[i]) & 1u)) {
            char msg[96];
            snprintf(msg, sizeof msg, "block %u: method %u is not decoded on the device", i, methods[i]);
            set_err(msg);
            return KOLM_EARG;
        }
        if (payload_off[i + 1] < payload_off[i]) return KOLM_EARG;
        total += orig_lens[i];
    }
    if (total >= (1ull << 31)) {
        set_err("decoded batch larger than 2^31-1 bytes");
        return KOLM_EARG;
    }
    if (total > out_cap) {
        set_err("output capacity too small");
        return KOLM_ECAP;
    }
    return KOLM_OK;
}

// Decodes nb blocks whose payloads are resident at dpay (+ payload_off[i] - payload_off[0])
// into dout (device).  Per-decoder block lists are built on the host; every kernel
// runs on the context stream.  ms (optional) = device time of the decode kernels.
static int decode_batch(kolm_ctx* c, const u8* dpay, const uint64_t* payload_off, const uint32_t* methods,
                        const uint32_t* orig_lens, u32 nb, u64 total, u8* dout, double* ms) {
    hipStream_t s = c->stream;
    std::vector<u64> poff(nb + 1);
    std::vector<u32> obase(nb + 1);
    obase[0] = 0;
    for (u32 i = 0; i <= nb; ++i) poff[i] = payload_off[i] - payload_off[0];
    for (u32 i = 0; i < nb; ++i) obase[i + 1] = obase[i] + orig_lens[i];
    // blocks per decoder
    std::vector<u32> lists[KOLM_NCAND];
    for (u32 i = 0; i < nb; ++i) lists[methods[i]].push_back(i);
    std::vector<u32> flat;
    u32 lstart[KOLM_NCAND + 1];
    for (u32 m = 0; m < KOLM_NCAND; ++m) {
        lstart[m] = (u32)flat.size();
        flat.insert(flat.end(), lists[m].begin(), lists[m].end());
    }
    lstart[KOLM_NCAND] = (u32)flat.size();
    // BBWT family: one list over ids 2..6 (the flags come from each block's id)
    std::vector<u32> bwl;
    u32 maxn = 0;
    for (u32 m = KOLM_M_BBWT; m <= KOLM_M_BBWT_GRAY; ++m)
        for (u32 i : lists[m]) {
            bwl.push_back(i);
            maxn = std::max(maxn, orig_lens[i]);
        }
    std::vector<u32> vb(nb + 1);
    vb[0] = 0;
    for (u32 i = 0; i < nb; ++i) vb[i + 1] = vb[i] + (methods[i] == KOLM_M_BBWT_BP ? 8 * ((orig_lens[i] + 7) / 8) : 0u);
    u64* dpoff = c->get<u64>("dec_poff", nb + 1);
    u32* dob = c->get<u32>("dec_obase", nb + 1);
    u32* dlist = c->get<u32>("dec_list", nb);
    u32* dst = c->get<u32>("dec_status", nb);
    KOLM_HIP_CHECK(hipMemcpyAsync(dpoff, poff.data(), sizeof(u64) * (nb + 1), hipMemcpyHostToDevice, s));
    KOLM_HIP_CHECK(hipMemcpyAsync(dob, obase.data(), sizeof(u32) * (nb + 1), hipMemcpyHostToDevice, s));
    KOLM_HIP_CHECK(hipMemcpyAsync(dlist, flat.data(), sizeof(u32) * nb, hipMemcpyHostToDevice, s));
    KOLM_HIP_CHECK(hipMemsetAsync(dst, 0, sizeof(u32) * nb, s));
    BwArgs a{};
    const u64 T = total + 16;
    if (!bwl.empty()) {
        u32* dmeth = c->get<u32>("dec_meth", nb);
        u32* dvb = c->get<u32>("dec_vbase", nb + 1);
        u32* dbwl = c->get<u32>("dec_bwlist", bwl.size());
        KOLM_HIP_CHECK(hipMemcpyAsync(dmeth, methods, sizeof(u32) * nb, hipMemcpyHostToDevice, s));
        KOLM_HIP_CHECK(hipMemcpyAsync(dvb, vb.data(), sizeof(u32) * (nb + 1), hipMemcpyHostToDevice, s));
        KOLM_HIP_CHECK(hipMemcpyAsync(dbwl, bwl.data(), sizeof(u32) * bwl.size(), hipMemcpyHostToDevice, s));
        a.d = DecArgs{dpay, dpoff, dob, dout, dst, dbwl, (u32)bwl.size()};
        a.meth = dmeth;
        a.vbase = dvb;
        a.vals = c->get<u8>("dec_vals", (u64)vb[nb] + 16);
        a.mi = c->get<u8>("dec_mi", T);
        a.bw = c->get<u8>("dec_bw", T);
        a.cpb = (maxn + MTF_CHUNK - 1) / MTF_CHUNK;
        const u64 nch = (u64)bwl.size() * a.cpb;
        a.summ = c->get<u8>("dec_summ", nch * 256 + 16);
        a.states = c->get<u8>("dec_states", nch * 256 + 16);
        a.X[0] = c->get<u32>("dec_x0", T);
        a.X[3] = c->get<u32>("dec_x3", T);
        a.X[4] = c->get<u32>("dec_x4", T);
        a.so = c->get<u64>("dec_so", T);
        a.tpb = (maxn + BWI_TILE - 1) / BWI_TILE;
        a.th = c->get<u32>("dec_th", (u64)bwl.size() * a.tpb * 256 + 16);
        a.sshift = 6;
        while (((u64)maxn + (1ull << a.sshift) - 1) >> a.sshift > BWI_NODES) ++a.sshift;
        a.nnmax = (u32)(((u64)maxn + (1ull << a.sshift) - 1) >> a.sshift);
        a.nd = c->get<u32>("dec_nodes", 5ull * bwl.size() * a.nnmax + 16);
        std::vector<u32> wb(bwl.size() + 1);
        wb[0] = 0;
        a.wmax = 0;
        for (size_t li = 0; li < bwl.size(); ++li) {
            const u64 nw = (poff[bwl[li] + 1] - poff[bwl[li]] + 7) / 8;
            a.wmax = std::max(a.wmax, (u32)nw);
            wb[li + 1] = wb[li] + (u32)nw;
        }
        u32* dwb = c->get<u32>("dec_wbase", wb.size());
        KOLM_HIP_CHECK(hipMemcpyAsync(dwb, wb.data(), sizeof(u32) * wb.size(), hipMemcpyHostToDevice, s));
        a.wbase = dwb;
        a.fw = c->get<u32>("dec_fw", (u64)wb.back() + 16);
        a.es = c->get<u8>("dec_es", (u64)wb.back() + 16);
        a.vbw = c->get<u32>("dec_vbw", (u64)wb.back() + 16);
    }
    u32 *tpos = nullptr, *tval = nullptr, *ntok = nullptr, *mark = nullptr, *src = nullptr;
    if (!lists[KOLM_M_LZ77].empty()) {
        tpos = c->get<u32>("dec_tpos", T);
        tval = c->get<u32>("dec_tval", T);
        ntok = c->get<u32>("dec_ntok", nb);
        mark = c->get<u32>("dec_mark", T);
        src = c->get<u32>("dec_src", T);
    }
    u32 *rvals = nullptr, *rnval = nullptr, *recnt = nullptr, *rlen = nullptr;
    u64 *rea = nullptr, *reb = nullptr;
    if (!lists[KOLM_M_REPAIR].empty()) {
        const u64 P = poff[nb] + 16;
        rvals = c->get<u32>("dec_rvals", P);
        rlen = c->get<u32>("dec_rlen", P);
        rnval = c->get<u32>("dec_rnval", nb);
        recnt = c->get<u32>("dec_recnt", lists[KOLM_M_REPAIR].size());
        rea = c->get<u64>("dec_rea", T);
        reb = c->get<u64>("dec_reb", T);
    }
    auto args = [&](u32 m) { return DecArgs{dpay, dpoff, dob, dout, dst, dlist + lstart[m], lstart[m + 1] - lstart[m]}; };
    if (ms) KOLM_HIP_CHECK(hipEventRecord(c->ev[0], s));
    launch_dec_raw(args(KOLM_M_RAW), s);
    launch_dec_uleb(args(KOLM_M_XOR), false, s);
    launch_dec_uleb(args(KOLM_M_LFSR), true, s);
    if (!lists[KOLM_M_LZ77].empty()) launch_dec_lz77(args(KOLM_M_LZ77), tpos, tval, ntok, mark, src, s);
    if (!bwl.empty()) launch_dec_bw(a, s);
    if (rvals) launch_dec_repair(args(KOLM_M_REPAIR), rvals, rnval, recnt, rlen, rea, reb, s);
    if (ms) KOLM_HIP_CHECK(hipEventRecord(c->ev[1], s));
    std::vector<u32> st(nb);
    KOLM_HIP_CHECK(hipMemcpyAsync(st.data(), dst, sizeof(u32) * nb, hipMemcpyDeviceToHost, s));
    c->sync();
    if (ms) {
        float f = 0.f;
        KOLM_HIP_CHECK(hipEventElapsedTime(&f, c->ev[0], c->ev[1]));
        *ms = f;
    }
    for (u32 i = 0; i < nb; ++i)
        if (st[i]) {
            char msg[128];
            snprintf(msg, sizeof msg, "block %u (method %u): %s", i, methods[i],
                     st[i] == DEC_ELEN ? "decoded length mismatch" : "malformed payload");
            set_err(msg);
            return KOLM_EARG;
        }
    return KOLM_OK;
}

int kolm_decode_blocks(const uint8_t* payloads, const uint64_t* payload_off, const uint32_t* methods,
                       const uint32_t* orig_lens, uint32_t nblocks, uint8_t* out, uint64_t out_cap) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if (nblocks && (!payloads || !payload_off || !methods || !orig_lens || !out)) return KOLM_EARG;
    u64 total = 0;
    if (int rc = check_decode(payload_off, methods, orig_lens, nblocks, out_cap, total)) return rc;
    if (nblocks == 0) return KOLM_OK;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        const u32 nb = nblocks;
        const u64 ptotal = payload_off[nb] - payload_off[0];
        u8* dpay = c->get<u8>("dec_pay", ptotal + 64);
        u8* dout = c->get<u8>("dec_out", total + 64);
        if (ptotal)
            KOLM_HIP_CHECK(hipMemcpyAsync(dpay, payloads + payload_off[0], ptotal, hipMemcpyHostToDevice, c->stream));
        if (int rc = decode_batch(c, dpay, payload_off, methods, orig_lens, nb, total, dout, nullptr)) return rc;
        KOLM_HIP_CHECK(hipMemcpy(out, dout, total, hipMemcpyDeviceToHost));
        return KOLM_OK;
    });
}

int kolm_decode_blocks_device(kolm_ctx* c, const void* d_payloads, const uint64_t* payload_off,
                              const uint32_t* methods, const uint32_t* orig_lens, uint32_t nblocks, void* d_out,
                              uint64_t out_cap, double* ms) {
    if (!c) return KOLM_EARG;
    if (nblocks && (!d_payloads || !payload_off || !methods || !orig_lens || !d_out)) return KOLM_EARG;
    u64 total = 0;
    if (int rc = check_decode(payload_off, methods, orig_lens, nblocks, out_cap, total)) return rc;
    if (ms) *ms = 0.0;
    if (nblocks == 0) return KOLM_OK;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        return decode_batch(c, static_cast<const u8*>(d_payloads) + payload_off[0], payload_off, methods, orig_lens,
                            nblocks, total, static_cast<u8*>(d_out), ms);
    });
}

int kolm_bbwt_forward(const uint8_t* in, size_t n, uint8_t* out) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if ((n && (!in || !out))) return KOLM_EARG;
    if (n == 0) return KOLM_OK;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (int e = check_geom(n, (u32)n)) return e;
        Geom geo;
        geom_init(geo, n, (u32)n);
        u8* d = upload(c, in, n);
        Pipeline P{c, geo, d};
        u8* bw = P.bbwt();
        KOLM_HIP_CHECK(hipMemcpyAsync(out, bw, n, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        return KOLM_OK;
    });
}

int kolm_mtf_encode(const uint8_t* in, size_t n, uint8_t* out) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if ((n && (!in || !out))) return KOLM_EARG;
    if (n == 0) return KOLM_OK;
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (int e = check_geom(n, (u32)n)) return e;
        Geom geo;
        geom_init(geo, n, (u32)n);
        u8* d = upload(c, in, n);
        Pipeline P{c, geo, d};
        u8* m = P.mtf(d);
        KOLM_HIP_CHECK(hipMemcpyAsync(out, m, n, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        return KOLM_OK;
    });
}

static int rice_common(kolm_ctx* c, const Geom& geo, const u8* d_seq, int k, uint8_t* out, size_t cap,
                       size_t* out_len) {
    const u64 n = geo.N;
    const u64 worst = (n * ((255u >> k) + 1 + k) + 7) / 8 + 64;
    u8* dout = c->get<u8>("rice_out", worst + 64);
    KOLM_HIP_CHECK(hipMemsetAsync(dout, 0, worst + 64, c->stream));
    const u64 ntiles = (u64)((geo.bs + TILE - 1) / TILE) * geo.nb + 16;
    u32* t1 = c->get<u32>("tile_tmp", 2 * ntiles + 16);
    u32* t2 = c->get<u32>("tile_tmp2", 2 * ntiles + 2 * geo.nb + 16);
    u32* cnt = c->get<u32>("counters", C_N);
    launch_rice_only(geo, d_seq, k, dout, t1, t2, cnt + C_RICE, c->stream);
    KOLM_HIP_CHECK(hipMemcpyAsync(c->h_cnt, cnt, sizeof(u32) * C_N, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    const u32 sz = c->h_cnt[C_RICE];
    if (out_len) *out_len = sz;
    if (sz > cap) {
        set_err("rice output capacity too small");
        return KOLM_ECAP;
    }
    if (sz) {
        KOLM_HIP_CHECK(hipMemcpyAsync(out, dout, sz, hipMemcpyDeviceToHost, c->stream));
        c->sync();
    }
    return KOLM_OK;
}

int kolm_rice_encode(const uint8_t* in, size_t n, int k, uint8_t* out, size_t cap, size_t* out_len) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if (k < 0 || k > 15 || (n && (!in || !out))) return KOLM_EARG;
    if (n == 0) {
        if (out_len) *out_len = 0;
        return KOLM_OK;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (int e = check_geom(n, (u32)n)) return e;
        Geom geo;
        geom_init(geo, n, (u32)n);
        u8* d = upload(c, in, n);
        return rice_common(c, geo, d, k, out, cap, out_len);
    });
}

int kolm_bbwt_mtf_rice(const uint8_t* in, size_t n, int flags, int k, uint8_t* out, size_t cap,
                       size_t* out_len) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if (k < 0 || k > 15 || (n && (!in || !out))) return KOLM_EARG;
    if (flags != 0 && flags != 1 && flags != 4 && flags != 8 && flags != 16) return KOLM_EARG;
    if (n == 0) {
        if (out_len) *out_len = 0;
        return KOLM_OK;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (int e = check_geom(n, (u32)n)) return e;
        Geom geo;
        geom_init(geo, n, (u32)n);
        u8* d = upload(c, in, n);
        Pipeline P{c, geo, d};
        u8* m = P.mtf(P.bbwt());
        if (flags == 0) return rice_common(c, geo, m, k, out, cap, out_len);
        // bitwise variant through the batched path with a forced method
        const int32_t force = flags == 1 ? 3 : flags == 4 ? 4 : flags == 8 ? 5 : 6;
        if (k != 2) {
            set_err("bitwise variants are only defined with k=2 in the batched path");
            return KOLM_EARG;
        }
        const u64 dcap = 9 * n + 256;
        u8* arena = c->get<u8>("arena", dcap);
        std::vector<u64> off(2);
        int r = encode_batch(c, d, n, (u32)n, nullptr, 0, 1u << force, &force, arena, dcap, nullptr, nullptr,
                             off.data(), nullptr);
        if (r) return r;
        if (out_len) *out_len = off[1];
        if (off[1] > cap) {
            set_err("output capacity too small");
            return KOLM_ECAP;
        }
        KOLM_HIP_CHECK(hipMemcpyAsync(out, arena, off[1], hipMemcpyDeviceToHost, c->stream));
        c->sync();
        return KOLM_OK;
    });
}

int kolm_lz77_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    kolm_ctx* c = need_default();
    if (!c) return KOLM_ENOINIT;
    if (n && (!in || !out)) return KOLM_EARG;
    if (n == 0) {
        if (out_len) *out_len = 0;
        return KOLM_OK;
    }
    return guarded([&] {
        std::lock_guard<std::mutex> g(c->mu);
        KOLM_HIP_CHECK(hipSetDevice(c->device));
        if (int e = check_geom(n, (u32)n)) return e;
        Geom geo;
        geom_init(geo, n, (u32)n);
        u8* d = upload(c, in, n);
        Pipeline P{c, geo, d};
        LzArgs z = P.lz_args();
        P.lz(z);
        u32 sz = 0;
        KOLM_HIP_CHECK(hipMemcpyAsync(&sz, z.lz_size, sizeof(u32), hipMemcpyDeviceToHost, c->stream));
        c->sync();
        if (out_len) *out_len = sz;
        if (sz > cap) {
            set_err("lz77 output capacity too small");
            return KOLM_ECAP;
        }
        u8* dout = c->get<u8>("lz_out", (u64)sz + 64);
        u64* doff = c->get<u64>("lz_off", 2);
        KOLM_HIP_CHECK(hipMemsetAsync(doff, 0, sizeof(u64) * 2, c->stream));
        launch_lz_emit(z, nullptr, doff, dout, c->stream);
        KOLM_HIP_CHECK(hipMemcpyAsync(out, dout, sz, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        return KOLM_OK;
    });
}

}  // extern "C"
