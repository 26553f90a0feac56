// Re-Pair (candidate 9, PY:1817-1911) on gfx950: one 1024-thread workgroup per block runs
// the batched exact Re-Pair of repair_core.h (see its header for the formulation and
// why the batches reproduce the reference's sequential rounds bit for bit).
//
// Work per block is O(n) amortised: every pair id is chosen at most once and its region
// of occurrence positions is read once; the sequential depth is the number of batches
// (944 for 1 MiB of enwik-style text, 912 for random bytes, 16935 for the gradient image
// against 18863 / 54287 / 133138 reference rounds).  The kernel is latency-bound (block-
// local barriers + dependent global accesses), so blocks run concurrently, one per CU.
#include "kolm_internal.h"

#define RP_HD __host__ __device__
#include "repair_core.h"

namespace kolm {

static_assert(RP_RS_N == rp::RS_N && RP_RS_SIZE == rp::RS_SIZE && RP_RS_ERR == rp::RS_ERR, "result layout");
static_assert(RP_P_N == rp::P_N && RP_MAX_N == rp::MAX_N, "profile sections / block limit");

namespace {

struct DevExec {
    rp::Shared* sh;
    u64* prof;      // [P_N] per block, or null
    u32* trace;     // per-batch records (block 0 only), or null
    u32* rec = nullptr;
    u64 last = 0;   // thread 0: time of the previous mark
    u32 last_id = 0;
    __device__ inline void mark(u32 id) {
        if ((prof || trace) && threadIdx.x == 0) {
            const u64 now = wall_clock64();
            if (last) {
                if (prof) prof[last_id] += now - last;
                if (rec) rec[8 + last_id] += (u32)(now - last);
            }
            last = now;
            last_id = id;
        }
    }
    // debug trace: it = loop iteration (a record per iteration), then the batch's fields
    __device__ inline void begin(u32 it) {
        if (trace && threadIdx.x == 0) rec = it < RP_TR_CAP ? trace + (u64)it * RP_TR_W : nullptr;
    }
    __device__ inline void record(const u32 (&f)[8]) {
        if (rec && threadIdx.x == 0)
            for (u32 k = 0; k < 8; ++k) rec[k] = f[k];
    }
    template <class F>
    __device__ inline void par(F f) {
        f(threadIdx.x);
        __syncthreads();
    }
    // exclusive scan of a[0..NT) in place; *total = sum (both visible after the barrier)
    __device__ inline void scan(u32* a, u32* total) {
        const u32 t = threadIdx.x, lane = t & 63, w = t >> 6;
        const u32 v = a[t];
        const u32 incl = wave_incl_scan(v, OpAddU(), 0u);
        if (lane == 63) sh->wtot[w] = incl;
        __syncthreads();
        u32 pre = 0, tot = 0;
#pragma unroll
        for (u32 i = 0; i < rp::NT / 64; ++i) {
            const u32 x = sh->wtot[i];
            pre += i < w ? x : 0u;
            tot += x;
        }
        a[t] = pre + incl - v;
        if (t == 0) *total = tot;
        __syncthreads();
    }
    // two exclusive scans sharing their barriers (a: totals in *ta, b: in *tb)
    __device__ inline void scan2(u32* a, u32* b, u32* ta, u32* tb) {
        const u32 t = threadIdx.x, lane = t & 63, w = t >> 6;
        const u32 va = a[t], vb = b[t];
        const u32 ia = wave_incl_scan(va, OpAddU(), 0u), ib = wave_incl_scan(vb, OpAddU(), 0u);
        if (lane == 63) {
            sh->wtot[w] = ia;
            sh->wtot2[w] = ib;
        }
        __syncthreads();
        u32 pa = 0, sa = 0, pb = 0, sb = 0;
#pragma unroll
        for (u32 i = 0; i < rp::NT / 64; ++i) {
            const u32 x = sh->wtot[i], y = sh->wtot2[i];
            pa += i < w ? x : 0u;
            sa += x;
            pb += i < w ? y : 0u;
            sb += y;
        }
        a[t] = pa + ia - va;
        b[t] = pb + ib - vb;
        if (t == 0) {
            *ta = sa;
            *tb = sb;
        }
        __syncthreads();
    }
    // wave-aggregated append: one atomic per wave, slots in lane order among pred lanes
    __device__ inline u32 append(u32* ctr, bool pred) {
        const u64 m = __ballot(pred);
        if (!m) return rp::NIL;
        const u32 lane = __lane_id();
        const u32 leader = (u32)__ffsll((unsigned long long)m) - 1;
        u32 base = 0;
        if (lane == leader) base = atomicAdd(ctr, (u32)__popcll(m));
        base = (u32)__shfl((int)base, (int)leader);
        return pred ? base + (u32)__popcll(m & ((1ull << lane) - 1ull)) : rp::NIL;
    }
    // Lanes grouped by equal key (the active lanes only): this lane's group as a lane mask
    // (0 when inactive).  One iteration per distinct key in the wave.
    __device__ inline u64 peers(u64 key, bool act) {
        u64 rem = __ballot(act);
        u64 mine = 0;
        while (rem) {
            const u32 l = (u32)__ffsll((unsigned long long)rem) - 1;
            const u64 kl = ((u64)(u32)__builtin_amdgcn_readlane((int)(key >> 32), l) << 32) |
                           (u32)__builtin_amdgcn_readlane((int)(u32)key, l);
            const bool eq = act && key == kl;
            const u64 m = __ballot(eq);
            if (eq) mine = m;
            rem &= ~m;
        }
        return mine;
    }
    // wave-aggregated atomics (agg, wave-uniform): lanes hitting the same word combine into
    // one atomic by the group's first lane (text has a few hot pairs per big batch:
    // thousands of +-1 on one word); without agg every lane does its own
    __device__ inline void add_agg(u32* p, bool act, bool agg) {
        if (!agg) {
            if (act) atomicAdd(p, 1u);
            return;
        }
        const u64 m = peers((u64)(uintptr_t)p, act);
        if (act && __lane_id() == (u32)__ffsll((unsigned long long)m) - 1) atomicAdd(p, (u32)__popcll(m));
    }
    __device__ inline void sub_agg(u32* p, bool act, bool agg) {
        if (!agg) {
            if (act) atomicSub(p, 1u);
            return;
        }
        const u64 m = peers((u64)(uintptr_t)p, act);
        if (act && __lane_id() == (u32)__ffsll((unsigned long long)m) - 1) atomicSub(p, (u32)__popcll(m));
    }
    // slot = old value + this lane's rank among the group (as if every lane did atomicAdd(p, 1))
    __device__ inline u32 slot_agg(u32* p, bool act, bool agg) {
        if (!agg) return act ? atomicAdd(p, 1u) : 0u;
        const u32 lane = __lane_id();
        const u64 m = peers((u64)(uintptr_t)p, act);
        const u32 ld = act ? (u32)__ffsll((unsigned long long)m) - 1 : lane;
        u32 base = 0;
        if (act && lane == ld) base = atomicAdd(p, (u32)__popcll(m));
        base = (u32)__shfl((int)base, (int)ld);
        return base + (u32)__popcll(m & ((1ull << lane) - 1ull));
    }
    // one representative lane per distinct key: leader lane of this lane's group
    __device__ inline u32 leader(u64 key, bool act, bool agg) {
        if (!agg) return __lane_id();
        const u64 m = peers(key, act);
        return act ? (u32)__ffsll((unsigned long long)m) - 1 : __lane_id();
    }
    __device__ inline bool is_leader(u32 ld) const { return __lane_id() == ld; }
    __device__ inline u32 from_leader(u32 v, u32 ld) const { return (u32)__shfl((int)v, (int)ld); }
    __device__ inline u32 add(u32* p, u32 v) { return atomicAdd(p, v); }
    __device__ inline u32 sub(u32* p, u32 v) { return atomicSub(p, v); }
    __device__ inline u32 min(u32* p, u32 v) { return atomicMin(p, v); }
    __device__ inline u32 max(u32* p, u32 v) { return atomicMax(p, v); }
    __device__ inline u32 cas32(u32* p, u32 cmp, u32 v) { return atomicCAS(p, cmp, v); }
    __device__ inline u64 cas64(u64* p, u64 cmp, u64 v) {
        return (u64)atomicCAS((unsigned long long*)p, (unsigned long long)cmp, (unsigned long long)v);
    }
};

__global__ __launch_bounds__(rp::NT) void k_repair(RpArgs a, u32 b0) {
    __shared__ rp::Shared sh;
    const u32 b = b0 + blockIdx.x;
    const u32 base = a.geo.base(b);
    rp::Block B{};
    rp::workspace_layout(a.ws + (u64)blockIdx.x * a.ws_stride, a.geo.bs, B);
    B.text = a.text + base;
    B.n = a.geo.end(b) - base;
    B.out = a.out + (u64)b * a.out_stride;
    B.out_cap = a.out_stride;
    B.result = a.result + (u64)b * rp::RS_N;
    DevExec ex{&sh, a.prof ? a.prof + (u64)b * rp::P_N : nullptr, b == 0 ? a.trace : nullptr};
    rp::repair_block(ex, B, sh);
    ex.mark(0);
}

// winners' Re-Pair payloads -> arena (one workgroup per block, 16-byte copies where aligned)
__global__ __launch_bounds__(WG) void k_rp_emit(RpArgs a, const u32* method, const u64* off, u8* arena) {
    const u32 b = blockIdx.x;
    if (method[b] != 9u) return;
    const u32 size = a.result[(u64)b * rp::RS_N + rp::RS_SIZE];
    const u8* src = a.out + (u64)b * a.out_stride;
    u8* dst = arena + off[b];
    for (u32 i = threadIdx.x; i < size; i += WG) dst[i] = src[i];
}

}  // namespace

u64 repair_ws_bytes(u32 bs) {
    rp::Block B{};
    return rp::workspace_layout(nullptr, bs, B);
}

void launch_repair(const RpArgs& a, u32 b0, u32 nblk, hipStream_t s) {
    if (!nblk) return;
    k_repair<<<nblk, rp::NT, 0, s>>>(a, b0);
}

void launch_rp_emit(const RpArgs& a, const u32* method, const u64* off, u8* arena, hipStream_t s) {
    if (!a.geo.nb) return;
    k_rp_emit<<<a.geo.nb, WG, 0, s>>>(a, method, off, arena);
}

}  // namespace kolm
