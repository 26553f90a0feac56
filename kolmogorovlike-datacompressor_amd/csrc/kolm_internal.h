// Internal declarations of libkolm_hip.so (MI355X / gfx950 only).
//
// Data layout in HBM for one batch: the batch is the concatenation
// of nb fixed-size blocks (block b = global positions [b*bs, min((b+1)*bs, N))).
// Global position g and global suffix-array index i share the same index space [0, N):
// block b's suffix array occupies SA[b*bs .. b*bs+n_b).  All per-position arrays are
// structure-of-arrays, u32 unless noted.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace kolm {

void set_err(const std::string& s);  // message returned by kolm_last_error()

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;

constexpr int TILE = 2048;        // elements per sort/scan tile (one 256-thread workgroup)
constexpr int WG = 256;           // threads per workgroup
constexpr int PER_THREAD = TILE / WG;
constexpr int NCLASS = 12;        // small-segment size classes: len in (2^(c-1), 2^c], c = 0..11
constexpr u32 NONE = 0xFFFFFFFFu;
constexpr int LZ_WINDOW = 4096;   // PY:1723 WINDOW_MAX
constexpr int LZ_MIN = 3;         // PY:1724 MIN_MATCH
constexpr int LZ_CAP = 32;        // per-lane capped compare; longer candidates are extended by the wave
constexpr int MTF_CHUNK = 1024;   // bytes replayed per thread by the MTF kernel
constexpr u32 NCAND = 11;         // candidate ids 0..10 computed on the device (10 = v2_new, opt-in)

// Segment of the suffix array still to be refined: SA[start .. start+len).  Bit 31 of
// len (SEG_FIRST) marks a segment that begins at the start of its round group, so its
// first run of equal keys keeps the group's rank (no RK rewrite needed).
constexpr u32 SEG_FIRST = 0x80000000u;
constexpr u32 SEG_LEN = 0x7FFFFFFFu;
struct Seg {
    u32 start;
    u32 len;
};
// Segment that needs MSD radix passes (len > TILE), with its tile range.
struct LSeg {
    u32 start;
    u32 len;
    u32 tile_base;
    u32 ntiles;
};
// One MSD tile: segment index in the level's LSeg list and tile number k within it.
struct LTile {
    u32 seg;
    u32 k;
};

// Block geometry of a batch.  Fixed mode (vb == null): blocks of bs bytes (the last may be
// short), block_of by a fast u32 division.  Variable mode (content-defined chunks, PY:2213):
// block b = [vb[b], vb[b+1]), bs = the longest block (it sizes the per-block tile/chunk
// counts; the tiles past a shorter block's end are empty), block_of by a granule map
// (vmap[g >> vshift] = block of the granule's first position) plus a short forward walk.
// Every kernel addresses blocks through base()/end()/block_of() only.
struct Geom {
    u64 N;        // total bytes (< 2^31)
    u32 bs;       // block size (variable mode: longest block)
    u32 nb;       // number of blocks
    u64 magic;    // fastdiv: block_of(g) = g * magic >> shift, exact for g < 2^31
    u32 shift;
    const u32* vb = nullptr;    // variable mode: device bounds [nb + 1]
    const u32* hvb = nullptr;   // variable mode: the same bounds in host memory
    const u32* vmap = nullptr;  // variable mode: device granule -> block map
    u32 vshift = 0;
    __host__ __device__ inline const u32* bounds() const {
#if defined(__HIP_DEVICE_COMPILE__)
        return vb;
#else
        return hvb;
#endif
    }
    __host__ __device__ inline u32 block_of(u32 g) const {
        if (const u32* v = bounds()) {
#if defined(__HIP_DEVICE_COMPILE__)
            u32 b = vmap[g >> vshift];
#else
            u32 lo = 0, hi = nb;  // host: binary search (no host copy of the map)
            while (hi - lo > 1) {
                const u32 m = (lo + hi) >> 1;
                if (v[m] <= g) lo = m; else hi = m;
            }
            u32 b = lo;
#endif
            while (v[b + 1] <= g) ++b;
            return b;
        }
        return (u32)(((u64)g * magic) >> shift);
    }
    __host__ __device__ inline u32 base(u32 b) const {
        if (const u32* v = bounds()) return v[b];
        return b * bs;
    }
    __host__ __device__ inline u32 end(u32 b) const {
        if (const u32* v = bounds()) return v[b + 1];
        u64 e = (u64)(b + 1) * bs;
        return (u32)(e < N ? e : N);
    }
};

void geom_init(Geom& g, u64 N, u32 bs);
// Variable-mode geometry over host bounds hb[0..nb] (hb[0] = 0, strictly increasing,
// hb[nb] = N < 2^31); d_vb / d_vmap hold nb + 1 and (N >> vshift) + 1 words.  Blocking
// upload + map build on stream s; hb must outlive every host use of the geometry.
void geom_init_var(Geom& g, const u32* hb, u32 nb, u32* d_vb, u32* d_vmap, u32 vshift, hipStream_t s);
u32 geom_var_shift(const u32* hb, u32 nb);

// ---- wave64 scans on DPP (gfx9 row shifts + row broadcasts): VALU only, no LDS permute
// (__shfl_up/__shfl_xor compile to ds_bpermute + address math per step) ----
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_SHL1 = 0x101, DPP_ROW_SHL2 = 0x102, DPP_ROW_SHL4 = 0x104, DPP_ROW_SHL8 = 0x108;
constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143, DPP_WAVE_SHR1 = 0x138, DPP_WAVE_SHL1 = 0x130;

#define KOLM_DPP(old, v, ctrl, rmask) \
    ((u32)__builtin_amdgcn_update_dpp((int)(old), (int)(v), (ctrl), (rmask), 0xF, false))

// inclusive scan in lane order (lane 63 ends with the total)
template <class Op>
__device__ inline u32 wave_incl_scan(u32 v, Op op, u32 ident) {
    v = op(v, KOLM_DPP(ident, v, DPP_ROW_SHR1, 0xF));
    v = op(v, KOLM_DPP(ident, v, DPP_ROW_SHR2, 0xF));
    v = op(v, KOLM_DPP(ident, v, DPP_ROW_SHR4, 0xF));
    v = op(v, KOLM_DPP(ident, v, DPP_ROW_SHR8, 0xF));
    v = op(v, KOLM_DPP(ident, v, DPP_ROW_BCAST15, 0xA));
    v = op(v, KOLM_DPP(ident, v, DPP_ROW_BCAST31, 0xC));
    return v;
}
template <class Op>
__device__ inline u32 wave_excl_scan(u32 v, Op op, u32 ident) {
    return KOLM_DPP(ident, wave_incl_scan(v, op, ident), DPP_WAVE_SHR1, 0xF);
}
// reverse order (lane 0 ends with the total): mirror the lane index through the scan
template <class Op>
__device__ inline u32 wave_incl_scan_rev(u32 v, Op op, u32 ident) {
    const u32 lane = __lane_id();
    // bpermute-free reversal is not available in DPP across rows; use one permute each way
    const u32 r = (u32)__builtin_amdgcn_ds_bpermute((int)((63 - lane) << 2), (int)v);
    const u32 s = wave_incl_scan(r, op, ident);
    return (u32)__builtin_amdgcn_ds_bpermute((int)((63 - lane) << 2), (int)s);
}
template <class Op>
__device__ inline u32 wave_excl_scan_rev(u32 v, Op op, u32 ident) {
    return KOLM_DPP(ident, wave_incl_scan_rev(v, op, ident), DPP_WAVE_SHL1, 0xF);
}

template <class Op>
__device__ inline u32 wave_reduce(u32 v, Op op, u32 ident) {
    return (u32)__builtin_amdgcn_readlane((int)wave_incl_scan(v, op, ident), 63);
}
struct OpAddU {
    __device__ u32 operator()(u32 a, u32 b) const { return a + b; }
};
struct OpMaxU {
    __device__ u32 operator()(u32 a, u32 b) const { return a > b ? a : b; }
};
struct OpMinU {
    __device__ u32 operator()(u32 a, u32 b) const { return a < b ? a : b; }
};

// Optional per-kernel timing hook for launchers that issue several kernels (null = off).
// Families are include/kolm.h's KOLM_KT_*; names are the kernel symbols as rocprof shows
// them; bytes are the algorithmic bytes of the launch.
struct KTimer {
    virtual void begin(int fam, const char* name, u64 bytes) = 0;
    virtual void end() = 0;
};
struct KScope {
    KTimer* t;
    KScope(KTimer* t_, int fam, const char* name, u64 bytes) : t(t_) {
        if (t) t->begin(fam, name, bytes);
    }
    ~KScope() {
        if (t) t->end();
    }
};
enum : int { KT_CLASSIFY = 0, KT_KEYGEN, KT_MSD, KT_SMALLSORT, KT_LSD, KT_LZPARSE, KT_MTF, KT_SIZES, KT_EMIT, KT_LYNDON,
             KT_REPAIR, KT_CDC };

// XCD-aware workgroup -> tile remap (speed only, never correctness): workgroups are dealt
// round-robin over the 8 XCDs, so give each XCD a contiguous range of tiles — tiles of
// one block then share an L2 (random accesses inside a block's arrays stay L2-local).
// Bijective for any grid size.
// workgroup w of a range of G workgroups -> tile index such that the workgroups one XCD runs
// (consecutive dispatches go round-robin over the 8 XCDs) take contiguous tiles
__device__ inline u32 xcd_map(u32 w, u32 G) {
    const u32 x = w & 7, j = w >> 3, q = G >> 3, r = G & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}
__device__ inline u32 xcd_tile() { return xcd_map(blockIdx.x, gridDim.x); }

// Lyndon factors of every block as sorted factor-start lists (k_duval_merge): block b's
// count[b] starts sit at start[geo.base(b) ..], the first one = base(b).  Read only where
// a rotation wraps (within a few characters of a factor end), so a block's few dozen
// starts stay in L2 and no per-position factor record is materialised.
struct Factors {
    const u32* start;
    const u32* count;
    // p's factor: start fs and length m (binary search over the block's starts)
    __device__ inline void locate(const Geom& geo, u32 p, u32& fs, u32& m) const {
        const u32 b = geo.block_of(p);
        const u32* s = start + geo.base(b);
        const u32 n = count[b];
        u32 lo = 0, len = n;
        while (len > 1) {
            const u32 half = len >> 1;
            if (s[lo + half] <= p) lo += half;
            len -= half;
        }
        fs = s[lo];
        m = (lo + 1 < n ? s[lo + 1] : geo.end(b)) - fs;
    }
};

// Everything the suffix-sorting kernels touch for one pass (linear or cyclic).
struct SortArgs {
    Geom geo;
    const u8* text;
    u32* SA;
    u32* RK;
    u32* K2;
    u32* SA2;
    u32* K22;
    Factors fac;       // cyclic: Lyndon factor starts per block
    const u8* FEd;     // cyclic: min(distance to the factor end, 255): fac is read only near the end
    u32* blk_split;    // [nb] set to 1 when a group of block b split this round
    u32 med;           // large groups of at most MED_T elements sorted by the medium form (launch_med_sort)
    const u32* blk_done;  // [nb] cyclic: block converged (no further splits possible)
    int cyclic;
    int initial;       // round 0: keys are packed characters
    u32 h;             // doubling offset of this round (round >= 1)
    const u32* KP;     // [N] this round's key by position (k_keypos), or null: keys gathered directly
    u32 key_bits;      // keys of this round are < 2^key_bits (small sort packs key|index in 32 bits)
    u32* KA;           // cyclic round 0 with 8 characters: k_keypos also writes characters 4..7 here
    u32 cls_chunk;     // k_classify: one contiguous share of the list per workgroup (else grid-stride)
    u32 xcd;           // class lists are position-ordered: per-class kernels map workgroups to
                       // XCD-contiguous list ranges (k_classify_bins)
};

// Position-ordered class lists: k_classify bins every small segment by start >> bsh (at most
// CLS_NBIN bins per class), so a class list is in (coarse) position order and the per-class
// kernels' KP gathers / RK scatters of concurrent workgroups on one XCD stay inside a few
// blocks (L2 locality).
constexpr u32 CLS_NBIN = 1024;
struct Bins {
    u32* cnt;   // [NCLASS][CLS_NBIN] counts, then class-local offsets
    u32* fill;  // [NCLASS][CLS_NBIN] placement counters
    u32 bsh;
};

// Append-only lists written by the classify / MSD / small-sort kernels.
struct Lists {
    Seg* cls[NCLASS];      // small segments per class
    u32* cls_cnt;          // [NCLASS]
    u32* next_cnt;         // [1] segments for the next round
    Seg* next;
    u32* eq_cnt;           // [1] equal-key runs longer than TILE (finalised directly)
    Seg* eq;
    u32* misc;             // [1] active elements of the round
    u32* cls_elems;        // [NCLASS] elements per small class (timing/bytes bookkeeping)
    u32* lmax;             // [1] the round's longest large segment (k_classify)
};

struct Level {
    LSeg* segs;
    u32* nseg;       // device counter
    LTile* tiles;
    u32* ntiles;     // device counter
    u32* nelem;      // device counter: elements in the level's segments
};

// ---- launchers (k_sort.hip) ----
void launch_iota(u32* SA, u64 N, hipStream_t s);
void launch_block_segs(Seg* segs, const Geom& geo, hipStream_t s);
// Up to 6 u32 ranges zeroed by one launch (a round's counters: one kernel instead of 4-6
// hipMemsetAsync fills, each a ~4.5 us launch on the sort stream)
struct ZeroSpans {
    u32* p[6];
    u32 n[6];
    // optional (done != null): p[3] holds the per-block split flags of the previous round, which
    // fold into done / last (k_update_done's rule for round `round`) before they are zeroed
    u32* done = nullptr;
    u32* last = nullptr;
    u32 round = 0;
};
void launch_zero_spans(const ZeroSpans& z, hipStream_t s);
// Up to 6 u32 ranges (p[k], n[k] words) copied to dst + o[k] by one launch: the small results
// of a batch (offsets, winners, counters) gathered for a single device-to-host copy
struct PackSpans {
    const u32* p[6];
    u32 n[6];
    u32 o[6];
};
void launch_pack_spans(const PackSpans& ps, u32* dst, hipStream_t s);
// the spans into coherent host memory, then `seq` into hseq[w] for each of the returned waves
u32 launch_spans_to_host(const PackSpans& ps, u32* hdst, u32* hseq, u32 seq, hipStream_t s);
// ncur: the list length, or (ncur_dev set) a bound for the grid with the length in ncur_dev
void launch_classify_bins(const Seg* cur, u32 ncur, const u32* ncur_dev, const SortArgs& a, const Lists& L,
                          const Level& lv0, const Bins& bn, hipStream_t s, bool bins_zeroed = false);
void launch_keypos(const SortArgs& a, u32* KP, hipStream_t s);
// the round's key gathers of every small class in one launch: class c's segments segs[c] (count[c]
// of them; 0 = not launched), wg0 filled by the launcher
struct KgClasses {
    const Seg* segs[NCLASS];
    u32 count[NCLASS];
    u32 wg0[NCLASS + 1];
};
void launch_keygen_small(KgClasses kc, const SortArgs& a, hipStream_t s);
void launch_keygen_large(const LTile* tiles, u32 ntiles, const LSeg* segs, const SortArgs& a,
                         hipStream_t s);
constexpr u32 MED_T = 8192;  // the medium sort's capacity (one 1024-thread workgroup per large group)
// the medium sort of an MSD level's groups of at most MED_T elements (count in ndev when set)
void launch_med_sort(const LSeg* segs, u32 nseg, const u32* ndev, const SortArgs& a, const Lists& L,
                     hipStream_t s);
// MSD levels: ntiles / nseg is the count, or (ndev set) a bound with the count in ndev
void launch_msd_hist(const LTile* tiles, u32 ntiles, const u32* ndev, const LSeg* segs, const SortArgs& a,
                     u32 shift, u32 width, u32* hist, hipStream_t s);
void launch_msd_scan(const LSeg* segs, u32 nseg, const u32* ndev, const SortArgs& a, u32 width, u32* hist,
                     bool last_level, const Lists& L, const Level& next, hipStream_t s);
void launch_msd_scatter(const LTile* tiles, u32 ntiles, const u32* ndev, const LSeg* segs, const SortArgs& a,
                        u32 shift, u32 width, const u32* hist, hipStream_t s);
void launch_copy_back(const LTile* tiles, u32 ntiles, const u32* ndev, const LSeg* segs, const SortArgs& a,
                      hipStream_t s);
constexpr int TINY_C = 5;  // classes 1..TINY_C (<= 32 elements): one thread per segment
void launch_tiny_sort(int c, const Seg* segs, u32 count, const SortArgs& a, const Lists& L, hipStream_t s);
void launch_small_sort(int c, const Seg* segs, u32 count, const SortArgs& a, const Lists& L,
                       hipStream_t s);
// classes 5..11 of a round in one launch (those with count 0 skipped; wg0 filled by the launcher),
// 32-bit (w32) or 64-bit sort words for all of them
struct SsClasses {
    const Seg* segs[NCLASS];
    u32 count[NCLASS];
    u32 wg0[NCLASS + 1];
};
void launch_small_sorts(SsClasses sc, bool w32, const SortArgs& a, const Lists& L, hipStream_t s);
void launch_finalize_eq(const Seg* eq, u32 count, const SortArgs& a, const Lists& L, hipStream_t s);
void launch_rounds_sum(const u32* blk_last, u32 nb, u64* out, hipStream_t s);
void launch_update_done(u32* blk_done, u32* blk_last, const u32* blk_split, u32 nb, u32 round, hipStream_t s);

// ---- k_blocks.hip: per-block scans, Lyndon factors, BBWT gather ----
u32 duval_span_bytes(const Geom& geo);  // bytes per Duval span of this batch (launch_lyndon's choice)
void launch_lyndon(const Geom& geo, const u8* text, u8* flag, u8* FEd, u32* fstart, uint4* fpre, u32* nfac,
                   u32* stack, u32* fcount, u32* tile_tmp, hipStream_t s, KTimer* kt = nullptr);
void launch_prevc(const Geom& geo, const u8* text, const u8* flag, Factors fac, u8* prevc, hipStream_t s);
void launch_bbwt_gather(const Geom& geo, const u32* SA, const u8* prevc, u8* out, hipStream_t s);
// early BBWT gather: bm[slot] bit = the slot lies in one of the *ncur_dev (<= bound) segments of cur;
// the masked gather writes out[g] = prevc[SA[g]] for the slots whose bit is set
u32 bbwt_early_round();
void launch_mark_active(const Seg* cur, const u32* ncur_dev, u32 bound, u64* bm, hipStream_t s);
void launch_bbwt_gather_masked(const Geom& geo, const u32* SA, const u8* prevc, u8* out, const u64* bm,
                               hipStream_t s);

// ---- k_lsd.hip: per-block LSD radix passes: round 0 of the cyclic sort ----
u32 lsd_tiles(const Geom& geo);
struct R0Bufs {
    const u8* text;
    const u8* FEd;    // min(distance to the factor end, 255)
    Factors fac;      // Lyndon factor starts (read only where the C characters wrap)
    const u8* code;   // [nb * 256] per-block byte -> code (launch_alpha)
    u32 chars;        // C rotation characters per key
    u32 w;            // bits per code
    u32* KP;   // [N] scratch: high key bits by position (KB)
    u32* K2;   // [N] out: sorted keys (scratch)
    u32* SA;   // [N] out: positions in C-character order (ties by position)
    u32* K22;  // [N] scratch
    u32* SA2;  // [N] scratch
    u32* RK;   // [N] out: group start slot of every position (low key bits KA by position first)
    u32* hist;                    // [lsd_tiles * 256]
    u32 *tmax, *tmin, *cmax, *cmin;  // [lsd_tiles]
    u32* HF;   // [lsd_tiles * WG] group-head masks (LSD_T / WG slots per thread)
    u32* swc = nullptr;  // [2 * nb * 16 * 256] per-(block, part) digit totals of the LSD scans / sweep passes
    u64* rec[2] = {nullptr, nullptr};  // [N] each: the LSD passes' (key, position) records (record mode)
};
// per-block code tables for round 0 (alphabet compaction), max code width of the batch
u32 launch_alpha(const Geom& geo, const u8* text, u32* pres, u8* code, u32* d_w, u32* h_w, bool compact,
                 hipStream_t s, KTimer* kt = nullptr);
// the same without the host wait: the width lands in *h_w (pinned) once stream s passes this point;
// alpha_width() turns it into the width launch_alpha returns
void launch_alpha_async(const Geom& geo, const u8* text, u32* pres, u8* code, u32* d_w, u32* h_w, hipStream_t s,
                        KTimer* kt = nullptr, bool zeroed = false);
u32 alpha_width(u32 h_w);
void launch_round0(const Geom& geo, const R0Bufs& t, Seg* next, u32* next_cnt, u32* blk_split, hipStream_t s,
                   KTimer* kt = nullptr);



// ---- k_mtf.hip ----
// bits (optional, [nb * 8], zeroed by the caller): the replay also adds each block's Rice-k
// bit counts of the 5 BBWT candidates (counters 0..4, see k_entropy.hip) — no extra pass
bool mtf_wave_mode(const Geom& geo);  // position-parallel MTF replay (batches of few blocks)
u32 mtf_chunk_bytes(const Geom& geo);  // bytes per MTF chunk of this batch (launch_mtf's choice)
u64 mtf_cp_words(const Geom& geo);    // its scratch (u32 words)
// cp_scratch ([mtf_cp_words]): range states of the three-launch compose
void launch_mtf(const Geom& geo, const u8* in, u8* out, u8* summary, u16* summary_cnt, u8* states,
                hipStream_t s, KTimer* kt = nullptr, u64* bits = nullptr, int rice_k = 2, u32* cp_scratch = nullptr);

// ---- k_entropy.hip: cheap sizes, Rice sizes / emission, MDL, emission of simple models ----
struct EmitArgs {
    Geom geo;
    const u8* text;
    const u8* mtf;
    u32* sizes;        // [nb * NCAND]
    u64* bits;         // [nb * 8] scratch (bit counters)
    u32* method;       // [nb]
    const int32_t* force;  // [nb] or null
    u32 cand_mask;
    u64* off;          // [nb + 1] payload offsets
    u8* arena;
    u64 arena_cap;
    u32* tile_tmp;     // per-tile scratch
    u32* tile_tmp2;
    int rice_k;
};
// xor / lfsr_pred size counters (5, 6) only, from the text: runs on the index stream
void launch_cheap_sizes(const EmitArgs& e, hipStream_t s);
void launch_mdl(const EmitArgs& e, const u32* lz_sizes, const u32* rp_result, const u32* v2_size, u32* status,
                hipStream_t s);
void launch_emit_simple(const EmitArgs& e, hipStream_t s);
void launch_emit_rice(const EmitArgs& e, hipStream_t s);
void launch_rice_only(const Geom& geo, const u8* in, int k, u8* out, u32* tile_tmp, u32* tile_tmp2,
                      u32* out_size, hipStream_t s);

// ---- k_v2.hip: candidate 10 (v2_new, opt-in: the reference raises NameError) ----
constexpr u32 V2_META = 11;  // per-block plane decisions (k_v2_size)
// automaton histograms + choice per block, mapped bytes as 8 plane blocks per block in U
void launch_v2_sizes(const Geom& geo, const u8* text, u32* hist, u32* sel, u8* U, hipStream_t s,
                     KTimer* kt = nullptr);
// per plane block (bounds d_pb[nplanes + 1], absolute in L): Rice bits of the runs for k 0..15, first bit
void launch_v2_runs(u32 nplanes, const u32* d_pb, const u8* L, u64* rbits, u32* b1, hipStream_t s, KTimer* kt,
                    u64 bytes);
void launch_v2_size(const Geom& geo, const u32* sel, const u64* rbits, const u32* b1, u32* meta, u32* size,
                    hipStream_t s);
// payloads of the blocks whose method is 10 (method == null: every block)
void launch_v2_emit(const Geom& geo, const u32* d_pb, const u32* meta, const u32* method, const u64* off,
                    const u8* U, const u8* L, u8* arena, hipStream_t s);

// ---- k_lz77.hip ----
// k_lz_local: a workgroup owns LZL_HOME consecutive positions
// of one block, indexes its window [home - 4096 - LZL_LEAD, home end) in LDS, and parses the
// home with LZL_HOME / LZL_CHUNK chains of 16 lanes (4 per wave)
constexpr int LZL_HOME = 4096;
constexpr int LZL_CHUNK = 256;
constexpr int LZL_LEAD = 64;    // speculative lead-in parsed before a chain's chunk start
constexpr int LZL_CAPX = 256;   // speculative matches are compared up to this far past the chunk end
constexpr u32 LZ_UNRES = 0x80000000u;  // c_exit flag: the chunk's last token reached LZL_CAPX (length unresolved)

struct LzArgs {
    Geom geo;
    const u8* text;
    // speculative tokens of chunk c live in slots [chunk start, chunk start + ntok[c])
    u32* tok_pos;      // [N] token start position
    u32* tok_len;      // [N] match length (0 = literal)
    u32* tok_dist;     // [N] match distance
    u32* tok_off;      // [N] byte offset of the token inside its chunk's speculative stream
    // fix-up tokens (true path from the real chunk entry until it meets the speculative path)
    u32* fix_pos;      // [N]
    u32* fix_len;      // [N]
    u32* fix_dist;     // [N]
    u32* fix_off;      // [N] byte offset inside the chunk's output
    u32* c_ntok;       // [nchunks] speculative token count
    u32* c_exit;       // [nchunks] first path position >= chunk end
    u32* c_bytes;      // [nchunks] speculative stream bytes
    u32* c_first;      // [nchunks] first speculative token on the true path
    u32* c_fix0;       // [nchunks] index of the first fix-up token (fix_* arrays)
    u32* c_nfix;       // [nchunks]
    u32* c_fixbytes;   // [nchunks]
    u32* c_off;        // [nchunks] byte offset of the chunk's output in the block payload
    u32* b_nfix;       // [nb] fix-up tokens of the block (fix_* slots [base, base + b_nfix))
    u32* ntok;         // [nb] total tokens of the block
    u32* lz_size;      // [nb] stream size
    u32* nlong;        // [1]
    u32 cpb;           // chunks per block
    u32 cshift;        // chunk = 1 << cshift bytes (LZL_CHUNK)
    u32* nfix;         // [1] fix-up tokens computed by the stitch (statistics)
    u64* prof;         // [8] optional k_lz_local phase clocks (KOLM_LZ_PROF=1), null = off
    u32 stitch_runs;   // k_lz_stitch_l takes runs of whole chunks lane-parallel (KOLM_STITCH_RUNS=0: off)
    // 4 KiB tile index (k_lz_tiles): rank[x] = x's stable rank among its tile's positions of the
    // same 3-gram hash, tcnt[tile * 1024 + h] = the tile's count of hash h
    u16* rank;         // [N]
    u16* tcnt;         // [nb * tiles per block * 1024]
};
// the window-index form of k_lz_local for a batch of nb blocks (KOLM_LZ_IDX; 0 = no tile index);
// launch_lz_parse runs the tile index (k_lz_tiles) first for forms 1 and 2
int lz_index_form(u32 nb);
void launch_lz_parse(const LzArgs& z, hipStream_t s, KTimer* kt = nullptr);
const char* lz_spec_name();  // the speculative-parse kernel in use (timing / roofline)
u32 lz_chunk_shift();        // log2 of the parse's chunk bytes (LzArgs::cshift) for the form in use
void launch_lz_emit(const LzArgs& z, const u32* method, const u64* off, u8* arena, hipStream_t s);

// ---- k_repair.hip: exact Re-Pair (candidate 9), one workgroup per block ----
constexpr u32 RP_RS_N = 6;       // result words per block (repair_core.h RS_*)
constexpr u32 RP_RS_SIZE = 0, RP_RS_RULES = 1, RP_RS_FINAL = 2, RP_RS_BATCHES = 3, RP_RS_ERR = 4;
constexpr u32 RP_MAX_N = 1u << 22;  // block length limit of the device Re-Pair
struct RpArgs {
    Geom geo;
    const u8* text;
    char* ws;          // workspace of the blocks of one launch group
    u64 ws_stride;     // repair_ws_bytes(bs)
    u8* out;           // [nb * out_stride] per-block payload
    u64 out_stride;    // 4 * bs + 64
    u32* result;       // [nb * RP_RS_N]
    u64* prof;         // [nb * RP_P_N] wall-clock ticks per section (KOLM_RP_PROF=1), or null
    u32* trace;        // [RP_TR_CAP * RP_TR_W] per-batch records of block 0 (KOLM_RP_TRACE=file), or null
};
constexpr u32 RP_P_N = 12;
constexpr u32 RP_TR_W = 20;        // trace record: 8 batch fields + per-section ticks
constexpr u32 RP_TR_CAP = 1u << 16;
u64 repair_ws_bytes(u32 bs);
void launch_repair(const RpArgs& a, u32 b0, u32 nblk, hipStream_t s);
void launch_rp_emit(const RpArgs& a, const u32* method, const u64* off, u8* arena, hipStream_t s);

// ---- k_cdc.hip: FastCDC chunk boundaries (PY:140-309) ----
struct CdcParams {
    const u8* d;     // device text
    u32 n;           // bytes (< 2^31)
    u32 mn, av, mx;  // min / avg / max chunk size (validated by the caller, PY:227-230)
    u32 ms, ml;      // MaskS / MaskL (PY:233-240)
};
struct CdcBufs {
    const u32* gear;       // [256] PY's GEAR table (PY:152-167)
    u64 *WS, *WL, *C, *F;  // [nw = ceil(n / 64)] bitmaps
    u32 *exitp, *join;     // [nseg = ceil(n / cdc_segment(avg, max))]
    u32* wgcnt;            // [ceil(nw / 256)]
    u32* cuts;             // [n / mn + 2] out: cut positions (chunk starts after 0), ascending
    u32* total;            // [1] out: number of cuts
};
u32 cdc_segment(u32 avg, u32 mx);
void launch_cdc(const CdcParams& p, const CdcBufs& b, hipStream_t s, KTimer* kt = nullptr);

// ---- k_decode.hip: block decoders (PY:2194-2207), one workgroup per block ----
enum : u32 { DEC_OK = 0, DEC_ELEN = 1, DEC_EFORMAT = 2 };
struct DecArgs {
    const u8* pay;    // payload arena
    const u64* poff;  // [nb + 1] payload offsets
    const u32* obase; // [nb + 1] output offsets (prefix of the original lengths)
    u8* out;          // decoded bytes
    u32* status;      // [nb] DEC_* per block (zeroed by the caller)
    const u32* list;  // blocks of this decoder
    u32 nlist;
};
void launch_dec_raw(const DecArgs& a, hipStream_t s);
void launch_dec_uleb(const DecArgs& a, bool lfsr, hipStream_t s);
// scratch arrays tpos/tval/mark/src: one u32 per output byte; ntok: [nb]
void launch_dec_lz77(const DecArgs& a, u32* tpos, u32* tval, u32* ntok, u32* mark, u32* src, hipStream_t s);
// Re-Pair (id 9): vals / rlen one u32 per payload byte (at the payload offset), ea / eb one
// u64 per output byte, nval [nb], ecount [nlist]
void launch_dec_repair(const DecArgs& a, u32* vals, u32* nval, u32* ecount, u32* rlen, u64* ea, u64* eb,
                       hipStream_t s);
// BBWT family (ids 2..6): Rice -> inverse map -> MTF decode -> inverse BBWT
struct BwArgs {
    DecArgs d;         // list = the blocks with ids 2..6
    const u32* meth;   // [nb] method ids
    const u32* vbase;  // [nb + 1] Rice value offsets (bit-plane blocks: 8 * ceil(n / 8) values)
    u8* vals;          // Rice values of bit-plane blocks
    u8* mi;            // [N] MTF indices (at obase)
    u8* bw;            // [N] BBWT string (at obase)
    u8* summ;          // [nlist * cpb * 256] MTF chunk summaries
    u8* states;        // [nlist * cpb * 256] MTF chunk entry tables
    u32 cpb;           // MTF chunks per block slot (longest block / MTF_CHUNK)
    u32* X[5];         // [N] u32 scratch of the inverse BBWT: PI, -, -, D (cycle lengths), OFF
    u64* so;           // [N] segment | offset << 32 of every slot (inverse BBWT)
    u32* th;           // [nlist * tpb * 256] counting-sort tile histograms / offsets
    u32* nd;           // [5 * nlist * nnmax] ruling-set node arrays (next, length, min, cycle min, rank)
    u32 tpb;           // counting-sort tiles per block slot
    u32 sshift;        // splitters: elements whose local index is a multiple of 1 << sshift
    u32 nnmax;         // nodes per block slot (<= BWI_NODES)
    const u32* wbase;  // [nlist + 1] first 64-bit payload word of each listed block
    u32 wmax;          // most words of one payload
    u32* fw;           // [words] Rice phase function per word (8 bits per entry phase)
    u8* es;            // [words] entry phase per word
    u32* vbw;          // [words] index of the first value starting in the word
};
constexpr u32 BWI_TILE = 4096;    // counting-sort tile of the inverse BBWT
constexpr u32 BWI_NODES = 16384;  // ruling-set nodes per block (LDS-resident in k_bwi_nodes)
void launch_dec_bw(const BwArgs& a, hipStream_t s);

}  // namespace kolm

#define KOLM_HIP_CHECK(x)                                              \
    do {                                                               \
        hipError_t e_ = (x);                                           \
        if (e_ != hipSuccess) throw ::kolm::HipError(e_, #x, __LINE__); \
    } while (0)

namespace kolm {
struct HipError {
    hipError_t err;
    const char* what;
    int line;
    HipError(hipError_t e, const char* w, int l) : err(e), what(w), line(l) {}
};
}  // namespace kolm

// host-side links between kolm_api.cpp and kolm_comm.cpp (RCCL)
#include <vector>
struct kolm_ctx;
namespace kolm {
int ctx_device(const kolm_ctx* c);
// kolm_encode_blocks_multi's reassembly over the process's devices (kolm_comm.cpp)
int multi_rccl_gather(const std::vector<int>& devs, const std::vector<const u8*>& d_pay, const std::vector<u64>& nbytes,
                      u8* host, u64 cap);
void comm_shutdown();
}  // namespace kolm
