/* kolm.h — C ABI of libkolm_hip.so, the MI355X (gfx950) block-transform hot path of
 * KolmogorovLike-DataCompressor v2-2.
 *
 * Reference interfaces replaced (PY = final_researched/kolm_final_researched_v2-2.py):
 *   kolm_bbwt_forward      <- bbwt_forward(bytes)->bytes                PY:351-423
 *   kolm_mtf_encode        <- mtf_encode(bytes)->List[int]              PY:460-468
 *   kolm_rice_encode       <- rice_encode(seq, k)->bytes                PY:1413-1421
 *   kolm_lz77_encode       <- encode_lz77(bytes)->(bytes, {})           PY:1686-1763
 *   kolm_bbwt_mtf_rice     <- encode_bbwt_mtf_rice(block, flags, k=2)   PY:2028-2073
 *   kolm_encode_blocks     <- the per-block MDL loop of compress_blocks_fixed
 *                             (candidates 0..9 of _select_encoders, argmin with
 *                             ties -> lowest id)                        PY:2152-2178, 2332-2369
 *                             candidate 9 = repair_compress            PY:1817-1911
 *   kolm_encode_blocks_device: same, input already resident in device memory
 *                             (bench / multi-GPU path; PY has no equivalent).
 *   kolm_encode_blocks_multi: same as kolm_encode_blocks over several devices of one
 *                             process (contiguous block shards, one host thread and
 *                             context per device).
 *   kolm_toc_write / kolm_toc_read: the KOLR container's header + TOC on the host
 *                             (PY:2375-2445 writer, PY:2451-2530 reader; kolm_toc.cpp).
 *   kolm_comm_* / kolm_gather_payloads: RCCL over xGMI (kolm_comm.cpp) — the reassembly
 *                             of independently encoded block shards (PY:2350-2369 blocks,
 *                             PY:2375-2445 the container they feed) onto one rank.
 *
 * Conventions: plain pointers and sizes; caller-allocated buffers with explicit
 * capacities; every function returns 0 (KOLM_OK) or a negative code; no exception
 * crosses the ABI.  One context per device; calls on one context are serialised
 * (internally locked).  The free functions (kolm_bbwt_forward, ...) use the default
 * context created by kolm_init().
 */
#ifndef KOLM_H
#define KOLM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KOLM_OK 0
#define KOLM_EARG (-1)     /* bad argument */
#define KOLM_ECAP (-2)     /* output capacity too small */
#define KOLM_EHIP (-3)     /* HIP runtime error (message: kolm_last_error) */
#define KOLM_ERCCL (-4)    /* RCCL (collective) error (message: kolm_last_error) */
#define KOLM_ENOINIT (-5)  /* kolm_init not called */
#define KOLM_EFORMAT (-6)  /* malformed container (message: PY's ValueError text) */
#define KOLM_ERANGE (-7)   /* a container field overflows (PY: struct.error) */

/* Candidate method ids (index into PY _select_encoders(), PY:2152-2165). */
#define KOLM_M_RAW 0
#define KOLM_M_XOR 1
#define KOLM_M_BBWT 2
#define KOLM_M_BBWT_BP 3
#define KOLM_M_BBWT_NIB 4
#define KOLM_M_BBWT_BR 5
#define KOLM_M_BBWT_GRAY 6
#define KOLM_M_LZ77 7
#define KOLM_M_LFSR 8
#define KOLM_M_REPAIR 9
#define KOLM_M_V2NEW 10
#define KOLM_NCAND 11          /* ids 0..10 are computed on the GPU */
#define KOLM_DEFAULT_MASK 0x3FFu  /* the reference's candidate set as shipped, ids 0..9 (v2_new raises in PY) */
#define KOLM_FULL_MASK 0x7FFu     /* + v2_new (id 10) with the automaton evaluated serially (opt-in) */
#define KOLM_HOTPATH_MASK 0x1FFu  /* BBWT / MTF+Rice / LZ77 path of the north star, ids 0..8 */
#define KOLM_REPAIR_MAX_BLOCK (1u << 22)  /* candidate 9 handles blocks up to 4 MiB */

typedef struct kolm_ctx kolm_ctx;

/* Kernel families timed with HIP events when timing is enabled (kolm_ctx_set_timing). */
#define KOLM_KT_CLASSIFY 0   /* k_classify */
#define KOLM_KT_KEYGEN 1     /* k_keypos, k_keygen_small, k_keygen_large */
#define KOLM_KT_MSD 2        /* k_msd_hist, k_msd_scan, k_msd_scatter, k_copy_back */
#define KOLM_KT_SMALLSORT 3  /* k_small_sort<1..11>, k_single, k_finalize_eq */
#define KOLM_KT_LSD 4        /* per-block LSD radix passes of the cyclic round 0: k_lsd_*, k_r0_* */
#define KOLM_KT_LZPARSE 5    /* k_lz_local (LDS 3-gram index + speculative parse), k_lz_stitch */
#define KOLM_KT_MTF 6        /* k_mtf_summary, k_mtf_compose, k_mtf_replay */
#define KOLM_KT_SIZES 7      /* k_sizes, k_mdl, k_offsets */
#define KOLM_KT_EMIT 8       /* emission kernels */
#define KOLM_KT_LYNDON 9     /* k_duval_*, Lyndon scans, k_prevc, k_bbwt_gather */
#define KOLM_KT_REPAIR 10    /* k_repair (one workgroup per block), k_rp_emit */
#define KOLM_KT_CDC 11       /* k_cdc_flags, k_cdc_spec, k_cdc_stitch, k_cdc_count/scan/emit */
#define KOLM_NKT 12

typedef struct kolm_ktime {
    double ms;          /* summed launch durations (HIP events on the library stream) */
    uint64_t launches;
    uint64_t bytes;     /* algorithmic HBM bytes of those launches */
} kolm_ktime;

/* Per-batch statistics reported by the encode entry points. */
typedef struct kolm_stats {
    uint32_t lin_rounds;      /* linear suffix-order rounds: 0 (Lyndon factors by Duval, LZ77 index in LDS) */
    uint32_t cyc_rounds;      /* prefix-doubling rounds, cyclic omega-order (max over blocks) */
    uint64_t lin_active;      /* 0 (kept for ABI stability) */
    uint64_t cyc_active;      /* same, cyclic */
    uint64_t lz_tokens;       /* LZ77 tokens over all blocks */
    uint64_t lz_long;         /* LZ77 parse positions that needed exact long-match resolution */
    double ms_total;          /* device time of the whole batch (HIP events) */
    double ms_sa;             /* of which: linear + cyclic suffix sorting */
    double ms_lz;             /* of which: LZ77 match + parse */
    double ms_entropy;        /* of which: BBWT gather + MTF + Rice sizes */
    double ms_emit;           /* of which: MDL + payload emission */
    kolm_ktime kt[KOLM_NKT];  /* per kernel family, filled when timing is enabled */
    double ms_repair;         /* Re-Pair (candidate 9) on its own stream, overlapping the rest */
    uint64_t rp_rules;        /* Re-Pair rules over all blocks */
    uint64_t rp_batches;      /* Re-Pair batches (sequential depth) summed over blocks */
    uint64_t rp_final;        /* Re-Pair final sequence symbols over all blocks */
    uint64_t lz_fix;          /* LZ77 tokens the stitch computed off the speculative paths */
    uint64_t cyc_rounds_sum;  /* sum over blocks of the rounds each block needed: round 0 through
                                 the last round that split one of its groups (>= 1; independent of
                                 how blocks are batched; SURVEY §8d's per-block R, used for the
                                 byte contract) */
} kolm_stats;

/* ---- library / default context ------------------------------------------------ */
int kolm_init(int device);
int kolm_shutdown(void);
const char* kolm_last_error(void);
int kolm_device_count(int* count);

/* ---- single-block kernels on the default context (host buffers) --------------- */
/* out: n bytes. */
int kolm_bbwt_forward(const uint8_t* in, size_t n, uint8_t* out);
/* out: n bytes (MTF indices 0..255). */
int kolm_mtf_encode(const uint8_t* in, size_t n, uint8_t* out);
/* Rice code of the byte sequence, parameter k in [0, 15]; worst case
 * n*(255/2^k + 1 + k)/8 + 1 bytes. */
int kolm_rice_encode(const uint8_t* in, size_t n, int k, uint8_t* out, size_t cap, size_t* out_len);
/* LZ77 stream (worst case 2n bytes). */
int kolm_lz77_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
/* BBWT -> MTF -> bitwise map -> Rice k (flags: 0, 1 bit-plane, 4 nibble, 8 bitrev, 16 gray). */
int kolm_bbwt_mtf_rice(const uint8_t* in, size_t n, int flags, int k, uint8_t* out, size_t cap,
                       size_t* out_len);

/* ---- content-defined chunking (FastCDC) ------------------------------------------ */
/* Chunk boundaries of data[0, n) exactly as cdc_fast_boundaries_strict (PY:210-309,
 * replaces the loop at PY:247-298 + the orphan-tail merge PY:300-306): starts[0 ..
 * *nchunks] receives the chunk starts followed by n (chunk i = [starts[i], starts[i+1])).
 * cap = entries available in starts (n / min_size + 2 always suffices).  KOLM_EARG with
 * PY's messages for the parameters it rejects (0 < min <= avg <= max, avg >= 64). */
int kolm_cdc_boundaries(const uint8_t* data, uint64_t n, uint32_t min_size, uint32_t avg_size,
                        uint32_t max_size, int merge_orphan_tail, uint64_t* starts, uint64_t cap,
                        uint64_t* nchunks);

/* ---- decode side (host buffers, default context) -------------------------------- */
/* Decodes nblocks payloads of a container on the device (the decoder registry
 * _select_decoders, PY:2194-2207): block i = payloads[payload_off[i], payload_off[i+1]),
 * method id methods[i], original length orig_lens[i]; the blocks are written back to back
 * into out (sum of orig_lens bytes, out_cap available).  Method ids outside
 * KOLM_DECODE_MASK return KOLM_EARG; so do malformed payloads (message names the block). */
#define KOLM_DECODE_MASK 0x3FFu  /* every candidate id 0..9 (raw, xor, bbwt family 2..6, lz77, lfsr_pred, repair) */
int kolm_decode_blocks(const uint8_t* payloads, const uint64_t* payload_off, const uint32_t* methods,
                       const uint32_t* orig_lens, uint32_t nblocks, uint8_t* out, uint64_t out_cap);

/* ---- container (host only: no device call, usable without a GPU) ---------------- */
/* Header + TOC of a KOLR container (PY:2213-2326 CDC, PY:2332-2445 fixed): mode 0 fixed /
 * 1 CDC, size_field = block size (fixed) or avg_size (CDC), nblocks entries of method id,
 * original length and payload length.  Writes every byte that precedes the payload area
 * (the payloads follow back to back) into out[0, cap); *out_len receives the count (out
 * may be NULL to query it).  KOLM_ERANGE when nblocks > 65535 or total_len >= 2^32. */
int kolm_toc_write(int mode, uint32_t size_field, uint64_t total_len, uint32_t nblocks,
                   const uint32_t* methods, const uint32_t* orig_lens, const uint64_t* payload_lens,
                   uint8_t* out, uint64_t cap, uint64_t* out_len);
/* Parses a whole container buf[0, n): fields[4] = {mode, size_field, total_len, nblocks},
 * *payload_start = offset of the payload area, methods / orig_lens (cap >= nblocks
 * entries) and payload_off (nblocks + 1 entries, relative to the payload area).  Checks
 * exactly what PY's decompress checks before decoding (magic, truncations, RLE size, EF
 * sum, trailing bytes): KOLM_EFORMAT with PY's message otherwise; KOLM_ECAP (fields and
 * *payload_start filled) when cap < nblocks. */
int kolm_toc_read(const uint8_t* buf, uint64_t n, uint32_t* fields, uint64_t* payload_start,
                  uint32_t* methods, uint32_t* orig_lens, uint64_t* payload_off, uint32_t cap);

/* ---- batched hot entry (host buffers, default context) ------------------------- */
/* Encodes nblocks blocks of `data` (block i = data[starts[i] .. starts[i]+lens[i]);
 * blocks contiguous and non-empty: fixed chunking when all lens are equal except a
 * shorter last one, otherwise content-defined chunks, e.g. kolm_cdc_boundaries' output
 * for compress_blocks_cdc, PY:2213-2326).
 * sizes[i*KOLM_NCAND + m] receives the payload size of candidate m (UINT32_MAX if the
 * candidate is disabled by cand_mask).  method[i] receives the MDL winner, or the
 * forced method when force_method != NULL and force_method[i] >= 0.  The winners'
 * payloads are written back to back into payload_arena in block order;
 * payload_off[i] / payload_off[i+1] delimit block i (nblocks+1 entries). */
int kolm_encode_blocks(const uint8_t* data, const uint64_t* starts, const uint32_t* lens,
                       uint32_t nblocks, uint32_t cand_mask, const int32_t* force_method,
                       uint32_t* sizes, uint32_t* method, uint8_t* payload_arena,
                       uint64_t arena_cap, uint64_t* payload_off, kolm_stats* stats);

/* compress_blocks_fixed (PY:2332-2445) in one call on the default context: the host
 * buffer data[0, n) goes up through a ring of pinned staging chunks (parallel host copies
 * beside the DMA), every block of block_size bytes is encoded (candidates cand_mask, MDL),
 * and the KOLR container (header + TOC by kolm_toc_write, then the winners' payloads copied
 * straight from device memory) is assembled in a pinned host buffer owned by the context:
 * *out / *out_len describe it until the next call on the default context: callers on
 * several threads must serialise the call AND their read of *out (the Python binding holds
 * one lock across both), since the next call reuses the buffer.  Inputs above
 * 2^31 bytes run as several device batches.  KOLM_ERANGE when the block count exceeds
 * 65535 or n >= 2^32 (PY's struct.error). */
int kolm_compress_fixed(const uint8_t* data, uint64_t n, uint32_t block_size, uint32_t cand_mask,
                        const uint8_t** out, uint64_t* out_len, kolm_stats* stats);

/* Second phase of kolm_compress_fixed: copy the container it described (*out, *out_len)
 * into the caller's buffer dst[0, n) (n <= *out_len) with the context's host copy
 * threads (page faults of a fresh destination and the memcpy itself spread over them).
 * Same serialisation rule as kolm_compress_fixed's *out.  KOLM_ECAP when n exceeds the
 * container. */
int kolm_result_copy(uint8_t* dst, uint64_t n);

/* kolm_encode_blocks over ngpu devices (0..ngpu-1, clamped to the device count and the
 * block count) of this process: fixed blocks of block_size over data[0, total), block i
 * of shard r lives on device r, shards are contiguous block ranges, one host thread and
 * context per device.  The shards' payloads are reassembled with RCCL: one
 * ncclCommInitAll communicator over the devices (created on first use, kept until
 * kolm_shutdown), every device's payload arena received into device 0 in one group over
 * xGMI, then one copy into payload_arena (KOLM_MULTI_GATHER=host: each device copies its
 * own payloads to the host instead).  Outputs exactly as kolm_encode_blocks (block order;
 * sizes [nblocks*KOLM_NCAND], method [nblocks], payload_off [nblocks+1]).  stats
 * (optional) sums counts and takes the max of times over devices.  KOLM_ERCCL on a
 * collective error. */
int kolm_encode_blocks_multi(int ngpu, const uint8_t* data, uint64_t total, uint32_t block_size,
                             uint32_t cand_mask, const int32_t* force_method, uint32_t* sizes,
                             uint32_t* method, uint8_t* payload_arena, uint64_t arena_cap,
                             uint64_t* payload_off, kolm_stats* stats);

/* ---- explicit contexts and device-resident batches ------------------------------ */
int kolm_ctx_create(int device, kolm_ctx** out);
int kolm_ctx_destroy(kolm_ctx* ctx);
/* Pre-allocates device scratch for batches of up to total_bytes with blocks of up to
 * max_block bytes (optional: buffers grow on demand otherwise). */
int kolm_ctx_reserve(kolm_ctx* ctx, uint64_t total_bytes, uint32_t max_block);
/* Allocate / free / copy device memory through the context's HIP runtime. */
int kolm_dev_alloc(kolm_ctx* ctx, uint64_t bytes, void** dptr);
int kolm_dev_free(kolm_ctx* ctx, void* dptr);
int kolm_memcpy_h2d(kolm_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int kolm_memcpy_d2h(kolm_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int kolm_ctx_sync(kolm_ctx* ctx);
/* Enable (1) / disable (0) per-launch HIP-event timing of the kernel families. */
int kolm_ctx_set_timing(kolm_ctx* ctx, int enable);
/* 1: run every launch of the next batches on one stream (kernels serialised: each kernel's
 * solo duration, for profiling); 0 (default, or KOLM_SERIAL=1 at context creation): the
 * sort chain, the LZ77 parse and Re-Pair overlap on their own streams. */
int kolm_ctx_set_serial(kolm_ctx* ctx, int serial);
/* Per-kernel timing accumulated since timing was enabled, as JSON text
 * {"k_name": {"ms": .., "launches": .., "bytes": .., "family": KOLM_KT_*, "stream":
 * "sort"|"index"|"repair"}, ...} (bytes = algorithmic HBM bytes; stream = the
 * HIP stream the kernel ran on).  *len receives the length; buf may be NULL to query it. */
int kolm_ctx_kernel_times(kolm_ctx* ctx, char* buf, size_t cap, size_t* len);
/* Fixed-size blocks of d_data (device pointer, total bytes, block_size).  Payloads go
 * to the device arena d_arena (cap bytes); h_sizes / h_method / h_off are host arrays
 * as in kolm_encode_blocks.  Blocks until the batch is complete. */
int kolm_encode_blocks_device(kolm_ctx* ctx, const uint8_t* d_data, uint64_t total,
                              uint32_t block_size, uint32_t cand_mask,
                              const int32_t* force_method, uint8_t* d_arena, uint64_t arena_cap,
                              uint32_t* h_sizes, uint32_t* h_method, uint64_t* h_off,
                              kolm_stats* stats);
/* Content-defined blocks of d_data: block i = [h_bounds[i], h_bounds[i+1]), h_bounds[0] = 0,
 * strictly increasing, nblocks + 1 entries (PY:2213-2326).  Outputs as
 * kolm_encode_blocks_device. */
int kolm_encode_blocks_device_var(kolm_ctx* ctx, const uint8_t* d_data, const uint32_t* h_bounds,
                                  uint32_t nblocks, uint32_t cand_mask, const int32_t* force_method,
                                  uint8_t* d_arena, uint64_t arena_cap, uint32_t* h_sizes,
                                  uint32_t* h_method, uint64_t* h_off, kolm_stats* stats);
/* kolm_cdc_boundaries over a device-resident buffer; h_starts are host u32 entries. */
int kolm_cdc_boundaries_device(kolm_ctx* ctx, const uint8_t* d_data, uint64_t n, uint32_t min_size,
                               uint32_t avg_size, uint32_t max_size, int merge_orphan_tail,
                               uint32_t* h_starts, uint64_t cap, uint64_t* nchunks);
/* kolm_decode_blocks over device-resident payloads (e.g. an encode arena): block i =
 * d_payloads[payload_off[i], payload_off[i+1]) with payload_off / methods / orig_lens on
 * the host; the blocks are written back to back into d_out (device, out_cap bytes).
 * ms (optional) receives the device time of the decode kernels (HIP events). */
int kolm_decode_blocks_device(kolm_ctx* ctx, const void* d_payloads, const uint64_t* payload_off,
                              const uint32_t* methods, const uint32_t* orig_lens, uint32_t nblocks,
                              void* d_out, uint64_t out_cap, double* ms);

/* ---- collectives: RCCL over xGMI, one process per GPU (kolm_comm.cpp) ------------- */
/* The only data exchange of the multi-GPU path: blocks are independent (PY:2350-2369), so
 * each rank encodes its block shard alone and the payloads are gathered onto one rank to
 * write the container (PY:2375-2445).  Every function returns KOLM_ERCCL on an RCCL error
 * (message: kolm_last_error).  Calls on one communicator are serialised. */
#define KOLM_COMM_ID_BYTES 128
typedef struct kolm_comm kolm_comm;
/* A fresh communicator id (ncclGetUniqueId): one rank creates it, every rank passes the
 * same KOLM_COMM_ID_BYTES bytes to kolm_comm_init (the caller moves them between the
 * processes: kolm.parallel does it over a TCP socket at MASTER_ADDR). */
int kolm_comm_unique_id(uint8_t* id);
/* Rank `rank` of an nranks-rank communicator on ctx's device (ncclCommInitRank: returns
 * when every rank has joined).  One rank per device. */
int kolm_comm_init(kolm_ctx* ctx, int nranks, int rank, const uint8_t* id, kolm_comm** out);
int kolm_comm_destroy(kolm_comm* comm);
int kolm_comm_rank(kolm_comm* comm, int* rank, int* nranks);
/* values[0, count) (host memory, 8-byte elements: dtype 0 uint64, 1 double) reduced over
 * every rank in place (op 0 sum, 1 max); synchronous.  kolm_comm_barrier: an all-reduce of
 * one word. */
int kolm_comm_allreduce(kolm_comm* comm, void* values, uint32_t count, int dtype, int op);
int kolm_comm_barrier(kolm_comm* comm);
/* Gathers every rank's payloads onto rank dst.  Each rank passes its payload arena
 * d_arena[0, nbytes) (device memory of its context, complete — e.g. as
 * kolm_encode_blocks_device returned it) and its nblocks method ids / nblocks + 1 payload
 * offsets (host arrays, as kolm_encode_blocks_device returned them).  On dst, d_dst
 * (device, dst_cap bytes) receives the ranks' payloads back to back in rank order,
 * method_all / off_all (host, dst_cap_blocks / dst_cap_blocks + 1 entries; either may be
 * NULL) the ranks' ids in rank order and their offsets into d_dst (off_all[total blocks] =
 * total bytes).  On every rank rank_bytes / rank_blocks (nranks entries, optional)
 * receive each rank's sizes.  When the payloads or ids do not fit dst's capacities every
 * rank returns KOLM_ECAP (sizes filled) and nothing is transferred.  async_op != 0:
 * returns once the transfers are queued on the communicator's stream; d_arena must stay
 * unmodified and the outputs are valid only after kolm_comm_wait (or the next call on the
 * communicator) — the transfer of one batch then runs while the next one encodes. */
int kolm_gather_payloads(kolm_comm* comm, const void* d_arena, uint64_t nbytes, const uint32_t* method,
                         const uint64_t* payload_off, uint32_t nblocks, int dst, void* d_dst, uint64_t dst_cap,
                         uint32_t dst_cap_blocks, uint64_t* rank_bytes, uint32_t* rank_blocks,
                         uint32_t* method_all, uint64_t* off_all, int async_op);
/* Completes the communicator's asynchronous gather, if any (every rank). */
int kolm_comm_wait(kolm_comm* comm);

#ifdef __cplusplus
}
#endif
#endif /* KOLM_H */
