#!/usr/bin/env python3
"""Benchmark: compress MB/s at fixed block size, bit-exact path, 1..8 GPUs.

Workload (BASELINE.json north star / SURVEY.md §8d configs 3-4): per GPU, 256 MiB of
synthetic enwik-style text (kolm.datagen.enwik_like, seed 20251212 + rank) resident in
HBM, 1 MiB fixed blocks, all candidates 0..8 evaluated per block, MDL winner emitted.
One step = one full compress of the rank's batch from HBM to a device payload arena
(+ for N > 1 the RCCL gather of every rank's payloads and method ids to rank 0).
Weak scaling: per-GPU work is fixed; value = all ranks' input bytes / max-over-ranks time.
The timed steps run with kernel timing OFF; a separate pass of --kt-steps steps records
HIP events around every launch (per-kernel durations), and at N=1 one more step runs
with the streams serialised (each kernel's solo duration).

Also reported:
  roofline      the critical path: the SORT STREAM (Lyndon -> omega-order sort -> BBWT
                gather -> MTF + Rice sizes; the LZ77 parse runs beside it on the index
                stream and is hidden).  achieved = SURVEY §8d contract bytes of that stream
                per step / summed device time of its kernels per step (HIP events on that
                stream); traffic = PMC-measured HBM bytes of the same kernels per step
                (profiles/pmc_summary.json, tools/pmc_traffic.py).  The dominant single
                kernel and the LZ77 parse (overlapped and solo) are reported beside it.
  cpu_baseline  the oracle (faithful C++ restatement of the reference CPU path, 5x BBWT
                as in PY) on a bounded sample of the same stream, rank 0 at N=1 only.
  detail.parity_blocks  every block of the timed output (sizes of ids 0..8, winner, winner
                sha256) against tests/golden/bench_stream.json (oracle answers).

  detail.config4_shard (N = 1) / detail.config4 (N > 1)  BASELINE config 4: 256 MiB TOTAL of
                rank 0's stream in 1 MiB blocks round-robin over the GPUs (block i on rank
                i mod N) with the async RCCL gather (payloads, ids, offsets) to rank 0; at N = 1
                the shard one GPU of the 8-GPU run encodes (blocks i = 0 mod 8, 32 MiB), timed
                alone, parity per block against the rank-0 fixture.
  --strong      makes config 4 the headline (scaling "strong"): every rank encodes its
                round-robin shard of the one 256 MiB stream; value = 256 MiB / time.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 via
python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
(the launcher only sets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*: this process uses no PyTorch —
device memory, the RCCL communicator, barriers and reductions all go through libkolm_hip.so's
C ABI, kolm.parallel.Comm; the communicator id travels over TCP at MASTER_ADDR:MASTER_PORT+1)
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

if os.environ.get("KOLM_BENCH_TORCH_RT"):  # A/B only: bind to torch's bundled HIP runtime instead
    import torch  # noqa: F401
import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "kolmogorovlike-datacompressor_amd"))

from kolm import _lib, datagen  # noqa: E402
from kolm.parallel import Comm  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GOLDEN = os.path.join(REPO, "tests", "golden")
# what stops a kernel short of the HBM roof when it is not bandwidth (measured)
LIMITER = {
    "k_lz_local": "instruction issue + LDS latency (SQ counters of this build, profiles/r06/sq_lz_local.txt): "
                  "per wave 20.8 K VALU, 8.7 K SALU, 1.3 K LDS instructions; a wave issues 47 % of its cycles, "
                  "waits on data 33 %, stalls on issue 20 %, 35 % of its LDS cycles are bank conflicts; 4 waves "
                  "per SIMD (33 KB of LDS per workgroup: the text window, its 3-gram index and the slot of every "
                  "home position); HBM traffic is only the text window and the token records (PMC 1.53 GB per "
                  "launch), so the HBM contract fraction is not its bound",
    "k_repair": "latency: one workgroup per block, barrier-separated batches of dependent global accesses",
    "k_duval_span": "LDS latency: sequential Duval over each thread's 128-byte chunk, then tree merges of "
                    "adjacent factorisations (dependent LDS byte compares / bitmap scans); reads the text once",
    "k_lsd_scatter_w<3, 2, 1>": "random 4-byte gathers of the next key by position (one 32-64 B request each) "
                                "beside the streaming LSD scatter",
}
SORT_STREAM_LIMITER = ("random 4-byte gathers / scatters of ranks and keys by position (one 32-64 B HBM "
                       "request per element in the doubling rounds and the RK scatter), streaming LSD passes at "
                       "2-3 TB/s, and latency-bound Lyndon / MTF-compose chains (DESIGN.md §4)")
MB = 1e6


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(data: bytes, bs: int, budget_s: float):
    """Oracle (reference algorithms) on whole 1 MiB blocks of the same stream: every
    candidate 0..8 + MDL, as the reference's per-block loop (Re-Pair excluded).  Timed
    block-parallel on T threads (ctypes releases the GIL; blocks are independent, SURVEY
    §8d) and on 1 thread, each for about half the budget."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    nblk = max(1, len(data) // bs)

    def one(i):
        blk = data[(i % nblk) * bs:(i % nblk + 1) * bs]
        sizes = [len(oracle.candidate(m, blk)) for m in range(9)]
        _ = int(np.argmin(sizes))
        return len(blk)

    # Re-Pair (id 9) per block, for the full-candidate comparison: the oracle's O(n log n)
    # restatement (the reference's own O(n * rules) recount is far slower), 1 thread
    t0 = time.time()
    nr = 0
    for i in range(2):
        oracle.repair_fast(data[(i % nblk) * bs:(i % nblk + 1) * bs])
        nr += 1
    rp_s = (time.time() - t0) / nr

    # per stage on one 1 MiB block of the stream, 1 thread (BBWT once; the candidates 2..6 run it
    # once each, as PY does), beside SURVEY §6's extracted-reference times for a 1 MiB text block
    blk0 = data[:bs]
    stage = {}
    t0 = time.time()
    bw = oracle.bbwt_forward(blk0)
    stage["bbwt"] = time.time() - t0
    t0 = time.time()
    oracle.rice_encode(oracle.mtf_encode(bw), 2)
    stage["mtf_rice"] = time.time() - t0
    t0 = time.time()
    oracle.encode_lz77(blk0)
    stage["lz77"] = time.time() - t0
    t0 = time.time()
    oracle.encode_xor(blk0)
    oracle.encode_lfsr(blk0)
    stage["xor_lfsr"] = time.time() - t0
    per_block = 5 * (stage["bbwt"] + stage["mtf_rice"]) + stage["lz77"] + stage["xor_lfsr"]

    # 1 thread
    t0 = time.time()
    n1 = b1 = 0
    while True:
        n1 += one(b1)
        b1 += 1
        if time.time() - t0 >= budget_s / 2 or b1 >= nblk:
            break
    el1 = time.time() - t0
    # T threads, whole waves of T blocks
    T = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16
    t0 = time.time()
    nt = bt = 0
    with ThreadPoolExecutor(T) as ex:
        while True:
            nt += sum(ex.map(one, range(bt, bt + T)))
            bt += T
            if time.time() - t0 >= budget_s / 2:
                break
    elt = time.time() - t0
    model = _cpu_model()
    return {"value": round(nt / elt / MB, 5), "unit": "MB/s", "cores": T, "kind": "port",
            "sample": f"{bt} x {bs >> 20} MiB blocks on {T} threads ({elt:.1f} s) and {b1} on 1 thread "
                      f"({el1:.1f} s) of the bench stream, candidates 0..8 (5x BBWT, list MTF, bit-serial "
                      f"Rice, exhaustive 4 KiB LZ77), Re-Pair (id 9) excluded as in the GPU path; {model}",
            "single_thread": {"value": round(n1 / el1 / MB, 5), "cores": 1},
            "per_stage_s": {k: round(v, 3) for k, v in stage.items()},
            "per_stage_note": (f"one {bs >> 20} MiB block of the stream, 1 thread: ids 0..8 = 5 x (BBWT + MTF/Rice) + LZ77 "
                               f"+ xor/lfsr = {per_block:.2f} s per block; SURVEY §6 extracted reference C++ on a 1 MiB "
                               "text block (Xeon, 8 vCPU, g++ -O3 -march=native): BBWT 4.181 s, MTF+Rice 0.035 s, LZ77 "
                               "2.147 s = 23.1 s per block for the same candidate set.  Same algorithms (comparison-"
                               "sort prefix doubling of each Lyndon factor's rotations, heap merge, list MTF, "
                               "exhaustive 4 KiB LZ77); the gap is the BBWT stage (DESIGN.md §6) and the CPU ("
                               + model + " here)"),
            "survey_extracted_ref_s": {"bbwt": 4.181, "mtf_rice": 0.035, "lz77": 2.147},
            "full_candidates": {
                "value": round(1.0 / (el1 / max(b1, 1) + rp_s) * (bs / MB) * T, 5), "unit": "MB/s", "cores": T,
                "sample": f"per-block time of ids 0..8 (1 thread, above) + Re-Pair by the O(n log n) oracle "
                          f"({rp_s:.2f} s per {bs >> 20} MiB block, 2 blocks), scaled to {T} block-parallel threads"}}


def load_golden_stream(rank: int, n: int, bs: int):
    """Per-block oracle answers for this rank's stream (make_golden_bench.py), or None."""
    path = os.path.join(GOLDEN, "bench_stream.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        g = json.load(f).get("ranks", {}).get(str(rank))
    if not g or g["bytes"] != n or g["block_size"] != bs:
        return None
    return g


def golden_subset(g, idx):
    """The oracle records of the blocks idx of a stream (a rank's round-robin shard)."""
    return {"blocks": [g["blocks"][i] for i in idx]} if g else None


def check_blocks(g, sizes, method, arena_host, off, ncand, wkey, shakey):
    """Blocks whose sizes (ids < ncand), winner and winner sha256 all match the oracle."""
    ok = 0
    for i, rec in enumerate(g["blocks"]):
        if list(map(int, sizes[i][:ncand])) != rec["sizes"][:ncand] or int(method[i]) != rec[wkey]:
            continue
        pay = arena_host[int(off[i]):int(off[i + 1])]
        if hashlib.sha256(pay).hexdigest() == rec.get(shakey, rec["sha9"]):
            ok += 1
    return ok


COMM = None  # kolm.parallel.Comm (RCCL behind the C ABI) when WORLD_SIZE > 1


def sync_max(el, world):
    if world > 1:
        el = float(COMM.allreduce([float(el)], op="max")[0])
    return el


def sum_all(v, world):
    if world > 1:
        v = int(COMM.allreduce([int(v)])[0])
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mib", type=int, default=256, help="input MiB per GPU")
    ap.add_argument("--bs", type=int, default=1 << 20, help="block size")
    ap.add_argument("--kt-steps", type=int, default=2, help="steps of the kernel-timed pass (HIP events per launch)")
    ap.add_argument("--no-serial-pass", action="store_true", help="skip the serialised-streams step (N=1)")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of oracle CPU work (N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--full-steps", type=int, default=2,
                    help="timed steps of the full candidate list 0..9 (Re-Pair included); 0 = skip")
    ap.add_argument("--decode-steps", type=int, default=3,
                    help="timed device decode passes over the hot-path payloads (0: skip)")
    ap.add_argument("--cdc-steps", type=int, default=2,
                    help="timed steps of the content-defined (FastCDC) mode; 0 = skip")
    ap.add_argument("--v2-steps", type=int, default=1,
                    help="timed steps of the candidate list 0..10 (+ v2_new, opt-in) on --v2-mib MiB; 0 = skip")
    ap.add_argument("--v2-mib", type=int, default=32, help="input MiB of the v2_new leg")
    ap.add_argument("--config-steps", type=int, default=3,
                    help="timed repetitions of the config-2 / config-5 legs (gradient block, mixed corpus); 0 = skip")
    ap.add_argument("--host-steps", type=int, default=2,
                    help="timed kolm.compress_blocks_fixed(bytes) calls on the host buffer (PCIe-inclusive); 0 = skip")
    ap.add_argument("--strong", action="store_true",
                    help="headline = BASELINE config 4's shape: --mib MiB TOTAL (rank 0's stream) in 1 MiB blocks "
                         "round-robin over the ranks (block i on rank i mod N), RCCL gather to rank 0; strong scaling")
    ap.add_argument("--c4-steps", type=int, default=5,
                    help="timed steps of the config-4 leg (N=1: the 8-GPU shard, blocks i = 0 mod 8 of the stream; "
                         "N>1: the whole config, --mib MiB total round-robin); 0 = skip")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(rank, f"warning: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    global COMM
    if world > 1:
        COMM = Comm.from_env(device=local)
    n = a.mib << 20
    t = time.time()
    stream0 = None  # rank 0's stream: the config-4 data (256 MiB total, sharded)
    if a.strong or a.c4_steps > 0:
        stream0 = datagen.enwik_like(n, seed=datagen.ENWIK_SEED)
    data = stream0 if rank == 0 and stream0 is not None else datagen.enwik_like(n, seed=datagen.ENWIK_SEED + rank)
    log(rank, f"[bench] generated {a.mib} MiB per rank in {time.time() - t:.1f}s")
    nb_stream = (n + a.bs - 1) // a.bs
    golden_full = load_golden_stream(rank, n, a.bs)
    if a.strong:  # this rank's round-robin shard of rank 0's stream is the workload
        mine = list(range(rank, nb_stream, world))
        data = b"".join(stream0[i * a.bs:(i + 1) * a.bs] for i in mine)
        golden_full = golden_subset(load_golden_stream(0, n, a.bs), mine)
        n = len(data)

    L = _lib.load()
    ctx = _lib.device_ctx(local)

    def dsync():
        _lib.check(L.kolm_ctx_sync(ctx))

    d_in = _lib.input_buffer(ctx, data)
    cap = n + (4 << 20)
    # payload arenas: N > 1 double-buffers them, so the RCCL gather of step k (over xGMI,
    # on the communicator's stream) overlaps step k+1's encoding instead of serialising behind it
    arenas = [_lib.DeviceBuffer(ctx, cap) for _ in range(2 if world > 1 else 1)]
    pending = [None] * len(arenas)
    nstep = [0]
    arena = arenas[0]
    nb = (n + a.bs - 1) // a.bs
    sizes = np.zeros((nb, _lib.KOLM_NCAND), np.uint32)
    method = np.zeros(nb, np.uint32)
    off = np.zeros(nb + 1, np.uint64)
    dsync()

    def step(st, mask=_lib.KOLM_HOTPATH_MASK):
        j = nstep[0] % len(arenas)
        nstep[0] += 1
        buf = arenas[j]
        if pending[j] is not None:  # the gather of two steps ago still reads this buffer
            pending[j].wait()
            pending[j] = None
        _lib.check(L.kolm_encode_blocks_device(ctx, d_in.ptr, n, a.bs, mask, None, buf.ptr, cap,
                                               sizes.ctypes.data, method.ctypes.data, off.ctypes.data,
                                               ctypes.byref(st)))
        if world > 1:
            pending[j] = COMM.gather_payloads(buf.ptr, int(off[-1]), method, off, dst=0, async_op=True,
                                              dst_cap_blocks=nb)
        return buf

    def drain():
        """every gather in flight completed (inside the timed region for timed steps)"""
        for j, w in enumerate(pending):
            if w is not None:
                w.wait()
                pending[j] = None
        dsync()

    def timed(fn, k):
        """k calls of fn between barriers + device syncs; max over ranks of the wall time"""
        drain()
        if world > 1:
            COMM.barrier()
        dsync()
        t0 = time.perf_counter()
        res = [fn() for _ in range(k)]
        drain()
        if world > 1:
            COMM.barrier()
        return sync_max(time.perf_counter() - t0, world), res

    for _ in range(a.warmup):
        step(_lib.Stats())
    # ---- the headline: K steps, no per-launch timing events ----
    el, _ = timed(lambda: step(_lib.Stats()), a.steps)
    arena = arenas[(nstep[0] - 1) % len(arenas)]
    ms_step = el / a.steps * 1e3
    ntot = sum_all(n, world)  # whole-job input bytes per step
    value = ntot * a.steps / el / MB

    # ---- parity of the timed output, block by block, against the oracle's answers ----
    golden = golden_full
    arena_host = arena.download(int(off[-1])) if golden else None
    parity_ok = check_blocks(golden, sizes, method, arena_host, off, 9, "w9", "sha9") if golden else 0
    parity_checked = nb if golden else 0
    parity = {"ok": sum_all(parity_ok, world), "checked": sum_all(parity_checked, world), "blocks": sum_all(nb, world)}
    log(rank, f"[bench] parity {parity}")

    # BASELINE config 4 (256 MiB TOTAL in 1 MiB blocks, round-robin over the GPUs, RCCL
    # gather to rank 0).  N > 1: the whole config, every rank its shard i = rank (mod N)
    # of rank 0's stream, gathered asynchronously into rank 0 as in the headline.  N = 1:
    # what one GPU of the 8-GPU run encodes — the 32 blocks i = 0 (mod 8) — timed alone,
    # so the per-GPU rate of config 4's shard size is measured beside the 256 MiB one.
    c4 = None
    if a.c4_steps > 0 and not a.strong and stream0 is not None:
        G = world if world > 1 else 8
        r4 = rank if world > 1 else 0
        mine4 = list(range(r4, nb_stream, G))
        n4 = len(mine4) * a.bs  # 1 MiB blocks of a whole-MiB stream: every block full
        d4 = _lib.input_buffer(ctx, b"".join(stream0[i * a.bs:(i + 1) * a.bs] for i in mine4))
        cap4 = n4 + (4 << 20)
        ar4 = [_lib.DeviceBuffer(ctx, cap4) for _ in range(2)]
        pend4 = [None, None]
        cnt4 = [0]
        sz4 = np.zeros((len(mine4), _lib.KOLM_NCAND), np.uint32)
        m4 = np.zeros(len(mine4), np.uint32)
        o4 = np.zeros(len(mine4) + 1, np.uint64)

        def c4_step():
            j = cnt4[0] % 2
            cnt4[0] += 1
            if pend4[j] is not None:
                pend4[j].wait()
                pend4[j] = None
            _lib.check(L.kolm_encode_blocks_device(ctx, d4.ptr, n4, a.bs, _lib.KOLM_HOTPATH_MASK, None,
                                                   ar4[j].ptr, cap4, sz4.ctypes.data, m4.ctypes.data,
                                                   o4.ctypes.data, None))
            if world > 1:
                pend4[j] = COMM.gather_payloads(ar4[j].ptr, int(o4[-1]), m4, o4, dst=0, async_op=True,
                                                dst_cap_blocks=nb_stream)

        def c4_drain():
            for j in range(2):
                if pend4[j] is not None:
                    pend4[j].wait()
                    pend4[j] = None

        c4_step()
        c4_drain()
        drain()
        if world > 1:
            COMM.barrier()
        dsync()
        t0 = time.perf_counter()
        for _ in range(a.c4_steps):
            c4_step()
        c4_drain()
        dsync()
        if world > 1:
            COMM.barrier()
        el4 = sync_max(time.perf_counter() - t0, world)
        g4 = golden_subset(load_golden_stream(0, a.mib << 20, a.bs), mine4)
        ok4 = 0
        if g4:
            ok4 = check_blocks(g4, sz4, m4, ar4[(cnt4[0] - 1) % 2].download(int(o4[-1])), o4, 9, "w9", "sha9")
        tot4 = sum_all(n4, world)
        c4 = {"value": round(tot4 * a.c4_steps / el4 / MB, 2), "unit": "MB/s", "steps": a.c4_steps,
              "ms_per_step": round(el4 / a.c4_steps * 1e3, 3), "blocks_per_gpu": len(mine4),
              "bytes_per_gpu": n4, "partition": f"round_robin over {G}",
              "parity_blocks": f"{sum_all(ok4, world)}/{sum_all(len(mine4), world)}" if g4 else None,
              "note": ("config 4 whole: rank 0's stream, block i on rank i mod N, async RCCL gather (payloads, ids, "
                       "offsets) to rank 0 inside the timed region") if world > 1 else
                      ("config 4's per-GPU shard at N = 8 (blocks i = 0 mod 8 of the 256 MiB stream, 32 MiB) on one "
                       "GPU, no collective; MB/s of this GPU alone")}
        del d4, ar4


    # ---- kernel-timed pass (HIP events around every launch) ----
    _lib.check(L.kolm_ctx_set_timing(ctx, 1))
    kt_stats = []

    def kt_step():
        kt_stats.append(_lib.Stats())
        return step(kt_stats[-1])

    elk, _ = timed(kt_step, max(1, a.kt_steps))
    _lib.check(L.kolm_ctx_set_timing(ctx, 0))
    ktimes = _lib.kernel_times(ctx)
    ks = max(1, a.kt_steps)
    stats = [s.as_dict() for s in kt_stats]
    s0 = stats[-1]

    # ---- one serialised step (N=1): every kernel's solo duration ----
    solo = None
    if world == 1 and not a.no_serial_pass:
        _lib.check(L.kolm_ctx_set_serial(ctx, 1))
        _lib.check(L.kolm_ctx_set_timing(ctx, 1))
        els, _ = timed(lambda: step(_lib.Stats()), 1)
        _lib.check(L.kolm_ctx_set_timing(ctx, 0))
        _lib.check(L.kolm_ctx_set_serial(ctx, 0))
        solo = {"times": _lib.kernel_times(ctx), "ms_step": els * 1e3}

    # ---- roofline of the critical path: the sort stream, SURVEY §8d byte contract ----
    pmc_path = os.path.join(REPO, "profiles", "pmc_summary.json")
    pmc = {}
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f).get("kernels", {})
    idx_k = ("k_lz_local", "k_lz_stitch", "k_cheap_sizes", "k_prevc", "k_lz_emit", "k_repair", "k_rp_")
    sort_k = {k: v for k, v in ktimes.items() if v.get("stream") == "sort"}
    if not sort_k:  # streams serialised (KOLM_SERIAL=1): every kernel but the index stream's
        sort_k = {k: v for k, v in ktimes.items() if not k.startswith(idx_k) and v.get("stream") != "repair"}
    sort_ms = max(sum(v["ms"] for v in sort_k.values()) / ks, 1e-9)
    rsum = s0["cyc_rounds_sum"]  # sum over blocks of the doubling rounds each block needed
    lens = np.full(nb, a.bs, np.int64)
    lens[-1] = n - a.bs * (nb - 1)
    r_avg = rsum / nb  # equal blocks: sum_b n_b R_b = bs * rsum
    out_w = int(sizes[:, 2:7].min(axis=1).astype(np.int64).sum())  # the BBWT family's emitted size
    # per block: n(44 R_lin + 8) Lyndon (R_lin = 0: Duval, no linear SA) + n(44 R + 7)
    # cyclic SA + BBWT gather + 2n MTF + n Rice size pass + (n + out_w) winner emit
    contract = int(n * (8 + 7 + 2 + 1 + 1) + 44 * float((lens * r_avg).sum()) + out_w)
    achieved = contract / (sort_ms * 1e-3) / 1e9
    builder = sum(v["bytes"] for v in sort_k.values()) / ks
    # PMC traffic of the sort stream per step: every profiled kernel except the index
    # stream's (LZ77 parse + stitch, cheap sizes, predecessor bytes) and the runtime's copy /
    # fill kernels, per encode batch of the profiled run (tools/pmc_traffic.py BATCHES)
    per_batch = [v["bytes_per_batch"] for k, v in pmc.items()
                 if "bytes_per_batch" in v and not k.startswith("__amd") and not k.startswith(idx_k)]
    traffic = int(sum(per_batch)) if per_batch else None
    # the dominant kernel: the largest summed device time over the kernel-timed steps, any stream.
    # Its contract bytes per launch: k_lz_local's SURVEY §8d term 35n + out_lz, every other
    # kernel's algorithmic bytes as the library counts them.  frac from the
    # overlapped launches (HIP events on its own stream beside the sort stream) and from the
    # serialised step (the kernel alone, N = 1); traffic = PMC HBM bytes per launch
    # (profiles/pmc_summary.json) and its ratio to the contract.
    dom_name, dom = max(ktimes.items(), key=lambda kv: kv[1]["ms"]) if ktimes else ("", {"ms": 0, "launches": 1,
                                                                                            "bytes": 0})
    dom_avg = dom["ms"] / max(dom["launches"], 1)
    if dom_name == "k_lz_local":
        dom_contract = int(35 * n + int(sizes[:, 7].astype(np.int64).sum()))
        dom_cterm = "SURVEY 8d LZ77 term 35n + out_lz per launch"
    else:
        dom_contract = int(dom["bytes"] / max(dom["launches"], 1))
        dom_cterm = "the library's algorithmic bytes per launch (DESIGN.md §4)"
    dom_solo = None
    if solo and dom_name in solo["times"]:
        st = solo["times"][dom_name]
        dom_solo = st["ms"] / max(st["launches"], 1)
    dom_pmc = next((v for k, v in pmc.items() if k.split("<")[0] == dom_name and "hbm_bytes_per_launch" in v), None)

    def _frac(ms):
        return round(dom_contract / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if ms else None
    roof_dom = {"name": dom_name, "avg_launch_ms": round(dom_avg, 4),
                "avg_launch_ms_solo": round(dom_solo, 4) if dom_solo else None,
                "launches_per_step": dom["launches"] // ks,
                "contract_bytes_per_launch": dom_contract, "contract": dom_cterm,
                "achieved_GBs": round(dom_contract / (dom_avg * 1e-3) / 1e9, 2) if dom_avg else None,
                "frac": _frac(dom_avg),
                "achieved_GBs_solo": round(dom_contract / (dom_solo * 1e-3) / 1e9, 2) if dom_solo else None,
                "frac_solo": _frac(dom_solo),
                "builder_bytes_per_launch": int(dom["bytes"] / max(dom["launches"], 1)),
                "traffic_pmc_bytes_per_launch": int(dom_pmc["hbm_bytes_per_launch"]) if dom_pmc else None,
                "traffic_over_contract": round(dom_pmc["hbm_bytes_per_launch"] / dom_contract, 4)
                if dom_pmc and dom_contract else None,
                "limiter": LIMITER.get(dom_name, "random 4-byte gathers / scatters")}
    sdom_name, sdom = max(sort_k.items(), key=lambda kv: kv[1]["ms"]) if sort_k else ("", {"ms": 0, "launches": 1,
                                                                                           "bytes": 0})
    sdom_avg = sdom["ms"] / max(sdom["launches"], 1)
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": f"sort stream (critical path: {len(sort_k)} kernels, Lyndon -> omega-order sort -> "
                      "BBWT gather -> MTF + Rice sizes)",
            "kernel_ms_per_step": round(sort_ms, 3),
            "contract_bytes_per_step": contract,
            "contract": f"SURVEY 8d: n(44 R_lin + 8) + n(44 R + 7) + 2n + n + (n + out_w) per block, R_lin = 0 "
                        f"(Duval), R = per-block doubling rounds (mean {r_avg:.2f}), out_w = {out_w}",
            "builder_bytes_per_step": int(builder),
            "builder_frac": round(builder / (sort_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if sort_ms else None,
            "traffic_frac": round(traffic / (sort_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if traffic else None,
            "traffic_over_contract": round(traffic / contract, 4) if traffic and contract else None,
            "stream_span_ms": round(s0["ms_sa"] + s0["ms_entropy"], 3),
            "limiter": SORT_STREAM_LIMITER,
            "dominant_kernel": roof_dom,
            "sort_stream_largest_kernel": {"name": sdom_name, "avg_launch_ms": round(sdom_avg, 4),
                                           "launches_per_step": sdom["launches"] // ks,
                                           "achieved_GBs": round(sdom["bytes"] / max(sdom["launches"], 1) /
                                                                 (sdom_avg * 1e-3) / 1e9, 2) if sdom_avg else None}}
    lz = ktimes.get("k_lz_local")
    lz_detail = None
    if lz:
        lz_avg = lz["ms"] / lz["launches"]
        lz_detail = {"avg_launch_ms_overlapped": round(lz_avg, 3),
                     "avg_launch_ms_solo": round(solo["times"]["k_lz_local"]["ms"], 3)
                     if solo and "k_lz_local" in solo["times"] else None,
                     "algorithmic_bytes_per_launch": int(lz["bytes"] / lz["launches"]),
                     "contract_bytes_per_launch": int(35 * n + int(sizes[:, 7].astype(np.int64).sum())),  # 35n + out_lz
                     "limiter": LIMITER["k_lz_local"]}
    # whole pipeline: every kernel's algorithmic bytes per step / wall time per step
    alg_step = sum(v["bytes"] for v in ktimes.values()) / ks
    pipe = {"algorithmic_bytes_per_step": int(alg_step),
            "achieved_GBs": round(alg_step / (ms_step * 1e-3) / 1e9, 2),
            "frac": round(alg_step / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}

    # Decode side (decompress, PY:2451-2550): the payloads still resident in the arena
    # decoded back on the device (kolm_decode_blocks_device, every id 0..9); checked
    # against the input once, then timed with the same discipline.
    blens = np.full(nb, a.bs, np.uint32)
    blens[-1] = n - a.bs * (nb - 1)
    cur_arena = [arenas[(nstep[0] - 1) % len(arenas)]]

    def decode_leg():
        d_out = _lib.DeviceBuffer(ctx, n + 64)
        dms = ctypes.c_double(0.0)
        acc = [0.0]

        def dstep():
            _lib.check(L.kolm_decode_blocks_device(ctx, cur_arena[0].ptr, off.ctypes.data, method.ctypes.data,
                                                   blens.ctypes.data, nb, d_out.ptr, n + 64, ctypes.byref(dms)))
            acc[0] += dms.value

        dstep()
        dsync()
        ok = d_out.download(n) == data
        if not ok:
            raise SystemExit("decode leg: device round trip differs from the input")
        acc[0] = 0.0
        eld, _ = timed(dstep, a.decode_steps)
        d_out.free()
        return {"value": round(ntot * a.decode_steps / eld / MB, 2), "unit": "MB/s", "steps": a.decode_steps,
                "ms_per_step": round(eld / a.decode_steps * 1e3, 2),
                "kernel_ms_per_step": round(acc[0] / a.decode_steps, 2), "round_trip_exact": ok,
                "methods": np.bincount(method, minlength=10).tolist()}

    dec = decode_leg() if a.decode_steps > 0 else None

    # The reference's FULL candidate list (ids 0..9: + exact Re-Pair, its own stream beside
    # the hot path): same data, same timing discipline; reported beside the hot-path value.
    full = None
    if a.full_steps > 0:
        method_hot, off_hot, sizes_hot = method.copy(), off.copy(), sizes.copy()
        step(_lib.Stats(), _lib.KOLM_DEFAULT_MASK)
        fst = []

        def full_step():
            fst.append(_lib.Stats())
            return step(fst[-1], _lib.KOLM_DEFAULT_MASK)

        elf, _ = timed(full_step, a.full_steps)
        cur_arena[0] = arenas[(nstep[0] - 1) % len(arenas)]
        f0 = fst[-1].as_dict()
        full = {"value": round(ntot * a.full_steps / elf / MB, 2), "unit": "MB/s", "steps": a.full_steps,
                "ms_per_step": round(elf / a.full_steps * 1e3, 2), "candidates": "0..9 (PY's full list)",
                "ms_repair": round(f0["ms_repair"], 2), "ratio": round(float(off[-1]) / n, 4),
                "methods": np.bincount(method, minlength=10).tolist(),
                "repair_rules_per_block": round(f0["rp_rules"] / nb, 1),
                "repair_batches_per_block": round(f0["rp_batches"] / nb, 1)}
        if golden:
            fh = cur_arena[0].download(int(off[-1]))
            fok = check_blocks(golden, sizes, method, fh, off, 10, "w10", "sha10")
            full["parity_blocks"] = f"{sum_all(fok, world)}/{sum_all(nb, world)}"
        # decode of those payloads (Re-Pair wins every text block): grammar expansion on the device
        if a.decode_steps > 0:
            full["decode"] = decode_leg()
        method[:], off[:], sizes[:] = method_hot, off_hot, sizes_hot

    # Content-defined mode (compress_blocks_cdc, PY:2213-2326): FastCDC boundaries on the
    # device (PY's default 4096/8192/16384) + candidates 0..8 over the variable-length
    # chunks, same resident data, same timing discipline; reported beside the value.
    cdc = None
    if a.cdc_steps > 0:
        ccap = n // 4096 + 3
        hst = np.zeros(ccap, np.uint32)
        nch = ctypes.c_uint64(0)
        csz = np.zeros((ccap, _lib.KOLM_NCAND), np.uint32)
        cmeth = np.zeros(ccap, np.uint32)
        coff = np.zeros(ccap + 1, np.uint64)
        cst = {}

        def cdc_step():
            t_b = time.perf_counter()
            _lib.check(L.kolm_cdc_boundaries_device(ctx, d_in.ptr, n, 4096, 8192, 16384, 1, hst.ctypes.data,
                                                    ccap, ctypes.byref(nch)))
            cst["ms_bounds"] = (time.perf_counter() - t_b) * 1e3
            st = _lib.Stats()
            _lib.check(L.kolm_encode_blocks_device_var(ctx, d_in.ptr, hst.ctypes.data, int(nch.value),
                                                       _lib.KOLM_HOTPATH_MASK, None, arenas[0].ptr, cap,
                                                       csz.ctypes.data, cmeth.ctypes.data, coff.ctypes.data,
                                                       ctypes.byref(st)))

        cdc_step()
        elc, _ = timed(cdc_step, a.cdc_steps)
        nbc = int(nch.value)
        cdc = {"value": round(ntot * a.cdc_steps / elc / MB, 2), "unit": "MB/s", "steps": a.cdc_steps,
               "ms_per_step": round(elc / a.cdc_steps * 1e3, 2), "ms_boundaries": round(cst["ms_bounds"], 2),
               "params": [4096, 8192, 16384], "chunks_per_gpu": nbc, "candidates": "0..8",
               "ratio": round(float(coff[nbc]) / n, 4)}

    # Candidate 10 (v2_new, opt-in: PY as shipped raises before computing it) on a prefix of
    # the resident input: the automaton + 8 bit planes, the BBWT of every plane (8x the
    # positions of the hot path, binary alphabet), run-length Rice; ids 0..10 + MDL.
    v2 = None
    if a.v2_steps > 0:
        n2 = min(n, a.v2_mib << 20)
        nb2 = (n2 + a.bs - 1) // a.bs
        sz2 = np.zeros((nb2, _lib.KOLM_NCAND), np.uint32)
        m2 = np.zeros(nb2, np.uint32)
        o2 = np.zeros(nb2 + 1, np.uint64)

        def v2_step():
            st = _lib.Stats()
            _lib.check(L.kolm_encode_blocks_device(ctx, d_in.ptr, n2, a.bs, _lib.KOLM_FULL_MASK, None,
                                                   arenas[0].ptr, cap, sz2.ctypes.data, m2.ctypes.data,
                                                   o2.ctypes.data, ctypes.byref(st)))

        v2_step()
        el2, _ = timed(v2_step, a.v2_steps)
        v2 = {"value": round(world * n2 * a.v2_steps / el2 / MB, 2), "unit": "MB/s", "steps": a.v2_steps,
              "ms_per_step": round(el2 / a.v2_steps * 1e3, 2), "mib_per_gpu": n2 >> 20,
              "candidates": "0..10 (v2_new opt-in)", "ratio": round(float(o2[-1]) / n2, 4),
              "methods": np.bincount(m2, minlength=11).tolist(),
              "v2_new_size_ratio": round(float(sz2[:, 10].astype(np.float64).sum()) / n2, 4)}

    # BASELINE configs 2 and 5 at their stated shapes (rank-local, resident in HBM): the
    # gradient BMP's first 1 MiB as one block, and the mixed corpus (sine WAV || checker
    # BMP || 1 MiB random) in 1 MiB blocks (3 blocks, a short tail) with per-block model
    # selection; both checked against tests/golden/mixed_corpus.json (oracle answers).
    configs = None
    if a.config_steps > 0:
        configs = {}
        mg_path = os.path.join(GOLDEN, "mixed_corpus.json")
        mg = json.load(open(mg_path)) if os.path.exists(mg_path) else {}
        for name, gen in (("gradient_1m", lambda: datagen.gradient_bmp()[: 1 << 20]),
                          ("mixed_corpus", datagen.mixed_corpus)):
            cdata = gen()
            cn = len(cdata)
            cbs = 1 << 20
            cnb = (cn + cbs - 1) // cbs
            d_c = _lib.input_buffer(ctx, cdata)
            ccap2 = 9 * cn + 4096
            d_ar = _lib.DeviceBuffer(ctx, ccap2)
            res = {}
            for label, mask, wkey, shakey, ncand in (("ids0_8", _lib.KOLM_HOTPATH_MASK, "w9", "sha9", 9),
                                                     ("ids0_9", _lib.KOLM_DEFAULT_MASK, "w10", "sha10", 10)):
                csz = np.zeros((cnb, _lib.KOLM_NCAND), np.uint32)
                cm = np.zeros(cnb, np.uint32)
                co = np.zeros(cnb + 1, np.uint64)
                cst = [_lib.Stats()]

                def cstep():
                    cst[0] = _lib.Stats()
                    _lib.check(L.kolm_encode_blocks_device(ctx, d_c.ptr, cn, cbs, mask, None, d_ar.ptr,
                                                           ccap2, csz.ctypes.data, cm.ctypes.data, co.ctypes.data,
                                                           ctypes.byref(cst[0])))

                cstep()
                elx, _ = timed(cstep, a.config_steps)
                sd = cst[0].as_dict()
                r = {"value": round(world * cn * a.config_steps / elx / MB, 2), "unit": "MB/s",
                     "ms_per_call": round(elx / a.config_steps * 1e3, 3), "device_ms": round(sd["ms_total"], 3),
                     "ms_sa": round(sd["ms_sa"], 3), "ms_lz": round(sd["ms_lz"], 3),
                     "cyclic_rounds": sd["cyc_rounds"], "ratio": round(float(co[-1]) / cn, 4),
                     "methods": cm.tolist()}
                if mask == _lib.KOLM_DEFAULT_MASK:
                    r["ms_repair"] = round(sd["ms_repair"], 3)
                g = mg.get(name)
                if g and g["input"]["len"] == cn:
                    hostp = d_ar.download(int(co[-1]))
                    r["parity_blocks"] = f"{check_blocks(g, csz, cm, hostp, co, ncand, wkey, shakey)}/{cnb}"
                res[label] = r
            res["bytes"] = cn
            res["blocks"] = cnb
            configs[name] = res
            del d_c, d_ar

    # The reference's own API on a host buffer (PCIe-inclusive, never the headline):
    # kolm.compress_blocks_fixed(bytes, 1 MiB) -> container bytes, on the bench stream.
    host = None
    if a.host_steps > 0 and world == 1:
        import kolm
        kolm._lib.ensure_init(local)
        blob = kolm.compress_blocks_fixed(data, a.bs, hot_path=True)  # warm-up (allocations)
        t0 = time.perf_counter()
        for _ in range(a.host_steps):
            blob = kolm.compress_blocks_fixed(data, a.bs, hot_path=True)
        elh = (time.perf_counter() - t0) / a.host_steps
        # its parts: PCIe H2D of the input and D2H of the payloads (pageable host memory,
        # as the API receives it), and the device encode of the same batch
        dsync()
        t0 = time.perf_counter()
        d_in.upload(data)
        h2d = time.perf_counter() - t0
        t0 = time.perf_counter()
        _ = arena.download(int(off[-1]))
        d2h = time.perf_counter() - t0
        # the reference's own call: its full candidate list 0..9 (Re-Pair included), the
        # container PY itself returns (PY:2332)
        blob_full = kolm.compress_blocks_fixed(data, a.bs)  # warm-up
        t0 = time.perf_counter()
        for _ in range(a.host_steps):
            blob_full = kolm.compress_blocks_fixed(data, a.bs)
        elf_h = (time.perf_counter() - t0) / a.host_steps
        host_full = {"value": round(n / elf_h / MB, 2), "unit": "MB/s", "ms_per_call": round(elf_h * 1e3, 2),
                     "container_bytes": len(blob_full), "device_ms_of_call": round(kolm.last_stats().get("ms_total", 0.0), 2),
                     "note": "kolm.compress_blocks_fixed(bytes, 1 MiB): PY's default candidate list 0..9 (Re-Pair "
                             "included), the container the reference's compress_blocks_fixed returns, PCIe included"}
        del blob_full
        host = {"value": round(n / elh / MB, 2), "unit": "MB/s", "steps": a.host_steps,
                "ms_per_call": round(elh * 1e3, 2), "container_bytes": len(blob),
                "device_ms_of_call": round(kolm.last_stats().get("ms_total", 0.0), 2),
                "ms_h2d_pageable": round(h2d * 1e3, 2), "ms_d2h_pageable": round(d2h * 1e3, 2),
                "ms_device_step": round(ms_step, 2),
                "pcie_share": round((h2d + d2h) / elh, 3),
                "ids0_9": host_full,
                "note": "kolm.compress_blocks_fixed(bytes, 1 MiB, hot_path=True) on the bench stream = one "
                        "kolm_compress_fixed call: the pageable input staged through pinned chunks (parallel host "
                        "copies beside the DMA), the batched device encode, TOC + payloads D2H into a pinned "
                        "container buffer, one copy into the returned bytes; ms_h2d/d2h_pageable: plain "
                        "hipMemcpy of the same bytes (kolm_memcpy_h2d/d2h) for comparison"}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(data, a.bs, a.cpu_budget)

    if rank == 0:
        hot = {kk: round(v["ms"] / ks, 3) for kk, v in sorted(ktimes.items(), key=lambda kv: -kv[1]["ms"])[:14]}
        out = {
            "metric": "compress MB/s at fixed block size, bit-exact vs reference; 1/2/4/8-GPU scaling",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_step, 2), "higher_is_better": True, "scaling": "strong" if a.strong else "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": ("BASELINE config 4: enwik-style synthetic text (kolm.datagen.enwik_like, seed "
                                    f"20251212), {a.mib} MiB TOTAL in {a.bs >> 20} MiB blocks sharded round-robin "
                                    f"over {world} GPU(s), resident in HBM, candidates 0..8 + MDL, payloads emitted "
                                    "in HBM" + (", RCCL gather to rank 0" if world > 1 else "")) if a.strong else
                                   ("enwik-style synthetic text (kolm.datagen.enwik_like, seed 20251212+rank), "
                                    f"{a.mib} MiB per GPU resident in HBM, {a.bs >> 20} MiB fixed blocks, "
                                    "candidates 0..8 + MDL, payloads emitted in HBM"
                                    + (", RCCL gather to rank 0" if world > 1 else "")),
                       "block_size": a.bs, "bytes_per_gpu": n, "blocks_per_gpu": nb,
                       "parallelism": f"block-shard x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "detail": {"parity_blocks": f"{parity['ok']}/{parity['blocks']}"
                                        + ("" if parity["checked"] == parity["blocks"]
                                           else f" ({parity['checked']} with fixtures)"),
                       "ratio": round(float(off[-1]) / n, 4),
                       "methods": np.bincount(method, minlength=10).tolist(),
                       "kernel_timed_pass_ms_per_step": round(elk / ks * 1e3, 2),
                       "serialised_step_ms": round(solo["ms_step"], 2) if solo else None,
                       "lz77_parse": lz_detail,
                       "decode": dec,
                       "full_candidates": full,
                       "cdc_mode": cdc,
                       "v2_new": v2,
                       "configs": configs,
                       "host_e2e": host,
                       "config4" if world > 1 else "config4_shard": c4,
                       "device_ms": {k: round(s0[k], 2) for k in ("ms_total", "ms_sa", "ms_lz", "ms_entropy", "ms_emit")},
                       "cyclic_rounds": s0["cyc_rounds"], "cyclic_rounds_mean_per_block": round(r_avg, 3),
                       "lz77": {"tokens": s0["lz_tokens"], "stitch_fixups": s0["lz_fix"],
                                "long_extensions": s0["lz_long"]},
                       "pipeline_roofline": pipe,
                       "families_ms_per_step": {KN: round(sum(v["ms"] for v in ktimes.values()
                                                              if _lib.KT_NAMES[v["family"]] == KN) / ks, 2)
                                                for KN in _lib.KT_NAMES
                                                if any(_lib.KT_NAMES[v["family"]] == KN for v in ktimes.values())},
                       "kernels_ms_per_step": hot,
                       "sort_stream_kernels_ms_per_step": {kk: round(v["ms"] / ks, 3) for kk, v in
                                                           sorted(sort_k.items(), key=lambda kv: -kv[1]["ms"])},
                       "solo_kernels_ms": {kk: round(v["ms"], 3) for kk, v in
                                           sorted(solo["times"].items(), key=lambda kv: -kv[1]["ms"])[:14]}
                       if solo else None},
        }
        if os.environ.get("KOLM_BENCH_ALLK"):  # A/B tooling (tools/kab.sh): every kernel
            out["detail"]["kernels_all_ms_per_step"] = {kk: round(v["ms"] / ks, 3) for kk, v in ktimes.items()}
        if cpu:
            out["detail"]["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        COMM.close()


if __name__ == "__main__":
    main()
