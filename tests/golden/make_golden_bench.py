#!/usr/bin/env python3
"""Per-block known answers for the benchmarked stream.

The bench encodes ``kolm.datagen.enwik_like(256 MiB, seed=ENWIK_SEED + rank)`` in
1 MiB fixed blocks (bench.py).  The reference itself (PY) needs hours per 1 MiB block
for that volume, so these answers come from the oracle (oracle/kolm_oracle.cpp), which
is pinned to PY's own outputs by tests/test_oracle.py (goldens from make_golden.py /
make_golden_large.py).  Per block this records the reference's per-block MDL loop
(PY:2350-2369) over the candidate list truncated to ids 0..8 (the hot path) and over
PY's full list 0..9 (Re-Pair by the O(n log n) restatement, checked against the
O(n*rules) one in tests/test_oracle.py):

    sizes    len(payload) of ids 0..9
    w9/w10   MDL winner over ids 0..8 / 0..9 (strict '<', ties -> lowest id)
    sha9     sha256 of the ids-0..8 winner's payload
    sha10    sha256 of the ids-0..9 winner's payload (only when it differs from w9)
    lz       sha256 of the LZ77 stream (id 7, PY:1711-1763), whatever wins

Usage (build container, 8 CPUs; ~10 min per 256 blocks):
    python tests/golden/make_golden_bench.py [--ranks 0] [--mib 256]
Writes tests/golden/bench_stream.json (merging ranks already present).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kolmogorovlike-datacompressor_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.dont_write_bytecode = True

OUT = os.path.join(HERE, "bench_stream.json")


def block_record(block: bytes) -> dict:
    import oracle
    pays = [oracle.candidate(m, block) for m in range(10)]
    sizes = [len(p) for p in pays]
    w9 = min(range(9), key=lambda m: (sizes[m], m))
    w10 = min(range(10), key=lambda m: (sizes[m], m))
    rec = {"sizes": sizes, "w9": w9, "w10": w10,
           "sha9": hashlib.sha256(pays[w9]).hexdigest(),
           "lz": hashlib.sha256(pays[7]).hexdigest()}
    if w10 != w9:
        rec["sha10"] = hashlib.sha256(pays[w10]).hexdigest()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="0", help="comma-separated bench ranks (seed = ENWIK_SEED + rank)")
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--bs", type=int, default=1 << 20)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    from kolm import datagen
    out = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            out = json.load(f)
    out.setdefault("generator", "kolm.datagen.enwik_like(mib << 20, seed=ENWIK_SEED + rank)")
    out.setdefault("oracle", "oracle/kolm_oracle.cpp (PY-pinned), Re-Pair by oracle/repair_lm.cpp")
    out.setdefault("ranks", {})
    for r in (int(x) for x in a.ranks.split(",")):
        n = a.mib << 20
        data = datagen.enwik_like(n, seed=datagen.ENWIK_SEED + r)
        nb = (n + a.bs - 1) // a.bs
        t0 = time.time()
        with ThreadPoolExecutor(a.threads) as ex:
            recs = list(ex.map(lambda i: block_record(data[i * a.bs:(i + 1) * a.bs]), range(nb)))
        out["ranks"][str(r)] = {"seed": datagen.ENWIK_SEED + r, "bytes": n, "block_size": a.bs,
                                "input_sha256": hashlib.sha256(data).hexdigest(), "blocks": recs}
        print(f"rank {r}: {nb} blocks in {time.time() - t0:.0f} s", flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
