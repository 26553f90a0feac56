#!/usr/bin/env python3
"""Known answers at scale computed by the Python reference itself (adds to large.json).

Run only in the build container (needs /root/reference; tens of minutes):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_scale.py

Adds to tests/golden/large.json, without touching the entries make_golden_large.py wrote:
  * "lz77" for enwik_256k and gradient_1m: PY's encode_lz77 (PY:1711-1763) on 256 KiB of
    enwik-style text and on the gradient BMP's first 1 MiB;
  * case "enwik_128k_repair": PY's repair_compress (PY:1841-1911, the O(n * rules)
    recount) on 128 KiB of enwik-style text (seed 77), "repair" {len, sha256};
  * case "bench_block0_repair": the same on block 0 of bench.py's stream (1 MiB);
  * case "bench_block0": PY's encode_lz77 on that block.
Arguments (optional): the case names to (re)compute.
The GPU and the oracle are checked against these in test_gpu_parity.py / test_oracle.py.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kolmogorovlike-datacompressor_amd"))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

REPAIR_CASE = "enwik_128k_repair"


def inputs():
    from kolm import datagen as D
    return {
        ("enwik_256k", "lz77"): lambda: D.enwik_like(1 << 18),
        ("gradient_1m", "lz77"): lambda: D.gradient_bmp()[: 1 << 20],
        (REPAIR_CASE, "repair"): lambda: D.enwik_like(1 << 17, seed=77),
        # block 0 of bench.py's rank-0 stream (enwik_like(n)[:1 MiB] does not depend on n):
        # PY's Re-Pair of a whole 1 MiB bench block (about an hour)
        ("bench_block0_repair", "repair"): lambda: D.enwik_like(1 << 20),
        # PY's LZ77 of the same bench block (round 6: the bench's LZ77 stream at 1 MiB rests on PY
        # itself, not only on the oracle; about 5 minutes)
        ("bench_block0", "lz77"): lambda: D.enwik_like(1 << 20),
    }


def run(key):
    from make_golden import load_reference
    ref = load_reference()
    name, kind = key
    data = inputs()[key]()
    t0 = time.time()
    out = ref.encode_lz77(data)[0] if kind == "lz77" else ref.repair_compress(data)[0]
    return key, {"input": {"len": len(data), "sha256": hashlib.sha256(data).hexdigest()},
                 kind: {"len": len(out), "sha256": hashlib.sha256(out).hexdigest()},
                 "_seconds": round(time.time() - t0, 1)}


def main():
    path = os.path.join(HERE, "large.json")
    with open(path) as f:
        large = json.load(f)
    keys = [k for k in inputs() if len(sys.argv) < 2 or k[0] in sys.argv[1:]]
    with ProcessPoolExecutor(max_workers=len(keys)) as ex:
        for (name, kind), res in ex.map(run, keys):
            print(name, kind, res["_seconds"], "s", flush=True)
            ent = large.setdefault(name, {"input": res["input"]})
            if ent["input"] != res["input"]:
                raise SystemExit(f"{name}: input differs from the recorded one")
            ent[kind] = res[kind]
            ent.setdefault("_seconds", {})[kind] = res["_seconds"]
    with open(path, "w") as f:
        json.dump(large, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
