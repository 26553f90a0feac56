#!/usr/bin/env python3
"""Golden fixtures for the content-defined (FastCDC) block path, made by importing PY.

PY = /root/reference/final_researched/kolm_final_researched_v2-2.py (read-only).  Run
ONLY in the build container (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_cdc.py

Outputs (committed, data only):
  tests/golden/cdc.npz        per case: cdc_fast_boundaries_strict (PY:210-309) as int64
                              (start, end) pairs (inputs rebuilt by boundary_cases() from
                              kolm.datagen, sha256 in cdc.json), and for the container cases the
                              compress_blocks_cdc (PY:2213-2326) container with PY's full
                              candidate list ("full") and with the list truncated to ids
                              0..8 ("ids0_8", same ids, SURVEY.md §8d config 5 note)
  tests/golden/cdc.json       parameters, lengths and sha256 of every array above
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kolmogorovlike-datacompressor_amd"))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

from kolm import datagen  # noqa: E402
from make_golden import HOBBIT, load_reference  # noqa: E402


def boundary_cases() -> dict:
    """name -> (data, (min, avg, max), merge_orphan_tail)."""
    enw = datagen.enwik_like(1 << 20)
    grad = datagen.gradient_bmp()
    rnd = datagen.splitmix64_bytes(1 << 19)
    sine = datagen.sine_wav()
    chk = datagen.checker_bmp()
    return {
        "enwik1m_default": (enw, (4096, 8192, 16384), True),
        "enwik128k_small": (enw[:1 << 17], (64, 128, 256), True),
        "enwik64k_min1": (enw[:1 << 16], (1, 64, 1024), True),
        "enwik1m_odd": (enw, (3000, 5000, 20000), True),
        "enwik300k_nomerge": (enw[:300007], (4096, 8192, 16384), False),
        "enwik200k_eq": (enw[:200000], (1000, 1000, 1000), True),
        "enwik1m_big": (enw, (16384, 65536, 262144), True),
        "grad512k_2k": (grad[:1 << 19], (1024, 2048, 8192), True),
        "random512k": (rnd, (4096, 8192, 16384), True),
        "sine_full": (sine, (4096, 8192, 16384), True),
        "checker_full": (chk, (2048, 4096, 8192), True),
        "zeros_tail": (bytes(16384 * 3 + 100), (4096, 8192, 16384), True),
        "zeros_tail_nomerge": (bytes(16384 * 3 + 100), (4096, 8192, 16384), False),
        "zeros_odd": (bytes(100000), (1000, 3000, 12345), True),
        "tiny_le_min": (b"abc" * 10, (64, 128, 256), True),
        "tiny_min_plus1": (enw[:65], (64, 128, 256), True),
        "one_byte": (b"\x07", (64, 128, 256), True),
    }


def container_cases() -> dict:
    """name -> (data, (min, avg, max)); small enough for PY's pure-Python candidates."""
    enw = datagen.enwik_like(1 << 16)
    rnd = datagen.splitmix64_bytes(4096)
    mix = (HOBBIT * 8)[:2048] + rnd[:2048] + bytes(3000) + bytes(i & 0xFF for i in range(2048)) + enw[:3000]
    return {
        "hobbit_64": (HOBBIT * 10, (64, 256, 1024)),
        "mix_512": (mix, (512, 1024, 4096)),
        "enwik12k_default": (enw[:12288], (4096, 8192, 16384)),
        "zeros20k_default": (bytes(20480), (4096, 8192, 16384)),
        "empty": (b"", (4096, 8192, 16384)),
        "one": (b"\x07", (4096, 8192, 16384)),
    }


def main():
    ref = load_reference()
    arrays, man = {}, {"reference": "final_researched/kolm_final_researched_v2-2.py",
                       "boundaries": {}, "containers": {}}

    def put(key, data):
        arr = data if isinstance(data, np.ndarray) else np.frombuffer(bytes(data), dtype=np.uint8)
        arrays[key] = arr
        return {"len": int(arr.size), "sha256": hashlib.sha256(arr.tobytes()).hexdigest()}

    t_all = time.time()
    for name, (data, (mn, av, mx), merge) in boundary_cases().items():
        t0 = time.time()
        b = ref.cdc_fast_boundaries_strict(data, mn, av, mx, merge)
        # inputs are rebuilt by boundary_cases() (kolm.datagen); only their hash is kept
        man["boundaries"][name] = {
            "params": [mn, av, mx], "merge": merge,
            "input": {"len": len(data), "sha256": hashlib.sha256(data).hexdigest()},
            "bounds": put(f"{name}/bounds", np.array(b, dtype="<i8").reshape(-1, 2)), "nchunks": len(b)}
        print(f"bounds {name:20s} n={len(data):8d} chunks={len(b):6d} {time.time() - t0:6.2f}s", flush=True)

    full = ref._select_encoders

    def truncated():
        return full()[:9]

    for name, (data, (mn, av, mx)) in container_cases().items():
        t0 = time.time()
        ref._select_encoders = full
        c_full = ref.compress_blocks_cdc(data, mn, av, mx)
        ref._select_encoders = truncated
        c_09 = ref.compress_blocks_cdc(data, mn, av, mx)
        ref._select_encoders = full
        assert ref.decompress(c_full) == data
        man["containers"][name] = {"params": [mn, av, mx], "input": put(f"c_{name}/input", data),
                                   "full": put(f"c_{name}/full", c_full), "ids0_8": put(f"c_{name}/ids0_8", c_09)}
        print(f"container {name:18s} full={len(c_full)} ids0_8={len(c_09)} {time.time() - t0:6.2f}s", flush=True)

    np.savez_compressed(os.path.join(HERE, "cdc.npz"), **arrays)
    with open(os.path.join(HERE, "cdc.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print(f"done in {time.time() - t_all:.1f}s")


if __name__ == "__main__":
    main()
