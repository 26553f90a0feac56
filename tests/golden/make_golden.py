#!/usr/bin/env python3
"""Generate golden fixtures by importing the Python reference (PY).

PY = /root/reference/final_researched/kolm_final_researched_v2-2.py (read-only).
Run ONLY in the build container (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Outputs (committed, data only):
  tests/golden/kernels.npz     per-input outputs of the reference hot-path functions:
                               duval_lyndon (PY:326), bbwt_forward (PY:351),
                               mtf_encode (PY:460), encode_bbwt_mtf_rice flags
                               0/1/4/8/16 (PY:2028, candidates 2..6 of PY:2152),
                               encode_lz77 (PY:1711), encode_xor (PY:2105),
                               encode_lfsr_predict (PY:1984), repair_compress (PY:1841)
  tests/golden/containers.npz  compress_blocks_fixed (PY:2332) containers, with PY's
                               full candidate list and with the list truncated to ids
                               0..8 (SURVEY.md §8d config 5 note)
  tests/golden/manifest.json   names, sizes, sha256 of every array above

Inputs are rebuilt from closed formulas by ``golden_inputs()`` (no reference data file
is copied).  The reference is imported with ``sys.modules`` registration (needed by
``@dataclass`` at PY:649) and without writing bytecode into /root/reference.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kolmogorovlike-datacompressor_amd"))
sys.dont_write_bytecode = True

from kolm import datagen  # noqa: E402

REF_PY = "/root/reference/final_researched/kolm_final_researched_v2-2.py"

HOBBIT = (
    "In a hole in the ground there lived a hobbit. Not a nasty, dirty, wet "
    "hole, filled with the ends of worms and an oozy smell, nor yet a dry, "
    "bare, sandy hole with nothing in it to sit down on or to eat: it was a "
    "hobbit-hole, and that means comfort."
).encode("utf-8")
UTF8 = "数据压缩 data compression 可逆性 reversibility —— Kolmogorov-style.".encode("utf-8")


def load_reference():
    spec = importlib.util.spec_from_file_location("kolm_ref_v22", REF_PY)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["kolm_ref_v22"] = mod
    spec.loader.exec_module(mod)
    return mod


def golden_inputs() -> dict:
    """Name -> bytes.  Shared with tests (tests/golden_inputs.py re-creates them)."""
    pat = datagen.pattern_blocks()
    grad = datagen.gradient_bmp()
    sine = datagen.sine_wav()
    chk = datagen.checker_bmp()
    d = {
        "empty": b"",
        "one": b"\x07",
        "two_ba": b"ba",
        "two_ab": b"ab",
        "aaaa": b"aaaa",
        "banana": b"banana",
        "mississippi": b"mississippi",
        "abracadabra": b"abracadabra",
        "zyx": b"zyxwvu",
        "abcabcab": b"abcabcab",
        "text_hobbit": HOBBIT * 10,
        "repetitive": b"a" * 20480,
        "abab": b"ab" * 10000,
        "abcabc": b"abc" * 6000,
        "zero16k": bytes(16384),
        "ramp8k": bytes(i & 0xFF for i in range(8192)),
        "utf8_mixed": UTF8 * 40,
        "rand4k": datagen.splitmix64_bytes(4096),
        "rand1k_seed7": datagen.splitmix64_bytes(1000, seed=7),
        "grad4k": grad[:4096],
        "grad_px4k": grad[54 + 3072 * 100: 54 + 3072 * 100 + 4096],
        "sine4k": sine[:4096],
        "checker8k": chk[:8192],
        "enwik16k": datagen.enwik_like(16384),
    }
    for b in (0, 1, 2, 6, 10, 15):
        d[f"pattern{b}_4k"] = pat[b * 65536: b * 65536 + 4096]
    # small random strings over tiny alphabets: BBWT tie / Lyndon corner cases
    rng = np.random.default_rng(12345)
    for i in range(60):
        alpha = [2, 2, 3, 4][i % 4]
        n = int(rng.integers(1, 70))
        d[f"tiny{i:02d}"] = bytes((rng.integers(0, alpha, n) + 97).astype(np.uint8))
    return d


# inputs whose LZ77 in pure Python would take > a minute are skipped there
LZ77_SKIP = set()


def container_cases(inputs: dict) -> dict:
    """Name -> (data, block_size)."""
    mix = (inputs["text_hobbit"][:2048] + inputs["rand4k"][:2048] + bytes(2048)
           + inputs["ramp8k"][:2048] + inputs["abab"][:2048] + inputs["rand4k"][2048:4096]
           + inputs["utf8_mixed"][:2048])
    return {
        "config1_zero64k": (bytes(65536), 65536),
        "hobbit_b512": (inputs["text_hobbit"], 512),
        "hobbit_b2470": (inputs["text_hobbit"], 2470),
        "mix_b2048": (mix, 2048),
        "mix_b1000": (mix, 1000),
        "small_b3": (b"abracadabra", 3),
        "empty": (b"", 2048),
        "one": (b"\x07", 2048),
        "pattern10_b1024": (inputs["pattern10_4k"], 1024),
        "sine_b2048": (inputs["sine4k"], 2048),
    }


def main():
    ref = load_reference()
    inputs = golden_inputs()
    arrays = {}
    manifest = {"reference": REF_PY, "kernels": {}, "containers": {}}

    def put(key, data):
        arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        arrays[key] = arr
        return {"len": int(arr.size), "sha256": hashlib.sha256(arr.tobytes()).hexdigest()}

    flags = {0: (False, False, False, False, False), 1: (True, False, False, False, False),
             4: (False, False, True, False, False), 8: (False, False, False, True, False),
             16: (False, False, False, False, True)}
    t_all = time.time()
    for name, data in inputs.items():
        t0 = time.time()
        ent = {"input": put(f"{name}/input", data)}
        facs = ref.duval_lyndon(data)
        ent["duval"] = put(f"{name}/duval", np.array(facs, dtype=np.int64).reshape(-1, 2).ravel().astype("<i8").view(np.uint8))
        ent["bbwt"] = put(f"{name}/bbwt", ref.bbwt_forward(data))
        ent["mtf"] = put(f"{name}/mtf", bytes(ref.mtf_encode(ref.bbwt_forward(data))))
        for f, fl in flags.items():
            payload, _ = ref.encode_bbwt_mtf_rice(data, fl[0], False, fl[2], fl[3], fl[4], rice_param=2)
            ent[f"rice{f}"] = put(f"{name}/rice{f}", payload)
        if name not in LZ77_SKIP:
            ent["lz77"] = put(f"{name}/lz77", ref.encode_lz77(data)[0])
        ent["xor"] = put(f"{name}/xor", ref.encode_xor(data)[0])
        ent["lfsr"] = put(f"{name}/lfsr", ref.encode_lfsr_predict(data)[0])
        ent["repair"] = put(f"{name}/repair", ref.repair_compress(data)[0])
        manifest["kernels"][name] = ent
        print(f"{name:16s} n={len(data):6d} {time.time() - t0:7.2f}s", flush=True)
    np.savez_compressed(os.path.join(HERE, "kernels.npz"), **arrays)

    carrays = {}
    full = ref._select_encoders

    def truncated():
        return full()[:9]

    for cname, (data, bs) in container_cases(inputs).items():
        t0 = time.time()
        ref._select_encoders = full
        c_full = ref.compress_blocks_fixed(data, bs)
        ref._select_encoders = truncated
        c_09 = ref.compress_blocks_fixed(data, bs)
        ref._select_encoders = full
        assert ref.decompress(c_full) == data
        if cname != "mix_b2048" and cname != "mix_b1000":
            assert ref.decompress(c_09) == data
        carrays[f"{cname}/input"] = np.frombuffer(data, dtype=np.uint8)
        carrays[f"{cname}/full"] = np.frombuffer(c_full, dtype=np.uint8)
        carrays[f"{cname}/ids0_8"] = np.frombuffer(c_09, dtype=np.uint8)
        manifest["containers"][cname] = {
            "block_size": bs, "input_len": len(data),
            "full": {"len": len(c_full), "sha256": hashlib.sha256(c_full).hexdigest()},
            "ids0_8": {"len": len(c_09), "sha256": hashlib.sha256(c_09).hexdigest()},
        }
        print(f"container {cname:18s} full={len(c_full)} ids0_8={len(c_09)} {time.time() - t0:6.2f}s", flush=True)
    np.savez_compressed(os.path.join(HERE, "containers.npz"), **carrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(f"done in {time.time() - t_all:.1f}s")


if __name__ == "__main__":
    main()
