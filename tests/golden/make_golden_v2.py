#!/usr/bin/env python3
"""Golden fixtures for candidate 10 (v2_new, encode_new_pipeline PY:1498-1576) by
importing the Python reference (PY).

As shipped, PY's pipeline calls circuit_map_automaton_forward(block) with its default
parallel=True and raises NameError (os / ProcessPoolExecutor are never imported,
PY:1037-1043), so PY itself never emits id 10.  SURVEY §8f row 3 defines
the candidate "with parallel=False semantics": here the module's
circuit_map_automaton_forward is rebound to the same function with parallel=False (the
serial branch at PY:1033-1035 — the reference code is otherwise unchanged; the selection
result is the same as the parallel one, _best_choice folds the same candidates).

Run ONLY in the build container:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_v2.py

Outputs (committed, data only):
  tests/golden/v2new.npz    per input: the v2_new payload, the automaton (mode, param);
                            containers of compress_blocks_fixed with PY's candidate list
                            0..10 (v2_new enabled) for small inputs
  tests/golden/v2new.json   names, sizes, sha256, automaton choices
"""
from __future__ import annotations

import functools
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

from make_golden import golden_inputs, load_reference  # noqa: E402

MAX_V2_INPUT = 8192  # PY's bbwt_forward on 8 binary planes is slow beyond this


def v2_cases(inputs: dict) -> dict:
    return {k: v for k, v in inputs.items() if len(v) <= MAX_V2_INPUT}


def container_cases(inputs: dict) -> dict:
    mix = (inputs["text_hobbit"][:1024] + inputs["rand4k"][:1024] + bytes(1024) + inputs["ramp8k"][:1024]
           + inputs["sine4k"][:1024] + inputs["grad4k"][:1024])
    return {
        "hobbit_b512": (inputs["text_hobbit"][:3000], 512),
        "mix_b1024": (mix, 1024),
        "sine_b1024": (inputs["sine4k"], 1024),
        "small_b3": (b"abracadabra", 3),
        "one": (b"\x07", 2048),
    }


def main():
    ref = load_reference()
    orig = ref.circuit_map_automaton_forward
    ref.circuit_map_automaton_forward = functools.partial(orig, parallel=False)
    arrays = {}
    manifest = {"reference": "final_researched/kolm_final_researched_v2-2.py", "automaton": "parallel=False",
                "kernels": {}, "containers": {}}

    def put(key, data):
        arr = np.frombuffer(bytes(data), dtype=np.uint8)
        arrays[key] = arr
        return {"len": int(arr.size), "sha256": hashlib.sha256(arr.tobytes()).hexdigest()}

    inputs = golden_inputs()
    for name, data in v2_cases(inputs).items():
        t0 = time.time()
        payload = ref.encode_new_pipeline(data)
        assert ref.decode_new_pipeline(payload, len(data)) == data
        _, theta = ref.circuit_map_automaton_forward(data) if data else (b"", {"mode": 0, "param": 0, "H0": 0.0})
        ent = {"input": put(f"{name}/input", data), "v2new": put(f"{name}/v2new", payload),
               "mode": int(theta["mode"]), "param": int(theta["param"]), "H0": float(theta["H0"])}
        manifest["kernels"][name] = ent
        print(f"{name:16s} n={len(data):6d} -> {len(payload):6d} mode={ent['mode']} param={ent['param']} "
              f"{time.time() - t0:6.2f}s", flush=True)
    for cname, (data, bs) in container_cases(inputs).items():
        t0 = time.time()
        c = ref.compress_blocks_fixed(data, bs)  # the full list, v2_new (id 10) included
        assert ref.decompress(c) == data
        arrays[f"C/{cname}/input"] = np.frombuffer(data, dtype=np.uint8)
        arrays[f"C/{cname}/full10"] = np.frombuffer(c, dtype=np.uint8)
        manifest["containers"][cname] = {"block_size": bs, "input_len": len(data),
                                         "full10": {"len": len(c), "sha256": hashlib.sha256(c).hexdigest()}}
        print(f"container {cname:14s} {len(c)} B {time.time() - t0:6.2f}s", flush=True)
    np.savez_compressed(os.path.join(HERE, "v2new.npz"), **arrays)
    with open(os.path.join(HERE, "v2new.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
