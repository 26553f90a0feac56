#!/usr/bin/env python3
"""Known answers for BASELINE configs 2 and 5 at their stated shapes.

config 5: kolm.datagen.mixed_corpus() (sine WAV || checker BMP || 1 MiB splitmix64
          random bytes, 2234874 bytes) in 1 MiB fixed blocks: 3 blocks, the last one
          short.  Per block: sizes of ids 0..9, the MDL winners over ids 0..8 and 0..9
          (PY:2350-2369), the winners' sha256; and the whole KOLR container
          (PY:2332-2445) for both candidate lists (len + sha256).
config 2: bytes [0, 1 MiB) of the gradient BMP as one block, same fields.

Answers come from the oracle (PY-pinned by tests/test_oracle.py; the sine / checker /
gradient BBWT+Rice and the checker LZ77 are also pinned to PY directly by large.json).
    python tests/golden/make_golden_mixed.py      (build container, ~2 min)
Writes tests/golden/mixed_corpus.json.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kolmogorovlike-datacompressor_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.dont_write_bytecode = True


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main():
    import oracle
    from kolm import datagen as D
    cases = {"mixed_corpus": D.mixed_corpus(), "gradient_1m": D.gradient_bmp()[: 1 << 20]}
    bs = 1 << 20
    out = {}
    for name, data in cases.items():
        nb = (len(data) + bs - 1) // bs
        blocks = [data[i * bs:(i + 1) * bs] for i in range(nb)]
        with ThreadPoolExecutor(8) as ex:
            pays = list(ex.map(lambda bm: oracle.candidate(bm[1], blocks[bm[0]]),
                               [(i, m) for i in range(nb) for m in range(10)]))
        recs, w9s, w10s = [], [], []
        for i in range(nb):
            p = pays[i * 10:(i + 1) * 10]
            sizes = [len(x) for x in p]
            w9 = min(range(9), key=lambda m: (sizes[m], m))
            w10 = min(range(10), key=lambda m: (sizes[m], m))
            w9s.append(p[w9])
            w10s.append(p[w10])
            recs.append({"len": len(blocks[i]), "sizes": sizes, "w9": w9, "w10": w10,
                         "sha9": sha(p[w9]), "sha10": sha(p[w10])})
        lens = [len(b) for b in blocks]
        c9 = oracle.write_container_fixed(len(data), bs, [r["w9"] for r in recs], lens, w9s)
        c10 = oracle.write_container_fixed(len(data), bs, [r["w10"] for r in recs], lens, w10s)
        out[name] = {"input": {"len": len(data), "sha256": sha(data)}, "block_size": bs, "blocks": recs,
                     "container_ids0_8": {"len": len(c9), "sha256": sha(c9)},
                     "container_full": {"len": len(c10), "sha256": sha(c10)}}
        print(name, [(r["w9"], r["w10"]) for r in recs], len(c9), len(c10), flush=True)
    with open(os.path.join(HERE, "mixed_corpus.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
