"""GPU probe of the device Re-Pair (candidate 9): correctness vs the oracle on 1 MiB
blocks of each data kind and the device time of Re-Pair alone and beside the full
candidate set (run on the GPU box: python tools/rp_probe.py [nblocks])."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd"), os.path.join(REPO, "oracle")]
import numpy as np
import oracle as O
from kolm import _lib, datagen as D

_lib.ensure_init(0)
MB = 1 << 20
kinds = {"enwik": lambda: D.enwik_like(MB, seed=5), "gradient": lambda: D.gradient_bmp()[:MB],
         "random": lambda: D.splitmix64_bytes(MB), "zeros": lambda: bytes(MB), "pattern": lambda: D.pattern_blocks()}
for k, f in kinds.items():
    data = f()
    t = time.time()
    _, _, pays, st = _lib.encode_blocks(data, MB, cand_mask=1 << 9, force=[9])
    el = time.time() - t
    ok = pays[0] == O.repair_fast(data)
    print(f"{k}: {'ok' if ok else 'MISMATCH'} size={len(pays[0])} rules={st['rp_rules']} batches={st['rp_batches']} "
          f"ms_repair={st['ms_repair']:.1f} wall={el:.2f}s", flush=True)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
data = D.enwik_like(nb * MB, seed=20251212)
for mask, label in [(1 << 9, "repair only"), (_lib.KOLM_HOTPATH_MASK, "ids 0..8"), (_lib.KOLM_DEFAULT_MASK, "ids 0..9")]:
    for rep in range(2):
        t = time.time()
        sizes, method, pays, st = _lib.encode_blocks(data, MB, cand_mask=mask)
        el = time.time() - t
    print(f"{nb} x 1 MiB enwik, {label}: ms_total={st['ms_total']:.1f} ms_repair={st['ms_repair']:.1f} "
          f"wall={el:.2f}s methods={np.bincount(method, minlength=10).tolist()} batches/blk={st['rp_batches']/nb:.0f}",
          flush=True)
