"""Experiment: one 256 MiB device batch vs k sequential sub-batches (L2/MALL locality of
the per-round gathers).  python tools/batch_split.py [mib] [iters]"""
import ctypes, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd")]
import torch
import numpy as np
from kolm import _lib, datagen as D

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = mib << 20
bs = 1 << 20
data = D.enwik_like(n)
L = _lib.load()
torch.cuda.set_device(0)
ctx = ctypes.c_void_p()
_lib.check(L.kolm_ctx_create(0, ctypes.byref(ctx)))
d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
d_in[:n].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
arena = torch.empty(n + (8 << 20), dtype=torch.uint8, device="cuda")
for k in (1, 2, 4, 8, 1):
    sub = n // k
    nb = sub // bs
    sizes = np.zeros((nb, _lib.KOLM_NCAND), np.uint32)
    method = np.zeros(nb, np.uint32)
    off = np.zeros(nb + 1, np.uint64)
    ts = []
    for it in range(iters + 1):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for j in range(k):
            _lib.check(L.kolm_encode_blocks_device(ctx, d_in.data_ptr() + j * sub, sub, bs, _lib.KOLM_HOTPATH_MASK, None,
                                                   arena.data_ptr() + j * (sub + (1 << 20)), sub + (1 << 20),
                                                   sizes.ctypes.data, method.ctypes.data, off.ctypes.data, None))
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    el = min(ts[1:])
    print(f"k={k}: {el * 1e3:.1f} ms  {n / el / 1e6:.0f} MB/s", flush=True)
