"""Profiling driver: encode a resident batch of 1 MiB enwik-style blocks a few times.

    python tools/profile_run.py [--mib 256] [--iters 2] [--data enwik|gradient|mixed]
"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd")]
import numpy as np  # noqa: E402

from kolm import _lib, datagen as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--bs", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--data", default="enwik")
    a = ap.parse_args()
    n = a.mib << 20
    t = time.time()
    if a.data == "enwik":
        data = D.enwik_like(n)
    elif a.data == "gradient":
        g = D.gradient_bmp()
        data = (g * (n // len(g) + 1))[:n]
    else:
        m = D.mixed_corpus()
        data = (m * (n // len(m) + 1))[:n]
    print(f"generated {n >> 20} MiB in {time.time() - t:.1f}s", flush=True)
    L = _lib.load()
    _lib.ensure_init(0)
    ctx = ctypes.c_void_p()
    _lib.check(L.kolm_ctx_create(0, ctypes.byref(ctx)))
    dptr = ctypes.c_void_p()
    _lib.check(L.kolm_dev_alloc(ctx, n + 64, ctypes.byref(dptr)))
    _lib.check(L.kolm_memcpy_h2d(ctx, dptr, data, n))
    cap = n + (1 << 20)
    arena = ctypes.c_void_p()
    _lib.check(L.kolm_dev_alloc(ctx, cap, ctypes.byref(arena)))
    nb = (n + a.bs - 1) // a.bs
    sizes = np.zeros((nb, _lib.KOLM_NCAND), np.uint32)
    method = np.zeros(nb, np.uint32)
    off = np.zeros(nb + 1, np.uint64)
    for it in range(a.iters):
        st = _lib.Stats()
        t = time.time()
        _lib.check(L.kolm_encode_blocks_device(ctx, dptr, n, a.bs, 0x1FF, None, arena, cap,
                                               sizes.ctypes.data, method.ctypes.data, off.ctypes.data,
                                               ctypes.byref(st)))
        el = time.time() - t
        d = st.as_dict()
        print(f"iter {it}: {el * 1e3:.1f} ms wall, {n / el / 1e6:.1f} MB/s, out {int(off[-1])} B "
              f"(ratio {int(off[-1]) / n:.3f}), methods {np.bincount(method, minlength=9).tolist()}", flush=True)
        print("  ", {k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items()}, flush=True)


if __name__ == "__main__":
    main()
