"""Per-kernel device times of one batch of a named input (debug): which kernels a small,
latency-bound input (BASELINE config 5: the mixed corpus) spends its time in.

  on the GPU box:  python tools/lz_probe.py [mixed|gradient] [mask]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd")]
from kolm import _lib, datagen  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "mixed"
    mask = int(sys.argv[2], 0) if len(sys.argv) > 2 and sys.argv[2] != "-" else _lib.KOLM_HOTPATH_MASK
    part = int(sys.argv[3]) if len(sys.argv) > 3 else -1  # one 1 MiB block of the input only
    data = {"mixed": datagen.mixed_corpus, "gradient": lambda: datagen.gradient_bmp()[: 1 << 20],
            "wav": datagen.sine_wav, "checker": datagen.checker_bmp,
            "text": lambda: datagen.enwik_like(256 << 20), "text32": lambda: datagen.enwik_like(32 << 20),
            # BASELINE config 4's per-GPU shard at N = 8: blocks i = 0 (mod 8) of the 256 MiB stream
            "c4shard": lambda: b"".join(memoryview(datagen.enwik_like(256 << 20))[i << 20:(i + 1) << 20]
                                        for i in range(0, 256, 8))}[kind]()
    if part >= 0:
        data = data[part << 20:(part + 1) << 20]
    _lib.ensure_init(0)
    L = _lib.load()
    ctx = ctypes.c_void_p()
    _lib.check(L.kolm_ctx_create(0, ctypes.byref(ctx)))
    n, bs = len(data), 1 << 20
    nb = (n + bs - 1) // bs
    d = _lib.input_buffer(ctx, data)
    cap = 9 * n + 4096
    ar = _lib.DeviceBuffer(ctx, cap)
    sz = np.zeros((nb, _lib.KOLM_NCAND), np.uint32)
    m = np.zeros(nb, np.uint32)
    o = np.zeros(nb + 1, np.uint64)
    iters = int(os.environ.get("PROBE_ITERS", "3"))
    for it in range(iters):
        st = _lib.Stats()
        if it == iters - 1:
            _lib.check(L.kolm_ctx_set_timing(ctx, 1))
        _lib.check(L.kolm_encode_blocks_device(ctx, d.ptr, n, bs, mask, None, ar.ptr, cap,
                                               sz.ctypes.data, m.ctypes.data, o.ctypes.data, ctypes.byref(st)))
    _lib.check(L.kolm_ctx_set_timing(ctx, 0))
    sd = st.as_dict()
    print(kind, part, len(data), "stats", {k: v for k, v in sd.items() if k != "kernels"}, "methods", m.tolist())
    kt = _lib.kernel_times(ctx)
    for k, v in sorted(kt.items(), key=lambda kv: -kv[1]["ms"])[:40]:
        print(f"  {k:32s} {v['ms']:8.3f} {v['launches']}")


if __name__ == "__main__":
    main()
