"""Host-buffer API phases (debug): kolm.compress_blocks_fixed on the bench stream with
KOLM_HOST_PROF=1 set by the caller.   python tools/host_probe.py [MiB]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd")]
import kolm  # noqa: E402
from kolm import datagen  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
data = datagen.enwik_like(mib << 20)
for it in range(4):
    t = time.perf_counter()
    blob = kolm.compress_blocks_fixed(data, 1 << 20, hot_path=True)
    dt = time.perf_counter() - t
    print(f"call {it}: {1e3 * dt:.2f} ms  {len(data) / dt / 1e6:.0f} MB/s  out {len(blob)}", file=sys.stderr, flush=True)
