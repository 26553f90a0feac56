"""Quick GPU diagnostics: runs each kernel on small golden inputs and reports mismatches
(no asserts) so one gpurun call shows every broken stage."""
import os, sys, time, traceback
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd"), os.path.join(REPO, "oracle")]
import numpy as np
import kolm, oracle as O
from kolm import _lib, datagen as D

_lib.ensure_init(0)
K = np.load(os.path.join(REPO, "tests/golden/kernels.npz"))
names = sorted({k.split("/")[0] for k in K.files})
bad = {}
def chk(kind, name, got, want):
    if got != want:
        bad.setdefault(kind, []).append(name)
t0 = time.time()
for name in names:
    inp = K[f"{name}/input"].tobytes()
    for kind, fn, want in [
        ("bbwt", lambda: kolm.bbwt_forward(inp), K[f"{name}/bbwt"].tobytes()),
        ("mtf", lambda: bytes(kolm.mtf_encode(K[f"{name}/bbwt"].tobytes())), K[f"{name}/mtf"].tobytes()),
        ("rice_k2", lambda: kolm.rice_encode(K[f"{name}/mtf"].tobytes(), 2), K[f"{name}/rice0"].tobytes()),
        ("lz77", lambda: kolm.encode_lz77(inp)[0], K[f"{name}/lz77"].tobytes()),
    ]:
        try:
            chk(kind, name, fn(), want)
        except Exception as e:
            bad.setdefault(kind + "_exc", []).append(f"{name}: {e!r}")
    if inp:
        try:
            sizes, method, pays, st = _lib.encode_blocks(inp, len(inp))
            want = [len(O.candidate(m, inp)) for m in range(9)]
            if list(map(int, sizes[0])) != want:
                bad.setdefault("sizes", []).append(f"{name}: got {list(map(int, sizes[0]))} want {want}")
        except Exception as e:
            bad.setdefault("batch_exc", []).append(f"{name}: {e!r}")
print(f"small goldens done in {time.time()-t0:.1f}s")
for k, v in bad.items():
    print("FAIL", k, len(v), v[:12])
# a 1 MiB block and a multi-block batch
for label, data, bs in [("grad1m", D.gradient_bmp()[:1 << 20], 1 << 20), ("enwik4x256k", D.enwik_like(1 << 20), 1 << 18)]:
    try:
        t = time.time()
        sizes, method, pays, st = _lib.encode_blocks(data, bs)
        el = time.time() - t
        print(label, "sizes", sizes.tolist()[:2], "method", method.tolist(), f"{el:.2f}s", {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()})
        blk = data[:bs]
        want = [len(O.candidate(m, blk)) for m in (0, 1, 2, 3, 4, 5, 6, 8)]
        print(label, "oracle sizes (no lz)", want)
    except Exception:
        traceback.print_exc()
print("sanity done")
