"""Decode side on the GPU (kolm_decode_blocks, the decoder registry PY:2194-2207): every
PY golden container (fixed and CDC mode) decompresses to its input; device and host
decoders agree block for block on seeded payloads of every device-decoded method;
malformed payloads are rejected with the block named.  The host decoders (kolm/decode.py)
are themselves pinned to PY by tests/test_host.py."""
import os

import numpy as np
import pytest

from kolm import datagen as D
from kolm import decode as H

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_golden_containers_fixed(kolm_gpu, golden_containers, manifest):
    for cname in manifest["containers"]:
        inp = golden_containers[f"{cname}/input"].tobytes()
        for kind in ("full", "ids0_8"):
            blob = golden_containers[f"{cname}/{kind}"].tobytes()
            assert kolm_gpu.decompress(blob) == inp, (cname, kind)


def test_golden_containers_cdc(kolm_gpu):
    import json
    z = np.load(os.path.join(GOLDEN, "cdc.npz"))
    with open(os.path.join(GOLDEN, "cdc.json")) as f:
        man = json.load(f)
    for name in man["containers"]:
        inp = z[f"c_{name}/input"].tobytes()
        for kind in ("full", "ids0_8"):
            assert kolm_gpu.decompress(z[f"c_{name}/{kind}"].tobytes()) == inp, (name, kind)


def _blocks():
    yield D.enwik_like(200_000, seed=3)
    yield D.splitmix64_bytes(70_001)
    yield bytes(65_536)
    yield D.gradient_bmp()[:100_000]
    yield D.sine_wav()[:50_000]
    yield b"a"
    yield b"ab" * 3000 + b"c"
    yield bytes(i & 0xFF for i in range(4099))


@pytest.mark.parametrize("mid", list(range(10)))
def test_device_vs_host_per_method(kolm_gpu, mid):
    """Payloads of method `mid` (forced through the batched encoder) for assorted blocks,
    decoded in ONE device batch: equal to the inputs and to the host decoders."""
    from kolm import _lib
    blocks = list(_blocks())
    pays = []
    for blk in blocks:
        _, _, p, _ = _lib.encode_blocks(blk, len(blk), cand_mask=1 << mid, force=[mid])
        pays.append(p[0])
        assert H.decode_block(mid, p[0], len(blk)) == blk
    got = _lib.decode_blocks(pays, [mid] * len(blocks), [len(b) for b in blocks])
    assert got == b"".join(blocks)


def test_mixed_batch_large(kolm_gpu):
    """64 MiB of 1 MiB blocks, hot-path candidates, one device batch; round trip exact."""
    data = D.enwik_like(24 << 20) + D.splitmix64_bytes(8 << 20) + bytes(4 << 20)
    blob = kolm_gpu.compress_blocks_fixed(data, 1 << 20, hot_path=True)
    assert kolm_gpu.decompress(blob) == data
    assert kolm_gpu.decompress(blob, device=False) == data


def test_mixed_methods_one_batch(kolm_gpu):
    """Every device-decoded id in ONE batch, blocks of different lengths interleaved (the
    BBWT family shares one list; its MTF chunk grid is sized by the longest block)."""
    from kolm import _lib
    blocks = list(_blocks())
    pays, mids = [], []
    for j, blk in enumerate(blocks * 2):
        mid = j % 10
        _, _, p, _ = _lib.encode_blocks(blk, len(blk), cand_mask=1 << mid, force=[mid])
        pays.append(p[0])
        mids.append(mid)
    got = _lib.decode_blocks(pays, mids, [len(b) for b in blocks * 2])
    assert got == b"".join(blocks * 2)


@pytest.mark.parametrize("mid", [2, 3, 5])
def test_bbwt_family_large(kolm_gpu, mid):
    """4 MiB blocks (4096 MTF chunks, multi-tile inverse BBWT, long Lyndon cycles)."""
    from kolm import _lib
    blocks = [D.enwik_like(4 << 20, seed=11), bytes(1 << 20) + b"x", b"ab" * (1 << 20)]
    pays = []
    for blk in blocks:
        _, _, p, _ = _lib.encode_blocks(blk, len(blk), cand_mask=1 << mid, force=[mid])
        pays.append(p[0])
    assert _lib.decode_blocks(pays, [mid] * len(blocks), [len(b) for b in blocks]) == b"".join(blocks)


def test_lz77_long_overlaps(kolm_gpu):
    """Copy chains through overlapping matches (dist 1..3 runs of 1 MiB) and the maximal
    window distance: pointer jumping must resolve every chain."""
    from kolm import _lib
    blocks = [bytes(1 << 20), b"xyz" * 349_525, (b"q" + bytes(4095)) * 64, D.enwik_like(1 << 20, seed=9)]
    pays = []
    for blk in blocks:
        _, _, p, _ = _lib.encode_blocks(blk, len(blk), cand_mask=1 << 7, force=[7])
        pays.append(p[0])
    assert _lib.decode_blocks(pays, [7] * len(blocks), [len(b) for b in blocks]) == b"".join(blocks)


def test_malformed_payloads(kolm_gpu):
    from kolm import _lib
    cases = [
        (0, b"abc", 4),                 # raw length mismatch
        (1, b"\x05\x80", 2),            # truncated 2-byte ULEB value
        (1, b"\x01\x02\x03", 2),        # too many values
        (7, b"\x01\x03\x01", 3),        # first token a copy (distance > output)
        (7, b"\x02\x41", 1),            # unknown flag
        (7, b"\x00\x41", 2),            # short output
        (8, b"\x01", 2),                # too few values
    ]
    for mid, pay, n in cases:
        with pytest.raises(_lib.KolmError):
            _lib.decode_blocks([pay], [mid], [n])
    for mid in (2, 3, 6):
        with pytest.raises(_lib.KolmError):   # Rice: unary run past 63 bits
            _lib.decode_blocks([b"\xff" * 16], [mid], [4])
        with pytest.raises(_lib.KolmError):   # Rice: too few values
            _lib.decode_blocks([b"\x00"], [mid], [100])
    def u(v):
        out = bytearray()
        while True:
            out.append((v & 0x7F) | (0x80 if v >= 128 else 0))
            v >>= 7
            if not v:
                return bytes(out)
    rp = [
        (b"XP" + u(256) + u(0) + u(1) + u(65), 1),                     # magic
        (b"RP" + u(255) + u(0) + u(1) + u(65), 1),                     # terminal alphabet
        (b"RP" + u(256) + u(5), 4),                                    # truncated rules
        (b"RP" + u(256) + u(1) + u(256) + u(65) + u(1) + u(256), 2),   # self-referencing rule
        (b"RP" + u(256) + u(1) + u(65) + u(66) + u(1) + u(257), 2),    # undefined symbol
        (b"RP" + u(256) + u(0) + u(2) + u(65) + u(66), 3),             # length mismatch
        (b"RP" + u(256) + u(0) + u(2) + u(65) + b"\x80", 2),           # truncated value
    ]
    for pay, n in rp:
        with pytest.raises(_lib.KolmError):
            _lib.decode_blocks([pay], [9], [n])
    ok = b"RP" + u(256) + u(1) + u(65) + u(66) + u(3) + u(256) + u(67) + u(256)
    assert _lib.decode_blocks([ok], [9], [5]) == b"ABCAB" == H.decode_block(9, ok, 5)
    # hand-made grammars PY (PY:1945-1970) accepts although the encoder never writes them:
    # forward references, and unused rules that do not resolve (undefined symbol, cycle)
    def rp_pay(rules, seq):
        body = b"".join(u(x) + u(y) for x, y in rules)
        return b"RP" + u(256) + u(len(rules)) + body + u(len(seq)) + b"".join(u(s) for s in seq)
    accepted = [
        (rp_pay([(257, 67), (65, 66)], [256, 257]), b"ABCAB"),                    # forward reference
        (rp_pay([(258, 257), (65, 66), (259, 67), (68, 69)], [256, 257]), b"DECABAB"),  # forward chain
        (rp_pay([(65, 66), (999, 65)], [256]), b"AB"),                           # unused, undefined symbol
        (rp_pay([(65, 66), (258, 65), (257, 66)], [256, 256]), b"ABAB"),          # unused cycle
    ]
    for pay, want in accepted:
        assert H.decode_block(9, pay, len(want)) == want
        assert _lib.decode_blocks([pay], [9], [len(want)]) == want
    # the same chains beside 40000 backward rules (the forward pass starts mid-grammar, past
    # the rule lengths kept in LDS)
    big = [(65, 66)] + [(256 + r - 1, 67) for r in range(1, 40000)]
    tail = len(big)
    big += [(256 + tail + 1, 68), (69, 256 + tail + 2), (70, 71)]
    pay = rp_pay(big, [256 + tail, 256 + 5])
    want = b"EFGD" + b"AB" + b"C" * 5
    assert _lib.decode_blocks([pay], [9], [len(want)]) == want == H.decode_block(9, pay, len(want))
    with pytest.raises(_lib.KolmError):  # a USED cycle (PY would not terminate on it)
        _lib.decode_blocks([rp_pay([(257, 65), (256, 66)], [256])], [9], [4])
    with pytest.raises(_lib.KolmError):  # method id outside the decoder registry
        _lib.decode_blocks([b"x"], [10], [1])
    # a bad block in a batch fails the batch and names the block
    good = b"hello"
    with pytest.raises(_lib.KolmError, match="block 1"):
        _lib.decode_blocks([good, b"\x02"], [0, 7], [5, 1])


def test_decode_device_entry(kolm_gpu):
    """kolm_decode_blocks_device: payloads resident in device memory (an encode arena),
    output to device memory, kernel time reported; round trip exact."""
    import ctypes
    from kolm import _lib
    L = _lib.load()
    blocks = list(_blocks())
    pays, mids = [], []
    for j, blk in enumerate(blocks):
        mid = (2, 7, 3, 0, 6, 1, 8, 9)[j % 8]
        _, _, p, _ = _lib.encode_blocks(blk, len(blk), cand_mask=1 << mid, force=[mid])
        pays.append(p[0])
        mids.append(mid)
    arena = b"".join(pays)
    off = np.zeros(len(pays) + 1, np.uint64)
    off[1:] = np.cumsum([len(p) for p in pays])
    meth = np.asarray(mids, np.uint32)
    lens = np.asarray([len(b) for b in blocks], np.uint32)
    total = int(lens.sum())
    ctx = ctypes.c_void_p()
    _lib.check(L.kolm_ctx_create(0, ctypes.byref(ctx)))
    try:
        dp, do = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(L.kolm_dev_alloc(ctx, len(arena) + 64, ctypes.byref(dp)))
        _lib.check(L.kolm_dev_alloc(ctx, total + 64, ctypes.byref(do)))
        _lib.check(L.kolm_memcpy_h2d(ctx, dp, arena, len(arena)))
        ms = ctypes.c_double(-1.0)
        _lib.check(L.kolm_decode_blocks_device(ctx, dp, off.ctypes.data, meth.ctypes.data, lens.ctypes.data,
                                               len(blocks), do, total, ctypes.byref(ms)))
        out = ctypes.create_string_buffer(total)
        _lib.check(L.kolm_memcpy_d2h(ctx, out, do, total))
        assert out.raw == b"".join(blocks)
        assert ms.value > 0.0
        with pytest.raises(_lib.KolmError):  # capacity
            _lib.check(L.kolm_decode_blocks_device(ctx, dp, off.ctypes.data, meth.ctypes.data, lens.ctypes.data,
                                                   len(blocks), do, total - 1, None))
        L.kolm_dev_free(ctx, dp)
        L.kolm_dev_free(ctx, do)
    finally:
        L.kolm_ctx_destroy(ctx)


def _payload_of_L(L: bytes) -> bytes:
    """Candidate-2 payload whose MTF+Rice layer decodes to the BBWT string L (any L has
    an inverse BBWT: the cycles of its stable sort permutation)."""
    import oracle as O
    return O.rice_encode(O.mtf_encode(L), 2)


def _L_with_permutation(P):
    """A string L whose stable counting sort is the permutation P (F-slot x -> index
    P[x]): split x at the descents of P and give each run the next byte value."""
    n = len(P)
    L = bytearray(n)
    g = 0
    for x in range(n):
        if x and P[x] < P[x - 1]:
            g += 1
        L[P[x]] = g
    assert g < 256
    return bytes(L)


def test_inverse_bbwt_arbitrary_strings(kolm_gpu):
    """Inverse BBWT of arbitrary BBWT strings (not produced by the encoder): random bytes,
    sorted runs (n one-slot cycles), two symbols, and a permutation whose one long cycle
    avoids every splitter slot (multiples of 64) — decoded by the splitter-free path —
    against the host decoder (PY:425-454)."""
    from kolm import _lib
    rng = np.random.default_rng(5)
    cases = [rng.integers(0, 256, 100_000, dtype=np.uint8).tobytes(),
             bytes(sorted(rng.integers(0, 256, 50_000, dtype=np.uint8).tobytes())),
             rng.integers(0, 2, 70_000, dtype=np.uint8).tobytes(),
             bytes(range(256)) * 40, bytes(1)]
    n = 4096
    S = [x for x in range(n) if x % 64]
    pos = {s: j for j, s in enumerate(S)}
    P = [x if x % 64 == 0 else S[(pos[x] + 7) % len(S)] for x in range(n)]
    cases.append(_L_with_permutation(P))
    pays = [_payload_of_L(L) for L in cases]
    lens = [len(L) for L in cases]
    got = _lib.decode_blocks(pays, [2] * len(cases), lens)
    want = b"".join(H.decode_block(2, p, m) for p, m in zip(pays, lens))
    assert got == want


def test_repair_containers_large(kolm_gpu):
    """Full candidate list (Re-Pair wins on text): 8 x 1 MiB text blocks + zeros + a
    period-3 pattern decoded on the device (deep and wide grammars) == input == host."""
    data = D.enwik_like(8 << 20, seed=21) + bytes(1 << 20) + b"abc" * 349_525
    blob = kolm_gpu.compress_blocks_fixed(data, 1 << 20)
    assert kolm_gpu.decompress(blob) == data


def test_toc_cases_on_device(kolm_gpu):
    """The PY-written corner-case containers of tests/golden/toc_cases.json through the device
    decoders: long / shifted / oversubscribed prefix codes decode as PY decodes them, and the
    bit-plane blocks with n % 8 != 0 (where PY raises IndexError: the pinned divergence of
    kolm/decode.py) decode to their input."""
    import json
    with open(os.path.join(GOLDEN, "toc_cases.json")) as f:
        cases = json.load(f)
    for name, c in cases.items():
        blob = bytes.fromhex(c["container"])
        if name.startswith("bitplane"):
            assert kolm_gpu.decompress(blob) == bytes.fromhex(c["input"]), name
        elif "ok" in c["py"]:
            assert kolm_gpu.decompress(blob) == bytes.fromhex(c["py"]["ok"]), name
        else:
            with pytest.raises(ValueError, match=c["py"]["message"]):
                kolm_gpu.decompress(blob)
