"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors
(tests/golden, produced by importing PY), PY's own 1 MiB known answers, and the oracle
(faithful CPU restatement) on seeded inputs.  Bit-exact everywhere (integer/byte work).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
from kolm import datagen as D

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "manifest.json")) as _f:
    _MAN = json.load(_f)
KNAMES = sorted(_MAN["kernels"])
CNAMES = sorted(_MAN["containers"])
FLAG_OF_MID = {2: 0, 3: 1, 4: 4, 5: 8, 6: 16}


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def gk(golden_kernels, name, kind) -> bytes:
    return golden_kernels[f"{name}/{kind}"].tobytes()


@pytest.mark.parametrize("name", KNAMES)
def test_bbwt_golden(kolm_gpu, golden_kernels, name):
    inp = gk(golden_kernels, name, "input")
    assert kolm_gpu.bbwt_forward(inp) == gk(golden_kernels, name, "bbwt")


@pytest.mark.parametrize("name", KNAMES)
def test_mtf_golden(kolm_gpu, golden_kernels, name):
    bw = gk(golden_kernels, name, "bbwt")
    assert bytes(kolm_gpu.mtf_encode(bw)) == gk(golden_kernels, name, "mtf")


@pytest.mark.parametrize("name", KNAMES)
def test_lz77_golden(kolm_gpu, golden_kernels, name):
    inp = gk(golden_kernels, name, "input")
    assert kolm_gpu.encode_lz77(inp)[0] == gk(golden_kernels, name, "lz77")


@pytest.mark.parametrize("name", KNAMES)
def test_batched_candidates_golden(kolm_gpu, golden_kernels, name):
    """All 10 candidate payloads of one block (ids 0..9, Re-Pair included) through the
    batched entry (forced method), against PY's own outputs."""
    inp = gk(golden_kernels, name, "input")
    if not inp:
        return
    from kolm import _lib
    want = {0: inp, 1: gk(golden_kernels, name, "xor"), 7: gk(golden_kernels, name, "lz77"),
            8: gk(golden_kernels, name, "lfsr"), 9: gk(golden_kernels, name, "repair")}
    for mid, f in FLAG_OF_MID.items():
        want[mid] = gk(golden_kernels, name, f"rice{f}")
    for mid in range(10):
        sizes, method, payloads, _ = _lib.encode_blocks(inp, len(inp), force=[mid])
        assert int(method[0]) == mid
        assert payloads[0] == want[mid], f"candidate {mid}"
        assert int(sizes[0][mid]) == len(want[mid]), f"size of candidate {mid}"
    # un-forced: MDL winner = argmin, ties -> lowest id (PY:2359)
    sizes, method, payloads, _ = _lib.encode_blocks(inp, len(inp))
    lens = [len(want[m]) for m in range(10)]
    assert list(map(int, sizes[0][:10])) == lens
    assert int(method[0]) == int(np.argmin(lens))
    # hot path (ids 0..8): candidate 9 disabled, argmin over the rest
    sizes, method, payloads, _ = _lib.encode_blocks(inp, len(inp), cand_mask=_lib.KOLM_HOTPATH_MASK)
    assert int(sizes[0][9]) == 0xFFFFFFFF
    assert int(method[0]) == int(np.argmin(lens[:9]))


@pytest.mark.parametrize("name", KNAMES)
def test_repair_golden(kolm_gpu, golden_kernels, name):
    """repair_compress (PY:1841-1911) on the GPU vs PY's payload."""
    inp = gk(golden_kernels, name, "input")
    assert kolm_gpu.repair_compress(inp)[0] == gk(golden_kernels, name, "repair")


@pytest.mark.parametrize("name", ["text_hobbit", "rand4k", "enwik16k", "utf8_mixed", "zero16k"])
@pytest.mark.parametrize("k", [0, 1, 2, 3, 5, 7])
def test_rice_param(kolm_gpu, golden_kernels, name, k):
    mtf = gk(golden_kernels, name, "mtf")
    assert kolm_gpu.rice_encode(mtf, k) == O.rice_encode(mtf, k)


@pytest.mark.parametrize("cname", CNAMES)
def test_container_golden(kolm_gpu, golden_containers, manifest, cname):
    inp = golden_containers[f"{cname}/input"].tobytes()
    bs = manifest["containers"][cname]["block_size"]
    got = kolm_gpu.compress_blocks_fixed(inp, bs)
    assert got == golden_containers[f"{cname}/full"].tobytes()  # PY's container, byte for byte
    assert kolm_gpu.decompress(got) == inp
    hot = kolm_gpu.compress_blocks_fixed(inp, bs, hot_path=True)
    assert hot == golden_containers[f"{cname}/ids0_8"].tobytes()


LARGE = {
    "gradient_1m": lambda: D.gradient_bmp()[: 1 << 20],
    "pattern_1m": lambda: D.pattern_blocks(),
    "checker_full": lambda: D.checker_bmp(),
    "sine_full": lambda: D.sine_wav(),
    "enwik_256k": lambda: D.enwik_like(1 << 18),
}


@pytest.mark.parametrize("case", sorted(LARGE))
def test_large_known_answers(kolm_gpu, large_known, case):
    """1 MiB-class blocks against sha256 of PY's own outputs (tests/golden/large.json)."""
    from kolm import _lib
    data = LARGE[case]()
    ref = large_known[case]
    assert sha(data) == ref["input"]["sha256"]
    bw = kolm_gpu.bbwt_forward(data)
    assert sha(bw) == ref["bbwt"]["sha256"], "bbwt"
    mt = bytes(kolm_gpu.mtf_encode(bw))
    assert sha(mt) == ref["mtf"]["sha256"], "mtf"
    for mid, f in FLAG_OF_MID.items():
        _, _, payloads, _ = _lib.encode_blocks(data, len(data), force=[mid])
        assert len(payloads[0]) == ref[f"rice{f}"]["len"], f"rice{f} len"
        assert sha(payloads[0]) == ref[f"rice{f}"]["sha256"], f"rice{f}"
    if "lz77" in ref:
        z = kolm_gpu.encode_lz77(data)[0]
        assert len(z) == ref["lz77"]["len"] and sha(z) == ref["lz77"]["sha256"], "lz77"


def test_bench_block0_lz77_vs_py(kolm_gpu, large_known):
    """Block 0 of the bench stream (enwik_like, 1 MiB): the LZ77 stream against sha256 of PY's own
    encode_lz77 on it (make_golden_scale.py), so the bench's LZ77 at 1 MiB rests on PY itself."""
    ref = large_known.get("bench_block0")
    if ref is None or "lz77" not in ref:
        pytest.skip("no PY LZ77 known answer for bench block 0")
    data = D.enwik_like(1 << 20)
    assert sha(data) == ref["input"]["sha256"]
    z = kolm_gpu.encode_lz77(data)[0]
    assert len(z) == ref["lz77"]["len"] and sha(z) == ref["lz77"]["sha256"]


def _oracle_all(block: bytes):
    return [O.candidate(m, block) for m in range(10)]


@pytest.mark.parametrize("seed,bs,n", [(1, 65536, 4 * 65536 + 12345), (2, 4096, 65536 + 17), (3, 1000, 20011),
                                       (4, 7, 301), (5, 1, 40), (6, 3, 64), (7, 8, 800)])
def test_multiblock_vs_oracle(kolm_gpu, seed, bs, n):
    """Several blocks in one batch, all candidate sizes + the emitted winners vs oracle."""
    from kolm import _lib
    rng = np.random.default_rng(seed)
    parts = [D.enwik_like(n // 2, seed=seed), rng.integers(0, 4, n // 4).astype(np.uint8).tobytes(),
             bytes(n // 8), D.splitmix64_bytes(n, seed=seed)]
    data = b"".join(parts)[:n]
    sizes, method, payloads, _ = _lib.encode_blocks(data, bs)
    nb = (n + bs - 1) // bs
    assert len(payloads) == nb
    for i in range(nb):
        blk = data[i * bs:(i + 1) * bs]
        cand = _oracle_all(blk)
        lens = [len(c) for c in cand]
        assert list(map(int, sizes[i][:10])) == lens, f"block {i}"
        m = int(np.argmin(lens))
        assert int(method[i]) == m, f"block {i}"
        assert payloads[i] == cand[m], f"block {i} payload"


def test_container_vs_oracle_multiblock(kolm_gpu):
    data = D.mixed_corpus()[:300_000]
    bs = 65536
    got = kolm_gpu.compress_blocks_fixed(data, bs)
    assert got == O.compress_blocks_fixed(data, bs, range(10))
    assert kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True) == O.compress_blocks_fixed(data, bs, range(9))


@pytest.mark.parametrize("seed", [11, 12])
def test_full_size_enwik_properties(kolm_gpu, seed):
    """Full-size blocks (1 MiB, BASELINE configs 3/4): exact vs oracle on one block, and
    size-independent properties on a 16-block batch (BBWT is a permutation of each
    block, MTF round trip on a sample, container decodes)."""
    from kolm import _lib
    data = D.enwik_like(16 << 20, seed=seed)
    bs = 1 << 20
    sizes, method, payloads, st = _lib.encode_blocks(data, bs)
    assert len(payloads) == 16
    blk = data[:bs]
    cand = _oracle_all(blk)
    assert list(map(int, sizes[0][:10])) == [len(c) for c in cand]
    assert payloads[0] == cand[int(method[0])]
    for i in range(16):
        assert int(sizes[i][int(method[i])]) == len(payloads[i])
        assert int(method[i]) == int(np.argmin(sizes[i]))
    # BBWT of one block is a permutation and inverts back
    from kolm import decode
    b3 = data[3 * bs:4 * bs]
    bw = kolm_gpu.bbwt_forward(b3)
    assert np.array_equal(np.bincount(np.frombuffer(bw, np.uint8), minlength=256),
                          np.bincount(np.frombuffer(b3, np.uint8), minlength=256))
    assert decode.bbwt_inverse(bw) == b3


@pytest.mark.parametrize("data,bs", [(b"", 16), (b"\x00", 1), (b"ab", 1), (b"abc" * 5, 4), (bytes(range(256)) * 3, 100)])
def test_edge_cases(kolm_gpu, data, bs):
    got = kolm_gpu.compress_blocks_fixed(data, bs)
    assert got == O.compress_blocks_fixed(data, bs, range(10))
    assert kolm_gpu.decompress(got) == data


def _fib_word(n: int) -> bytes:
    a, b = b"a", b"ab"
    while len(b) < n:
        a, b = b, b + a
    return b[:n]


def _thue_morse(n: int) -> bytes:
    return bytes(97 + (bin(i).count("1") & 1) for i in range(n))


def _adversarial(kind: str, n: int) -> bytes:
    rng = np.random.default_rng(len(kind))
    if kind == "decreasing":      # every byte its own Lyndon factor inside a run
        return (bytes(range(255, -1, -1)) * (n // 256 + 1))[:n]
    if kind == "fibonacci":       # LCPs ~ n: many doubling rounds, few factors
        return _fib_word(n)
    if kind == "thue_morse":
        return _thue_morse(n)
    if kind == "period7":         # equal factors repeated, every rotation tied
        return (rng.integers(0, 256, 7).astype(np.uint8).tobytes() * (n // 7 + 1))[:n]
    if kind == "runs":            # long runs with sparse breaks: huge factors spanning spans
        out = bytearray(b"a" * n)
        for p in rng.integers(0, n, 40):
            out[int(p)] = 98 + int(p) % 3
        return bytes(out)
    if kind == "zeros":
        return bytes(n)
    if kind == "two_symbols":
        return rng.integers(0, 2, n).astype(np.uint8).tobytes()
    if kind == "short_words":     # Lyndon factors of 1..10 bytes: the 8 round-0 characters wrap
        out = bytearray()         # inside the factor at every offset
        c = 250
        while len(out) < n:
            ln = int(rng.integers(1, 11))
            out.append(c)
            out += rng.integers(c + 1, 256, ln - 1).astype(np.uint8).tobytes()
            c = c - 1 if c > 1 else 250
        return bytes(out[:n])
    raise ValueError(kind)


ADV = ["decreasing", "fibonacci", "thue_morse", "period7", "runs", "zeros", "two_symbols", "short_words"]


@pytest.mark.parametrize("kind", ADV)
def test_adversarial_bbwt_lz77(kolm_gpu, kind):
    """Structures the reference's own tests do not cover but the GPU formulation is
    sensitive to: Lyndon factors spanning many 32 KiB Duval spans (or one factor per
    byte), LCPs of the whole block (doubling to the last round), every rotation tied,
    matches running to the block end.  One block (200 KB; 100 KB for the two slow
    oracle cases), vs the oracle."""
    data = _adversarial(kind, 100_000 if kind in ("fibonacci", "thue_morse") else 200_000)
    assert kolm_gpu.bbwt_forward(data) == O.bbwt_forward(data), "bbwt"
    assert kolm_gpu.encode_lz77(data)[0] == O.encode_lz77(data), "lz77"


@pytest.mark.parametrize("kind", ["decreasing", "period7", "runs", "two_symbols", "short_words"])
def test_adversarial_batched(kolm_gpu, kind):
    """Same structures through the batched entry: 4 blocks of 65536 + a ragged tail."""
    from kolm import _lib
    data = _adversarial(kind, 4 * 65536 + 1234)
    bs = 65536
    sizes, method, payloads, _ = _lib.encode_blocks(data, bs)
    for i in range((len(data) + bs - 1) // bs):
        blk = data[i * bs:(i + 1) * bs]
        cand = _oracle_all(blk)
        assert list(map(int, sizes[i][:10])) == [len(c) for c in cand], f"block {i}"
        assert payloads[i] == cand[int(method[i])], f"block {i}"


def _merge_stack_block(z: int, swap: bool) -> bytes:
    """A 65536-byte block whose two 32 KiB Duval spans factorise into exactly z + 2 span
    factors: span 0 = "\\x01" + text (one Lyndon word: its minimum byte occurs once, at
    the front), span 1 = "\\x01" + text + z zero bytes (one word + z factors "\\x00").  The
    two words merge across the spans when the first is smaller (swap picks the order)."""
    t0 = D.enwik_like(32767, seed=31)
    t1 = D.enwik_like(32767 - z, seed=32)
    if swap:
        t0, t1 = D.enwik_like(32767, seed=32), D.enwik_like(32767 - z, seed=31)
    blk = b"\x01" + t0 + b"\x01" + t1 + bytes(z)
    assert len(blk) == 65536
    return blk


def test_lyndon_merge_stack_boundary(kolm_gpu):
    """k_duval_merge keeps its factor stack in LDS while the span factorisations total at
    most MERGE_LDS (8192) entries and in global memory past that: blocks at 8191, 8192 and
    8193 span factors, with and without the cross-span merge, in ONE batch, vs the oracle."""
    from kolm import _lib
    blocks = [_merge_stack_block(z, sw) for z in (8189, 8190, 8191) for sw in (False, True)]
    data = b"".join(blocks)
    _, method, payloads, _ = _lib.encode_blocks(data, 65536, force=[2] * len(blocks))
    for i, blk in enumerate(blocks):
        assert payloads[i] == O.candidate(2, blk), f"block {i}"
    assert kolm_gpu.bbwt_forward(blocks[3]) == O.bbwt_forward(blocks[3])


@pytest.mark.parametrize("ngpu", [1, 2])
def test_encode_blocks_multi(kolm_gpu, ngpu):
    """Single-process multi-device entry (kolm_encode_blocks_multi): same outputs as the
    single-device batch (ngpu is clamped to the visible device count)."""
    from kolm import _lib
    data = D.mixed_corpus()[:700_000]
    bs = 65536
    a = _lib.encode_blocks(data, bs)
    b = _lib.encode_blocks_multi(data, bs, ngpu)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    assert kolm_gpu.compress_blocks_fixed(data, bs, devices=ngpu) == O.compress_blocks_fixed(data, bs, range(10))


def test_encode_blocks_multi_threads(kolm_gpu):
    """Two host threads calling kolm_encode_blocks_multi at once (each device's
    payloads wait in its context's arena between the encode and the gather; the calls are
    serialised inside the library, so neither sees the other's payloads)."""
    import threading
    from kolm import _lib
    ins = [(D.enwik_like(300_000, seed=11), 32768), (D.mixed_corpus()[:500_000], 65536)]
    want = [_lib.encode_blocks(d, bs) for d, bs in ins]
    got = [None, None]
    errs = []

    def run(i):
        try:
            for _ in range(3):
                got[i] = _lib.encode_blocks_multi(ins[i][0], ins[i][1], 1)
                assert np.array_equal(got[i][1], want[i][1]) and got[i][2] == want[i][2]
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs


RP_LARGE = {
    "enwik_1m": lambda: D.enwik_like(1 << 20, seed=5),
    "gradient_1m": lambda: D.gradient_bmp()[: 1 << 20],
    "random_1m": lambda: D.splitmix64_bytes(1 << 20),
    "pattern_1m": lambda: D.pattern_blocks(),
    "zeros_1m": lambda: bytes(1 << 20),
}


def test_repair_full_size_batch(kolm_gpu):
    """Re-Pair on 1 MiB blocks (text: 18.9k rules in ~950 batches; gradient: 133k rules in
    ~17k batches; random; runs of zeros; the pattern file), all in ONE batch of 5 blocks
    run concurrently, vs the oracle's exact O(n log n) Re-Pair."""
    from kolm import _lib
    names = sorted(RP_LARGE)
    blocks = [RP_LARGE[k]() for k in names]
    data = b"".join(blocks)
    sizes, method, payloads, st = _lib.encode_blocks(data, 1 << 20, cand_mask=1 << 9,
                                                     force=[9] * len(blocks))
    for name, blk, pay in zip(names, blocks, payloads):
        assert pay == O.repair_fast(blk), name


@pytest.mark.parametrize("kind", ADV)
def test_adversarial_repair(kolm_gpu, kind):
    """Re-Pair on the adversarial structures (long (a,a) runs, periodic text, two symbols):
    one 200 KB block vs the oracle."""
    data = _adversarial(kind, 200_000)
    assert kolm_gpu.repair_compress(data)[0] == O.repair_fast(data)


def _lz_edge(kind: str) -> bytes:
    """Inputs aimed at the workgroup-local LZ77 parse (k_lz77.hip): 4 KiB homes, 256-byte
    chunks with 48-byte lead-ins, matches resolved exactly only 256 bytes past a chunk."""
    rng = np.random.default_rng(7 + len(kind))
    if kind == "long_copies":     # copies of 300..5000 bytes with sparse mutations: matches
        out = bytearray(rng.integers(0, 256, 6000).astype(np.uint8).tobytes())  # past the cap
        while len(out) < 150_000:
            L = int(rng.integers(300, 5000))
            d = int(rng.integers(L, min(len(out), 4096) + 1)) if L <= 4096 else len(out) - 1
            seg = bytearray(out[len(out) - d:len(out) - d + L])
            for _ in range(int(rng.integers(0, 3))):
                seg[int(rng.integers(0, L))] ^= 0x5A
            out += seg + rng.integers(0, 256, int(rng.integers(1, 40))).astype(np.uint8).tobytes()
        return bytes(out)
    if kind in ("period4096", "period4097"):  # a match only at exactly the window edge (or none)
        per = int(kind[6:])
        unit = rng.integers(0, 256, per).astype(np.uint8).tobytes()
        return (unit * (150_000 // per + 1))[:150_000]
    if kind == "text_zero_runs":  # tokens spanning many chunks and homes, then text again
        parts = []
        for i, z in enumerate((9000, 300, 70_000, 4096, 257)):
            parts += [D.enwik_like(6000 + 1000 * i, seed=40 + i), bytes(z)]
        return b"".join(parts)
    if kind == "random":          # all literals: every chain trivially in sync
        return rng.integers(0, 256, 120_000).astype(np.uint8).tobytes()
    if kind == "text":
        return D.enwik_like(200_000, seed=99)
    if kind in ("ab_random", "acgt_random"):  # few distinct 3-grams: buckets of ~1000 window
        sym = np.frombuffer(b"ab" if kind == "ab_random" else b"ACGT", np.uint8)  # positions
        return sym[rng.integers(0, len(sym), 60_000)].tobytes()
    raise ValueError(kind)


LZ_EDGE_KINDS = ["long_copies", "period4096", "period4097", "text_zero_runs", "random", "text", "ab_random",
                 "acgt_random"]


@pytest.mark.parametrize("kind", LZ_EDGE_KINDS)
def test_lz77_local_edges(kolm_gpu, kind):
    data = _lz_edge(kind)
    assert kolm_gpu.encode_lz77(data)[0] == O.encode_lz77(data)


@pytest.mark.parametrize("bs", [15, 16, 17, 255, 256, 257, 4095, 4096, 4097, 4096 + 256 + 63, 12288 + 5])
def test_lz77_local_block_geometry(kolm_gpu, bs):
    """Block sizes around the 16-byte first compare, the chunk (256) and home (4096) sizes in one
    batch: the last chunk / home of every block is partial; candidates must never cross a block."""
    from kolm import _lib
    data = (D.enwik_like(30_000, seed=5) + bytes(700) + D.enwik_like(20_000, seed=6))
    nb = (len(data) + bs - 1) // bs
    _, method, payloads, st = _lib.encode_blocks(data, bs, force=[7] * nb)
    for i in range(nb):
        blk = data[i * bs:(i + 1) * bs]
        assert payloads[i] == O.encode_lz77(blk), f"block {i}"


@pytest.mark.parametrize("idx", [0, 2])
def test_lz77_index_forms(kolm_gpu, monkeypatch, idx):
    """The two ways k_lz_local gets its window's 3-gram index (KOLM_LZ_IDX, k_lz77.hip): the
    workgroup's own LDS sort (0) and the tile index with u8 ranks + bucket starts (2, ranks of
    255 or more by binary search: the few-3-gram inputs) — every edge input
    and the block geometries around the tile size, against the oracle (PY:1686-1763)."""
    from kolm import _lib
    monkeypatch.setenv("KOLM_LZ_IDX", str(idx))
    for kind in LZ_EDGE_KINDS:
        data = _lz_edge(kind)
        assert kolm_gpu.encode_lz77(data)[0] == O.encode_lz77(data), kind
    data = (D.enwik_like(30_000, seed=5) + bytes(700) + D.enwik_like(20_000, seed=6))
    for bs in (255, 4095, 4097, 8192 + 3, 12288 + 5):
        nb = (len(data) + bs - 1) // bs
        _, _, payloads, _ = _lib.encode_blocks(data, bs, force=[7] * nb)
        for i in range(nb):
            assert payloads[i] == O.encode_lz77(data[i * bs:(i + 1) * bs]), (bs, i)


# ---- candidate 10 (v2_new, opt-in; PY:1498-1576 with the automaton evaluated serially) ----

def _v2_golden():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    return np.load(os.path.join(here, "v2new.npz")), json.load(open(os.path.join(here, "v2new.json")))


def test_v2new_golden_payloads(kolm_gpu):
    """Every PY v2_new payload (85 inputs: every automaton model selected somewhere) through
    the batched device entry, candidate 10 forced."""
    from kolm import _lib
    z, m = _v2_golden()
    bad = []
    for n in m["kernels"]:
        inp = z[f"{n}/input"].tobytes()
        if not inp:
            continue
        _, _, payloads, _ = _lib.encode_blocks(inp, len(inp), cand_mask=1 << 10, force=[10])
        if payloads[0] != z[f"{n}/v2new"].tobytes():
            bad.append(n)
    assert not bad, bad


def test_v2new_golden_containers(kolm_gpu):
    """PY's containers with its full candidate list 0..10 (v2_new enabled) — v2_new wins
    blocks there — byte for byte, and decoded back."""
    z, m = _v2_golden()
    for c, e in m["containers"].items():
        data = z[f"C/{c}/input"].tobytes()
        got = kolm_gpu.compress_blocks_fixed(data, e["block_size"], v2_new=True)
        assert got == z[f"C/{c}/full10"].tobytes(), c
        assert kolm_gpu.decompress(got) == data


@pytest.mark.parametrize("bs", [16384, 5000])
def test_v2new_multiblock_vs_oracle(kolm_gpu, bs):
    """Several blocks (text, image rows, audio, zeros, random, ramp) in one batch, each
    block's candidate-10 payload and the MDL winner over ids 0..10 vs the oracle."""
    from kolm import _lib
    data = (D.enwik_like(bs + 77, seed=3) + D.gradient_bmp()[54:54 + bs] + D.sine_wav()[44:44 + bs]
            + bytes(bs // 2) + D.splitmix64_bytes(bs, seed=4) + bytes(i & 0xFF for i in range(bs)))
    nb = (len(data) + bs - 1) // bs
    sizes, method, payloads, _ = _lib.encode_blocks(data, bs, cand_mask=_lib.KOLM_FULL_MASK)
    for i in range(nb):
        blk = data[i * bs:(i + 1) * bs]
        want10 = O.candidate(10, blk)
        assert int(sizes[i][10]) == len(want10), f"block {i}"
        if int(method[i]) == 10:
            assert payloads[i] == want10, f"block {i}"
    _, _, forced, _ = _lib.encode_blocks(data, bs, cand_mask=1 << 10, force=[10] * nb)
    for i in range(nb):
        assert forced[i] == O.candidate(10, data[i * bs:(i + 1) * bs]), f"block {i}"

@pytest.mark.gpu
@pytest.mark.parametrize("sigma", [1, 2, 3, 5, 16, 17, 33, 64, 65, 129, 256])
def test_round0_alphabet_widths(kolm_gpu, sigma):
    """Round 0 packs C = min(32, 64 / w) alphabet-compacted characters (w = bits of the
    block's distinct-byte count): every code width 1..8 and its boundaries, on random text
    over sigma scattered byte values (short Lyndon factors: the C characters wrap)."""
    rng = np.random.default_rng(sigma)
    vals = rng.choice(256, sigma, replace=False).astype(np.uint8)
    data = vals[rng.integers(0, sigma, 30000)].tobytes()
    assert kolm_gpu.bbwt_forward(data) == O.bbwt_forward(data)


@pytest.mark.gpu
def test_round0_alphabet_mixed_batch(kolm_gpu):
    """One batch whose blocks have different alphabets (1, 3, 17, 50, 256 distinct bytes):
    the batch's code width is the widest block's, every block keeps its own code table."""
    from kolm import _lib
    rng = np.random.default_rng(7)
    bs = 8192
    parts = [bytes(bs), rng.choice([7, 99, 200], bs).astype(np.uint8).tobytes(),
             rng.choice(np.arange(40, 57), bs).astype(np.uint8).tobytes(), D.enwik_like(bs, seed=5),
             rng.integers(0, 256, bs).astype(np.uint8).tobytes(), b"ab" * 1000]
    data = b"".join(parts)
    sizes, method, payloads, _ = _lib.encode_blocks(data, bs)
    for i in range((len(data) + bs - 1) // bs):
        blk = data[i * bs:(i + 1) * bs]
        cand = _oracle_all(blk)
        assert list(map(int, sizes[i][:10])) == [len(c) for c in cand], f"block {i}"
        assert payloads[i] == cand[int(method[i])], f"block {i}"


REPAIR_SCALE = {"enwik_128k_repair": lambda: D.enwik_like(1 << 17, seed=77),
                "bench_block0_repair": lambda: D.enwik_like(1 << 20)}


@pytest.mark.parametrize("case", sorted(REPAIR_SCALE))
def test_repair_at_scale_vs_py(kolm_gpu, large_known, case):
    """Device Re-Pair (candidate 9) against PY's own repair_compress at 128 KiB and on the
    bench stream's block 0 (1 MiB): sha256 of PY's payload (make_golden_scale.py)."""
    if case not in large_known:
        pytest.skip(f"{case} not generated yet")
    ref = large_known[case]
    out = kolm_gpu.repair_compress(REPAIR_SCALE[case]())[0]
    assert (len(out), sha(out)) == (ref["repair"]["len"], ref["repair"]["sha256"])


def _image_like(kind: str, n: int) -> bytes:
    """Periodic image / audio structures of BASELINE config 5 at other periods: long
    periodic Lyndon factors (merge batch absorption, text LCP memo), rotation groups of
    2-8 K tied positions (the medium sort), LZ77 matches of KBs with short periods (the
    stitch's fingerprint filter), deep MTF indices (the position-parallel replay)."""
    if kind.startswith("checker"):
        run, rows_band, row = {"checker96": (48, 16, 1920), "checker12": (6, 5, 600),
                               "checker_odd": (37, 3, 999)}[kind]
        out = bytearray()
        y = 0
        while len(out) < n:
            flip = (y // rows_band) & 1
            x = np.arange(row)
            out += np.where(((x // run) + flip) % 2 == 0, 240, 40).astype(np.uint8).tobytes()
            y += 1
        return bytes(out[:n])
    if kind == "sine16":
        i = np.arange(n // 2 + 1)
        return (np.round(32767 * np.sin(2 * np.pi * 440 * i / 44100)).astype("<i2")).tobytes()[:n]
    if kind == "stripes":  # a 2 KiB random tile repeated with sparse mutations
        rng = np.random.default_rng(3)
        base = bytearray(rng.integers(0, 256, 2048).astype(np.uint8).tobytes() * (n // 2048 + 1))
        for p in rng.integers(0, n, 24):
            base[int(p)] ^= 0x55
        return bytes(base[:n])
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["checker96", "checker12", "checker_odd", "sine16", "stripes"])
def test_image_like_batches_vs_oracle(kolm_gpu, kind):
    """Batches of few blocks (the small-batch kernels) on periodic images and audio: the
    hot-path container against the oracle's, and the per-kernel BBWT / LZ77 of one block."""
    data = _image_like(kind, 2 * 65536 + 4321)
    bs = 65536
    assert kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True) == O.compress_blocks_fixed(data, bs, range(9))
    blk = data[bs:2 * bs]
    assert kolm_gpu.bbwt_forward(blk) == O.bbwt_forward(blk), "bbwt"
    assert kolm_gpu.encode_lz77(blk)[0] == O.encode_lz77(blk), "lz77"
