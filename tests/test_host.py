"""Host-side product logic (no GPU): input generators, KOLR container writer/reader,
host decoders, candidate registry semantics."""
import hashlib

import numpy as np
import pytest

import kolm
from kolm import container, datagen as D, decode
from kolm.parallel import shard_blocks


@pytest.mark.parametrize("name", sorted(D.REFERENCE_FILES))
def test_reference_file_regenerators(name):
    data = D.REFERENCE_FILES[name]()
    assert hashlib.sha256(data).hexdigest() == D.REFERENCE_SHA256[name]


def test_enwik_deterministic():
    a = D.enwik_like(1 << 20)
    b = D.enwik_like(1 << 20)
    assert a == b and len(a) == 1 << 20
    assert hashlib.sha256(a).hexdigest() == hashlib.sha256(D.enwik_like(1 << 20, seed=D.ENWIK_SEED)).hexdigest()
    assert D.enwik_like(1 << 16, seed=1) != D.enwik_like(1 << 16, seed=2)
    h = np.bincount(np.frombuffer(a, np.uint8), minlength=256) / len(a)
    h = h[h > 0]
    assert 3.5 < float(-(h * np.log2(h)).sum()) < 4.5  # text-like order-0 entropy


def test_container_roundtrip_goldens(golden_containers, manifest):
    """Our TOC writer re-serialises every PY container byte-for-byte; our decoders
    decompress every PY container (full candidate list, incl. Re-Pair blocks)."""
    for cname in manifest["containers"]:
        for kind in ("full", "ids0_8"):
            blob = golden_containers[f"{cname}/{kind}"].tobytes()
            inp = golden_containers[f"{cname}/input"].tobytes()
            mode, sz, tot, mids, orig, pays = container.read_container(blob)
            assert container.write_container(mode, sz, tot, mids, orig, pays) == blob
            assert kolm.decompress(blob, device=False) == inp


def test_container_errors():
    with pytest.raises(ValueError):
        kolm.decompress(b"NOPE" + bytes(20), device=False)
    blob = container.write_container(container.MODE_FIXED, 4, 3, [0], [3], [b"abc"])
    with pytest.raises(ValueError):
        kolm.decompress(blob + b"\x00", device=False)  # strict trailing-bytes check (PY:2545-2547)
    import struct
    with pytest.raises(struct.error):
        container.write_container(container.MODE_FIXED, 1, 70000, [0] * 70000, [1] * 70000, [b"a"] * 70000)


def test_huffman_ties_many_ids():
    """>= 3 distinct run symbols exercise PY's heapq tie behaviour (App. C.6)."""
    ids = [7, 7, 2, 0, 0, 0, 2, 6, 6, 1, 7, 8, 8, 2, 7]
    pays = [bytes([i]) * (i + 1) for i in range(len(ids))]
    blob = container.write_container(container.MODE_FIXED, 16, 16 * (len(ids) - 1) + 5, ids,
                                     [16] * (len(ids) - 1) + [5], pays)
    _, _, _, mids, orig, p2 = container.read_container(blob)
    assert mids == ids and p2 == pays


@pytest.mark.parametrize("name", ["text_hobbit", "banana", "tiny07", "zero16k", "enwik16k", "abab"])
def test_host_decoders_invert_golden_kernels(golden_kernels, name):
    g = lambda k: golden_kernels[f"{name}/{k}"].tobytes()  # noqa: E731
    inp = g("input")
    assert decode.bbwt_inverse(g("bbwt")) == inp
    assert decode.mtf_decode(list(g("mtf"))) == g("bbwt")
    for mid, f in decode.BBWT_FLAGS.items():
        assert decode.decode_bbwt_mtf_rice(g(f"rice{f}"), len(inp), f) == inp
    assert decode.decode_lz77(g("lz77"), len(inp)) == inp
    assert decode.decode_xor(g("xor"), len(inp)) == inp
    assert decode.decode_lfsr(g("lfsr"), len(inp)) == inp
    assert decode.repair_decompress(g("repair"), len(inp)) == inp


def test_fixed_boundaries_matches_reference_semantics():
    assert kolm.fixed_boundaries(b"", 4) == []
    assert kolm.fixed_boundaries(b"abcdefghij", 4) == [(0, 4), (4, 8), (8, 10)]
    with pytest.raises(ValueError):
        kolm.fixed_boundaries(b"ab", 0)


def test_registry_ids_stable():
    names = [n for _, n in kolm._select_encoders()]
    assert names == kolm.CANDIDATE_NAMES
    assert len(kolm._select_decoders()) == 11
    kolm.G_NO_LZ77 = True
    try:
        assert kolm.candidate_mask() == 0x3FF & ~(1 << 7)
        assert kolm.candidate_mask(hot_path=True) == 0x1FF & ~(1 << 7)
        assert [n for _, n in kolm._select_encoders()] == kolm.CANDIDATE_NAMES  # ids unchanged
    finally:
        kolm.G_NO_LZ77 = False
    kolm.G_ONLY_METHOD = "lz77"
    try:
        assert kolm.candidate_mask() == 1 << 7
        kolm.G_ONLY_METHOD = "repair"
        assert kolm.candidate_mask() == 1 << 9
    finally:
        kolm.G_ONLY_METHOD = None
    with pytest.raises(NameError):
        kolm._select_encoders()[10][0](b"x")  # v2_new raises as in PY
    kolm.G_ONLY_METHOD = "v2_new"
    try:
        with pytest.raises(NameError):  # PY: the only candidate and its fallback raise
            kolm.candidate_mask()
        kolm.G_V2_NEW = True
        assert kolm.candidate_mask() == 1 << 10
    finally:
        kolm.G_ONLY_METHOD = None
        kolm.G_V2_NEW = False
    kolm.G_V2_NEW = True
    try:
        assert kolm.candidate_mask() == 0x7FF
        assert kolm.candidate_mask(hot_path=True) == 0x1FF
    finally:
        kolm.G_V2_NEW = False


@pytest.mark.parametrize("nb,world", [(0, 2), (1, 2), (7, 2), (256, 8), (5, 8), (1000, 3)])
def test_shard_blocks_cover(nb, world):
    seen = []
    for r in range(world):
        f, c = shard_blocks(nb, r, world)
        seen.extend(range(f, f + c))
    assert seen == list(range(nb))
    counts = [shard_blocks(nb, r, world)[1] for r in range(world)]
    assert max(counts) - min(counts) <= 1


def test_uleb128():
    for v in [0, 1, 127, 128, 255, 16383, 16384, 2 ** 31]:
        b = kolm.uleb128_encode(v)
        assert kolm.uleb128_decode_stream(b, 0) == (v, len(b))
    with pytest.raises(ValueError):
        kolm.uleb128_encode(-1)


def test_host_v2new_decoder_goldens():
    """decode_new_pipeline (PY:1578-1648) + automaton inverse (PY:1056-1092) on the host
    inverts every PY v2_new payload, and decompress(device=False) PY's id-10 containers."""
    import json
    import os
    from kolm.decode import decode_new_pipeline
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(here, "v2new.npz"))
    m = json.load(open(os.path.join(here, "v2new.json")))
    for n in m["kernels"]:
        data = z[f"{n}/input"].tobytes()
        assert decode_new_pipeline(z[f"{n}/v2new"].tobytes(), len(data)) == data, n
    for c in m["containers"]:
        assert kolm.decompress(z[f"C/{c}/full10"].tobytes(), device=False) == z[f"C/{c}/input"].tobytes(), c


@pytest.mark.parametrize("seed", range(40))
def test_toc_writer_matches_reference_heapq(seed):
    """The native TOC writer (kolm_toc.cpp) against the oracle's restatement of PY's writer
    (Python heapq + _HuffNode ordering, PY:1267-1300, 2375-2445) on random method-id
    sequences built to produce many equal-weight merged entries (2..11 distinct ids, runs
    of 1..4): fixed and CDC mode, byte for byte, and read back."""
    import oracle
    rng = np.random.default_rng(seed)
    k = int(rng.integers(2, 12))
    alphabet = rng.choice(11, k, replace=False)
    ids = []
    while len(ids) < int(rng.integers(1, 400)):
        ids += [int(rng.choice(alphabet))] * int(rng.integers(1, 5))
    nb = len(ids)
    bs = int(rng.integers(1, 5000))
    cdc = bool(seed & 1)
    lens = ([int(x) for x in rng.integers(1, 3 * bs, nb)] if cdc else [bs] * (nb - 1) + [int(rng.integers(1, bs + 1))])
    pays = [bytes(int(rng.integers(0, 40))) for _ in range(nb)]
    want = oracle.write_container_fixed(sum(lens), bs, ids, lens, pays, cdc=cdc)
    got = container.write_container(container.MODE_CDC if cdc else container.MODE_FIXED, bs, sum(lens), ids, lens, pays)
    assert got == want
    mode, sz, tot, mids, orig, p2 = container.read_container(got)
    assert (mode, sz, tot, mids, orig, p2) == (int(cdc), bs, sum(lens), ids, lens, pays)


def test_toc_reader_errors():
    blob = container.write_container(container.MODE_FIXED, 8, 20, [2, 7, 7], [8, 8, 4], [b"ab", b"c", b"def"])
    for bad, msg in ((b"KOLX" + blob[4:], "Invalid magic"), (blob[:-1], "Truncated payload area"),
                     (blob + b"\0\0", "Extra trailing 2 bytes"), (blob[:16], "Truncated")):
        with pytest.raises(ValueError, match=msg):
            container.read_container(bad)
    assert kolm.uleb128_decode_stream(b"\x80\x80\x01", 0) == (16384, 3)
    with pytest.raises(ValueError):
        kolm.uleb128_decode_stream(b"\x80\x80", 0)


def test_bench_stream_fixture_consistent():
    """tests/golden/bench_stream.json (make_golden_bench.py) describes bench.py's rank-0
    stream: same input bytes, winners = argmin of the recorded sizes (ties -> lowest id)."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_stream.json")))["ranks"]["0"]
    data = D.enwik_like(g["bytes"], seed=g["seed"])
    assert hashlib.sha256(data).hexdigest() == g["input_sha256"] and g["seed"] == D.ENWIK_SEED
    for rec in g["blocks"]:
        s = rec["sizes"]
        assert rec["w9"] == min(range(9), key=lambda m: (s[m], m))
        assert rec["w10"] == min(range(10), key=lambda m: (s[m], m))
        assert s[0] == g["block_size"]


@pytest.mark.parametrize("nb,world", [(0, 2), (7, 2), (256, 8), (5, 8), (1000, 3)])
def test_rank_blocks_partitions(nb, world):
    from kolm.parallel import rank_blocks
    for part in ("contiguous", "round_robin"):
        seen = sorted(i for r in range(world) for i in rank_blocks(nb, r, world, part))
        assert seen == list(range(nb))
    assert list(rank_blocks(10, 1, 4, "round_robin")) == [1, 5, 9]


def _with_code_len(blob: bytes, new_len: int) -> bytes:
    """blob (one method id, so one prefix-code entry) with that entry's code length
    replaced: the TOC header is ULEB(hdr_len) ULEB(toc_bits) ULEB(U) then
    [n_runs, K, sym, len, ...]; every field here is one byte."""
    assert blob[14] < 0x80 and blob[15] < 0x80 and blob[16] < 0x80
    hdr = bytearray(blob[17:17 + blob[14]])
    assert hdr[1] == 1  # K
    hdr[3] = new_len
    return blob[:17] + bytes(hdr) + blob[17 + blob[14]:]


def test_toc_reader_hostile_code_lengths():
    """Code lengths past 32 / 64 bits are read as PY reads them (any size, PY:1302-1329): the
    one-symbol code of this container then needs that many zero bits, which its 1-bit stream
    does not hold, so decoding fails (as in PY) instead of wrapping a 64-bit code value.  PY's
    own containers with 40- and 70-bit codes decode: test_toc_prefix_code_lengths_as_py."""
    blob = container.write_container(container.MODE_FIXED, 8, 24, [7, 7, 7], [8, 8, 8], [b"a", b"b", b"c"])
    assert container.read_container(_with_code_len(blob, 1))[3] == [7, 7, 7]
    for bad in (33, 64, 127):
        with pytest.raises(ValueError):
            container.read_container(_with_code_len(blob, bad))


def test_toc_reader_many_codes_fast():
    """A header with thousands of prefix-code entries (repeated symbols, as a hostile
    container could carry) is parsed in linear time: the symbols are deduplicated through
    a hash map, not pairwise."""
    import time
    from kolm.container import uleb128_encode as U
    body = bytearray()
    K = 40000
    body += U(1) + U(K)
    for i in range(K):
        body += U(i % 5000) + U(1 + i % 20)
    body += U(0) + U(8)  # k_runs, tail (last block length)
    hdr = bytes(body)
    blob = b"KOLR" + (8).to_bytes(4, "little") + (8).to_bytes(4, "little") + (1).to_bytes(2, "little") \
        + U(len(hdr)) + U(8) + U(0) + hdr + b"\0"
    t0 = time.time()
    with pytest.raises(ValueError):
        container.read_container(blob)
    assert time.time() - t0 < 2.0


def _toc_cases():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "toc_cases.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["huff_40", "huff_70", "huff_len0", "huff_oversub"])
def test_toc_prefix_code_lengths_as_py(name):
    """Method-id prefix codes with lengths PY's writer never produces (40 / 70 bits, a length-0
    symbol that shifts the numbering, an oversubscribed set) written by PY itself
    (make_golden_toc.py): the native reader decodes exactly what PY's decompress decodes, or
    fails where it fails (PY:1302-1329, 2451-2500)."""
    c = _toc_cases()[name]
    blob = bytes.fromhex(c["container"])
    if "ok" in c["py"]:
        assert kolm.decompress(blob, device=False) == bytes.fromhex(c["py"]["ok"])
    else:
        with pytest.raises(ValueError, match=c["py"]["message"]):
            kolm.decompress(blob, device=False)


@pytest.mark.parametrize("name", ["bitplane_n13", "bitplane_n16", "bitplane_n21"])
def test_bitplane_partial_group_divergence(name):
    """Deliberate divergence, pinned: a bit-plane BBWT block (id 3) whose length is not a multiple
    of 8.  PY's own container (make_golden_toc.py) makes PY's decompress raise IndexError (it
    reads n Rice values where its encoder wrote 8*ceil(n/8), then indexes past the last partial
    group, PY:1122-1134, 2075-2089); this decoder reads the padded count and returns the input.
    At n % 8 == 0 both decode."""
    c = _toc_cases()[name]
    blob, inp = bytes.fromhex(c["container"]), bytes.fromhex(c["input"])
    n = len(inp)
    assert ("error" in c["py"]) == (n % 8 != 0)
    if n % 8:
        assert c["py"]["error"] == "IndexError"
    else:
        assert bytes.fromhex(c["py"]["ok"]) == inp
    assert kolm.decompress(blob, device=False) == inp
    assert decode.decode_block(3, container.read_container(blob)[5][0], n) == inp
