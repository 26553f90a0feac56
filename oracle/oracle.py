"""ORACLE — TEST INFRASTRUCTURE ONLY (checker and CPU baseline; never the product).

ctypes wrapper over ``libkolm_oracle.so`` (kolm_oracle.cpp: faithful C++ restatement of
the reference hot path) plus a pure-Python restatement of the reference's KOLR
container writer / reader, so the tests can build expected containers from oracle
payloads.  Citations: PY = final_researched/kolm_final_researched_v2-2.py.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes
import heapq
import math
import os
import struct
import subprocess
from collections import Counter
from typing import Dict, List, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkolm_oracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_char_p
        i64 = ctypes.c_int64
        for name in ("oracle_bbwt", "oracle_mtf", "oracle_lz77", "oracle_xor", "oracle_lfsr", "oracle_repair"):
            f = getattr(L, name)
            f.argtypes = [P, i64, ctypes.c_void_p, i64]
            f.restype = i64
        L.oracle_duval.argtypes = [P, i64, ctypes.c_void_p, i64]
        L.oracle_duval.restype = i64
        L.oracle_rice.argtypes = [P, i64, ctypes.c_int, ctypes.c_void_p, i64]
        L.oracle_rice.restype = i64
        L.oracle_bbwt_mtf_rice.argtypes = [P, i64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, i64]
        L.oracle_bbwt_mtf_rice.restype = i64
        L.oracle_candidate.argtypes = [ctypes.c_int, P, i64, ctypes.c_void_p, i64]
        L.oracle_candidate.restype = i64
        L.oracle_repair_fast.argtypes = [P, i64, ctypes.c_void_p, i64, ctypes.c_void_p]
        L.oracle_repair_fast.restype = i64
        L.oracle_cdc.argtypes = [P, i64, i64, i64, i64, ctypes.c_int, ctypes.c_void_p, i64]
        L.oracle_cdc.restype = i64
        _lib = L
    return _lib


def _call(fn, data: bytes, cap: int, *extra) -> bytes:
    buf = ctypes.create_string_buffer(max(cap, 1))
    if extra:
        r = fn(data, len(data), *extra, buf, cap)
    else:
        r = fn(data, len(data), buf, cap)
    if r < 0:
        raise RuntimeError(f"oracle call failed ({r})")
    return buf.raw[:r]


def duval_starts(s: bytes) -> List[int]:
    arr = (ctypes.c_int64 * max(len(s), 1))()
    r = lib().oracle_duval(s, len(s), arr, len(s))
    return list(arr[:r])


def bbwt_forward(s: bytes) -> bytes:
    return _call(lib().oracle_bbwt, s, len(s))


def mtf_encode(s: bytes) -> bytes:
    return _call(lib().oracle_mtf, s, len(s))


def rice_encode(seq: bytes, k: int = 2) -> bytes:
    return _call(lib().oracle_rice, seq, (len(seq) * ((255 >> k) + 1 + k) + 7) // 8 + 16, k)


def encode_bbwt_mtf_rice(block: bytes, flags: int, k: int = 2) -> bytes:
    return _call(lib().oracle_bbwt_mtf_rice, block, len(block) * 9 + 64, flags, k)


def encode_lz77(block: bytes) -> bytes:
    return _call(lib().oracle_lz77, block, 2 * len(block) + 16)


def encode_xor(block: bytes) -> bytes:
    return _call(lib().oracle_xor, block, 2 * len(block) + 16)


def encode_lfsr(block: bytes) -> bytes:
    return _call(lib().oracle_lfsr, block, 2 * len(block) + 16)


def repair_compress(block: bytes) -> bytes:
    return _call(lib().oracle_repair, block, 6 * len(block) + 64)


def repair_fast(block: bytes, with_stats: bool = False):
    """Exact Re-Pair (PY:1817-1911) in O(n log n) (repair_lm.cpp); same bytes as
    repair_compress.  with_stats -> (payload, (nrules, final_len, freq2_rounds, max_freq))."""
    cap = 6 * len(block) + 64
    buf = ctypes.create_string_buffer(cap)
    st = (ctypes.c_int64 * 4)()
    r = lib().oracle_repair_fast(block, len(block), buf, cap, st)
    if r < 0:
        raise RuntimeError(f"oracle call failed ({r})")
    return (buf.raw[:r], tuple(st)) if with_stats else buf.raw[:r]


def cdc_boundaries(data: bytes, min_size: int = 4096, avg_size: int = 8192, max_size: int = 16384,
                   merge_orphan_tail: bool = True) -> List[Tuple[int, int]]:
    """FastCDC chunks (PY:210-309) by cdc_oracle.cpp; PY's ValueErrors (PY:227-230)."""
    n = len(data)
    if n == 0:
        return []
    if not (min_size > 0 and min_size <= avg_size <= max_size):
        raise ValueError("Require 0 < min_size <= avg_size <= max_size")
    if avg_size < 64:
        raise ValueError("avg_size too small; use >= 64")
    cap = n // min_size + 2
    arr = (ctypes.c_int64 * (2 * cap))()
    r = lib().oracle_cdc(data, n, min_size, avg_size, max_size, 1 if merge_orphan_tail else 0, arr, cap)
    if r < 0:
        raise RuntimeError(f"oracle_cdc failed ({r})")
    return [(arr[2 * i], arr[2 * i + 1]) for i in range(r)]


BBWT_FLAGS = (0, 1, 4, 8, 16)  # candidates 2..6 (PY:2156-2160)


def candidate(mid: int, block: bytes) -> bytes:
    """Payload of candidate `mid`; Re-Pair (9) through the O(n log n) restatement
    (repair_lm.cpp, checked against the O(n*rules) one in tests/test_oracle.py)."""
    if mid == 9:
        return repair_fast(block)
    cap = 9 * len(block) + 64
    buf = ctypes.create_string_buffer(cap)
    r = lib().oracle_candidate(mid, block, len(block), buf, cap)
    if r < 0:
        raise RuntimeError(f"candidate {mid} unavailable ({r})")
    return buf.raw[:r]


# ---------------------------------------------------------------------------
# Container restatement (PY:1204-1411, 2128-2146, 2332-2550)
# ---------------------------------------------------------------------------

def uleb128(n: int) -> bytes:  # PY:111-124
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def uleb128_decode(data: bytes, pos: int) -> Tuple[int, int]:  # PY:126-137
    shift = result = 0
    while True:
        if pos >= len(data):
            raise ValueError("Truncated ULEB128")
        b = data[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


class _Bits:
    def __init__(self):
        self.buf = bytearray()
        self.cur = 0
        self.bitpos = 0

    def bit(self, b):
        self.cur |= (b & 1) << (7 - self.bitpos)
        self.bitpos += 1
        if self.bitpos == 8:
            self.buf.append(self.cur)
            self.cur = 0
            self.bitpos = 0

    def kbits(self, v, k):
        for i in range(k - 1, -1, -1):
            self.bit((v >> i) & 1)

    def value(self):
        return bytes(self.buf) + (bytes([self.cur]) if self.bitpos else b""), len(self.buf) * 8 + self.bitpos


class _HuffNode:  # PY:1267-1276
    __slots__ = ("w", "sym", "left", "right")

    def __init__(self, w, sym=None, left=None, right=None):
        self.w, self.sym, self.left, self.right = w, sym, left, right

    def __lt__(self, other):
        if self.w != other.w:
            return self.w < other.w
        a = self.sym if self.sym is not None else -1
        b = other.sym if other.sym is not None else -1
        return a < b


def huff_lengths(freq: Dict[int, int]) -> Dict[int, int]:  # PY:1278-1300
    heap = [_HuffNode(max(1, f), sym=s) for s, f in freq.items()]
    if not heap:
        return {}
    if len(heap) == 1:
        return {heap[0].sym: 1}
    heapq.heapify(heap)
    while len(heap) > 1:
        a = heapq.heappop(heap)
        b = heapq.heappop(heap)
        heapq.heappush(heap, _HuffNode(a.w + b.w, left=a, right=b))
    lengths = {}
    stack = [(heap[0], 0)]
    while stack:
        nd, d = stack.pop()
        if nd.sym is not None:
            lengths[nd.sym] = max(1, d)
        else:
            stack.append((nd.left, d + 1))
            stack.append((nd.right, d + 1))
    return lengths


def huff_canonical(lengths):  # PY:1302-1311
    items = sorted(lengths.items(), key=lambda kv: (kv[1], kv[0]))
    enc, dec = {}, {}
    code = prev = maxlen = 0
    for sym, L in items:
        if L != prev:
            code <<= (L - prev)
            prev = L
        enc[sym] = (code, L)
        dec[(L, code)] = sym
        maxlen = max(maxlen, L)
        code += 1
    return enc, dec, maxlen


def rice_write(bw: _Bits, seq, k):  # PY:1331-1338
    M = 1 << k
    for n in seq:
        q, r = (n // M, n % M) if k > 0 else (n, 0)
        for _ in range(q):
            bw.bit(1)
        bw.bit(0)
        if k > 0:
            bw.kbits(r, k)


def ef_choose_l(U, n):  # PY:1352-1357
    if n <= 0 or U <= 1:
        return 0
    avg = U // n
    if avg <= 1:
        return 0
    return max(0, int(math.floor(math.log2(avg))))


def ef_write(bw: _Bits, P, U):  # PY:1359-1375
    n = len(P)
    l = ef_choose_l(U, n)
    for x in P:
        bw.kbits(x & ((1 << l) - 1), l)
    m = (U + ((1 << l) - 1)) >> l
    bits = [0] * (m + n)
    for i, x in enumerate(P):
        bits[(x >> l) + i] = 1
    for b in bits:
        bw.bit(b)


def rle_ids(ids):  # PY:1403-1410
    if not ids:
        return [], []
    syms, runs = [ids[0]], [1]
    for x in ids[1:]:
        if x == syms[-1]:
            runs[-1] += 1
        else:
            syms.append(x)
            runs.append(1)
    return syms, runs


def zz_enc(x: int) -> int:  # PY:1261-1262
    return (x << 1) if x >= 0 else ((-x) << 1) - 1


def write_container_fixed(total_len: int, block_size: int, method_ids: Sequence[int],
                          orig_lens: Sequence[int], payloads: Sequence[bytes], cdc: bool = False) -> bytes:
    """PY:2332-2445 (FIXED mode) given the per-block MDL winners; cdc=True: PY:2213-2326
    (CDC mode, block_size = avg_size: mode bit, ZigZag/Rice orig-length deltas)."""
    out = bytearray(b"KOLR")
    out += struct.pack("<I", ((1 << 31) if cdc else 0) | (block_size & 0x7FFFFFFF))
    out += struct.pack("<I", total_len)
    out += struct.pack("<H", len(method_ids))
    payload_lens = [len(p) for p in payloads]
    total_payload = sum(payload_lens)
    run_syms, run_lens = rle_ids(list(method_ids))
    lengths = huff_lengths(Counter(run_syms))
    enc_tbl, _, _ = huff_canonical(lengths)
    best_k, best_bits = 0, 1 << 60
    for k in range(8):
        bw = _Bits()
        rice_write(bw, run_lens, k)
        _, bits = bw.value()
        if bits < best_bits:
            best_bits, best_k = bits, k
    hdr = bytearray()
    hdr += uleb128(len(run_syms))
    hdr += uleb128(len(enc_tbl))
    for sym, L in sorted(lengths.items(), key=lambda kv: (kv[1], kv[0])):
        hdr += uleb128(sym) + uleb128(L)
    hdr += uleb128(best_k)
    deltas = None
    if not cdc:
        hdr += uleb128(orig_lens[-1] if orig_lens else 0)
    else:
        deltas = [zz_enc(ol - block_size) for ol in orig_lens]
        best_k2, best_bits2 = 0, 1 << 60
        for k in range(8):
            bw = _Bits()
            rice_write(bw, deltas, k)
            _, bits = bw.value()
            if bits < best_bits2:
                best_bits2, best_k2 = bits, k
        hdr += uleb128(best_k2)
    bw = _Bits()
    for s in run_syms:
        c, L = enc_tbl[s]
        bw.kbits(c, L)
    rice_write(bw, run_lens, best_k)
    if deltas is not None:
        rice_write(bw, deltas, best_k2)
    P, acc = [], 0
    for L in payload_lens:
        acc += L
        P.append(acc)
    ef_write(bw, P, total_payload)
    toc_bits, toc_bitlen = bw.value()
    out += uleb128(len(hdr)) + uleb128(toc_bitlen) + uleb128(total_payload)
    out += hdr + toc_bits
    for p in payloads:
        out += p
    return bytes(out)


def compress_blocks_fixed(data: bytes, block_size: int = 8192, ids: Sequence[int] = range(9)) -> bytes:
    """Oracle compress: per-block MDL argmin over candidate ids (PY:2350-2369)."""
    if block_size <= 0:
        raise ValueError("block_size must be positive")
    n = len(data)
    mids, lens, pays = [], [], []
    for start in range(0, n, block_size):
        block = data[start:start + block_size]
        best = None
        for mid in ids:
            p = candidate(mid, block)
            if best is None or len(p) < len(best[0]):
                best = (p, mid)
        mids.append(best[1])
        lens.append(len(block))
        pays.append(best[0])
    return write_container_fixed(n, block_size, mids, lens, pays)


def compress_blocks_cdc(data: bytes, min_size: int = 4096, avg_size: int = 8192, max_size: int = 16384,
                        ids: Sequence[int] = range(9)) -> bytes:
    """Oracle compress in CDC mode (PY:2213-2326): FastCDC chunks, per-chunk MDL argmin."""
    mids, lens, pays = [], [], []
    for s, e in cdc_boundaries(data, min_size, avg_size, max_size):
        block = data[s:e]
        best = None
        for mid in ids:
            p = candidate(mid, block)
            if best is None or len(p) < len(best[0]):
                best = (p, mid)
        mids.append(best[1])
        lens.append(len(block))
        pays.append(best[0])
    return write_container_fixed(len(data), avg_size, mids, lens, pays, cdc=True)


FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3


def fnv1a64(data: bytes) -> int:
    """FNV-1a-64 (SURVEY.md §8c known answers), numpy-vectorised per 8 lanes is not
    possible (sequential), so done in chunks via Python ints."""
    h = FNV_OFFSET
    for b in data:
        h ^= b
        h = (h * FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h
