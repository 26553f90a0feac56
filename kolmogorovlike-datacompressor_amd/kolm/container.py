"""KOLR container: header + TOC (host side; a few hundred bytes per 65535 blocks).

Same byte format as the reference (PY = kolm_final_researched_v2-2.py):
  b'KOLR' | <I mode<<31 | size | <I total_len | <H nblocks          PY:2333-2339, 2128-2146
  ULEB toc_hdr_len | ULEB toc_bitlen | ULEB total_payload           PY:2436-2438
  toc_header: ULEB n_runs, ULEB K, K x (ULEB sym, ULEB len) in canonical order,
              ULEB rice_k(run lengths), FIXED: ULEB last_orig_len   PY:2392-2406
              (CDC: ULEB rice_k(zigzag(orig_len - avg)))
  toc_bits (MSB-first): canonical Huffman of the run symbols of the method ids,
              Rice(k) run lengths, [CDC: Rice(k2) deltas], Elias-Fano of the
              cumulative payload ends (low bits first, then the high bitvector)
                                                                     PY:2409-2426, 1359-1375
  payloads back to back.
Tie semantics of PY's Huffman (heapq over _HuffNode, internal nodes compare as
sym = -1, Counter insertion order, PY:1267-1300) are reproduced by using the same
algorithm on the same data structures.
"""
from __future__ import annotations

import heapq
import math
import struct
from collections import Counter
from typing import Dict, List, Sequence, Tuple

MAGIC = b"KOLR"
MODE_FIXED = 0
MODE_CDC = 1


def uleb128_encode(n: int) -> bytes:
    """PY:111-124."""
    if n < 0:
        raise ValueError("ULEB128 only supports unsigned integers")
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def uleb128_decode_stream(data: bytes, pos: int = 0) -> Tuple[int, int]:
    """PY:126-137."""
    shift = result = 0
    while True:
        if pos >= len(data):
            raise ValueError("Truncated ULEB128")
        b = data[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if (b & 0x80) == 0:
            return result, pos
        shift += 7


def pack_mode_and_size(mode: int, size: int) -> int:
    if mode not in (MODE_FIXED, MODE_CDC):
        raise ValueError("invalid mode")
    if size < 0 or size > 0x7FFFFFFF:
        raise ValueError("size out of range (must fit in 31 bits)")
    return ((mode & 1) << 31) | (size & 0x7FFFFFFF)


class BitWriter:
    """MSB-first bit writer (PY:1231-1254)."""

    __slots__ = ("buf", "cur", "bitpos")

    def __init__(self):
        self.buf = bytearray()
        self.cur = 0
        self.bitpos = 0

    def write_bit(self, b: int):
        self.cur |= (b & 1) << (7 - self.bitpos)
        self.bitpos += 1
        if self.bitpos == 8:
            self.buf.append(self.cur)
            self.cur = 0
            self.bitpos = 0

    def write_kbits(self, val: int, k: int):
        for i in range(k - 1, -1, -1):
            self.write_bit((val >> i) & 1)

    def getvalue_bits(self) -> Tuple[bytes, int]:
        return (bytes(self.buf) + (bytes([self.cur]) if self.bitpos else b""),
                len(self.buf) * 8 + self.bitpos)


class BitReader:
    __slots__ = ("buf", "byte", "bit")

    def __init__(self, buf: bytes):
        self.buf = buf
        self.byte = 0
        self.bit = 0

    def read_bit(self) -> int:
        if self.byte >= len(self.buf):
            raise ValueError("BitReader: out of data")
        v = (self.buf[self.byte] >> (7 - self.bit)) & 1
        self.bit += 1
        if self.bit == 8:
            self.bit = 0
            self.byte += 1
        return v


class _HuffNode:
    __slots__ = ("w", "sym", "left", "right")

    def __init__(self, w, sym=None, left=None, right=None):
        self.w, self.sym, self.left, self.right = w, sym, left, right

    def __lt__(self, other):
        if self.w != other.w:
            return self.w < other.w
        a = self.sym if self.sym is not None else -1
        b = other.sym if other.sym is not None else -1
        return a < b


def huff_lengths(freq: Dict[int, int]) -> Dict[int, int]:
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
    lengths: Dict[int, int] = {}
    stack = [(heap[0], 0)]
    while stack:
        nd, d = stack.pop()
        if nd.sym is not None:
            lengths[nd.sym] = max(1, d)
        else:
            stack.append((nd.left, d + 1))
            stack.append((nd.right, d + 1))
    return lengths


def huff_canonical(lengths: Dict[int, int]):
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


def rice_write_values(bw: BitWriter, seq: Sequence[int], k: int):
    M = 1 << k
    for n in seq:
        q, r = (n // M, n % M) if k > 0 else (n, 0)
        for _ in range(q):
            bw.write_bit(1)
        bw.write_bit(0)
        if k > 0:
            bw.write_kbits(r, k)


def rice_bits(seq: Sequence[int], k: int) -> int:
    return sum((n >> k) + 1 + k for n in seq)


def rice_read_n(br: BitReader, k: int, nvals: int) -> List[int]:
    M = 1 << k
    out = []
    for _ in range(nvals):
        q = 0
        while br.read_bit() == 1:
            q += 1
        r = 0
        for _ in range(k):
            r = (r << 1) | br.read_bit()
        out.append(q * M + r)
    return out


def ef_choose_l(U: int, n: int) -> int:
    if n <= 0 or U <= 1:
        return 0
    avg = U // n
    if avg <= 1:
        return 0
    return max(0, int(math.floor(math.log2(avg))))


def ef_write_positions(bw: BitWriter, P: Sequence[int], U: int):
    n = len(P)
    l = ef_choose_l(U, n)
    for x in P:
        bw.write_kbits(x & ((1 << l) - 1), l)
    m = (U + ((1 << l) - 1)) >> l
    bits = [0] * (m + n)
    for i, x in enumerate(P):
        bits[(x >> l) + i] = 1
    for b in bits:
        bw.write_bit(b)


def ef_read_positions(br: BitReader, U: int, n: int) -> List[int]:
    l = ef_choose_l(U, n)
    lows = []
    for _ in range(n):
        v = 0
        for _ in range(l):
            v = (v << 1) | br.read_bit()
        lows.append(v)
    m = (U + ((1 << l) - 1)) >> l
    ones = []
    total = m + n
    for idx in range(total):
        if br.read_bit() == 1:
            ones.append(idx)
            if len(ones) == n:
                for _ in range(idx + 1, total):
                    br.read_bit()
                break
    return [((ones[i] - i) << l) | lows[i] for i in range(n)]


def rle_ids(ids: Sequence[int]):
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


def zz_enc(x: int) -> int:
    return (x << 1) if x >= 0 else ((-x) << 1) - 1


def zz_dec(n: int) -> int:
    return (n >> 1) if (n & 1) == 0 else -((n + 1) >> 1)


def write_container(mode: int, size_field: int, total_len: int, method_ids: Sequence[int],
                    orig_lens: Sequence[int], payloads: Sequence[bytes]) -> bytes:
    """Assemble a KOLR container (PY:2213-2326 CDC, PY:2332-2445 FIXED)."""
    nblocks = len(method_ids)
    out = bytearray(MAGIC)
    out += struct.pack("<I", pack_mode_and_size(mode, size_field))
    out += struct.pack("<I", total_len)
    out += struct.pack("<H", nblocks)  # struct.error above 65535, as in PY
    payload_lens = [len(p) for p in payloads]
    total_payload = sum(payload_lens)
    run_syms, run_lens = rle_ids(list(method_ids))
    lengths = huff_lengths(Counter(run_syms))
    enc_tbl, _, _ = huff_canonical(lengths)
    best_k, best_bits = 0, 1 << 60
    for k in range(8):
        bits = rice_bits(run_lens, k)
        if bits < best_bits:
            best_bits, best_k = bits, k
    hdr = bytearray()
    hdr += uleb128_encode(len(run_syms))
    hdr += uleb128_encode(len(enc_tbl))
    for sym, L in sorted(lengths.items(), key=lambda kv: (kv[1], kv[0])):
        hdr += uleb128_encode(sym) + uleb128_encode(L)
    hdr += uleb128_encode(best_k)
    deltas = None
    if mode == MODE_FIXED:
        hdr += uleb128_encode(orig_lens[-1] if nblocks > 0 else 0)
    else:
        deltas = [zz_enc(ol - size_field) for ol in orig_lens]
        best_k2, best_bits2 = 0, 1 << 60
        for k in range(8):
            bits = rice_bits(deltas, k)
            if bits < best_bits2:
                best_bits2, best_k2 = bits, k
        hdr += uleb128_encode(best_k2)
    bw = BitWriter()
    for s in run_syms:
        c, L = enc_tbl[s]
        bw.write_kbits(c, L)
    rice_write_values(bw, run_lens, best_k)
    if deltas is not None:
        rice_write_values(bw, deltas, best_k2)
    P, acc = [], 0
    for L in payload_lens:
        acc += L
        P.append(acc)
    ef_write_positions(bw, P, total_payload)
    toc_bits, toc_bitlen = bw.getvalue_bits()
    out += uleb128_encode(len(hdr)) + uleb128_encode(toc_bitlen) + uleb128_encode(total_payload)
    out += hdr + toc_bits
    for p in payloads:
        out += p
    return bytes(out)


def read_container(container: bytes):
    """Parse a KOLR container (PY:2451-2524).  Returns (mode, size_field, total_len,
    method_ids, orig_lens, payload_bytes_list)."""
    if len(container) < 4 or container[:4] != MAGIC:
        raise ValueError("Invalid magic")
    pos = 4
    packed = struct.unpack_from("<I", container, pos)[0]
    pos += 4
    mode, size_field = (packed >> 31) & 1, packed & 0x7FFFFFFF
    total_len = struct.unpack_from("<I", container, pos)[0]
    pos += 4
    nblocks = struct.unpack_from("<H", container, pos)[0]
    pos += 2
    toc_hdr_len, pos = uleb128_decode_stream(container, pos)
    toc_bitlen, pos = uleb128_decode_stream(container, pos)
    total_payload, pos = uleb128_decode_stream(container, pos)
    if pos + toc_hdr_len > len(container):
        raise ValueError("Truncated TOC header")
    hdr = container[pos:pos + toc_hdr_len]
    pos += toc_hdr_len
    nbits_bytes = (toc_bitlen + 7) // 8
    if pos + nbits_bytes > len(container):
        raise ValueError("Truncated TOC bits")
    bits = container[pos:pos + nbits_bytes]
    pos += nbits_bytes
    p = 0
    n_runs, p = uleb128_decode_stream(hdr, p)
    K, p = uleb128_decode_stream(hdr, p)
    lengths = {}
    for _ in range(K):
        sym, p = uleb128_decode_stream(hdr, p)
        L, p = uleb128_decode_stream(hdr, p)
        lengths[sym] = L
    k_runs, p = uleb128_decode_stream(hdr, p)
    if mode == MODE_FIXED:
        last_len, p = uleb128_decode_stream(hdr, p)
    else:
        k_orig, p = uleb128_decode_stream(hdr, p)
    _, dec, maxlen = huff_canonical(lengths)
    br = BitReader(bits)
    run_syms = []
    for _ in range(n_runs):
        c = 0
        for L in range(1, maxlen + 1):
            c = (c << 1) | br.read_bit()
            if (L, c) in dec:
                run_syms.append(dec[(L, c)])
                break
        else:
            raise ValueError("Huffman decode failed")
    run_lens = rice_read_n(br, k_runs, n_runs)
    method_ids = []
    for s, r in zip(run_syms, run_lens):
        method_ids.extend([s] * r)
    if len(method_ids) != nblocks:
        raise ValueError("Method id RLE expands to wrong size")
    if mode == MODE_FIXED:
        orig_lens = [size_field] * (nblocks - 1) + ([last_len] if nblocks > 0 else [])
    else:
        orig_lens = [size_field + zz_dec(x) for x in rice_read_n(br, k_orig, nblocks)]
    ends = ef_read_positions(br, total_payload, nblocks)
    if ends and ends[-1] != total_payload:
        raise ValueError("Payload EF sum mismatch")
    if pos + total_payload > len(container):
        raise ValueError("Truncated payload area")
    area = container[pos:pos + total_payload]
    pos += total_payload
    if pos != len(container):
        raise ValueError(f"Extra trailing {len(container) - pos} bytes after container end")
    payloads, start = [], 0
    for e in ends:
        payloads.append(area[start:e])
        start = e
    return mode, size_field, total_len, method_ids, orig_lens, payloads
