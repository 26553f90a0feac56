"""Block decoders for ``decompress()`` — host side.

The decode direction is outside the north-star hot path (SURVEY.md §8f row 4 lists GPU
decode kernels as "next"); these host decoders exist so that ``kolm.decompress`` keeps
the reference block API and so that round trips can be tested.  They follow the
reference decoders (PY = kolm_final_researched_v2-2.py), with one deliberate fix:
PY's bit-plane decoder reads ``orig_len`` Rice values although the encoder emitted
8*ceil(n/8); here the padded count is read so every container the
reference encoder can produce decodes.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from .container import uleb128_decode_stream


def decode_raw(payload: bytes, n: int) -> bytes:  # PY:2101
    if len(payload) != n:
        raise ValueError("raw payload length mismatch")
    return bytes(payload)


def _uleb_bytes(payload: bytes, n: int) -> np.ndarray:
    """Decode n ULEB values < 2^14 (each 1 or 2 bytes)."""
    out = np.empty(n, dtype=np.int64)
    pos = 0
    for i in range(n):
        v, pos = uleb128_decode_stream(payload, pos)
        out[i] = v
    if pos != len(payload):
        raise ValueError("trailing bytes in ULEB stream")
    return out


def decode_xor(payload: bytes, n: int) -> bytes:  # PY:2113-2122
    d = _uleb_bytes(payload, n)
    return (np.cumsum(d) & 0xFF).astype(np.uint8).tobytes()


_LFSR = None


def _lfsr_table() -> np.ndarray:
    global _LFSR
    if _LFSR is None:
        s, tab = 1, []
        for _ in range(255):
            tab.append(s)
            fb = 0
            for bit in range(8):
                if (0x96 >> bit) & 1:
                    fb ^= (s >> bit) & 1
            s = ((s << 1) & 0xFF) | fb
        _LFSR = np.array(tab, dtype=np.int64)
    return _LFSR


def decode_lfsr(payload: bytes, n: int) -> bytes:  # PY:2005-2019
    d = _uleb_bytes(payload, n)
    st = _lfsr_table()[np.arange(n) % 255]
    return ((d + st) & 0xFF).astype(np.uint8).tobytes()


def rice_decode(data: bytes, k: int, nvals: int) -> np.ndarray:  # PY:1423-1460
    bits = np.unpackbits(np.frombuffer(data, dtype=np.uint8))
    zeros = np.flatnonzero(bits == 0)
    out = np.empty(nvals, dtype=np.int64)
    pos = 0
    nb = bits.size
    for i in range(nvals):
        j = np.searchsorted(zeros, pos)
        if j >= zeros.size:
            raise ValueError("rice: truncated unary")
        z = int(zeros[j])
        q = z - pos
        pos = z + 1
        r = 0
        if k:
            if pos + k > nb:
                raise ValueError("rice: truncated remainder")
            for t in range(k):
                r = (r << 1) | int(bits[pos + t])
            pos += k
        out[i] = (q << k) | r
    return out


def bitplane_deinterleave(data: bytes, orig_len: int) -> bytes:  # PY:1122-1134
    a = np.frombuffer(data, dtype=np.uint8).reshape(-1, 8)
    bits = np.unpackbits(a, axis=1).reshape(-1, 8, 8)  # [group][plane][byte i]
    return np.packbits(bits.transpose(0, 2, 1).reshape(-1, 8), axis=1).ravel()[:orig_len].tobytes()


_BITREV = np.array([int(f"{i:08b}"[::-1], 2) for i in range(256)], dtype=np.uint8)


def mtf_decode(seq) -> bytes:  # PY:470-478
    table = list(range(256))
    out = bytearray(len(seq))
    for i, idx in enumerate(seq):
        b = table.pop(int(idx))
        out[i] = b
        table.insert(0, b)
    return bytes(out)


def bbwt_inverse(L: bytes) -> bytes:  # PY:425-454
    n = len(L)
    if n == 0:
        return b""
    arr = np.frombuffer(L, dtype=np.uint8)
    pi = np.argsort(arr, kind="stable")
    seen = np.zeros(n, dtype=bool)
    factors: List[Tuple[int, bytes]] = []
    for i in range(n):
        if seen[i]:
            continue
        cyc = []
        cur = i
        while not seen[cur]:
            seen[cur] = True
            cyc.append(cur)
            cur = int(pi[cur])
        # i is the minimum of its cycle (cycles are discovered in increasing min order)
        seq = arr[pi[np.array(cyc)]]
        factors.append((i, seq.tobytes()))
    return b"".join(f for _, f in reversed(factors))


def decode_bbwt_mtf_rice(payload: bytes, n: int, flags: int, k: int = 2) -> bytes:  # PY:2075-2089
    length = 8 * ((n + 7) // 8) if flags & 1 else n
    seq = rice_decode(payload, k, length).astype(np.uint8)
    if flags & 16:
        g = seq.copy()
        g ^= g >> 1
        g ^= g >> 2
        g ^= g >> 4
        seq = g
    if flags & 8:
        seq = _BITREV[seq]
    if flags & 4:
        seq = ((seq & 0x0F) << 4) | (seq >> 4)
    if flags & 1:
        seq = np.frombuffer(bitplane_deinterleave(seq.tobytes(), n), dtype=np.uint8)
    return bbwt_inverse(mtf_decode(seq.tolist()))


def decode_lz77(data: bytes, orig_len: int) -> bytes:  # PY:1765-1812
    out = bytearray()
    i, n = 0, len(data)
    while i < n and len(out) < orig_len:
        flag = data[i]
        i += 1
        if flag == 0:
            if i >= n:
                raise ValueError("LZ77 truncated literal")
            out.append(data[i])
            i += 1
        elif flag == 1:
            length, i = uleb128_decode_stream(data, i)
            dist, i = uleb128_decode_stream(data, i)
            if dist == 0 or dist > min(len(out), 4096):
                raise ValueError("LZ77 invalid distance")
            start = len(out) - dist
            for t in range(min(length, orig_len - len(out))):
                out.append(out[start + t])
        else:
            raise ValueError("LZ77 unknown flag")
    if len(out) != orig_len:
        raise ValueError("LZ77 output length mismatch")
    return bytes(out)


def _uleb_values(buf: bytes) -> Tuple[np.ndarray, np.ndarray]:
    """Every ULEB128 value of buf at once: (values, end offset of each value)."""
    a = np.frombuffer(buf, dtype=np.uint8)
    ends = np.flatnonzero(a < 0x80)  # the last byte of every value
    starts = np.concatenate([[0], ends[:-1] + 1]).astype(np.int64)
    vals = np.zeros(ends.size, dtype=object)
    # values of up to 9 groups fit in 63 bits and are summed vectorised; longer ones
    # (never produced by the encoder) are folded one by one
    width = ends - starts + 1
    short = width <= 9
    acc = np.zeros(ends.size, dtype=np.int64)
    for g in range(9):
        sel = short & (width > g)
        acc[sel] |= (a[starts[sel] + g].astype(np.int64) & 0x7F) << (7 * g)
    vals[short] = acc[short].tolist()
    for j in np.flatnonzero(~short):
        vals[j] = sum((int(b) & 0x7F) << (7 * g) for g, b in enumerate(a[starts[j]:ends[j] + 1]))
    return vals, ends + 1


def repair_decompress(data: bytes, orig_len: int) -> bytes:
    """Re-Pair grammar expansion (inverse of repair_compress, PY:1913-1978): rules are
    materialised children-first in a topological order of the rules the sequence reaches
    (a rule referencing an undefined symbol or itself is rejected), then the sequence is
    a join of its symbols' expansions."""
    if len(data) < 2 or data[:2] != b"RP":
        raise ValueError("Bad magic")
    vals, ends = _uleb_values(bytes(data[2:]))

    def field(i: int) -> int:
        if i >= len(vals):
            raise ValueError("Truncated ULEB128")
        return int(vals[i])

    if field(0) != 256:
        raise ValueError("Unsupported terminal alphabet")
    nrules = field(1)
    pairs = 2 + 2 * nrules
    seq_len = field(pairs)
    field(pairs + seq_len)  # the last symbol exists
    rhs = {256 + r: (field(2 + 2 * r), field(3 + 2 * r)) for r in range(nrules)}
    seq = vals[pairs + 1:pairs + 1 + seq_len]
    # children-first order of the reachable rules (iterative DFS, gray = on the path)
    order: List[int] = []
    state: Dict[int, int] = {}
    for root in {int(s) for s in seq if s >= 256}:
        if state.get(root) == 2:
            continue
        path = [(root, 0)]
        state[root] = 1
        while path:
            sym, k = path[-1]
            if k == 2:
                path.pop()
                state[sym] = 2
                order.append(sym)
                continue
            path[-1] = (sym, k + 1)
            if sym not in rhs:
                raise ValueError(f"Re-Pair: undefined symbol {sym}")
            child = rhs[sym][k]
            if child >= 256:
                st = state.get(child, 0)
                if st == 1:
                    raise ValueError(f"Re-Pair: rule {child} expands into itself")
                if st == 0:
                    state[child] = 1
                    path.append((child, 0))
    table: Dict[int, bytes] = {t: bytes((t,)) for t in range(256)}
    for sym in order:
        a, b = rhs[sym]
        table[sym] = table[a] + table[b]
    out = b"".join(table[int(s)] for s in seq)
    if len(out) != orig_len:
        raise RuntimeError(f"RePair output length mismatch: got {len(out)}, expect {orig_len}")
    return out


BBWT_FLAGS = {2: 0, 3: 1, 4: 4, 5: 8, 6: 16}


# ---- v2_new (id 10): decode_new_pipeline PY:1578-1648 + circuit_map_automaton_inverse
# PY:1056-1092.  Every model predicts byte i from the decoded bytes before it, so the
# inverse is a sequential recurrence (PY's own backward loops).
def _dil(x: int) -> int:
    return ((((x << 1) & 0xFE) | x) | (((x >> 1) & 0x7F) | x)) & 0xFF


def _ero(x: int) -> int:
    return ~_dil(~x & 0xFF) & 0xFF


def _v2_inverse(y: bytes, mode: int, param: int) -> bytes:
    n = len(y)
    if mode == 0 or mode > 5 or n == 0 or (mode == 1 and param == 0):
        return bytes(y)
    r = bytearray(n)
    for i in range(n):
        if mode == 1:    # Delta-k PY:679-690
            p = 0 if i < param else r[i - param]
        elif mode in (2, 3):  # Gray family PY:727-752, nibble interleave PY:805-826
            if i == 0:
                p = 0
            elif i == 1:
                p = r[0]
            else:
                a, b = r[i - 1], r[i - 2]
                if mode == 3:
                    p = (a & 0xF0) | (b & 0x0F)  # mux(select, cross, run) == cross for every a, b
                else:
                    v = param & 3
                    x = a if v == 0 else b if v == 1 else (a ^ b) if v == 2 else (a | b)
                    p = x ^ (x >> 1)
        elif mode == 4:  # Majority-of-3 PY:849-866
            if i == 0:
                p = 0
            elif i < 3:
                p = r[i - 1]
            else:
                a, b, c = r[i - 1], r[i - 2], r[i - 3]
                p = (a & b) | (a & c) | (b & c)
        else:            # Morpho-Predict PY:887-900
            if i == 0:
                p = 0
            else:
                d = r[i - 1]
                m = _ero(_dil(d)) if (param & 1) == 0 else _dil(_ero(d))
                e = _dil(d) ^ _ero(d)
                p = (m & e) | (d & ~e & 0xFF)
        r[i] = y[i] ^ p
    return bytes(r)


def _rice_runs_until(bits: np.ndarray, pos: int, k: int, target: int) -> Tuple[List[int], int]:
    """PY:1462-1487 _rice_decode_until_len over an unpacked bit array from bit `pos`."""
    runs: List[int] = []
    total = 0
    nb = bits.size
    zeros = np.flatnonzero(bits[pos:] == 0) + pos
    zi = 0
    while total < target:
        zi = int(np.searchsorted(zeros, pos, side="left"))
        if zi >= zeros.size:
            raise ValueError("BitReader: out of data")
        z = int(zeros[zi])
        q = z - pos
        pos = z + 1
        r = 0
        if k:
            if pos + k > nb:
                raise ValueError("BitReader: out of data")
            for t in range(k):
                r = (r << 1) | int(bits[pos + t])
            pos += k
        val = (q << k) | r
        if val <= 0:
            raise ValueError("Invalid Rice value (non-positive)")
        runs.append(val)
        total += val
        if total > target:
            raise ValueError("RLE overrun: sum(runs) > target_len")
    return runs, pos


def decode_new_pipeline(payload: bytes, n: int) -> bytes:  # PY:1578-1648
    if n == 0:
        return b""
    if len(payload) < 3:
        raise ValueError("V2 slim header truncated")
    h0 = payload[0]
    mode, plen = (h0 >> 5) & 7, h0 & 7
    if plen > 4:
        raise ValueError("V2 slim header invalid param_len (>4)")
    if len(payload) < 1 + plen + 2:
        raise ValueError("V2 slim header truncated (param/raw/b1)")
    param = int.from_bytes(payload[1:1 + plen], "little")
    pos = 1 + plen
    raw_mask, b1_mask = payload[pos], payload[pos + 1]
    pos += 2
    nenc = 8 - bin(raw_mask).count("1")
    if pos + nenc > len(payload):
        raise ValueError("V2 slim header k_list truncated")
    ks = list(payload[pos:pos + nenc])
    data = payload[pos + nenc:]
    bits = np.unpackbits(np.frombuffer(data, dtype=np.uint8)) if data else np.zeros(0, np.uint8)
    dpos = 0  # byte position in data
    planes = np.zeros((8, n), dtype=np.uint8)
    ki = 0
    for j in range(8):
        if (raw_mask >> j) & 1:
            need = (n + 7) // 8
            if dpos + need > len(data):
                raise ValueError("V2 payload truncated in RAW plane")
            planes[j] = np.unpackbits(np.frombuffer(data[dpos:dpos + need], dtype=np.uint8))[:n]
            dpos += need
        else:
            k = ks[ki]
            ki += 1
            runs, bitpos = _rice_runs_until(bits, 8 * dpos, k, n)
            dpos = (bitpos + 7) // 8
            b = (b1_mask >> j) & 1
            lbits = np.repeat((np.arange(len(runs)) + b) & 1, runs).astype(np.uint8)
            u = np.frombuffer(bbwt_inverse(lbits.tobytes()), dtype=np.uint8)
            planes[j, :min(n, u.size)] = u[:n]
    mapped = np.packbits(planes.T, axis=1).ravel().tobytes()
    return _v2_inverse(mapped, mode, param)


def decode_block(mid: int, payload: bytes, n: int) -> bytes:
    """Decoder registry aligned with the encoder ids (PY:2194-2207)."""
    if mid == 0:
        return decode_raw(payload, n)
    if mid == 1:
        return decode_xor(payload, n)
    if mid in BBWT_FLAGS:
        return decode_bbwt_mtf_rice(payload, n, BBWT_FLAGS[mid])
    if mid == 7:
        return decode_lz77(payload, n)
    if mid == 8:
        return decode_lfsr(payload, n)
    if mid == 9:
        return repair_decompress(payload, n)
    if mid == 10:
        return decode_new_pipeline(payload, n)
    raise ValueError(f"Unknown method_id {mid}")
