"""KOLR container (host side): the header + TOC come from the native writer / reader of
libkolm_hip.so (csrc/kolm_toc.cpp: kolm_toc_write / kolm_toc_read, host code only, so
these work without a GPU); this module only moves bytes in and out of it.

Byte format (PY = kolm_final_researched_v2-2.py; details in kolm_toc.cpp's header):
  b'KOLR' | <I mode<<31 | size | <I total_len | <H nblocks          PY:2333-2339, 2128-2146
  ULEB toc_hdr_len | ULEB toc_bitlen | ULEB total_payload           PY:2436-2438
  toc_header | toc_bits (prefix-coded method-id runs, Rice run lengths, [CDC length
  deltas], Elias-Fano payload ends)                                 PY:2375-2435
  payloads back to back.
Errors as PY's: ValueError for malformed containers (PY's messages), struct.error when a
block count or length overflows its field.
"""
from __future__ import annotations

import ctypes
import struct
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib

MAGIC = b"KOLR"
MODE_FIXED = 0
MODE_CDC = 1
MAX_BLOCKS = 0xFFFF  # the '<H' block-count field


def uleb128_encode(n: int) -> bytes:
    """Unsigned LEB128 (PY:111-124): 7-bit groups, least significant first."""
    if n < 0:
        raise ValueError("ULEB128 only supports unsigned integers")
    groups = [(n >> s) & 0x7F for s in range(0, max(n.bit_length(), 1), 7)]
    return bytes(g | 0x80 for g in groups[:-1]) + bytes(groups[-1:])


def uleb128_decode_stream(data: bytes, pos: int = 0) -> Tuple[int, int]:
    """(value, position after it) of the ULEB128 number at data[pos] (PY:126-137)."""
    end = pos
    while end < len(data) and data[end] & 0x80:
        end += 1
    if end >= len(data):
        raise ValueError("Truncated ULEB128")
    value = 0
    for b in reversed(data[pos:end + 1]):
        value = (value << 7) | (b & 0x7F)
    return value, end + 1


def pack_mode_and_size(mode: int, size: int) -> int:
    """PY:2128-2141: bit 31 = mode, low 31 bits = block size / avg size."""
    if mode not in (MODE_FIXED, MODE_CDC):
        raise ValueError("invalid mode")
    if not 0 <= size <= 0x7FFFFFFF:
        raise ValueError("size out of range (must fit in 31 bits)")
    return (mode << 31) | size


def _raise(rc: int):
    msg = _lib.load().kolm_last_error()
    text = msg.decode() if msg else f"kolm error {rc}"
    if rc == _lib.KOLM_ERANGE:
        raise struct.error(text)
    if rc == _lib.KOLM_EFORMAT:
        raise ValueError(text)
    raise _lib.KolmError(rc, text)


def write_container(mode: int, size_field: int, total_len: int, method_ids: Sequence[int],
                    orig_lens: Sequence[int], payloads: Sequence[bytes]) -> bytes:
    """Assemble a KOLR container (PY:2213-2326 CDC, PY:2332-2445 FIXED)."""
    pack_mode_and_size(mode, size_field)
    nb = len(method_ids)
    if nb > MAX_BLOCKS:
        raise struct.error("'H' format requires 0 <= number <= 65535")
    if not 0 <= total_len <= 0xFFFFFFFF:
        raise struct.error("'I' format requires 0 <= number <= 4294967295")
    mids = np.ascontiguousarray(np.asarray(method_ids, dtype=np.uint32).reshape(-1))
    lens = np.ascontiguousarray(np.asarray(orig_lens, dtype=np.uint32).reshape(-1))
    plen = np.fromiter((len(p) for p in payloads), dtype=np.uint64, count=len(payloads))
    if not (len(mids) == len(lens) == len(plen) == nb):
        raise ValueError("method_ids, orig_lens and payloads must have one entry per block")
    L = _lib.load()
    n = ctypes.c_uint64(0)
    args = (mode, size_field, total_len, nb, mids.ctypes.data, lens.ctypes.data, plen.ctypes.data)
    rc = L.kolm_toc_write(*args, None, 0, ctypes.byref(n))
    if rc:
        _raise(rc)
    head = ctypes.create_string_buffer(max(n.value, 1))
    rc = L.kolm_toc_write(*args, head, n.value, ctypes.byref(n))
    if rc:
        _raise(rc)
    return b"".join([head.raw[:n.value], *payloads])


def read_toc(container: bytes):
    """Header + TOC of a container: (mode, size_field, total_len, method_ids u32[nb],
    orig_lens u32[nb], payload_off u64[nb + 1] relative to the payload area,
    payload_start)."""
    L = _lib.load()
    fields = np.zeros(4, np.uint32)
    start = ctypes.c_uint64(0)
    mids = np.zeros(MAX_BLOCKS, np.uint32)
    lens = np.zeros(MAX_BLOCKS, np.uint32)
    off = np.zeros(MAX_BLOCKS + 1, np.uint64)
    rc = L.kolm_toc_read(container, len(container), fields.ctypes.data, ctypes.byref(start), mids.ctypes.data,
                         lens.ctypes.data, off.ctypes.data, MAX_BLOCKS)
    if rc:
        _raise(rc)
    mode, size_field, total_len, nb = (int(x) for x in fields)
    return mode, size_field, total_len, mids[:nb], lens[:nb], off[:nb + 1], int(start.value)


def read_container(container: bytes):
    """Parse a KOLR container (PY:2451-2524).  Returns (mode, size_field, total_len,
    method_ids, orig_lens, payload_bytes_list)."""
    container = bytes(container)
    mode, size_field, total_len, mids, lens, off, start = read_toc(container)
    area = memoryview(container)[start:]
    payloads: List[bytes] = [bytes(area[int(a):int(b)]) for a, b in zip(off[:-1], off[1:])]
    return mode, size_field, total_len, mids.tolist(), lens.tolist(), payloads
