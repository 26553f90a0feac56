"""Deterministic input generators for the benchmark/parity configurations.

Two families:

* ``pattern_blocks()``, ``gradient_bmp()``, ``checker_bmp()``, ``sine_wav()`` regenerate
  the four files of the reference's ``test_binary_files/`` byte-for-byte from closed
  formulas (the sha256 of each output is pinned in
  ``REFERENCE_SHA256`` and checked by ``tests/test_datagen.py``).  Nothing at run time
  reads ``/root/reference``.
* ``enwik_like(nbytes, seed)`` is this build's own synthetic "enwik-style" text
  generator for configs 3/4: a 5000-word vocabulary built from 30
  English syllables (1-4 per word), Zipf(1) word sampling, sentences of 5-25 words,
  3 % of words replaced by ``[[a|b]]`` links and 5 % of sentences preceded by a
  ``<page><title>..</title><id>..</id></page>`` record.  It is vectorised with numpy
  (256 MiB in a few seconds) and fully determined by ``seed``.
"""
from __future__ import annotations

import hashlib
import math
import struct

import numpy as np

REFERENCE_SHA256 = {
    "example_pattern_blocks.bin": "368f2b15db06185c9305e4558ae183555261c19eea8a9088a407f287a6f96225",
    "example_gradient_1024x768.bmp": "1a88d0eb78f836dd0498a36b97b5b7a93f9a7f4f1744a9c5f9e9b4150439a561",
    "example_checker_640x480.bmp": "3acaccaee5c795d967ade9986a71fdefaa08ec3a5a99588c6916a18e748c364c",
    "example_sine_44k_3s.wav": "e46d948d8511890025773aaebc1d93e2a27cf1f62aa329afd2aa8118aae77cdf",
}

ENWIK_SEED = 20251212
RANDOM_SEED = 0x9E3779B97F4A7C15


def sha256(data: bytes) -> str:
    return hashlib.sha256(data).hexdigest()


# ---------------------------------------------------------------------------
# test_binary_files/ regenerators
# ---------------------------------------------------------------------------

def pattern_blocks() -> bytes:
    """16 x 64 KiB: zeros, 0xFF, 4 x ramp, 4 x Fibonacci mod 256, 6 x records."""
    blk = 65536
    parts = [bytes(blk), b"\xff" * blk]
    parts.append((np.arange(4 * blk, dtype=np.uint32) & 0xFF).astype(np.uint8).tobytes())
    fib = np.empty(4 * blk, dtype=np.uint8)
    a, b = 1, 1
    for i in range(4 * blk):
        fib[i] = a
        a, b = b, (a + b) & 0xFF
    parts.append(fib.tobytes())
    rec = bytearray()
    for i in range(4000):
        L = 32 + (7 * i) % 97
        rec += struct.pack("<IH", i, L) + bytes([i % 13]) * L
    rec += b"\xab" * (6 * blk - len(rec))
    parts.append(bytes(rec))
    return b"".join(parts)


def _bmp(width: int, height: int, pixel_rows) -> bytes:
    row_bytes = width * 3
    pad = (4 - row_bytes % 4) % 4
    body = bytearray()
    for y in range(height - 1, -1, -1):  # bottom-up
        body += pixel_rows(y)
        body += b"\x00" * pad
    hdr = struct.pack("<2sIHHI", b"BM", 54 + len(body), 0, 0, 54)
    info = struct.pack("<IiiHHIIiiII", 40, width, height, 1, 24, 0, len(body), 2835, 2835, 0, 0)
    return hdr + info + bytes(body)


def gradient_bmp() -> bytes:
    w, h = 1024, 768
    x = np.arange(w, dtype=np.int64)

    def row(y):
        px = np.empty((w, 3), dtype=np.uint8)
        px[:, 0] = (x ^ y) & 0xFF
        px[:, 1] = y * 255 // 767
        px[:, 2] = x * 255 // 1023
        return px.tobytes()

    return _bmp(w, h, row)


def checker_bmp() -> bytes:
    w, h = 640, 480
    x = np.arange(w, dtype=np.int64)

    def row(y):
        g = np.where(((x // 16) + (y // 16)) % 2 == 0, 240, 40).astype(np.uint8)
        return np.repeat(g, 3).tobytes()

    return _bmp(w, h, row)


def sine_wav() -> bytes:
    n = 132300
    samples = bytearray()
    for i in range(n):
        samples += struct.pack("<h", int(32767 * math.sin(2 * math.pi * 440 * i / 44100)))
    fmt = struct.pack("<4sIHHIIHH", b"fmt ", 16, 1, 1, 44100, 88200, 2, 16)
    data = struct.pack("<4sI", b"data", len(samples)) + bytes(samples)
    return struct.pack("<4sI4s", b"RIFF", 4 + len(fmt) + len(data), b"WAVE") + fmt + data


REFERENCE_FILES = {
    "example_pattern_blocks.bin": pattern_blocks,
    "example_gradient_1024x768.bmp": gradient_bmp,
    "example_checker_640x480.bmp": checker_bmp,
    "example_sine_44k_3s.wav": sine_wav,
}


# ---------------------------------------------------------------------------
# Other synthetic inputs
# ---------------------------------------------------------------------------

def splitmix64_bytes(nbytes: int, seed: int = RANDOM_SEED) -> bytes:
    """Random bytes from splitmix64 (little-endian 8-byte words), vectorised."""
    nwords = (nbytes + 7) // 8
    m = np.uint64(0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        idx = np.arange(1, nwords + 1, dtype=np.uint64)
        z = (np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)) & m
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:nbytes]


_SYLLABLES = [
    "th", "er", "on", "an", "re", "he", "in", "ed", "nd", "ha",
    "at", "en", "es", "of", "or", "nt", "ea", "ti", "to", "it",
    "st", "io", "le", "is", "ou", "ar", "as", "de", "rt", "ve",
]


def _enwik_tables(rng: np.random.Generator):
    nvocab = 5000
    words = []
    seen = set()
    while len(words) < nvocab:
        k = int(rng.integers(1, 5))
        w = "".join(_SYLLABLES[int(i)] for i in rng.integers(0, len(_SYLLABLES), k))
        if w in seen:
            continue
        seen.add(w)
        words.append(w)
    # capitalised variants for sentence starts / titles
    ranks = np.arange(1, nvocab + 1, dtype=np.float64)
    p = 1.0 / ranks
    p /= p.sum()
    return words, p


def enwik_like(nbytes: int, seed: int = ENWIK_SEED) -> bytes:
    """Deterministic enwik-style text of exactly ``nbytes`` bytes (see module doc)."""
    if nbytes <= 0:
        return b""
    rng = np.random.default_rng(seed)
    words, p = _enwik_tables(rng)
    nv = len(words)
    # token table: 0..nv-1 "word ", nv..2nv-1 "Word " (sentence start),
    # then links, then xml records, then punctuation.
    tokens = [w + " " for w in words] + [w.capitalize() + " " for w in words]
    nlinks = 4000
    la = rng.choice(nv, nlinks, p=p)
    lb = rng.choice(nv, nlinks, p=p)
    link_base = len(tokens)
    tokens += [f"[[{words[a].capitalize()} {words[b]}|{words[b]}]] " for a, b in zip(la, lb)]
    nrec = 20000
    ta = rng.choice(nv, nrec, p=p)
    tb = rng.choice(nv, nrec, p=p)
    rec_base = len(tokens)
    tokens += [
        f"\n<page>\n  <title>{words[a].capitalize()} {words[b].capitalize()}</title>\n"
        f"  <id>{1000 + 37 * i}</id>\n  <revision>\n    <text>"
        for i, (a, b) in enumerate(zip(ta, tb))
    ]
    punct_base = len(tokens)
    tokens += [". ", ".\n", ", ", "; ", "</text>\n  </revision>\n</page>\n"]
    tok_bytes = [t.encode("ascii") for t in tokens]
    tok_len = np.array([len(t) for t in tok_bytes], dtype=np.int64)
    tok_off = np.concatenate([[0], np.cumsum(tok_len)[:-1]])
    table = np.frombuffer(b"".join(tok_bytes), dtype=np.uint8)

    out_parts = []
    produced = 0
    while produced < nbytes:
        # one chunk of sentences (~ 4 MiB of text)
        nsent = 60000
        slen = rng.integers(5, 26, nsent)
        nw = int(slen.sum())
        wid = rng.choice(nv, nw, p=p).astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(slen)[:-1]])
        wid[starts] += nv  # capitalised sentence start
        link_mask = rng.random(nw) < 0.03
        wid[link_mask] = link_base + rng.integers(0, nlinks, int(link_mask.sum()))
        # sentence terminators
        term = punct_base + rng.choice(4, nsent, p=[0.55, 0.25, 0.12, 0.08])
        # xml records before 5 % of sentences (closing tag after the sentence)
        rec_mask = rng.random(nsent) < 0.05
        # assemble: per sentence [rec?] words... term [close?]
        counts = slen + 1 + 2 * rec_mask.astype(np.int64)
        total = int(counts.sum())
        seq = np.empty(total, dtype=np.int64)
        sent_off = np.concatenate([[0], np.cumsum(counts)[:-1]])
        word_sent = np.repeat(np.arange(nsent), slen)
        word_rank = np.arange(nw) - np.repeat(starts, slen)
        seq[sent_off[word_sent] + rec_mask[word_sent] + word_rank] = wid
        seq[sent_off + rec_mask + slen] = term
        rs = np.nonzero(rec_mask)[0]
        seq[sent_off[rs]] = rec_base + rng.integers(0, nrec, rs.size)
        seq[sent_off[rs] + slen[rs] + 2] = punct_base + 4
        lens = tok_len[seq]
        ends = np.cumsum(lens)
        nb = int(ends[-1])
        src = np.repeat(tok_off[seq] - (ends - lens), lens) + np.arange(nb)
        out_parts.append(table[src])
        produced += nb
    return np.concatenate(out_parts)[:nbytes].tobytes()


def mixed_corpus() -> bytes:
    """Config 5: sine WAV || checker BMP || 1 MiB splitmix64 random bytes."""
    return sine_wav() + checker_bmp() + splitmix64_bytes(1 << 20)
