"""Synthetic corpus / query generator.

Pure-Python statement of the generator used by the fixtures and the CPU tests. The
bench uses the byte-identical C implementation in ``csrc/synth.c`` (10M rows in Python
would take minutes); ``tests/test_synth.py`` checks the two agree.

Stream: splitmix64, seed 42. Alphabet ``A`` (37 symbols, space included). Per word,
draws in this order: ``L = min_len + r % span``; ``L`` chars ``A[r % 37]``;
``w[0] = A[r % 26]``; ``w[L-1] = A[r % 26]``; ``weight = 0.5f + (float)(r >> 40) / 2^24``
(always drawn). A row is ``row_size`` consecutive words (the first is the key, the rest
aliases). After all rows, per query: ``row = r % rows``; the row's key is the source;
``l = min(qlen, len)``; ``o = r % (len - l + 1)``; ``q = key[o:o+l]``;
``p = r % l``; ``q[p] = A[r % 26]`` (one substitution; 4 draws per query).
"""
from __future__ import annotations

import struct

ALPHABET = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 "
MASK64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int = 42):
        self.s = seed & MASK64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)


def _f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def weight_from_draw(r: int) -> float:
    # 0.5f + (float)(r >> 40) / 2^24, evaluated in fp32 like the C generator
    hi = _f32(float(r >> 40))
    return _f32(0.5 + _f32(hi / 16777216.0))


def gen_corpus(rows: int, seed: int = 42, min_len: int = 8, span: int = 17, row_size: int = 1,
               rng: SplitMix64 | None = None):
    """Returns (words: list[bytes], weights: list[float], rng) with len(words) == rows*row_size."""
    rng = rng or SplitMix64(seed)
    words, weights = [], []
    for _ in range(rows * row_size):
        L = min_len + rng.next() % span
        w = bytearray(ALPHABET[rng.next() % 37] for _ in range(L))
        w[0] = ALPHABET[rng.next() % 26]
        w[L - 1] = ALPHABET[rng.next() % 26]
        words.append(bytes(w))
        weights.append(weight_from_draw(rng.next()))
    return words, weights, rng


def gen_queries(words, row_size: int, nq: int, rng: SplitMix64, qlen: int = 12):
    keys = words[::row_size]
    out = []
    for _ in range(nq):
        src = keys[rng.next() % len(keys)]
        l = min(qlen, len(src))
        o = rng.next() % (len(src) - l + 1)
        q = bytearray(src[o:o + l])
        p = rng.next() % l
        q[p] = ALPHABET[rng.next() % 26]
        out.append(bytes(q))
    return out
