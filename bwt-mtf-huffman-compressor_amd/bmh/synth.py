"""Synthetic inputs of SURVEY.md Appendix D (integer-only, reproducible).

These generate the benchmark configs' data (BASELINE.json configs 3-5): uniform-random bytes
from splitmix64 and integer-Zipf text. Pure numpy; counter-based so any byte range of the
stream can be produced independently (used to give each rank its own blocks).
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def splitmix64_words(seed: int, start_word: int, count: int) -> np.ndarray:
    """Words z_k for k in [start_word, start_word+count) of splitmix64(seed): x_k = seed + (k+1)*GAMMA."""
    with np.errstate(over="ignore"):
        k = np.arange(start_word + 1, start_word + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z ^= z >> np.uint64(31)
    return z


def splitmix64_bytes(seed: int, offset: int, nbytes: int) -> np.ndarray:
    """Bytes [offset, offset+nbytes) of the little-endian splitmix64(seed) byte stream."""
    w0 = offset // 8
    w1 = (offset + nbytes + 7) // 8
    words = splitmix64_words(seed, w0, w1 - w0)
    b = words.astype("<u8").view(np.uint8)
    s = offset - w0 * 8
    return np.ascontiguousarray(b[s:s + nbytes])


class _Stream:
    def __init__(self, seed: int):
        self.seed = seed
        self.pos = 0

    def take(self, n: int) -> np.ndarray:
        w = splitmix64_words(self.seed, self.pos, n)
        self.pos += n
        return w


def zipf_vocab(vocab_size: int = 8192) -> list[bytes]:
    s = _Stream(1)
    words = []
    for _ in range(vocab_size):
        r = int(s.take(1)[0])
        ln = 2 + r % 9
        letters = s.take(ln) % np.uint64(26)
        words.append(bytes((97 + letters).astype(np.uint8)))
    return words


def zipf_text(nbytes: int, vocab_size: int = 8192) -> np.ndarray:
    """First nbytes of the integer-Zipf word stream (App. D): token word = first k with cdf[k] > x."""
    words = zipf_vocab(vocab_size)
    w = np.array([(1 << 32) // (k + 1) for k in range(vocab_size)], dtype=np.uint64)
    cdf = np.cumsum(w, dtype=np.uint64)
    total = cdf[-1]
    lens = np.array([len(x) + 1 for x in words], dtype=np.int64)
    blob = b"".join(x + b" " for x in words)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    flat = np.frombuffer(blob, dtype=np.uint8)
    out = np.empty(nbytes, dtype=np.uint8)
    filled = 0
    tok = _Stream(2)
    batch = max(1 << 16, nbytes // 5)
    while filled < nbytes:
        x = tok.take(batch) % total
        kk = np.searchsorted(cdf, x, side="right")
        ln = lens[kk]
        ends = np.cumsum(ln)
        need = nbytes - filled
        cut = int(np.searchsorted(ends, need, side="left")) + 1
        kk, ln = kk[:cut], ln[:cut]
        # gather the token bytes
        off = np.repeat(starts[kk] - np.concatenate([[0], np.cumsum(ln)[:-1]]), ln)
        idx = np.arange(int(ln.sum()), dtype=np.int64) + off
        chunk = flat[idx]
        m = min(need, chunk.size)
        out[filled:filled + m] = chunk[:m]
        filled += m
    return out
