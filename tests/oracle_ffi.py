"""ctypes access to oracle/liboracle.so — the TEST-ONLY C restatement of the reference.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")
GOLDEN = os.path.join(REPO, "tests", "golden")
CALGARY = ["bib", "book1", "book2", "geo", "news", "obj1", "obj2", "paper1", "paper2",
           "pic", "progc", "progl", "progp", "trans"]


def ensure_built() -> None:
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", ORACLE_DIR, "liboracle.so"], check=True, capture_output=True)


class Oracle:
    def __init__(self):
        ensure_built()
        L = C.CDLL(LIB)
        u8p = C.c_void_p
        L.orc_bwt_ref.argtypes = [u8p, C.c_size_t, u8p, C.POINTER(C.c_uint64)]
        L.orc_bwt_fast.argtypes = [u8p, C.c_size_t, u8p, C.POINTER(C.c_uint64)]
        L.orc_mtf.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_mtf_inverse.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_bwt_inverse.argtypes = [u8p, C.c_size_t, C.c_uint64, u8p]
        L.orc_histogram.argtypes = [u8p, C.c_size_t, u8p, u8p]
        L.orc_encode_record.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.c_int]
        L.orc_encode_record.restype = C.c_int64
        L.orc_record_bound.argtypes = [C.c_size_t]
        L.orc_record_bound.restype = C.c_size_t
        L.orc_decode_record.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t]
        L.orc_decode_record.restype = C.c_int64
        L.orc_decode_to_mtf.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t]
        L.orc_decode_to_mtf.restype = C.c_int64
        L.orc_huffman_build.argtypes = [u8p, u8p, u8p, u8p, u8p, C.c_size_t]
        L.orc_huffman_build.restype = C.c_int
        L.orc_zipf_state_size.restype = C.c_size_t
        L.orc_zipf_init.argtypes = [u8p]
        L.orc_zipf_fill.argtypes = [u8p, u8p, C.c_size_t]
        self.L = L

    @staticmethod
    def _a(x) -> np.ndarray:
        if isinstance(x, np.ndarray):
            return np.ascontiguousarray(x, dtype=np.uint8).reshape(-1)
        return np.frombuffer(bytes(x), dtype=np.uint8).copy()

    def bwt(self, data, faithful: bool = False) -> tuple[int, bytes]:
        a = self._a(data)
        out = np.empty(a.size, np.uint8)
        p = C.c_uint64()
        f = self.L.orc_bwt_ref if faithful else self.L.orc_bwt_fast
        if f(a.ctypes.data, a.size, out.ctypes.data, C.byref(p)) != 0:
            raise ValueError("oracle bwt failed")
        return p.value, out.tobytes()

    def mtf(self, data) -> bytes:
        a = self._a(data)
        out = np.empty(a.size, np.uint8)
        self.L.orc_mtf(a.ctypes.data, a.size, out.ctypes.data)
        return out.tobytes()

    def mtf_inverse(self, data) -> bytes:
        a = self._a(data)
        out = np.empty(a.size, np.uint8)
        self.L.orc_mtf_inverse(a.ctypes.data, a.size, out.ctypes.data)
        return out.tobytes()

    def histogram(self, data):
        a = self._a(data)
        freq = np.zeros(256, np.uint64)
        first = np.zeros(256, np.uint64)
        self.L.orc_histogram(a.ctypes.data, a.size, freq.ctypes.data, first.ctypes.data)
        return freq, first

    def huffman_build(self, freq, first):
        """Code lengths, codes and tree bytes of the reference's tree (main.cpp:245-254)."""
        f = np.ascontiguousarray(freq, dtype=np.uint64)
        fi = np.ascontiguousarray(first, dtype=np.uint64)
        ln = np.zeros(256, np.uint8)
        code = np.zeros(256, np.uint64)
        tree = np.zeros(320, np.uint8)
        r = self.L.orc_huffman_build(f.ctypes.data, fi.ctypes.data, ln.ctypes.data, code.ctypes.data,
                                     tree.ctypes.data, tree.size)
        if r < 0:
            raise ValueError("oracle huffman_build failed")
        return ln, code, tree[:r].tobytes()

    def encode(self, data, faithful: bool = False) -> bytes:
        a = self._a(data)
        cap = self.L.orc_record_bound(a.size)
        out = np.empty(cap, np.uint8)
        r = self.L.orc_encode_record(a.ctypes.data, a.size, out.ctypes.data, cap, 1 if faithful else 0)
        if r < 0:
            raise ValueError("oracle encode failed")
        return out[:r].tobytes()

    def decode(self, rec) -> bytes:
        a = self._a(rec)
        n = int.from_bytes(a[8:16].tobytes(), "little")
        out = np.empty(max(n, 1), np.uint8)
        r = self.L.orc_decode_record(a.ctypes.data, a.size, out.ctypes.data, n)
        if r < 0:
            raise ValueError("oracle decode failed")
        return out[:r].tobytes()

    def decode_to_mtf(self, rec) -> bytes:
        a = self._a(rec)
        n = int.from_bytes(a[8:16].tobytes(), "little")
        out = np.empty(max(n, 1), np.uint8)
        r = self.L.orc_decode_to_mtf(a.ctypes.data, a.size, out.ctypes.data, n)
        if r < 0:
            raise ValueError("oracle decode failed")
        return out[:r].tobytes()


class ZipfStream:
    """SURVEY App. D Zipf text, read sequentially from the oracle's C generator."""

    def __init__(self, oracle: "Oracle"):
        self.L = oracle.L
        self.st = C.create_string_buffer(self.L.orc_zipf_state_size())
        self.L.orc_zipf_init(C.addressof(self.st))

    def read(self, n: int) -> np.ndarray:
        out = np.empty(n, np.uint8)
        self.L.orc_zipf_fill(C.addressof(self.st), out.ctypes.data, n)
        return out


def golden_calgary():
    for fn in CALGARY:
        with open(os.path.join(GOLDEN, "calgary", fn), "rb") as f:
            data = f.read()
        with open(os.path.join(GOLDEN, "calgary_records", fn + ".bzap"), "rb") as f:
            rec = f.read()
        yield fn, data, rec


def golden_small():
    d = os.path.join(GOLDEN, "small")
    for fn in sorted(os.listdir(d)):
        if fn.endswith(".bzap"):
            continue
        with open(os.path.join(d, fn), "rb") as f:
            data = f.read()
        with open(os.path.join(d, fn + ".bzap"), "rb") as f:
            rec = f.read()
        yield fn, data, rec


def manifest(name: str) -> dict:
    import json
    with open(os.path.join(GOLDEN, "manifests", name + ".json")) as f:
        return json.load(f)
