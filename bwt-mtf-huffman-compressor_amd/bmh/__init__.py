"""bmh — Python binding of libbmh (MI355X BWT -> MTF -> Huffman block encoder).

Mirrors the reference's stage functions (komour/bwt-mtf-huffman-compressor main.cpp) with
the same names and argument meaning, running on the GPU through the C ABI in include/bmh.h:

    bwt(data)             -> (primary, L)         main.cpp:77-91
    move_to_front(L)      -> mtf                  main.cpp:93-112
    huffman(mtf)          -> (payload, table)     main.cpp:229-257
    tree_to_bytes(table)  -> tree bytes           main.cpp:189-196
    compress(in, out)     prints the reference metrics line, writes the record  main.cpp:300-325
    decompress(in, out)                                                          main.cpp:327-345

There is no CPU fallback: if libbmh.so or a gfx950 device is missing, calls raise BmhError.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("BMH_LIB") or os.path.join(PKG_ROOT, "lib", "libbmh.so")
CLI_PATH = os.path.join(PKG_ROOT, "bin", "bmh")

BMH_OK, BMH_EINVAL, BMH_ENOMEM, BMH_EHIP, BMH_ERANGE, BMH_ECORRUPT, BMH_ENODEV = range(7)


class BmhError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{msg} [status {status}]")
        self.status = status


class CodeTable(C.Structure):
    """bmh_code_table: per-block Huffman code words, lengths and preorder tree bytes."""
    _fields_ = [("code", C.c_uint64 * 256), ("len", C.c_uint8 * 256), ("tree", C.c_uint8 * 320),
                ("tree_len", C.c_uint32), ("leaves", C.c_uint32)]

    @property
    def tree_bytes(self) -> bytes:
        return bytes(self.tree[: self.tree_len])


_lib = None

P = C.c_void_p
U64 = C.c_uint64
U32 = C.c_uint32
PU64 = C.POINTER(C.c_uint64)

_SIGS = {
    "bmh_version": (C.c_char_p, []),
    "bmh_status_str": (C.c_char_p, [C.c_int]),
    "bmh_last_error": (C.c_char_p, []),
    "bmh_device_count": (C.c_int, []),
    "bmh_ctx_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "bmh_ctx_destroy": (None, [P]),
    "bmh_ctx_stream": (P, [P]),
    "bmh_dev_alloc": (C.c_int, [P, U64, C.POINTER(P)]),
    "bmh_dev_free": (C.c_int, [P, P]),
    "bmh_host_alloc": (C.c_int, [P, U64, C.POINTER(P)]),
    "bmh_host_free": (C.c_int, [P, P]),
    "bmh_memcpy_h2d": (C.c_int, [P, P, P, U64]),
    "bmh_memcpy_d2h": (C.c_int, [P, P, P, U64]),
    "bmh_bwt_dev": (C.c_int, [P, P, PU64, U32, P, PU64]),
    "bmh_mtf_dev": (C.c_int, [P, P, PU64, U32, P, PU64, PU64]),
    "bmh_histogram_dev": (C.c_int, [P, P, PU64, U32, PU64, PU64]),
    "bmh_huffman_build": (C.c_int, [PU64, PU64, C.POINTER(CodeTable)]),
    "bmh_huffman_build_sized": (C.c_int, [PU64, PU64, U64, C.POINTER(CodeTable)]),
    "bmh_node_ranks": (C.c_int, [U64, U32, C.POINTER(C.c_uint16)]),
    "bmh_payload_bytes": (U64, [C.POINTER(CodeTable), PU64]),
    "bmh_pack_dev": (C.c_int, [P, P, PU64, U32, C.POINTER(CodeTable), P, U64, PU64, PU64]),
    "bmh_encode_blocks_dev": (C.c_int, [P, P, PU64, U32, P, U64, PU64]),
    "bmh_record_bound": (U64, [U64]),
    "bmh_encode_pipelines": (U32, [P, U64, U32]),
    "bmh_ctx_last_pipelines": (U32, [P]),
    "bmh_ctx_spec_fallbacks": (U32, [P]),
    "bmh_compress_host": (C.c_int, [P, P, U64, U64, P, U64, PU64]),
    "bmh_compress_host_multi": (C.c_int, [C.POINTER(P), U32, P, U64, U64, P, U64, PU64]),
    "bmh_compress_bound": (U64, [U64, U64]),
    "bmh_host_cpus": (U32, []),
    "bmh_copy_threads": (U32, [U32, U32]),
    "bmh_decompress_host": (C.c_int, [P, U64, P, U64, PU64]),
    "bmh_record_to_mtf": (C.c_int, [P, U64, P, U64, PU64]),
    "bmh_decode_blocks_dev": (C.c_int, [P, P, PU64, U32, P, U64, PU64]),
    "bmh_decompress_dev": (C.c_int, [P, P, U64, P, U64, PU64]),
    "bmh_is_container": (C.c_int, [P, U64]),
    "bmh_container_info": (C.c_int, [P, U64, PU64, PU64]),
    "bmh_container_record": (C.c_int, [P, U64, U64, C.POINTER(P), PU64]),
    "bmh_ctx_set_timing": (C.c_int, [P, C.c_int]),
    "bmh_ctx_set_option": (C.c_int, [P, U32, U64]),
    "bmh_ctx_reset_stats": (C.c_int, [P]),
    "bmh_ctx_kernel_stats": (C.c_int, [P, P, PU64, C.POINTER(C.c_double), C.c_int]),
    "bmh_synth_splitmix64_dev": (C.c_int, [P, P, U64, U64, U64]),
    "bmh_synth_zipf_dev": (C.c_int, [P, P, U64, U64]),
    "bmh_check_violations": (C.c_int64, [P, U32]),
}


def lib() -> C.CDLL:
    """Load libbmh.so (built in-tree by `make -C bwt-mtf-huffman-compressor_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BmhError(BMH_ENODEV, f"libbmh.so not built at {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            try:
                f = getattr(L, name)
            except AttributeError:  # an older library under BMH_LIB (A/B runs); the export test checks ours
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(st: int, what: str) -> None:
    if st != BMH_OK:
        L = lib()
        raise BmhError(st, f"{what}: {L.bmh_status_str(st).decode()} ({L.bmh_last_error().decode()})")


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(PU64)


def as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


class DevBuf:
    """A device allocation owned by a Context."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = C.c_void_p()
        _check(lib().bmh_dev_alloc(ctx.h, max(1, self.nbytes), C.byref(p)), "dev_alloc")
        self.ptr = p

    def upload(self, host: np.ndarray, offset: int = 0) -> None:
        host = as_u8(host)
        _check(lib().bmh_memcpy_h2d(self.ctx.h, C.c_void_p(self.ptr.value + offset), _ptr(host), host.nbytes), "h2d")

    def download(self, nbytes: int | None = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(n, dtype=np.uint8)
        _check(lib().bmh_memcpy_d2h(self.ctx.h, _ptr(out), C.c_void_p(self.ptr.value + offset), n), "d2h")
        return out

    def free(self) -> None:
        if self.ptr:
            lib().bmh_dev_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if getattr(self, "ptr", None) and self.ctx.h:
                self.free()
        except Exception:
            pass


class _PinnedBlock:
    """One bmh_host_alloc block. It is the base object of every numpy view of it, so the block
    is released only when the HostBuf and the last view (hout.a[:n], slices kept by callers)
    are gone: a view can never read freed pinned memory."""

    def __init__(self, ctx: "Context", nbytes: int):
        p = C.c_void_p()
        _check(lib().bmh_host_alloc(ctx.h, max(1, nbytes), C.byref(p)), "host_alloc")
        self.ptr = p

    def __del__(self):
        try:
            if self.ptr:
                lib().bmh_host_free(None, self.ptr)  # no context needed (include/bmh.h)
                self.ptr = None
        except Exception:
            pass


class HostBuf:
    """Page-locked host memory (bmh_host_alloc) viewed as a numpy uint8 array (`.a`).
    free() drops this object's hold; the memory itself goes when no view of it is left."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        blk = _PinnedBlock(ctx, self.nbytes)
        arr = (C.c_uint8 * max(1, self.nbytes)).from_address(blk.ptr.value)
        arr._owner = blk  # numpy views keep arr alive, arr keeps the block
        self.ptr = blk.ptr
        self.a = np.frombuffer(arr, dtype=np.uint8)[: self.nbytes]

    def free(self) -> None:
        self.a = None
        self.ptr = None
class Context:
    """One GPU (bmh_ctx). Not thread-safe; use one per device/thread."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(lib().bmh_ctx_create(device, C.byref(h)), f"ctx_create(device {device})")
        self.h = h
        self.device = device

    def close(self) -> None:
        if self.h:
            lib().bmh_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def alloc(self, nbytes: int) -> DevBuf:
        return DevBuf(self, nbytes)

    def alloc_host(self, nbytes: int) -> HostBuf:
        return HostBuf(self, nbytes)

    def compress_into(self, src: np.ndarray, block_size: int, out: np.ndarray) -> int:
        """bmh_compress_host from `src` into `out` (numpy uint8 views, e.g. HostBuf.a for the
        DMA-only path); returns the output length."""
        n = C.c_uint64()
        _check(lib().bmh_compress_host(self.h, _ptr(src), src.size, block_size, _ptr(out), out.size, C.byref(n)),
               "compress_host")
        return n.value

    def pipelines(self, total: int, nblocks: int) -> int:
        """Pipelines (streams) the library's rule gives a device batch of this shape (before the
        data probe: see last_pipelines)."""
        return int(lib().bmh_encode_pipelines(self.h, total, nblocks))

    def last_pipelines(self) -> int:
        """Pipelines the last encode_blocks_dev call ran on."""
        return int(lib().bmh_ctx_last_pipelines(self.h))

    def spec_fallbacks(self) -> int:
        """Batches re-encoded after their speculative list round left work (bmh.h)."""
        return int(lib().bmh_ctx_spec_fallbacks(self.h))

    # ---- tuning options (include/bmh.h BMH_OPT_*; 0 restores the library's rule)
    OPTIONS = {"pipelines": 1, "stream_batch": 2, "max_batch": 3, "mtf_chunk": 4, "check_lists": 5, "one_pipeline": 6,
               "copy_threads": 7}

    def set_option(self, name: str, value: int) -> None:
        _check(lib().bmh_ctx_set_option(self.h, self.OPTIONS[name], int(value)), f"set_option({name})")

    def set_options(self, spec: str) -> None:
        """Options from a "name=value,name=value" string (experiment tools pass theirs this way;
        the library itself reads no environment)."""
        for item in filter(None, (x.strip() for x in (spec or "").split(","))):
            k, v = item.split("=", 1)
            self.set_option(k.strip(), int(v))

    # ---- measurement
    def set_timing(self, on: bool) -> None:
        _check(lib().bmh_ctx_set_timing(self.h, 1 if on else 0), "set_timing")

    def reset_stats(self) -> None:
        _check(lib().bmh_ctx_reset_stats(self.h), "reset_stats")

    def kernel_stats(self) -> dict[str, tuple[int, float]]:
        cap = 128
        names = (C.c_char * 64 * cap)()
        la = (C.c_uint64 * cap)()
        ms = (C.c_double * cap)()
        n = lib().bmh_ctx_kernel_stats(self.h, C.cast(names, C.c_void_p), la, ms, cap)
        return {bytes(names[i]).split(b"\0")[0].decode(): (int(la[i]), float(ms[i])) for i in range(min(n, cap))}

    # ---- device-buffer stage calls (batched)
    def bwt_dev(self, d_in, offs: np.ndarray, d_L) -> np.ndarray:
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        prim = np.zeros(len(offs) - 1, dtype=np.uint64)
        _check(lib().bmh_bwt_dev(self.h, _dp(d_in), _u64p(offs), len(offs) - 1, _dp(d_L), _u64p(prim)), "bwt")
        return prim

    def mtf_dev(self, d_L, offs: np.ndarray, d_mtf):
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        nb = len(offs) - 1
        freq = np.zeros(nb * 256, dtype=np.uint64)
        first = np.zeros(nb * 256, dtype=np.uint64)
        _check(lib().bmh_mtf_dev(self.h, _dp(d_L), _u64p(offs), nb, _dp(d_mtf), _u64p(freq), _u64p(first)), "mtf")
        return freq.reshape(nb, 256), first.reshape(nb, 256)

    def histogram_dev(self, d_in, offs: np.ndarray):
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        nb = len(offs) - 1
        freq = np.zeros(nb * 256, dtype=np.uint64)
        first = np.zeros(nb * 256, dtype=np.uint64)
        _check(lib().bmh_histogram_dev(self.h, _dp(d_in), _u64p(offs), nb, _u64p(freq), _u64p(first)), "histogram")
        return freq.reshape(nb, 256), first.reshape(nb, 256)

    def encode_blocks_dev(self, d_in, offs: np.ndarray, d_out, out_cap: int) -> np.ndarray:
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        ro = np.zeros(len(offs), dtype=np.uint64)
        _check(lib().bmh_encode_blocks_dev(self.h, _dp(d_in), _u64p(offs), len(offs) - 1, _dp(d_out), out_cap,
                                           _u64p(ro)), "encode_blocks")
        return ro

    def decode_blocks_dev(self, d_rec, rec_offs: np.ndarray, d_out, out_cap: int) -> np.ndarray:
        """GPU decode of records in device memory; returns the output offsets (nblocks+1)."""
        rec_offs = np.ascontiguousarray(rec_offs, dtype=np.uint64)
        oo = np.zeros(len(rec_offs), dtype=np.uint64)
        _check(lib().bmh_decode_blocks_dev(self.h, _dp(d_rec), _u64p(rec_offs), len(rec_offs) - 1, _dp(d_out),
                                           out_cap, _u64p(oo)), "decode_blocks")
        return oo

    def decompress_bytes(self, data) -> bytes:
        """decompress() (main.cpp:327-345) of a record or container, decoded on this GPU."""
        a = as_u8(data)
        n = C.c_uint64()
        _check(lib().bmh_decompress_dev(self.h, _ptr(a), a.size, None, 0, C.byref(n)), "decompress_dev(size)")
        out = np.empty(max(n.value, 1), dtype=np.uint8)
        _check(lib().bmh_decompress_dev(self.h, _ptr(a), a.size, _ptr(out), n.value, C.byref(n)), "decompress_dev")
        return out[: n.value].tobytes()

    def synth_splitmix64(self, d_out, nbytes: int, seed: int = 0, offset: int = 0) -> None:
        _check(lib().bmh_synth_splitmix64_dev(self.h, _dp(d_out), nbytes, seed, offset), "synth")

    def synth_zipf(self, d_out, nbytes: int, offset: int = 0) -> None:
        """Bytes [offset, offset + nbytes) of the App. D Zipf text stream, generated in HBM."""
        _check(lib().bmh_synth_zipf_dev(self.h, _dp(d_out), nbytes, offset), "synth")

    # ---- host convenience
    def encode_blocks(self, blocks: Sequence) -> list[bytes]:
        """Encode independent blocks (host bytes) -> one reference record each."""
        arrs = [as_u8(b) for b in blocks]
        offs = np.zeros(len(arrs) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([a.size for a in arrs])
        total = int(offs[-1])
        cap = sum(int(lib().bmh_record_bound(a.size)) for a in arrs)
        d_in, d_out = self.alloc(total), self.alloc(cap)
        try:
            d_in.upload(np.concatenate(arrs) if arrs else np.zeros(0, np.uint8))
            ro = self.encode_blocks_dev(d_in, offs, d_out, cap)
            raw = d_out.download(int(ro[-1]))
        finally:
            d_in.free()
            d_out.free()
        return [raw[int(ro[i]):int(ro[i + 1])].tobytes() for i in range(len(arrs))]

    def compress_bytes(self, data, block_size: int = 0) -> bytes:
        a = as_u8(data)
        cap = int(lib().bmh_compress_bound(a.size, block_size))
        out = np.empty(max(cap, 1), dtype=np.uint8)
        olen = C.c_uint64()
        _check(lib().bmh_compress_host(self.h, _ptr(a), a.size, block_size, _ptr(out), cap, C.byref(olen)),
               "compress")
        return out[: olen.value].tobytes()


def _dp(x) -> C.c_void_p:
    if isinstance(x, DevBuf):
        return x.ptr
    if isinstance(x, int):
        return C.c_void_p(x)
    if hasattr(x, "data_ptr"):  # torch tensor on the context's device
        return C.c_void_p(x.data_ptr())
    return x


def compress_bytes_multi(ctxs: Sequence[Context], data, block_size: int) -> bytes:
    a = as_u8(data)
    cap = int(lib().bmh_compress_bound(a.size, block_size))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    olen = C.c_uint64()
    arr = (C.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
    _check(lib().bmh_compress_host_multi(arr, len(ctxs), _ptr(a), a.size, block_size, _ptr(out), cap,
                                         C.byref(olen)), "compress_multi")
    return out[: olen.value].tobytes()


# ---------------------------------------------------------------- host-only functions
def decompress_bytes(data) -> bytes:
    """decompress() (main.cpp:327-345) on a record or BMH container held in memory."""
    a = as_u8(data)
    n = C.c_uint64()
    _check(lib().bmh_decompress_host(_ptr(a), a.size, None, 0, C.byref(n)), "decompress(size)")
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    _check(lib().bmh_decompress_host(_ptr(a), a.size, _ptr(out), n.value, C.byref(n)), "decompress")
    return out[: n.value].tobytes()


def record_to_mtf(rec) -> bytes:
    """huffman_reverse (main.cpp:259-281): record -> MTF stream."""
    a = as_u8(rec)
    n = C.c_uint64()
    _check(lib().bmh_record_to_mtf(_ptr(a), a.size, None, 0, C.byref(n)), "record_to_mtf(size)")
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    _check(lib().bmh_record_to_mtf(_ptr(a), a.size, _ptr(out), n.value, C.byref(n)), "record_to_mtf")
    return out[: n.value].tobytes()


def huffman_build(freq: np.ndarray, first: np.ndarray, n: int = 0) -> CodeTable:
    """The tree of huffman() (main.cpp:245-254) for a block of n bytes (n = 0: size unknown,
    the closed-form tie-break of SURVEY App. B.3; below 128 KiB the order of the reference's
    heap history for that size, include/bmh.h bmh_huffman_build_sized)."""
    f = np.ascontiguousarray(freq, dtype=np.uint64)
    fi = np.ascontiguousarray(first, dtype=np.uint64)
    t = CodeTable()
    _check(lib().bmh_huffman_build_sized(_u64p(f), _u64p(fi), n, C.byref(t)), "huffman_build")
    return t


def node_ranks(n: int, L: int) -> tuple[list[int], bool]:
    """Address ranks of the 2L - 1 tree nodes of an n-byte block, and whether they come from the
    reference's heap history (True) or the closed form (False)."""
    buf = (C.c_uint16 * 511)()
    r = lib().bmh_node_ranks(n, L, buf)
    if r < 0:
        raise BmhError(BMH_EINVAL, "node_ranks: L must be 1..256")
    return list(buf[: 2 * L - 1]), r == 1


def payload_bytes(table: CodeTable, freq: np.ndarray) -> int:
    f = np.ascontiguousarray(freq, dtype=np.uint64)
    return int(lib().bmh_payload_bytes(C.byref(table), _u64p(f)))


def container_records(data) -> list[bytes]:
    a = as_u8(data)
    nb = C.c_uint64()
    _check(lib().bmh_container_info(_ptr(a), a.size, C.byref(nb), None), "container_info")
    out = []
    for b in range(nb.value):
        p = C.c_void_p()
        ln = C.c_uint64()
        _check(lib().bmh_container_record(_ptr(a), a.size, b, C.byref(p), C.byref(ln)), "container_record")
        off = p.value - a.ctypes.data
        out.append(a[off:off + ln.value].tobytes())
    return out


def is_container(data) -> bool:
    a = as_u8(data)
    return bool(lib().bmh_is_container(_ptr(a), a.size))


# ------------------------------------------------------- reference-named stage functions
_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def bwt(data, ctx: Context | None = None) -> tuple[int, bytes]:
    """bwt() (main.cpp:77-91): (primary row, last column) of the cyclic-rotation BWT."""
    ctx = ctx or default_context()
    a = as_u8(data)
    if a.size == 0:
        raise BmhError(BMH_EINVAL, "bwt: empty input (the reference segfaults)")
    d_in, d_L = ctx.alloc(a.size), ctx.alloc(a.size)
    try:
        d_in.upload(a)
        prim = ctx.bwt_dev(d_in, np.array([0, a.size], dtype=np.uint64), d_L)
        return int(prim[0]), d_L.download().tobytes()
    finally:
        d_in.free()
        d_L.free()


def move_to_front(data, ctx: Context | None = None) -> bytes:
    """move_to_front() (main.cpp:93-112)."""
    ctx = ctx or default_context()
    a = as_u8(data)
    if a.size == 0:
        return b""
    d_L, d_m = ctx.alloc(a.size), ctx.alloc(a.size)
    try:
        d_L.upload(a)
        ctx.mtf_dev(d_L, np.array([0, a.size], dtype=np.uint64), d_m)
        return d_m.download().tobytes()
    finally:
        d_L.free()
        d_m.free()


def huffman(mtf, ctx: Context | None = None) -> tuple[bytes, CodeTable]:
    """huffman() (main.cpp:229-257): (payload bytes, code table incl. tree)."""
    ctx = ctx or default_context()
    a = as_u8(mtf)
    if a.size == 0:
        raise BmhError(BMH_EINVAL, "huffman: empty input (the reference segfaults)")
    offs = np.array([0, a.size], dtype=np.uint64)
    d_m = ctx.alloc(a.size)
    try:
        d_m.upload(a)
        freq, first = ctx.histogram_dev(d_m, offs)
        freq, first = freq[0], first[0]
        t = huffman_build(freq, first, a.size)  # the MTF stream has the block's size
        cap = (payload_bytes(t, freq) + 3) & ~3  # the pack writes whole 4-byte words
        d_out = ctx.alloc(cap)
        try:
            tabs = (CodeTable * 1)(t)
            nbytes = np.zeros(1, dtype=np.uint64)
            _check(lib().bmh_pack_dev(ctx.h, d_m.ptr, _u64p(offs), 1, tabs, d_out.ptr, cap, None, _u64p(nbytes)),
                   "pack")
            return d_out.download(int(nbytes[0])).tobytes(), t
        finally:
            d_out.free()
    finally:
        d_m.free()


def tree_to_bytes(table: CodeTable) -> bytes:
    """tree_to_bytes() (main.cpp:189-196)."""
    return table.tree_bytes


def metrics_line(out_name: str, n: int, size: int, header: int) -> str:
    """The stdout line of compress() (main.cpp:321, 402-413), C++ ostream default formatting."""
    return (f"header size: {_g(header)} $$ file_name: {out_name} $$ initial_data_size: {n} $$ "
            f"encoded_file_size: {size} $$ bits_avg: {_g(8 * size / n)} $$ compress_rate = {_g(size / n)}")


def _g(x: float) -> str:
    s = f"{x:.6g}"
    return s


def compress(initial_file_name: str, encoded_file_name: str, block_size: int = 0,
             ctx: Context | None = None) -> None:
    """compress() (main.cpp:300-325)."""
    ctx = ctx or default_context()
    with open(initial_file_name, "rb") as f:
        data = f.read()
    out = ctx.compress_bytes(data, block_size)
    if is_container(out):
        recs = container_records(out)
        header = 32 + 8 * len(recs) + sum(24 + int.from_bytes(r[16:24], "little") for r in recs)
    else:
        header = 24 + int.from_bytes(out[16:24], "little")
    print(metrics_line(encoded_file_name, len(data), len(out), header))
    with open(encoded_file_name, "wb") as f:
        f.write(out)


def decompress(encoded_file_name: str, decoded_file_name: str) -> None:
    """decompress() (main.cpp:327-345)."""
    with open(encoded_file_name, "rb") as f:
        data = f.read()
    with open(decoded_file_name, "wb") as f:
        f.write(decompress_bytes(data))


__all__ = ["BmhError", "CodeTable", "Context", "DevBuf", "lib", "bwt", "move_to_front", "huffman",
           "tree_to_bytes", "compress", "decompress", "compress_bytes_multi", "decompress_bytes",
           "record_to_mtf", "huffman_build", "node_ranks", "payload_bytes", "container_records", "is_container",
           "metrics_line", "default_context"]
