"""the small-input bands (3-20 B, 100-256 B random, 4-10 KB,
39.8-43 KB, 63.6-64.5 KB) where the reference's Huffman tie-break follows glibc heap history
(main.cpp:232-253, std::pair<long, BTree*> ordered by heap address).

Fixtures: tests/golden/manifests/bands.json + tests/golden/bands/*.bzap, written by the real
reference (tests/golden/make_bands.py). Parity asserted here, for every case:
  * size: the record length equals the reference's (it does not depend on the tie-break,
    SURVEY §0.4);
  * cross-decode: the reference's records decode to the input with our decoders, and our
    records decode to the input with the reference's decoder (ref_DECOMPRESS, when built);
  * header: primary index, n and tree length equal the reference's;
  * byte-exact records wherever the manifest records that the model reproduces the reference;
  * byte-exact records everywhere from the library (host bmh_huffman_build_sized and the GPU
    encode): the node address order of the reference's heap history for the block size
    (csrc/heap_order.cpp), checked against the glibc restatement of oracle/alloc_trace, itself
    pinned to the reference's records here and call by call against traces of the reference
    binary (oracle/alloc_trace/band_trace.py --validate, this container only).
"""
import json
import os
import subprocess

import numpy as np
import pytest

import bmh
from bmh import synth
from oracle_ffi import GOLDEN, REF_DIR, REPO

import sys
sys.path.insert(0, os.path.join(REPO, "oracle", "alloc_trace"))
import band_trace  # noqa: E402  (test infrastructure: the glibc heap restatement)

MAN = json.load(open(os.path.join(GOLDEN, "manifests", "bands.json")))
REF_DEC = os.path.join(REF_DIR, "ref_DECOMPRESS")
_Z = synth.zipf_text(70_000).tobytes()
_R = synth.splitmix64_bytes(0, 0, 70_000).tobytes()


def band_input(kind: str, n: int) -> bytes:
    return (_R if kind == "random" else _Z)[:n]


def ref_record(e) -> bytes | None:
    if "file" not in e:
        return None
    with open(os.path.join(GOLDEN, e["file"]), "rb") as f:
        return f.read()


def header(rec: bytes):
    return tuple(int.from_bytes(rec[i:i + 8], "little") for i in (0, 8, 16))


def check_against_reference(e, rec: bytes, exact: bool = False) -> None:
    import hashlib
    assert len(rec) == e["record_len"], (e["kind"], e["n"])
    assert header(rec) == (e["primary"], e["n"], e["tree_len"]), (e["kind"], e["n"])
    if exact or e["oracle_exact"]:
        assert hashlib.sha256(rec).hexdigest() == e["sha256"], (e["kind"], e["n"])


def record_from_table(primary: int, mtf: np.ndarray, t) -> bytes:
    """write_bytes (io_utilities.h:7-27) of encode_with_huffman's payload (main.cpp:158-172)."""
    code = np.frombuffer(bytes(t.code), np.uint64)[mtf]
    ln = np.frombuffer(bytes(t.len), np.uint8)[mtf].astype(np.int64)
    start = np.cumsum(ln) - ln
    sym = np.repeat(np.arange(mtf.size), ln)
    k = np.arange(int(ln.sum())) - start[sym]
    bits = ((code[sym] >> (ln[sym] - 1 - k).astype(np.uint64)) & np.uint64(1)).astype(np.uint8)
    pay = np.packbits(bits).tobytes() or b"\x00"
    hdr = b"".join(int(v).to_bytes(8, "little") for v in (primary, mtf.size, t.tree_len))
    return hdr + t.tree_bytes + pay


def test_band_fixtures_cover_the_bands():
    ns = {(e["kind"], e["n"]) for e in MAN["cases"]}
    assert len(ns) == len(MAN["cases"]) >= 150
    for lo, hi in ((3, 20), (100, 256), (4000, 10000), (39800, 43000), (63600, 64500)):
        assert any(lo <= n <= hi for _, n in ns), (lo, hi)
    for e in MAN["cases"]:
        assert e["oracle_exact"] or os.path.exists(os.path.join(GOLDEN, e["file"]))


def test_band_reference_records_decode_with_our_decoders(oracle):
    for e in MAN["cases"]:
        rec = ref_record(e)
        if rec is None:
            continue
        data = band_input(e["kind"], e["n"])
        assert bmh.decompress_bytes(rec) == data, (e["kind"], e["n"])
        assert oracle.decode(rec) == data, (e["kind"], e["n"])


def test_band_oracle_records_size_header_and_ref_cross_decode(oracle, tmp_path):
    for e in MAN["cases"]:
        data = band_input(e["kind"], e["n"])
        rec = oracle.encode(data)
        check_against_reference(e, rec)
    if not os.path.exists(REF_DEC):
        pytest.skip("oracle/_ref/ref_DECOMPRESS not built (needs /root/reference)")
    for e in MAN["cases"][::3]:
        data = band_input(e["kind"], e["n"])
        (tmp_path / "r.bzap").write_bytes(oracle.encode(data))
        subprocess.run([REF_DEC, "r.bzap", "r.out"], cwd=tmp_path, check=True, capture_output=True, timeout=60)
        assert (tmp_path / "r.out").read_bytes() == data, (e["kind"], e["n"])


@pytest.mark.gpu
def test_band_gpu_records_and_decode(ctx, tmp_path):
    """GPU encode of every band input in one batch: every record byte-exact against the
    reference's (heap-history node order per block size); the GPU decodes the reference's records; the
    reference's decoder (when it travelled with the tree) decodes ours."""
    datas = [band_input(e["kind"], e["n"]) for e in MAN["cases"]]
    recs = ctx.encode_blocks(datas)
    for e, rec in zip(MAN["cases"], recs):
        check_against_reference(e, rec, exact=True)
    # one block at a time too (a batch of one size class; a fresh layout each call)
    for e in MAN["cases"][::7]:
        check_against_reference(e, ctx.encode_blocks([band_input(e["kind"], e["n"])])[0], exact=True)
    for e, data in zip(MAN["cases"], datas):
        r = ref_record(e)
        if r is not None:
            assert ctx.decompress_bytes(r) == data, (e["kind"], e["n"])
    if os.path.exists(REF_DEC):
        for e, data, rec in list(zip(MAN["cases"], datas, recs))[::5]:
            (tmp_path / "r.bzap").write_bytes(rec)
            subprocess.run([REF_DEC, "r.bzap", "r.out"], cwd=tmp_path, check=True, capture_output=True, timeout=60)
            assert (tmp_path / "r.out").read_bytes() == data, (e["kind"], e["n"])


def test_band_host_huffman_sized_exact(oracle):
    """bmh_huffman_build_sized (heap-history order for the block size) reproduces every band
    record of the reference byte for byte; the closed form alone reproduces 5 of 180."""
    for e in MAN["cases"]:
        data = band_input(e["kind"], e["n"])
        primary, L = oracle.bwt(data)
        mtf = np.frombuffer(oracle.mtf(L), np.uint8)
        freq, first = oracle.histogram(mtf.tobytes())
        rec = record_from_table(primary, mtf, bmh.huffman_build(freq, first, len(data)))
        check_against_reference(e, rec, exact=True)


def test_node_ranks_match_glibc_restatement():
    """libbmh's C++ heap replay (heap_order.cpp) gives the same node ranks as the test-only
    Python restatement (oracle/alloc_trace/glibc_heap.py), in the bands and past them."""
    rng = np.random.default_rng(5)
    ns = list(range(1, 25)) + [100, 212, 4000, 9000, 21000, 31000, 39900, 42000, 63700, 64400, 64600, 100000,
                                131071] + [int(x) for x in rng.integers(25, 131072, 12)]
    hist = 0
    for n in ns:
        for L in sorted({min(n, x) for x in (1, 2, 3, 17, 128, 129, 256)}):  # L <= n
            ranks, from_history = bmh.node_ranks(n, L)
            assert ranks == band_trace.node_ranks(n, L), (n, L)
            if not from_history:
                assert ranks == band_trace.model_ranks(L), (n, L)
            hist += from_history
    assert hist > 0
    # the closed form holds from 64.6 KB up
    for n in (64600, 65536, 100000, 131071, 1 << 17, 1 << 20):
        assert not any(bmh.node_ranks(n, L)[1] for L in (2, 64, 128, 129, 200, 256)), n


def test_glibc_restatement_pins_band_records(oracle):
    """The Python heap restatement's ranks reproduce the reference's band records (a spread of
    the 180 cases; all 180 by oracle/alloc_trace/band_trace.py --validate)."""
    for e in MAN["cases"][::9]:
        data = band_input(e["kind"], e["n"])
        rec = band_trace.record_with_ranks(data, band_trace.node_ranks)
        check_against_reference(e, rec, exact=True)
