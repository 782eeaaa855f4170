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
  * byte-exact records wherever the manifest records that the model reproduces the reference.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import bmh
from bmh import synth
from oracle_ffi import GOLDEN, REF_DIR

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


def check_against_reference(e, rec: bytes) -> None:
    import hashlib
    assert len(rec) == e["record_len"], (e["kind"], e["n"])
    assert header(rec) == (e["primary"], e["n"], e["tree_len"]), (e["kind"], e["n"])
    if e["oracle_exact"]:
        assert hashlib.sha256(rec).hexdigest() == e["sha256"], (e["kind"], e["n"])


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
    """GPU encode of every band input in one batch: size / header parity with the reference,
    byte-exact where the model holds; the GPU decodes the reference's records; the
    reference's decoder (when it travelled with the tree) decodes ours."""
    datas = [band_input(e["kind"], e["n"]) for e in MAN["cases"]]
    recs = ctx.encode_blocks(datas)
    for e, rec in zip(MAN["cases"], recs):
        check_against_reference(e, rec)
    for e, data in zip(MAN["cases"], datas):
        r = ref_record(e)
        if r is not None:
            assert ctx.decompress_bytes(r) == data, (e["kind"], e["n"])
    if os.path.exists(REF_DEC):
        for e, data, rec in list(zip(MAN["cases"], datas, recs))[::5]:
            (tmp_path / "r.bzap").write_bytes(rec)
            subprocess.run([REF_DEC, "r.bzap", "r.out"], cwd=tmp_path, check=True, capture_output=True, timeout=60)
            assert (tmp_path / "r.out").read_bytes() == data, (e["kind"], e["n"])
