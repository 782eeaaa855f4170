"""CPU: the test-only oracle (oracle/oracle.c) pinned to the reference's own outputs.

Every expectation here was produced by the real reference (oracle/_ref/ref_COMPRESS, compiled
from /root/reference/main.cpp in the build container) and committed under tests/golden/ by
tests/golden/make_golden.py; SURVEY.md Appendix C lists the same values.
"""
import hashlib

import numpy as np
import pytest

from bmh import synth
import os

from oracle_ffi import GOLDEN, golden_calgary, golden_small, manifest

# (primary, tree bytes, payload bytes, total) per Calgary file
APPENDIX_C = {
    "bib": (20021, 138, 33043, 33205), "book1": (176914, 137, 267002, 267163),
    "book2": (126853, 152, 186818, 186994), "geo": (62253, 320, 69219, 69563),
    "news": (69906, 154, 133339, 133517), "obj1": (7292, 320, 11441, 11785),
    "obj2": (5164, 320, 88389, 88733), "paper1": (11627, 143, 18057, 18224),
    "paper2": (16446, 149, 27963, 28136), "pic": (71709, 253, 101231, 101508),
    "progc": (13575, 148, 13527, 13699), "progl": (31494, 147, 18574, 18745),
    "progp": (43017, 145, 12657, 12826), "trans": (48011, 154, 22222, 22400),
}


def test_golden_records_match_appendix_c():
    agg = hashlib.sha256()
    for name, data, rec in golden_calgary():
        prim, tree, pay, total = APPENDIX_C[name]
        assert len(rec) == total
        assert int.from_bytes(rec[0:8], "little") == prim
        assert int.from_bytes(rec[8:16], "little") == len(data)
        assert int.from_bytes(rec[16:24], "little") == tree
        assert total - 24 - tree == pay
        agg.update(rec)
    assert agg.hexdigest() == "744bbe9f0adbbf155cbe2dc36d7b5e5fbe458f7293b335bcb0c94d98e50e3c2c"


@pytest.mark.parametrize("name", sorted(APPENDIX_C))
def test_oracle_encode_calgary(oracle, name):
    data, rec = next((d, r) for n, d, r in golden_calgary() if n == name)
    assert oracle.encode(data) == rec


def test_oracle_faithful_bwt_agrees_with_fast(oracle):
    # the merge-sort restatement of std::stable_sort vs prefix doubling, incl. periodic inputs
    rng = np.random.default_rng(5)
    cases = [b"banana", b"a", b"ab" * 50, bytes(300), b"abc" * 77 + b"ab",
             rng.integers(0, 4, 2000, dtype=np.uint8).tobytes(),
             rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()]
    for c in cases:
        assert oracle.bwt(c, faithful=True) == oracle.bwt(c)


def test_oracle_small_known_answers(oracle):
    for name, data, rec in golden_small():
        assert oracle.encode(data) == rec, name
    # SURVEY.md §4 table
    assert oracle.bwt(b"banana") == (3, b"nnbaaa")
    a = oracle.encode(b"a")
    assert len(a) == 27 and a[24:] == bytes([0x30, 0x80, 0x00])


def test_oracle_decode_golden(oracle):
    for name, data, rec in golden_calgary():
        assert oracle.decode(rec) == data, name
        assert oracle.mtf_inverse(oracle.decode_to_mtf(rec)) == oracle.bwt(data)[1], name


def test_oracle_calgary_256k_manifest(oracle):
    man = manifest("calgary_256k")
    blocks = []
    for _, data, _ in golden_calgary():
        blocks += [data[i:i + 262144] for i in range(0, len(data), 262144)]
    agg = hashlib.sha256()
    for b, e in zip(blocks, man["blocks"]):
        r = oracle.encode(b)
        assert hashlib.sha256(r).hexdigest() == e["sha256"]
        agg.update(r)
    assert agg.hexdigest() == man["aggregate_sha256"]


def test_oracle_random_block0_manifest(oracle):
    man = manifest("random_1g_4m")["blocks"]
    for b in (0, 255):
        r = oracle.encode(synth.splitmix64_bytes(0, b << 22, 1 << 22))
        assert len(r) == man[b]["record_len"]
        assert int.from_bytes(r[:8], "little") == man[b]["primary"]
        assert hashlib.sha256(r).hexdigest() == man[b]["sha256"]


def test_oracle_zipf_1m_block0_manifest(oracle):
    man = manifest("zipf100m_1m")["blocks"][0]
    r = oracle.encode(synth.zipf_text(1 << 20))
    assert hashlib.sha256(r).hexdigest() == man["sha256"]


def test_synth_hashes():
    # SURVEY.md Appendix D
    w = synth.splitmix64_words(0, 0, 1)
    assert int(w[0]) == 0xE220A8397B1DCDAF
    assert synth.splitmix64_bytes(0, 0, 8).tobytes() == bytes.fromhex("afcd1d7b39a820e2")
    # counter-based: any window equals the same slice of the stream
    s = synth.splitmix64_bytes(0, 0, 4096)
    assert synth.splitmix64_bytes(0, 1001, 777).tobytes() == s[1001:1778].tobytes()
    z = synth.zipf_text(16 << 20)
    assert hashlib.sha256(z.tobytes()).hexdigest() == \
        "b8b5a2980d7a3c0ec97b8eafa08eaf2423aa1696be1fb47b191566c737d2b889"


def test_oracle_zipf_stream_pinned(oracle):
    """The oracle's sequential App. D Zipf generator (config 5's input, used to make the 512-block
    zipf_16m manifest): App. D's sha256 of the first 16 MiB, the numpy generator's bytes, and
    reads of any length continue the same stream (tokens cut across reads)."""
    from oracle_ffi import ZipfStream
    z = ZipfStream(oracle)
    parts = [z.read(n) for n in (1, 5, 1000003, 17, (16 << 20) - 1000026)]
    a = np.concatenate(parts)
    assert hashlib.sha256(a.tobytes()).hexdigest() == \
        "b8b5a2980d7a3c0ec97b8eafa08eaf2423aa1696be1fb47b191566c737d2b889"
    assert (a[: 1 << 21] == synth.zipf_text(1 << 21)).all()
    man = manifest("zipf_16m")
    assert len(man["blocks"]) == 512 and all(b["n"] == 16 << 20 for b in man["blocks"])
    assert man["blocks"][0]["primary"] == 6326714 and man["blocks"][0]["record_len"] == 5038328


def test_full_pipeline_fixture_sizes_and_decode(oracle):
    """The reference's FULL_PIPELINE records (tests/golden/full_pipeline, make_full_pipeline.py):
    same sizes and headers as its standalone COMPRESS records, tree bytes may differ (heap
    history across files); each decodes to its input with the oracle and the host decoder."""
    import bmh
    fp = os.path.join(GOLDEN, "full_pipeline")
    differ = 0
    for name, data, rec in golden_calgary():
        with open(os.path.join(fp, name + ".bzap"), "rb") as f:
            full = f.read()
        assert len(full) == len(rec) and full[:24] == rec[:24], name
        differ += full != rec
        assert oracle.decode(full) == data, name
        assert bmh.decompress_bytes(full) == data, name
    assert differ == 13
