"""Run-heavy blocks (csrc/bwt_runs.hip): in batches up to 64 MiB, blocks of 64 KiB .. 16 MiB with
at most n / 4 cyclic runs take the run-length BWT instead of the rotation sorter. The BWT (L and
primary index) and the records must equal the oracle's (the C restatement of reference
main.cpp:77-91 and the encode pipeline) on every shape the run path has to get right: runs that
wrap around the block end, identical rotations (periodic blocks, where the primary is the first
slot of rotation 0's tie group, as std::stable_sort leaves it), one byte value, two runs, the
64 KiB floor, and batches that mix run blocks with sorter blocks (contiguous on either side or
interleaved, which gathers the sorter blocks into one sub-batch)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import bmh

pytestmark = pytest.mark.gpu


def geometric_runs(seed: int, n: int, alphabet: int, mean_run: float) -> bytes:
    rng = np.random.default_rng(seed)
    out = bytearray()
    prev = -1
    while len(out) < n:
        c = int(rng.integers(0, alphabet))
        if c == prev:
            c = (c + 1) % alphabet
        out += bytes([c]) * int(rng.geometric(1.0 / mean_run))
        prev = c
    return bytes(out[:n])


def sparse_bitmap(seed: int, n: int) -> bytes:
    """Mostly zero bytes with short non-zero bursts (a scanned page, like Calgary pic)."""
    rng = np.random.default_rng(seed)
    a = np.zeros(n, np.uint8)
    for s in rng.integers(0, n - 40, n // 400):
        a[s:s + int(rng.integers(1, 40))] = rng.integers(1, 256, 1)[0]
    return a.tobytes()


def wrap_run(seed: int, n: int) -> bytes:
    """A long run of 'z' split across the block end, runs inside."""
    body = bytearray(geometric_runs(seed, n - 9000, 4, 20))
    return b"z" * 5000 + bytes(body) + b"z" * 4000


RUN_CASES = {
    "geometric_a3": lambda: geometric_runs(1, 200_003, 3, 12.0),
    "geometric_a200": lambda: geometric_runs(2, 131_072, 200, 6.0),
    "sparse_bitmap": lambda: sparse_bitmap(3, 300_000),
    "wrap_run": lambda: wrap_run(4, 150_000),
    "periodic_runs": lambda: (b"\x00" * 700 + b"\x01\x02") * 120,
    "periodic_short": lambda: (b"a" * 9 + b"b") * 20_000,
    "one_value": lambda: b"\x07" * 100_000,
    "two_runs": lambda: b"\x05" * 70_000 + b"\x09" * 50_000,
    "floor_64k": lambda: geometric_runs(5, 1 << 16, 2, 8.0),
}


def runs_of(data: bytes) -> int:
    a = np.frombuffer(data, np.uint8)
    return int(np.count_nonzero(a != np.roll(a, 1)))


@pytest.mark.parametrize("name", sorted(RUN_CASES))
def test_run_block_bwt_matches_oracle(ctx, oracle, name):
    data = RUN_CASES[name]()
    assert len(data) >= 1 << 16 and runs_of(data) * 4 <= len(data), "case must take the run path"
    ctx.reset_stats()
    ctx.set_timing(True)
    prim, L = bmh.bwt(data, ctx)
    st = ctx.kernel_stats()
    ctx.set_timing(False)
    oprim, oL = oracle.bwt(data)
    assert L == oL and prim == oprim, (name, prim, oprim)
    assert "bwt_run_count" in st and "bwt_g1_scatter" not in st, sorted(st)


def test_run_blocks_in_mixed_batches(ctx, oracle):
    """Sorter blocks before, between and after run blocks: one record per block, each the
    oracle's."""
    rng = np.random.default_rng(7)
    run_a = RUN_CASES["sparse_bitmap"]()
    run_b = RUN_CASES["geometric_a3"]()
    txt = [rng.integers(0, 40, int(s)).astype(np.uint8).tobytes() for s in (90_000, 70_001, 5_000, 120_000)]
    layouts = [
        [txt[0], run_a, txt[1], run_b, txt[2]],  # interleaved: sorter blocks gathered
        [run_a, txt[0], txt[1]],                 # contiguous sorter blocks after a run block
        [txt[0], txt[3], run_b],                 # contiguous sorter blocks first
        [run_a, run_b],                          # run blocks only
        [txt[2], run_a, run_b, txt[3]],
    ]
    for lay in layouts:
        recs = ctx.encode_blocks(lay)
        for blk, rec in zip(lay, recs):
            assert rec == oracle.encode(blk), [len(b) for b in lay]


def test_run_blocks_sorted_together(ctx, oracle):
    """Every run shape in one batch (run blocks only, then with sorter blocks between): the run
    path sorts all of a batch's run blocks together (block index above every key, one host wait
    a doubling round for all), one-value blocks included. BWT and records equal the oracle's."""
    blocks = [RUN_CASES[k]() for k in sorted(RUN_CASES)]
    blocks += [sparse_bitmap(21, 262_144), sparse_bitmap(22, 251_072)]  # Calgary pic's 256 KiB halves' shape
    offs = np.cumsum([0] + [len(b) for b in blocks]).astype(np.uint64)
    d_in, d_L = ctx.alloc(int(offs[-1])), ctx.alloc(int(offs[-1]))
    d_in.upload(np.frombuffer(b"".join(blocks), np.uint8))
    ctx.reset_stats()
    ctx.set_timing(True)
    prim = ctx.bwt_dev(d_in, offs, d_L)
    st = ctx.kernel_stats()
    ctx.set_timing(False)
    L = d_L.download()
    d_in.free()
    d_L.free()
    assert "bwt_g1_scatter" not in st, sorted(st)
    for i, b in enumerate(blocks):
        op, oL = oracle.bwt(b)
        assert int(prim[i]) == op and L[int(offs[i]):int(offs[i + 1])].tobytes() == oL, (i, len(b))
    # sorter blocks between them, past kBandCeil (128 KiB) so the oracle's closed-form Huffman
    # tie-break is the reference's (below it the reference follows its heap history, which
    # heap_order.cpp replays and tests/test_bands.py pins against the reference's own records)
    rng = np.random.default_rng(3)
    mixed = []
    for b in blocks[:6]:
        mixed += [b, rng.integers(0, 30, 140_000).astype(np.uint8).tobytes()]
    recs = ctx.encode_blocks(mixed)
    for blk, rec in zip(mixed, recs):
        assert rec == oracle.encode(blk)


def test_run_path_compress_roundtrip(ctx):
    """compress_bytes over a run-heavy stream (blocks cut at 1 MiB, batches <= 64 MiB are
    screened) round-trips and matches the single-block-per-call records."""
    data = sparse_bitmap(11, 3_000_000)
    out = ctx.compress_bytes(data, block_size=1 << 20)
    assert ctx.decompress_bytes(out) == data
    recs = bmh.container_records(out)
    blocks = [data[i:i + (1 << 20)] for i in range(0, len(data), 1 << 20)]
    assert recs == ctx.encode_blocks(blocks)


def test_calgary_pic_takes_run_path(ctx):
    """Calgary pic (513 KB, 76 K runs) through the run path: the reference's record, no
    rotation-sorter passes."""
    from oracle_ffi import GOLDEN
    pic = open(os.path.join(GOLDEN, "calgary", "pic"), "rb").read()
    gold = open(os.path.join(GOLDEN, "calgary_records", "pic.bzap"), "rb").read()
    ctx.reset_stats()
    ctx.set_timing(True)
    rec = ctx.encode_blocks([pic])[0]
    st = ctx.kernel_stats()
    ctx.set_timing(False)
    assert rec == gold
    assert "bwt_run_sort" in st and "bwt_g1_scatter" not in st, sorted(st)


def _np_runs(seed: int, n: int, alphabet: int, mean_run: float) -> np.ndarray:
    """Geometric runs (consecutive runs differ) built with numpy, for multi-MiB blocks."""
    rng = np.random.default_rng(seed)
    k = int(n / mean_run * 1.5) + 64
    lens = rng.geometric(1.0 / mean_run, k)
    vals = np.cumsum(rng.integers(1, alphabet, k)) % alphabet
    return np.repeat(vals.astype(np.uint8), lens)[:n]


def test_run_heavy_blocks_in_four_pipeline_batch(ctx, oracle):
    """a batch past the run screen (> 64 MiB) of >= 16 blocks runs on four pipelines,
    the fourth on stream D, the run path's side stream. The screen is decided on the whole batch
    (Ctx::screen_total), so its run-heavy blocks (1-4 MiB, <= n/4 runs) stay on the rotation sorter
    and never queue behind pipeline 3. Every record equals the same block encoded alone (where the
    screen sends it down the run path), and one block equals the oracle."""
    sizes = [(4 << 20) - 3 * b * 7919 if b % 3 else (1 << 20) + b * 4099 for b in range(24)]
    blocks = [_np_runs(100 + b, n, (3, 17, 200)[b % 3], (6.0, 12.0, 40.0)[b % 3]) for b, n in enumerate(sizes)]
    assert sum(sizes) > 64 << 20 and len(blocks) >= 16
    for b in blocks:  # run-heavy by the screen's rule (runs <= n / 4)
        assert int(np.count_nonzero(b != np.roll(b, 1))) * 4 <= b.size
    recs = ctx.encode_blocks(blocks)
    for i, blk in enumerate(blocks):
        assert recs[i] == ctx.encode_blocks([blk])[0], i
    assert recs[0] == oracle.encode(blocks[0])
