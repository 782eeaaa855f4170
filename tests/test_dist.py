"""CPU: the N > 1 path (one process per device, blocks dealt round-robin, no data-path
collective) rehearsed with world_size 2 over gloo on 127.0.0.1.

The per-block encoder here is the test-only oracle standing in for a device; what is under
test is the sharding / timing / parity logic — bench.py's own rank_plan, encode_leg and
parity_leg, the code the driver's N-GPU runs execute around the GPU encoder.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

from bmh import dist


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _blocks():
    from bmh import synth
    z = synth.zipf_text(7 * 20000 + 123).tobytes()
    return [z[i:i + 20000] for i in range(0, len(z), 20000)]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from oracle_ffi import Oracle
    r = dist.init()
    try:
        orc = Oracle()
        blocks = _blocks()
        mine = dist.rank_blocks(len(blocks), r.rank, r.world)
        out = {}

        def step():
            for b in mine:
                out[b] = orc.encode(blocks[b])
        dt = dist.timed_steps(r, step, 2, 1, lambda: None)
        tot = dist.sum_over_ranks(r, float(sum(len(blocks[b]) for b in mine)))
        gathered = [None] * r.world
        r.dist.all_gather_object(gathered, out)
        if r.rank == 0:
            merged = {}
            for g in gathered:
                merged.update(g)
            q.put((dt, tot, [merged[b] for b in range(len(blocks))]))
    finally:
        dist.finalize(r)


class _OracleEncoder:
    """bench.DeviceEncoder's interface with the oracle in place of the GPU (test only)."""

    def __init__(self, mine, bs):
        from bmh import synth
        from oracle_ffi import Oracle
        self.orc, self.mine, self.bs = Oracle(), mine, bs
        self.blocks = [synth.splitmix64_bytes(0, b * bs, bs) for b in mine]
        self.in_bytes = len(mine) * bs
        self.recs = []

    def step(self):
        self.recs = [self.orc.encode(b) for b in self.blocks]

    def sync(self):
        pass

    def out_bytes(self):
        return sum(map(len, self.recs))

    def records(self):
        return self.recs


def _bench_worker(rank, world, port, q, scaling):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import bench
    r = dist.init()
    try:
        bs = 1 << 22
        # strong: 2 blocks in total dealt over the ranks; weak: 1 block per rank
        mine = bench.rank_plan(r.rank, r.world, bs, scaling, bytes_per_gpu=bs, total_bytes=2 * bs)
        enc = _OracleEncoder(mine, bs)
        res = bench.encode_leg(r, enc, 1, 0)
        parity = bench.parity_leg(r, enc.records(), mine, bs)
        if r.rank == 0:
            q.put((mine, res, parity))
    finally:
        dist.finalize(r)


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_world2_gloo_bench_legs(scaling):
    """bench.py's N-rank legs with 2 gloo ranks: the round-robin plan, the barrier-bracketed
    max-over-ranks timing, bytes summed over ranks, and every rank's records checked against
    the reference manifest (config 4, 4 MiB blocks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q, scaling)) for r in range(2)]
    for p in procs:
        p.start()
    mine, res, parity = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mine == [0]
    assert res["in_bytes"] == 2 * (1 << 22) and res["dt"] > 0
    assert res["out_bytes"] > res["in_bytes"]  # random data: records slightly larger
    assert parity == "2/2 records byte-identical to the reference manifest"


def test_bench_rank_plan():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    bs = 1 << 22
    for world in (1, 2, 4, 8):
        strong = [bench.rank_plan(r, world, bs, "strong", 1 << 30, 1 << 30) for r in range(world)]
        assert sorted(b for m in strong for b in m) == list(range(256))
        assert all(len(m) == 256 // world for m in strong)
        weak = [bench.rank_plan(r, world, bs, "weak", 1 << 30, 1 << 30) for r in range(world)]
        assert sorted(b for m in weak for b in m) == list(range(256 * world))
        assert weak[world - 1][:2] == [world - 1, 2 * world - 1]


def test_rank_blocks_partition():
    for world in (1, 2, 3, 8):
        seen = sorted(b for r in range(world) for b in dist.rank_blocks(37, r, world))
        assert seen == list(range(37))
        assert dist.rank_blocks(37, 1, world) == list(range(1, 37, world))


def test_world2_gloo_matches_single_process(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    dt, tot, recs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blocks = _blocks()
    assert tot == float(sum(map(len, blocks)))
    assert dt > 0
    assert recs == [oracle.encode(b) for b in blocks]


def test_single_rank_defaults(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    r = dist.init()
    assert (r.rank, r.world, r.dist) == (0, 1, None)
    assert dist.max_over_ranks(r, 3.5) == 3.5
    calls = []
    assert dist.timed_steps(r, lambda: calls.append(1), 3, 2, lambda: None) >= 0
    assert len(calls) == 5
