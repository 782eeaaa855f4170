"""CPU: the N > 1 path (one process per device, blocks dealt round-robin, no data-path
collective) rehearsed with world_size 2 over gloo on 127.0.0.1.

The per-block encoder here is the test-only oracle standing in for a device; what is under
test is the sharding / timing / reassembly logic bench.py and the multi-GPU driver use.
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
    r = dist.init("gloo")
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
