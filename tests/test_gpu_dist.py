"""GPU: bench.py's N-rank path with the real libbmh encoder — 2 ranks under
torch.distributed.run sharing the test box's GPU, launched exactly as the driver launches the
scaling runs (ranks map to device local_rank mod device_count; the gloo process group carries
only the barriers and the max-over-ranks / sum-over-ranks reductions, never block data — the
same control plane as on 8 GPUs, bmh/dist.py). Each rank checks its own records against the
reference manifest (config 4, SURVEY §8e: block b -> rank b mod N); the weak case also runs
the default line's decode, PCIe-inclusive and Calgary legs, so every leg of the driver's N > 1
line has run under a test.

The ranks are started as child processes of this (GPU-initialised) pytest process; nothing
here replaces a running program."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_world2_bench_on_gpu(scaling):
    env = dict(os.environ)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--scaling", scaling, "--cpu-procs", "2"]
    if scaling == "weak":  # 64 blocks per rank, every leg of the default line
        cmd += ["--bytes-per-gpu", str(256 << 20), "--decode-steps", "1", "--pcie-steps", "1", "--calgary-steps", "1"]
    else:  # config 4 as written (1 GiB dealt over the ranks) + the 1 GiB-per-GPU leg, here 256 MiB
        cmd += ["--decode-steps", "0", "--pcie-steps", "0", "--calgary-steps", "0", "--bytes-per-gpu",
                str(256 << 20), "--weak-steps", "1"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.strip().splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["value"] > 0 and line["ms_per_step"] > 0
    nblk = 128 if scaling == "weak" else 256  # blocks over both ranks
    assert line["parity"] == f"{nblk}/{nblk} records byte-identical to the reference manifest", line["parity"]
    # rank 0 times the reference CPU path at any world size (here on 2 processes to stay short)
    cb = line["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] == 2 and cb["kind"] == "reference", cb
    # the pipelines the library really ran the rank's batch on (capi.cpp encode_blocks): 4 by the
    # size rule for 512 MiB (strong: 128 blocks a rank), 1 for a dense 256 MiB batch (weak)
    assert line["config"]["streams_per_gpu"] == (4 if scaling == "strong" else 1)
    if scaling == "strong":
        w = line["weak_scaling"]
        assert w["bytes_per_gpu"] == 256 << 20 and w["value"] > 0 and w["streams_per_gpu"] == 1
        assert w["parity"] == "128/128 records byte-identical to the reference manifest", w
    else:
        assert line["weak_scaling"] is None
    if scaling == "weak":
        assert line["decode"]["roundtrip_bit_exact"]
        assert line["pcie_inclusive"]["records_equal_device_encode"]
        assert line["calgary"]["whole_files"]["records_byte_identical_to_reference"]
        assert line["calgary"]["blocks_256k"]["records_byte_identical_to_reference"]
