#!/usr/bin/env python3
"""Headline benchmark: BWT -> MTF -> Huffman block encode on MI355X.

Metric (BASELINE.json): encode MB/s (and ratio) — workload = BASELINE config 4, 1 GiB of
uniform-random bytes (splitmix64 seed 0) in 4 MiB blocks per GPU. A "step"
encodes the rank's whole 1 GiB batch (256 blocks) from HBM to reference records in HBM.
Weak scaling: rank r owns global blocks r, r+N, r+2N, ... of the N GiB stream (round-robin,
no collective on the data path); value = bytes of all ranks / max-over-ranks time.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

Prints ONE JSON line on rank 0 (plus diagnostics on stderr).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "bwt-mtf-huffman-compressor_amd")
sys.path.insert(0, PKG)

import bmh  # noqa: E402
from bmh import dist, synth  # noqa: E402

METRIC = "encode MB/s and ratio on Calgary + 1 GiB synthetic at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

# Algorithmic HBM bytes per input byte of the batch for the kernels that sweep the whole
# batch once per launch (DESIGN.md §4 states and justifies each figure).
# roofline.achieved uses SURVEY.md §8(d)'s graded per-unit figure: 1 algorithmic HBM byte per
# input byte ("HBM-read roofline"), times the input bytes one launch processes. Every kernel
# below processes the whole batch per launch. STAGE_BYTES_PER_INPUT_BYTE is the
# diagnostic per-stage traffic model (minimum bytes each kernel must move).
ALGO_BYTES_PER_INPUT_BYTE = 1.0
STAGE_BYTES_PER_INPUT_BYTE = {
    "bwt_g1_hist": 1.0,         # read input
    "bwt_g1_scatter": 9.0,      # read input 1 B, write the 8-byte rotation record
    "bwt_finish_dense": 9.0,    # read the 8-byte record, write L 1 B
    "mtf_recency": 1.0,         # read L
    "mtf_encode": 2.0,          # read L 1 B, write MTF 1 B
    "mtf_hist": 1.0,            # read MTF
    "pack_write": 2.0,          # read MTF 1 B, write payload ~1 B (random data)
}
PMC_TRAFFIC = os.path.join(REPO, "profiles", "pmc_traffic.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(block_size: int, nsample: int) -> dict:
    """The reference CPU path (oracle/_ref/ref_COMPRESS, compiled from the reference sources)
    on a bounded sample of the same workload, one process per block, all in parallel."""
    ref = os.path.join(REPO, "oracle", "_ref", "ref_COMPRESS")
    tmp = tempfile.mkdtemp(prefix="bmh_cpu_")
    files = []
    for b in range(nsample):
        p = os.path.join(tmp, f"b{b:04d}")
        synth.splitmix64_bytes(0, b * block_size, block_size).tofile(p)
        files.append(p)
    kind = "reference"
    t0 = time.perf_counter()
    if os.path.exists(ref):
        procs = [subprocess.Popen([ref, f, f + ".bzap"], stdout=subprocess.DEVNULL) for f in files]
        rcs = [p.wait() for p in procs]
        wall = time.perf_counter() - t0
        ok = all(rc == 0 for rc in rcs)
    else:  # the from-scratch C port (oracle.c), one thread per block
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from concurrent.futures import ThreadPoolExecutor

        from oracle_ffi import Oracle
        orc = Oracle()
        kind = "port"

        def one(f):
            rec = orc.encode(np.fromfile(f, np.uint8), faithful=True)
            with open(f + ".bzap", "wb") as g:
                g.write(rec)
        with ThreadPoolExecutor(nsample) as ex:
            list(ex.map(one, files))
        wall = time.perf_counter() - t0
        ok = True
    # parity of the baseline itself against the committed manifest
    try:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from oracle_ffi import manifest
        man = manifest("random_1g_4m")["blocks"] if block_size == 1 << 22 else None
        if man:
            for b, f in enumerate(files):
                with open(f + ".bzap", "rb") as g:
                    ok &= hashlib.sha256(g.read()).hexdigest() == man[b]["sha256"]
    except Exception as e:  # pragma: no cover
        log("cpu_baseline manifest check skipped:", e)
    for f in files:
        for x in (f, f + ".bzap"):
            if os.path.exists(x):
                os.remove(x)
    os.rmdir(tmp)
    return {"value": round(nsample * block_size / wall / 1e6, 3), "unit": "MB/s", "cores": nsample,
            "kind": kind, "sample": f"{nsample} x {block_size >> 20} MiB splitmix64 blocks (global blocks "
            f"0..{nsample - 1}), one process per block, wall {wall:.2f} s, records match manifest: {ok}"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--block-size", type=int, default=4 << 20)
    ap.add_argument("--bytes-per-gpu", type=int, default=1 << 30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="blocks in the CPU sample (default: host threads, <=16)")
    ap.add_argument("--decode-steps", type=int, default=3, help="timed GPU decode steps of the same records (0: skip)")
    a = ap.parse_args()

    # BMH_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin);
    # the driver's runs use the default (RCCL, one rank per GPU).
    r = dist.init(os.environ.get("BMH_DIST_BACKEND") or None)
    world = r.world
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    dev = r.local_rank % max(1, int(bmh.lib().bmh_device_count()))
    ctx = bmh.Context(dev)

    bs = a.block_size
    nblk = a.bytes_per_gpu // bs
    mine = [r.rank + world * i for i in range(nblk)]  # global blocks of this rank
    total = nblk * bs
    offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
    d_in = ctx.alloc(total)
    for i, b in enumerate(mine):  # synthetic input generated straight into HBM
        ctx.synth_splitmix64(d_in.ptr.value + i * bs, bs, 0, b * bs)
    cap = int(sum(int(bmh.lib().bmh_record_bound(bs)) for _ in range(nblk)))
    d_out = ctx.alloc(cap)
    rec_offs = [None]

    def step():
        rec_offs[0] = ctx.encode_blocks_dev(d_in, offs, d_out, cap)

    def sync():
        # every call is host-synchronous on the context stream; also drain the device
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(dev)
        except Exception:
            pass

    for _ in range(a.warmup):
        step()
    # the timed region runs without per-kernel events ...
    dt = dist.timed_steps(r, step, a.steps, 0, sync)
    # ... then a separate pass with HIP events around every launch for the kernel breakdown.
    # The timed region splits each batch over 2 streams (kernels overlap, which stretches
    # their individual durations); the per-kernel pass runs one stream so each kernel's
    # duration (and so its roofline) is its own.
    ksteps = max(1, min(a.steps, 5))
    streams_env = os.environ.get("BMH_STREAMS")
    os.environ["BMH_STREAMS"] = "1"
    ctx.reset_stats()
    ctx.set_timing(True)
    for _ in range(ksteps):
        step()
    sync()
    stats = ctx.kernel_stats()
    ctx.set_timing(False)
    if streams_env is None:
        del os.environ["BMH_STREAMS"]
    else:
        os.environ["BMH_STREAMS"] = streams_env
    walls = {k[5:]: v for k, v in stats.items() if k.startswith("wall:")}
    stats = {k: v for k, v in stats.items() if not k.startswith("wall:")}

    ro = rec_offs[0]
    out_bytes = dist.sum_over_ranks(r, float(ro[-1]))
    # decode of the same records on the same GPU (GPU decode), timed the same way,
    # with a full round-trip check of this rank's batch; reported beside the encode line
    dec = None
    if a.decode_steps > 0:
        d_dec = ctx.alloc(total)
        ro_host = np.ascontiguousarray(ro, dtype=np.uint64)

        def dstep():
            ctx.decode_blocks_dev(d_out, ro_host, d_dec, total)
        dstep()
        ddt = dist.timed_steps(r, dstep, a.decode_steps, 0, sync)
        ok = d_dec.download().tobytes() == d_in.download().tobytes()
        ok = dist.sum_over_ranks(r, float(ok)) == world
        dec = {"value": round(float(total) * world * a.decode_steps / ddt / 1e6, 2), "unit": "MB/s (decoded bytes)",
               "ms_per_step": round(ddt / a.decode_steps * 1e3, 3), "steps": a.decode_steps,
               "roundtrip_bit_exact": bool(ok)}
        d_dec.free()
    in_bytes = float(total) * world
    # parity spot check: this rank's first block vs the reference manifest
    parity = None
    if bs == 1 << 22:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        try:
            from oracle_ffi import manifest
            man = manifest("random_1g_4m")["blocks"]
            checks = [(i, b) for i, b in enumerate(mine) if b < len(man)][:4]
            okc = 0
            for i, b in checks:
                rec = d_out.download(int(ro[i + 1] - ro[i]), int(ro[i]))
                okc += hashlib.sha256(rec.tobytes()).hexdigest() == man[b]["sha256"]
            parity = f"{okc}/{len(checks)} records byte-identical to the reference manifest"
        except Exception as e:
            parity = f"unchecked ({e})"

    if r.rank == 0:
        steps = a.steps
        value = in_bytes * steps / dt / 1e6
        # dominant kernel over the timed region
        dom = max(stats.items(), key=lambda kv: kv[1][1]) if stats else None
        roof = None
        if dom:
            name, (launches, ms) = dom
            lps = launches / ksteps
            avg_s = ms / launches / 1e3
            per_launch = ALGO_BYTES_PER_INPUT_BYTE * total / lps  # batch bytes per launch
            ach = per_launch / avg_s / 1e9
            traffic = None
            try:  # HBM bytes per launch from the committed PMC summary of this workload
                pm = json.load(open(PMC_TRAFFIC))
                if pm.get("workload_bytes") == total and name in pm.get("kernels", {}):
                    traffic = pm["kernels"][name]["hbm_bytes_per_launch"]
            except (OSError, ValueError, KeyError):
                pass
            stage = STAGE_BYTES_PER_INPUT_BYTE.get(name)
            roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "measured": "HIP events on the kernel's stream, 1-stream kernel pass of the same workload",
                    "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": name,
                    "avg_launch_ms": round(avg_s * 1e3, 4), "launches_per_step": lps,
                    "algorithmic_bytes_per_launch": per_launch,
                    "stage_model_bytes_per_launch": stage * total if stage else None,
                    "stage_model_frac": round(stage * total / avg_s / 1e9 / HBM_PEAK_GBS, 4) if stage else None}
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": steps,
            "warmup": a.warmup, "ms_per_step": round(dt / steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: splitmix64(seed 0) bytes (SURVEY App. D), generated in HBM",
            "config": {"workload": "BASELINE config 4: 1 GiB uniform-random bytes per GPU, 4 MiB blocks, "
                                   "round-robin block deal", "block_size": bs, "blocks_per_gpu": nblk,
                       "bytes_per_gpu": total, "parallelism": f"{world} independent GPU(s), no collective",
                       "streams_per_gpu": int(os.environ.get("BMH_STREAMS", "2"))},
            "ratio": round(out_bytes / in_bytes, 7),
            "roofline": roof,
            "kernels_ms_per_step": {k: round(v[1] / ksteps, 3) for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])},
            "host_wall_ms_per_step": {k: round(v[1] / ksteps, 3) for k, v in walls.items()},
            "parity": parity,
            "decode": dec,
        }
        if world == 1 and not a.no_cpu_baseline:
            ns = a.cpu_sample or min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 8)))
            line["cpu_baseline"] = cpu_baseline(bs, ns)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    ctx.close()
    dist.finalize(r)


if __name__ == "__main__":
    main()
