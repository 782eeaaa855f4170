#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: the per-rank batches of the driver's
default N > 1 runs (`bench.py --scaling strong`: 1 GiB dealt over N GPUs, block b -> rank b mod N)
are 1024 / N MiB = 256 / N blocks of 4 MiB. Each is run here as its own N = 1 bench process
(`--total-bytes`), repeated in fresh processes; the predicted N-GPU line is
    value(N) = 1 GiB / max-over-ranks step time ~= 1 GiB / t(1024/N MiB)
(ranks never exchange data and each has its own GPU, PCIe link and hardware queues), and the
predicted efficiency is value(N) / (N * value(1)).

  python3 tools/strong_rehearsal.py OUT.json [--reps 2] [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(total: int, steps: int, pcie_steps: int) -> dict:
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(steps), "--warmup", "3",
           "--total-bytes", str(total), "--no-cpu-baseline", "--decode-steps", "0",
           "--pcie-steps", str(pcie_steps), "--calgary-steps", "0"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-3000:])
        raise SystemExit(r.returncode)
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    return {"ms_per_step": d["ms_per_step"], "value": d["value"], "parity": d["parity"],
            "streams_per_gpu": d["config"]["streams_per_gpu"], "blocks": d["config"]["blocks_per_gpu"],
            "kernels_ms_per_step": d["kernels_ms_per_step"],
            "kernel_sum_ms": round(sum(d["kernels_ms_per_step"].values()), 3),
            "pcie_ms_per_step": (d["pcie_inclusive"] or {}).get("ms_per_step")}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--pcie-steps", type=int, default=3)
    a = ap.parse_args()
    rows = {}
    for n in (1, 2, 4, 8):
        mib = 1024 // n
        reps = [run(mib << 20, a.steps, a.pcie_steps) for _ in range(a.reps)]
        for x in reps:
            print(f"N={n} per-rank {mib} MiB: {x['ms_per_step']} ms, streams {x['streams_per_gpu']}, "
                  f"kernels {x['kernel_sum_ms']} ms, pcie {x['pcie_ms_per_step']} ms, {x['parity']}", flush=True)
        rows[n] = {"per_rank_mib": mib, "runs": reps,
                   "median_ms": round(statistics.median(x["ms_per_step"] for x in reps), 4),
                   "min_ms": min(x["ms_per_step"] for x in reps),
                   "median_pcie_ms": (statistics.median(x["pcie_ms_per_step"] for x in reps)
                                      if a.pcie_steps else None)}
    t1, m1 = rows[1]["median_ms"], rows[1]["min_ms"]
    for n, row in rows.items():
        t = row["median_ms"]
        row["predicted_value_MBps"] = round((1 << 30) / (t / 1e3) / 1e6, 1)
        row["predicted_efficiency"] = round(t1 / (n * t), 3)
        row["predicted_efficiency_min"] = round(m1 / (n * row["min_ms"]), 3)  # fastest process each
        row["cost_vs_ideal"] = round(t / (t1 / n), 3)
        if row["median_pcie_ms"]:
            p1 = rows[1]["median_pcie_ms"]
            row["predicted_pcie_inclusive_MBps"] = round((1 << 30) / (row["median_pcie_ms"] / 1e3) / 1e6, 1)
            row["predicted_pcie_efficiency"] = round(p1 / (n * row["median_pcie_ms"]), 3)
    out = {"what": "strong-scaling rehearsal on one MI355X: each N's per-rank batch (1 GiB / N in 4 MiB blocks) "
                   "as an N = 1 bench process; predicted N-GPU value = 1 GiB / per-rank step time",
           "reps": a.reps, "steps": a.steps, "rows": rows}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for n, row in rows.items():
        print(f"N={n}: {row['median_ms']} ms -> predicted {row['predicted_value_MBps']} MB/s, "
              f"efficiency {row['predicted_efficiency']}, pcie {row.get('predicted_pcie_inclusive_MBps')} "
              f"eff {row.get('predicted_pcie_efficiency')}", flush=True)


if __name__ == "__main__":
    main()
