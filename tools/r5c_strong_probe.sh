export TMPDIR=/tmp
o=gpurun_out/r5c; mkdir -p $o
for p in 1 2 3 4; do
  timeout -k 10 120 python3 bench.py --total-bytes $((128<<20)) --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --pipelines $p > $o/b$p.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$o/b$p.json').read().strip().splitlines()[-1]); print('pipes $p', d['ms_per_step'], d['parity'][:6], d['host_wall_ms_per_step'])"
done
for p in 1 4; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t$p -o run --output-format csv -- python3 tools/trace_run.py 128 4 3 pipelines=$p > $o/t$p.log 2>&1 || exit 1
  python3 tools/stream_trace.py $o/t$p 3 > $o/s$p.txt; cat $o/t$p.log | tail -1; cat $o/s$p.txt
done
