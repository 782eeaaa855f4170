set -e
export TMPDIR=/tmp
for cfg in "BMH_MTF_CHUNK=4096 BMH_STREAM_BATCH=268435456" "BMH_STREAM_BATCH=268435456" "BMH_MTF_CHUNK=4096 BMH_STREAM_BATCH=67108864" "BMH_STREAM_BATCH=67108864"; do
  env $cfg timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --calgary-steps 0 --pcie-steps 5 > gpurun_out/ab.json 2>/dev/null
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); p=d['pcie_inclusive']; print(sys.argv[1], p['value'], p['ms_per_step'])" "$cfg"
done
