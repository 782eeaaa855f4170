set -e
mkdir -p gpurun_out/mtfsw
for c in 0 2048 1024; do
  for cfg in "100 1" "128 16"; do
    if [ $c = 0 ]; then timeout -k 10 120 python3 tools/text_bench.py $cfg > gpurun_out/mtfsw/t_${c}_${cfg// /_}.json
    else timeout -k 10 120 python3 tools/text_bench.py $cfg mtf_chunk=$c > gpurun_out/mtfsw/t_${c}_${cfg// /_}.json; fi
  done
done
python3 - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/mtfsw/*.json")):
    d=json.load(open(f)); k=d["kernels"] if "kernels" in d else d.get("kernels_ms",{})
    print(f.split('/')[-1], d["ms"], "ms", d.get("parity"), {x:k[x] for x in k if "mtf" in x})
P
