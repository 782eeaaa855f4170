export TMPDIR=/tmp
ALL="bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans"
for r in 1 2; do
for s in 2 3; do
  echo "streams $s"
  BMH_STREAMS=$s timeout -k 10 60 python3 tools/cal_subset_time.py $ALL || exit 1
  BMH_STREAMS=$s timeout -k 10 100 python3 tools/text_bench.py 100 1 > gpurun_out/t100_$s.json || exit 1
  BMH_STREAMS=$s timeout -k 10 100 python3 tools/text_bench.py 128 16 > gpurun_out/t128_$s.json || exit 1
  BMH_STREAMS=$s timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > gpurun_out/b_$s.json 2>/dev/null || exit 1
  python3 -c "
import json
for f in ['t100_$s','t128_$s']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['ms'], d['MBps'], d.get('parity'))
d=json.loads(open('gpurun_out/b_$s.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'])"
done
done
