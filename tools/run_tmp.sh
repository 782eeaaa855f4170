bash tools/gpu_round.sh r3a || exit 1
timeout -k 10 100 python3 tools/calgary_prof.py --mode whole > gpurun_out/cal_whole.json
timeout -k 10 100 python3 tools/calgary_prof.py --mode 256k > gpurun_out/cal_256k.json
python3 -c "
import json
for f in ['cal_whole','cal_256k']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['ms'])"
