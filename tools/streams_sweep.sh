set -e
for s in 1 2 3 4 6 8; do
  echo "streams=$s"
  BMH_STREAMS=$s timeout -k 10 100 python3 tools/text_bench.py 100 1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('  zipf100m/1m', d['ms'], 'ms', d['MBps'], 'MB/s')"
  BMH_STREAMS=$s timeout -k 10 100 python3 tools/text_bench.py 128 16 | python3 -c "import json,sys; d=json.load(sys.stdin); print('  zipf128m/16m', d['ms'], 'ms', d['MBps'], 'MB/s')"
  BMH_STREAMS=$s timeout -k 10 100 python3 tools/calgary_prof.py --mode whole | python3 -c "import json,sys; d=json.load(sys.stdin); print('  calgary whole', d['ms'], 'ms')"
done
