set -e
timeout -k 10 200 python -u tools/stress_calgary.py 100 bwt > gpurun_out/bis_cur.log 2>&1
for c in f35772d 7644f7a 8f4863d 97b7106 144c5fc; do
  BMH_LIB=variants/at_$c/libbmh.so timeout -k 10 200 python -u tools/stress_calgary.py 100 bwt > gpurun_out/bis_$c.log 2>&1
done
for f in gpurun_out/bis_*.log; do echo $f; tail -1 $f; done
