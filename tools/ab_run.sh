# A/B of an engine env switch: bitwise check + A and C benches with VAR=1 and VAR=0.  bash tools/ab_run.sh OUT VAR
set -e
out=gpurun_out/$1; mkdir -p $out
if [ "$2" = MDA_BN_FIN ]; then
  timeout -k 10 200 python tools/fin_check.py MTL 32 > $out/check.log 2>&1
  timeout -k 10 300 python tools/fin_check.py multi_classifier 8 >> $out/check.log 2>&1
fi
for v in 1 0; do
  echo "== $2=$v" >> $out/bench.log
  env $2=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 >> $out/bench.log 2>&1
  env $2=$v timeout -k 10 200 python tools/phase_times.py MTL >> $out/bench.log 2>&1
  env $2=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 >> $out/bench.log 2>&1
done
