# A/B of the working-tree extension against an older build (tools/build_alt.sh): A and C benches + A phase
# times for each.   bash tools/ab_so.sh OUT ALT_SO [--tests]
set -e
out=gpurun_out/$1; mkdir -p $out
if [ "$3" = --tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
fi
export MDA_SYNTH_BACKEND=torch
for v in new old; do
  if [ $v = old ]; then export MDA_EXT_PATH=$2; fi
  echo "== $v" >> $out/bench.log
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 >> $out/bench.log 2>&1
  timeout -k 10 200 python tools/phase_times.py MTL >> $out/bench.log 2>&1
  timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 >> $out/bench.log 2>&1
done
