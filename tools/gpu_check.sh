# One GPU call: the whole GPU test suite, then A and C benches with an optional env A/B.
#   bash tools/gpu_check.sh OUTDIR [ENVVAR]   (ENVVAR: benches run with ENVVAR=1 and ENVVAR=0)
set -e
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
for v in 1 0; do
  [ -z "$2" ] && [ $v = 0 ] && break
  env_set=${2:+$2=$v}
  echo "== ${env_set:-default}" >> $out/bench.log
  env $env_set timeout -k 10 200 python bench.py --steps 300 --warmup 30 >> $out/bench.log 2>&1
  env $env_set timeout -k 10 200 python tools/phase_times.py MTL >> $out/bench.log 2>&1
  env $env_set timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 >> $out/bench.log 2>&1
done
