# GPU-box A/B runner for the performance work (docs/PERF.md).  All output goes to gpurun_out/OUT/.
#
#   bash tools/gpu_ab.sh env   OUT VAR            A and C benches (+ A phase times) with VAR=1 and VAR=0
#   bash tools/gpu_ab.sh so    OUT ALT.so         ... with the working-tree extension and an older build
#                                                 (tools/build_alt.sh REV; loaded through MDA_EXT_PATH)
#   bash tools/gpu_ab.sh table OUT ALT.json       ... with the shipped tuned table and an alternative one
#   bash tools/gpu_ab.sh retune OUT               conv config tests, a from-scratch retune, benches on it
#
# Every GPU step has its own time limit and the steps are chained with set -e (a failure ends the run).
set -e
mode=$1; out=gpurun_out/$2; arg=$3
mkdir -p $out
export MDA_SYNTH_BACKEND=${MDA_SYNTH_BACKEND:-torch}   # the same data for every variant (and older builds)

benches() {  # $1: label
  echo "== $1" >> $out/bench.log
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 >> $out/bench.log 2>&1
  timeout -k 10 200 python tools/phase_times.py MTL >> $out/bench.log 2>&1
  timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 >> $out/bench.log 2>&1
}

case $mode in
  env)
    for v in 1 0; do ( export $arg=$v; benches "$arg=$v" ); done ;;
  so)
    benches new
    ( export MDA_EXT_PATH=$arg; benches "old ($arg)" ) ;;
  table)
    benches shipped
    cp $arg mtl_das_pytorch_amd/engine/tuned_cfgs.json
    benches "$arg" ;;
  retune)
    timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_cfgs_gpu.py tests/test_kernels_gpu.py -x -q \
      --timeout 120 --timeout-method thread > $out/tests.log 2>&1
    timeout -k 10 900 python -u tools/retune.py --out $out/tuned_cfgs.json > $out/retune.log 2>&1
    cp $out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
    benches retuned ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
