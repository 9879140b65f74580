# Kernel config tests, a from-scratch retune, then the A and C benches on the new table.
#   bash tools/retune_bench.sh OUT
set -e
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_cfgs_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
MDA_SYNTH_BACKEND=torch timeout -k 10 900 python -u tools/retune.py --out $out/tuned_cfgs.json > $out/retune.log 2>&1
cp $out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > $out/bench.log 2>&1
timeout -k 10 200 python tools/phase_times.py MTL >> $out/bench.log 2>&1
timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 >> $out/bench.log 2>&1
