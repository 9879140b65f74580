# Round-4 GPU session helper: full GPU test suite, then A / C / B benches with phase splits.
#   gpurun --timeout 1200 -- 'bash tools/r4_gpu.sh [tests|bench|all]'
source tools/gpu_round.sh
what=${1:-all}
if [ "$what" = tests ] || [ "$what" = all ]; then
  step gputests timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 120 --timeout-method thread || exit $?
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  step benchA timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step phaseA timeout -k 10 200 python tools/phase_times.py MTL && \
  step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 && \
  step phaseC timeout -k 10 300 python tools/phase_times.py multi_classifier && \
  step benchBd timeout -k 10 200 python bench.py --model single_distance --steps 300 --warmup 30 && \
  step benchBe timeout -k 10 200 python bench.py --model single_event --steps 300 --warmup 30
fi
if [ "$what" = faults ]; then
  # runtime-fault diagnostics (docs/PERF.md "Runtime faults"): riskiest step last, the chain stops at a failure
  step hwq_default timeout -k 10 120 python -X faulthandler tools/hwq_repro.py --streams 4 && \
  step exitA timeout -k 10 200 python -X faulthandler bench.py --steps 50 --warmup 10 --heldout 0 && \
  step exitC timeout -k 10 300 python -X faulthandler bench.py --model multi_classifier --steps 20 --warmup 5 --heldout 0 && \
  step hwq2_repro env GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -X faulthandler tools/hwq_repro.py --streams 4 && \
  step hwq2_benchA env GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -X faulthandler bench.py --steps 50 --warmup 10 --heldout 0 && \
  step hwq2_benchC env GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -X faulthandler bench.py --model multi_classifier --steps 20 --warmup 5 --heldout 0
fi
if [ "$what" = retune_keep ]; then
  # fill the tuned table's missing signatures (new fused convs) by isolated timing, then bench on it
  step retune timeout -k 10 900 python -u tools/retune.py --keep --models MTL,single_event,single_distance,multi_classifier \
      --out gpurun_out/tuned_cfgs.json && cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json && \
  step benchA_rt timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step benchC_rt timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20
fi
if [ "$what" = prof ]; then
  source tools/profile_round.sh
  step prof_A timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_A \
      -- python bench.py --steps 12 --warmup 2 --no-tune --heldout 0 && \
  step kernels_A python tools/prof_summary.py gpurun_out/prof_A 6 && \
  step prof_C timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_C \
      -- python bench.py --model multi_classifier --steps 12 --warmup 2 --no-tune --heldout 0 && \
  step kernels_C python tools/prof_summary.py gpurun_out/prof_C 6 && \
  step timelineA timeout -k 10 200 python tools/timeline.py MTL
fi
