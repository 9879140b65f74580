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
