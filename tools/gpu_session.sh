#!/bin/bash
# Generic GPU-box session for the performance / validation work (replaces the round-specific tools/r4_gpu.sh).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_session.sh MODE [ARGS...]'
#
# MODE
#   tests                       the whole GPU suite (pytest -m gpu)
#   bench  [N]                  N x (A, C, B_event, B_distance) benches (default 1), plus A/C phase splits
#   ab  "SPEC_A" "SPEC_B" [N] [MODELS]
#                               N interleaved pairs of bench runs per model (default 2; MODELS default "MTL
#                               multi_classifier") under two sets of class-switch overrides, e.g.
#                               ab "" "engine.mtl.MTLProgram.SIDE_WGRAD_GRID=0" 3 MTL      (tools/variant.py)
#   dp                          the per-rank program of an 8-GPU run on a 1-rank RCCL group (bench --dp-shape 8)
#                               next to the single-GPU benches, A and C
#   prof   [MODEL TAG]          rocprofv3 kernel table + counter passes (tools/profile_round.sh)
#   timeline [MODEL]            tools/timeline.py and tools/kernel_phases.py (in-step phase timers)
#   faults                      HIP-runtime fault diagnostics; the riskiest step last
#   multiprog                   the round-4 crash sequence: 6 programs trained + evaluated in one process
#   retune [OUT]                conv config tests, a from-scratch retune (tools/retune.py), benches on it
#
# Every GPU step runs under its own time limit and the steps are chained: the first failure (a fault, a
# time limit) ends the session (tools/gpu_round.sh `step`).  Outputs: gpurun_out/<step>.log.
source tools/gpu_round.sh
mode=${1:-bench}
shift || true
V="python tools/variant.py"

bench_model() {  # name model extra-args...
  local name=$1 model=$2; shift 2
  local steps="--steps 300 --warmup 30"
  [ "$model" = multi_classifier ] && steps="--steps 100 --warmup 20"
  TAILN=${TAILN:-2} step "$name" timeout -k 10 300 python bench.py --model "$model" $steps "$@"
}

case $mode in
  tests)
    step gputests timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread ;;
  bench)
    n=${1:-1}
    for i in $(seq 1 "$n"); do
      bench_model "A_$i" MTL && bench_model "C_$i" multi_classifier && \
      bench_model "Be_$i" single_event && bench_model "Bd_$i" single_distance || exit $?
    done
    step phaseA timeout -k 10 200 python tools/phase_times.py MTL && \
    step phaseC timeout -k 10 300 python tools/phase_times.py multi_classifier ;;
  ab)
    a=$1; b=$2; n=${3:-2}; models=${4:-"MTL multi_classifier"}
    for m in $models; do
      steps="--steps 300 --warmup 30"
      [ "$m" = multi_classifier ] && steps="--steps 100 --warmup 20"
      for i in $(seq 1 "$n"); do
        TAILN=1 step "ab_${m}_A$i" timeout -k 10 300 $V $a -- --model "$m" $steps && \
        TAILN=1 step "ab_${m}_B$i" timeout -k 10 300 $V $b -- --model "$m" $steps || exit $?
      done
    done ;;
  dp)
    # the per-rank program of an 8-GPU run on a 1-rank RCCL group (bench --dp-shape 8): the model's bucket count
    # (A: 2 side-stream buckets behind external events) vs one bucket, next to the single-GPU benches
    bench_model A1 MTL && \
    TAILN=2 step A_w8 env MDA_DIST_BACKEND=nccl timeout -k 10 300 python bench.py --steps 300 --warmup 30 --dp-shape 8 && \
    TAILN=2 step A_w8b1 env MDA_DIST_BACKEND=nccl timeout -k 10 300 python bench.py --steps 300 --warmup 30 --dp-shape 8 --buckets 1 && \
    TAILN=2 step A_w8sbn env MDA_DIST_BACKEND=nccl timeout -k 10 300 python bench.py --steps 300 --warmup 30 --dp-shape 8 --sync_bn && \
    bench_model C1 multi_classifier && \
    TAILN=2 step C_w8 env MDA_DIST_BACKEND=nccl timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --dp-shape 8 && \
    TAILN=2 step C_w8sbn env MDA_DIST_BACKEND=nccl timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --dp-shape 8 --sync_bn ;;
  prof)
    source tools/profile_round.sh
    prof_model "${1:-MTL}" "${2:-A}" ;;
  timeline)
    m=${1:-MTL}
    step "timeline_$m" timeout -k 10 200 python tools/timeline.py "$m" && \
    step "phases_$m" timeout -k 10 300 python tools/kernel_phases.py "$m" --all ;;
  faults)
    step hwq_default timeout -k 10 120 python -X faulthandler tools/hwq_repro.py --streams 4 && \
    step hwq2_repro2 env GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -X faulthandler tools/hwq_repro.py --streams 2 && \
    step hwq2_benchA env GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -X faulthandler bench.py --steps 50 --warmup 10 --heldout 0 && \
    step hwq2_benchC env GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -X faulthandler bench.py --model multi_classifier --steps 20 --warmup 5 --heldout 0 ;;
  multiprog)
    step multiprog timeout -k 10 900 python -X faulthandler tools/accuracy_table.py --rows A,B_distance,C --seeds 0,1 \
        --out gpurun_out/multiprog ;;
  retune)
    out=${1:-gpurun_out/tuned_cfgs.json}
    step retune_tests timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_cfgs_gpu.py tests/test_kernels_gpu.py -x -q \
        --timeout 120 --timeout-method thread && \
    step retune timeout -k 10 900 python -u tools/retune.py --out "$out" && \
    cp "$out" mtl_das_pytorch_amd/engine/tuned_cfgs.json && \
    bench_model A_retuned MTL && bench_model C_retuned multi_classifier ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
