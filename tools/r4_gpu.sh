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
  step hwq2_repro2 env GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -X faulthandler tools/hwq_repro.py --streams 2 && \
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
if [ "$what" = wgbig ]; then
  # large-tile weight-gradient kernels: numerics, then re-time every wgrad choice and bench before / after
  step wgtests timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py \
      -k "big or batched_wgrad" -v --timeout 120 --timeout-method thread && \
  step benchA0 timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step benchC0 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 && \
  step retune_wg timeout -k 10 900 python -u tools/retune.py --keep --drop wgrad \
      --models MTL,single_event,single_distance,multi_classifier --out gpurun_out/tuned_wg.json && \
  cp gpurun_out/tuned_wg.json mtl_das_pytorch_amd/engine/tuned_cfgs.json && \
  step benchA_wg timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step benchC_wg timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 && \
  step phaseC_wg timeout -k 10 300 python tools/phase_times.py multi_classifier && \
  step benchA_upb0 env MDA_PATCH_UPB=0 timeout -k 10 200 python bench.py --steps 300 --warmup 30
fi
if [ "$what" = upb ]; then
  # same-box A/B of the patch wgrad unit cap (ops/functional.py PATCH_MAX_UNITS)
  for r in 1 2; do
    for u in 3 0; do
      step benchA_upb${u}_$r env MDA_PATCH_UPB=$u timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
    done
  done
  for u in 3 0; do
    step benchC_upb${u} env MDA_PATCH_UPB=$u timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
fi
if [ "$what" = wgassign ]; then
  step wgassignC timeout -k 10 400 python -u tools/wgrad_assign.py multi_classifier table,big,table,big --min-px 256,1024 && \
  step wgassignA timeout -k 10 300 python -u tools/wgrad_assign.py MTL table,big,bigall --min-px 256
fi
if [ "$what" = wgtune ]; then
  # weight-gradient configs chosen by their batched launches' time, then A / C benches on the new table
  step benchA_pre timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
  step benchC_pre timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
  step wgtune timeout -k 10 900 python -u tools/retune.py --keep --wgrad-batches \
      --models MTL,multi_classifier --out gpurun_out/tuned_wgb.json && \
  cp gpurun_out/tuned_wgb.json mtl_das_pytorch_amd/engine/tuned_cfgs.json && \
  step benchA_wgb timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
  step benchC_wgb timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
  step wgjobsC timeout -k 10 300 python tools/wgrad_assign.py multi_classifier table --min-px 256
fi
if [ "$what" = spill ]; then
  # share of stream 0's weight gradients moved to the spill stream (engine/lowering.py spill_wgrads)
  for f in 0 0.3 0.5 0.7 0.85 0; do
    step benchA_spill$f env MDA_WGSPILL=$f timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
  done
  for f in 0 0.5 0.7 0.9 0; do
    step benchC_spill$f env MDA_WGSPILL=$f timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
fi
if [ "$what" = spill2 ]; then
  # spilled weight gradients with their blocks per CU capped by extra LDS (MDA_SPILL_LDS bytes)
  for cfg in "0 0" "0.5 98304" "0.85 98304" "0.85 65536" "0.5 65536" "0.85 0" "0 0"; do
    set -- $cfg
    step benchA_spill$1_lds$2 env MDA_WGSPILL=$1 MDA_SPILL_LDS=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
  done
fi
if [ "$what" = spill3 ]; then
  for f in 0 0.5 0.7 0.85 0; do
    step benchA_sp$f env MDA_WGSPILL=$f MDA_SPILL_LDS=0 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
  done
  step benchA_sp0.7_lds env MDA_WGSPILL=0.7 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
  MDA_WGSPILL=0.7 MDA_SPILL_LDS=0 step tl_sp70 timeout -k 10 200 python tools/timeline.py MTL bwd,adam && \
  for f in 0 0.7 0.9; do
    step benchC_sp$f env MDA_WGSPILL=$f MDA_SPILL_LDS=0 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
fi
if [ "$what" = wg0 ]; then
  for v in 0 1 0 1; do
    step benchA_wg0_$v env MDA_WG_STREAM0=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
  done
  for v in 0 1; do
    step benchC_wg0_$v env MDA_WG_STREAM0=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
fi
if [ "$what" = opt ]; then
  step opttests timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_rccl_gpu.py tests/test_mtl_layer_local_gpu.py \
      -x -v --timeout 120 --timeout-method thread && \
  step rccl2 timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 120 --timeout-method thread && \
  step rccl3 timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 120 --timeout-method thread && \
  step inc timeout -k 10 300 python -u -m pytest tests/test_inception_gpu.py -x -v --timeout 120 --timeout-method thread && \
  step benchA timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
  step phaseA timeout -k 10 200 python tools/phase_times.py MTL && \
  step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
  step phaseC timeout -k 10 300 python tools/phase_times.py multi_classifier
fi
if [ "$what" = scratch ]; then
  # verdict item 7: the whole table re-derived from an EMPTY table (isolated, then in-context for A and C)
  step scratch timeout -k 10 1100 python -u tools/retune.py --models MTL,single_event,single_distance,multi_classifier \
      --in-context --topk 3 --passes cfg,tail --out gpurun_out/tuned_scratch.json && \
  cp gpurun_out/tuned_scratch.json mtl_das_pytorch_amd/engine/tuned_scratch.json && \
  for r in 1 2; do
    step benchA_ship$r timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
    step benchA_scr$r env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_scratch.json timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
  done
fi
if [ "$what" = scratch_ab ]; then
  # shipped table vs the from-scratch one, interleaved on one box
  for r in 1 2; do
    step benchA_ship$r timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
    step benchA_scr$r env MDA_TUNED_CFGS=gpurun_out/tuned_scratch.json timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
    step benchC_ship$r timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
    step benchC_scr$r env MDA_TUNED_CFGS=gpurun_out/tuned_scratch.json timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
fi
if [ "$what" = acc ]; then
  step accuracy timeout -k 10 1100 python -u tools/accuracy_table.py --out gpurun_out/accuracy
fi
if [ "$what" = tailab ]; then
  for r in 1 2 3; do
    for v in 0 1; do
      step benchC_tb${v}_$r env MDA_TAIL_BATCH=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
    done
  done
  for v in 0 1; do
    step phaseC_tb$v env MDA_TAIL_BATCH=$v timeout -k 10 300 python tools/phase_times.py multi_classifier || exit $?
  done
fi
if [ "$what" = scratch2 ]; then
  # second from-scratch stage: batch-level weight-gradient configs and a wider in-context search on top of
  # the isolated-only scratch table (no shipped-table input)
  step scratch2 env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_scratch.json timeout -k 10 1000 python -u tools/retune.py \
      --keep --wgrad-batches --in-context --topk 6 --margin 0.001 --reps 30 --passes cfg,xcd,tail \
      --models MTL,single_event,single_distance,multi_classifier --out gpurun_out/tuned_scratch2.json && \
  cp gpurun_out/tuned_scratch2.json mtl_das_pytorch_amd/engine/tuned_scratch2.json && \
  for r in 1 2; do
    step benchA_ship$r timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
    step benchA_scr2_$r env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_scratch2.json timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 || exit $?
  done
fi
if [ "$what" = wgb ]; then
  # weight-gradient configs chosen by their batched launches' time on top of the shipped table, then A/B
  step wgb timeout -k 10 600 python -u tools/retune.py --keep --wgrad-batches --models MTL,multi_classifier \
      --out gpurun_out/tuned_wgb2.json && \
  cp gpurun_out/tuned_wgb2.json mtl_das_pytorch_amd/engine/tuned_wgb2.json && \
  for r in 1 2; do
    step benchA_ship$r timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
    step benchA_wgb$r env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_wgb2.json timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
    step benchC_ship$r timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
    step benchC_wgb$r env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_wgb2.json timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
fi
if [ "$what" = accev_prof ]; then
  for sd in 0 1 2; do
    step accuracy_ev$sd timeout -k 10 300 python -X faulthandler -u tools/accuracy_table.py --rows A,B_distance,C --seeds $sd \
        --out gpurun_out/accuracy_ev$sd || exit $?
  done

  source tools/profile_round.sh && \
  prof_model MTL A && prof_model multi_classifier C
fi
if [ "$what" = gclear ]; then
  step gctests timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py tests/test_rccl_gpu.py \
      tests/test_guard_gpu.py tests/test_mtl_layer_local_gpu.py tests/test_inference_gpu.py -x -v --timeout 120 --timeout-method thread && \
  step benchA1 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
  step benchA2 timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step phaseA timeout -k 10 200 python tools/phase_times.py MTL && \
  step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
  step phaseC timeout -k 10 300 python tools/phase_times.py multi_classifier
fi
if [ "$what" = tbwd ]; then
  step tbtests timeout -k 10 400 python -u -m pytest tests/test_inception_gpu.py tests/test_rccl_gpu.py -x -v --timeout 120 --timeout-method thread && \
  for r in 1 2; do
    for v in 0 1; do
      step benchC_tbw${v}_$r env MDA_TAIL_BATCH=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
    done
  done
  step phaseC timeout -k 10 300 python tools/phase_times.py multi_classifier
fi
if [ "$what" = final ]; then
  step gputests timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=5 -q --timeout 120 --timeout-method thread && \
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
  step benchA1 timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step benchA2 timeout -k 10 200 python bench.py && \
  step benchBe timeout -k 10 200 python bench.py --model single_event --steps 300 --warmup 30 --heldout 0 && \
  step benchBd timeout -k 10 200 python bench.py --model single_distance --steps 300 --warmup 30 --heldout 0 && \
  step benchC1 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 && \
  step benchC2 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
  step phaseA timeout -k 10 200 python tools/phase_times.py MTL && \
  step phaseC timeout -k 10 300 python tools/phase_times.py multi_classifier && \
  export MDA_CLEAN_EXIT=1 && \
  step prof_C timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_C \
      -- python bench.py --model multi_classifier --steps 12 --warmup 2 --no-tune --heldout 0 && \
  step kernels_C python tools/prof_summary.py gpurun_out/prof_C 6
fi
if [ "$what" = final2 ]; then
  step benchA1 timeout -k 10 200 python bench.py --steps 300 --warmup 30 && \
  step benchA2 timeout -k 10 200 python bench.py && \
  step benchBe timeout -k 10 200 python bench.py --model single_event --steps 300 --warmup 30 --heldout 0 && \
  step benchBd timeout -k 10 200 python bench.py --model single_distance --steps 300 --warmup 30 --heldout 0 && \
  step benchC1 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 && \
  step phaseA timeout -k 10 200 python tools/phase_times.py MTL && \
  step engtests timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_mtl_layer_local_gpu.py tests/test_rccl_gpu.py -q -x --timeout 120 --timeout-method thread
fi
if [ "$what" = wgbig2 ]; then
  step wgb3 timeout -k 10 600 python -u tools/retune.py --keep --wgrad-batches --wgrad-big-init --models multi_classifier \
      --out gpurun_out/tuned_wgb3.json && \
  cp gpurun_out/tuned_wgb3.json mtl_das_pytorch_amd/engine/tuned_wgb3.json && \
  for r in 1 2 3; do
    step benchC_ship$r timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 && \
    step benchC_wgb3_$r env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_wgb3.json timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
  done
  step wgassign_ship timeout -k 10 300 python tools/wgrad_assign.py multi_classifier table && \
  step wgassign_wgb3 env MDA_TUNED_CFGS=mtl_das_pytorch_amd/engine/tuned_wgb3.json timeout -k 10 300 python tools/wgrad_assign.py multi_classifier table
fi
if [ "$what" = final3 ]; then
  step gputests timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=5 -q --timeout 120 --timeout-method thread && \
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
  step benchA timeout -k 10 200 python bench.py && \
  step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20
fi
if [ "$what" = sidefin ]; then
  for r in 1 2; do
    for v in 0 1; do
      step benchA_sf${v}_$r env MDA_SIDE_FINALIZE=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --heldout 0 && \
      step benchC_sf${v}_$r env MDA_SIDE_FINALIZE=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 --heldout 0 || exit $?
    done
  done
fi
if [ "$what" = sidefin2 ]; then
  for r in 1 2 3; do
    for v in 1 0; do
      step benchC_sfb${v}_$r env MDA_SIDE_FINALIZE=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 200 --warmup 20 --heldout 0 || exit $?
    done
  done
  for v in 1 0; do
    step benchA_sfb${v} env MDA_SIDE_FINALIZE=$v timeout -k 10 200 python bench.py --steps 500 --warmup 30 --heldout 0 || exit $?
  done
fi
if [ "$what" = early ]; then
  step eatests timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_rccl_gpu.py tests/test_inception_gpu.py \
      tests/test_mtl_layer_local_gpu.py -x -v --timeout 120 --timeout-method thread && \
  for r in 1 2 3; do
    for v in 1 0; do
      step benchC_ea${v}_$r env MDA_EARLY_ADAM=$v timeout -k 10 300 python bench.py --model multi_classifier --steps 200 --warmup 20 --heldout 0 || exit $?
    done
  done
  for v in 1 0; do
    step benchA_ea${v} env MDA_EARLY_ADAM=$v timeout -k 10 200 python bench.py --steps 500 --warmup 30 --heldout 0 || exit $?
  done
fi
if [ "$what" = earlyA ]; then
  for r in 1 2 3; do
    for v in 1 0; do
      step benchA_eb${v}_$r env MDA_EARLY_ADAM=$v timeout -k 10 200 python bench.py --steps 500 --warmup 30 --heldout 0 || exit $?
    done
  done
fi
if [ "$what" = accfinal ]; then
  for sd in 0 1 2; do
    step accf$sd timeout -k 10 400 python -X faulthandler -u tools/accuracy_table.py --seeds $sd --out gpurun_out/accf$sd || exit $?
  done
fi
