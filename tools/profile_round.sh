#!/bin/bash
# Profiling passes for one model on a GPU box (sourced by a gpurun command after tools/gpu_round.sh):
#
#   gpurun --timeout 900 -- 'source tools/gpu_round.sh; source tools/profile_round.sh; prof_model MTL A'
#
# 1. rocprofv3 --kernel-trace --stats of a short bench run      -> gpurun_out/prof_<tag>/ + kernels_<tag>.txt
# 2. one --pmc pass per counter group (rocprofv3 does not split passes; each within the per-block slot
#    limits: TCC 4 -- FETCH_SIZE uses 3, WRITE_SIZE 2 -- SQ 8, GRBM 2)  -> gpurun_out/pmc_<tag>_<group>/
# 3. tools/pmc_table.py over the passes                           -> gpurun_out/pmc_<tag>.txt
# Every rocprofv3 run has its own hard time limit (a counter request beyond the hardware's capacity hangs).
export MDA_CLEAN_EXIT=1  # bench.py: normal interpreter exit, so rocprofv3 flushes its trace
PROF_ARGS=${PROF_ARGS:-"--steps 12 --warmup 2 --no-tune --heldout 0"}
prof_model() {
  local model=$1 tag=$2
  step "prof_$tag" timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$tag" \
      -- python bench.py --model "$model" $PROF_ARGS || return 1
  step "kernels_$tag" python tools/prof_summary.py "gpurun_out/prof_$tag" 6 || return 1
  local groups=("FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU"
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE")
  local names=(fetch write mfma lds) dirs=()
  for i in 0 1 2 3; do
    step "pmc_${tag}_${names[$i]}" timeout -s KILL 120 rocprofv3 --pmc ${groups[$i]} --kernel-trace --output-format csv \
        -d "gpurun_out/pmc_${tag}_${names[$i]}" -- python bench.py --model "$model" $PROF_ARGS || return 1
    dirs+=("gpurun_out/pmc_${tag}_${names[$i]}")
  done
  TAILN=${TAILN:-15} step "pmc_$tag" python tools/pmc_table.py "${dirs[@]}" --top 15
}
