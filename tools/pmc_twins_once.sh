source tools/gpu_round.sh
export MDA_CLEAN_EXIT=1
PA="--steps 12 --warmup 2 --no-tune --heldout 0"
step pmc_ship timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_ship -- python bench.py $PA || exit 1
MDA_TUNED_CFGS=tools/tables/tuned_leanbig_twins.json step pmc_twin timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_twin -- python bench.py $PA || exit 1
TAILN=12 step pmc_ship_t python tools/pmc_table.py gpurun_out/pmc_ship --top 6 && TAILN=12 step pmc_twin_t python tools/pmc_table.py gpurun_out/pmc_twin --top 6
