# Kernel-trace the Model A bench under several variants (env assignments), one rocprofv3 run each, and
# summarise per kernel.   bash tools/kt_variants.sh OUT "NAME1:VAR=a,VAR2=b" "NAME2:..." ...   (MODEL env: bench model)
export MDA_CLEAN_EXIT=1  # bench.py: normal interpreter exit, so rocprofv3 flushes its trace
set -e
out=gpurun_out/$1; shift; mkdir -p $out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  exports=$(echo "$envs" | tr ',' ' ')
  ( export $exports; timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $out/kt_$name -- \
      python bench.py --model ${MODEL:-MTL} --steps 20 --warmup 5 --no-tune --heldout 0 > $out/bench_$name.log 2>&1 )
  python tools/prof_summary.py $out/kt_$name > $out/kernels_$name.txt
  rm -rf $out/kt_$name
done
