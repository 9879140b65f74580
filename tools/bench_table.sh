# A and C benches with the shipped tuned table and with an alternative one.   bash tools/bench_table.sh OUT ALT.json
set -e
out=gpurun_out/$1; mkdir -p $out
for t in shipped alt; do
  if [ $t = alt ]; then cp $2 mtl_das_pytorch_amd/engine/tuned_cfgs.json; fi
  echo "== $t" >> $out/bench.log
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 >> $out/bench.log 2>&1
  timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 >> $out/bench.log 2>&1
done
