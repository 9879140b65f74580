source tools/gpu_round.sh
export TAILN=1
for f in 0 0.3 0.5 0.7 0.85; do
  MDA_WGRAD_STAGE=$f step stage_$f timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
done
