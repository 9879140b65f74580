#!/bin/bash
# Same-box A/B of the world > 1 all-reduce issue form on the per-rank program of 8 GPUs (1-rank RCCL,
# bench.py --dp-shape 8): FlatGradAllReducer default (async work per bucket) vs ON_COMM_STREAM.
source tools/gpu_round.sh
V="python tools/variant.py"
for m in MTL multi_classifier; do
  steps="--steps 300 --warmup 30"; [ $m = multi_classifier ] && steps="--steps 100 --warmup 20"
  for i in 1 2; do
    TAILN=1 step comm_${m}_A$i env MDA_DIST_BACKEND=nccl timeout -k 10 300 python bench.py --model $m $steps --dp-shape 8 || exit 1
    TAILN=1 step comm_${m}_B$i env MDA_DIST_BACKEND=nccl timeout -k 10 300 $V parallel.dist.FlatGradAllReducer.ON_COMM_STREAM=True -- --model $m $steps --dp-shape 8 || exit 1
  done
done
