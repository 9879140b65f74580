#!/bin/bash
# A/B of two builds of the HIP extension on one box (kernel changes that no class switch can toggle):
#
#   gpurun -- 'bash tools/ab_ext.sh ab/_mda_hip_base.so [pairs A] [pairs C] [pytest files...]'
#
# Build the baseline from a clean tree first (git worktree add /tmp/base HEAD; python -m
# mtl_das_pytorch_amd.csrc.build there; copy its _mda_hip*.so to ab/).  The in-tree build is "new", the other
# one is loaded through MDA_EXT_PATH (ops/hip.py).  Optional pytest files run first against the new build.
source tools/gpu_round.sh
base=${1:?baseline .so}; na=${2:-3}; nc=${3:-2}; shift 3 || shift $#
if [ $# -gt 0 ]; then
  step t_new timeout -k 10 800 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread || exit 1
fi
for i in $(seq 1 "$na"); do
  TAILN=1 step abA_new$i timeout -k 10 300 python bench.py --steps 300 --warmup 30 || exit 1
  TAILN=1 step abA_base$i env MDA_EXT_PATH="$base" timeout -k 10 300 python bench.py --steps 300 --warmup 30 || exit 1
done
for i in $(seq 1 "$nc"); do
  TAILN=1 step abC_new$i timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 || exit 1
  TAILN=1 step abC_base$i env MDA_EXT_PATH="$base" timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 || exit 1
done
