#!/bin/bash
# Same-box comparison of several builds of the HIP extension, interleaved (kernel changes no class switch toggles):
#   gpurun -- 'bash tools/ab_multi.sh ROUNDS_A ROUNDS_C tree ab/_mda_hip_base.so ab/_v1.so ...'
# "tree" is the in-tree build; the others load through MDA_EXT_PATH (ops/hip.py).  Each build first prints
# the bitwise digest of 5 captured Model A steps (tools/ext_digest.py), then A (300 steps) and C (100 steps)
# benches run round-robin over the builds.
source tools/gpu_round.sh
na=${1:?}; nc=${2:?}; shift 2
run() {  # run NAME SO CMD...
  local name=$1 so=$2; shift 2
  if [ "$so" = tree ]; then step "$name" "$@"; else step "$name" env MDA_EXT_PATH="$so" "$@"; fi
}
i=0
for so in "$@"; do
  i=$((i + 1))
  TAILN=1 run dg$i "$so" timeout -k 10 300 python -u tools/ext_digest.py --model MTL || exit 1
done
for r in $(seq 1 "$na"); do
  i=0
  for so in "$@"; do
    i=$((i + 1))
    TAILN=0 run A${r}_$i "$so" timeout -k 10 300 python bench.py --steps 300 --warmup 30 || exit 1
  done
done
for r in $(seq 1 "$nc"); do
  i=0
  for so in "$@"; do
    i=$((i + 1))
    TAILN=0 run C${r}_$i "$so" timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 20 || exit 1
  done
done
i=0
for so in "$@"; do
  i=$((i + 1))
  echo "build $i = $so: A $(grep -ho '"value": [0-9.]*' gpurun_out/A*_$i.log | cut -d' ' -f2 | tr '\n' ' ')" \
       "C $(grep -ho '"value": [0-9.]*' gpurun_out/C*_$i.log | cut -d' ' -f2 | tr '\n' ' ')" \
       "$(grep -ho 'DIGEST.*' gpurun_out/dg$i.log | cut -c1-70)"
done
