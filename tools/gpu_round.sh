#!/bin/bash
# Step runner for GPU-box sessions (sourced by the one-line commands given to gpurun):
#
#   gpurun --timeout 900 -- 'source tools/gpu_round.sh; \
#       step gpu   timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
#       step bench timeout -k 10 300 python bench.py'
#
# Each step writes gpurun_out/<name>.log, prints its last $TAILN lines and stops the session at the first
# failure (so nothing else touches the GPU after a fault or a time limit).  Every GPU step carries its own
# `timeout -k`.
set -o pipefail
mkdir -p gpurun_out
step() {
  local name=$1; shift
  echo "== $name"
  "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -"${TAILN:-15}" "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; exit $rc; fi
}
