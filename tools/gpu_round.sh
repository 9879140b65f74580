#!/bin/bash
# One GPU-box session: tests, bench, profile.  Every GPU step has its own time limit; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; echo "== $name"; "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -${TAILN:-15} gpurun_out/$name.log; if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; exit $rc; fi; }
