#!/bin/bash
# last check of the final tree: the GPU suite, smoke, the default bench line
set -u
cd "$(dirname "$0")/.."
F=gpurun_out/r06/last
mkdir -p $F
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall smoke \
  "timeout -k 10 400 python bench.py > $F/bench.json 2> $F/bench.log"
rc=$?
cp gpurun_out/pytest_gpu.log $F/pytest_gpu.log
cp gpurun_out/smoke.log $F/smoke.log
exit $rc
