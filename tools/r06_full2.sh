#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall smoke
cp gpurun_out/pytest_gpu.log gpurun_out/r06/pytest_gpu_full2.log
