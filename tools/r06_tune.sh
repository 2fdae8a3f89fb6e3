#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
: > gpurun_out/r06/tune_wsum_sizes.txt
steps=()
for P in 8000000 12000000 15000000 18000000 20000000 23520848 25000000 28000000 32000000; do
  steps+=("echo P=$P >> gpurun_out/r06/tune_wsum_sizes.txt && P=$P VARS=3,9,5,11 GRIDS=0 PVARS= NOREAD=1 ROUNDS=9 timeout -k 10 200 python tools/tune_wsum.py >> gpurun_out/r06/tune_wsum_sizes.txt")
done
bash tools/gpu_job.sh "${steps[@]}"
