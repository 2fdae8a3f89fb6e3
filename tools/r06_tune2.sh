#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
: > gpurun_out/r06/tune_wsum_sizes3.txt
steps=()
for NP in 100:1690236 100:2000000 100:4000000 100:6603900 200:6603900 50:6603900 200:1690236 100:12000000 100:14000000; do
  N=${NP%%:*}; P=${NP##*:}
  steps+=("echo N=$N P=$P >> gpurun_out/r06/tune_wsum_sizes3.txt && N=$N P=$P VARS=12,16,3,9,5,11 GRIDS=0 PVARS= NOREAD=1 ROUNDS=9 timeout -k 10 200 python tools/tune_wsum.py >> gpurun_out/r06/tune_wsum_sizes3.txt")
done
bash tools/gpu_job.sh "${steps[@]}"
