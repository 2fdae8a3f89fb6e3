#!/bin/bash
# Host phases of Krum's distance matrix + certified selection at C4.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/time_krum_host.py > gpurun_out/krum_host.json"
