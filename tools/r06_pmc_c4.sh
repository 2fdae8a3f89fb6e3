#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh "timeout -k 10 500 bash tools/pmc_gram2.sh c4_stages tools/ab_gram_stages.py 50"
