#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh "timeout -k 10 300 python tools/probe_upload_cost.py > gpurun_out/r06/upload_cost.json"
