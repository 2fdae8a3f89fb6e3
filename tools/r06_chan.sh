#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh "timeout -k 10 400 python tools/probe_channels.py > gpurun_out/r06/probe_channels.jsonl"
