#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
export FSAGG_ERR_LOG=$PWD/gpurun_out/r06/trimmed_err_final.jsonl
rm -f $FSAGG_ERR_LOG
bash tools/gpu_job.sh pytest smoke \
  "timeout -k 10 500 python -u tools/bench_robust.py dropin dropin_fresh > gpurun_out/r06/dropin2.jsonl" \
  "timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases2.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases2_fresh.txt 2>&1" \
  "timeout -k 10 300 python tools/probe_upload_cost.py > gpurun_out/r06/upload_cost2.json"
