#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_world2.py tests/test_gpu_server.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/host_tests.log 2>&1" \
  "timeout -k 10 300 python tools/bench_share.py --aggregate --world 8 > gpurun_out/r06/share_aggregate_n8_hosttab.jsonl" \
  "timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline > gpurun_out/r06/bench_hosttab.json"
