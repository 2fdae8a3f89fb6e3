#!/bin/bash
# new flat weighted-sum width rule: tests, the layout-B probe with row-set
# widths, a bench line without PMC / CPU baseline
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rows.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/width_tests.log 2>&1" \
  "timeout -k 10 400 python tools/probe_layout_b.py --rows-widths 0,24,8 > gpurun_out/r06/layout_b_widths.jsonl" \
  "timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline > gpurun_out/r06/bench_width.json 2> gpurun_out/r06/bench_width.log"
