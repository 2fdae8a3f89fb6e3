#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_orderstat_pair.py tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_rows.py tests/test_gpu_fullsize.py tests/test_gpu_pairgram.py -x -v --timeout 120 --timeout-method thread -k 'pair or median or trimmed or refinement or nonfinite or bulyan or order or c5 or repair'" \
  "bash tools/r05_ab_os.sh"
