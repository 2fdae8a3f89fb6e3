#!/bin/bash
# the l2 metric's partial kernel with 16 loads in flight per lane
set -u
cd "$(dirname "$0")/.."
F=gpurun_out/r06/l2
mkdir -p $F
export TMPDIR=/tmp
P=/tmp/r06l2
bash tools/gpu_job.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- python tools/bench_wire.py dissim > $F/dissim_traced.jsonl"
rc=$?
find $P -name '*kernel_stats.csv' -exec cp {} $F/dissim_kernel_stats.csv \; 2>/dev/null
exit $rc
