#!/bin/bash
# Interleaved A/B of the order-statistic kernels: the previous commit's
# library (tools/probe/old, FSAGG_LIB) against the working tree's, each
# running tools/bench_pair.py (one-wave vs two-wave in-process), two rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then L=tools/probe/old/libfsagg.so; else L=federatedscope_amd/lib/libfsagg.so; fi
    FSAGG_LIB=$L timeout -k 10 200 python -u tools/bench_pair.py 128 200 255 \
      | sed "s/^{/{\"lib\": \"$lib\", \"round\": $r, /" >> gpurun_out/ab_os.jsonl || exit $?
  done
done
