# stream kernel load depth A/B; Krum/Bulyan drop-ins with the init table
# built under the distance kernels
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "median or orderstat or trimmed or krum or Krum or bulyan or Bulyan" > gpurun_out/t_sel.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_sel.log
[ $rc -eq 0 ] || exit $rc
KAB_VARIANTS='FSAGG_OS_UNROLL=16|FSAGG_OS_UNROLL=32|FSAGG_OS_UNROLL=64' timeout -k 10 600 bash tools/kab.sh orderstat_large
timeout -k 10 300 python3 tools/bench_robust.py dropin > gpurun_out/dropin.jsonl 2> gpurun_out/dropin.err; echo "dropin rc=$?"; cut -c1-100 gpurun_out/dropin.jsonl
