# streaming kernel with a sampled digit base: tests, then the n > 255 sweep
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "median or orderstat or trimmed or bulyan or Bulyan" > gpurun_out/t_sel.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_sel.log
[ $rc -eq 0 ] || exit $rc
KAB_VARIANTS='FSAGG_OS_UNROLL=32' timeout -k 10 300 bash tools/kab.sh orderstat_large
