# streaming order-statistic kernel (n > 255): GPU tests, then the n > 255
# sweep and the C5 regression check; Krum tests under the ds_read_b64 form
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "median or orderstat" > gpurun_out/t_os.log 2>&1; rc=$?; echo "os tests rc=$rc"; tail -3 gpurun_out/t_os.log
[ $rc -eq 0 ] || exit $rc
FSAGG_PAIR_LDS=dsr timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "krum or pairdist or bulyan or Krum or fullsize" > gpurun_out/t_krum.log 2>&1; rc=$?; echo "krum dsr tests rc=$rc"; tail -3 gpurun_out/t_krum.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 tools/bench_robust.py orderstat_large orderstat > gpurun_out/os_large.jsonl 2> gpurun_out/os_large.err; echo "bench rc=$?"
cat gpurun_out/os_large.jsonl | cut -c1-200
