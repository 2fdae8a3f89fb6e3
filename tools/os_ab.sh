set -u
R=$GRAFT_REPO_ROOT
cd $R
P=$R/tools/probe/lib/libfsagg.so
bash tools/gpu_job.sh "python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rows.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -q --timeout 120 --timeout-method thread -k 'median or trimmed or orderstat or bulyan'" "python -u tools/bench_robust.py orderstat" "FSAGG_LIB=$P python -u tools/bench_robust.py orderstat" "python -u tools/bench_robust.py orderstat" "FSAGG_LIB=$P python -u tools/bench_robust.py orderstat"
