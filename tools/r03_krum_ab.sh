# Round-3 job: Krum Gram path — GPU tests, C4 bench twice, kernel trace.
set -u
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_job.sh "python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_golden.py -q --timeout 120 --timeout-method thread" "python -u tools/bench_robust.py krum" "python -u tools/bench_robust.py krum" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_krum -o run -- python3 $R/tools/bench_robust.py krum > $R/gpurun_out/krum_prof.log 2>&1
