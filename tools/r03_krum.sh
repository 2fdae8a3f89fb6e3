set -u
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_job.sh "python -u -m pytest tests/test_gpu_pairgram.py -v --timeout 120 --timeout-method thread" "python -u tools/bench_robust.py krum"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_krum -o run -- python3 $R/tools/bench_robust.py krum > $R/gpurun_out/krum_prof.log 2>&1
