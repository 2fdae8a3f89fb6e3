set -u
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_job.sh bench
cp gpurun_out/bench.log gpurun_out/bench_default.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --no-pmc --no-cpu-baseline > $R/gpurun_out/bench_prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b64 -o run -- python3 $R/tools/bench_b64.py --uploads 8 --distinct 8 --reps 2 > $R/gpurun_out/b64_prof.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python3 tools/bench_share.py --world 8 --splits uniform4,taper0.5x4,4/3/2/1 --rates 0,350,550 > gpurun_out/rccl_share8.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_share.py --world 4 --splits uniform4,taper0.5x4 --rates 0,350,550 > gpurun_out/rccl_share4.log 2>&1 || exit $?
