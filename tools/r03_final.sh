# Round-3 evidence pass (one gpurun call): the GPU suite, smoke, the bench
# line, the robust-rule benches, kernel traces of every bench and the Krum
# PMC passes.  Summaries land in gpurun_out/ for copying into profiles/r03.
set -u
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_job.sh pytestall smoke bench "python -u tools/bench_robust.py krum orderstat orderstat_large dropin" "python -u tools/time_krum_host.py" || exit $?
bash tools/profile_all.sh || exit $?
bash tools/pmc.sh krum final
