# round-2 GPU pass: sanity (smoke, GPU tests, bench), Krum operand-read A/B,
# drop-in host phases, the n > 255 order-statistic sweep
bash tools/gpu_job.sh smoke pytest bench && \
KAB_VARIANTS='FSAGG_NONE=0|FSAGG_PAIR_LDS=dsr|FSAGG_NONE=0|FSAGG_PAIR_LDS=dsr' timeout -k 10 400 bash tools/kab.sh krum > gpurun_out/kab_krum.txt 2>&1 && \
timeout -k 10 120 python3 tools/time_dropin_host.py > gpurun_out/dropin_host.txt 2>&1 && \
timeout -k 10 300 python3 tools/bench_robust.py orderstat_large > gpurun_out/os_large.jsonl 2> gpurun_out/os_large.err
