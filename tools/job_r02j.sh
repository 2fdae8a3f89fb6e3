# small-bucket weighted sum (V = 1, U client rows in flight): FedAvg GPU
# tests, then the strong-scaling per-rank shares under U = 1 / 4 / 8
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fedavg or weighted or golden or wsum or server or sharded or world2" > gpurun_out/t_ws.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_ws.log
[ $rc -eq 0 ] || exit $rc
for U in 1 4 8; do
for P in 6250000 3125000; do
  for C in 4 8; do
    FSAGG_WSUM_SMALL_U=$U timeout -k 10 120 python3 bench.py --params $P --chunks $C --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/share.json 2> gpurun_out/share.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/share.json')); print('U=$U P=$P chunks=$C ms/step', d['ms_per_step'], 'kernel ms', d['per_rank_kernel_ms'])"
  done
done
done
