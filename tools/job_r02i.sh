# per-rank share of the strong-scaling bench on one GPU: the fixed model's
# P/N parameters in `chunks` pipeline pieces (no collective at N=1), i.e. the
# compute side of T_N for N = 2, 4, 8
mkdir -p gpurun_out
for P in 12500000 6250000 3125000; do
  for C in 1 4 8; do
    timeout -k 10 120 python3 bench.py --params $P --chunks $C --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/share_${P}_${C}.json 2> gpurun_out/share_${P}_${C}.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/share_${P}_${C}.json')); print('P=$P chunks=$C ms/step', d['ms_per_step'], 'kernel ms', d['per_rank_kernel_ms'], 'GB/s', d['value'])"
  done
done
