# strong-scaling pipeline pieces on side streams: the per-rank share on one
# GPU (P/N parameters, C pieces, S streams; no collective at N = 1)
mkdir -p gpurun_out
for cfg in "3125000 4 1" "3125000 4 2" "3125000 4 3" "3125000 8 2" "6250000 4 1" "6250000 4 2" "6250000 8 2" "12500000 4 2" "25000000 4 2"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --params $1 --chunks $2 --streams $3 --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/share.json 2> gpurun_out/share.err || { cat gpurun_out/share.err | tail -5; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/share.json')); print('P=$1 chunks=$2 streams=$3 ms/step', d['ms_per_step'], 'bit-exact', d['assembled_bit_exact'])"
done
