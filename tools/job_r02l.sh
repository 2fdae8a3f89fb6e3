# side-stream pieces: sharded GPU tests, an 8-rank gloo rehearsal of the
# strong-scaling bench on one GPU (781k-param pieces: two side streams), the
# one-GPU share and the default bench line
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sharded or world2" > gpurun_out/t_sh.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_sh.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --no-weak > gpurun_out/w8.json 2> gpurun_out/w8.err; rc=$?; echo "w8 rc=$rc"; grep "\[bench\] rank 0\|bit-exact" gpurun_out/w8.err | head -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 bench.py --params 3125000 --chunks 4 --no-cpu-baseline > gpurun_out/share.json 2> gpurun_out/share.err; python3 -c "import json; d=json.load(open('gpurun_out/share.json')); print('share 3.125M x4 auto', d['ms_per_step'], d['assembled_bit_exact'])"
timeout -k 10 200 python3 bench.py > gpurun_out/bench_line.json 2> gpurun_out/bench_line.err; echo "bench rc=$?"; cut -c1-150 gpurun_out/bench_line.json
