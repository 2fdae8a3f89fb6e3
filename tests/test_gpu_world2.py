"""Two ranks (gloo, sharing the box's one GPU) through the multi-GPU code
paths with the real libfsagg kernels:

* bench.py's strong-scaling step (PipelinedAssembly: block-cyclic
  parameter pieces, an all-gather per round) must assemble the full
  FedAvg result bit-exact on every rank;
* the drop-in aggregators in ``aggregator.shard_by_param_range`` mode
  (tests/_world2_worker.py) must reproduce the reference's goldens.

On the 8-GPU node the same code runs over RCCL (bench.py's default
backend); the collectives differ only in core/sharding.Comm."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run2(args, timeout=110, nproc=2):
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes', '1',
           '--nproc-per-node', str(nproc), '--master-addr', '127.0.0.1',
           '--master-port', str(_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS='4')
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    # the ranks' own tracebacks (torchrun prefixes them with [rankN])
    tb = '\n'.join(ln for ln in p.stderr.splitlines()
                   if ln.startswith('[rank'))
    assert p.returncode == 0, (p.stdout[-2000:], tb[-6000:] or
                               p.stderr[-4000:])
    # every JSON object in the output (the two ranks' lines can interleave)
    dec, out, i = json.JSONDecoder(), [], p.stdout.find('{')
    while i >= 0:
        try:
            obj, j = dec.raw_decode(p.stdout, i)
        except json.JSONDecodeError:
            j = i + 1
        else:
            out.append(obj)
        i = p.stdout.find('{', j)
    return out


def test_bench_strong_scaling_world2():
    recs = _run2(['bench.py', '--gpus', '2', '--backend', 'gloo',
                  '--clients', '10', '--params', '1000003', '--steps', '3',
                  '--warmup', '1', '--no-cpu-baseline', '--no-weak'])
    assert len(recs) == 1
    r = recs[0]
    assert r['n_gpus'] == 2 and r['scaling'] == 'strong'
    assert r['assembled_bit_exact'] is True
    assert r['config']['params'] == 1000003


def test_bench_self_launch():
    """A bare ``bench.py --gpus 2`` (no torchrun) starts its own two rank
    processes and prints ONE n_gpus 2 line, bit-exact after the assembly;
    with RCCL on a box with fewer GPUs than ranks it refuses (non-zero exit,
    no line)."""
    import torch
    env = dict(os.environ, OMP_NUM_THREADS='4')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, 'bench.py', '--gpus', '2',
                        '--backend', 'gloo', '--assembly', 'p2p',
                        '--clients', '10', '--params', '1000003', '--steps',
                        '3', '--warmup', '1', '--no-cpu-baseline',
                        '--no-weak'], cwd=ROOT, capture_output=True,
                       text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r['n_gpus'] == 2 and r['assembled_bit_exact'] is True
    assert r['roofline']['peak'] == 2 * 8000.0
    if torch.cuda.device_count() < 2:
        q = subprocess.run([sys.executable, 'bench.py', '--gpus', '2',
                            '--steps', '1', '--warmup', '0'], cwd=ROOT,
                           capture_output=True, text=True, timeout=110,
                           env=env)
        assert q.returncode != 0
        assert not [ln for ln in q.stdout.splitlines()
                    if ln.startswith('{')]


@pytest.mark.parametrize('world,clients,params', [
    (2, 100, 25_000_000),       # configs[2] itself: 5 GB per rank
    (4, 10, 1_000_003)])
def test_bench_peer_assembly(world, clients, params):
    """bench.py's peer assembly (core/sharding.PeerAssembly): each rank's
    kernel stores its piece into every rank's uncached output buffer through
    IPC-imported pointers, then the flag barrier — here 2 / 4 processes on
    one GPU (same-device IPC), on the 8-GPU node the same code over xGMI.
    Every rank's assembled result must be bit-exact, and the barrier must
    not have timed out (bench.py calls PeerAssembly.check())."""
    recs = _run2(['bench.py', '--gpus', str(world), '--backend', 'gloo',
                  '--assembly', 'p2p', '--clients', str(clients),
                  '--params', str(params), '--steps', '5', '--warmup', '2',
                  '--no-cpu-baseline', '--no-weak'], nproc=world)
    assert len(recs) == 1
    r = recs[0]
    assert r['n_gpus'] == world
    assert 'peer assembly' in r['config']['parallelism'], r['config']
    assert r['assembled_bit_exact'] is True


@pytest.mark.parametrize('mode', ['rccl', 'p2p'])
def test_sharded_aggregators_world2(mode):
    """The reference's goldens through aggregate() sharded over two ranks,
    assembled by the pipelined all-gathers ('rccl') and by the peer
    assembly ('p2p')."""
    recs = _run2([os.path.join('tests', '_world2_worker.py'), mode])
    assert sorted(r['rank'] for r in recs) == [0, 1]
    for r in recs:
        assert 'synthetic' in r['ok'] and len(r['ok']) >= 18, r
        assert r['mode'] == mode


@pytest.mark.parametrize('world', [2, 4])
def test_peer_assembly_aggregate(world):
    """aggregate() on device dicts through the peer assembly (fused
    broadcast for one-key FedAvg, pushed pieces for the other rules), three
    rounds each: bit-identical to the unsharded call on every rank."""
    recs = _run2([os.path.join('tests', '_peer_worker.py'), 'aggregate'],
                 nproc=world)
    assert sorted(r['rank'] for r in recs) == list(range(world))
    for r in recs:
        assert r['ok'] == ['fedavg_one_key', 'fedavg_multi_key', 'median',
                           'trimmed_mean', 'krum'], r


@pytest.mark.parametrize('mode', ['lost', 'lost_views'])
def test_peer_assembly_lost_rank(mode):
    """Rank 1 never runs its round: rank 0's barrier gives up after the 1 s
    timeout, run_bucket raises naming rank 1 (with result views the call
    itself returns — its barrier has not run yet — and check() raises), and
    both ranks release the peer buffers and exit 0."""
    recs = _run2([os.path.join('tests', '_peer_worker.py'), mode])
    by = {r['rank']: r for r in recs}
    assert set(by) == {0, 1}
    assert by[1]['raised'] is None
    assert 'rank 1' in (by[0]['raised'] or ''), by[0]
    if mode == 'lost_views':
        assert by[0]['views_call'] == 'returned', by[0]
    assert 0.9 <= by[0]['waited_s'] <= 30.0, by[0]
    # once the late rank has caught up, the next round succeeds everywhere
    assert by[0]['second_round_ok'] is True, by[0]
    assert by[1]['second_round_ok'] is True, by[1]
