"""bench.py's launcher contract: ``--gpus N`` must
produce an N-rank line or fail, however it is started.  Without a GPU only
the refusal path can run: N RCCL ranks need N visible GPUs, and a
WORLD_SIZE that disagrees with --gpus is an error, never a smaller-N
line.  The N-rank line itself is tests/test_gpu_world2.py::
test_bench_self_launch (gloo, one GPU)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')]
                          + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _visible_gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_visible_gpus() >= 8, reason='an 8-GPU node runs it')
def test_too_few_gpus_for_rccl_ranks_is_an_error():
    p = _bench(['--gpus', '8', '--steps', '1', '--warmup', '0'])
    assert p.returncode != 0
    assert '{' not in p.stdout
    assert 'visible GPUs' in p.stderr


def test_world_size_mismatch_is_an_error():
    p = _bench(['--gpus', '4', '--steps', '1', '--warmup', '0',
                '--no-pmc'], env={'WORLD_SIZE': '1', 'RANK': '0',
                                  'LOCAL_RANK': '0'})
    assert p.returncode == 2
    assert '{' not in p.stdout
    assert 'WORLD_SIZE 1' in p.stderr
