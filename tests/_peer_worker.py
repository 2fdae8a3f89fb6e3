"""Rank body of tests/test_gpu_world2.py's peer-assembly cases (run under
torch.distributed.run, gloo for the handle exchange, every rank on the
box's one GPU: same-device IPC stands in for the xGMI peers).

argv[1] = 'aggregate': the drop-in aggregators with
``aggregator.shard_by_param_range`` and ``shard_assembly = 'p2p'`` on
device-resident client dicts — FedAvg on one key (the fused broadcast
epilogue), FedAvg on several keys, median, trimmed mean, Krum (the pushed
piece) — every rank's result bit-identical to the unsharded aggregate() on
the same dicts.

argv[1] = 'lost': rank 1 never runs its round; rank 0's flag barrier must
give up within the timeout, ``run_bucket`` must raise, and both ranks must
release the peer buffers and exit cleanly.

argv[1] = 'lost_views': the same with result views
(``run_bucket(copy=False)``, ``aggregator.shard_result_views``): the call
returns before its barrier has run, so it cannot raise; the failure
surfaces at ``check()`` (or the next run_bucket), naming rank 1."""
import json
import os
import sys
import time
from collections import OrderedDict
from types import SimpleNamespace

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def cfg(sharded, f=0, agg_num=1, ratio=0.2, n=1000):
    bft = SimpleNamespace(krum_agg_num=agg_num,
                          trimmedmean_excluded_ratio=ratio,
                          normbounding_norm_bound=1.0)
    agg = SimpleNamespace(byzantine_node_num=f, BFT_args=bft,
                          shard_by_param_range=sharded,
                          shard_assembly='p2p', shard_chunks=2)
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=n, sample_client_rate=1.0),
        aggregator=agg)


class DictModel(torch.nn.Module):
    def __init__(self, sd):
        super().__init__()
        self.sd = sd

    def state_dict(self, *a, **kw):
        return self.sd


def clients(shapes, n, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    return [(int(1 + (7 * i) % 13), OrderedDict(
        (k, torch.randn(s, device='cuda', generator=g))
        for k, s in shapes)) for i in range(n)]


def aggregate_mode(rank, world):
    from federatedscope_amd.core.aggregators import (ClientsAvgAggregator,
                                                     KrumAggregator,
                                                     MedianAggregator,
                                                     TrimmedmeanAggregator)
    from federatedscope_amd.core.sharding import PeerAssembly
    done = []
    one = [('w', (1_000_003, ))]
    multi = [('a', (300_001, )), ('b', (64, 70)), ('c', (1, )),
             ('d', (70_000, ))]
    # the same init model on every rank (each rank reduces its piece of
    # init + update)
    g = torch.Generator(device='cuda').manual_seed(99)
    init1 = OrderedDict((k, torch.randn(s, device='cuda', generator=g))
                        for k, s in one)
    initm = OrderedDict((k, torch.randn(s, device='cuda', generator=g))
                        for k, s in multi)
    cases = [
        ('fedavg_one_key', ClientsAvgAggregator, one, None, {}, 20),
        ('fedavg_multi_key', ClientsAvgAggregator, multi, None, {}, 20),
        ('median', MedianAggregator, multi, initm, {'f': 1}, 21),
        ('trimmed_mean', TrimmedmeanAggregator, one, init1, {'f': 1}, 30),
        ('krum', KrumAggregator, multi, initm, {'f': 2, 'agg_num': 3}, 12),
    ]
    for name, cls, shapes, init, kw, n in cases:
        fb = clients(shapes, n, seed=len(name) + n)
        info = {'client_feedback': fb, 'recover_fun': None}
        model = DictModel(init) if init is not None else None
        a = cls(model=model, device='cuda', config=cfg(True, **kw))
        b = cls(model=model, device='cuda', config=cfg(False, **kw))
        for rnd in range(3):       # rounds rotate the double buffers
            got = a.aggregate(info)
            want = b.aggregate(info)
            for k in want:
                if not torch.equal(got[k], want[k]):
                    bad = (got[k] != want[k]).reshape(-1).nonzero()
                    pa = next(iter(a._plans.values()))
                    lay = next(iter(a._layouts.values()), None)
                    off = lay.offsets[k] if lay is not None else None
                    raise AssertionError(
                        (name, k, rnd, 'rank', rank, 'bad', bad.numel(),
                         'first', bad[:4].reshape(-1).tolist(),
                         'key offset', off, 'pieces',
                         [pa.piece(r) for r in range(world)],
                         got[k].reshape(-1)[bad[:2].reshape(-1)].tolist(),
                         want[k].reshape(-1)[bad[:2].reshape(-1)].tolist()))
        assert all(isinstance(p, PeerAssembly) for p in a._plans.values())
        if name == 'krum':
            assert a.last_selection == b.last_selection
        done.append(name)
    return {'ok': done}


def lost_mode(rank, world, views=False):
    from federatedscope_amd.core.sharding import Comm, PeerAssembly
    pa = PeerAssembly(4096, comm=Comm(), device=torch.device('cuda', 0),
                      timeout_s=1.0, buffers=3 if views else 2)
    raised = None
    at_call = None
    t0 = time.time()
    def compute(lo, hi, own, peers):
        own[lo:hi].fill_(1.0)
        return False

    if rank == 0:
        try:
            pa.run_bucket(compute, copy=not views)
            if views:
                at_call = 'returned'
                pa.check()
        except RuntimeError as e:
            raised = str(e)
    waited = time.time() - t0
    dist.barrier()
    # the late rank runs the round it missed (rank 0's flag for it is
    # already up), then both run the next round: it must succeed on every
    # rank (check() cleared the timed-out status) and assemble both pieces
    if rank == 1:
        pa.run_bucket(compute)

    def compute2(lo, hi, own, peers):
        own[lo:hi].fill_(2.0 + rank)
        return False
    second = None
    try:
        res = pa.run_bucket(compute2)
        want = torch.cat([torch.full((pa.piece(r)[1] - pa.piece(r)[0], ),
                                     2.0 + r, device=res.device)
                          for r in range(world)])
        second = bool(torch.equal(res, want))
    except RuntimeError as e:
        second = 'raised: %s' % e
    dist.barrier()
    pa.close()
    return {'raised': raised, 'waited_s': round(waited, 3),
            'second_round_ok': second, 'views_call': at_call}


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    mode = sys.argv[1]
    res = aggregate_mode(rank, world) if mode == 'aggregate' else \
        lost_mode(rank, world, views=mode == 'lost_views')
    res.update(rank=rank, world=world, mode=mode)
    sys.stdout.write(json.dumps(res) + '\n')
    sys.stdout.flush()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
