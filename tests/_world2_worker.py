"""Rank body of tests/test_gpu_world2.py (run under torch.distributed.run
with the gloo backend: two ranks sharing the box's one GPU).  argv[1]:
the assembly (``aggregator.shard_assembly``), 'rccl' (pipelined
all-gathers) or 'p2p' (peer assembly: IPC-imported output copies, stores
from the reducing kernel or a push, flag barrier).

Every rank builds the drop-in aggregators with
``aggregator.shard_by_param_range`` and calls aggregate() on the same client
list (SPMD): each rank stages and reduces only its parameter-range pieces
with the libfsagg kernels, the pieces are all-gathered (Krum / norm bounding
add their one all-reduce), and every rank must hold the reference's result —
the golden fixtures generated from FederatedScope itself."""
import json
import os
import sys
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    import oracle as O
    import trimmed_bounds as TB
    from golden_io import load_case
    from test_gpu_golden import (DictModel, assert_bit_exact, cfg, feedback,
                                 to_np)
    from federatedscope_amd.core.aggregators import (
        BulyanAggregator, ClientsAvgAggregator, KrumAggregator,
        MedianAggregator, NormboundingAggregator, TrimmedmeanAggregator)

    mode = sys.argv[1] if len(sys.argv) > 1 else 'rccl'

    def sharded(c, chunks=2):
        c.aggregator.shard_by_param_range = True
        c.aggregator.shard_chunks = chunks
        c.aggregator.shard_assembly = mode
        return c

    done = []
    for name in ('fedavg_n100_iw0', 'fedavg_n7_iw1', 'fedavg_missing_key',
                 'fedavg_dtypes'):
        meta, clients, out, _, _ = load_case(name)
        for dev in ('cuda', 'cpu'):
            agg = ClientsAvgAggregator(config=sharded(cfg(
                iw=meta['ignore_weight'])))
            got = agg.aggregate({'client_feedback': feedback(clients, dev),
                                 'recover_fun': None})
            assert_bit_exact(got, out, name + '/' + dev)
            done.append(name + '/' + dev)
    for name in ('orderstat_n200_p51', 'orderstat_n7_p48',
                 'orderstat_n51_p51'):
        meta, clients, out, init, extra = load_case(name)
        for chunks in (1, 3):
            agg = MedianAggregator(model=DictModel(init),
                                   config=sharded(cfg(f=1), chunks))
            got = agg.aggregate({'client_feedback': feedback(clients, 'cpu')})
            assert_bit_exact(got, out, name)
        k = int(len(clients) * 0.2)
        got = TrimmedmeanAggregator(model=DictModel(init), config=sharded(
            cfg(f=1, ratio=0.2))).aggregate(
                {'client_feedback': feedback(clients)})
        want = O.add_init(init, O.trimmed_mean_update(clients, k))
        for key in got:
            g, o = to_np(got[key]).astype(np.float64), np.asarray(want[key])
            T = np.stack([np.asarray(d[key], np.float64).reshape(-1)
                          for _, d in clients])
            TB.check_vs_oracle('world2|%s|%s' % (name, key), g.reshape(-1),
                               o.reshape(-1), T, len(clients) - 2 * k,
                               init=np.asarray(init[key]).reshape(-1))
        done.append(name)
    for name in ('krum_n50_f10_a5', 'krum_n12_f2_a3', 'krum_n10_f10_a1'):
        meta, clients, out, init, extra = load_case(name)
        agg = KrumAggregator(model=DictModel(init), config=sharded(cfg(
            f=meta['f'], agg_num=meta['agg_num'],
            client_num=max(2 * meta['f'] + 3, 50))))
        got = agg.aggregate({'client_feedback': feedback(clients, 'cpu')})
        assert agg.last_selection == [int(i) for i in
                                      extra['order'][:meta['agg_num']]], name
        assert_bit_exact(got, out, name)
        done.append(name)
    for name in ('bulyan_n40_f9', 'bulyan_n20_f4'):
        meta, clients, out, init, extra = load_case(name)
        agg = BulyanAggregator(model=DictModel(init), config=sharded(cfg(
            f=meta['f'], rate=meta['rate'], client_num=4 * meta['f'] + 3)))
        got = agg.aggregate({'client_feedback': feedback(clients)})
        keep = len(clients) - int(2 * meta['rate'] * meta['f'])
        assert agg.last_selection == [int(i) for i in extra['order'][:keep]]
        for key in out:
            np.testing.assert_allclose(to_np(got[key]), out[key], rtol=1e-5,
                                       atol=1e-6)
        done.append(name)
    for name in ('normbound_0.5', 'normbound_5'):
        meta, clients, out, init, _ = load_case(name)
        got = NormboundingAggregator(model=DictModel(init), config=sharded(
            cfg(bound=meta['bound']))).aggregate(
                {'client_feedback': feedback(clients, 'cpu')})
        for key in out:
            np.testing.assert_allclose(to_np(got[key]), out[key], rtol=1e-6,
                                       atol=1e-7)
        done.append(name)
    # larger multi-key host dicts: sharded == unsharded, bit for bit
    g = torch.Generator().manual_seed(5)
    shapes = [(300_001, ), (64, 70), (1, ), (70_000, )]
    clients = [(i + 1, OrderedDict(('k%d' % j, torch.randn(s, generator=g))
                                   for j, s in enumerate(shapes)))
               for i in range(30)]
    a = ClientsAvgAggregator(config=sharded(cfg(), 4)).aggregate(
        {'client_feedback': clients, 'recover_fun': None})
    b = ClientsAvgAggregator(config=cfg()).aggregate(
        {'client_feedback': clients, 'recover_fun': None})
    for k in b:
        assert torch.equal(a[k], b[k]), k
    done.append('synthetic')
    from federatedscope_amd.core.sharding import (PeerAssembly,
                                                  PipelinedAssembly)
    kind = PeerAssembly if mode == 'p2p' else PipelinedAssembly
    plans = [p for p in agg._plans.values()]
    assert plans and all(isinstance(p, kind) for p in plans), plans
    sys.stdout.write(json.dumps({'rank': rank, 'world': world, 'ok': done,
                                 'mode': mode})
                     + '\n')  # one write: the ranks share the pipe
    sys.stdout.flush()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
