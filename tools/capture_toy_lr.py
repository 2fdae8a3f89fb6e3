#!/usr/bin/env python3
"""Capture the aggregation inputs/outputs of the reference's own toy-LR
course (tests/test_toy_lr.py:16-53, configs[0] C1: 5 clients, 20 rounds,
CPU standalone runner) → tests/golden/toy_lr_rounds.npz.

Runs ONLY in the build container (imports /root/reference).  Two harness
shims, both outside the reference's arithmetic: protobuf's pure-Python
implementation (the generated gRPC module predates protobuf >= 3.20) and a
stub `pympler.asizeof` (message-size logging only, message.py:264).

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference \
        python3 /root/repo/tools/capture_toy_lr.py
"""
import copy
import json
import os
import sys
import tempfile
import types

os.environ['PROTOCOL_BUFFERS_PYTHON_IMPLEMENTATION'] = 'python'
pymp = types.ModuleType('pympler')
pymp.asizeof = types.SimpleNamespace(asizeof=lambda x: 0)
sys.modules['pympler'] = pymp
sys.modules['pympler.asizeof'] = pymp.asizeof

import numpy as np  # noqa: E402
import torch  # noqa: E402

from federatedscope.core.aggregators import ClientsAvgAggregator  # noqa
from federatedscope.core.auxiliaries.data_builder import get_data  # noqa
from federatedscope.core.auxiliaries.utils import setup_seed  # noqa
from federatedscope.core.auxiliaries.logging import update_logger  # noqa
from federatedscope.core.configs.config import global_cfg  # noqa
from federatedscope.core.auxiliaries.runner_builder import get_runner  # noqa
from federatedscope.core.auxiliaries.worker_builder import (  # noqa
    get_server_cls, get_client_cls)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests',
                   'golden', 'toy_lr_rounds.npz')

captured = []
_orig = ClientsAvgAggregator.aggregate


def spy(self, agg_info):
    ins = [(int(s), {k: v.detach().clone().numpy() for k, v in d.items()})
           for s, d in agg_info['client_feedback']]
    out = _orig(self, agg_info)
    captured.append((ins, {k: v.detach().clone().numpy()
                           for k, v in out.items()}))
    return out


def main():
    ClientsAvgAggregator.aggregate = spy
    torch.set_num_threads(1)
    cfg = global_cfg.clone()
    cfg.use_gpu = False
    cfg.federate.mode = 'standalone'
    cfg.federate.total_round_num = 20
    cfg.federate.make_global_eval = False
    cfg.federate.client_num = 5
    cfg.eval.freq = 10
    cfg.data.type = 'toy'
    cfg.trainer.type = 'general'
    cfg.model.type = 'lr'
    cfg.outdir = tempfile.mkdtemp()
    setup_seed(cfg.seed)
    update_logger(cfg, True)
    data, modified = get_data(cfg.clone())
    cfg.merge_from_other_cfg(modified)
    runner = get_runner(data=data, server_class=get_server_cls(cfg),
                        client_class=get_client_cls(cfg), config=cfg.clone())
    best = runner.run()
    loss = float(best['client_summarized_weighted_avg']['test_loss'])
    arrs = {}
    meta = {'rounds': len(captured), 'test_loss': loss, 'rounds_meta': []}
    for r, (ins, out) in enumerate(captured):
        meta['rounds_meta'].append({'sizes': [s for s, _ in ins],
                                    'keys': list(ins[0][1].keys())})
        for i, (_, d) in enumerate(ins):
            for k, v in d.items():
                arrs['r%d|x|%d|%s' % (r, i, k)] = v
        for k, v in out.items():
            arrs['r%d|out|%s' % (r, k)] = v
    arrs['meta'] = np.array(json.dumps(meta))
    np.savez_compressed(OUT, **arrs)
    print('captured %d rounds, test_loss %.4f -> %s' % (len(captured), loss,
                                                       OUT))


if __name__ == '__main__':
    main()
