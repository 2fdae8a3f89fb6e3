"""The server counterpart's host logic (core/workers/server.py), on CPU with
spy aggregators (no staging, no kernels): the reference's
_perform_federated_aggregation (federatedscope/core/workers/server.py:
437-490) loops over model_num internal models, hands each aggregator the
clients' part for that model, passes the server's recover_fun, calls the
monitor's calc_model_metric hook first, and keeps no unbounded history."""
from collections import OrderedDict

import pytest
import torch

from federatedscope_amd.core.workers.server import AggregationServer


class Spy:
    def __init__(self, tag):
        self.tag = tag
        self.calls = []

    def aggregate(self, agg_info):
        self.calls.append(agg_info)
        # the size-weighted mean of key 'w' (host arithmetic, a stand-in)
        tot = sum(s for s, _ in agg_info['client_feedback'])
        w = sum(s * d['w'] for s, d in agg_info['client_feedback']) / tot
        return OrderedDict(w=w)


class Model(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(3))


class Monitor:
    def __init__(self):
        self.calls = []

    def calc_model_metric(self, global_state, msg_list, rnd):
        self.calls.append((rnd, len(msg_list)))


def _para(v):
    return OrderedDict(w=torch.full((3, ), float(v)))


def test_model_num_loop_recover_fun_monitor():
    models = [Model(), Model()]
    aggs = [Spy(0), Spy(1)]
    mon = Monitor()

    def recover(x):
        return x

    srv = AggregationServer(models, aggs, sample_client_num=2,
                            stage_on_arrival=False, recover_fun=recover,
                            monitor=mon, staleness_toleration=1)
    assert srv.model_num == 2
    srv.callback_funcs_model_para(0, 1, (1, [_para(1), _para(10)]))
    assert srv.callback_funcs_model_para(0, 2, (3, [_para(5), _para(50)]))
    # model i got the clients' i-th part, in arrival order
    assert [d['w'][0].item() for _, d in
            aggs[0].calls[0]['client_feedback']] == [1.0, 5.0]
    assert [d['w'][0].item() for _, d in
            aggs[1].calls[0]['client_feedback']] == [10.0, 50.0]
    for a in aggs:
        assert a.calls[0]['recover_fun'] is recover
        assert a.calls[0]['staleness'] == [(1, 0), (2, 0)]
    assert torch.allclose(models[0].w, torch.full((3, ), 4.0))
    assert torch.allclose(models[1].w, torch.full((3, ), 40.0))
    assert mon.calls == [(0, 2), (0, 2)]        # once per model, round 0
    # round 1 with a stale upload from round 0 (tolerated)
    srv.callback_funcs_model_para(0, 3, (2, [_para(7), _para(70)]))
    srv.callback_funcs_model_para(1, 1, (1, [_para(2), _para(20)]))
    srv.callback_funcs_model_para(1, 2, (1, [_para(4), _para(40)]))
    assert srv.state == 2
    assert aggs[1].calls[1]['staleness'] == [(1, 0), (2, 0), (3, 1)]
    assert srv.history is None                  # no history kept by default


@pytest.mark.parametrize('keep', [1, 3])
def test_history_is_bounded(keep):
    agg = Spy(0)
    srv = AggregationServer(Model(), agg, sample_client_num=1,
                            stage_on_arrival=False, keep_history=keep)
    for r in range(5):
        srv.callback_funcs_model_para(r, 1, (1, _para(r)))
    assert len(srv.history) == keep
    assert srv.history[-1]['w'][0].item() == 4.0


def test_model_num_mismatch_raises():
    with pytest.raises(ValueError):
        AggregationServer([Model(), Model()], [Spy(0)], sample_client_num=1,
                          stage_on_arrival=False)


def test_normbound_rates_match_torch_rtruediv():
    """NormboundingAggregator._rates rounds as the reference's
    ``self.norm_bound / torch.norm(param)`` (normbounding_aggregator.py:
    39-44): a Python float over a 0-dim fp32 tensor, i.e.
    reciprocal() * bound — checked bit for bit against torch itself."""
    import numpy as np
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import NormboundingAggregator
    rng = np.random.default_rng(7)
    for bound in (0.5, 1.0, 5.0, 3.3):
        cfg = SimpleNamespace(aggregator=SimpleNamespace(
            BFT_args=SimpleNamespace(normbounding_norm_bound=bound)),
            federate=SimpleNamespace(ignore_weight=False, use_ss=False))
        agg = NormboundingAggregator(model=torch.nn.Linear(1, 1), config=cfg)
        sq = rng.uniform(0.3, 400.0, 5000) ** 2
        got = agg._rates(sq)
        for v, r in zip(sq, got):
            norm = torch.tensor(float(np.float32(np.sqrt(v))),
                                dtype=torch.float32)
            if float(norm) > bound:
                want = (bound / norm).item()
                assert r == want, (bound, float(norm), r, want)
            else:
                assert r is None
