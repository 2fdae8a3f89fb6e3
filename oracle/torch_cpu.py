"""TEST INFRASTRUCTURE ONLY — torch-CPU, op-for-op restatement of the
reference's FedAvg loop, used as ``bench.py``'s timed CPU baseline.

SURVEY §8(d) asks for the build's own CPU restatement of
``ClientsAvgAggregator._para_weighted_avg``
(federatedscope/core/aggregators/clients_avg_aggregator.py:60-100) timed with
torch's CPU kernels at ``torch.set_num_threads(1)`` — what StandaloneRunner
sets (federatedscope/core/fed_runner.py:297-299) — and at all the host's
cores.  This is that loop: per key, per client in list order,
``tmp = x * w`` then ``acc = tmp`` (client 0) or ``acc += tmp``, every op an
ATen CPU kernel with its own temporary, exactly as the reference executes it
(the numpy port in fsagg_oracle.py has no such temporaries and runs ~6x
faster than the reference).  The product never imports this module.
"""
import torch


def para_weighted_avg_torch(models, weights):
    """models: list of (sample_size, OrderedDict[str, torch.Tensor]) on the
    CPU; weights: the reference's per-client Python doubles.  Returns a new
    dict (the reference aliases client 0's; the inputs are left intact)."""
    avg = {}
    keys = list(models[0][1].keys())
    for key in keys:
        acc = None
        for i, (_, local) in enumerate(models):
            if key not in local:
                continue
            tmp = local[key] * weights[i]
            if acc is None:
                acc = tmp
            else:
                acc += tmp
        avg[key] = acc
    return avg
