#!/usr/bin/env python3
"""cProfile of the quantised-upload ingress (tools/bench_wire.py quant_leg's
server loop: 100 ResNet-50 int8 uploads through
AggregationServer.callback_funcs_model_para with stage-on-arrival).
tools only."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import bench_wire  # noqa: E402


def main():
    import torch
    calls = []
    orig = bench_wire.time.perf_counter
    pr = cProfile.Profile()

    class Hook:
        on = False
    # profile the second and later rounds of run(True): wrap the server's
    # callback through the module's AggregationServer
    from federatedscope_amd.core.workers import server as S
    cb = S.AggregationServer.callback_funcs_model_para

    def wrapped(self, *a, **k):
        pr.enable()
        try:
            return cb(self, *a, **k)
        finally:
            pr.disable()
    S.AggregationServer.callback_funcs_model_para = wrapped
    bench_wire.quant_leg(n=100, reps=2)
    torch.cuda.synchronize()
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
        print(s.getvalue())


if __name__ == '__main__':
    main()
