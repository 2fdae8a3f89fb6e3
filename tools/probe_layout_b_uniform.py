import sys, os, json, time, statistics
sys.path.insert(0, '/root/repo')
os.chdir('/root/repo')
import torch
from collections import OrderedDict
from types import SimpleNamespace
import bench
from federatedscope_amd import ops
from federatedscope_amd.core.aggregators import ClientsAvgAggregator
from federatedscope_amd.core.aggregators._engine import fedavg_weights
from federatedscope_amd.layout import BucketLayout
dev = torch.device('cuda', 0)
with open('tools/resnet50_layout.json') as f:
    keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta')) for k, s in keys))
sizes = bench.sample_sizes(100)
n, P = 100, lay.numel
ld = ops.round_up(P, 64)
slab = torch.empty((n, ld), dtype=torch.float32, device=dev)
ops.fill_uniform(slab, ld, seed=1)
clients = [(sizes[i], OrderedDict((k, slab[i, lay.offsets[k]:lay.offsets[k] + lay.numels[k]].view(lay.shapes[k])) for k in lay.keys)) for i in range(n)]
cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False, use_ss=False))
agg = ClientsAvgAggregator(device=dev, config=cfg)
st = agg._staged_rows(clients)
print('uniform', st.rs.uniform, 'flat', ops._flat_rows(st.rs, None), 'aligned', st.rs.aligned16, 'missing', st.rs.missing)
info = {'client_feedback': clients, 'recover_fun': None}
w_dev = torch.tensor(fedavg_weights(sizes), dtype=torch.float32, device=dev)
rows = ops.RowTable.from_slab(slab, numel=ld)
flat = torch.empty(ld, dtype=torch.float32, device=dev)
for _ in range(5):
    agg.aggregate(info); ops.weighted_sum(rows, w_dev, flat)
torch.cuda.synchronize()
for rnd in range(3):
    for name, fn in (('agg', lambda: agg.aggregate(info)), ('flat', lambda: ops.weighted_sum(rows, w_dev, flat))):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(10): fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize(); t2 = time.perf_counter()
        print(name, 'host %.3f ms/call, total %.4f ms/call' % ((t1-t0)*100, (t2-t0)*100))
