"""Row sets on the GPU: the clients' own device tensors read in place
(include/fsagg.h fsagg_rows) must give exactly what the staged stack gives.

* the row-set kernels over a key table equal the same kernels over the
  stack rows bit for bit, and the flat kernels over the slab (weighted sum,
  median, trimmed mean: per coordinate, so bit-identical; Krum: the same
  chunking → identical, the flat form's padded segments → within 1e-6);
* NULL entries implement the reference's missing-key rule in one launch;
* the drop-in aggregators take the in-place path for device dicts (no
  stack is built) and return what they return for host dicts."""
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [1, 0, 1023, 5, 300_001, 3, 7, 65_537, 24_577, 16]


def _clients(n, sizes=SIZES, seed=9, scale=1.0):
    g = torch.Generator(device='cuda').manual_seed(seed)
    return [OrderedDict(('k%d' % j, scale * torch.randn(
        sz, device='cuda', generator=g)) for j, sz in enumerate(sizes))
        for _ in range(n)]


def _sets(clients):
    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout, ClientStack
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    st = ClientStack(lay, len(clients), 'cuda')
    st.slab.zero_()
    st.load_many(clients)
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    keyed = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=clients)
    stacked = ops.RowSet.from_stack(st, range(len(clients)))
    return lay, st, keyed, stacked


def _key_ranges(lay, a, b):
    return all(torch.equal(a[lay.offsets[k]:lay.offsets[k] + lay.numels[k]],
                           b[lay.offsets[k]:lay.offsets[k] + lay.numels[k]])
               for k in lay.keys)


@pytest.mark.parametrize('n', [1, 13, 100])
def test_weighted_sum_rows_matches_flat(n):
    from federatedscope_amd import ops
    clients = _clients(n)
    lay, st, keyed, stacked = _sets(clients)
    rng = np.random.default_rng(n)
    w = [float(x) for x in rng.random(n)]
    pre = [float(x) for x in rng.random(n) + 0.5]
    base = torch.randn(lay.numel, device='cuda')
    outs = []
    for rs in (keyed, stacked):
        for kw in ({}, {'prescale': pre},
                   {'base': ops.BaseRows.from_bucket(base)}):
            o = torch.full((lay.numel, ), 7.0, device='cuda')
            ops.weighted_sum_rows(rs, w, o, **kw)
            outs.append(o)
    flat = []
    for kw in ({}, {'prescale': pre}, {'base': base}):
        o = torch.full((lay.numel, ), 7.0, device='cuda')
        ops.weighted_sum(ops.RowTable.from_slab(st.slab, numel=lay.numel),
                         w, o, **kw)
        flat.append(o)
    for i in range(3):
        assert _key_ranges(lay, outs[i], flat[i])
        assert _key_ranges(lay, outs[3 + i], flat[i])
    # and the first against the oracle's op order
    want = O.para_weighted_avg([(0, OrderedDict((k, v.cpu().numpy())
                                                for k, v in c.items()))
                                for c in clients], weights=w)
    got = lay.unpack(outs[0])
    for k in lay.keys:
        assert got[k].cpu().numpy().tobytes() == want[k].tobytes(), k


def test_weighted_sum_rows_missing_keys_one_launch():
    """NULL entries: each key reduced over the clients that hold it, the
    weights not renormalised (clients_avg_aggregator.py:74-75)."""
    from federatedscope_amd import ops
    n = 9
    clients = _clients(n, seed=4)
    lay, st, _, _ = _sets(clients)
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    drop = [(3, 'k2'), (5, 'k4'), (8, 'k4'), (1, 'k0'), (6, 'k8')]
    for i, k in drop:
        ptrs[i, lay.keys.index(k)] = 0
    rs = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=clients)
    assert rs.missing == len(drop)
    w = [float(x) for x in np.random.default_rng(1).random(n)]
    out = torch.zeros(lay.numel, device='cuda')
    ops.weighted_sum_rows(rs, w, out)
    host = [(0, OrderedDict((k, v.cpu().numpy()) for k, v in c.items()
                            if (i, k) not in drop))
            for i, c in enumerate(clients)]
    want = O.para_weighted_avg(host, weights=w)
    got = lay.unpack(out)
    for k in lay.keys:
        assert got[k].cpu().numpy().tobytes() == want[k].tobytes(), k
    with pytest.raises(KeyError):
        ops.coord_median_rows(rs, out)


@pytest.mark.parametrize('n', [7, 64, 100, 200, 300])
def test_order_statistics_rows_match_flat(n):
    from federatedscope_amd import ops
    sizes = [1, 1023, 5, 70_001, 3, 257]
    clients = _clients(n, sizes=sizes, seed=n)
    lay, st, keyed, stacked = _sets(clients)
    base = torch.randn(lay.numel, device='cuda')
    rows = ops.RowTable.from_slab(st.slab, numel=lay.numel)
    k = int(n * 0.2)
    for rs in (keyed, stacked):
        a = torch.full((lay.numel, ), 3.0, device='cuda')
        b = torch.full((lay.numel, ), 3.0, device='cuda')
        ops.coord_median_rows(rs, a, base=ops.BaseRows.from_bucket(base))
        ops.coord_median(rows, b, base=base)
        assert _key_ranges(lay, a, b)
        ops.trimmed_mean_rows(rs, k, a)
        ops.trimmed_mean(rows, k, b)
        assert _key_ranges(lay, a, b)
        ops.trimmed_mean_rows(rs, k, a, divisor=3.0,
                              base=ops.BaseRows.from_bucket(base))
        ops.trimmed_mean(rows, k, b, divisor=3.0, base=base)
        assert _key_ranges(lay, a, b)


@pytest.mark.parametrize('n', [5, 50])
def test_pairdist_rows(n):
    from federatedscope_amd import ops
    clients = _clients(n, sizes=[1, 1023, 5, 300_001, 3, 65_537], seed=2,
                       scale=0.1)
    lay, st, keyed, stacked = _sets(clients)
    D1 = ops.pairdist_rows(keyed)
    D2 = ops.pairdist_rows(stacked)
    assert torch.equal(D1, D2)     # same chunking → same sums
    D3 = ops.pairdist(ops.RowTable.from_slab(st.slab, numel=lay.numel),
                      lay.segments())
    off = ~torch.eye(n, dtype=torch.bool, device='cuda')
    assert torch.allclose(D1[off], D3[off], rtol=1e-6, atol=0)
    X = [np.concatenate([c[k].cpu().numpy().astype(np.float64).ravel()
                         for k in lay.keys]) for c in clients]
    sq = ops.rows_sqnorm(keyed).cpu().numpy()
    for i in range(n):
        for s, k in enumerate(lay.keys):
            v = clients[i][k].cpu().numpy().astype(np.float64)
            assert sq[i, s] == pytest.approx((v * v).sum(), rel=1e-12,
                                             abs=1e-300)
        assert sq[i].sum() == pytest.approx((X[i] ** 2).sum(), rel=1e-12)


@pytest.mark.parametrize('bound', [0.5, 1.0, 5.0, 3.3, 1e-3])
def test_normbound_prescale_matches_host_rates(bound):
    """fsagg_normbound_prescale_f32 against NormboundingAggregator._rates
    (itself pinned bit for bit to torch's ``bound / torch.norm(x)``,
    tests/test_server_logic.py): random norms around the bound, norms that
    round to exactly fl32(bound) or one ulp either side, 0, inf and NaN;
    the per-key sums added in the same order on both sides."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import NormboundingAggregator
    rng = np.random.default_rng(int(bound * 1000))
    b32 = np.float32(bound)
    edge = [np.nextafter(b32, np.float32(0)), b32,
            np.nextafter(b32, np.float32(np.inf))]
    norms = np.concatenate([rng.uniform(0.0, 4.0 * bound, 4000),
                            np.array(edge, dtype=np.float64)])
    sq = np.zeros((norms.size + 3, 3))
    sq[:norms.size, 0] = norms ** 2 * 0.25
    sq[:norms.size, 1] = norms ** 2 * 0.5
    sq[:norms.size, 2] = norms ** 2 * 0.25
    sq[-2, 1] = np.inf
    sq[-1, 2] = np.nan
    cfg = SimpleNamespace(aggregator=SimpleNamespace(
        BFT_args=SimpleNamespace(normbounding_norm_bound=bound)),
        federate=SimpleNamespace(ignore_weight=False, use_ss=False))
    agg = NormboundingAggregator(model=torch.nn.Linear(1, 1), config=cfg)
    host = [1.0 if r is None else r for r in
            agg._rates((sq[:, 0] + sq[:, 1]) + sq[:, 2])]
    got = ops.normbound_prescale(torch.from_numpy(sq).cuda(), bound)
    got = got.cpu().numpy()
    want = np.array(host, dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
        np.nonzero(got.view(np.uint32) != want.view(np.uint32))
    assert got[-3] == 1.0 and got[-2] == 0.0 and got[-1] == 1.0


def _cfg(**kw):
    bft = SimpleNamespace(krum_agg_num=kw.get('agg_num', 3),
                          trimmedmean_excluded_ratio=0.2,
                          normbounding_norm_bound=kw.get('bound', 5.0))
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=kw.get('client_num', 1000),
                                 sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=kw.get('f', 2),
                                   BFT_args=bft),
        asyn=SimpleNamespace(staleness_discount_factor=1.0))


def test_dropin_device_dicts_read_in_place():
    """Device dicts → no ClientStack is built; the results equal the host
    dicts' (staged) results bit for bit, for every rule; the server model
    on the device is read in place too."""
    from federatedscope_amd.core.aggregators import (
        BulyanAggregator, ClientsAvgAggregator, KrumAggregator,
        MedianAggregator, NormboundingAggregator, TrimmedmeanAggregator)
    n = 23
    sizes = [(5, 3), (1, ), (130, ), (33, 2), (4097, )]
    g = torch.Generator().manual_seed(21)
    host = [(int(torch.randint(1, 90, (1, ), generator=g)), OrderedDict(
        ('p%d' % j, 0.1 * torch.randn(s, generator=g))
        for j, s in enumerate(sizes))) for _ in range(n)]
    dev = [(s, OrderedDict((k, v.cuda()) for k, v in d.items()))
           for s, d in host]
    init_h = OrderedDict(('p%d' % j, torch.randn(s, generator=g))
                         for j, s in enumerate(sizes))
    init_d = OrderedDict((k, v.cuda()) for k, v in init_h.items())

    class M(torch.nn.Module):
        def __init__(self, sd):
            super().__init__()
            self.sd = sd

        def state_dict(self, *a, **kw):
            return self.sd

    rules = [(ClientsAvgAggregator, {}), (KrumAggregator, {}),
             (BulyanAggregator, {'f': 4, 'client_num': n}),
             (MedianAggregator, {}), (TrimmedmeanAggregator, {}),
             (NormboundingAggregator, {'bound': 0.5})]
    for cls, kw in rules:
        a = cls(model=M(init_d), device='cuda', config=_cfg(**kw))
        got = a.aggregate({'client_feedback': dev, 'recover_fun': None})
        assert not a._stacks, cls          # nothing staged
        b = cls(model=M(init_h), device='cuda', config=_cfg(**kw))
        want = b.aggregate({'client_feedback': host, 'recover_fun': None})
        assert list(got) == list(want)
        for k in want:
            assert got[k].device.type == 'cuda'
            assert torch.equal(got[k].cpu(), want[k]), (cls.__name__, k)
    # an unaligned view (4-B offset) is staged instead, same result
    off = [(s, OrderedDict((k, torch.cat([torch.zeros(1, device='cuda'),
                                           v.reshape(-1)])[1:].view(v.shape))
                           for k, v in d.items())) for s, d in dev]
    a = ClientsAvgAggregator(device='cuda', config=_cfg())
    got = a.aggregate({'client_feedback': off, 'recover_fun': None})
    want = ClientsAvgAggregator(device='cuda', config=_cfg()).aggregate(
        {'client_feedback': host, 'recover_fun': None})
    for k in want:
        assert torch.equal(got[k].cpu(), want[k]), k


def test_back_to_back_aggregates_without_sync():
    """Twenty aggregate() calls issued back to back with no host
    synchronisation, alternating two multi-key layouts and client sets of
    different sizes (so the row tables, weights and chunk lists the pinned
    ring copies on its side stream differ every call and their device
    blocks are freed and reused while earlier kernels may still run): every
    result equals the same call made alone, bit for bit."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    layouts = [[(513, 3), (7, ), (70_001, ), (64, 64)],
               [(5, ), (1000, 33), (4096, ), (3, 3, 3)]]
    sets = []
    g = torch.Generator(device='cuda').manual_seed(77)
    for j in range(4):
        shapes = layouts[j % 2]
        n = 9 + 7 * j
        sets.append([(1 + (5 * i + j) % 17, OrderedDict(
            ('w%d' % k, torch.randn(s, device='cuda', generator=g))
            for k, s in enumerate(shapes))) for i in range(n)])
    agg = ClientsAvgAggregator(device='cuda', config=_cfg())
    want = []
    for fb in sets:
        r = agg.aggregate({'client_feedback': fb, 'recover_fun': None})
        torch.cuda.synchronize()
        want.append({k: v.clone() for k, v in r.items()})
    got = []
    torch.cuda.synchronize()
    for c in range(20):
        got.append(agg.aggregate({'client_feedback': sets[c % 4],
                                  'recover_fun': None}))
    torch.cuda.synchronize()
    for c, r in enumerate(got):
        for k, v in want[c % 4].items():
            assert torch.equal(r[k], v), (c, k)


def test_uniform_row_sets_take_the_flat_kernel():
    """Clients whose keys are views of one storage laid out exactly as the
    bucket (a flat-parameter model, a slab row) form a uniform row set: the
    whole bucket is one contiguous range per client and FedAvg runs the
    flat kernel over it — bit-identical to the row-set kernel on separately
    allocated copies of the same keys.  Keys of one storage at other
    offsets, or of different storages, are not uniform."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.layout import BucketLayout
    shapes = [('a', (3, 5)), ('b', (7, )), ('c', (64, 33)), ('d', (1, ))]
    lay = BucketLayout(OrderedDict((k, torch.empty(s)) for k, s in shapes))
    n = 9
    g = torch.Generator(device='cuda').manual_seed(3)
    slab = torch.randn((n, lay.numel + 64), device='cuda', generator=g)

    def views(i, shift=0):
        return OrderedDict((k, slab[i, shift + lay.offsets[k]:shift +
                                    lay.offsets[k] + lay.numels[k]].view(s))
                           for k, s in shapes)
    uni = [views(i) for i in range(n)]
    sep = [OrderedDict((k, v.clone()) for k, v in d.items()) for d in uni]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    sizes = [i + 3 for i in range(n)]
    agg = ClientsAvgAggregator(device='cuda', config=cfg)
    st = agg._staged_rows([(s, d) for s, d in zip(sizes, uni)])
    assert st.rs.uniform and ops._flat_rows(st.rs, None)
    got = agg.aggregate({'client_feedback': list(zip(sizes, uni)),
                         'recover_fun': None})
    want = agg.aggregate({'client_feedback': list(zip(sizes, sep)),
                          'recover_fun': None})
    assert not agg._staged_rows(list(zip(sizes, sep))).rs.uniform
    for k in want:
        assert torch.equal(got[k], want[k]), k
    host = [(s, OrderedDict((k, v.cpu().numpy()) for k, v in d.items()))
            for s, d in zip(sizes, sep)]
    ref = O.para_weighted_avg(host)
    for k in ref:
        assert got[k].cpu().numpy().tobytes() == ref[k].tobytes(), k
    # one storage at other offsets (a gap of 4 after key 'a'): not uniform
    odd = []
    for i in range(n):
        d = views(i)
        d['b'] = slab[i, lay.offsets['b'] + 4:lay.offsets['b'] + 11]
        odd.append(d)
    assert not agg._staged_rows([(1, d) for d in odd]).rs.uniform
    # keys of different storages: not uniform
    mixed = [OrderedDict(d) for d in uni]
    for d in mixed:
        d['d'] = d['d'].clone()
    assert not agg._staged_rows([(1, d) for d in mixed]).rs.uniform


@pytest.mark.parametrize('n', [1, 7, 100, 128, 129])
def test_hosttab_weighted_sum(n):
    """The flat weighted sum with its row table, weights and prescales in
    the kernel arguments (fsagg_weighted_sum_hosttab_f32: up to 128 rows,
    host lists; 129 rows take the device-table kernel) equals the
    device-table kernel bit for bit — plain, with prescale and base, with
    several outputs (the peer-assembly epilogue) and over a sub-range
    (a rank's piece) with a ragged tail — and the oracle."""
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    P = 1_000_003
    slab = torch.empty((n, P + 61), dtype=torch.float32, device='cuda')
    ops.fill_uniform(slab, P + 61, seed=n)
    rows_dev = ops.RowTable.from_slab(slab, numel=P)
    from federatedscope_amd.layout import BucketLayout
    lay = BucketLayout(OrderedDict([('w', torch.empty(P, device='meta'))]))
    ptrs = np.array([[slab[i].data_ptr()] for i in range(n)], dtype=np.int64)
    rs = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=(slab, ))
    rng = np.random.default_rng(n)
    w = [float(x) for x in rng.random(n) / n]
    pre = [float(x) for x in rng.random(n) + 0.5]
    base = torch.randn(ops.round_up(P, 64), device='cuda')
    for kw in ({}, {'prescale': pre}, {'prescale': pre, 'base': True}):
        b = ops.BaseRows.from_bucket(base) if kw.get('base') else None
        got = torch.full((ops.round_up(P, 64), ), 7.0, device='cuda')
        ops.weighted_sum_rows(rs, w, got, prescale=kw.get('prescale'),
                              base=b)
        want = torch.empty_like(got)
        ops.weighted_sum(rows_dev, w, want, prescale=kw.get('prescale'),
                         base=base if b is not None else None)
        assert torch.equal(got[:P], want[:P]), (n, kw)
        # a sub-range (a rank's piece), with peers' copies
        lo, hi = 64 * 1001, P
        o1 = torch.full_like(got, 3.0)
        o2 = torch.full_like(got, 5.0)
        assert ops.weighted_sum_rows_bcast(
            rs, w, o1, [o2.data_ptr()], prescale=kw.get('prescale'), base=b,
            lo=lo, hi=hi)
        assert torch.equal(o1[lo:hi], want[lo:hi])
        assert torch.equal(o2[lo:hi], want[lo:hi])
        assert bool((o1[:lo] == 3.0).all()) and bool((o2[:lo] == 5.0).all())
    # the oracle on the first columns
    x = slab[:, :4096].cpu().numpy()
    ref = O.para_weighted_avg([(1, {'w': x[i]}) for i in range(n)],
                              weights=w)['w']
    got = torch.empty(ops.round_up(P, 64), device='cuda')
    ops.weighted_sum_rows(rs, w, got)
    assert got[:4096].cpu().numpy().tobytes() == ref.tobytes()
    if n > L.FSAGG_HOSTTAB_MAX_CLIENTS:
        arr = (ctypes_p() * 1)(got.data_ptr())
        tab = np.array([slab[i].data_ptr() for i in range(n)], np.uint64)
        wf = np.asarray(w, np.float32)
        assert L.load().fsagg_weighted_sum_hosttab_f32(
            tab.ctypes.data, wf.ctypes.data, None, n, P, None, arr, 1,
            None) != 0


def ctypes_p():
    import ctypes
    return ctypes.c_void_p


@pytest.mark.parametrize('n', [1, 5, 25])
def test_rows_hosttab_weighted_sum(n):
    """A small multi-key row set's weighted sum with its pointer table,
    weights, prescales and base table in the kernel arguments
    (fsagg_weighted_sum_rows_hosttab_f32: n <= 64, n·nseg <= 256) equals the
    device-table kernel bit for bit — keyed rows with absent keys, stack
    rows, prescales, a per-key base (device tensors) and a bucket base — and
    makes no table upload."""
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    clients = _clients(n, seed=n + 3)
    lay, st, keyed, stacked = _sets(clients)
    assert n * keyed.nseg <= L.FSAGG_HOSTTAB_ROWS_MAX_PTRS
    # absent keys: client 0 lacks k2, the last client k4
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    ptrs[0, lay.keys.index('k2')] = 0
    ptrs[-1, lay.keys.index('k4')] = 0
    holey = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=clients)
    rng = np.random.default_rng(n)
    w = [float(x) for x in rng.random(n)]
    pre = [float(x) for x in rng.random(n) + 0.5]
    server = OrderedDict((k, torch.randn(v.shape, device='cuda'))
                         for k, v in clients[0].items())
    bp = np.array([server[k].data_ptr() for k in lay.keys], dtype=np.int64)
    bases = [None, ops.BaseRows.from_pointers(lay, bp, 'cuda',
                                              keepalive=(server, )),
             ops.BaseRows.from_bucket(torch.randn(lay.numel, device='cuda'))]
    wd = torch.tensor(w, dtype=torch.float32, device='cuda')
    pd = torch.tensor(pre, dtype=torch.float32, device='cuda')
    # the layout's chunk list (cached per layout) exists before counting
    ops.weighted_sum_rows(keyed, w, torch.empty(lay.numel, device='cuda'))
    for rs in (keyed, holey, stacked):
        for b in bases:
            for use_pre in (False, True):
                got = torch.full((lay.numel, ), 7.0, device='cuda')
                before = ops._RING.uploads
                ops.weighted_sum_rows(rs, w, got, base=b,
                                      prescale=pre if use_pre else None)
                assert ops._RING.uploads == before
                want = torch.full((lay.numel, ), 7.0, device='cuda')
                ops.weighted_sum_rows(rs, wd, want, base=b,
                                      prescale=pd if use_pre else None)
                assert _key_ranges(lay, got, want), (n, use_pre, b)
