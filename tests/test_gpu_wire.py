"""§8(f) rows on the GPU: quantised uploads decoded into the device stack,
secret-sharing FedAvg, and the update-dissimilarity metrics — against the
reference's own outputs (tests/golden/{quant,ss,dissim}_*.npz, written by
tools/gen_golden_wire.py) and the CPU oracle.

Bit-exact: dequantisation, quantised FedAvg, secret-sharing recovery.
Tolerance: the dissimilarity metrics (the reference sums squares in fp32
with ATen's ISA-dependent reduction order; rtol 1e-5 / 1e-4 as in
tests/test_oracle_golden.py)."""
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import oracle as O
from golden_io import case_names, load_case

pytestmark = pytest.mark.gpu


def _cfg(use_ss=False):
    return SimpleNamespace(federate=SimpleNamespace(
        ignore_weight=False, use_ss=use_ss, client_num=1000,
        sample_client_rate=1.0))


def _torch_wire(d, device='cpu'):
    return OrderedDict((k, torch.from_numpy(np.array(v)).to(device))
                       for k, v in d.items())


def _same_bits(got, want):
    g = got.detach().cpu().numpy()
    w = np.asarray(want)
    assert g.dtype == w.dtype and g.shape == w.shape
    assert g.tobytes() == w.tobytes()


@pytest.mark.parametrize('name', case_names('quant_'))
@pytest.mark.parametrize('device', ['cpu', 'cuda'])
def test_dequantization_drop_in(name, device):
    from federatedscope_amd.core.compression import \
        symmetric_uniform_dequantization
    _, clients, _, _, extra = load_case(name)
    for i, (_, wire) in enumerate(clients):
        got = symmetric_uniform_dequantization(_torch_wire(wire, device))
        pre = 'deq|%d|' % i
        want = OrderedDict((k[len(pre):], v) for k, v in extra.items()
                           if k.startswith(pre))
        assert list(got.keys()) == [k.replace('weight_quant', 'weight')
                                    for k in wire if 'weight_scale' not in k]
        for k, v in want.items():
            assert got[k].device.type == device
            _same_bits(got[k], v)


@pytest.mark.parametrize('name', case_names('quant_'))
@pytest.mark.parametrize('stage', [True, False])
def test_quantized_uploads_through_server(name, stage):
    """Server.callback_funcs_model_para with quantization.method='uniform':
    staged uploads cross PCIe as int codes and are dequantised into the
    stack by fsagg_wire_unpack_f32; the round's FedAvg is bit-exact."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.workers.server import AggregationServer
    _, clients, out, _, _ = load_case(name)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.p = torch.nn.ParameterDict()

        def state_dict(self, *a, **kw):
            return OrderedDict()

        def load_state_dict(self, sd, strict=True):
            self.loaded = sd

    srv = AggregationServer(M(), ClientsAvgAggregator(config=_cfg()),
                            sample_client_num=len(clients),
                            stage_on_arrival=stage, dequantize=True,
                            keep_history=1)
    for sender, (s, wire) in enumerate(clients):
        srv.callback_funcs_model_para(0, sender, (s, _torch_wire(wire)))
    got = srv.history[-1]
    assert list(got.keys()) == list(out.keys())
    for k in out:
        _same_bits(got[k], out[k])


def test_wire_unpack_large_int8_int16_mix():
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    rng = np.random.default_rng(3)
    q8 = rng.integers(-127, 128, 1_000_003).astype(np.int8)
    q16 = rng.integers(-32767, 32768, 70_001).astype(np.int16)
    f = rng.standard_normal(4099).astype(np.float32)
    s8, s16 = np.float32(0.0123), np.float32(3.1e-5)
    off_f, off16 = 16, 16 + f.nbytes
    off8 = off16 + q16.nbytes
    buf = np.zeros(off8 + q8.nbytes, np.uint8)
    buf[:8].view(np.float32)[:] = [s8, s16]
    buf[off_f:off16].view(np.float32)[:] = f
    buf[off16:off8].view(np.int16)[:] = q16
    buf[off8:].view(np.int8)[:] = q8
    dev = torch.device('cuda')
    src = torch.from_numpy(buf).to(dev)
    out_n = 16 + 4099 + 70_001 + 1_000_003 + 64
    out = torch.full((out_n, ), -7.0, device=dev)
    d_f, d16, d8 = 16, 16 + 4099 + 3, 16 + 4099 + 3 + 70_001 + 5
    recs = [(off_f, d_f, 4099, L.FSAGG_WIRE_F32, -1),
            (off16, d16, 70_001, L.FSAGG_WIRE_I16, 1),
            (off8, d8, 1_000_003, L.FSAGG_WIRE_I8, 0)]
    segs = ops.wire_segments(recs, dev)
    scales = src[:8].view(torch.float32)
    ops.wire_unpack(src, segs, 3, 1_000_003, scales, out,
                    src_bytes=src.numel(), max_dst=out_n)
    o = out.cpu().numpy()
    assert o[d_f:d_f + 4099].tobytes() == f.tobytes()
    assert o[d16:d16 + 70_001].tobytes() == \
        (q16.astype(np.float32) * s16).tobytes()
    assert o[d8:d8 + 1_000_003].tobytes() == \
        (q8.astype(np.float32) * s8).tobytes()
    # untouched gaps keep their contents
    assert (o[:16] == -7.0).all() and (o[d_f + 4099:d16] == -7.0).all()


class _Recover:
    """Stands in for ``AdditiveSecretSharing(...).fixedpoint2float`` — the
    recover function the reference's server hands the aggregator.  The
    device path only reads its fixed-point constants (core/secret_sharing
    ss_params) and must never call it."""

    def __init__(self, meta):
        self.mod_number = int(meta['mod_number'])
        self.maximum = int(meta['maximum'])
        self.epsilon = meta['epsilon']

    def __call__(self, x):
        raise AssertionError('the device path called recover_fun')


@pytest.mark.parametrize('name', case_names('ss_'))
def test_secret_sharing_fedavg_bit_exact(name):
    """Shares written by the reference's clients (secret_split + the share
    exchange, tools/gen_golden_wire.py) through the use_ss branch, with and
    without ignore_weight (weight 1/n in float64, :77-82)."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    meta, clients, out, _, _ = load_case(name)
    iw = meta.get('ignore_weight', False)
    c = _cfg(use_ss=True)
    c.federate.ignore_weight = iw
    agg = ClientsAvgAggregator(device='cuda', config=c)
    got = agg.aggregate({'client_feedback': clients,
                         'recover_fun': _Recover(meta)})
    assert list(got.keys()) == list(out.keys())
    for k in out:
        _same_bits(got[k], out[k])
    # no recover function: the float64 weighted share sums (numpy's x*w)
    sums = agg.aggregate({'client_feedback': clients, 'recover_fun': None})
    w = 1.0 / len(clients) if iw else 1.0
    for k in out:
        acc = None
        for _, m in clients:
            x = np.asarray(m[k]).astype(np.float64) * w
            acc = x if acc is None else acc + x
        _same_bits(sums[k], acc)


@pytest.mark.parametrize('n,P', [(100, 1_000_000), (7, 1001), (3, 1)])
def test_secret_sharing_large_vs_oracle(n, P):
    """Parties' share sums (int64 and float64 rows, wrapped int64 sums
    included; odd lengths hit the kernel's single-element tail) against the
    oracle restatement."""
    from federatedscope_amd import ops
    rng = np.random.default_rng(11 + P)
    mod = 2 * 2**60 + 1
    shares = []
    for i in range(n):
        if i % 3:
            shares.append(rng.integers(-2**62, 2**62, P, dtype=np.int64))
        else:
            shares.append(rng.integers(0, mod, P).astype(np.float64))
    sizes = [int(s) for s in rng.integers(1, 500, n)]
    want = O.ss_fedavg([(s, {'w': x}) for s, x in zip(sizes, shares)], mod,
                       2**60, 1e8)['w']
    dev = torch.device('cuda')
    got = ops.ss_recover([torch.from_numpy(x).to(dev) for x in shares],
                         float(mod), float(2**60), 1e8, float(sum(sizes)))
    assert got.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize('name', case_names('dissim_'))
def test_dissimilarity_metrics(name):
    from federatedscope_amd.core.monitors import (calc_blocal_dissim,
                                                  calc_l2_dissim)
    _, clients, _, last, extra = load_case(name)
    tl = OrderedDict((k, torch.from_numpy(v)) for k, v in last.items())
    tc = [(s, OrderedDict((k, torch.from_numpy(v)) for k, v in m.items()))
          for s, m in clients]
    l2 = calc_l2_dissim(tl, tc)
    np.testing.assert_allclose(l2['raw'], extra['l2_raw'], rtol=1e-5)
    np.testing.assert_allclose(l2['mean'], extra['l2_mean'], rtol=1e-5)
    ol2 = O.calc_l2_dissim(last, clients)
    np.testing.assert_allclose(l2['raw'], ol2['raw'], rtol=1e-12)
    bl = calc_blocal_dissim(tl, tc)
    assert list(bl.keys()) == [str(k) for k in extra['blocal_keys']]
    np.testing.assert_allclose(list(bl.values()), extra['blocal'], rtol=1e-4)
    obl = O.calc_blocal_dissim(last, clients)
    np.testing.assert_allclose(list(bl.values()), list(obl.values()),
                               rtol=1e-9)


@pytest.mark.parametrize('name', case_names('quantlayout_'))
def test_quant_plan_layouts(name):
    """Wire dicts written by the reference's client-side quantisation for
    layouts with only quantised keys, only fp32 keys, int16 codes and odd
    sizes (region offsets, scale table, gaps) through WireStager, against
    the reference's own dequantisation."""
    from federatedscope_amd.core.compression import QuantPlan, WireStager
    _, clients, out, _, _ = load_case(name)
    wire = _torch_wire(clients[0][1])
    plan = QuantPlan(wire)
    st = WireStager(plan, 'cuda')
    row = torch.full((plan.layout.numel, ), 9.0, device='cuda')
    st.put(wire, row)
    st.finish()
    got = plan.layout.unpack(row)
    assert list(got.keys()) == list(out.keys())
    for k in out:
        _same_bits(got[k], np.asarray(out[k], np.float32))


@pytest.mark.parametrize('name', case_names('dissim_'))
def test_dissimilarity_metrics_in_place(name):
    """Device-resident client dicts take the key-table path (no staging);
    its sums are bit-identical to the staged path's."""
    from federatedscope_amd.core.monitors import (calc_blocal_dissim,
                                                  calc_l2_dissim)
    _, clients, _, last, extra = load_case(name)
    tl = OrderedDict((k, torch.from_numpy(v)) for k, v in last.items())
    host = [(s, OrderedDict((k, torch.from_numpy(v)) for k, v in m.items()))
            for s, m in clients]
    dev = [(s, OrderedDict((k, v.cuda()) for k, v in m.items()))
           for s, m in host]
    assert calc_l2_dissim(tl, dev)['raw'] == calc_l2_dissim(tl, host)['raw']
    np.testing.assert_allclose(calc_l2_dissim(tl, dev)['raw'],
                               extra['l2_raw'], rtol=1e-5)
    assert calc_blocal_dissim(tl, dev) == calc_blocal_dissim(tl, host)


def test_delta_keys_match_flat_odd_layouts():
    """KeyTable metric passes over odd-sized, empty and 4-byte-offset key
    tensors equal the flat (staged) passes bit for bit."""
    from federatedscope_amd import ops
    g = torch.Generator(device='cuda').manual_seed(9)
    sizes = [1, 0, 1023, 5, 300_001, 0, 7, 65_537]
    n = 13
    pool = torch.randn(n * (sum(sizes) + len(sizes)) + 8, device='cuda',
                       generator=g)
    clients, flat, off = [], [], 1   # start one element in: 4-B aligned
    for i in range(n):
        row = []
        for sz in sizes:
            row.append(pool[off:off + sz])
            off += sz + 1
        clients.append(row)
        flat.append(torch.cat(row))
    base = [torch.randn(sz, device='cuda', generator=g) for sz in sizes]
    kt = ops.KeyTable(clients, 'cuda')
    rows = ops.RowTable.from_tensors(flat)
    bflat = torch.cat(base)
    for b_keys, b_flat in ((base, bflat), (None, None)):
        want = ops.delta_sqnorm(rows, kt.offsets, base=b_flat)
        got = ops.delta_sqnorm_keys(kt, base=b_keys)
        assert torch.equal(got, want)
    w = [float(x) for x in np.random.default_rng(2).random(n)]
    out_k = torch.full((kt.numel, ), 7.0, device='cuda')
    out_f = torch.full((kt.numel, ), 7.0, device='cuda')
    ops.delta_wsum_keys(kt, w, base, out_k)
    ops.delta_wsum(rows, w, bflat, out_f)
    assert torch.equal(out_k, out_f)
    # the flat wsum against the oracle's op order (fp32, row order, from +0)
    x = torch.stack(flat).cpu().numpy()
    want = np.zeros(kt.numel, np.float32)
    b = bflat.cpu().numpy()
    for i in range(n):
        want = want + np.float32(w[i]) * (x[i] - b)
    assert out_f.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize('shift', [0, 1])
@pytest.mark.parametrize('n', [1, 2, 4, 5, 6, 13])
def test_delta_sqnorm_wsum_fused(n, shift):
    """calc_blocal_dissim's fused pass (one read of the clients): the global
    update is bit-identical to delta_wsum, the norms agree with
    delta_sqnorm to fp64 summation order, and the key-table and flat forms
    agree bit for bit — on whole 16-B-aligned chunks (shift 0), rows one
    element off alignment (shift 1: the guarded loads), chunk tails, empty
    and single-element keys."""
    from federatedscope_amd import ops
    g = torch.Generator(device='cuda').manual_seed(11 + n + shift)
    sizes = [1, 0, 1023, 5, 300_001, 0, 7, 65_537, 4096, 1024 * 37]
    pool = torch.randn(n * (sum(sizes) + 8 * len(sizes)) + 8, device='cuda',
                       generator=g)
    clients, flat, off = [], [], shift
    for i in range(n):
        row = []
        for sz in sizes:
            row.append(pool[off:off + sz])
            off += (sz + 3) // 4 * 4 + 4      # keys 16-B aligned + shift
            assert row[-1].numel() == sz
        clients.append(row)
        flat.append(torch.cat(row))
    base = [torch.randn(sz, device='cuda', generator=g) for sz in sizes]
    kt = ops.KeyTable(clients, 'cuda')
    rows = ops.RowTable.from_tensors(flat)
    bflat = torch.cat(base)
    w = [float(x) for x in np.random.default_rng(n).random(n)]
    want_sq = ops.delta_sqnorm(rows, kt.offsets, base=bflat)
    want_g = torch.empty(kt.numel, device='cuda')
    ops.delta_wsum(rows, w, bflat, want_g)
    out_k = torch.full((kt.numel, ), 7.0, device='cuda')
    out_f = torch.full((kt.numel, ), 7.0, device='cuda')
    sq_k = ops.delta_sqnorm_wsum_keys(kt, w, base, out_k)
    sq_f = ops.delta_sqnorm_wsum(rows, w, kt.offsets, bflat, out_f)
    assert torch.equal(out_k, want_g) and torch.equal(out_f, want_g)
    assert torch.equal(sq_k, sq_f)
    torch.testing.assert_close(sq_f, want_sq, rtol=1e-13, atol=0.0)
    # fp64 norms against a float64 numpy restatement of fl32(x − b)²
    x = torch.stack(flat).cpu().numpy()
    d = (x - bflat.cpu().numpy()).astype(np.float64)
    ref = np.add.reduceat(d * d, kt.offsets[:-1], axis=1)
    for s, sz in enumerate(sizes):      # reduceat gives d[off] for empties
        if sz == 0:
            ref[:, s] = 0.0
    np.testing.assert_allclose(sq_f.cpu().numpy(), ref, rtol=1e-12)


def test_wire_unpack_skips_malformed_segments():
    """The segment table is device data: segments that overrun the packed
    input or the row, or name an unknown kind / scale, are skipped on the
    device (nothing written, no fault); the valid ones still decode."""
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    dev = torch.device('cuda')
    f = np.arange(16, dtype=np.float32) + 1.0
    src = torch.from_numpy(f.view(np.uint8).copy()).to(dev)      # 64 B
    scales = torch.tensor([0.5], device=dev)
    recs = [(0, 0, 4, L.FSAGG_WIRE_F32, -1),      # valid
            (0, 98, 4, L.FSAGG_WIRE_F32, -1),     # row overrun
            (60, 10, 4, L.FSAGG_WIRE_F32, -1),    # input overrun
            (0, 20, 4, 7, -1),                    # unknown kind
            (0, 30, 4, L.FSAGG_WIRE_I8, 5),       # scale index out of range
            (0, 40, -3, L.FSAGG_WIRE_F32, -1),    # negative length
            (1, 50, 2, L.FSAGG_WIRE_I16, 0),      # misaligned int16 source
            (16, 60, 8, L.FSAGG_WIRE_I8, 0)]      # valid int8
    arr = np.zeros(len(recs), dtype=ops.WIRE_SEG_DTYPE)
    for i, r in enumerate(recs):
        arr[i] = r
    segs = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
    out = torch.full((100, ), -1.0, device=dev)
    ops.wire_unpack(src, segs, len(recs), 8, scales, out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert o[:4].tolist() == [1.0, 2.0, 3.0, 4.0]
    q = f.view(np.uint8)[16:24].view(np.int8).astype(np.float32)
    assert o[60:68].tobytes() == (q * np.float32(0.5)).tobytes()
    mask = np.ones(100, bool)
    mask[:4] = False
    mask[60:68] = False
    assert (o[mask] == -1.0).all()


# -- gRPC uploads: base64 text decoded on the device -------------------------
def _b64_device_puts():
    from federatedscope_amd.core.compression.b64wire import STATS
    return STATS['device_puts']


@pytest.mark.parametrize('name', case_names('b64_'))
def test_b64_fedavg_golden(name):
    """The reference's own gRPC uploads (str values from b64serializer)
    aggregated by ClientsAvgAggregator on the GPU: the fp32 keys' base64
    characters are decoded into the device stack by fsagg_b64_unpack_f32;
    the aggregate is bit-identical to the reference's."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    meta, clients, out, _, _ = load_case(name)
    c = _cfg()
    c.federate.ignore_weight = meta.get('ignore_weight', False)
    agg = ClientsAvgAggregator(device='cuda', config=c)
    before = _b64_device_puts()
    got = agg.aggregate({'client_feedback': [(s, OrderedDict(d))
                                             for s, d in clients],
                         'recover_fun': None})
    # every client went through the kernel (the views case's transposed
    # key alone is decoded on the host)
    assert _b64_device_puts() - before == len(clients)
    assert list(got.keys()) == list(out.keys())
    for k in out:
        _same_bits(got[k], out[k])


@pytest.mark.parametrize('name', ['b64_fedavg_n5', 'b64_iw_n3'])
def test_b64_uploads_through_server(name):
    """Server.callback_funcs_model_para with gRPC uploads: each upload's
    base64 is staged into its device-stack slot on arrival."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.workers.ingress import StagedUpdate
    from federatedscope_amd.core.workers.server import AggregationServer
    meta, clients, out, _, _ = load_case(name)
    c = _cfg()
    c.federate.ignore_weight = meta.get('ignore_weight', False)

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict()

        def load_state_dict(self, sd, strict=True):
            self.loaded = sd

    srv = AggregationServer(M(), ClientsAvgAggregator(device='cuda',
                                                      config=c),
                            sample_client_num=len(clients), keep_history=1)
    before = _b64_device_puts()
    for sender, (s, d) in enumerate(clients):
        srv.callback_funcs_model_para(0, sender, (s, OrderedDict(d)))
        if sender < len(clients) - 1:
            staged = srv.msg_buffer['train'][0][sender][1]
            assert isinstance(staged, StagedUpdate)
    assert _b64_device_puts() - before == len(clients)
    got = srv.history[-1]
    assert list(got.keys()) == list(out.keys())
    for k in out:
        _same_bits(got[k], out[k])


def _b64(t):
    import base64
    import pickle
    return base64.b64encode(pickle.dumps(t)).decode()


def test_b64_rows_every_phase_and_size():
    """HostStager's device decode of str uploads, row by row: keys of 1..40
    and a few thousand elements, sliced out of larger storages at offsets
    0..2 (so the data starts at every byte phase of a 4-char group), one
    absent key; the row holds exactly the tensors' bytes and zero
    padding."""
    from federatedscope_amd.layout import BucketLayout, ClientStack
    rng = np.random.default_rng(7)
    sizes = list(range(1, 41)) + [1000, 4097, 65536 + 3]
    tmpl = OrderedDict(('k%d' % i, torch.zeros(m))
                       for i, m in enumerate(sizes))
    lay = BucketLayout(tmpl)
    ups, want = [], []
    for c in range(3):
        d, w = OrderedDict(), torch.zeros(lay.numel)
        for i, m in enumerate(sizes):
            if c == 1 and i == 5:
                continue                       # an absent key
            base = torch.from_numpy(
                rng.standard_normal(m + 5).astype(np.float32))
            t = base[c:c + m]
            d['k%d' % i] = _b64(t)
            w[lay.offsets['k%d' % i]:lay.offsets['k%d' % i] + m] = t
        ups.append(d)
        want.append(w)
    st = ClientStack(lay, 3, 'cuda')
    st.slab.fill_(float('nan'))                # padding must be written
    before = _b64_device_puts()
    st.load_many(ups)
    torch.cuda.synchronize()
    assert _b64_device_puts() - before == 3
    for c in range(3):
        g = st.slab[c].cpu().numpy()
        assert g.tobytes() == want[c].numpy().tobytes(), c


def test_b64_large_round_trip():
    """A 25M-parameter key (the C3 model's size, 133 MB of base64): decode
    on the device == the tensor that was pickled (encode→decode round
    trip)."""
    from federatedscope_amd.layout import BucketLayout, ClientStack
    t = torch.randn(25_000_000)
    lay = BucketLayout({'w': torch.zeros(25_000_000)})
    st = ClientStack(lay, 1, 'cuda')
    st.load_many([{'w': _b64(t)}])
    torch.cuda.synchronize()
    assert torch.equal(st.slab[0, :t.numel()].cpu(), t)


def test_b64_bad_character_in_data_raises():
    """A character outside the base64 alphabet inside the tensor data (the
    host never reads those characters) is caught by the kernel and raised
    when the staging finishes."""
    from federatedscope_amd.core.compression.b64wire import FramingError
    from federatedscope_amd.layout import BucketLayout, ClientStack
    t = torch.randn(100_000)
    txt = _b64(t)
    mid = len(txt) // 2
    bad = txt[:mid] + '*' + txt[mid + 1:]
    lay = BucketLayout({'w': torch.zeros(100_000)})
    st = ClientStack(lay, 1, 'cuda')
    with pytest.raises(FramingError, match='alphabet'):
        st.load_many([{'w': bad}])
    st.load_many([{'w': txt}])                 # the stager state is clean
    torch.cuda.synchronize()
    assert torch.equal(st.slab[0, :100_000].cpu(), t)


def test_b64_rejected_upload_dropped_by_sender():
    """One sender's base64 carries a character outside the alphabet inside
    its tensor data: the server drops that sender's upload alone (recorded
    in rejected_uploads with its reason), keeps waiting, and aggregates
    once the sender re-uploads a clean one — bit-identical to the round
    without the bad upload."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.workers.server import AggregationServer
    meta, clients, out, _, _ = load_case('b64_fedavg_n5')
    c = _cfg()

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict()

        def load_state_dict(self, sd, strict=True):
            self.loaded = sd

    srv = AggregationServer(M(), ClientsAvgAggregator(device='cuda',
                                                      config=c),
                            sample_client_num=len(clients), keep_history=1)
    bad_sender = 2
    s2, d2 = clients[bad_sender]
    k = max(d2, key=lambda key: len(d2[key]) if isinstance(d2[key], str)
            else 0)
    txt = d2[k]
    mid = len(txt) // 2
    corrupt = OrderedDict(d2)
    corrupt[k] = txt[:mid] + '*' + txt[mid + 1:]
    for sender, (s, d) in enumerate(clients):
        moved = srv.callback_funcs_model_para(
            0, sender, (s, corrupt if sender == bad_sender else
                        OrderedDict(d)))
    assert moved is False and srv.state == 0
    assert [(r, snd) for r, snd, _ in srv.rejected_uploads] == \
        [(0, bad_sender)]
    assert 'alphabet' in srv.rejected_uploads[0][2]
    assert bad_sender not in srv.msg_buffer['train'][0]
    assert srv.callback_funcs_model_para(0, bad_sender, (s2, OrderedDict(d2)))
    got = srv.history[-1]
    # arrival order differs from the fixture's (the sender re-uploaded
    # last): the reference's result for this order
    order = [i for i in range(len(clients)) if i != bad_sender] + \
        [bad_sender]
    want = O.para_weighted_avg([(clients[i][0], OrderedDict(
        (kk, O.b64_tensor(v) if isinstance(v, str) else v)
        for kk, v in clients[i][1].items())) for i in order])
    for kk in want:
        _same_bits(got[kk], want[kk])


def test_b64_rejected_then_retried_before_round_fills():
    """A sender's corrupt upload followed, in the same round and before the
    buffer fills, by a clean retry into the same slot: only the sender's
    latest put decides, so nothing is dropped and the round aggregates the
    retry (rejections were matched by sender tag alone)."""
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.workers.server import AggregationServer
    meta, clients, out, _, _ = load_case('b64_fedavg_n5')
    c = _cfg()

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict()

        def load_state_dict(self, sd, strict=True):
            self.loaded = sd

    srv = AggregationServer(M(), ClientsAvgAggregator(device='cuda',
                                                      config=c),
                            sample_client_num=len(clients), keep_history=1)
    bad_sender = 2
    s2, d2 = clients[bad_sender]
    k = max(d2, key=lambda key: len(d2[key]) if isinstance(d2[key], str)
            else 0)
    txt = d2[k]
    mid = len(txt) // 2
    corrupt = OrderedDict(d2)
    corrupt[k] = txt[:mid] + '*' + txt[mid + 1:]
    assert srv.callback_funcs_model_para(0, bad_sender,
                                         (s2, corrupt)) is False
    assert srv.callback_funcs_model_para(0, bad_sender,
                                         (s2, OrderedDict(d2))) is False
    moved = False
    for sender, (s, d) in enumerate(clients):
        if sender != bad_sender:
            moved = srv.callback_funcs_model_para(0, sender,
                                                  (s, OrderedDict(d)))
    assert moved is True and srv.rejected_uploads == []
    got = srv.history[-1]
    # the buffer keeps the sender's first arrival position
    order = [bad_sender] + [i for i in range(len(clients))
                            if i != bad_sender]
    want = O.para_weighted_avg([(clients[i][0], OrderedDict(
        (kk, O.b64_tensor(v) if isinstance(v, str) else v)
        for kk, v in clients[i][1].items())) for i in order])
    for kk in want:
        _same_bits(got[kk], want[kk])
