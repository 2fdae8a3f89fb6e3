"""The native host pack (_fsagg_host.host_pack): host buffers and zero runs
packed into one destination by a persistent thread pool with non-temporal
stores — the host half of layout.HostStager's pinned staging.  CPU only:
the destination here is ordinary memory."""
import numpy as np
import pytest


def _ext():
    from federatedscope_amd.core.aggregators._engine import _host_ext
    h = _host_ext()
    if h is None or not hasattr(h, 'host_pack'):
        pytest.skip('_fsagg_host.so not built')
    return h


@pytest.mark.parametrize('threads', [1, 3, 16])
def test_host_pack_items_and_zeros(threads):
    h = _ext()
    rng = np.random.default_rng(threads)
    sizes = [1, 7, 4096, 3 << 20, 13, (5 << 20) + 3, 0, 64]
    srcs = [rng.standard_normal(s).astype(np.float32) for s in sizes]
    # layout: each item at a 4-B offset with gaps of zeros between some
    items, off, want = [], 0, []
    for i, a in enumerate(srcs):
        items.append((a, a.nbytes, off))
        want.append((off, a.view(np.uint8)))
        off += a.nbytes
        if i % 3 == 1:
            items.append((None, 4 * 1001, off))
            want.append((off, np.zeros(4 * 1001, np.uint8)))
            off += 4 * 1001
    dst = np.full(off + 64, 0xAB, dtype=np.uint8)
    h.host_pack(items, dst.ctypes.data, threads)
    for o, ref in want:
        assert np.array_equal(dst[o:o + ref.size], ref)
    assert (dst[off:] == 0xAB).all()          # nothing past the last item


def test_host_pack_repeated_and_unaligned():
    h = _ext()
    rng = np.random.default_rng(5)
    a = rng.standard_normal((9 << 20) // 4).astype(np.float32)
    for shift in (0, 4, 12, 60):
        dst = np.zeros(a.nbytes + 128, dtype=np.uint8)
        h.host_pack([(a, a.nbytes, shift)], dst.ctypes.data, 8)
        assert np.array_equal(dst[shift:shift + a.nbytes], a.view(np.uint8))
        assert not dst[:shift].any() and not dst[shift + a.nbytes:].any()


def test_host_pack_rejects_short_source():
    h = _ext()
    a = np.zeros(10, np.float32)
    dst = np.zeros(100, np.uint8)
    with pytest.raises(ValueError):
        h.host_pack([(a, 41, 0)], dst.ctypes.data, 2)


def test_native_pack_matches_pack_host():
    """layout._native_pack against BucketLayout.pack_host on a layout with
    padding, an absent key and a zero-size key (CPU tensors)."""
    import torch
    from collections import OrderedDict
    from federatedscope_amd.layout import BucketLayout, _native_pack
    _ext()
    g = torch.Generator().manual_seed(3)
    tmpl = OrderedDict([('a', torch.rand(1001, generator=g)),
                        ('b', torch.rand(3, 5, generator=g)),
                        ('e', torch.rand(0)),
                        ('c', torch.rand(70_000, generator=g))])
    lay = BucketLayout(tmpl)
    model = OrderedDict((k, torch.rand(v.shape, generator=g))
                        for k, v in tmpl.items() if k != 'b')
    want = torch.full((lay.numel,), 7.0)
    lay.pack_host(model, want)
    got = torch.full((lay.numel,), -3.0)
    assert _native_pack(lay, model, got)
    assert torch.equal(got, want)
    # a non-contiguous or non-fp32 key: not taken, nothing written
    bad = OrderedDict(model)
    bad['c'] = model['c'].double()
    got2 = torch.full((lay.numel,), -3.0)
    assert not _native_pack(lay, bad, got2)
    assert (got2 == -3.0).all()


def test_native_pack_range_stack():
    """The parameter-range shard's pack (RangeStack: this rank's pieces of
    every key) through host_pack equals RangeStack.pack_host."""
    import torch
    from collections import OrderedDict
    from federatedscope_amd.layout import (BucketLayout, RangeStack,
                                           _native_pack)
    _ext()
    g = torch.Generator().manual_seed(4)
    tmpl = OrderedDict([('a', torch.rand(1001, generator=g)),
                        ('b', torch.rand(3, 5, generator=g)),
                        ('c', torch.rand(70_000, generator=g))])
    lay = BucketLayout(tmpl)
    # the constructor's span bookkeeping, without its device slab
    rs = RangeStack.__new__(RangeStack)
    pieces = [(5, 900), (1010, 40_000), (60_000, lay.numel)]
    rs.layout = lay
    rs.pieces = pieces
    rs.loc, off = [], 0
    for a, b in pieces:
        rs.loc.append(off)
        off += -(-max(b - a, 0) // RangeStack.ALIGN) * RangeStack.ALIGN
    rs.numel = off
    rs.spans = []
    for (a, b), loc in zip(pieces, rs.loc):
        sp = []
        for k in lay.keys:
            o, m = lay.offsets[k], lay.numels[k]
            x, y = max(a, o), min(b, o + m)
            if y > x:
                sp.append((k, x - o, loc + x - a, y - x))
        rs.spans.append(sp)
    model = OrderedDict((k, torch.rand(v.shape, generator=g))
                        for k, v in tmpl.items())
    want = torch.full((rs.numel,), 5.0)
    rs.pack_host(model, want)
    got = torch.full((rs.numel,), 5.0)
    assert _native_pack(rs, model, got)
    assert torch.equal(got, want)


def test_quant_plan_native_pack_matches_cat():
    """QuantPlan.pack_host through host_pack (int8 / int16 codes and fp32
    keys at their regions) is byte-identical to the torch.cat path."""
    import torch
    from collections import OrderedDict
    from federatedscope_amd.core.compression import wire as W
    _ext()
    g = torch.Generator().manual_seed(6)

    def codes(shape, dt):
        lim = 127 if dt == torch.int8 else 32767
        return torch.randint(-lim, lim + 1, shape, generator=g).to(dt)
    tmpl = OrderedDict([
        ('conv.weight_quant', codes((64, 3, 3, 3), torch.int8)),
        ('conv.weight_scale', torch.tensor(0.01)),
        ('bn.bias', torch.rand(64, generator=g)),
        ('fc.weight_quant', codes((10, 5001), torch.int16)),
        ('fc.weight_scale', torch.tensor(0.002)),
        ('fc.bias', torch.rand(10, generator=g)),
        ('head.weight_quant', codes((777,), torch.int8)),
        ('head.weight_scale', torch.tensor(0.5))])
    plan = W.QuantPlan(tmpl)
    up = OrderedDict((k, (codes(v.shape, v.dtype) if v.dtype in
                          (torch.int8, torch.int16) else
                          torch.rand(v.shape, generator=g)))
                     for k, v in tmpl.items())
    want = torch.full((plan.nbytes,), 0x5A, dtype=torch.uint8)
    got = want.clone()
    plan.pack_host(up, got)
    assert plan._pack_native(up, got)
    ref = want.clone()
    # the torch.cat path on the same buffer bytes
    scales = ref[:4 * max(plan.nscale, 1)].view(torch.float32)
    for j, sk in enumerate(plan.scale_keys):
        scales[j] = float(up[sk])
    for dt, a, b, wkeys in plan.spans:
        torch.cat([up[wk].reshape(-1) for wk in wkeys], out=ref[a:b].view(dt))
    assert torch.equal(got, ref)


def test_quant_plan_checked_pack_rejects_like_check():
    """pack_host_checked packs exactly when QuantPlan.check would pass: a
    wrong dtype, a wrong size or a missing scale makes it return False (the
    caller then raises through check)."""
    import torch
    from collections import OrderedDict
    from federatedscope_amd.core.compression import wire as W
    _ext()
    tmpl = OrderedDict([
        ('conv.weight_quant', torch.zeros(8, 3, dtype=torch.int8)),
        ('conv.weight_scale', torch.tensor(0.01)),
        ('bias', torch.zeros(8))])
    plan = W.QuantPlan(tmpl)
    buf = torch.zeros(plan.nbytes, dtype=torch.uint8)
    good = OrderedDict([
        ('conv.weight_quant', torch.ones(8, 3, dtype=torch.int8)),
        ('conv.weight_scale', torch.tensor(0.5)),
        ('bias', torch.full((8,), 2.0))])
    assert plan.pack_host_checked(good, buf)
    ref = torch.zeros_like(buf)
    plan.pack_host(good, ref)
    assert torch.equal(buf, ref)
    for bad in (
            OrderedDict(good, **{'conv.weight_quant':
                                 torch.ones(8, 3, dtype=torch.int16)}),
            OrderedDict(good, bias=torch.zeros(9)),
            OrderedDict((k, v) for k, v in good.items()
                        if k != 'conv.weight_scale')):
        assert not plan.pack_host_checked(bad, buf)
        with pytest.raises((ValueError, KeyError)):
            plan.check(bad)
