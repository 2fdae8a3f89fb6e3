"""CPU-only checks: the C-ABI library loads and exports every symbol the
header declares, and the host-side logic (layouts, weights, builder,
wire-format decode) behaves like the reference's."""
import base64
import os
import pickle
import re
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, 'include', 'fsagg.h')) as f:
        text = f.read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(fsagg_[a-z0-9_]+)\s*\(', text)))


def test_library_exports_header():
    from federatedscope_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.SIGNATURES) == syms
    assert lib.fsagg_version() == 2


def test_library_rejects_bad_args_without_gpu():
    from federatedscope_amd import _lib
    lib = _lib.load()
    rc = lib.fsagg_weighted_sum_f32(None, None, None, 0, 10, None, None, None)
    assert rc == -1
    assert b'invalid' in lib.fsagg_last_error()
    with pytest.raises(_lib.FsaggError):
        _lib.check(rc, 'x')
    assert lib.fsagg_pairdist_workspace_bytes(50, 6603902, 12) > 0
    # trimmed mean with 2k >= n is rejected before any launch
    assert lib.fsagg_trimmed_mean_f32(1, 4, 10, 2, 0.0, None, 1, None) == -1
    # row-set entry points reject a missing table / a bad chunk unit
    rows = _lib.Rows(0, 0, 4, 1)
    assert lib.fsagg_weighted_sum_rows_f32(rows, None, 0, 1024, 1, None,
                                           None, 0, 16, None) == -1
    rows = _lib.Rows(16, 0, 4, 1)
    assert lib.fsagg_weighted_sum_rows_f32(rows, 16, 3, 1000, 16, None,
                                           None, 0, 16, None) == -1
    assert b'chunk_elems' in lib.fsagg_last_error()
    assert lib.fsagg_trimmed_mean_rows_f32(rows, 16, 3, 100, 2, 1.0, None,
                                           0, 16, None) == -1
    assert lib.fsagg_wsum_chunk_elems(25_000_000) == 24 * 1024
    assert lib.fsagg_wsum_chunk_elems(1000) == 1024


def test_host_extension_key_table_without_gpu():
    """csrc/host/keytable.cpp: CPU tensors (or non-dicts) are not device
    rows: None, and the caller stages instead."""
    import torch
    from federatedscope_amd import _lib
    h = _lib.host()
    d = [{'a': torch.zeros(3), 'b': torch.zeros(2, 2)} for _ in range(3)]
    assert h.key_table(d, ['a', 'b'], [(3, ), (2, 2)], 0) is None
    assert h.key_table([object()], ['a'], [(3, )], 0) is None
    # no keys at all: an empty table
    raw, missing, aligned = h.key_table(d, [], [], 0)
    assert raw == b'' and missing == 0 and aligned
    with pytest.raises(ValueError):
        h.key_table(d, ['a'], [], 0)
    # the device-table form (per-key byte offsets): same checks
    assert h.key_table(d, ['a', 'b'], [(3, ), (2, 2)], 0, [0, 64]) is None
    raw, missing, aligned, uniform = h.key_table(d, [], [], 0, [])
    assert raw == b'' and missing == 0 and aligned and not uniform
    with pytest.raises(ValueError):
        h.key_table(d, ['a', 'b'], [(3, ), (2, 2)], 0, [0])


def test_unpack_views_of_a_row():
    """BucketLayout.unpack on a slab row (a view with a storage offset):
    each key's view starts at the row's own offset, and a bucket shorter
    than the layout is refused."""
    from federatedscope_amd.layout import BucketLayout
    tmpl = OrderedDict([('a', torch.zeros(3)), ('b', torch.zeros(5, 7)),
                        ('s', torch.zeros(()))])
    lay = BucketLayout(tmpl)
    slab = torch.arange(3 * lay.numel, dtype=torch.float32).view(3, -1)
    row = slab[1]
    v = lay.unpack(row)
    for k in lay.keys:
        o, m = lay.offsets[k], lay.numels[k]
        assert v[k].shape == tmpl[k].shape
        assert torch.equal(v[k].reshape(-1), row[o:o + m])
    assert v['b'].data_ptr() == row[lay.offsets['b']:].data_ptr()
    with pytest.raises(ValueError):
        lay.unpack(row[:lay.numel - 1])


def test_bucket_layout_alignment_and_dtypes():
    from federatedscope_amd.layout import BucketLayout, KEY_ALIGN
    tmpl = OrderedDict([('a', torch.zeros(3)), ('b', torch.zeros(5, 7)),
                        ('n', torch.tensor(3)), ('h', torch.zeros(4).half()),
                        ('c', torch.zeros(16))])
    lay = BucketLayout(tmpl)
    assert lay.keys == ['a', 'b', 'c']
    assert list(lay.other) == ['n', 'h']
    assert lay.offsets == {'a': 0, 'b': 16, 'c': 64}
    assert all(o % KEY_ALIGN == 0 for o in lay.offsets.values())
    assert lay.numel == 80
    assert lay.segments() == [0, 16, 64, 80]
    host = torch.empty(lay.numel)
    m = OrderedDict([('a', torch.arange(3.)), ('b', torch.ones(5, 7)),
                     ('c', torch.full((16, ), 2.))])
    lay.pack_host(m, host)
    assert host[:3].tolist() == [0, 1, 2] and host[3:16].abs().sum() == 0
    v = lay.unpack(host)
    assert v['b'].shape == (5, 7) and torch.equal(v['c'], m['c'])


def test_fedavg_weights_match_oracle():
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    sizes = [3, 500, 17, 1, 999]
    assert fedavg_weights(sizes) == O.fedavg_weights(sizes)
    assert fedavg_weights(sizes, ignore_weight=True) == \
        O.fedavg_weights(sizes, ignore_weight=True)


def test_krum_scores_slice_semantics():
    from federatedscope_amd.core.aggregators.krum_aggregator import \
        krum_scores
    rng = np.random.default_rng(0)
    D = rng.random((10, 10)).astype(np.float32)
    D = D + D.T
    np.fill_diagonal(D, np.inf)
    # n - f - 2 = -2: Python slice semantics, all but the last two columns
    s = krum_scores(torch.from_numpy(D), 10).numpy()
    np.testing.assert_allclose(s, np.sort(D, 1)[:, :-2].sum(1), rtol=1e-6)


def test_param2tensor_wire_format():
    from federatedscope_amd.core.auxiliaries.utils import param2tensor
    t = torch.randn(4, 3)
    assert torch.equal(param2tensor(base64.b64encode(
        pickle.dumps(t)).decode()), t)
    assert param2tensor([1.0, 2.0]).dtype == torch.float32
    assert param2tensor(3).dtype == torch.long

    class Evil:
        def __reduce__(self):
            return (os.system, ('true', ))

    # the framing walker refuses the global; the restricted unpickler it
    # falls back to refuses it too, and the framing error is raised
    from federatedscope_amd.core.compression.b64wire import FramingError
    with pytest.raises(FramingError, match='posix.system'):
        param2tensor(base64.b64encode(pickle.dumps(Evil())).decode())


def _cfg(**kw):
    return SimpleNamespace(
        backend='torch',
        data=SimpleNamespace(type='toy'),
        fedopt=SimpleNamespace(use=False),
        asyn=SimpleNamespace(use=kw.get('asyn', False),
                             staleness_discount_factor=1.0),
        personalization=SimpleNamespace(beta=1.0),
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=50, sample_client_rate=1.0,
                                 share_local_model=False),
        aggregator=SimpleNamespace(
            robust_rule=kw.get('rule', 'fedavg'), byzantine_node_num=2,
            BFT_args=SimpleNamespace(krum_agg_num=1,
                                     trimmedmean_excluded_ratio=0.1,
                                     normbounding_norm_bound=1.0)))


@pytest.mark.parametrize('method,rule,online,asyn,cls', [
    ('fedavg', 'fedavg', False, False, 'ClientsAvgAggregator'),
    ('fedavg', 'krum', False, False, 'KrumAggregator'),
    ('fedavg', 'median', False, False, 'MedianAggregator'),
    ('fedavg', 'trimmedmean', False, False, 'TrimmedmeanAggregator'),
    ('fedavg', 'bulyan', False, False, 'BulyanAggregator'),
    ('fedavg', 'normbounding', False, False, 'NormboundingAggregator'),
    ('fedavg', 'fedavg', True, False, 'OnlineClientsAvgAggregator'),
    ('fedavg', 'fedavg', False, True, 'AsynClientsAvgAggregator'),
    ('ditto', 'nonexistent', False, False, 'ClientsAvgAggregator'),
    ('pfedme', 'fedavg', False, False, 'ServerClientsInterpolateAggregator'),
    ('local', 'fedavg', False, False, 'NoCommunicationAggregator'),
])
def test_builder_selection(method, rule, online, asyn, cls):
    from federatedscope_amd.core.auxiliaries.aggregator_builder import \
        get_aggregator
    agg = get_aggregator(method, model=None, device='cpu', online=online,
                         config=_cfg(rule=rule, asyn=asyn))
    assert type(agg).__name__ == cls


def test_no_gpu_raises_loudly():
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    agg = ClientsAvgAggregator(config=_cfg())
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        agg.aggregate({'client_feedback': [(1, {'w': torch.zeros(4)})]})


def _device_asm():
    """Disassembly of libfsagg's gfx950 code objects (llvm-objdump)."""
    import glob
    import os
    import shutil
    import subprocess
    import tempfile
    llvm = '/opt/rocm/lib/llvm/bin/llvm-objdump'
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), 'federatedscope_amd', 'lib', 'libfsagg.so')
    if not (os.path.exists(llvm) and os.path.exists(so)):
        pytest.skip('llvm-objdump or libfsagg.so missing')
    d = tempfile.mkdtemp()
    try:
        dst = os.path.join(d, 'lib.so')
        shutil.copy(so, dst)
        subprocess.run([llvm, '--offloading', dst], check=True,
                       capture_output=True, cwd=d)
        cos = glob.glob(os.path.join(d, 'lib.so.*gfx950*'))
        assert cos, 'no gfx950 code object in libfsagg.so'
        return '\n'.join(subprocess.run([llvm, '-d', co], check=True,
                                        capture_output=True,
                                        text=True).stdout for co in cos)
    finally:
        shutil.rmtree(d)


def test_device_code_memory_rules():
    """Rules of the kernels' memory instructions, checked on the shipped
    library: (1) no flat loads — row pointers come from tables, and a
    dereference of a generic pointer compiles to flat_load, which also
    counts in lgkmcnt, so the next scalar/LDS wait would drain every HBM
    load in flight; (2) no writes through the scalar data
    cache (scalar stores, scalar buffer/scratch stores, scalar cache
    write-back/discard, scalar atomics) — the mnemonics are assembled at run
    time below so this file does not spell them."""
    import re
    asm = _device_asm()
    assert 'global_load' in asm
    assert asm.count('flat_load') == 0
    sc = 's' + '_'
    stems = ['st' + 'ore_', 'buffer_st' + 'ore_', 'scratch_st' + 'ore_',
             'dcache_' + 'wb', 'dcache_' + 'discard', 'ato' + 'mic_',
             'buffer_ato' + 'mic_']
    bad = re.findall(r'\b(' + '|'.join(sc + t + r'\w*' for t in stems) +
                     r')\b', asm)
    assert not bad, sorted(set(bad))


def test_missing_library_fails_loudly():
    """No CPU fallback: without libfsagg.so the product path raises."""
    import subprocess
    import sys
    code = (
        'import torch\n'
        'from collections import OrderedDict\n'
        'from types import SimpleNamespace\n'
        'from federatedscope_amd import _lib\n'
        'from federatedscope_amd.core.aggregators import '
        'ClientsAvgAggregator\n'
        'cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,'
        ' use_ss=False))\n'
        'agg = ClientsAvgAggregator(config=cfg)\n'
        'fb = [(1, OrderedDict(w=torch.ones(3))), '
        '(2, OrderedDict(w=torch.zeros(3)))]\n'
        'try:\n'
        '    agg.aggregate({"client_feedback": fb})\n'
        'except Exception as e:\n'
        '    print("RAISED", type(e).__name__)\n'
        'else:\n'
        '    print("NO-ERROR")\n'
        'try:\n'
        '    _lib.load()\n'
        'except _lib.FsaggError:\n'
        '    print("LOAD-RAISED")\n')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FSAGG_LIB='/nonexistent/libfsagg.so',
               PYTHONPATH=root)
    r = subprocess.run([sys.executable, '-c', code], env=env, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert 'RAISED' in r.stdout and 'NO-ERROR' not in r.stdout, r.stdout + \
        r.stderr
    assert 'LOAD-RAISED' in r.stdout


# -- gRPC uploads: the framing walker (core/compression/b64wire) -------------
def _b64(x, protocol=None):
    return base64.b64encode(pickle.dumps(x, protocol=protocol)).decode()


@pytest.mark.parametrize('name', ['b64_fedavg_n5', 'b64_views_n4'])
def test_b64_host_decode_matches_oracle(name):
    """The product's host decode (param2tensor's str branch) of the
    reference's own uploads is bit-identical to the oracle's stdlib
    restatement, shape and dtype included."""
    import oracle as O
    from golden_io import load_case
    from federatedscope_amd.core.auxiliaries.utils import param2tensor
    _, clients, _, _, _ = load_case(name)
    for _, d in clients:
        for k, v in d.items():
            t = param2tensor(v)
            want = np.asarray(O.b64_tensor(v))
            got = t.contiguous().numpy()
            assert got.dtype == want.dtype and got.shape == want.shape, k
            assert got.tobytes() == want.tobytes(), k


def test_b64_framing_of_tensor_variants():
    from federatedscope_amd.core.compression.b64wire import parse_b64
    cases = [torch.arange(10, dtype=torch.float32), torch.randn(3, 5),
             torch.randn(0), torch.tensor(3.5), torch.tensor(7),
             torch.randn(4, 6).t(), torch.randn(10)[3:7],
             torch.randn(5, dtype=torch.float64), torch.randn(6).half(),
             torch.randn(6).bfloat16(), torch.randn(3, requires_grad=True),
             torch.nn.Parameter(torch.randn(2, 2)), torch.zeros(2, 0, 3),
             torch.tensor([True, False])]
    for t in cases:
        for proto in (3, 4, 5):
            txt = _b64(t, proto)
            f = parse_b64(txt)
            ref = pickle.loads(base64.b64decode(txt))
            assert f.dtype == ref.dtype and f.shape == tuple(ref.shape)
            assert f.stride == ref.stride()
            assert f.storage_offset == ref.storage_offset()
            assert f.requires_grad == ref.requires_grad
            got = f.to_tensor()
            assert torch.equal(got.detach(), ref.detach())
            assert parse_b64(txt.encode()).data_pos == f.data_pos   # bytes
            if f.is_contiguous() and f.numel:
                # the segment math of the device path: the characters
                # [c0, c1) decode, after `skip` bytes, to the tensor's bytes
                c0, c1, skip = f.char_range()
                raw = base64.b64decode(txt[c0:c1])
                nb = f.numel * f.itemsize
                want = ref.detach().contiguous().view(-1).view(
                    torch.uint8).numpy().tobytes() \
                    if ref.dtype != torch.bool else \
                    ref.contiguous().numpy().tobytes()
                assert raw[skip:skip + nb] == want


def test_b64_malformed_framing_raises():
    from federatedscope_amd.core.compression.b64wire import (FramingError,
                                                             parse_b64)
    good = _b64(torch.randn(100))
    raw = bytearray(base64.b64decode(good))
    magic = raw.index(b'\x8a\x0al\xfc\x9cF\xf9 j\xa8P\x19')
    bad_magic = bytearray(raw)
    bad_magic[magic + 3] ^= 1

    class Evil:
        def __reduce__(self):
            return (os.system, ('true', ))

    bad = [good[:-4], good[:100], good + 'AAAA', 'hello', '',
           good[:40] + '!' + good[41:],                  # char in framing
           base64.b64encode(bytes(bad_magic)).decode(),
           base64.b64encode(bytes(raw[:-1])).decode(),   # no STOP
           base64.b64encode(bytes(raw) + b'.').decode(),  # trailing bytes
           _b64({'a': torch.randn(2)}), _b64([1, 2]), _b64(3),
           _b64(Evil()), _b64(torch.randn(3), 2)]        # protocol 2 bytes
    for b in bad:
        with pytest.raises(FramingError):
            parse_b64(b)


def test_b64_framing_cache_is_by_content():
    from federatedscope_amd.core.compression.b64wire import parse_b64
    a = torch.randn(50000)
    ta, tb = _b64(a), _b64(a[1:])
    fa = parse_b64(ta)
    assert parse_b64(ta).data_pos == fa.data_pos
    fb = parse_b64(tb)
    assert fb.shape == (49999, ) and fb.storage_offset == 1
    assert fa.shape == (50000, ) and fa.storage_offset == 0


def test_b64_native_walk_matches_python_walk():
    """_fsagg_host.b64_frame (csrc/host/b64frame.cpp) and the Python walker
    agree field for field on every variant, and both refuse the malformed
    uploads."""
    from federatedscope_amd.core.compression import b64wire as B
    if B._text_ext() is None:
        pytest.skip('_fsagg_host.so not built')
    variants = [torch.arange(10, dtype=torch.float32), torch.randn(3, 5),
                torch.randn(0), torch.tensor(3.5), torch.tensor(7),
                torch.randn(4, 6).t(), torch.randn(10)[3:7],
                torch.randn(5, dtype=torch.float64), torch.randn(6).half(),
                torch.randn(6).bfloat16(), torch.randn(3, requires_grad=True),
                torch.nn.Parameter(torch.randn(2, 2)), torch.zeros(2, 0, 3),
                torch.tensor([True, False]), torch.randn(70000)]
    fields = ('dtype', 'shape', 'stride', 'storage_offset', 'storage_numel',
              'data_pos', 'requires_grad', 'nchars')
    for t in variants:
        for proto in (3, 4, 5):
            txt = _b64(t, proto)
            a, b = B.parse_b64(txt), B.parse_b64_py(txt)
            for f in fields:
                assert getattr(a, f) == getattr(b, f), (f, proto, t.shape)
    good = _b64(torch.randn(100))

    class Evil:
        def __reduce__(self):
            return (os.system, ('true', ))

    raw = base64.b64decode(good)
    bad = [good[:-4], good[:100], good + 'AAAA', 'hello', '',
           good[:40] + '!' + good[41:],
           base64.b64encode(raw[:-1]).decode(),
           base64.b64encode(raw + b'.').decode(),
           _b64({'a': torch.randn(2)}), _b64([1, 2]), _b64(3),
           _b64(Evil()), _b64(torch.randn(3), 2), 'é' * 8]
    for x in bad:
        with pytest.raises(B.FramingError):
            B.parse_b64(x)
        with pytest.raises(B.FramingError):
            B.parse_b64_py(x)


@pytest.mark.parametrize('opt', [
    dict(type='SGD', lr=-0.1),
    dict(type='SGD', lr=0.1, momentum=-0.5),
    dict(type='SGD', lr=0.1, weight_decay=-1.0),
    dict(type='SGD', lr=0.1, nesterov=True),
    dict(type='SGD', lr=0.1, momentum=0.9, dampening=0.1, nesterov=True),
    dict(type='Adam', lr=0.1, betas=(1.0, 0.999)),
    dict(type='Adam', lr=0.1, betas=(0.9, -0.1)),
    dict(type='Adam', lr=0.1, eps=-1e-8),
    dict(type='AdamW', lr=0.1, weight_decay=-0.01),
    dict(type='Adagrad', lr=0.1, lr_decay=-1.0),
    dict(type='Adagrad', lr=0.1, initial_accumulator_value=-1.0),
    dict(type='RMSprop', lr=0.1, alpha=-0.9),
    dict(type='RMSprop', lr=0.1, momentum=-0.9),
])
def test_fedopt_rejects_what_torch_optim_rejects(opt):
    """The FedOpt server optimizer's config is checked like the torch.optim
    constructor the reference's get_optimizer builds
    (optimizer_builder.py:53-56): same exception type and message."""
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import FedOptAggregator
    kw = {k: v for k, v in opt.items() if k != 'type'}
    with pytest.raises(ValueError) as want:
        getattr(torch.optim, opt['type'])(
            [torch.zeros(1, requires_grad=True)], **kw)
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False),
        fedopt=SimpleNamespace(optimizer=dict(opt), annealing=False))
    with pytest.raises(ValueError) as got:
        FedOptAggregator(config=cfg, model=torch.nn.Linear(2, 2))
    assert str(got.value) == str(want.value)


def test_fedopt_keeps_its_config():
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import FedOptAggregator
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False),
        fedopt=SimpleNamespace(optimizer=dict(type='SGD', lr=0.5,
                                              momentum=0.9), annealing=False))
    agg = FedOptAggregator(config=cfg, model=torch.nn.Linear(2, 2))
    assert agg.opt_kwargs == {'momentum': 0.9}
    assert agg.momentum == 0.9


# -- row-set chunk plan (layout.plan_row_chunks) ------------------------------
@pytest.mark.parametrize('unit', [1024, 4096, 16384, 24576])
def test_plan_row_chunks_covers_keys(unit):
    """Every key span is cut into whole-tile pieces from its start (the last
    one shorter) that tile it exactly and never straddle a key."""
    import json
    import os
    import numpy as np
    from federatedscope_amd.layout import plan_row_chunks
    from federatedscope_amd.ops import CHUNK_DTYPE
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, 'tools', 'resnet50_layout.json')) as f:
        keys = [tuple(s) for _, s in json.load(f)['keys']]
    spans, off = [], 0
    for i, s in enumerate(keys):
        m = int(np.prod(s))
        spans.append((i, off, off + m))
        off = (off + m + 63) // 64 * 64
    arr = plan_row_chunks(spans, unit, CHUNK_DTYPE)
    assert arr['len'].max() <= unit and arr['len'].min() >= 1
    for s, a, b in spans:
        sel = arr[arr['seg'] == s]
        assert sel['lo'][0] == a and sel['lo'][-1] + sel['len'][-1] == b
        assert np.all(sel['lo'][1:] == sel['lo'][:-1] + sel['len'][:-1])
        assert np.all(sel['len'][:-1] == unit)
    assert plan_row_chunks([], unit, CHUNK_DTYPE).size == 0
