"""Client buckets: flattening per-client state_dicts into device rows.

A :class:`BucketLayout` maps the fp32 keys of a model (client 0's key order —
the order every reference aggregator iterates, e.g.
clients_avg_aggregator.py:70) to ``(offset, numel, shape)`` inside one flat
fp32 bucket.  Every key starts on a 16-element (64-byte) boundary so that any
key is itself a 16-byte-aligned sub-bucket (per-key launches for keys some
clients lack reuse the same rows).  Keys of other dtypes (fp16, bf16, fp64,
int64 — SURVEY A5) are listed separately and reduced per key.

A :class:`ClientStack` is the device-resident ``[capacity][numel]`` slab the
server fills as client updates arrive (host dicts are staged through pinned
buffers and copied asynchronously) and the aggregators stream over.
"""
import os
from collections import OrderedDict

import torch

from .core.auxiliaries.utils import param2tensor, param_meta

KEY_ALIGN = 16  # elements


def plan_row_chunks(spans, unit, dtype):
    """The chunk list of key spans [(seg, lo, hi)]: pieces of exactly
    ``unit`` coordinates (a whole tile of the row-set kernel) from each
    key's start, its last piece shorter, in key order.  Measured and not
    kept at the ResNet-50 layout (tools/probe_layout_b.py, profiles/r04/):
    balanced equal pieces (slower: nearly every piece then takes the
    kernel's guarded partial-tile path), short pieces first (no change) and
    longest first (2.5 % slower than key order, whose row-set kernel runs
    at the flat kernel's time on that box)."""
    import numpy as np
    parts = []
    for s, a, b in spans:
        st = np.arange(a, b, unit, dtype=np.int64)
        part = np.zeros(len(st), dtype=dtype)
        part['lo'] = st
        part['len'] = np.minimum(unit, b - st)
        part['seg'] = s
        parts.append(part)
    return np.concatenate(parts) if parts else np.zeros(0, dtype=dtype)


class BucketLayout:
    def __init__(self, template):
        self.keys = []          # fp32 keys in template order
        self.offsets = {}
        self.numels = {}
        self.shapes = {}
        self.other = OrderedDict()  # key -> dtype (non-fp32 keys)
        self.order = list(template.keys())
        off = 0
        for k, v in template.items():
            t = param_meta(v)
            if not isinstance(t, torch.Tensor):
                t = torch.as_tensor(t)
            if t.dtype == torch.float32:
                self.keys.append(k)
                self.offsets[k] = off
                self.numels[k] = t.numel()
                self.shapes[k] = tuple(t.shape)
                off += -(-t.numel() // KEY_ALIGN) * KEY_ALIGN
            else:
                self.other[k] = t.dtype
                self.shapes[k] = tuple(t.shape)
        self.numel = max(off, KEY_ALIGN)

    def signature(self):
        sig = self.__dict__.get('_signature')
        if sig is None:
            sig = self.__dict__['_signature'] = (
                tuple(self.order), tuple((k, self.shapes[k])
                                         for k in self.keys),
                tuple(self.other.items()))
        return sig

    @property
    def key_numels(self):
        """[(key, numel)] of the fp32 keys in layout order."""
        kn = self.__dict__.get('_key_numels')
        if kn is None:
            kn = self.__dict__['_key_numels'] = [(k, self.numels[k])
                                                 for k in self.keys]
        return kn

    def chunk_tables(self, device):
        """Device tables for fsagg_gather_rows_f32: key offsets, key lengths
        and the bucket as chunks of <= FSAGG_STACK_CHUNK coordinates that
        never straddle a key (built once per layout and device)."""
        from .ops import _h2d
        from ._lib import FSAGG_STACK_CHUNK as CH
        device = torch.device(device)
        cache = self.__dict__.setdefault('_chunk_tables', {})
        if str(device) not in cache:
            ck, cs = [], []
            for s, k in enumerate(self.keys):
                for st in range(0, self.numels[k], CH):
                    ck.append(s)
                    cs.append(st)
            cache[str(device)] = (
                _h2d([self.offsets[k] for k in self.keys], torch.int64,
                     device),
                _h2d([self.numels[k] for k in self.keys], torch.int64,
                     device),
                _h2d(ck, torch.int32, device), _h2d(cs, torch.int64, device))
        return cache[str(device)]

    def row_chunks(self, unit, device, lo=0, hi=None):
        """Device chunk table (struct fsagg_chunk, include/fsagg.h) of the
        fp32 keys' coordinates inside [lo, hi), cut into pieces of at most
        ``unit`` that never straddle a key (padding between keys is never
        part of a chunk; plan_row_chunks).  Cached per (unit, range,
        device); returns (uint8 device tensor, nchunk)."""
        from .ops import CHUNK_DTYPE, _h2d_bytes
        hi = self.numel if hi is None else hi
        device = torch.device(device)
        cache = self.__dict__.setdefault('_row_chunks', {})
        ck = (int(unit), int(lo), int(hi), str(device))
        if ck not in cache:
            spans = []
            for s, k in enumerate(self.keys):
                a = max(self.offsets[k], lo)
                b = min(self.offsets[k] + self.numels[k], hi)
                if b > a:
                    spans.append((s, a, b))
            arr = plan_row_chunks(spans, unit, CHUNK_DTYPE)
            cache[ck] = (_h2d_bytes(arr, device) if len(arr) else None,
                         len(arr))
        return cache[ck]

    def seg_bounds(self, device, lo=0, hi=None, keep=None):
        """Device int64 arrays (seg_lo, seg_end) of each fp32 key's exact
        coordinates clipped to [lo, hi) (empty segments where a key lies
        outside, or where ``keep`` — a predicate on the key's element count
        — is false), cached per range, predicate and device."""
        hi = self.numel if hi is None else hi
        device = torch.device(device)
        cache = self.__dict__.setdefault('_seg_bounds', {})
        ck = (int(lo), int(hi), str(device), keep)
        if ck not in cache:
            from .ops import _h2d
            a = [min(max(self.offsets[k], lo), hi) for k in self.keys]
            b = [min(max(self.offsets[k] + self.numels[k], lo), hi)
                 if keep is None or keep(self.numels[k]) else
                 min(max(self.offsets[k], lo), hi) for k in self.keys]
            cache[ck] = (_h2d(a, torch.int64, device),
                         _h2d(b, torch.int64, device))
        return cache[ck]

    def segments(self, keys=None):
        """Element offsets [0, ..., numel] splitting the bucket per key
        (padding folded into the preceding key; zeros add nothing to sums of
        squares)."""
        ks = self.keys if keys is None else keys
        offs = [self.offsets[k] for k in ks] + [self.numel]
        offs[0] = 0
        return offs

    def pack_host(self, model, out):
        """Copy the fp32 keys of ``model`` into the flat CPU tensor ``out``
        (padding and missing keys zero)."""
        ends = [self.offsets[k] for k in self.keys[1:]] + [self.numel]
        for k, end in zip(self.keys, ends):
            o, m = self.offsets[k], self.numels[k]
            if k not in model:
                out[o:end].zero_()
                continue
            out[o:o + m].copy_(param2tensor(model[k]).reshape(-1))
            if end > o + m:
                out[o + m:end].zero_()
        return out

    def pack_device(self, model, out_row):
        """Pack into a device row (``out_row`` 1-D fp32 cuda tensor)."""
        devs = {param_meta(model[k]).device.type for k in self.keys
                if k in model}
        if devs <= {'cuda'}:
            # device-resident update: per-key device copies (padding and
            # absent keys keep whatever the row holds; stacks start zeroed)
            for k in self.keys:
                if k not in model:
                    continue
                t = param2tensor(model[k])
                o, m = self.offsets[k], self.numels[k]
                out_row[o:o + m].copy_(t.reshape(-1), non_blocking=True)
            return out_row
        st = HostStager(out_row.device, nbuf=1)
        st.put(self, model, out_row)
        st.finish()      # the consumer stream waits for the copy
        return out_row

    def unpack(self, flat, keys=None):
        """Views of the flat bucket, one per fp32 key, in the given order
        (one as_strided per key: a third of slice + view's host time, which
        the drop-in's result emission pays per key every call)."""
        if flat.dim() != 1 or not flat.is_contiguous() or \
                flat.numel() < self.numel:
            raise ValueError('unpack needs a flat contiguous bucket of %d '
                             'elements' % self.numel)
        spec = self.__dict__.get('_view_spec')
        if spec is None:
            spec = {}
            for k in self.keys:
                shp = tuple(self.shapes[k])
                st, acc = [], 1
                for d in reversed(shp):
                    st.append(acc)
                    acc *= d
                spec[k] = (shp, tuple(reversed(st)), self.offsets[k])
            self.__dict__['_view_spec'] = spec
        ks = self.keys if keys is None else keys
        if len(ks) > 8:
            # many keys: every view in one native call
            packed = self.__dict__.get('_view_pack')
            if packed is None or packed[0] is not ks and packed[0] != ks:
                import numpy as np
                rec = []
                for k in ks:
                    shp, st, off = spec[k]
                    rec += [len(shp)] + list(shp) + list(st) + [off]
                packed = (list(ks), np.asarray(rec, np.int64).tobytes())
                self.__dict__['_view_pack'] = packed
            host = _views_ext()
            if host is not None:
                return OrderedDict(zip(ks, host.views(flat, packed[1])))
        view = flat.as_strided
        base = flat.storage_offset()
        return OrderedDict([(k, view(spec[k][0], spec[k][1],
                                     base + spec[k][2])) for k in ks])


_VIEWS = []


def _views_ext():
    """_fsagg_host (its ``views``), or None when it was not built."""
    if not _VIEWS:
        try:
            from . import _lib
            h = _lib.host()
            _VIEWS.append(h if hasattr(h, 'views') else None)
        except Exception:  # noqa: BLE001 (no extension: per-key views)
            _VIEWS.append(None)
    return _VIEWS[0]


# Pinned staging buffers are shared by every HostStager of the process, so
# the event of the last DMA that read each slot lives next to the slot: a
# stager must not overwrite a buffer an earlier stager's copy is still
# reading (e.g. the init model packed right after the client uploads).
_PINNED = {}
_PINNED_EV = {}


def _pinned(numel, slot=0):
    ev = _PINNED_EV.pop(slot, None)
    if ev is not None:
        ev.synchronize()              # the DMA that last read this slot
    b = _PINNED.get(slot)
    if b is None or b.numel() < numel:
        b = torch.empty(numel, dtype=torch.float32, pin_memory=True)
        _PINNED[slot] = b
    return b[:numel]


# pinned staging buffers per HostStager (A/B: FSAGG_STAGE_BUFFERS)
_STAGE_BUFFERS = max(1, int(os.environ.get('FSAGG_STAGE_BUFFERS', '2')))

# c10::ScalarType codes of the dtypes the host pack takes
_SCALAR_CODE = {torch.int8: 1, torch.int16: 2, torch.float32: 6}

# A/B: FSAGG_NATIVE_PACK=0 packs through torch copies (BucketLayout.pack_host)
_NATIVE_PACK_OFF = os.environ.get('FSAGG_NATIVE_PACK', '1') == '0'


def _native_pack(layout, model, host):
    """layout.pack_host through the host extension (_fsagg_host.host_pack:
    a persistent thread pool, non-temporal stores into the pinned buffer)
    when every present key is a contiguous CPU fp32 tensor of its layout
    size; False (nothing written) otherwise.  Byte-identical to pack_host:
    keys at their offsets, absent keys and padding zero."""
    if _NATIVE_PACK_OFF or not isinstance(layout, (BucketLayout, RangeStack)):
        return False
    from .core.aggregators._engine import _host_ext
    h = _host_ext()
    if h is None or not hasattr(h, 'host_pack'):
        return False
    f32 = torch.float32
    if isinstance(layout, BucketLayout) and isinstance(model, dict) and \
            hasattr(h, 'host_pack_dict'):
        # the dict walk in C++ (one call per upload)
        spec = layout.__dict__.get('_pack_spec')
        if spec is None:
            keys = layout.keys
            ends = [layout.offsets[k] for k in keys[1:]] + [layout.numel]
            spec = ([(k, 4 * layout.offsets[k], 4 * layout.numels[k],
                      _SCALAR_CODE[f32], 1) for k in keys],
                    [(4 * (layout.offsets[k] + layout.numels[k]),
                      4 * (e - layout.offsets[k] - layout.numels[k]))
                     for k, e in zip(keys, ends)
                     if e > layout.offsets[k] + layout.numels[k]])
            layout.__dict__['_pack_spec'] = spec
        return h.host_pack_dict(model, spec[0], spec[1], host.data_ptr(),
                                torch.get_num_threads())
    items = []
    if isinstance(layout, RangeStack):
        # this rank's pieces only, as RangeStack.pack_host (absent keys are
        # left as they are: the presence matrix masks them)
        lay = layout.layout
        arrs = {}
        for sp in layout.spans:
            for k, src, dst, ln in sp:
                if k not in model:
                    continue
                a = arrs.get(k)
                if a is None:
                    v = model[k]
                    if not isinstance(v, torch.Tensor) or \
                            v.dtype is not f32 or v.device.type != 'cpu' or \
                            v.numel() != lay.numels[k] or \
                            not v.is_contiguous():
                        return False
                    a = arrs[k] = v.detach().reshape(-1).numpy()
                items.append((a[src:src + ln], 4 * ln, 4 * dst))
        h.host_pack(items, host.data_ptr(), torch.get_num_threads())
        return True
    keys = layout.keys
    ends = [layout.offsets[k] for k in keys[1:]] + [layout.numel]
    for k, end in zip(keys, ends):
        o, m = layout.offsets[k], layout.numels[k]
        v = model.get(k)
        if v is None:
            if k in model:
                return False
            items.append((None, 4 * (end - o), 4 * o))
            continue
        if not isinstance(v, torch.Tensor) or v.dtype is not f32 or \
                v.device.type != 'cpu' or v.numel() != m or \
                not v.is_contiguous():
            return False
        if m:
            items.append((v.detach().numpy(), 4 * m, 4 * o))
        if end > o + m:
            items.append((None, 4 * (end - o - m), 4 * (o + m)))
    h.host_pack(items, host.data_ptr(), torch.get_num_threads())
    return True


class HostStager:
    """Double-buffered host→device staging of client buckets.

    Packing client i+1 into one pinned buffer (a multi-threaded host copy)
    overlaps the DMA of client i out of the other buffer; the copies run on
    a side stream and the consumer stream waits on it once at the end."""

    def __init__(self, device, nbuf=None):
        if nbuf is None:
            nbuf = _STAGE_BUFFERS
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        # the rows being overwritten may still be read by kernels queued on
        # the consumer stream (the stack is reused across rounds)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.nbuf = nbuf
        self.last = None
        self.i = 0
        self._b64 = None

    def put(self, layout, model, dst_row, tag=None):
        """Stage one upload into ``dst_row``; ``tag`` names it when its
        device-side base64 decode is rejected (:meth:`rejected`)."""
        slot = self.i % self.nbuf
        self.i += 1
        if isinstance(layout, BucketLayout) and self._put_b64(
                layout, model, dst_row, slot, tag):
            return
        host = _pinned(layout.numel, slot)
        if not _native_pack(layout, model, host):
            layout.pack_host(model, host)
        with torch.cuda.stream(self.stream):
            dst_row.copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        _PINNED_EV[slot] = ev
        self.last = ev

    def _put_b64(self, layout, model, dst_row, slot, tag=None):
        """gRPC uploads (every fp32 key base64 text, core/compression/
        b64wire): the base64 characters cross PCIe and are decoded into the
        row on the device.  False when the upload is not of that form."""
        from .core.compression.b64wire import B64Stager, is_b64
        if not any(is_b64(model.get(k)) for k in layout.keys):
            return False
        framings, host_keys = B64Stager.plan(layout, model)
        if not framings:
            return False
        if self._b64 is None:
            self._b64 = B64Stager(self.device, self.stream)
        ev = self._b64.put(layout, framings, dst_row,
                           lambda nb: _pinned(-(-nb // 4), slot).view(
                               torch.uint8),
                           host={k: model[k] for k in host_keys}, tag=tag)
        if ev is not None:
            _PINNED_EV[slot] = ev
            self.last = ev
        return True

    def finish(self):
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        if self._b64 is not None:
            self._b64.finish()

    def rejected(self):
        """[(tag, reason)] of the uploads whose device decode was rejected
        since the last check (waits for the decodes; does not raise)."""
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        return self._b64.collect() if self._b64 is not None else []


class ClientStack:
    """Device slab ``[capacity][layout.numel]`` of packed client updates."""

    def __init__(self, layout, capacity, device):
        self.layout = layout
        self.device = torch.device(device)
        self.slab = torch.empty((max(1, capacity), layout.numel),
                                dtype=torch.float32, device=self.device)

    @property
    def capacity(self):
        return self.slab.shape[0]

    def ensure(self, capacity):
        """Grow to ``capacity`` rows, keeping the rows already staged."""
        if capacity > self.capacity:
            slab = torch.zeros((capacity, self.layout.numel),
                               dtype=torch.float32, device=self.device)
            slab[:self.capacity].copy_(self.slab)
            self.slab = slab

    def load(self, i, model):
        self.layout.pack_device(model, self.slab[i])

    def load_many(self, models):
        """Stage every client: device-resident fp32 dicts in ONE gather
        launch (fsagg_gather_rows_f32), host dicts through the
        double-buffered pinned stager, anything else (other dtypes, other
        devices) by per-key device copies."""
        stager = None
        gather = []
        for i, m in enumerate(models):
            srcs = self._device_keys(m)
            if srcs is not None:
                gather.append((i, srcs))
                continue
            on_host = any(param_meta(m[k]).device.type != 'cuda'
                          for k in self.layout.keys if k in m)
            if on_host:
                if stager is None:
                    stager = HostStager(self.device)
                stager.put(self.layout, m, self.slab[i])
            else:
                self.layout.pack_device(m, self.slab[i])
        if gather:
            self._gather(gather)
        if stager is not None:
            stager.finish()

    def _device_keys(self, model):
        """Data pointers of the model's fp32 keys when every present key is a
        contiguous fp32 tensor of the layout's size on this stack's device
        (0 for absent keys); else None.  (A hot loop: one pass, one lookup
        and the fewest tensor attribute reads per key.)"""
        dev = self.device.index if self.device.index is not None else \
            torch.cuda.current_device()
        f32 = torch.float32
        Tensor = torch.Tensor
        get = model.get
        ptrs = []
        push = ptrs.append
        for k, nm in self.layout.key_numels:
            t = get(k)
            if t is None:
                if k in model:      # an explicit None value: not ours
                    return None
                push(0)
                continue
            if t.__class__ is not Tensor and not isinstance(t, Tensor):
                return None
            if t.dtype is not f32 or t.get_device() != dev or \
                    t.numel() != nm or not t.is_contiguous():
                return None
            push(t.data_ptr() if nm else 0)
        return ptrs

    def _gather(self, gather):
        from . import _lib as L
        from .ops import _h2d, _stream
        lay = self.layout
        if not lay.keys:
            return
        tabs = lay.chunk_tables(self.device)
        base = self.slab.data_ptr()
        ld = self.slab.stride(0) * 4
        for b in range(0, len(gather), 65535):   # grid.y limit
            part = gather[b:b + 65535]
            src = _h2d([p for _, ptrs in part for p in ptrs], torch.int64,
                       self.device)
            dst = _h2d([base + i * ld for i, _ in part], torch.int64,
                       self.device)
            L.check(L.load().fsagg_gather_rows_f32(
                src.data_ptr(), len(part), len(lay.keys), dst.data_ptr(),
                tabs[0].data_ptr(), tabs[1].data_ptr(), tabs[2].data_ptr(),
                tabs[3].data_ptr(), tabs[2].numel(), _stream(self.device)),
                'fsagg_gather_rows_f32')

    def rows(self, idx=None, key=None):
        from .ops import RowTable
        if key is None:
            return RowTable.from_slab(self.slab, rows=idx,
                                      numel=self.layout.numel)
        return RowTable.from_slab(self.slab, rows=idx,
                                  col_offset=self.layout.offsets[key],
                                  numel=self.layout.numels[key])


class RangeStack:
    """Device slab ``[capacity][local]`` holding, per client, this rank's
    pieces of the bucket (global coordinate ranges ``pieces``), back to
    back at ``loc[j]`` — the parameter-range shard of the client stack
    (SURVEY §8(e)).  Duck-types the layout interface HostStager packs
    through (``numel``, ``pack_host``)."""

    ALIGN = 64

    def __init__(self, layout, pieces, capacity, device):
        self.layout = layout
        self.pieces = [(int(a), int(b)) for a, b in pieces]
        self.loc = []
        off = 0
        for a, b in self.pieces:
            self.loc.append(off)
            off += -(-max(b - a, 0) // self.ALIGN) * self.ALIGN
        self.numel = max(off, self.ALIGN)
        self.device = torch.device(device)
        self.slab = torch.zeros((max(1, capacity), self.numel),
                                dtype=torch.float32, device=self.device)
        # per piece: [(key, key elem start, local start, length)]
        self.spans = []
        for (a, b), loc in zip(self.pieces, self.loc):
            sp = []
            for k in layout.keys:
                o, m = layout.offsets[k], layout.numels[k]
                x, y = max(a, o), min(b, o + m)
                if y > x:
                    sp.append((k, x - o, loc + x - a, y - x))
            self.spans.append(sp)

    @property
    def capacity(self):
        return self.slab.shape[0]

    def offset(self, j):
        """Row element of bucket coordinate 0 for piece j (RowSet offset)."""
        return self.loc[j] - self.pieces[j][0]

    def pack_host(self, model, out):
        for sp in self.spans:
            for k, src, dst, ln in sp:
                if k in model:
                    out[dst:dst + ln].copy_(
                        param2tensor(model[k]).reshape(-1)[src:src + ln])
        return out

    def load_many(self, models):
        """Stage each client's pieces: host dicts through the pinned
        double-buffered stager (only this rank's share crosses PCIe),
        device tensors by slice copies."""
        stager = None
        for i, m in enumerate(models):
            on_host = any(param_meta(m[k]).device.type != 'cuda'
                          for k in self.layout.keys if k in m)
            if on_host:
                if stager is None:
                    stager = HostStager(self.device)
                stager.put(self, m, self.slab[i])
            else:
                row = self.slab[i]
                for sp in self.spans:
                    for k, src, dst, ln in sp:
                        if k in m:
                            row[dst:dst + ln].copy_(
                                param2tensor(m[k]).reshape(-1)[src:src + ln],
                                non_blocking=True)
        if stager is not None:
            stager.finish()
