"""Quantised uploads decoded straight into the device client stack.

The reference server dequantises every upload on the host
(Server.callback_funcs_model_para → symmetric_uniform_dequantization,
server.py:946-960; compression/utils.py:64-90) and aggregates fp32 dicts.
Here an upload's wire form — int8/int16 codes of the ``*.weight_quant`` keys,
their fp32 ``*.weight_scale`` scalars, and the unquantised fp32 keys — is
packed into one pinned byte buffer, copied to the GPU in ONE DMA (about
1 B per quantised parameter instead of 4), and expanded by one
fsagg_wire_unpack_f32 launch into the client's fp32 row of the stack:
``fl32(float(q) * scale)``, exactly the reference's ``value * alpha``.

Packed buffer: [scales: nscale × f32][f32 keys][int16 codes][int8 codes],
each region 16-byte aligned.
"""
from collections import OrderedDict

import torch

from ... import _lib as L
from ... import ops
from ...layout import BucketLayout
from .utils import scale_to_f32

_QUANT_KINDS = {torch.int8: L.FSAGG_WIRE_I8, torch.int16: L.FSAGG_WIRE_I16}


def _align(x, a=16):
    return -(-x // a) * a


class QuantPlan:
    """Static decode plan of one quantised model layout.

    ``template`` is a wire dict (the output of
    symmetric_uniform_quantization); the dequantised layout keeps the
    wire order with ``x.weight_quant`` renamed ``x.weight`` and the
    ``x.weight_scale`` entries dropped (utils.py:80-89)."""

    def __init__(self, template):
        deq = OrderedDict()
        self.quant = OrderedDict()   # dequantised key -> (wire key, dtype)
        self.plain = []              # fp32 keys sent as is
        for key, value in template.items():
            if 'weight_quant' in key:
                t = value if isinstance(value, torch.Tensor) else \
                    torch.as_tensor(value)
                if t.dtype not in _QUANT_KINDS:
                    raise TypeError('%s: codes must be int8/int16, got %s' %
                                    (key, t.dtype))
                k = key.replace('weight_quant', 'weight')
                deq[k] = torch.empty(t.shape, dtype=torch.float32)
                self.quant[k] = (key, t.dtype)
            elif 'weight_scale' in key:
                continue
            else:
                t = value if isinstance(value, torch.Tensor) else \
                    torch.as_tensor(value)
                if t.dtype != torch.float32:
                    raise NotImplementedError(
                        'wire staging of non-fp32 key %r (%s)' % (key,
                                                                  t.dtype))
                deq[key] = torch.empty(t.shape, dtype=torch.float32)
                self.plain.append(key)
        self.layout = BucketLayout(deq)
        lay = self.layout
        self.scale_keys = [self.quant[k][0].replace('weight_quant',
                                                     'weight_scale')
                           for k in lay.keys if k in self.quant]
        nscale = len(self.scale_keys)
        off = _align(4 * max(nscale, 1))
        recs = []
        self.regions = []            # (key, wire key, byte offset, dtype)
        for want in (torch.float32, torch.int16, torch.int8):
            width = torch.empty((), dtype=want).element_size()
            for k in lay.keys:
                if k in self.quant:
                    wk, dt = self.quant[k]
                    if dt == want:
                        recs.append((off, lay.offsets[k], lay.numels[k],
                                     _QUANT_KINDS[dt],
                                     self.scale_keys.index(
                                         wk.replace('weight_quant',
                                                    'weight_scale'))))
                        self.regions.append((k, wk, off, dt))
                        off += lay.numels[k] * width
                elif want == torch.float32:
                    recs.append((off, lay.offsets[k], lay.numels[k],
                                 L.FSAGG_WIRE_F32, -1))
                    self.regions.append((k, k, off, torch.float32))
                    off += lay.numels[k] * 4
            off = _align(off)
        self.records = recs
        # regions of one dtype are back to back: one torch.cat per dtype
        self.spans = []              # (dtype, byte start, byte end, wire keys)
        for want in (torch.float32, torch.int16, torch.int8):
            rs = [r for r in self.regions if r[3] == want]
            if rs:
                w = torch.empty((), dtype=want).element_size()
                end = rs[-1][2] + self.layout.numels[rs[-1][0]] * w
                self.spans.append((want, rs[0][2], end, [r[1] for r in rs]))
        self.nbytes = max(off, 16)
        self.nscale = nscale
        self.max_len = max([r[2] for r in recs] + [0])
        self.wire_keys = list(template.keys())
        self._segs = {}

    def segs(self, device):
        d = str(device)
        if d not in self._segs:
            self._segs[d] = ops.wire_segments(self.records, device)
        return self._segs[d]

    def check(self, wire):
        """The upload must carry exactly the plan's wire keys and dtypes."""
        for k, (wk, dt) in self.quant.items():
            v = wire.get(wk)
            if not isinstance(v, torch.Tensor) or v.dtype != dt or \
                    v.numel() != self.layout.numels[k]:
                raise ValueError('upload key %r does not match the wire '
                                 'layout (%s, %d elements)' %
                                 (wk, dt, self.layout.numels[k]))
        for k in self.plain:
            v = wire.get(k)
            if not isinstance(v, torch.Tensor) or \
                    v.dtype != torch.float32 or \
                    v.numel() != self.layout.numels[k]:
                raise ValueError('upload key %r does not match the wire '
                                 'layout' % k)
        for sk in self.scale_keys:
            if sk not in wire:
                raise KeyError(sk)

    def pack_host_checked(self, wire, buf):
        """check + pack_host in one native pass when the upload is the
        common form (a dict of contiguous CPU tensors, 1-element fp32
        scales): host_pack_dict checks every region's tensor (dtype, byte
        size) as it packs, which implies :meth:`check`.  False (the caller
        then checks and packs the general way) otherwise."""
        if not isinstance(wire, dict):
            return False
        sv = [wire.get(sk) for sk in self.scale_keys]
        if not all(isinstance(v, torch.Tensor) and v.numel() == 1 and
                   v.dtype == torch.float32 and v.device.type == 'cpu'
                   for v in sv):
            return False
        if sv:
            scales = buf[:4 * self.nscale].view(torch.float32)
            torch.cat([v.reshape(1) for v in sv], out=scales)
        return self._pack_native(wire, buf)

    def pack_host(self, wire, buf):
        """Pack one upload into the pinned uint8 buffer ``buf``."""
        scales = buf[:4 * max(self.nscale, 1)].view(torch.float32)
        sv = [wire[sk] for sk in self.scale_keys]
        if sv and all(isinstance(v, torch.Tensor) and v.numel() == 1 and
                      v.dtype == torch.float32 and v.device.type == 'cpu'
                      for v in sv):
            torch.cat([v.reshape(1) for v in sv], out=scales[:len(sv)])
        else:
            for j, v in enumerate(sv):
                scales[j] = scale_to_f32(v)
        if not self._pack_native(wire, buf):
            for dt, a, b, wkeys in self.spans:
                torch.cat([wire[wk].detach().reshape(-1).to('cpu')
                           for wk in wkeys], out=buf[a:b].view(dt))
        return buf

    def _pack_native(self, wire, buf):
        """The code and fp32 regions through _fsagg_host.host_pack (a
        persistent thread pool, non-temporal stores) when every wire tensor
        is a contiguous CPU tensor of its region's dtype; False (nothing
        written) otherwise.  Byte-identical to the torch.cat path."""
        from ...layout import _NATIVE_PACK_OFF
        if _NATIVE_PACK_OFF:
            return False
        from ..aggregators._engine import _host_ext
        h = _host_ext()
        if h is None or not hasattr(h, 'host_pack'):
            return False
        if isinstance(wire, dict) and hasattr(h, 'host_pack_dict'):
            # the dict walk in C++: every region's wire key, offset, bytes
            from ...layout import _SCALAR_CODE
            spec = self.__dict__.get('_pack_spec')
            if spec is None:
                spec = self._pack_spec = [
                    (wk, off, self.layout.numels[k] *
                     torch.empty((), dtype=dt).element_size(),
                     _SCALAR_CODE[dt], 0)
                    for k, wk, off, dt in self.regions]
            return h.host_pack_dict(wire, spec, [], buf.data_ptr(),
                                    torch.get_num_threads())
        items = []
        for dt, a, b, wkeys in self.spans:
            off = a
            for wk in wkeys:
                t = wire[wk]
                if not isinstance(t, torch.Tensor) or t.dtype != dt or \
                        t.device.type != 'cpu' or not t.is_contiguous():
                    return False
                nb = t.numel() * t.element_size()
                if nb:
                    items.append((t.detach().reshape(-1).numpy(), nb, off))
                off += nb
            if off != b:
                return False
        h.host_pack(items, buf.data_ptr(), torch.get_num_threads())
        return True


class WireStager:
    """Double-buffered pinned → device staging of quantised uploads; the
    DMA and the decode kernel run on a side stream, ordered after the
    consumer stream's earlier work (stack rows are reused across rounds)."""

    def __init__(self, plan, device, nbuf=2):
        self.plan = plan
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.nbuf = nbuf
        self.host = [torch.empty(plan.nbytes, dtype=torch.uint8,
                                 pin_memory=True) for _ in range(nbuf)]
        self.dev = [torch.empty(plan.nbytes, dtype=torch.uint8,
                                device=self.device) for _ in range(nbuf)]
        self.events = [None] * nbuf
        self.i = 0

    def put(self, wire, dst_row):
        """Stage one upload (a wire dict of host or device tensors) into the
        fp32 row ``dst_row``."""
        plan = self.plan
        b = self.i % self.nbuf
        if self.events[b] is not None:
            self.events[b].synchronize()   # the DMA that last read host[b]
        if not plan.pack_host_checked(wire, self.host[b]):
            plan.check(wire)
            plan.pack_host(wire, self.host[b])
        self.i += 1
        with torch.cuda.stream(self.stream):
            self.dev[b].copy_(self.host[b], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            scales = self.dev[b][:4 * max(plan.nscale, 1)].view(torch.float32)
            ops.wire_unpack(self.dev[b], plan.segs(self.device),
                            len(plan.records), plan.max_len, scales, dst_row,
                            src_bytes=plan.nbytes,
                            max_dst=plan.layout.numel)
        self.events[b] = ev

    def finish(self):
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
