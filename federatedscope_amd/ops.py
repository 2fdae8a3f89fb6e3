"""Tensor-level wrappers around libfsagg's C ABI.

Every function validates shapes, dtypes, devices and alignment on the host
BEFORE anything is launched (a malformed launch on a GPU box can fault the
whole node), then calls the HIP kernel on the current torch stream of the
tensors' device.  PyTorch is only the device-memory / stream container here.
"""
import ctypes
import math

import torch

from . import _lib as L

ALIGN_BYTES = 16


class _PinnedRing:
    """Reusable pinned staging for the small host tables every call uploads
    (row pointers, weights, chunk lists): NSLOT slots of SLOT bytes, used
    round robin, each backed by a slot of a device ring.  An upload is ONE
    native call (fsagg_upload_h2d): the bytes go into the pinned slot, a
    side stream copies them into the device slot and the caller's stream
    waits for that copy — the copy never sits behind the previous call's
    kernel on the caller's stream, and the host spends a few microseconds
    where the torch-level sequence (stream switch, allocation, copy, event)
    cost ~33 (profiles/r06/upload_cost.json).  A device slot is rewritten
    only after the consumer work enqueued within NSLOT/2 uploads of its
    previous use (the library's per-slot events).  Slots of 1 MiB hold the
    key table of up to ~800 clients of the ResNet-50 layout."""
    SLOT = 1 << 20
    NSLOT = 64
    # Content-addressed cache of the uploaded tables (the kernels only read
    # them): a table whose bytes were uploaded before is handed out again
    # without a copy.  Row tables hold the clients' tensor addresses, which
    # stay the same from call to call whenever the clients' tensors do (the
    # standalone simulator's persistent client models, a server's stack
    # slots, and every repeated aggregate() over the same dicts); weights,
    # chunk lists and selections repeat likewise.  A table enters the cache
    # on its SECOND sighting (a persistent device tensor of its own); the
    # first goes through the ring, so tables that never repeat (fresh
    # upload tensors every round) cost one native copy and nothing else.
    # Entries are immutable device tensors; each is marked used
    # (record_stream) by every stream it is handed to, so the caching
    # allocator recycles an evicted entry's block only after the work that
    # read it, and a stream an entry was not uploaded for first waits for
    # the entry's copy (fsagg_upload_wait on its slot: every copy runs in
    # order on one side stream, so the slot's latest copy completes after
    # the entry's).  The cache is bounded by bytes (host keys plus device
    # tables), not only by entries.
    CACHE_MAX_BYTES = 1 << 20      # = SLOT: the ResNet-50 key table fits
    CACHE_ENTRIES = 512
    CACHE_TOTAL_BYTES = 32 << 20
    SEEN_ENTRIES = 1024

    def __init__(self):
        from collections import OrderedDict
        self.buf = None
        self.i = 0
        self.streams = {}
        self.rings = {}
        self.cache = OrderedDict()
        self.seen = OrderedDict()
        self.cache_bytes = 0
        self.cache_on = True
        self.hits = 0
        self.misses = 0
        self.uploads = 0

    def _cached(self, key, device):
        hit = self.cache.get(key)
        if hit is None:
            return None
        self.cache.move_to_end(key)
        t, seen, slot = hit
        s = torch._C._cuda_getCurrentRawStream(device.index)
        if s not in seen:
            L.check(L.load().fsagg_upload_wait(slot, ctypes_ptr(s)),
                    'fsagg_upload_wait')
            t.record_stream(torch.cuda.current_stream(device))
            seen.add(s)
        self.hits += 1
        return t

    def _insert(self, key, t, slot, device):
        self.cache[key] = (t, {torch._C._cuda_getCurrentRawStream(
            device.index)}, slot)
        self.cache_bytes += 2 * len(key[3])
        while len(self.cache) > self.CACHE_ENTRIES or \
                self.cache_bytes > self.CACHE_TOTAL_BYTES:
            old, _ = self.cache.popitem(last=False)
            self.cache_bytes -= 2 * len(old[3])

    def clear(self):
        self.cache.clear()
        self.seen.clear()
        self.cache_bytes = 0

    def _copy_stream(self, device):
        s = self.streams.get(device.index)
        if s is None:
            s = self.streams[device.index] = torch.cuda.Stream(device=device)
        return s

    def upload(self, arr, device, ephemeral=False):
        """numpy array -> device tensor of its dtype and shape (async, see
        the class docstring).  ``ephemeral``: the caller launches the
        kernels that read it before NSLOT/2 further uploads and keeps no
        reference beyond that (per-call tables) — it may then come from the
        device ring (a view that later uploads overwrite) unless it is
        cached; otherwise it is a device tensor of its own."""
        import numpy as np
        if device.index is None:
            device = torch.device('cuda', torch.cuda.current_device())
        arr = np.ascontiguousarray(arr)
        raw = arr.reshape(-1).view(np.uint8)
        nb = raw.size
        key = None
        if self.cache_on and 0 < nb <= self.CACHE_MAX_BYTES:
            key = (device.index, arr.dtype.str, arr.shape, raw.tobytes())
            t = self._cached(key, device)
            if t is not None:
                return t
            self.misses += 1
            if ephemeral:
                if key in self.seen:
                    del self.seen[key]
                else:
                    self.seen[key] = None
                    while len(self.seen) > self.SEEN_ENTRIES:
                        self.seen.popitem(last=False)
                    key = None       # first sighting: the ring
        self.uploads += 1
        if nb == 0 or nb > self.SLOT or \
                device.index != torch.cuda.current_device():
            host = torch.from_numpy(raw.copy())
            return host.pin_memory().to(device, non_blocking=True).view(
                _TORCH_OF[arr.dtype.str]).reshape(arr.shape)
        if self.buf is None:
            self.buf = torch.empty(self.SLOT * self.NSLOT, dtype=torch.uint8,
                                   pin_memory=True)
            self.buf_ptr = self.buf.data_ptr()
        k = self.i
        self.i = (k + 1) % self.NSLOT
        lo = k * self.SLOT
        side = self._copy_stream(device)
        if key is None and ephemeral:
            ring = self.rings.get(device.index)
            if ring is None:
                ring = self.rings[device.index] = torch.empty(
                    self.SLOT * self.NSLOT, dtype=torch.uint8, device=device)
            dst = ring[lo:lo + nb]
        else:
            # a persistent entry: allocated from the copy stream's pool and
            # marked used by the caller's stream
            with torch.cuda.stream(side):
                dst = torch.empty(nb, dtype=torch.uint8, device=device)
            dst.record_stream(torch.cuda.current_stream(device))
        L.check(L.load().fsagg_upload_h2d(
            dst.data_ptr(), raw.ctypes.data, nb, self.buf_ptr + lo, k,
            self.NSLOT, ctypes_ptr(side.cuda_stream),
            ctypes_ptr(torch._C._cuda_getCurrentRawStream(device.index))),
            'fsagg_upload_h2d')
        t = dst.view(_TORCH_OF[arr.dtype.str]).reshape(arr.shape)
        if key is not None:
            self._insert(key, t, k, device)
        return t


_TORCH_OF = {'<i8': torch.int64, '<i4': torch.int32, '<i2': torch.int16,
             '|i1': torch.int8, '<f4': torch.float32, '<f8': torch.float64,
             '<f2': torch.float16, '|u1': torch.uint8, '|b1': torch.bool}
_NP_OF = {}
_RING = _PinnedRing()


def _h2d(values, dtype, device, ephemeral=False):
    """A small host table (row pointers, weights, offsets) on ``device``:
    staged through pinned memory and copied asynchronously, so a call never
    blocks the host on the GPU's queue (``ephemeral``: _PinnedRing.upload)."""
    import numpy as np
    device = torch.device(device)
    if device.type != 'cuda':
        return torch.tensor(values, dtype=dtype).to(device)
    npt = _NP_OF.get(dtype)
    if npt is None:
        npt = _NP_OF[dtype] = torch.empty(0, dtype=dtype).numpy().dtype
    return _RING.upload(np.asarray(values, dtype=npt), device,
                        ephemeral=ephemeral)


def _h2d_bytes(arr, device):
    """A numpy record array as a uint8 device tensor (pinned, async)."""
    import numpy as np
    return _RING.upload(np.ascontiguousarray(arr).view(np.uint8).reshape(-1),
                        torch.device(device))


def _h2d_np(arr, device, ephemeral=False):
    """A numpy array as a flat device tensor of its dtype (pinned, async)."""
    import numpy as np
    return _RING.upload(np.ascontiguousarray(arr).reshape(-1),
                        torch.device(device), ephemeral=ephemeral)


def _stream(device):
    """The raw current stream of ``device`` (an int, 0 = the null stream),
    without building a torch Stream object (~2 us each)."""
    idx = device.index if device.index is not None else \
        torch.cuda.current_device()
    return ctypes_ptr(torch._C._cuda_getCurrentRawStream(idx))


def ctypes_ptr(x):
    return int(x) if x else None


def _check_f32_cuda(t, what, align=ALIGN_BYTES):
    if not isinstance(t, torch.Tensor):
        raise TypeError('%s must be a torch.Tensor' % what)
    if t.device.type != 'cuda':
        raise ValueError('%s must live on a GPU (got %s)' % (what, t.device))
    if t.dtype != torch.float32:
        raise ValueError('%s must be float32 (got %s)' % (what, t.dtype))
    if not t.is_contiguous():
        raise ValueError('%s must be contiguous' % what)
    if t.data_ptr() % align:
        raise ValueError('%s must be %d-byte aligned' % (what, align))


class RowTable:
    """A device array of client row pointers (see include/fsagg.h).

    Row i is a flat fp32 bucket of ``numel`` elements that starts at
    ``ptrs[i]``; table order is the reduction order.  The table keeps the
    tensors it points into alive.
    """

    def __init__(self, ptrs, numel, device, keepalive=()):
        if len(ptrs) < 1:
            raise ValueError('RowTable needs at least one row')
        for p in ptrs:
            if p % 4:
                raise ValueError('client row pointer 0x%x is not 4-byte '
                                 'aligned' % p)
        # the streaming weighted sum reads 16 B per lane; the order-statistic
        # and distance kernels read 4 B per lane and take any fp32 row
        self.aligned16 = all(p % ALIGN_BYTES == 0 for p in ptrs)
        self.ptrs = list(ptrs)
        self.n = len(ptrs)
        self.numel = int(numel)
        self.device = torch.device(device)
        self.table = _h2d(self.ptrs, torch.int64, self.device)
        self._keep = tuple(keepalive)

    @classmethod
    def from_slab(cls, slab, rows=None, col_offset=0, numel=None):
        """Rows of a 2-D [n][ld] fp32 slab; ``rows`` selects/reorders."""
        _check_f32_cuda(slab, 'slab', align=4)
        if slab.dim() != 2:
            raise ValueError('slab must be 2-D [clients, ld]')
        n, ld = slab.shape
        numel = ld - col_offset if numel is None else int(numel)
        if col_offset < 0 or col_offset + numel > ld:
            raise ValueError('column range [%d, %d) outside ld=%d' %
                             (col_offset, col_offset + numel, ld))
        idx = range(n) if rows is None else [int(r) for r in rows]
        for r in idx:
            if not 0 <= r < n:
                raise IndexError('row %d outside slab of %d rows' % (r, n))
        base = slab.data_ptr()
        rowb = slab.stride(0) * 4
        ptrs = [base + r * rowb + col_offset * 4 for r in idx]
        return cls(ptrs, numel, slab.device, keepalive=(slab, ))

    @classmethod
    def from_tensors(cls, tensors, numel=None, offset=0):
        """One flat fp32 device tensor per client."""
        if not tensors:
            raise ValueError('no client tensors')
        dev = tensors[0].device
        m = min(t.numel() for t in tensors)
        numel = m - offset if numel is None else int(numel)
        ptrs = []
        for i, t in enumerate(tensors):
            _check_f32_cuda(t, 'client tensor %d' % i, align=4)
            if t.device != dev:
                raise ValueError('client tensors on different devices')
            if offset + numel > t.numel():
                raise ValueError('client tensor %d shorter than numel' % i)
            ptrs.append(t.data_ptr() + 4 * offset)
        return cls(ptrs, numel, dev, keepalive=tuple(tensors))

    def ptr(self):
        return self.table.data_ptr()


def _fp32_dev(values, device):
    """Per-call weights / prescales (read by the launch that follows)."""
    return _h2d([float(v) for v in values], torch.float32, device,
                ephemeral=True)


def _check_out(out, numel, device, what='out', align=ALIGN_BYTES):
    _check_f32_cuda(out, what, align=align)
    if out.device != device:
        raise ValueError('%s on %s, rows on %s' % (what, out.device, device))
    if out.numel() < numel:
        raise ValueError('%s has %d elements < numel %d' %
                         (what, out.numel(), numel))


def weighted_sum(rows, weights, out, prescale=None, base=None, stream=None):
    """out = [base +] Σ_i fl32(fl32(x_i·s_i)·w_i) in row order (no FMA).

    ``weights``/``prescale`` are Python floats (the reference's doubles); they
    are rounded to fp32 here exactly as ATen reads a wrapped scalar."""
    if len(weights) != rows.n:
        raise ValueError('%d weights for %d rows' % (len(weights), rows.n))
    if not rows.aligned16:
        raise ValueError('weighted_sum needs 16-byte aligned client rows '
                         '(pack them with BucketLayout / ClientStack)')
    _check_out(out, rows.numel, rows.device)
    if base is not None:
        _check_out(base, rows.numel, rows.device, 'base')
    w = weights if isinstance(weights, torch.Tensor) else _fp32_dev(
        weights, rows.device)
    s = None
    if prescale is not None:
        if len(prescale) != rows.n:
            raise ValueError('prescale length mismatch')
        s = prescale if isinstance(prescale, torch.Tensor) else _fp32_dev(
            prescale, rows.device)
    st = stream if stream is not None else _stream(rows.device)
    L.check(L.load().fsagg_weighted_sum_f32(
        rows.ptr(), w.data_ptr(), s.data_ptr() if s is not None else None,
        rows.n, rows.numel, base.data_ptr() if base is not None else None,
        out.data_ptr(), st), 'fsagg_weighted_sum_f32')
    return out


def weighted_sum_bcast(rows, weights, outs, prescale=None, base=None,
                       stream=None):
    """weighted_sum whose result is written to every device address in
    ``outs`` (this GPU's buffer and peers' imported buffers, each holding
    ``rows.numel`` fp32, 16-byte aligned): the assembly epilogue of the
    strong-scaled path (core/sharding.PeerAssembly)."""
    if len(weights) != rows.n:
        raise ValueError('%d weights for %d rows' % (len(weights), rows.n))
    if not rows.aligned16:
        raise ValueError('weighted_sum_bcast needs 16-byte aligned rows')
    if not 1 <= len(outs) <= L.FSAGG_MAX_PEERS:
        raise ValueError('1..%d outputs, got %d' % (L.FSAGG_MAX_PEERS,
                                                    len(outs)))
    for p in outs:
        if not p or int(p) % ALIGN_BYTES:
            raise ValueError('output address 0x%x not 16-byte aligned' %
                             int(p or 0))
    if base is not None:
        _check_out(base, rows.numel, rows.device, 'base')
    w = weights if isinstance(weights, torch.Tensor) else _fp32_dev(
        weights, rows.device)
    s = None
    if prescale is not None:
        if len(prescale) != rows.n:
            raise ValueError('prescale length mismatch')
        s = prescale if isinstance(prescale, torch.Tensor) else _fp32_dev(
            prescale, rows.device)
    arr = (ctypes.c_void_p * len(outs))(*[int(p) for p in outs])
    st = stream if stream is not None else _stream(rows.device)
    L.check(L.load().fsagg_weighted_sum_bcast_f32(
        rows.ptr(), w.data_ptr(), s.data_ptr() if s is not None else None,
        rows.n, rows.numel, base.data_ptr() if base is not None else None,
        arr, len(outs), st), 'fsagg_weighted_sum_bcast_f32')


def peer_push(src, dsts, n, device, stream=None):
    """Store ``n`` fp32 from device address ``src`` into each device address
    of ``dsts`` (peer copies of the output; fsagg_peer_push_f32)."""
    if not 0 <= len(dsts) <= L.FSAGG_MAX_PEERS:
        raise ValueError('0..%d destinations, got %d' % (L.FSAGG_MAX_PEERS,
                                                         len(dsts)))
    arr = (ctypes.c_void_p * max(len(dsts), 1))(*[int(p) for p in dsts])
    st = stream if stream is not None else _stream(device)
    L.check(L.load().fsagg_peer_push_f32(int(src), arr, len(dsts), int(n),
                                         st), 'fsagg_peer_push_f32')


_TYPED = {
    torch.float16: (L.FSAGG_F16, torch.float16),
    torch.bfloat16: (L.FSAGG_BF16, torch.bfloat16),
    torch.float64: (L.FSAGG_F64, torch.float64),
    torch.int64: (L.FSAGG_I64, torch.float32),
}


def typed_out_dtype(dtype):
    return _TYPED[dtype][1]


def weighted_sum_typed(tensors, weights, out):
    """Non-fp32 keys (A5 dtype rules): tensors are per-client contiguous device
    tensors of one dtype; weights are Python floats (kept as doubles)."""
    dt = tensors[0].dtype
    if dt not in _TYPED:
        raise ValueError('unsupported dtype %s' % dt)
    code, odt = _TYPED[dt]
    numel = tensors[0].numel()
    dev = tensors[0].device
    for t in tensors:
        if t.dtype != dt or t.numel() != numel or t.device != dev or \
                not t.is_contiguous() or dev.type != 'cuda':
            raise ValueError('typed rows must be contiguous %s tensors of %d '
                             'elements on one GPU' % (dt, numel))
    if out.dtype != odt or out.numel() != numel or out.device != dev or \
            not out.is_contiguous():
        raise ValueError('out must be a contiguous %s tensor of %d elements' %
                         (odt, numel))
    if len(weights) != len(tensors):
        raise ValueError('weights length mismatch')
    tab = _h2d([t.data_ptr() for t in tensors], torch.int64, dev)
    w = _h2d([float(x) for x in weights], torch.float64, dev)
    L.check(L.load().fsagg_weighted_sum_typed(tab.data_ptr(), code,
                                              w.data_ptr(), len(tensors),
                                              numel, out.data_ptr(),
                                              _stream(dev)),
            'fsagg_weighted_sum_typed')
    return out


def online_inc(m, x, cnt, sample_size):
    """m = (cnt*m + s*x) / (cnt + s), every op rounded to fp32."""
    _check_f32_cuda(m, 'maintained')
    _check_f32_cuda(x, 'client update')
    if x.numel() < m.numel() or x.device != m.device:
        raise ValueError('client update does not cover the maintained bucket')
    L.check(L.load().fsagg_online_inc_f32(
        m.data_ptr(), x.data_ptr(), float(cnt), float(sample_size),
        float(cnt + sample_size), m.numel(), _stream(m.device)),
            'fsagg_online_inc_f32')
    return m


def add(a, b, out):
    for t, nm in ((a, 'a'), (b, 'b'), (out, 'out')):
        _check_f32_cuda(t, nm)
    if not (a.numel() == b.numel() == out.numel()):
        raise ValueError('add: size mismatch')
    L.check(L.load().fsagg_add_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                   out.numel(), _stream(out.device)),
            'fsagg_add_f32')
    return out


def coord_median(rows, out, base=None):
    _check_out(out, rows.numel, rows.device, align=4)
    if base is not None:
        _check_out(base, rows.numel, rows.device, 'base', align=4)
    L.check(L.load().fsagg_coord_median_f32(
        rows.ptr(), rows.n, rows.numel,
        base.data_ptr() if base is not None else None, out.data_ptr(),
        _stream(rows.device)), 'fsagg_coord_median_f32')
    return out


def trimmed_mean(rows, k, out, divisor=None, base=None):
    if k < 0 or 2 * k >= rows.n:
        raise ValueError('trimmed mean needs 0 <= 2k < n (k=%d n=%d)' %
                         (k, rows.n))
    _check_out(out, rows.numel, rows.device, align=4)
    if base is not None:
        _check_out(base, rows.numel, rows.device, 'base', align=4)
    div = float(rows.n - 2 * k if divisor is None else divisor)
    L.check(L.load().fsagg_trimmed_mean_f32(
        rows.ptr(), rows.n, rows.numel, int(k), div,
        base.data_ptr() if base is not None else None, out.data_ptr(),
        _stream(rows.device)), 'fsagg_trimmed_mean_f32')
    return out


class Workspace:
    """Grow-only device scratch owned by the caller (the library allocates
    nothing)."""

    def __init__(self):
        self.buf = {}

    def get(self, device, nbytes):
        key = str(device)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8,
                            device=device)
            self.buf[key] = b
        return b


_WS = Workspace()


def pairdist(rows, seg_offsets, workspace=None):
    """Krum distance matrix D[n][n] (fp32, device): sum over key segments of
    per-key L2 distances; D[a][a] = +inf."""
    if rows.n < 2:
        raise ValueError('Krum needs at least two clients')
    offs = [int(o) for o in seg_offsets]
    if offs[0] != 0 or offs[-1] != rows.numel or \
            any(b < a for a, b in zip(offs, offs[1:])):
        raise ValueError('segment offsets must rise from 0 to numel')
    nseg = len(offs) - 1
    lib = L.load()
    need = lib.fsagg_pairdist_workspace_bytes(rows.n, rows.numel, nseg)
    ws = (workspace or _WS).get(rows.device, need)
    seg = _h2d(offs, torch.int64, rows.device)
    D = torch.empty((rows.n, rows.n), dtype=torch.float32, device=rows.device)
    L.check(lib.fsagg_pairdist_f32(rows.ptr(), rows.n, rows.numel,
                                   seg.data_ptr(), nseg, D.data_ptr(),
                                   ws.data_ptr(), ws.numel(),
                                   _stream(rows.device)), 'fsagg_pairdist_f32')
    return D


def pairdist_segsq(rows, seg_offsets, workspace=None):
    """Per-key squared pair distances [nseg][n][n] (fp64, device) — the
    shard-local half of Krum's distance matrix (summed across ranks by the
    caller, then :func:`pairdist_finish`)."""
    if rows.n < 2:
        raise ValueError('Krum needs at least two clients')
    offs = [int(o) for o in seg_offsets]
    if offs[0] != 0 or offs[-1] != rows.numel or \
            any(b < a for a, b in zip(offs, offs[1:])):
        raise ValueError('segment offsets must rise from 0 to numel')
    nseg = len(offs) - 1
    lib = L.load()
    need = lib.fsagg_pairdist_workspace_bytes(rows.n, rows.numel, nseg)
    ws = (workspace or _WS).get(rows.device, need)
    seg = _h2d(offs, torch.int64, rows.device)
    sq = torch.empty((nseg, rows.n, rows.n), dtype=torch.float64,
                     device=rows.device)
    L.check(lib.fsagg_pairdist_segsq_f32(rows.ptr(), rows.n, rows.numel,
                                         seg.data_ptr(), nseg, sq.data_ptr(),
                                         ws.data_ptr(), ws.numel(),
                                         _stream(rows.device)),
            'fsagg_pairdist_segsq_f32')
    return sq


def pairdist_finish(segsq):
    """D[a][b] = Σ_seg fl32(sqrt(segsq[seg][a][b])), D[a][a] = +inf."""
    if segsq.dtype != torch.float64 or segsq.dim() != 3 or \
            segsq.shape[1] != segsq.shape[2] or segsq.device.type != 'cuda' \
            or not segsq.is_contiguous():
        raise ValueError('segsq must be a contiguous [nseg][n][n] float64 '
                         'GPU tensor')
    nseg, n, _ = segsq.shape
    D = torch.empty((n, n), dtype=torch.float32, device=segsq.device)
    L.check(L.load().fsagg_pairdist_finish_f64(segsq.data_ptr(), n, nseg,
                                               D.data_ptr(),
                                               _stream(segsq.device)),
            'fsagg_pairdist_finish_f64')
    return D


def row_sqnorm(rows, workspace=None):
    """Per-row Σx² in float64 (device tensor [n])."""
    lib = L.load()
    need = lib.fsagg_rownorm_workspace_bytes(rows.n, rows.numel)
    ws = (workspace or _WS).get(rows.device, need)
    sq = torch.empty(rows.n, dtype=torch.float64, device=rows.device)
    L.check(lib.fsagg_row_sqnorm_f32(rows.ptr(), rows.n, rows.numel,
                                     sq.data_ptr(), ws.data_ptr(), ws.numel(),
                                     _stream(rows.device)),
            'fsagg_row_sqnorm_f32')
    return sq


def fill_uniform(slab, numel, seed, index_offset=0):
    """Deterministic synthetic updates into a [n][ld] slab (benchmarks)."""
    _check_f32_cuda(slab, 'slab')
    n, ld = slab.shape
    if numel > ld:
        raise ValueError('numel > ld')
    L.check(L.load().fsagg_fill_uniform_f32(slab.data_ptr(), n, int(numel),
                                            ld, int(seed) & (2**64 - 1),
                                            int(index_offset),
                                            _stream(slab.device)),
            'fsagg_fill_uniform_f32')
    return slab


def round_up(x, a):
    return int(math.ceil(x / a) * a)


# -- wire formats and secret sharing ----------------
WIRE_SEG_DTYPE = [('src', '<i8'), ('dst', '<i8'), ('len', '<i8'),
                  ('kind', '<i4'), ('scale_idx', '<i4')]


def wire_segments(records, device):
    """Device table of (src_byte_off, dst_elem_off, len, kind, scale_idx)
    records (32 B each, the layout fsagg_wire_unpack_f32 reads)."""
    import numpy as np
    arr = np.zeros(len(records), dtype=WIRE_SEG_DTYPE)
    for i, (src, dst, ln, kind, sidx) in enumerate(records):
        if kind not in (L.FSAGG_WIRE_F32, L.FSAGG_WIRE_I8, L.FSAGG_WIRE_I16):
            raise ValueError('unknown wire kind %r' % kind)
        width = {L.FSAGG_WIRE_F32: 4, L.FSAGG_WIRE_I8: 1,
                 L.FSAGG_WIRE_I16: 2}[kind]
        if src % width:
            raise ValueError('segment %d source offset %d is not %d-byte '
                             'aligned' % (i, src, width))
        arr[i] = (src, dst, ln, kind, sidx)
    return torch.from_numpy(arr.view(np.uint8).copy()).to(device)


def wire_unpack(src, segs, nseg, max_len, scales, out, src_bytes=None,
                max_dst=None):
    """Decode one client's packed upload (``src``: device uint8 buffer) into
    its fp32 row ``out`` per the device segment table ``segs``.  The caller
    (which built ``segs`` with :func:`wire_segments`) states the extents it
    checked: ``src_bytes`` ≤ src.numel(), every dst + len ≤ ``max_dst``."""
    _check_f32_cuda(out, 'out', align=4)
    if src.device != out.device or segs.device != out.device or \
            scales.device != out.device:
        raise ValueError('wire buffers on different devices')
    if src.dtype != torch.uint8 or segs.dtype != torch.uint8 or \
            scales.dtype != torch.float32:
        raise ValueError('src/segs must be uint8, scales float32')
    if segs.numel() != 32 * nseg:
        raise ValueError('segment table holds %d bytes, expected %d' %
                         (segs.numel(), 32 * nseg))
    if src_bytes is not None and src_bytes > src.numel():
        raise ValueError('packed upload larger than the staging buffer')
    if max_dst is not None and max_dst > out.numel():
        raise ValueError('segments write past the end of the row')
    # the kernel re-checks every segment against these extents on the device
    L.check(L.load().fsagg_wire_unpack_f32(
        src.data_ptr(), int(src.numel() if src_bytes is None else src_bytes),
        segs.data_ptr(), scales.data_ptr(), int(scales.numel()), int(nseg),
        int(max_len), out.data_ptr(),
        int(out.numel() if max_dst is None else max_dst),
        _stream(out.device)), 'fsagg_wire_unpack_f32')
    return out


def ss_recover(shares, mod, maximum, epsilon, total, recover=True,
               weight=1.0):
    """Secret-sharing FedAvg of one key: ``shares`` are per-client device
    tensors (float64 or int64, same shape), each multiplied by ``weight``
    (float64) and summed in list order.  Returns fp32 (recovered, divided
    by ``total``) or, with ``recover=False``, the float64 sums."""
    if not shares:
        raise ValueError('no shares')
    dev = shares[0].device
    shape = shares[0].shape
    numel = shares[0].numel()
    for i, t in enumerate(shares):
        if t.device != dev or dev.type != 'cuda' or t.shape != shape or \
                not t.is_contiguous() or t.dtype not in (torch.float64,
                                                         torch.int64):
            raise ValueError('share %d must be a contiguous float64/int64 '
                             'tensor of shape %s on one GPU' % (i, shape))
    # the kernel reads two elements per lane (16-B loads)
    shares = [t if t.data_ptr() % ALIGN_BYTES == 0 else t.clone()
              for t in shares]
    tab = _h2d([t.data_ptr() for t in shares], torch.int64, dev)
    is_int = _h2d([t.dtype == torch.int64 for t in shares], torch.uint8, dev)
    out = torch.empty(shape, dtype=torch.float32 if recover else
                      torch.float64, device=dev)
    L.check(L.load().fsagg_ss_recover_f32(
        tab.data_ptr(), is_int.data_ptr(), len(shares), numel,
        float(weight), float(mod),
        float(maximum), float(epsilon), float(total), 1 if recover else 0,
        out.data_ptr() if recover else None,
        None if recover else out.data_ptr(), _stream(dev)),
        'fsagg_ss_recover_f32')
    return out


def delta_sqnorm(rows, seg_offsets, base=None, workspace=None):
    """sq[i][s] = Σ_{p in key s} fl32(x_i[p] - base[p])² in float64 (device
    tensor [n][nseg])."""
    offs = [int(o) for o in seg_offsets]
    if offs[0] != 0 or offs[-1] != rows.numel or \
            any(b < a for a, b in zip(offs, offs[1:])):
        raise ValueError('segment offsets must rise from 0 to numel')
    if base is not None:
        _check_out(base, rows.numel, rows.device, what='base', align=4)
    nseg = len(offs) - 1
    lib = L.load()
    need = lib.fsagg_delta_sqnorm_workspace_bytes(rows.n, rows.numel, nseg)
    ws = (workspace or _WS).get(rows.device, need)
    seg = _h2d(offs, torch.int64, rows.device)
    sq = torch.empty((rows.n, nseg), dtype=torch.float64, device=rows.device)
    L.check(lib.fsagg_delta_sqnorm_f32(
        rows.ptr(), rows.n, rows.numel,
        None if base is None else base.data_ptr(), seg.data_ptr(), nseg,
        sq.data_ptr(), ws.data_ptr(), ws.numel(), _stream(rows.device)),
        'fsagg_delta_sqnorm_f32')
    return sq


def delta_wsum(rows, weights, base, out):
    """out = Σ_i fl32(w_i · fl32(x_i − base)) (fp32, list order)."""
    _check_out(base, rows.numel, rows.device, what='base', align=4)
    _check_out(out, rows.numel, rows.device, align=4)
    if len(weights) != rows.n:
        raise ValueError('%d weights for %d rows' % (len(weights), rows.n))
    w = _fp32_dev(weights, rows.device)
    L.check(L.load().fsagg_delta_wsum_f32(rows.ptr(), w.data_ptr(), rows.n,
                                          rows.numel, base.data_ptr(),
                                          out.data_ptr(),
                                          _stream(rows.device)),
            'fsagg_delta_wsum_f32')
    return out


def delta_sqnorm_wsum(rows, weights, seg_offsets, base, out,
                      workspace=None):
    """:func:`delta_sqnorm` and :func:`delta_wsum` in one read of the rows
    (calc_blocal_dissim's two passes): returns sq [n][nseg] (fp64, within
    ~1e-15 relative of delta_sqnorm's order) and fills ``out``
    (bit-identical to delta_wsum)."""
    offs = [int(o) for o in seg_offsets]
    if offs[0] != 0 or offs[-1] != rows.numel or \
            any(b < a for a, b in zip(offs, offs[1:])):
        raise ValueError('segment offsets must rise from 0 to numel')
    _check_out(base, rows.numel, rows.device, what='base', align=4)
    _check_out(out, rows.numel, rows.device, align=4)
    if len(weights) != rows.n:
        raise ValueError('%d weights for %d rows' % (len(weights), rows.n))
    nseg = len(offs) - 1
    lib = L.load()
    need = lib.fsagg_delta_sqnorm_wsum_workspace_bytes(rows.n, rows.numel,
                                                       nseg)
    ws = (workspace or _WS).get(rows.device, need)
    seg = _h2d(offs, torch.int64, rows.device)
    w = _fp32_dev(weights, rows.device)
    sq = torch.empty((rows.n, nseg), dtype=torch.float64, device=rows.device)
    L.check(lib.fsagg_delta_sqnorm_wsum_f32(
        rows.ptr(), w.data_ptr(), rows.n, rows.numel, base.data_ptr(),
        seg.data_ptr(), nseg, sq.data_ptr(), out.data_ptr(), ws.data_ptr(),
        ws.numel(), _stream(rows.device)), 'fsagg_delta_sqnorm_wsum_f32')
    return sq


class KeyTable:
    """Per-client, per-key device tensors addressed in place: an n x nseg
    pointer table (entry [i][s] = client i's fp32 tensor for key s) plus the
    keys' flat offsets.  No staging copy — the form of the metric passes for
    client dicts that are already on the GPU.  Raises ValueError/TypeError
    if a tensor is not a contiguous fp32 tensor of the first client's key
    sizes on ``device`` (one lean pass: this runs once per client key)."""

    def __init__(self, clients, device):
        if not clients or not clients[0]:
            raise ValueError('KeyTable needs at least one client and key')
        device = torch.device(device)
        if device.type != 'cuda':
            raise ValueError('KeyTable needs a GPU device')
        idx = torch.cuda.current_device() if device.index is None \
            else device.index
        self.device = torch.device('cuda', idx)
        self.nseg = len(clients[0])
        self.sizes = [int(t.numel()) for t in clients[0]]
        f32 = torch.float32
        ptrs = []
        for i, row in enumerate(clients):
            if len(row) != self.nseg:
                raise ValueError('client %d has %d keys, client 0 has %d' %
                                 (i, len(row), self.nseg))
            for s, t in enumerate(row):
                if t.dtype is not f32 or not t.is_contiguous() or \
                        t.get_device() != idx or t.numel() != self.sizes[s]:
                    raise ValueError(
                        'client %d key %d must be a contiguous float32 '
                        'tensor of %d elements on %s' %
                        (i, s, self.sizes[s], self.device))
                p = t.data_ptr()
                if p % 4:
                    raise ValueError('client %d key %d is not 4-byte '
                                     'aligned' % (i, s))
                ptrs.append(p)
        self.n = len(clients)
        offs = [0]
        for sz in self.sizes:
            offs.append(offs[-1] + sz)
        self.offsets = offs
        self.numel = offs[-1]
        self.table = _h2d(ptrs, torch.int64, self.device)
        self.seg = _h2d(offs, torch.int64, self.device)
        self._keep = clients

    def base_table(self, base):
        """Device pointer table of the base model's per-key tensors."""
        if len(base) != self.nseg:
            raise ValueError('base has %d keys, clients %d' %
                             (len(base), self.nseg))
        for s, t in enumerate(base):
            _check_f32_cuda(t, 'base key %d' % s, align=4)
            if t.device != self.device or t.numel() != self.sizes[s]:
                raise ValueError('base key %d does not match the clients' % s)
        return _h2d([t.data_ptr() for t in base], torch.int64, self.device)


def delta_sqnorm_keys(keys, base=None, workspace=None):
    """:func:`delta_sqnorm` over a :class:`KeyTable` (``base``: per-key
    tensors or None); bit-identical to the staged form."""
    lib = L.load()
    need = lib.fsagg_delta_sqnorm_workspace_bytes(keys.n, keys.numel,
                                                  keys.nseg)
    ws = (workspace or _WS).get(keys.device, need)
    btab = keys.base_table(base) if base is not None else None
    sq = torch.empty((keys.n, keys.nseg), dtype=torch.float64,
                     device=keys.device)
    L.check(lib.fsagg_delta_sqnorm_keys_f32(
        keys.table.data_ptr(), keys.n, keys.numel,
        None if btab is None else btab.data_ptr(), keys.seg.data_ptr(),
        keys.nseg, sq.data_ptr(), ws.data_ptr(), ws.numel(),
        _stream(keys.device)), 'fsagg_delta_sqnorm_keys_f32')
    return sq


def delta_sqnorm_wsum_keys(keys, weights, base, out, workspace=None):
    """:func:`delta_sqnorm_wsum` over a :class:`KeyTable` (``base``: per-key
    tensors; ``out`` flat)."""
    _check_out(out, keys.numel, keys.device, align=4)
    if len(weights) != keys.n:
        raise ValueError('%d weights for %d rows' % (len(weights), keys.n))
    lib = L.load()
    need = lib.fsagg_delta_sqnorm_wsum_workspace_bytes(keys.n, keys.numel,
                                                       keys.nseg)
    ws = (workspace or _WS).get(keys.device, need)
    btab = keys.base_table(base)
    w = _fp32_dev(weights, keys.device)
    sq = torch.empty((keys.n, keys.nseg), dtype=torch.float64,
                     device=keys.device)
    L.check(lib.fsagg_delta_sqnorm_wsum_keys_f32(
        keys.table.data_ptr(), w.data_ptr(), keys.n, keys.numel,
        btab.data_ptr(), keys.seg.data_ptr(), keys.nseg, sq.data_ptr(),
        out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(keys.device)),
        'fsagg_delta_sqnorm_wsum_keys_f32')
    return sq


def delta_wsum_keys(keys, weights, base, out):
    """:func:`delta_wsum` over a :class:`KeyTable`; ``out`` is flat (keys
    concatenated in table order)."""
    _check_out(out, keys.numel, keys.device, align=4)
    if len(weights) != keys.n:
        raise ValueError('%d weights for %d clients' % (len(weights), keys.n))
    btab = keys.base_table(base)
    w = _fp32_dev(weights, keys.device)
    L.check(L.load().fsagg_delta_wsum_keys_f32(
        keys.table.data_ptr(), w.data_ptr(), keys.n, keys.numel,
        btab.data_ptr(), keys.seg.data_ptr(), keys.nseg, out.data_ptr(),
        _stream(keys.device)), 'fsagg_delta_wsum_keys_f32')
    return out


# -- row sets: client key tensors read in place (include/fsagg.h) -----------
import numpy as _np  # noqa: E402

CHUNK_DTYPE = _np.dtype([('lo', '<i8'), ('len', '<i4'), ('seg', '<i4')])


def _cuda_index(device):
    d = torch.device(device)
    if d.type == 'cuda' and d.index is None:
        d = torch.device('cuda', torch.cuda.current_device())
    return d


def absent(layout, table):
    """[n][m] bool: the NULL entries of a row table that name a non-empty
    key (an empty tensor's NULL pointer is never dereferenced: no chunk
    covers it)."""
    table = _np.asarray(table)
    if table.shape[1] == 1:
        return table == 0
    nonempty = _np.array([layout.numels[k] > 0 for k in layout.keys],
                         dtype=bool)
    return (table == 0) & nonempty[None, :]


class RowSet:
    """``n`` clients x the fp32 key segments of a :class:`BucketLayout`,
    addressed in place (struct fsagg_rows): entry (i, s) is client i's
    virtual base for key s — its key tensor's address minus 4 x the key's
    bucket offset, or its stack row (where bucket coordinates are row
    coordinates).  0 = the client lacks the key.  ``table`` is the host
    copy ([n][1] for a stack without absent keys, else [n][nseg])."""

    def __init__(self, layout, table, device, keepalive=(), aligned16=True,
                 missing=None, segmajor=None, uniform=False, ephemeral=False):
        if segmajor is not None:
            # the device layout built by the caller ([nseg][n]); the host
            # copy is its transposed view
            segmajor = _np.ascontiguousarray(segmajor, dtype=_np.int64)
            table = segmajor.T
        else:
            table = _np.ascontiguousarray(table, dtype=_np.int64)
        if table.ndim != 2 or table.shape[0] < 1:
            raise ValueError('row table must be [n][1] or [n][nseg]')
        self.layout = layout
        self.host = table
        self.n = table.shape[0]
        self.nseg = max(len(layout.keys), 1)
        # on the device the table is segment-major: one chunk's n client
        # pointers are contiguous (batched scalar loads, a small
        # scalar-cache footprint per workgroup)
        if table.shape[1] == 1:
            self.ss = 0
        elif table.shape[1] == self.nseg:
            self.ss = self.n
        else:
            raise ValueError('row table has %d columns for %d keys' %
                             (table.shape[1], self.nseg))
        self.device = _cuda_index(device)
        self.aligned16 = bool(aligned16)
        self.missing = int(absent(layout, table).sum()) if missing is None \
            else int(missing)
        # the device table is uploaded on first use: the flat weighted sum
        # of up to FSAGG_HOSTTAB_MAX_CLIENTS rows passes the host copy in
        # its kernel arguments and never needs it
        self._segmajor = segmajor
        self._tab = None
        self._struct = None
        # a per-call row set (the engine's): its device table may come from
        # the upload ring (see _PinnedRing.upload); persist() before keeping
        # it beyond the call
        self.ephemeral = bool(ephemeral)
        self._keep = tuple(keepalive)
        # uniform: every client's keys lie in ONE storage at their bucket
        # offsets (csrc/host/keytable.cpp), so client i's bucket is the
        # contiguous range at its virtual base — the flat kernels apply
        self.uniform = bool(uniform) and self.missing == 0 and \
            self.host.shape[1] == self.nseg

    @classmethod
    def from_stack(cls, stack, slots, present=None, offset=0,
                   ephemeral=False):
        """Rows ``slots`` of a ClientStack; ``present`` (bool [n][nseg])
        marks absent keys (NULL entries).  Bucket coordinate p is at row
        element p + ``offset`` (a range stack holds a piece of the bucket)."""
        _check_f32_cuda(stack.slab, 'stack')
        base = stack.slab.data_ptr() + 4 * int(offset)
        ld = stack.slab.stride(0) * 4
        rows = _np.array([base + int(s) * ld for s in slots], dtype=_np.int64)
        tab = rows[:, None]
        if present is not None and not _np.all(present):
            tab = _np.where(_np.asarray(present, bool), tab, 0)
        return cls(stack.layout, tab, stack.device, keepalive=(stack.slab, ),
                   aligned16=ld % ALIGN_BYTES == 0 and
                   base % ALIGN_BYTES == 0, ephemeral=ephemeral)

    @classmethod
    def from_pointers(cls, layout, ptrs, device, keepalive=(),
                      aligned16=True, missing=None):
        """[n][nseg] real data pointers of the clients' key tensors (0:
        absent), in layout key order (``missing``: the count of absent
        non-empty keys, when the caller has it)."""
        ptrs = _np.asarray(ptrs, dtype=_np.int64)
        offs = layout.__dict__.get('_offs4')
        if offs is None:
            offs = layout.__dict__['_offs4'] = 4 * _np.array(
                [layout.offsets[k] for k in layout.keys], dtype=_np.int64)
        virt = _np.where(ptrs != 0, ptrs - offs[None, :], 0)
        return cls(layout, virt, device, keepalive=keepalive,
                   aligned16=aligned16, missing=missing)

    @classmethod
    def from_virtual(cls, layout, segmajor, device, keepalive=(),
                     aligned16=True, missing=None, uniform=False,
                     ephemeral=False):
        """[nseg][n] virtual bases (0: absent), i.e. the device table as
        csrc/host/keytable.cpp builds it with offsets (``uniform``: its
        report that each client's keys are views of one storage at their
        bucket offsets)."""
        return cls(layout, None, device, keepalive=keepalive,
                   aligned16=aligned16, missing=missing, segmajor=segmajor,
                   uniform=uniform, ephemeral=ephemeral)

    @property
    def tab(self):
        """The device table ([nseg][n], or [1][n] for ss = 0)."""
        if self._tab is None:
            self._tab = _h2d_np(self.host.T if self._segmajor is None
                                else self._segmajor, self.device,
                                ephemeral=self.ephemeral)
        return self._tab

    def persist(self):
        """Give the row set a device table of its own (for holders beyond
        the call, e.g. a captured launch chain)."""
        if self.ephemeral:
            self.ephemeral = False
            self._tab = self._struct = None
        return self

    @property
    def struct(self):
        if self._struct is None:
            self._struct = L.Rows(self.tab.data_ptr(), self.ss, self.n,
                                  self.nseg)
        return self._struct

    def subset(self, sel):
        """The clients ``sel`` (indices, in the new reduction order)."""
        idx = _np.asarray([int(i) for i in sel], dtype=_np.int64)
        if len(idx) == 0 or idx.min() < 0 or idx.max() >= self.n:
            raise IndexError('row selection outside the %d clients' % self.n)
        # a subset of a table without absent entries has none; each client
        # of a uniform set is uniform on its own
        return RowSet(self.layout, self.host[idx], self.device,
                      keepalive=self._keep, aligned16=self.aligned16,
                      missing=0 if self.missing == 0 else None,
                      uniform=self.uniform, ephemeral=self.ephemeral)

    def ptr(self):
        return ctypes.byref(self.struct)


class BaseRows:
    """The ``base`` operand of the row-set kernels (the server's init model
    of the robust rules' init + update): per-key virtual bases of device
    tensors, or one flat bucket."""

    def __init__(self, host, bss, device, keepalive=(), ephemeral=False):
        self.bss = bss
        self.host = host      # the per-key virtual bases (host copy)
        self.device = device
        self.ephemeral = bool(ephemeral)
        self._tab = None
        self._keep = tuple(keepalive)

    @classmethod
    def from_bucket(cls, flat):
        _check_f32_cuda(flat, 'base bucket')
        return cls([flat.data_ptr()], 0, flat.device, keepalive=(flat, ))

    @classmethod
    def from_pointers(cls, layout, ptrs, device, keepalive=(),
                      ephemeral=False):
        ptrs = _np.asarray(ptrs, dtype=_np.int64).reshape(-1)
        offs = _np.array([layout.offsets[k] for k in layout.keys],
                         dtype=_np.int64)
        virt = ptrs - 4 * offs
        return cls([int(v) for v in virt], 1, _cuda_index(device),
                   keepalive=keepalive, ephemeral=ephemeral)

    @property
    def tab(self):
        """The device table, uploaded on first use (the kernel-argument
        paths read the host copy and never need it)."""
        if self._tab is None:
            self._tab = _h2d_np(_np.asarray(self.host, dtype=_np.int64),
                                self.device, ephemeral=self.ephemeral)
        return self._tab

    def ptr(self):
        return self.tab.data_ptr()


def _rows_out(rs, out, align):
    _check_f32_cuda(out, 'out', align=align)
    if out.device != rs.device or out.numel() < rs.layout.numel:
        raise ValueError('out must hold the %d-element bucket on %s' %
                         (rs.layout.numel, rs.device))


def weighted_sum_rows(rs, weights, out, prescale=None, base=None, lo=0,
                      hi=None):
    """:func:`weighted_sum` over a row set, on the keys' coordinates in
    [lo, hi) of the flat ``out`` bucket; absent keys are skipped per
    client (the reference's missing-key rule, in the same launch)."""
    if len(weights) != rs.n:
        raise ValueError('%d weights for %d rows' % (len(weights), rs.n))
    if not rs.aligned16:
        raise ValueError('weighted_sum_rows needs 16-byte aligned key '
                         'tensors')
    _rows_out(rs, out, ALIGN_BYTES)
    lib = L.load()
    if _flat_rows(rs, base):
        # one key, every client holding it (a flat model, configs[2]): the
        # row set IS a row table — the flat streaming kernel runs on it
        # directly, without the chunk list
        return _weighted_sum_rows_flat(rs, weights, out, prescale, base, lo,
                                       hi, lib)
    unit = lib.fsagg_wsum_chunk_elems_n(rs.layout.numel, rs.n)
    chunks, nchunk = rs.layout.row_chunks(unit, rs.device, lo, hi)
    if nchunk == 0:
        return out
    if _rows_hosttab(rs, weights, prescale, base):
        # a small row set: its tables in the kernel arguments, no upload
        tab = rs._segmajor if rs._segmajor is not None else rs.host.T
        if tab.shape[0] != rs.nseg:          # a stack row: every key
            tab = _np.broadcast_to(tab, (rs.nseg, rs.n))
        tab = _np.ascontiguousarray(tab, dtype=_np.int64)
        w = _np.asarray(weights, dtype=_np.float32)
        pre = None if prescale is None else _np.asarray(prescale,
                                                        dtype=_np.float32)
        if pre is not None and len(pre) != rs.n:
            raise ValueError('prescale length mismatch')
        bt = None
        if base is not None:
            bt = _np.asarray(base.host, dtype=_np.int64)
            if base.bss == 0:
                bt = _np.full(rs.nseg, bt[0], dtype=_np.int64)
        L.check(lib.fsagg_weighted_sum_rows_hosttab_f32(
            tab.ctypes.data, rs.n, rs.nseg, chunks.data_ptr(), nchunk, unit,
            w.ctypes.data, pre.ctypes.data if pre is not None else None,
            bt.ctypes.data if bt is not None else None, out.data_ptr(),
            _stream(rs.device)), 'fsagg_weighted_sum_rows_hosttab_f32')
        return out
    w = weights if isinstance(weights, torch.Tensor) else _fp32_dev(
        weights, rs.device)
    pre = None
    if prescale is not None:
        if len(prescale) != rs.n:
            raise ValueError('prescale length mismatch')
        pre = prescale if isinstance(prescale, torch.Tensor) else _fp32_dev(
            prescale, rs.device)
    L.check(lib.fsagg_weighted_sum_rows_f32(
        rs.ptr(), chunks.data_ptr(), nchunk, unit, w.data_ptr(),
        pre.data_ptr() if pre is not None else None,
        base.ptr() if base is not None else None,
        base.bss if base is not None else 0, out.data_ptr(),
        _stream(rs.device)), 'fsagg_weighted_sum_rows_f32')
    return out


def _rows_hosttab(rs, weights, prescale, base):
    """Whether a multi-key row set's weighted sum takes its tables in the
    kernel arguments (fsagg_weighted_sum_rows_hosttab_f32): few rows, host
    weights and prescales, a base with a host table."""
    return rs.n <= L.FSAGG_HOSTTAB_ROWS_MAX_CLIENTS and \
        rs.n * rs.nseg <= L.FSAGG_HOSTTAB_ROWS_MAX_PTRS and \
        not isinstance(weights, torch.Tensor) and \
        not isinstance(prescale, torch.Tensor) and (
            base is None or (base.host is not None and
                             rs.nseg <= L.FSAGG_HOSTTAB_ROWS_MAX_SEGS and
                             len(base.host) in (1, rs.nseg)))


def _flat_rows(rs, base):
    """Whether a row set runs the flat streaming kernel: one key every
    client holds, or a uniform row set (each client's keys laid out in one
    storage exactly as the bucket: its bucket is one contiguous range, the
    padding between keys included, which lies inside that storage)."""
    return (rs.nseg == 1 or getattr(rs, 'uniform', False)) and \
        not rs.missing and bool(rs.layout.keys) and (
            base is None or (base.host is not None and len(base.host) == 1))


def weighted_sum_rows_bcast(rs, weights, out, peers, prescale=None,
                            base=None, lo=0, hi=None):
    """:func:`weighted_sum_rows` whose result also lands in the peer copies
    ``peers`` (device addresses of other GPUs' output buckets, same
    coordinates) from the reducing kernel's own epilogue
    (fsagg_weighted_sum_bcast_f32, core/sharding.PeerAssembly).  Returns
    False, computing nothing, when the row set has no fused form (several
    keys or absent keys): the caller then computes and pushes."""
    if len(weights) != rs.n:
        raise ValueError('%d weights for %d rows' % (len(weights), rs.n))
    if not (rs.aligned16 and _flat_rows(rs, base)) or \
            len(peers) + 1 > L.FSAGG_MAX_PEERS:
        return False
    _rows_out(rs, out, ALIGN_BYTES)
    _weighted_sum_rows_flat(rs, weights, out, prescale, base, lo, hi,
                            L.load(), peers=peers)
    return True


def _weighted_sum_rows_flat(rs, weights, out, prescale, base, lo, hi, lib,
                            peers=None):
    if rs.nseg == 1:
        k = rs.layout.keys[0]
        o, m = rs.layout.offsets[k], rs.layout.numels[k]
    else:          # uniform: the bucket up to the last key's end (the
        # storage holds every key, so everything before it too)
        last = rs.layout.keys[-1]
        o, m = 0, rs.layout.offsets[last] + rs.layout.numels[last]
    a = max(int(lo), o)
    b = min(int(hi) if hi is not None else rs.layout.numel, o + m)
    if b <= a:
        return out
    if a % 4:
        raise ValueError('row range start %d is not 16-byte aligned' % a)
    if rs.n <= L.FSAGG_HOSTTAB_MAX_CLIENTS and \
            not isinstance(weights, torch.Tensor) and \
            not isinstance(prescale, torch.Tensor):
        # host tables in the kernel arguments: nothing to upload
        return _weighted_sum_hosttab(rs, weights, out, prescale, base, a, b,
                                     lib, peers)
    # entry i = the client's virtual base: coordinate p at entry + 4·p
    if a == 0:
        table = rs.tab
    else:
        table = _h2d_np(rs.host[:, 0] + 4 * a, rs.device, ephemeral=True)
    w = weights if isinstance(weights, torch.Tensor) else _fp32_dev(
        weights, rs.device)
    pre = None
    if prescale is not None:
        if len(prescale) != rs.n:
            raise ValueError('prescale length mismatch')
        pre = prescale if isinstance(prescale, torch.Tensor) else _fp32_dev(
            prescale, rs.device)
    bptr = None
    if base is not None:
        bptr = int(base.host[0]) + 4 * a
        if bptr % ALIGN_BYTES:
            raise ValueError('base is not 16-byte aligned at %d' % a)
    if peers is not None:
        outs = [out.data_ptr() + 4 * a] + [int(p) + 4 * a for p in peers]
        arr = (ctypes.c_void_p * len(outs))(*outs)
        L.check(lib.fsagg_weighted_sum_bcast_f32(
            table.data_ptr(), w.data_ptr(),
            pre.data_ptr() if pre is not None else None, rs.n, b - a, bptr,
            arr, len(outs), _stream(rs.device)),
            'fsagg_weighted_sum_bcast_f32')
        return out
    L.check(lib.fsagg_weighted_sum_f32(
        table.data_ptr(), w.data_ptr(),
        pre.data_ptr() if pre is not None else None, rs.n, b - a, bptr,
        out.data_ptr() + 4 * a, _stream(rs.device)), 'fsagg_weighted_sum_f32')
    return out


def _weighted_sum_hosttab(rs, weights, out, prescale, base, a, b, lib,
                          peers):
    """The flat weighted sum of ``rs``'s coordinates [a, b) with its row
    table, weights and prescales in the kernel arguments
    (fsagg_weighted_sum_hosttab_f32)."""
    n = rs.n
    if len(weights) != n:
        raise ValueError('%d weights for %d rows' % (len(weights), n))
    rows = _np.ascontiguousarray(rs.host[:, 0] + 4 * a, dtype=_np.uint64)
    w = _np.asarray(weights, dtype=_np.float32)
    pre = None
    if prescale is not None:
        if len(prescale) != n:
            raise ValueError('prescale length mismatch')
        pre = _np.asarray(prescale, dtype=_np.float32)
    bptr = None
    if base is not None:
        bptr = int(base.host[0]) + 4 * a
        if bptr % ALIGN_BYTES:
            raise ValueError('base is not 16-byte aligned at %d' % a)
    outs = [out.data_ptr() + 4 * a]
    if peers is not None:
        outs += [int(p) + 4 * a for p in peers]
    arr = (ctypes.c_void_p * len(outs))(*outs)
    L.check(lib.fsagg_weighted_sum_hosttab_f32(
        rows.ctypes.data, w.ctypes.data,
        pre.ctypes.data if pre is not None else None, n, b - a, bptr, arr,
        len(outs), _stream(rs.device)), 'fsagg_weighted_sum_hosttab_f32')
    return out


def _require_all(rs, what):
    if rs.missing:
        raise KeyError('%s needs every client to hold every key (%d absent)'
                       % (what, rs.missing))


def coord_median_rows(rs, out, base=None, lo=0, hi=None):
    _require_all(rs, 'median')
    _rows_out(rs, out, 4)
    chunks, nchunk = rs.layout.row_chunks(L.FSAGG_ROWS_OS_CHUNK, rs.device,
                                          lo, hi)
    if nchunk == 0:
        return out
    L.check(L.load().fsagg_coord_median_rows_f32(
        rs.ptr(), chunks.data_ptr(), nchunk, rs.layout.numel,
        base.ptr() if base is not None else None,
        base.bss if base is not None else 0, out.data_ptr(),
        _stream(rs.device)), 'fsagg_coord_median_rows_f32')
    return out


def trimmed_mean_rows(rs, k, out, divisor=None, base=None, lo=0, hi=None):
    _require_all(rs, 'trimmed mean')
    if k < 0 or 2 * k >= rs.n:
        raise ValueError('trimmed mean needs 0 <= 2k < n (k=%d n=%d)' %
                         (k, rs.n))
    _rows_out(rs, out, 4)
    chunks, nchunk = rs.layout.row_chunks(L.FSAGG_ROWS_OS_CHUNK, rs.device,
                                          lo, hi)
    if nchunk == 0:
        return out
    div = float(rs.n - 2 * k if divisor is None else divisor)
    L.check(L.load().fsagg_trimmed_mean_rows_f32(
        rs.ptr(), chunks.data_ptr(), nchunk, rs.layout.numel, int(k), div,
        base.ptr() if base is not None else None,
        base.bss if base is not None else 0, out.data_ptr(),
        _stream(rs.device)), 'fsagg_trimmed_mean_rows_f32')
    return out


def pairdist_rows_segsq(rs, lo=0, hi=None, workspace=None, keep=None,
                        extent=None):
    """Per-key squared pair distances [nseg][n][n] (fp64) over the keys'
    coordinates in [lo, hi) (a rank's range: summed across ranks by the
    caller, then :func:`pairdist_finish`); ``keep``: a predicate on a key's
    element count — the other keys' entries are 0."""
    _require_all(rs, 'Krum')
    if rs.n < 2:
        raise ValueError('Krum needs at least two clients')
    lay = rs.layout
    hi = lay.numel if hi is None else hi
    seg_lo, seg_end = lay.seg_bounds(rs.device, lo, hi, keep)
    lib = L.load()
    # plans ~1000 chunks over the range (``extent``: the coordinates the
    # kept keys actually hold, when only some are)
    extent = max(hi - lo if extent is None else int(extent), 1)
    need = lib.fsagg_pairdist_workspace_bytes(rs.n, extent, rs.nseg)
    ws = (workspace or _WS).get(rs.device, need)
    sq = torch.empty((rs.nseg, rs.n, rs.n), dtype=torch.float64,
                     device=rs.device)
    L.check(lib.fsagg_pairdist_rows_segsq_f32(
        rs.ptr(), seg_lo.data_ptr(), seg_end.data_ptr(), extent,
        sq.data_ptr(), ws.data_ptr(), ws.numel(), _stream(rs.device)),
        'fsagg_pairdist_rows_segsq_f32')
    return sq


def pairgram_rows_segsq(rs, lo=0, hi=None, workspace=None, keep=None):
    """As :func:`pairdist_rows_segsq`, on the matrix cores (n <= 256,
    fsagg_pairgram_rows_segsq_f32): returns ``[2][nseg][n][n]`` fp64 —
    [0] the per-key squared distances, [1] their predicted absolute error
    bounds (both may be summed over ranks); :func:`pairgram_finish` turns
    them into D and the pairs to recompute."""
    _require_all(rs, 'Krum')
    if not 2 <= rs.n <= L.FSAGG_PAIRGRAM_MAX_CLIENTS:
        raise ValueError('the Gram path takes 2..%d clients' %
                         L.FSAGG_PAIRGRAM_MAX_CLIENTS)
    lay = rs.layout
    hi = lay.numel if hi is None else hi
    seg_lo, seg_end = lay.seg_bounds(rs.device, lo, hi, keep)
    lib = L.load()
    extent = max(hi - lo, 1)
    need = lib.fsagg_pairgram_workspace_bytes(rs.n, extent, rs.nseg)
    ws = (workspace or _WS).get(rs.device, need)
    out = torch.empty((2, rs.nseg, rs.n, rs.n), dtype=torch.float64,
                      device=rs.device)
    L.check(lib.fsagg_pairgram_rows_segsq_f32(
        rs.ptr(), seg_lo.data_ptr(), seg_end.data_ptr(), extent,
        out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(), ws.numel(),
        _stream(rs.device)), 'fsagg_pairgram_rows_segsq_f32')
    return out


def _gram_buf(n, device):
    """The finish's outputs in one int32 [5][n][n] device tensor (one copy
    to the host): planes 0-1 D64 (fp64 [n][n], first so that it is 8-byte
    aligned for any n), planes 2-4 D (fp32), ill, B (fp32).  Returns (buf,
    D, ill, B, D64) views (:func:`gram_views` of a host copy)."""
    buf = torch.empty((5, n, n), dtype=torch.int32, device=device)
    return (buf,) + gram_views(buf)


def gram_views(buf):
    """(D, ill, B, D64) views of a :func:`_gram_buf` buffer (device or a
    host copy)."""
    n = int(buf.shape[1])
    return buf[2].view(torch.float32), buf[3], buf[4].view(torch.float32), \
        buf[0:2].reshape(-1).view(torch.float64).view(n, n)


def pairgram_finish(sq2, tol):
    """D (fp32 [n][n], device, as :func:`pairdist_finish`), ill (int32
    [n][n]: the pairs whose bound exceeds ``tol``·D, or non-finite), B
    (fp32 [n][n]: each pair's worst-case bound on |Σ_key d_key − the exact
    distance|) and D64 (fp64 [n][n]: Σ_key d_key in fp64, what B bounds
    without D's own fp32 rounding) from :func:`pairgram_rows_segsq`'s
    output: returns (buf, D, ill, B, D64) as :func:`_gram_buf`."""
    if sq2.dim() != 4 or sq2.shape[0] != 2 or sq2.dtype != torch.float64 \
            or not sq2.is_contiguous():
        raise ValueError('sq2 must be a contiguous fp64 [2][nseg][n][n] '
                         'tensor')
    nseg, n = int(sq2.shape[1]), int(sq2.shape[2])
    buf, D, ill, B, D64 = _gram_buf(n, sq2.device)
    L.check(L.load().fsagg_pairgram_finish_f32(
        sq2[0].data_ptr(), sq2[1].data_ptr(), n, nseg, float(tol),
        D.data_ptr(), ill.data_ptr(), B.data_ptr(), D64.data_ptr(),
        _stream(sq2.device)), 'fsagg_pairgram_finish_f32')
    return buf, D, ill, B, D64


def _pairgram_rows_launch(rs, tol, seg_lo, seg_end, ws, sq2, buf):
    D, ill, B, D64 = gram_views(buf)
    L.check(L.load().fsagg_pairgram_rows_f32(
        rs.ptr(), seg_lo.data_ptr(), seg_end.data_ptr(),
        max(rs.layout.numel, 1), float(tol), sq2[0].data_ptr(),
        sq2[1].data_ptr(), D.data_ptr(), ill.data_ptr(), B.data_ptr(),
        D64.data_ptr(), ws.data_ptr(), ws.numel(), _stream(rs.device)),
        'fsagg_pairgram_rows_f32')


def pairgram_rows_dist(rs, tol, workspace=None):
    """:func:`pairgram_rows_segsq` and :func:`pairgram_finish` in one call
    (fsagg_pairgram_rows_f32).  Returns (buf, D, ill, B, D64, sq2) as those
    two."""
    _require_all(rs, 'Krum')
    if not 2 <= rs.n <= L.FSAGG_PAIRGRAM_MAX_CLIENTS:
        raise ValueError('the Gram path takes 2..%d clients' %
                         L.FSAGG_PAIRGRAM_MAX_CLIENTS)
    lay = rs.layout
    seg_lo, seg_end = lay.seg_bounds(rs.device, 0, lay.numel, None)
    need = L.load().fsagg_pairgram_workspace_bytes(rs.n, max(lay.numel, 1),
                                                   rs.nseg)
    ws = (workspace or _WS).get(rs.device, need)
    sq2 = torch.empty((2, rs.nseg, rs.n, rs.n), dtype=torch.float64,
                      device=rs.device)
    buf = _gram_buf(rs.n, rs.device)[0]
    _pairgram_rows_launch(rs, tol, seg_lo, seg_end, ws, sq2, buf)
    return (buf,) + gram_views(buf) + (sq2,)


class _GraphCache:
    """Captured launch chains (HIP graphs, through torch.cuda.CUDAGraph) of
    the multi-kernel paths whose launches cost more host time than their
    small kernels run: the Gram chain is six launches (~100 µs of host
    time at C4, against ~10 µs for one graph launch).  One entry per SHAPE
    — client count, table stride, the layout, the tolerance, the library's
    workgroup-form settings, the stream — owning everything the captured
    kernels' arguments name: a pinned host table, a device row table, the
    workspace, the per-key sums and the output buffer.  A call writes ITS
    row table (the clients' addresses, fresh or not) into the entry's
    pinned table, once the previous replay's fetch of it has completed (the
    entry's event), and replays; the graph's first kernel fetches the
    pinned table into the device table (fsagg_fetch_mapped_u64).  So rounds
    of freshly received uploads replay a graph as well as repeated calls
    over the same dicts do.  The outputs are overwritten by the next call
    of the same shape — a caller consumes them (copies them to the host)
    before its next call.  The first call of a shape runs the chain eagerly
    (its result) and captures it (the capture only records launches).  An
    evicted entry waits for its last fetch before its buffers go back to
    torch's allocators."""
    MAX_ENTRIES = 8

    def __init__(self):
        from collections import OrderedDict
        self.entries = OrderedDict()
        self.enabled = True
        self.captures = 0

    def lookup(self, key):
        e = self.entries.get(key)
        if e is not None:
            self.entries.move_to_end(key)
        return e

    def put(self, key, e):
        self.entries[key] = e
        self.captures += 1
        while len(self.entries) > self.MAX_ENTRIES:
            _, old = self.entries.popitem(last=False)
            # the evicted chain's last replay must have read its pinned
            # table before the pinned block can go back to torch's host
            # allocator (which does not see the kernel's read)
            fetch = old[3] if len(old) > 3 else None
            if isinstance(fetch, tuple) and len(fetch) == 2 and \
                    isinstance(fetch[1], torch.cuda.Event):
                fetch[1].synchronize()
        return e


_GRAPHS = _GraphCache()


def _copy_table(host, dst, device):
    """The row table ``host`` into the device buffer ``dst`` on the current
    stream (ordered after the work already queued there)."""
    import numpy as np
    raw = np.ascontiguousarray(host).reshape(-1).view(np.uint8)
    if raw.size > _RING.SLOT or raw.size != dst.numel() * dst.element_size():
        raise ValueError('row table of %d bytes for a %d-byte slot' %
                         (raw.size, dst.numel() * dst.element_size()))
    ring = _RING
    if ring.buf is None:
        ring.buf = torch.empty(ring.SLOT * ring.NSLOT, dtype=torch.uint8,
                               pin_memory=True)
        ring.buf_ptr = ring.buf.data_ptr()
    k = ring.i
    ring.i = (k + 1) % ring.NSLOT
    cur = ctypes_ptr(torch._C._cuda_getCurrentRawStream(device.index))
    L.check(L.load().fsagg_upload_h2d(
        dst.data_ptr(), raw.ctypes.data, raw.size,
        ring.buf_ptr + k * ring.SLOT, k, ring.NSLOT, cur, cur),
        'fsagg_upload_h2d')


def pairgram_rows_dist_graph(rs, tol):
    """:func:`pairgram_rows_dist` replayed from the captured chain of its
    shape (see _GraphCache): returns (buf, D, ill, B, D64) views of a buffer
    valid until the next call of the same shape."""
    if not _GRAPHS.enabled:
        return pairgram_rows_dist(rs, tol)[:5]
    _require_all(rs, 'Krum')
    if not 2 <= rs.n <= L.FSAGG_PAIRGRAM_MAX_CLIENTS:
        raise ValueError('the Gram path takes 2..%d clients' %
                         L.FSAGG_PAIRGRAM_MAX_CLIENTS)
    lay = rs.layout
    lib = L.load()
    stream = torch._C._cuda_getCurrentRawStream(rs.device.index)
    host = rs.host.T if rs._segmajor is None else rs._segmajor
    # the workgroup-form settings (A/B knobs) select the captured kernels
    key = ('pairgram', rs.device.index, stream, host.shape, rs.ss, rs.n,
           rs.nseg, lay.signature(), float(tol), lib.fsagg_pairgram_knobs())
    e = _GRAPHS.lookup(key)
    if e is None:
        need = max(int(lib.fsagg_pairgram_workspace_bytes(
            rs.n, max(lay.numel, 1), rs.nseg)), 1)
        ws = torch.empty(need, dtype=torch.uint8, device=rs.device)
        sq2 = torch.empty((2, rs.nseg, rs.n, rs.n), dtype=torch.float64,
                          device=rs.device)
        seg_lo, seg_end = lay.seg_bounds(rs.device, 0, lay.numel, None)
        buf = _gram_buf(rs.n, rs.device)[0]
        tab = torch.empty(host.size, dtype=torch.int64, device=rs.device)
        # the row table's pinned source: the graph's first kernel reads it
        # (fsagg_fetch_mapped_u64), the host refills it before each replay
        pin = torch.empty(host.size, dtype=torch.int64, pin_memory=True)
        pin_np = pin.numpy().reshape(host.shape)
        done = torch.cuda.Event()
        rows = L.Rows(tab.data_ptr(), rs.ss, rs.n, rs.nseg)
        pin_np[...] = host

        def launch():
            L.check(lib.fsagg_fetch_mapped_u64(
                pin.data_ptr(), tab.data_ptr(), host.size,
                _stream(rs.device)), 'fsagg_fetch_mapped_u64')
            L.check(lib.fsagg_pairgram_rows_f32(
                ctypes.byref(rows), seg_lo.data_ptr(), seg_end.data_ptr(),
                max(lay.numel, 1), float(tol), sq2[0].data_ptr(),
                sq2[1].data_ptr(), *[v.data_ptr() for v in gram_views(buf)],
                ws.data_ptr(), ws.numel(), _stream(rs.device)),
                'fsagg_pairgram_rows_f32')
        launch()              # this call's result (and the code objects)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            launch()
        done.record()
        _GRAPHS.put(key, (g, buf, tab, (pin_np, done),
                          (rows, ws, sq2, seg_lo, seg_end, pin)))
        rs._gram_tab = tab
        return (buf,) + gram_views(buf)
    g, buf, tab, (pin_np, done), _ = e
    # the previous replay's fetch has read the pinned table (a caller that
    # consumed that replay's outputs has waited for it already: no wait)
    done.synchronize()
    pin_np[...] = host
    g.replay()
    done.record()
    # the chain's own device copy of this call's row table (valid until the
    # next call of the shape): krum_select gathers the selection from it
    rs._gram_tab = tab
    return (buf,) + gram_views(buf)


def krum_select(buf, nseg, f, m, ordered, sizes, ignore_weight, tab, ss,
                nsegt, base=None):
    """Krum's certified selection on the device from a Gram finish buffer
    (fsagg_krum_select_f32), with the first min(m, n) clients' row table,
    fp32 weights and base table for :func:`weighted_sum_rows_devtab`.
    ``tab``: the clients' device table [nsegt][n] (ss = n) or [1][n]
    (ss = 0); ``base``: nseg virtual bases (host ints) or None.  Returns
    (sel, sub_tab, sub_w, sub_base) device views of one allocation: sel
    int32 [2 + n] = certified, valid, order."""
    n = int(buf.shape[1])
    msel = min(int(m), n)
    nsb = len(base) if base is not None else 0
    w_sel = (2 + n + 1) // 2
    w_tab = nsegt * msel
    w_w = (msel + 1) // 2
    blob = torch.empty(4 * n + w_sel + w_tab + w_w + nsb, dtype=torch.int64,
                       device=buf.device)
    work = blob[:4 * n]
    o = 4 * n
    sel = blob[o:o + w_sel].view(torch.int32)[:2 + n]
    o += w_sel
    sub_tab = blob[o:o + w_tab].view(nsegt, msel)
    o += w_tab
    sub_w = blob[o:o + w_w].view(torch.float32)[:msel]
    o += w_w
    sub_base = blob[o:o + nsb] if nsb else None
    sz = _np.ascontiguousarray(sizes, dtype=_np.float64)
    bt = _np.ascontiguousarray(base, dtype=_np.int64) if nsb else None
    L.check(L.load().fsagg_krum_select_f32(
        buf.data_ptr(), n, int(nseg), int(f), int(m), int(bool(ordered)),
        sz.ctypes.data, int(bool(ignore_weight)),
        bt.ctypes.data if bt is not None else None, tab.data_ptr(), int(ss),
        int(nsegt), work.data_ptr(), sel.data_ptr(), sub_tab.data_ptr(),
        sub_w.data_ptr(), sub_base.data_ptr() if nsb else None,
        _stream(buf.device)), 'fsagg_krum_select_f32')
    return sel, sub_tab, sub_w, sub_base


def weighted_sum_rows_devtab(layout, tab, ss, n, weights, out, base=None):
    """fsagg_weighted_sum_rows_f32 over a row table that already lives on
    the device ([nseg][n] virtual bases with ss = n, or [1][n] with ss = 0;
    device fp32 ``weights``; ``base`` a device [nseg] table or None) into
    the flat ``out`` bucket — the average behind :func:`krum_select`."""
    lib = L.load()
    dev = out.device
    unit = lib.fsagg_wsum_chunk_elems_n(layout.numel, n)
    chunks, nchunk = layout.row_chunks(unit, dev, 0, None)
    if nchunk == 0:
        return out
    rows = L.Rows(tab.data_ptr(), int(ss), int(n), max(len(layout.keys), 1))
    L.check(lib.fsagg_weighted_sum_rows_f32(
        ctypes.byref(rows), chunks.data_ptr(), nchunk, unit,
        weights.data_ptr(), None,
        base.data_ptr() if base is not None else None,
        1 if base is not None else 0, out.data_ptr(), _stream(dev)),
        'fsagg_weighted_sum_rows_f32')
    return out


def pairdist_rows(rs, workspace=None):
    """Krum's distance matrix D[n][n] (fp32, device) over a row set."""
    return pairdist_finish(pairdist_rows_segsq(rs, workspace=workspace))


def pairsel_rows_segsq(rs, sel, lo=0, hi=None, workspace=None):
    """Per-key squared distances [nseg][len(sel)][n] (fp64, device) of the
    clients ``sel`` (device int32) to every client over the keys'
    coordinates in [lo, hi), in fp64 throughout (fsagg_pairsel_rows_segsq_f64;
    summed across ranks by the caller, then :func:`pairsel_finish`)."""
    _require_all(rs, 'Krum')
    nsel = int(sel.numel())
    if not 2 <= rs.n <= L.FSAGG_PAIRSEL_MAX_CLIENTS or \
            not 1 <= nsel <= L.FSAGG_PAIRSEL_MAX_SEL:
        raise ValueError('the selected-rows kernel takes 2..%d clients and '
                         '1..%d selected' % (L.FSAGG_PAIRSEL_MAX_CLIENTS,
                                             L.FSAGG_PAIRSEL_MAX_SEL))
    if sel.dtype != torch.int32 or sel.device != rs.device or \
            not sel.is_contiguous():
        raise ValueError('sel must be a contiguous int32 tensor on the rows\' '
                         'device')
    lib = L.load()
    chunks, nchunk = rs.layout.row_chunks(L.FSAGG_PAIRSEL_CHUNK, rs.device,
                                          lo, hi)
    need = lib.fsagg_pairsel_workspace_bytes(nsel, rs.n, max(nchunk, 1))
    ws = (workspace or _WS).get(rs.device, need)
    sq = torch.empty((rs.nseg, nsel, rs.n), dtype=torch.float64,
                     device=rs.device)
    L.check(lib.fsagg_pairsel_rows_segsq_f64(
        rs.ptr(), sel.data_ptr(), nsel,
        chunks.data_ptr() if chunks is not None else None, nchunk,
        sq.data_ptr(), ws.data_ptr(), ws.numel(), _stream(rs.device)),
        'fsagg_pairsel_rows_segsq_f64')
    return sq


def pairsel_finish(segsq, sel):
    """D rows [len(sel)][n] (fp64, device): Σ_key sqrt of
    :func:`pairsel_rows_segsq`'s output in key order, +inf at each selected
    client's own column."""
    if segsq.dim() != 3 or segsq.dtype != torch.float64 or \
            not segsq.is_contiguous():
        raise ValueError('segsq must be a contiguous fp64 [nseg][nsel][n] '
                         'tensor')
    nseg, nsel, n = (int(x) for x in segsq.shape)
    D = torch.empty((nsel, n), dtype=torch.float64, device=segsq.device)
    L.check(L.load().fsagg_pairsel_finish_f64(
        segsq.data_ptr(), sel.data_ptr(), nsel, n, nseg, D.data_ptr(),
        _stream(segsq.device)), 'fsagg_pairsel_finish_f64')
    return D


def rows_sqnorm(rs, lo=0, hi=None, workspace=None):
    """[n][nseg] fp64 per-client, per-key Σx² over [lo, hi) (0 for absent
    keys)."""
    lib = L.load()
    unit = lib.fsagg_wsum_chunk_elems(rs.layout.numel)
    chunks, nchunk = rs.layout.row_chunks(unit, rs.device, lo, hi)
    need = lib.fsagg_rows_sqnorm_workspace_bytes(rs.n, max(nchunk, 1))
    ws = (workspace or _WS).get(rs.device, need)
    sq = torch.empty((rs.n, rs.nseg), dtype=torch.float64, device=rs.device)
    L.check(lib.fsagg_rows_sqnorm_f32(
        rs.ptr(), chunks.data_ptr() if chunks is not None else None, nchunk,
        sq.data_ptr(), ws.data_ptr(), ws.numel(), _stream(rs.device)),
        'fsagg_rows_sqnorm_f32')
    return sq


def normbound_prescale(sq, bound):
    """Norm bounding's per-client scale (fp32 [n], device) from
    :func:`rows_sqnorm`'s [n][nseg] fp64: fl32(fl32(1/norm)·fl32(bound))
    where norm = fl32(sqrt(Σ sq)) > fl32(bound), else 1."""
    lib = L.load()
    if sq.dim() != 2 or sq.dtype != torch.float64 or not sq.is_contiguous():
        raise ValueError('sq must be contiguous fp64 [n][nseg]')
    pre = torch.empty(sq.shape[0], dtype=torch.float32, device=sq.device)
    L.check(lib.fsagg_normbound_prescale_f32(
        sq.data_ptr(), sq.shape[0], sq.shape[1], float(_np.float32(bound)),
        pre.data_ptr(), _stream(sq.device)), 'fsagg_normbound_prescale_f32')
    return pre
