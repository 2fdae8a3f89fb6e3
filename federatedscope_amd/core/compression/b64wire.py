"""Base64 (gRPC) uploads decoded on the device.

With the gRPC transport every tensor of a ``model_para`` message travels as
``base64.b64encode(pickle.dumps(tensor))`` (federatedscope/core/message.py
:8-9 b64serializer, applied per tensor leaf by transform_to_list :110-124;
the protobuf string field hands the server a str, :187-188,236-249), and
the server decodes each one on the host inside the aggregation loop
(core/auxiliaries/utils.py:95-105 param2tensor, called per key at
clients_avg_aggregator.py:86-87): base64 → pickle → a second, legacy
``torch.save`` stream inside the pickle → the tensor.

Here the host reads only the *framing* of that byte stream — the pickle
opcodes around the storage record and the legacy header in front of the raw
storage bytes, a few hundred bytes at either end — and locates the raw
fp32 bytes inside the decoded image.  The base64 characters that cover them
then go to the GPU as they are (one pinned copy, one DMA) and
``fsagg_b64_unpack_f32`` decodes them straight into the client's row of the
device stack.  No pickle machinery runs: the framing walker below admits a
whitelist of opcodes and of four globals (the tensor and storage rebuild
helpers, OrderedDict, torch.<T>Storage) and never calls anything, so a
crafted upload cannot execute code, and malformed framing raises
:class:`FramingError`.

Byte stream of one tensor (protocol 2..5 outer pickle; what torch pickles
for a CPU tensor in both the reference's pinned torch 1.10 and this image's
torch):

  _rebuild_tensor_v2(                       torch/_utils.py
      _load_from_bytes(<BINBYTES payload>),  torch/storage.py
      storage_offset, size, stride, requires_grad, OrderedDict())

  payload = legacy torch.save stream (protocol-2 pickles, back to back):
      magic number 0x1950a86a20f9469cfc6c, protocol version 1001,
      sys_info {protocol_version, little_endian, type_sizes},
      the storage as a persistent id
          ('storage', torch.<T>Storage, key, location, numel, None),
      [key],
      then per storage: numel as 8 little-endian bytes + the raw elements.
"""
import base64
import binascii
import struct
from collections import OrderedDict

import torch

__all__ = ['FramingError', 'B64Tensor', 'parse_b64', 'is_b64',
           'B64Stager']


class FramingError(ValueError):
    """The upload is not a base64 pickled tensor this parser understands."""


_STORAGE_DTYPES = {
    'FloatStorage': torch.float32, 'DoubleStorage': torch.float64,
    'HalfStorage': torch.float16, 'BFloat16Storage': torch.bfloat16,
    'LongStorage': torch.int64, 'IntStorage': torch.int32,
    'ShortStorage': torch.int16, 'CharStorage': torch.int8,
    'ByteStorage': torch.uint8, 'BoolStorage': torch.bool,
    'ComplexFloatStorage': torch.complex64,
    'ComplexDoubleStorage': torch.complex128,
}
_MAGIC = 0x1950a86a20f9469cfc6c          # torch/serialization.py MAGIC_NUMBER
_LEGACY_PROTOCOL = 1001                  # torch/serialization.py PROTOCOL_VERSION
_WINDOW = 3072                           # decoded bytes per cached window
_MAX_OPS = 4096                          # opcodes per pickle (framing only)
_MAX_STR = 1 << 16                       # longest str the framing may hold


def is_b64(v):
    """An upload value the gRPC transport delivered as base64 text (a str,
    as param2tensor tests it: utils.py:103-104)."""
    return isinstance(v, str)


class _Text:
    """Random access to the bytes base64 ``text`` decodes to, decoding only
    the 4-character groups a read touches (windows of _WINDOW bytes)."""

    def __init__(self, text):
        if isinstance(text, memoryview):
            text = text.cast('B')
        n = len(text)
        if n == 0 or n % 4:
            raise FramingError('base64 text of %d characters is not a whole '
                               'number of 4-character groups' % n)
        tail = text[-2:]
        if isinstance(tail, str):
            pad = tail.count('=')
        else:
            pad = bytes(tail).count(b'=')
        self.text = text
        self.nchars = n
        self.size = 3 * (n // 4) - pad
        self._win = {}
        self.spans = []          # [lo, hi) decoded bytes the parse read

    def _window(self, w):
        b = self._win.get(w)
        if b is None:
            c0 = 4 * (w * _WINDOW // 3)
            c1 = min(self.nchars, c0 + 4 * (_WINDOW // 3))
            chunk = self.text[c0:c1]
            try:
                b = base64.b64decode(chunk, validate=True)
            except (binascii.Error, ValueError) as e:
                raise FramingError('invalid base64 in the tensor framing: '
                                   '%s' % e) from None
            self._win[w] = b
        return b

    def read_bulk(self, pos, n):
        """Decode bytes [pos, pos + n) in one pass (the storage bytes of a
        host decode).  Non-validating like the reference's b64decode, but a
        character outside the alphabet changes the decoded length, which is
        checked."""
        if pos < 0 or n < 0 or pos + n > self.size:
            raise FramingError('storage bytes outside the stream')
        c0 = 4 * (pos // 3)
        c1 = 4 * (-(-(pos + n) // 3))
        try:
            raw = binascii.a2b_base64(self.text[c0:c1])
        except (binascii.Error, ValueError) as e:
            raise FramingError('invalid base64 in the tensor data: %s' % e) \
                from None
        skip = pos - 3 * (c0 // 4)
        if len(raw) < skip + n or (c1 < self.nchars and
                                   len(raw) != 3 * ((c1 - c0) // 4)):
            raise FramingError('invalid base64 in the tensor data')
        return memoryview(raw)[skip:skip + n]

    def read(self, pos, n):
        if pos < 0 or n < 0 or pos + n > self.size:
            raise FramingError('tensor framing truncated (read of %d bytes '
                               'at %d, stream has %d)' % (n, pos, self.size))
        self.spans.append((pos, pos + n))
        out = []
        while n > 0:
            w, o = divmod(pos, _WINDOW)
            b = self._window(w)
            take = min(n, _WINDOW - o)
            out.append(b[o:o + take])
            pos += take
            n -= take
        return b''.join(out)


# -- a framing-only pickle walker --------------------------------------------
class _Global:
    __slots__ = ('module', 'name')

    def __init__(self, module, name):
        self.module, self.name = module, name

    def __repr__(self):
        return '%s.%s' % (self.module, self.name)


class _Bytes:
    """A bytes object of the stream, not read: (start, length)."""
    __slots__ = ('start', 'length')

    def __init__(self, start, length):
        self.start, self.length = start, length


class _StorageRef:
    __slots__ = ('payload',)

    def __init__(self, payload):
        self.payload = payload


class _PersId:
    __slots__ = ('pid',)

    def __init__(self, pid):
        self.pid = pid


class _TensorRef:
    __slots__ = ('storage', 'offset', 'size', 'stride', 'requires_grad')

    def __init__(self, storage, offset, size, stride, requires_grad):
        self.storage, self.offset = storage, offset
        self.size, self.stride = size, stride
        self.requires_grad = requires_grad


# globals the framing may name; anything else is refused
_OUTER_GLOBALS = {('torch._utils', '_rebuild_tensor_v2'),
                  ('torch._utils', '_rebuild_parameter'),
                  ('torch.storage', '_load_from_bytes'),
                  ('collections', 'OrderedDict')}


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, bool)


def _reduce(fn, args):
    if not isinstance(fn, _Global) or not isinstance(args, tuple):
        raise FramingError('REDUCE of a non-whitelisted callable')
    key = (fn.module, fn.name)
    if key == ('torch.storage', '_load_from_bytes'):
        if len(args) != 1 or not isinstance(args[0], _Bytes):
            raise FramingError('_load_from_bytes takes one bytes object')
        return _StorageRef(args[0])
    if key == ('collections', 'OrderedDict'):
        if args:
            raise FramingError('backward hooks are not part of an upload')
        return OrderedDict()
    if key == ('torch._utils', '_rebuild_tensor_v2'):
        if len(args) not in (6, 7):
            raise FramingError('_rebuild_tensor_v2 takes 6 or 7 arguments')
        st, off, size, stride, rg, hooks = args[:6]
        if len(args) == 7 and args[6] not in (None, {}):
            raise FramingError('tensor metadata is not supported')
        if not isinstance(st, _StorageRef) or not _is_int(off) or \
                not isinstance(size, tuple) or \
                not isinstance(stride, tuple) or \
                not isinstance(rg, bool) or not isinstance(hooks, dict) or \
                hooks:
            raise FramingError('malformed _rebuild_tensor_v2 arguments')
        if len(size) != len(stride) or not all(
                _is_int(x) for x in size + stride):
            raise FramingError('size and stride differ or are not ints')
        return _TensorRef(st, off, size, stride, rg)
    if key == ('torch._utils', '_rebuild_parameter'):
        if len(args) != 3 or not isinstance(args[0], _TensorRef) or \
                not isinstance(args[1], bool) or args[2] not in ({}, None):
            raise FramingError('malformed _rebuild_parameter arguments')
        t = args[0]
        t.requires_grad = args[1]
        return t
    raise FramingError('REDUCE of %s.%s' % key)


def _walk(src, pos, end, globals_ok):
    """Run one pickle of ``src`` (a _Text) from ``pos`` to its STOP, within
    ``end``; returns (value, position after STOP).  Only the opcodes a
    pickled tensor and torch's legacy save header use are admitted; byte
    payloads are skipped, not read."""
    stack = []
    marks = []
    memo = {}

    def rd(n):
        nonlocal pos
        if pos + n > end:
            raise FramingError('pickle runs past its frame')
        b = src.read(pos, n)
        pos += n
        return b

    def u(fmt, n):
        return struct.unpack(fmt, rd(n))[0]

    def pop_mark():
        if not marks:
            raise FramingError('no MARK on the stack')
        m = marks.pop()
        items = stack[m:]
        del stack[m:]
        return items

    def pop():
        if len(stack) <= (marks[-1] if marks else 0):
            raise FramingError('pickle stack underflow')
        return stack.pop()

    def text(n):
        if n > _MAX_STR:
            raise FramingError('string of %d bytes in the framing' % n)
        try:
            return rd(n).decode('utf-8')
        except UnicodeDecodeError:
            raise FramingError('string is not UTF-8') from None

    def line():
        nonlocal pos
        out = bytearray()
        while True:
            c = rd(1)
            if c == b'\n':
                break
            out += c
            if len(out) > 256:
                raise FramingError('GLOBAL name too long')
        return out.decode('ascii', 'strict')

    def global_(module, name):
        if (module, name) in globals_ok:
            return _Global(module, name)
        if ('torch', '*Storage') in globals_ok and module == 'torch' and \
                name in _STORAGE_DTYPES:
            return _Global(module, name)
        raise FramingError('refusing global %s.%s in a model update' %
                           (module, name))

    for _ in range(_MAX_OPS):
        op = rd(1)[0]
        if op == 0x80:                       # PROTO
            if rd(1)[0] > 5:
                raise FramingError('pickle protocol > 5')
        elif op == 0x95:                     # FRAME (framing hint only)
            rd(8)
        elif op == 0x2e:                     # STOP
            if len(stack) != 1 or marks:
                raise FramingError('pickle ends with %d values on the stack'
                                   % len(stack))
            return stack[0], pos
        elif op == 0x28:                     # MARK
            marks.append(len(stack))
        elif op == 0x29:                     # EMPTY_TUPLE
            stack.append(())
        elif op == 0x5d:                     # EMPTY_LIST
            stack.append([])
        elif op == 0x7d:                     # EMPTY_DICT
            stack.append({})
        elif op == 0x74:                     # TUPLE
            stack.append(tuple(pop_mark()))
        elif op in (0x85, 0x86, 0x87):       # TUPLE1..3
            k = op - 0x84
            if len(stack) - (marks[-1] if marks else 0) < k:
                raise FramingError('pickle stack underflow')
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif op == 0x61:                     # APPEND
            v = pop()
            lst = pop()
            if not isinstance(lst, list):
                raise FramingError('APPEND to a non-list')
            lst.append(v)
            stack.append(lst)
        elif op == 0x65:                     # APPENDS
            items = pop_mark()
            lst = pop()
            if not isinstance(lst, list):
                raise FramingError('APPENDS to a non-list')
            lst.extend(items)
            stack.append(lst)
        elif op == 0x73:                     # SETITEM
            v = pop()
            k = pop()
            d = pop()
            if not isinstance(d, dict) or not isinstance(k, str):
                raise FramingError('SETITEM on a non-dict')
            d[k] = v
            stack.append(d)
        elif op == 0x75:                     # SETITEMS
            items = pop_mark()
            d = pop()
            if not isinstance(d, dict) or len(items) % 2:
                raise FramingError('malformed SETITEMS')
            for i in range(0, len(items), 2):
                if not isinstance(items[i], str):
                    raise FramingError('dict key is not a str')
                d[items[i]] = items[i + 1]
            stack.append(d)
        elif op == 0x4e:                     # NONE
            stack.append(None)
        elif op == 0x88:                     # NEWTRUE
            stack.append(True)
        elif op == 0x89:                     # NEWFALSE
            stack.append(False)
        elif op == 0x4b:                     # BININT1
            stack.append(rd(1)[0])
        elif op == 0x4d:                     # BININT2
            stack.append(u('<H', 2))
        elif op == 0x4a:                     # BININT
            stack.append(u('<i', 4))
        elif op == 0x8a:                     # LONG1
            n = rd(1)[0]
            stack.append(int.from_bytes(rd(n), 'little', signed=True))
        elif op == 0x58:                     # BINUNICODE
            stack.append(text(u('<I', 4)))
        elif op == 0x8c:                     # SHORT_BINUNICODE
            stack.append(text(rd(1)[0]))
        elif op == 0x8d:                     # BINUNICODE8
            stack.append(text(u('<Q', 8)))
        elif op in (0x42, 0x43, 0x8e):       # BINBYTES, SHORT_, BINBYTES8
            n = u('<I', 4) if op == 0x42 else \
                (rd(1)[0] if op == 0x43 else u('<Q', 8))
            if pos + n > end:
                raise FramingError('bytes object runs past the stream')
            stack.append(_Bytes(pos, n))
            pos += n
        elif op == 0x63:                     # GLOBAL
            module = line()
            stack.append(global_(module, line()))
        elif op == 0x93:                     # STACK_GLOBAL
            name = pop()
            module = pop()
            if not isinstance(module, str) or not isinstance(name, str):
                raise FramingError('STACK_GLOBAL of non-strings')
            stack.append(global_(module, name))
        elif op == 0x94:                     # MEMOIZE
            if not stack:
                raise FramingError('MEMOIZE of an empty stack')
            memo[len(memo)] = stack[-1]
        elif op in (0x71, 0x72):             # BINPUT, LONG_BINPUT
            idx = rd(1)[0] if op == 0x71 else u('<I', 4)
            if not stack:
                raise FramingError('PUT of an empty stack')
            memo[idx] = stack[-1]
        elif op in (0x68, 0x6a):             # BINGET, LONG_BINGET
            idx = rd(1)[0] if op == 0x68 else u('<I', 4)
            if idx not in memo:
                raise FramingError('GET of an unset memo slot')
            stack.append(memo[idx])
        elif op == 0x52:                     # REDUCE
            args = pop()
            fn = pop()
            stack.append(_reduce(fn, args))
        elif op == 0x51:                     # BINPERSID
            stack.append(_PersId(pop()))
        else:
            raise FramingError('pickle opcode 0x%02x is not part of a '
                               'tensor upload' % op)
    raise FramingError('tensor framing longer than %d opcodes' % _MAX_OPS)


class B64Tensor:
    """The framing of one base64 pickled tensor: dtype, shape, stride,
    storage offset and where the raw storage bytes sit in the decoded
    stream.  ``text`` is kept (not copied) for the device decode."""

    __slots__ = ('text', 'nchars', 'dtype', 'shape', 'stride',
                 'storage_offset', 'storage_numel', 'data_pos',
                 'requires_grad')

    @property
    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n

    @property
    def itemsize(self):
        return self.dtype.itemsize

    def is_contiguous(self):
        expect = 1
        for s, st in zip(reversed(self.shape), reversed(self.stride)):
            if s != 1 and st != expect:
                return False
            expect *= s
        return True

    def char_range(self):
        """(c0, c1, skip): the base64 characters [c0, c1) that decode to the
        tensor's bytes (contiguous tensors), the first of them ``skip``
        (0..2) bytes into the decoded image of c0."""
        if not self.is_contiguous():
            raise FramingError('not a contiguous tensor')
        es = self.itemsize
        a = self.data_pos + es * self.storage_offset
        b = a + es * self.numel
        c0 = 4 * (a // 3)
        c1 = 4 * (-(-b // 3))
        return c0, max(c1, c0), a - 3 * (c0 // 4)

    def meta(self):
        """A storage-free tensor of this shape and dtype (layout building)."""
        return torch.empty(self.shape, dtype=self.dtype, device='meta')

    def to_tensor(self):
        """Host decode of the storage bytes alone, as the reference's
        param2tensor would return the tensor (same storage, offset, size
        and stride)."""
        es = self.itemsize
        nb = es * self.storage_numel
        if nb:
            raw = _Text(self.text).read_bulk(self.data_pos, nb)
            st = torch.frombuffer(bytearray(raw), dtype=self.dtype)
        else:
            st = torch.empty(0, dtype=self.dtype)
        t = st.as_strided(self.shape, self.stride, self.storage_offset)
        if self.requires_grad:
            t.requires_grad_(True)
        return t


_CACHE = OrderedDict()
_CACHE_MAX = 8192
_PREFIX = 2048
_SUFFIX = 512


def _cache_key(text):
    n = len(text)
    return (type(text), n, bytes(text[:_PREFIX]) if not isinstance(text, str)
            else text[:_PREFIX], bytes(text[-_SUFFIX:])
            if not isinstance(text, str) else text[-_SUFFIX:])


def parse_b64(text):
    """Parse the framing of one b64serializer payload (str or bytes-like)
    without decoding its data; raises FramingError on anything else.  The
    walk runs natively (_fsagg_host.b64_frame, csrc/host/b64frame.cpp,
    ~2 us per key); :func:`parse_b64_py` is the same walk in Python, used
    without the extension."""
    if not isinstance(text, (str, bytes, bytearray, memoryview)):
        raise FramingError('not base64 text: %s' % type(text).__name__)
    ext = _text_ext()
    if ext is None:
        return parse_b64_py(text)
    try:
        cls, shape, stride, off, snumel, pos, rg, nchars = ext.b64_frame(text)
    except ValueError as e:
        msg = str(e)
        raise FramingError(msg[9:] if msg.startswith('framing: ') else msg) \
            from None
    return _fill(B64Tensor(), text, (_STORAGE_DTYPES[cls], shape, stride,
                                     off, snumel, pos, rg, nchars))


def parse_b64_py(text):
    """parse_b64 in Python (framing results cached by the characters the
    walk read)."""
    if not isinstance(text, (str, bytes, bytearray, memoryview)):
        raise FramingError('not base64 text: %s' % type(text).__name__)
    key = _cache_key(text)
    hit = _CACHE.get(key)
    if hit is not None:
        _CACHE.move_to_end(key)
        return _fill(B64Tensor(), text, hit)
    src = _Text(text)
    val, end = _walk(src, 0, src.size, _OUTER_GLOBALS)
    if end != src.size:
        raise FramingError('%d bytes after the pickle' % (src.size - end))
    if not isinstance(val, _TensorRef):
        raise FramingError('the upload is not a tensor')
    dtype, snumel, data_pos = _legacy_storage(src, val.storage.payload)
    if val.offset < 0 or any(s < 0 for s in val.size) or \
            any(s < 0 for s in val.stride):
        raise FramingError('negative offset, size or stride')
    if all(s > 0 for s in val.size):
        last = val.offset + sum((s - 1) * st
                                for s, st in zip(val.size, val.stride))
        if last >= snumel:
            raise FramingError('tensor reaches past its storage (%d >= %d)'
                               % (last, snumel))
    fields = (dtype, tuple(val.size), tuple(val.stride), val.offset, snumel,
              data_pos, val.requires_grad, src.nchars)
    # the framing is a function of the characters the walk decoded: cache
    # it by them when they all lie in the key's prefix and suffix
    if all(4 * (-(-b // 3)) <= _PREFIX or 4 * (a // 3) >= src.nchars - _SUFFIX
           for a, b in src.spans):
        _CACHE[key] = fields
        if len(_CACHE) > _CACHE_MAX:
            _CACHE.popitem(last=False)
    return _fill(B64Tensor(), text, fields)


def _fill(t, text, fields):
    (t.dtype, t.shape, t.stride, t.storage_offset, t.storage_numel,
     t.data_pos, t.requires_grad, t.nchars) = fields
    t.text = text
    return t


def _legacy_storage(src, payload):
    """Walk torch's legacy save stream inside the storage payload; returns
    (dtype, numel, decoded position of element 0)."""
    pos, end = payload.start, payload.start + payload.length
    magic, pos = _walk(src, pos, end, set())
    if magic != _MAGIC:
        raise FramingError('storage payload has no torch magic number')
    proto, pos = _walk(src, pos, end, set())
    if proto != _LEGACY_PROTOCOL:
        raise FramingError('legacy save protocol %r' % (proto, ))
    info, pos = _walk(src, pos, end, set())
    if not isinstance(info, dict) or info.get('little_endian') is not True:
        raise FramingError('storage payload is not little-endian')
    rec, pos = _walk(src, pos, end, {('torch', '*Storage')})
    if not isinstance(rec, _PersId) or not isinstance(rec.pid, tuple) or \
            len(rec.pid) not in (5, 6) or rec.pid[0] != 'storage':
        raise FramingError('storage record is not a persistent id')
    _, cls, skey, _location, numel = rec.pid[:5]
    if len(rec.pid) == 6 and rec.pid[5] is not None:
        raise FramingError('storage views are not supported')
    if not isinstance(cls, _Global) or cls.name not in _STORAGE_DTYPES or \
            not isinstance(skey, str) or not _is_int(numel) or numel < 0:
        raise FramingError('malformed storage record')
    keys, pos = _walk(src, pos, end, set())
    if keys != [skey]:
        raise FramingError('storage key list %r does not match' % (keys, ))
    n = struct.unpack('<q', src.read(pos, 8))[0]
    if pos + 8 > end or n != numel:
        raise FramingError('storage element count %d != %d' % (n, numel))
    dtype = _STORAGE_DTYPES[cls.name]
    es = dtype.itemsize
    if pos + 8 + es * numel != end:
        raise FramingError('storage bytes do not fill the payload')
    return dtype, numel, pos + 8


def decode_b64(text):
    """The host decode (param2tensor's str branch): framing walk, then the
    storage bytes alone."""
    return parse_b64(text).to_tensor()


# -- device staging -----------------------------------------------------------
class B64Stager:
    """Stage base64 uploads into fp32 client-stack rows: the characters of
    each key's storage bytes are copied into one pinned buffer behind the
    segment table (``[segs: nseg × 32 B][text]``), crossing PCIe in ONE DMA,
    and ONE fsagg_b64_unpack_f32 launch decodes them into the row (the
    padding between keys and absent keys become zero segments).  The DMA
    and the launch run on ``stream`` (layout.HostStager owns both and the
    pinned buffers); a device status word collects decode errors and
    :meth:`finish` raises on them."""

    def __init__(self, device, stream):
        device = torch.device(device)
        if device.index is None:
            device = torch.device('cuda', torch.cuda.current_device())
        self.device = device
        self.stream = stream
        # one status word per upload since the last collect(): a rejected
        # upload is reported by its tag (the sender / stack slot), not as a
        # failure of the whole round
        self._status = []
        self.tags = []
        self.puts = 0

    _BLOCK = 256

    def _status_word(self, i):
        b, j = divmod(i, self._BLOCK)
        while len(self._status) <= b:
            with torch.cuda.stream(self.stream):
                self._status.append(torch.zeros(self._BLOCK,
                                                dtype=torch.int32,
                                                device=self.device))
        return self._status[b].data_ptr() + 4 * j

    @staticmethod
    def plan(layout, model):
        """(framings, host_keys) of an upload: the framings of its present
        fp32 keys that are contiguous fp32 base64 tensors of the layout's
        shape (decoded on the device), and the other present keys (decoded
        on the host: param2tensor, which also raises on malformed text)."""
        dev, host = {}, []
        keys = [k for k in layout.keys if k in model]
        texts = [k for k in keys if is_b64(model[k])]
        ext = _text_ext()
        if ext is not None and hasattr(ext, 'b64_frame_many') and texts:
            # every key's walk in one native call, over several threads
            fr = ext.b64_frame_many([model[k] for k in texts])
            parsed = {k: (None if f is None else _fill(
                B64Tensor(), model[k], (_STORAGE_DTYPES[f[0]], ) + f[1:]))
                      for k, f in zip(texts, fr)}
        else:
            parsed = {}
            for k in texts:
                try:
                    parsed[k] = parse_b64(model[k])
                except FramingError:
                    parsed[k] = None
        for k in keys:
            t = parsed.get(k)
            if t is not None and t.dtype == torch.float32 and \
                    tuple(t.shape) == tuple(layout.shapes[k]) and \
                    t.is_contiguous():
                dev[k] = t
            else:
                host.append(k)
        return dev, host

    def put(self, layout, framings, dst_row, pinned, host=None, tag=None):
        """Stage one upload (``framings`` from :meth:`plan`) into
        ``dst_row``; ``pinned(nbytes)`` returns a free pinned uint8 buffer.
        ``host``: {key: value} of the upload's keys :meth:`plan` left to the
        host decode; ``tag`` names the upload in :meth:`collect`'s report.
        Returns the event of the DMA that reads it."""
        host_keys = host or {}
        from ... import _lib as L
        from ...ops import WIRE_SEG_DTYPE, _stream
        import numpy as np
        if dst_row.device != self.device or dst_row.dtype != \
                torch.float32 or not dst_row.is_contiguous() or \
                dst_row.numel() < layout.numel:
            raise ValueError('destination row does not hold the layout')
        segs = []
        chunks = []
        toff = 0
        ends = [layout.offsets[k] for k in layout.keys[1:]] + [layout.numel]
        for k, end in zip(layout.keys, ends):
            o, m = layout.offsets[k], layout.numels[k]
            t = framings.get(k)
            if k in host_keys:
                if end > o + m:
                    segs.append((0, o + m, end - o - m, L.FSAGG_WIRE_ZERO,
                                 -1))
                continue
            if t is None:
                if end > o:
                    segs.append((0, o, end - o, L.FSAGG_WIRE_ZERO, -1))
                continue
            if m:
                c0, c1, skip = t.char_range()
                segs.append((3 * (toff // 4) + skip, o, m,
                             L.FSAGG_WIRE_B64_F32, -1))
                chunks.append((t.text, c0, c1, toff))
                toff += -(-(c1 - c0) // 16) * 16
            if end > o + m:
                segs.append((0, o + m, end - o - m, L.FSAGG_WIRE_ZERO, -1))
        if not segs:
            return None
        if len(segs) > 65535:
            raise ValueError('upload of %d segments' % len(segs))
        sb = -(-32 * len(segs) // 16) * 16
        tb = max(toff, 16)
        total = sb + tb
        buf = pinned(total)
        arr = np.zeros(len(segs), dtype=WIRE_SEG_DTYPE)
        for j, sg in enumerate(segs):
            arr[j] = sg
        buf[:32 * len(segs)].copy_(torch.from_numpy(arr.view(np.uint8)))
        base = buf.data_ptr() + sb
        ext = _text_ext()
        if ext is not None and hasattr(ext, 'text_copy_many'):
            # every key's characters in one call, the bytes split evenly
            # over the threads whatever the key sizes
            ext.text_copy_many(chunks, base)
            chunks = []
        for text, c0, c1, off in chunks:
            if ext is not None:
                ext.text_copy(text, c0, c1, base + off)
            else:
                piece = text[c0:c1]
                if isinstance(piece, str):
                    piece = piece.encode('ascii')
                buf[sb + off:sb + off + (c1 - c0)].copy_(
                    torch.frombuffer(bytearray(piece), dtype=torch.uint8))
        max_len = max(sg[2] for sg in segs)
        with torch.cuda.stream(self.stream):
            dev = torch.empty(total, dtype=torch.uint8, device=self.device)
            dev.copy_(buf[:total], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            L.check(L.load().fsagg_b64_unpack_f32(
                dev.data_ptr() + sb, int(tb), dev.data_ptr(), len(segs),
                int(max_len), dst_row.data_ptr(), int(layout.numel),
                self._status_word(self.puts), _stream(self.device)),
                'fsagg_b64_unpack_f32')
            for k, v in host_keys.items():
                # rare (a non-contiguous or non-fp32 key): decoded on the
                # host, copied as pack_host would (a cast into the row)
                from ..auxiliaries.utils import param2tensor
                o, m = layout.offsets[k], layout.numels[k]
                dst_row[o:o + m].copy_(param2tensor(v).reshape(-1))
        self.puts += 1
        self.tags.append(tag)
        STATS['device_puts'] += 1
        STATS['device_text_bytes'] += toff
        return ev

    _REASON = {1: 'a character outside the base64 alphabet in the tensor '
                  'data',
               2: 'a segment outside the staged text or the row'}

    def collect(self):
        """[(tag, reason)] of the uploads since the last collect that the
        device decode rejected (waits for their decodes); clears them."""
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        if not self.puts:
            return []
        words = torch.cat(self._status).cpu()[:self.puts].tolist()
        # a later put under the same tag (a sender's retry into the same
        # slot, ordered after the failed one on the staging stream) rewrites
        # the whole row: only each tag's latest put decides
        last = {}
        for t, w in zip(self.tags, words):
            last.pop(t, None)
            last[t] = w
        bad = [(t, self._REASON.get(w, 'status %d' % w))
               for t, w in last.items() if w]
        if bad:
            with torch.cuda.stream(self.stream):
                for st in self._status:
                    st.zero_()
        self.puts = 0
        self.tags = []
        return bad

    def finish(self):
        """Order the consumer stream after every decode and raise if one of
        them met a non-base64 character or an out-of-range segment (the
        error's ``rejected`` lists the offending uploads' tags)."""
        bad = self.collect()
        if bad:
            err = FramingError(
                'base64 upload(s) rejected on the device: %s' % '; '.join(
                    '%s: %s' % (t, r) for t, r in bad))
            err.rejected = [t for t, _ in bad]
            raise err


_EXT = []
# uploads decoded on the device and the base64 bytes they sent (tests and
# the bench read these to show which path ran)
STATS = {'device_puts': 0, 'device_text_bytes': 0}


def _text_ext():
    if not _EXT:
        try:
            from ..aggregators._engine import _host_ext
            _EXT.append(_host_ext())
        except ImportError:
            _EXT.append(None)
    return _EXT[0]
