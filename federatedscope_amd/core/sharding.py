"""Parameter-range sharding of the aggregation across the GPUs of one node.

SURVEY §8(e): FedAvg, median, trimmed mean and the robust rules' init + update
are per-coordinate, so GPU g owns the parameter range [lo_g, hi_g) of the
flat bucket, holds the [n × (hi_g − lo_g)] slice of every client and runs the
full client loop over it — no arithmetic crosses GPUs, so the result stays
bit-identical to the single-GPU (and the reference's) order.  The only
exchanges are:

* Krum / Bulyan: per-key squared pair distances are partial sums over each
  rank's range → one all-reduce(SUM) of an [nseg][n][n] fp64 tensor
  (≤ 12·50²·8 B = 240 KB at C4) before the distance matrix is finished;
* optionally assembling the full aggregated model on every rank: an
  all-gather of the disjoint output shards (a concatenation, not a reduce).

Backend-agnostic: the collectives are plain torch.distributed calls, RCCL
("nccl") over xGMI on the GPU node, gloo in the CPU tests.
"""
import contextlib
import ctypes
import math

import torch
import torch.distributed as dist

from .. import ops

ALIGN = 64  # elements (256 B): shard boundaries keep rows 16-B aligned
_nullctx = contextlib.nullcontext


def shard_ranges(numel, world, align=ALIGN):
    """Contiguous, aligned, near-equal [lo, hi) ranges covering [0, numel)."""
    if world < 1:
        raise ValueError('world must be >= 1')
    per = int(math.ceil(numel / world / align)) * align if numel else 0
    return [(min(r * per, numel), min((r + 1) * per, numel))
            for r in range(world)]


def local_segments(seg_offsets, lo, hi):
    """Global per-key offsets [0, .., numel] clipped to [lo, hi) and made
    local (same number of segments; segments outside the range are empty)."""
    return [min(max(int(o), lo), hi) - lo for o in seg_offsets]


class Comm:
    """The sharded path's two collectives over a torch.distributed group.

    On RCCL ("nccl", xGMI) device tensors go to the collective directly.
    The gloo backend (CPU tests, two ranks sharing one GPU in the GPU
    tests) takes host tensors: device operands are staged through host
    memory and the call completes synchronously."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() \
            else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.backend = dist.get_backend(group) if dist.is_initialized() \
            else None
        self.host_staged = self.backend == 'gloo'

    def all_gather_into(self, out, inp, async_op=False):
        """out = cat of every rank's ``inp`` (equal sizes), in rank order.
        Returns a work handle when asynchronous, else None."""
        if self.world == 1:
            out.copy_(inp)
            return None
        if not (self.host_staged and inp.device.type == 'cuda'):
            return dist.all_gather_into_tensor(out, inp, group=self.group,
                                               async_op=async_op)
        ci = inp.detach().cpu()
        parts = [torch.empty_like(ci) for _ in range(self.world)]
        dist.all_gather(parts, ci, group=self.group)
        out.copy_(torch.cat(parts))
        return None

    def all_gather_bytes(self, b):
        """Every rank's ``b`` (small host bytes: IPC handles), rank order."""
        if self.world == 1:
            return [bytes(b)]
        out = [None] * self.world
        dist.all_gather_object(out, bytes(b), group=self.group)
        return out

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def all_reduce_sum(self, t):
        if self.world == 1:
            return t
        if self.host_staged and t.device.type == 'cuda':
            c = t.detach().cpu()
            dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


def assemble(shard, ranges, numel=None, group=None):
    """All-gather disjoint output shards into the full vector (every rank)."""
    world = dist.get_world_size(group)
    if len(ranges) != world:
        raise ValueError('%d ranges for world %d' % (len(ranges), world))
    numel = ranges[-1][1] if numel is None else numel
    maxlen = max(hi - lo for lo, hi in ranges)
    padded = torch.zeros(maxlen, dtype=shard.dtype, device=shard.device)
    padded[:shard.numel()] = shard
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    out = torch.empty(numel, dtype=shard.dtype, device=shard.device)
    for (lo, hi), p in zip(ranges, parts):
        out[lo:hi] = p[:hi - lo]
    return out


def allreduce_segsq(segsq, group=None):
    """Sum the ranks' per-key squared pair distances (Krum's one exchange)."""
    dist.all_reduce(segsq, op=dist.ReduceOp.SUM, group=group)
    return segsq


class ShardedAggregation:
    """Rank-local driver over this rank's parameter range.

    ``rows`` arguments are RowTables over this rank's slice of every client
    (numel = hi − lo); ``seg_offsets`` are the GLOBAL per-key offsets of the
    full bucket (BucketLayout.segments())."""

    def __init__(self, numel, seg_offsets=None, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() \
            else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.numel = numel
        self.ranges = shard_ranges(numel, self.world)
        self.lo, self.hi = self.ranges[self.rank]
        self.seg_offsets = seg_offsets

    def fedavg(self, rows, weights, out_shard, base_shard=None):
        return ops.weighted_sum(rows, weights, out_shard, base=base_shard)

    def median(self, rows, out_shard, base_shard=None):
        return ops.coord_median(rows, out_shard, base=base_shard)

    def trimmed_mean(self, rows, k, out_shard, divisor=None,
                     base_shard=None):
        return ops.trimmed_mean(rows, k, out_shard, divisor=divisor,
                                base=base_shard)

    def krum_distance(self, rows):
        """The full n×n Krum matrix from this rank's rows (all-reduce of the
        per-key partials when world > 1)."""
        offs = local_segments(self.seg_offsets, self.lo, self.hi)
        segsq = ops.pairdist_segsq(rows, offs)
        if self.world > 1:
            allreduce_segsq(segsq, self.group)
        return ops.pairdist_finish(segsq)

    def gather(self, out_shard):
        if self.world == 1:
            return out_shard
        return assemble(out_shard, self.ranges, self.numel, self.group)


class PipelinedAssembly:
    """Strong-scaled aggregation whose full result is assembled on every
    rank, the gather overlapped with the compute.

    The flat bucket is cut into ``chunks`` rounds (block-cyclic); round j
    holds ``world`` equal pieces of ``pcs[j]`` coordinates, contiguous in
    the output: piece (j, r) = [off[j] + r·pcs[j], … + pcs[j]).  Rank r owns
    pieces (j, r) for every j.  Round j: the rank computes its piece
    straight into its slot of the output, then an asynchronous in-place
    all-gather of round j's ``world`` pieces runs on the collective's stream
    while round j+1 computes.  Pieces are disjoint coordinate ranges, so the
    result is bit-identical to the single-GPU reduction; the only traffic is
    the output itself (4·P bytes over xGMI).

    ``split`` sets the rounds' relative sizes (default: equal).  Only the
    last round's gather is exposed, so a plan that shrinks toward its end
    (e.g. :func:`tapered_split`) exposes less of it while the early, large
    pieces run at the one-launch rate."""

    # Pieces below this many coordinates run on two side streams: piece j + 1
    # starts while piece j's last workgroups drain.  One GPU's share of the
    # 100 x 25M model at 8 GPUs (4 pieces of 781k): 0.239 against 0.279 ms;
    # at 4 GPUs (1.56M pieces) one stream is faster (0.400 against 0.425 ms),
    # and larger pieces only compete for the CUs.
    SMALL_PIECE = 1 << 20

    def __init__(self, numel, chunks=4, group=None, align=ALIGN, comm=None,
                 streams=None, split=None):
        if split is not None:
            split = [float(f) for f in split]
            if not split or min(split) <= 0:
                raise ValueError('split needs positive round weights')
            chunks = len(split)
        if chunks < 1:
            raise ValueError('chunks must be >= 1')
        if streams is not None and streams < 1:
            raise ValueError('streams must be >= 1')
        self._streams = streams       # None: by piece size (SMALL_PIECE)
        self._side = {}
        self.comm = comm if comm is not None else Comm(group)
        self.group = self.comm.group
        self.world = self.comm.world
        self.rank = self.comm.rank
        self.numel = int(numel)
        self.chunks = int(chunks)
        self.pcs = _round_lengths(self.numel, self.world, self.chunks,
                                  split, align)
        self.off = [0]
        for pc in self.pcs:
            self.off.append(self.off[-1] + self.world * pc)
        self.padded = self.off[-1]
        self.pc = max(self.pcs)
        self.streams = int(self._streams) if self._streams is not None else (
            2 if self.chunks > 1 and min(self.pcs) < self.SMALL_PIECE else 1)

    def piece(self, j, r=None):
        """Global [lo, hi) of piece (j, r) (empty past numel)."""
        r = self.rank if r is None else r
        lo = self.off[j] + r * self.pcs[j]
        return min(lo, self.numel), min(lo + self.pcs[j], self.numel)

    def slot(self, j, r=None):
        """Offset of piece (j, r) in the padded output."""
        r = self.rank if r is None else r
        return self.off[j] + r * self.pcs[j]

    def local_pieces(self):
        return [self.piece(j) for j in range(self.chunks)]

    def local_numel(self):
        """Columns of this rank's client slab: its pieces back to back, each
        ``pcs[j]`` wide (so every piece starts 256-B aligned)."""
        return sum(self.pcs)

    def check(self):
        """Nothing to verify (the collectives report their own errors)."""

    def run(self, compute, out=None, dtype=torch.float32, device=None):
        """compute(j, lo, hi, out_view) writes piece (j, rank) = global
        coordinates [lo, hi) into ``out_view`` (hi − lo elements).  Returns
        the assembled [numel] result (every rank).

        Stream order: each piece runs on its side stream (or the current
        one), which first waits for the current stream; the collective of
        round j is issued under the piece's stream, so the backend orders it
        after the piece (RCCL: its stream waits on the issuing stream); at
        the end the current stream waits for every side stream and every
        collective's work handle."""
        if out is None:
            out = torch.empty(self.padded, dtype=dtype, device=device)
        if out.numel() < self.padded:
            raise ValueError('out needs %d elements (padded), got %d' %
                             (self.padded, out.numel()))
        works = []
        W = self.world
        side = None
        if self.streams > 1 and self.chunks > 1 and out.is_cuda:
            side = self._side.get(out.device)
            if side is None:
                side = self._side[out.device] = [
                    torch.cuda.Stream(out.device)
                    for _ in range(self.streams)]
            cur = torch.cuda.current_stream(out.device)
            for st in side:
                st.wait_stream(cur)
        for j in range(self.chunks):
            lo, hi = self.piece(j)
            slot, pc = self.slot(j), self.pcs[j]
            with (torch.cuda.stream(side[j % len(side)]) if side
                  else _nullctx()):
                if hi > lo:
                    compute(j, lo, hi, out[slot:slot + (hi - lo)])
                if W > 1:
                    # the collective waits for the piece's own stream
                    w = self.comm.all_gather_into(
                        out[self.off[j]:self.off[j + 1]],
                        out[slot:slot + pc], async_op=True)
                    if w is not None:
                        works.append(w)
        if side:
            for st in side:
                cur.wait_stream(st)
        for w in works:
            w.wait()
        return out[:self.numel]


def tapered_split(chunks, ratio=0.5):
    """Round weights that shrink geometrically (1, r, r², …): the early
    rounds run at the one-launch rate, the exposed last gather is small."""
    return [ratio ** j for j in range(chunks)]


def _round_lengths(numel, world, chunks, split, align):
    """Per-round piece lengths (aligned) covering ``numel`` coordinates in
    ``chunks`` rounds of ``world`` pieces, in proportion to ``split``; the
    last round takes the remainder (never negative, at least ``align``)."""
    if split is None:
        per = world * chunks
        pc = int(math.ceil(numel / per / align)) * align if numel else align
        return [pc] * chunks
    tot = sum(split)
    pcs = []
    done = 0
    for j in range(chunks - 1):
        want = numel * split[j] / tot / world
        pc = max(int(math.ceil(want / align)) * align, align)
        pcs.append(pc)
        done += world * pc
    rest = max(numel - done, 0)
    pcs.append(max(int(math.ceil(rest / world / align)) * align, align))
    return pcs


class PeerAssembly:
    """Strong-scaled aggregation assembled by the producing kernel itself
    (DESIGN §7).

    Rank r owns piece r = [r·pc, (r+1)·pc) of the bucket, reduces it in ONE
    launch and stores each output tile into every rank's copy of the
    result: its own buffer and the peers' buffers, imported through IPC
    handles and written over xGMI (ops.weighted_sum_bcast).  A flag barrier
    on the same stream (fsagg_peer_barrier) then waits until every peer's
    stores have landed.  No collective library call and no separate gather
    pass: the 4·P output bytes cross the links while the 4·n·P input bytes
    stream from HBM, every GPU pushing to all of its peers at once.

    The output copies are double-buffered (round k writes buffer k mod 2): a
    rank can be one round ahead, and the barrier of round k + 1 proves that
    every rank has finished round k — so a rank never writes into a buffer a
    peer is still reading.  A result of :meth:`run` is valid until this
    rank's next :meth:`run`, and only for reads enqueued on the stream
    before it: once this rank reaches barrier k + 1, a peer may start round
    k + 2 and store into the buffer of round k.  :meth:`run_bucket` (the
    Aggregator.aggregate() path) copies the assembled bucket out before it
    returns.

    Uploads stay where they are: each rank reads only its range of every
    client (device-resident, as in the reference's multi-GPU mode where
    uploads arrive on the ranks' GPUs, parallel_runner.py:243-302)."""

    TIMEOUT_S = 10.0       # a lost peer ends the barrier with an error
    CTRL_WORDS = 64        # flag words [0, world)

    def __init__(self, numel, comm=None, device=None, align=ALIGN,
                 group=None, buffers=2, timeout_s=None):
        from .. import _lib as L
        if timeout_s is not None:
            self.TIMEOUT_S = float(timeout_s)
        self.comm = comm if comm is not None else Comm(group)
        self.world = self.comm.world
        self.rank = self.comm.rank
        if self.world > L.FSAGG_MAX_PEERS:
            raise ValueError('peer assembly supports up to %d GPUs' %
                             L.FSAGG_MAX_PEERS)
        self.device = torch.device(device) if device is not None else \
            torch.device('cuda', torch.cuda.current_device())
        self.numel = int(numel)
        W = self.world
        self.pc = max(int(math.ceil(self.numel / W / align)) * align, align)
        self.padded = W * self.pc
        self.epoch = 0
        self._lib = L.load()
        self._L = L
        idx = self.device.index
        self._own = []
        self._opened = []
        # Every rank runs every exchange, whatever failed locally, and the
        # ranks agree at the end: all of them use the peer copies or none
        # does (a rank that gave up alone would leave the others waiting in
        # a collective or at the flag barrier).
        err = None
        hb = int(self._lib.fsagg_peer_handle_bytes())
        bus = ctypes.create_string_buffer(64)
        try:
            nbytes = self.padded * 4
            for _ in range(buffers):
                self._own.append(self._alloc(nbytes))
            self._own.append(self._alloc(self.CTRL_WORDS * 4))
            self._L.check(self._lib.fsagg_peer_pci_bus_id(idx, bus, 64),
                          'fsagg_peer_pci_bus_id')
        except Exception as e:          # noqa: BLE001 (agreed on below)
            err = e
        buses = self.comm.all_gather_bytes(bus.value if err is None else b'')
        mine = b''
        if err is None:
            try:
                for k, b in enumerate(buses):
                    if not b:
                        raise RuntimeError('rank %d has no peer buffers' % k)
                    ok = self._lib.fsagg_peer_can_access(idx, b)
                    if ok < 0:
                        self._L.check(ok, 'fsagg_peer_can_access')
                    if ok == 0:
                        raise RuntimeError('GPU %s cannot access rank %d\'s '
                                           'GPU %s' % (bus.value.decode(), k,
                                                       b.decode()))
                mine = b''.join(self._handle(p, hb) for p in self._own)
            except Exception as e:      # noqa: BLE001
                err = e
        every = self.comm.all_gather_bytes(mine)
        # ptr[k] = rank k's allocations (buffers..., ctrl) as seen here
        self._ptr = []
        if err is None:
            try:
                for k in range(W):
                    if k == self.rank:
                        self._ptr.append(list(self._own))
                        continue
                    if len(every[k]) != len(mine):
                        raise RuntimeError('rank %d sent %d handle bytes, '
                                           'expected %d' % (k, len(every[k]),
                                                            len(mine)))
                    row = []
                    for a in range(len(self._own)):
                        p = self._open(every[k][a * hb:(a + 1) * hb])
                        self._opened.append(p)
                        row.append(p)
                    self._ptr.append(row)
            except Exception as e:      # noqa: BLE001
                err = e
        verdicts = self.comm.all_gather_bytes(b'1' if err is None else b'0')
        if err is not None or b'0' in verdicts:
            self._release()
            if err is not None:
                raise err
            raise RuntimeError('peer assembly unavailable on rank(s) %s' %
                               [k for k, v in enumerate(verdicts)
                                if v == b'0'])
        host = L.host()
        self.buffers = [host.device_tensor(p, self.padded, 0, idx)
                        for p in self._own[:-1]]
        self.ctrl = host.device_tensor(self._own[-1], self.CTRL_WORDS, 1,
                                       idx)
        self._flags = (ctypes.c_void_p * W)(
            *[self._ptr[k][-1] for k in range(W)])
        # the barrier's status word lives in mapped pinned host memory: the
        # host reads it once the barrier has run (an event), with no
        # device-to-host copy on the stream
        hs, ds = ctypes.c_void_p(), ctypes.c_void_p()
        self._L.check(self._lib.fsagg_peer_status_alloc(ctypes.byref(hs),
                                                        ctypes.byref(ds)),
                      'fsagg_peer_status_alloc')
        self._st_host, self._st_dev = int(hs.value), int(ds.value)
        self._status = ctypes.c_uint32.from_address(self._st_host)
        self._done = ctypes.c_uint32.from_address(self._st_host + 4)
        self._pending = None       # a views-mode round not yet checked

    # -- allocation plumbing ------------------------------------------------
    def _alloc(self, nbytes):
        p = ctypes.c_void_p()
        self._L.check(self._lib.fsagg_peer_alloc(self.device.index, nbytes,
                                                 ctypes.byref(p)),
                      'fsagg_peer_alloc')
        return int(p.value)

    def _handle(self, ptr, hb):
        buf = ctypes.create_string_buffer(hb)
        self._L.check(self._lib.fsagg_peer_handle(ptr, buf),
                      'fsagg_peer_handle')
        return buf.raw

    def _open(self, handle):
        p = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(handle, len(handle))
        self._L.check(self._lib.fsagg_peer_open(self.device.index, buf,
                                                ctypes.byref(p)),
                      'fsagg_peer_open')
        return int(p.value)

    def _release(self):
        if getattr(self, '_st_host', None):
            self._lib.fsagg_peer_status_free(self._st_host)
            self._st_host = None
        for p in self._opened:
            self._lib.fsagg_peer_close(self.device.index, p)
        for p in self._own:
            self._lib.fsagg_peer_free(self.device.index, p)
        self._opened, self._own = [], []

    # -- the round ------------------------------------------------------------
    def piece(self, r=None):
        """Global [lo, hi) of rank r's piece (empty past numel)."""
        r = self.rank if r is None else r
        lo = r * self.pc
        return min(lo, self.numel), min(lo + self.pc, self.numel)

    def local_pieces(self):
        """This rank's pieces of the bucket (one), as PipelinedAssembly."""
        return [self.piece()]

    def run(self, compute):
        """compute(lo, hi, outs) launches, on the current stream, the
        reduction of this rank's piece [lo, hi) into every address of
        ``outs`` (own buffer first, then the peers'; hi − lo floats each).
        Returns this GPU's assembled [numel] result (valid until the next
        run(), see the class docstring)."""
        b = self.epoch % len(self.buffers)
        self.epoch += 1
        lo, hi = self.piece()
        W = self.world
        if hi > lo:
            outs = [self._ptr[(self.rank + k) % W][b] + 4 * lo
                    for k in range(W)]
            compute(lo, hi, outs)
        self._barrier()
        return self.buffers[b][:self.numel]

    def run_bucket(self, compute, copy=True):
        """The Aggregator.aggregate() form.  ``compute(lo, hi, own, peers)``
        reduces this rank's piece [lo, hi) of the bucket into ``own`` (this
        GPU's copy, a [padded] fp32 tensor in bucket coordinates) on the
        current stream; ``peers`` are the device addresses of the other
        GPUs' copies (same coordinates).  It returns True when its kernel
        stored the piece into the peers' copies itself (the fused broadcast
        epilogue of FedAvg), else the piece is pushed to them here
        (fsagg_peer_push_f32).

        ``copy`` (default): after the flag barrier the assembled bucket is
        copied into a fresh tensor the caller owns, and the barrier's status
        is checked before returning (raises if a peer never arrived).
        ``copy=False``: the result is a view of this round's copy, valid for
        work enqueued on the current stream before this rank's next-but-one
        run_bucket (a peer writes that copy again only in round epoch +
        len(buffers), which it starts after this rank's barrier of round
        epoch + len(buffers) − 1); nothing waits here — the round's status
        is checked at the end of the next run_bucket (after its launches)
        or by :meth:`check`."""
        from .. import ops
        b = self.epoch % len(self.buffers)
        self.epoch += 1
        lo, hi = self.piece()
        W = self.world
        own = self.buffers[b]
        peers = [self._ptr[(self.rank + k) % W][b] for k in range(1, W)]
        if hi > lo:
            if not compute(lo, hi, own, peers) and peers:
                ops.peer_push(own.data_ptr() + 4 * lo,
                              [p + 4 * lo for p in peers], hi - lo,
                              self.device)
        self._barrier()
        if copy:
            res = torch.empty(self.numel, dtype=torch.float32,
                              device=self.device)
            res.copy_(own[:self.numel])
            self.check()
            return res
        prev, self._pending = self._pending, self.epoch
        if prev is not None:
            self._wait_done(prev)
            self._raise_status()
        else:
            # no earlier round to wait for: still read the status word (a
            # non-blocking load of pinned memory) so that a failure already
            # reported is raised here, not one round later
            self._raise_status()
        return own[:self.numel]

    def _barrier(self):
        ticks = int(self.TIMEOUT_S * 1e8)
        self._L.check(self._lib.fsagg_peer_barrier(
            self._flags, self.world, self.rank, self.epoch & 0xFFFFFFFF,
            ticks, self._st_dev, ops._stream(self.device)),
            'fsagg_peer_barrier')
        self._issued = self.epoch

    def _wait_done(self, epoch):
        """Spin until the barrier of ``epoch`` has run (its status[1] word
        in pinned host memory), bounded by the barrier's own timeout plus a
        margin for the work queued before it."""
        import time
        want = epoch & 0xFFFFFFFF
        if ((self._done.value - want) & 0xFFFFFFFF) < 0x80000000:
            return
        t0 = time.perf_counter()
        limit = self.TIMEOUT_S + 60.0
        spins = 0
        while ((self._done.value - want) & 0xFFFFFFFF) >= 0x80000000:
            spins += 1
            if spins & 0xFFF:
                continue        # a plain spin first: a sleep costs ~60 us
            t = time.perf_counter() - t0
            if t > limit:
                raise RuntimeError('peer barrier of round %d never ran' %
                                   epoch)
            if t > 0.05:
                time.sleep(1e-4)

    def _raise_status(self):
        v = int(self._status.value)
        if v:
            self._status.value = 0
            raise RuntimeError('peer barrier timed out waiting for rank %d'
                               % (v - 1))

    def check(self):
        """Raise if a barrier gave up waiting for a peer (waits for this
        rank's last barrier).  The status word is cleared before raising: a
        peer that arrives late runs the round it missed against flags that
        are already up, and the ranks' epochs meet again at the next round,
        which then succeeds (the plan stays cached — rebuilding it would be
        a collective the late peer is not in)."""
        if getattr(self, '_issued', None) is not None:
            self._wait_done(self._issued)
        self._pending = None
        self._raise_status()

    def close(self):
        """Collective: unmap the peers' buffers and free this rank's."""
        if not self._own:
            return
        torch.cuda.synchronize(self.device)
        self.comm.barrier()
        self.buffers, self.ctrl = [], None
        self._release()
        self.comm.barrier()
