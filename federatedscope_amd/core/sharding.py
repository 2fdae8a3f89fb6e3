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

    The flat bucket is cut into ``chunks`` rounds of ``world`` equal pieces
    (block-cyclic): piece (j, r) = [(j·world + r)·pc, … + pc).  Rank r owns
    pieces (j, r) for every j.  Round j: the rank computes its piece
    straight into its slot of the output, then an asynchronous in-place
    all-gather of round j's ``world`` pieces (contiguous in the output)
    runs on the collective's stream while round j+1 computes.  Pieces are
    disjoint coordinate ranges, so the result is bit-identical to the
    single-GPU reduction; the only traffic is the output itself (4·P bytes,
    ring all-gather over xGMI)."""

    # Pieces below this many coordinates run on two side streams: piece j + 1
    # starts while piece j's last workgroups drain.  One GPU's share of the
    # 100 x 25M model at 8 GPUs (4 pieces of 781k): 0.239 against 0.279 ms;
    # at 4 GPUs (1.56M pieces) one stream is faster (0.400 against 0.425 ms),
    # and larger pieces only compete for the CUs.
    SMALL_PIECE = 1 << 20

    def __init__(self, numel, chunks=4, group=None, align=ALIGN, comm=None,
                 streams=None):
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
        per = self.world * self.chunks
        self.pc = int(math.ceil(self.numel / per / align)) * align \
            if self.numel else align
        self.padded = self.pc * per
        self.streams = int(self._streams) if self._streams is not None else (
            2 if self.chunks > 1 and self.pc < self.SMALL_PIECE else 1)

    def piece(self, j, r=None):
        """Global [lo, hi) of piece (j, r) (empty past numel)."""
        r = self.rank if r is None else r
        lo = (j * self.world + r) * self.pc
        return min(lo, self.numel), min(lo + self.pc, self.numel)

    def local_pieces(self):
        return [self.piece(j) for j in range(self.chunks)]

    def local_numel(self):
        """Columns of this rank's client slab: its pieces back to back, each
        ``pc`` wide (so every piece starts 256-B aligned)."""
        return self.chunks * self.pc

    def run(self, compute, out=None, dtype=torch.float32, device=None):
        """compute(j, lo, hi, out_view) writes piece (j, rank) = global
        coordinates [lo, hi) into ``out_view`` (hi − lo elements).  Returns
        the assembled [numel] result (every rank)."""
        if out is None:
            out = torch.empty(self.padded, dtype=dtype, device=device)
        if out.numel() < self.padded:
            raise ValueError('out needs %d elements (padded), got %d' %
                             (self.padded, out.numel()))
        works = []
        W, pc = self.world, self.pc
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
            slot = (j * W + self.rank) * pc
            with (torch.cuda.stream(side[j % len(side)]) if side
                  else _nullctx()):
                if hi > lo:
                    compute(j, lo, hi, out[slot:slot + (hi - lo)])
                if W > 1:
                    # the collective waits for the piece's own stream
                    w = self.comm.all_gather_into(
                        out[j * W * pc:(j + 1) * W * pc],
                        out[slot:slot + pc], async_op=True)
                    if w is not None:
                        works.append(w)
        if side:
            for st in side:
                cur.wait_stream(st)
        for w in works:
            w.wait()
        return out[:self.numel]
