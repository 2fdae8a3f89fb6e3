"""Device plumbing shared by the drop-in aggregators.

Every aggregator in this package runs its reduction on an MI355X through
libfsagg (federatedscope_amd/ops.py).  This mixin owns:

* the compute device (a GPU — there is no CPU path: without one the
  aggregators raise instead of silently computing elsewhere);
* cached bucket layouts and the persistent device client stack (reused
  across rounds; sized for HBM, grown on demand);
* the general weighted-average driver that mirrors
  ClientsAvgAggregator._para_weighted_avg (clients_avg_aggregator.py:60-100)
  including its per-key "skip missing client" rule and dtype rules;
* conversion of the flat device result back to a state_dict on the device
  the client updates came from (host dicts in → host dicts out, as the
  reference's CPU aggregators return).
"""
from collections import OrderedDict

import torch

from ... import ops
from ...layout import BucketLayout, ClientStack
from ..auxiliaries.utils import (as_float_tensor, as_float_upload,
                                 param2tensor, param_meta)


# the peer assembly's flag-barrier bound on the aggregate() path when
# aggregator.shard_peer_timeout_s is unset (torch.distributed's default
# process-group timeout is 10 min for RCCL)
PEER_TIMEOUT_DEFAULT_S = 300.0


def compute_device(device=None):
    if not torch.cuda.is_available():
        raise RuntimeError(
            'federatedscope_amd aggregators run on an AMD GPU (libfsagg); no '
            'GPU is visible and there is no CPU fallback')
    if device is not None:
        d = torch.device(device)
        if d.type == 'cuda':
            return torch.device('cuda', d.index if d.index is not None else
                                torch.cuda.current_device())
    return torch.device('cuda', torch.cuda.current_device())


def fedavg_weights(sizes, ignore_weight=False, use_ss=False):
    """The reference's per-client weights, as Python doubles
    (clients_avg_aggregator.py:64-84)."""
    total = 0
    for s in sizes:
        total += s
    n = len(sizes)
    if ignore_weight:
        return [1.0 / n] * n
    if use_ss:
        return [1.0] * n
    return [s / total for s in sizes]


def _first_device(model):
    for v in model.values():
        if isinstance(v, torch.Tensor):
            return v.device
    return torch.device('cpu')


class StagedSet:
    """The client list of one aggregate() call as row sets.  Unsharded: one
    piece, the whole bucket, whose row set is a slot of a ClientStack
    (staged uploads) or the clients' own device tensors (read in place).
    Sharded by parameter range: this rank's pieces of the
    bucket, each (j, lo, hi, rows), plus the PipelinedAssembly ``plan``
    that all-gathers the pieces of every rank."""

    def __init__(self, layout, rs=None, stack=None, slots=None, pieces=None,
                 plan=None):
        self.layout = layout
        self.rs = rs
        self.stack = stack
        self.slots = slots
        self.plan = plan
        self.pieces = pieces if pieces is not None else \
            [(0, 0, layout.numel, rs)]
        self.n = self.pieces[0][3].n

    def rows(self, sel=None):
        """The clients ``sel`` (indices into the client list, in reduction
        order; default all) as one RowSet over the whole bucket."""
        if self.plan is not None or self.rs is None:
            raise RuntimeError('a sharded client set has per-piece rows')
        return self.rs if sel is None else self.rs.subset(sel)

    def subset(self, sel):
        """The clients ``sel`` in the new reduction order (every piece)."""
        rs = None if self.rs is None else self.rs.subset(sel)
        pieces = [(j, lo, hi, rs if r is self.rs else r.subset(sel))
                  for j, lo, hi, r in self.pieces]
        return StagedSet(self.layout, rs, pieces=pieces, plan=self.plan)


class DeviceEngine:
    """Mixin: call ``_engine_init(device)`` from the constructor."""

    def _engine_init(self, device=None):
        self._dev_req = device
        self._dev = None
        self._layouts = {}
        self._fast_layouts = {}
        self._stacks = {}
        self._plans = {}

    # -- parameter-range sharding across the ranks of a process group --------
    def _shard(self):
        """(Comm, chunks) when the config asks for the aggregation to be
        sharded by parameter range over the default process group
        (``aggregator.shard_by_param_range``, pipelined over
        ``aggregator.shard_chunks`` rounds) and that group has > 1 rank;
        else None.  Every rank then calls aggregate() with the same client
        list (SPMD) and receives the full result."""
        agg = getattr(getattr(self, 'cfg', None), 'aggregator', None)
        if not getattr(agg, 'shard_by_param_range', False):
            return None
        import torch.distributed as dist
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return None
        from ..sharding import Comm
        comm = self.__dict__.get('_comm')
        if comm is None:
            comm = self._comm = Comm()
        return comm, int(getattr(agg, 'shard_chunks', 2) or 1)

    def _plan(self, layout, comm, chunks):
        """The assembly of a sharded call, cached per layout.
        ``aggregator.shard_assembly``: 'auto' (default) — the peer assembly
        (each rank's kernel stores its piece into every GPU's copy over
        xGMI, then a flag barrier: core/sharding.PeerAssembly), or, when the
        ranks agree it cannot be set up (a GPU that cannot reach a peer, no
        IPC), the pipelined all-gathers; 'p2p' — the peer assembly or an
        error; 'rccl' — the pipelined all-gathers.
        ``aggregator.shard_result_views`` (default False): the peer
        assembly returns views of its rotating output copies (three) instead
        of a fresh copy, and checks each round's barrier status at the next
        call — the result must be consumed (e.g. the server's
        load_state_dict, server.py:482-483) before the next-but-one
        aggregate() on this aggregator."""
        from ..sharding import PeerAssembly, PipelinedAssembly
        agg = getattr(getattr(self, 'cfg', None), 'aggregator', None)
        mode = str(getattr(agg, 'shard_assembly', 'auto') or 'auto')
        if mode not in ('auto', 'p2p', 'rccl'):
            raise ValueError("aggregator.shard_assembly must be 'auto', "
                             "'p2p' or 'rccl', got %r" % mode)
        views = bool(getattr(agg, 'shard_result_views', False))
        key = (layout.signature(), chunks, mode, views)
        pa = self._plans.get(key)
        if pa is not None:
            return pa
        if mode != 'rccl':
            # no collective precedes the flag barrier on this path, so any
            # host-side skew between the ranks (uneven staging, gRPC ingest
            # on one rank before it calls aggregate()) counts against the
            # bound: by default it is on the order of a process group's
            # timeout, not the bench's 10 s
            tmo = getattr(agg, 'shard_peer_timeout_s', None)
            if tmo is None:
                tmo = PEER_TIMEOUT_DEFAULT_S
            try:
                # collective: every rank takes the same branch (the
                # constructor agrees on success or failure across ranks)
                pa = PeerAssembly(
                    layout.numel, comm=comm, device=self.compute_device,
                    timeout_s=tmo, buffers=3 if views else 2)
            except Exception:  # noqa: BLE001 (agreed by every rank)
                if mode == 'p2p':
                    raise
                pa = None
        if pa is None:
            pa = PipelinedAssembly(layout.numel, chunks=chunks, comm=comm)
        self._plans[key] = pa
        return pa

    def _run_pieces(self, st, fn, bcast=None):
        """Flat result bucket on the compute device from fn(rows, out, lo,
        hi) over the set's pieces; sharded, every rank ends up holding the
        whole bucket: the peer assembly stores each rank's piece into every
        GPU's copy (``bcast(rows, out, peers, lo, hi)`` — a kernel whose
        epilogue does that itself, returning False when it has no such form
        — or fn followed by a push), the pipelined assembly all-gathers the
        pieces (the gather of round j overlapping round j+1).  Coordinates
        are bucket coordinates."""
        from ..sharding import PeerAssembly
        dev = self.compute_device
        if st.plan is None:
            out = torch.empty(st.layout.numel, dtype=torch.float32,
                              device=dev)
            for _, lo, hi, rs in st.pieces:
                fn(rs, out, lo, hi)
            return out
        if isinstance(st.plan, PeerAssembly):
            rows = st.pieces[0][3]

            def compute(lo, hi, own, peers):
                if bcast is not None and bcast(rows, own, peers, lo, hi):
                    return True
                fn(rows, own, lo, hi)
                return False
            agg = getattr(getattr(self, 'cfg', None), 'aggregator', None)
            return st.plan.run_bucket(compute, copy=not getattr(
                agg, 'shard_result_views', False))
        out = torch.empty(st.plan.padded, dtype=torch.float32, device=dev)
        rows = {j: rs for j, _, _, rs in st.pieces}
        st.plan.run(lambda j, lo, hi, view: fn(rows[j], out, lo, hi),
                    out=out)
        return out

    def _sum_pieces(self, st, fn):
        """Σ over this rank's pieces of fn(rows, lo, hi), summed across the
        ranks when sharded (the exchange Krum and norm bounding need)."""
        acc = None
        for _, lo, hi, rs in st.pieces:
            if hi <= lo and acc is not None:
                continue
            v = fn(rs, lo, max(hi, lo))
            acc = v if acc is None else acc.add_(v)
        if st.plan is not None:
            st.plan.comm.all_reduce_sum(acc)
        return acc

    def _pairdist(self, st):
        """Krum's distance matrix D (fp32 [n][n]) of a client set, as a
        pending result whose ``.cpu()`` waits for it.  Up to 256 clients: on
        the matrix cores (fsagg_pairgram_*: the Gram of the rows centred on a
        central client, fp32 split exactly into bf16 limbs), every pair with
        a worst-case bound on its error (``last_pair_bound``, host fp64
        [n][n]) that the callers certify their selection with
        (:meth:`_certified_order`); non-finite pairs are recomputed on the
        VALU kernel.  Above 256 clients: the VALU kernel (direct differences,
        ``last_pair_bound`` None)."""
        from ... import _lib
        self._pair_info = None
        if not 2 <= st.n <= _lib.FSAGG_PAIRGRAM_MAX_CLIENTS:
            return self._pairdist_valu(st)
        if st.plan is None:
            # one graph launch for the chain's eight kernels (ops._GRAPHS)
            rs = st.rows()
            buf = ops.pairgram_rows_dist_graph(rs, _GRAM_TOL)[0]
            return _PendingD(self, st, buf=buf,
                             tab=rs.__dict__.get('_gram_tab'))
        sq2 = self._sum_pieces(
            st, lambda rs, lo, hi: ops.pairgram_rows_segsq(rs, lo, hi))
        return _PendingD(self, st, buf=ops.pairgram_finish(sq2, _GRAM_TOL)[0])

    def _pairdist_valu(self, st):
        """D on the VALU kernel (fsagg_pairdist_*)."""
        self.last_pairdist_path = 'valu'
        self._pair_info = None
        segsq = self._sum_pieces(
            st, lambda rs, lo, hi: ops.pairdist_rows_segsq(rs, lo, hi))
        return _PendingD(self, st, D=ops.pairdist_finish(segsq))

    @property
    def last_pair_bound(self):
        """Host fp64 [n][n] bounds on the last Gram-path D's error (None
        after the VALU path)."""
        info = self.__dict__.get('_pair_info')
        return None if info is None else info.bound()

    @property
    def last_pair_cert(self):
        """(D64, B64) of the last Gram-path D: what selections are
        certified with (None after the VALU path)."""
        info = self.__dict__.get('_pair_info')
        return None if info is None else info.cert()

    def _certified_order(self, st, D, f, m, ordered):
        """(D, scores, order) for a Krum selection of ``m`` clients: from the
        Gram path's fp64 sums when their bounds certify the selection
        (:func:`certified_selection`, natively in
        ``_fsagg_host.gram_select`` when no pair was recomputed;
        ``ordered``: the order of the first ``m`` as well, which fixes a
        multi-Krum average's summation order); else with the ambiguous
        clients' rows recomputed in fp64 (:meth:`_refine_selection`); else
        from D recomputed on the VALU kernel."""
        import numpy as np
        from ... import _lib
        from .krum_aggregator import krum_scores
        info = self.__dict__.get('_pair_info')
        if info is None:
            scores = krum_scores(D, f)
            return D, scores, torch.sort(scores)[1]
        amb = None
        if info.raw:
            got = _lib.host().gram_select(info.host.numpy(), info.nseg, f, m,
                                          bool(ordered))
            if got is not None:
                sc, order, amb = got
                if not amb:
                    return D, torch.frombuffer(sc, dtype=torch.float64), \
                        torch.frombuffer(order, dtype=torch.int64)
        D64, B64 = info.cert()
        if amb is None:
            n = D64.shape[0]
            k = n - f - 2
            sc = np.sort(D64, 1)[:, :max(k, 0)].sum(1)
            order = np.argsort(sc, kind='stable')
            amb = ambiguous_clients(D64, B64, f, m, order, ordered)
            if amb is not None and not amb:
                return D, torch.from_numpy(sc), torch.from_numpy(order)
        got = self._refine_selection(st, D64, B64, f, m, ordered, amb)
        if got is not None:
            sc, o, nrows = got
            self.last_pairdist_path = 'mfma + exact rows %d of %d' % (
                nrows, st.n)
            return D, torch.from_numpy(sc), torch.from_numpy(o)
        D = self._pairdist_valu(st).cpu()
        self.last_pairdist_path = 'mfma, not certified: valu'
        scores = krum_scores(D, f)
        order = torch.sort(scores)[1]
        return D, scores, order

    def _refine_selection(self, st, D, B, f, m, ordered, amb):
        """:func:`refine_selection` with the ambiguous clients' rows from
        the fp64 kernel (fsagg_pairsel_*, summed across ranks when
        sharded); None when the client count is outside its range."""
        from ... import _lib
        if st.n > _lib.FSAGG_PAIRSEL_MAX_CLIENTS:
            return None
        nseg = max(1, len(st.layout.keys))
        big = max([st.layout.numels[key] for key in st.layout.keys] or [1])
        world = st.plan.comm.world if st.plan is not None else 1
        # fp64 differences and squares, sums of at most `big` terms per key
        # (+ slices, chunks and ranks), a sqrt and nseg adds per pair
        rel = ((big + 64 + world) / 2 + nseg + 8) * 2.0 ** -53
        # the rows kernel costs ~ n·rows, the full VALU matrix ~ n²/2: at
        # 50 × 6.6M, 8 rows 0.45 ms against 0.47 ms (tools/probe_pairsel.py)
        max_rows = min(_lib.FSAGG_PAIRSEL_MAX_SEL, max(4, st.n // 6))
        return refine_selection(D, B, f, m, ordered, amb,
                                lambda sel: self._exact_rows(st, sel), rel,
                                max_rows)

    def _exact_rows(self, st, sel):
        """fp64 host [len(sel)][n]: the selected clients' rows of D in fp64
        (summed across ranks when sharded)."""
        import numpy as np
        dev = self.compute_device
        sel_t = torch.from_numpy(np.asarray(sel, dtype=np.int32)).to(dev)
        sq = self._sum_pieces(
            st, lambda rs, lo, hi: ops.pairsel_rows_segsq(rs, sel_t, lo, hi))
        return ops.pairsel_finish(sq, sel_t).cpu().numpy()

    def _sqnorms(self, st):
        """[n][nseg] fp64 per-client, per-key squared norms."""
        return self._sum_pieces(
            st, lambda rs, lo, hi: ops.rows_sqnorm(rs, lo, hi))

    @property
    def compute_device(self):
        if self._dev is None:
            self._dev = compute_device(self._dev_req)
        return self._dev

    # -- layouts and stacks -------------------------------------------------
    def _layout(self, template, as_float=False):
        if as_float:
            template = OrderedDict(
                (k, _as_float_proto(v)) for k, v in template.items())
        sig = tuple((k, tuple(t.shape), t.dtype) for k, t in (
            (k, param_meta(v)) for k, v in template.items()))
        lay = self._layouts.get(sig)
        if lay is None:
            lay = BucketLayout(template)
            self._layouts[sig] = lay
        return lay

    def _stack(self, layout, models, as_float=False):
        """Pack the fp32 keys of each client dict into a device row."""
        key = layout.signature()
        st = self._stacks.get(key)
        if st is None or st.capacity < len(models):
            st = ClientStack(layout, max(len(models), 1), self.compute_device)
            st.slab.zero_()
            self._stacks[key] = st
        if as_float:
            models = [OrderedDict((k, as_float_upload(v))
                                  for k, v in m.items()) for m in models]
        st.load_many(models)
        return st

    def _bucket(self, layout, model, as_float=False):
        """A single model (e.g. the server's init model) as a device bucket;
        every layout key must be present."""
        flat = torch.zeros(layout.numel, dtype=torch.float32,
                           device=self.compute_device)
        src = OrderedDict()
        for k in layout.keys:
            if k not in model:
                raise KeyError(k)
            v = param2tensor(model[k])
            src[k] = as_float_tensor(v) if as_float else v
        layout.pack_device(src, flat)
        return flat

    def _key_table(self, layout, dicts, virtual=False):
        """(ptrs [n][nseg], aligned16, missing) when every present layout
        key of every dict is a contiguous fp32 tensor of the layout's shape
        on the compute device (the C++ walk of csrc/host/keytable.cpp), else
        None.  ``virtual``: the device row table instead — [nseg][n]
        virtual bases (ptr − 4·offset, 0 where absent)."""
        import numpy as np
        from ... import _lib
        dev = self.compute_device
        kl = layout.__dict__.get('_key_list')
        if kl is None:
            kl = layout.__dict__['_key_list'] = (
                list(layout.keys), [layout.shapes[k] for k in layout.keys],
                [4 * layout.offsets[k] for k in layout.keys])
        if not kl[0]:
            return None
        host = _host_ext()
        if host is None:      # no _fsagg_host.so: stage the dicts instead
            return None
        if virtual:
            res = host.key_table(dicts, kl[0], kl[1], dev.index, kl[2])
        else:
            res = host.key_table(dicts, kl[0], kl[1], dev.index)
        if res is None:
            return None
        raw, missing, aligned = res[:3]
        shape = (len(kl[0]), len(dicts)) if virtual else (len(dicts),
                                                            len(kl[0]))
        tab = np.frombuffer(raw, dtype=np.int64).reshape(shape)
        if virtual:
            return tab, aligned, missing, bool(res[3])
        return tab, aligned, missing

    def _base(self, layout, model, as_float=False):
        """The server model as the kernels' ``base`` operand: its own device
        tensors when they are fp32 on the compute device (no copy), else a
        packed device bucket."""
        if isinstance(model, dict):
            kt = self._key_table(layout, [model])
            if kt is not None and kt[1] and \
                    not ops.absent(layout, kt[0]).any():
                return ops.BaseRows.from_pointers(layout, kt[0][0],
                                                  self.compute_device,
                                                  keepalive=(model, ),
                                                  ephemeral=True)
        return ops.BaseRows.from_bucket(self._bucket(layout, model,
                                                     as_float=as_float))

    # -- result emission -----------------------------------------------------
    @staticmethod
    def _emit(layout, flat, keys, out_device, extra=None):
        """Views of ``flat`` per key, on ``out_device`` (one copy)."""
        if out_device.type != 'cuda' or out_device != flat.device:
            flat = flat.to(out_device)
        views = layout.unpack(flat)
        out = OrderedDict()
        for k in keys:
            if extra is not None and k in extra:
                out[k] = extra[k].to(out_device)
            elif k in views:
                out[k] = views[k]
        return out

    # -- the FedAvg core ----------------------------------------------------
    def _weighted_avg_device(self, models, weights, as_float=False,
                             base_model=None, prescale=None, staged=None):
        """Weighted average with the reference's per-key semantics.

        Returns (layout, flat fp32 bucket on the GPU, {non-fp32 key: tensor},
        key order).  ``models`` is the client_feedback list of
        (sample_size, dict); ``weights`` the per-client Python doubles.
        Keys some clients lack are reduced over the clients that have them,
        weights NOT renormalised (clients_avg_aggregator.py:74-75): their
        row-set entries are NULL and the kernel skips them."""
        dicts = [m for _, m in models]
        template = dicts[0]
        n = len(dicts)
        st = staged if staged is not None else self._staged(
            models, as_float=as_float)
        layout = st.layout
        base = None
        if base_model is not None:
            base = self._base(layout, base_model, as_float=as_float)
        out = self._run_pieces(
            st, lambda rs, o, lo, hi: ops.weighted_sum_rows(
                rs, weights, o, prescale=prescale, base=base, lo=lo, hi=hi),
            bcast=lambda rs, o, peers, lo, hi: ops.weighted_sum_rows_bcast(
                rs, weights, o, peers, prescale=prescale, base=base, lo=lo,
                hi=hi))
        extra = OrderedDict()
        for k, dt in layout.other.items():
            have = [i for i in range(n) if k in dicts[i]]
            ts = [param2tensor(dicts[i][k]).to(self.compute_device)
                  .contiguous() for i in have]
            o = torch.empty(ts[0].shape, dtype=ops.typed_out_dtype(dt),
                            device=self.compute_device)
            ops.weighted_sum_typed(ts, [weights[i] for i in have], o)
            if base_model is not None:
                raise NotImplementedError(
                    'init + update for non-fp32 key %r' % k)
            extra[k] = o
        return layout, out, extra, list(template.keys())

    def _staged(self, models, as_float=False, require_all=False):
        """The client list as row sets (sharded by parameter range when the
        config asks for it, see :meth:`_shard`)."""
        sh = self._shard()
        st = self._staged_rows(models, as_float, require_all,
                               whole=sh is None)
        if sh is None:
            return st
        comm, chunks = sh
        plan = self._plan(st.layout, comm, chunks)
        spans = plan.local_pieces()
        if st.rs is not None:          # whole-bucket rows: restrict
            pieces = [(j, lo, hi, st.rs) for j, (lo, hi) in enumerate(spans)]
            return StagedSet(st.layout, st.rs, pieces=pieces, plan=plan)
        # host (or foreign-device) dicts: stage this rank's pieces only
        from ...layout import RangeStack
        dicts = [m for _, m in models]
        if as_float:
            dicts = [OrderedDict((k, as_float_tensor(v))
                                 for k, v in m.items()) for m in dicts]
        # the spans differ between assemblies (one piece per rank for the
        # peer assembly, ``chunks`` for the pipelined one)
        key = ('range', st.layout.signature(), tuple(spans))
        rst = self._stacks.get(key)
        if rst is None or rst.capacity < len(dicts):
            rst = RangeStack(st.layout, spans, len(dicts),
                             self.compute_device)
            self._stacks[key] = rst
        rst.load_many(dicts)
        present = st.slots          # the presence matrix (see below)
        pieces = [(j, lo, hi, ops.RowSet.from_stack(
            rst, range(len(dicts)), present=present, offset=rst.offset(j),
            ephemeral=True)) for j, (lo, hi) in enumerate(spans)]
        return StagedSet(st.layout, pieces=pieces, plan=plan)

    def _staged_rows(self, models, as_float=False, require_all=False,
                     whole=True):
        """The client list as one row set: slots DeviceIngress staged on
        arrival, the clients' own device tensors read in place, or (host
        dicts, other devices, other dtypes) rows of a device stack.  With
        ``whole=False`` the stack is not built: the StagedSet then carries
        only the layout and, in ``slots``, the key-presence matrix."""
        from ..workers.ingress import StagedUpdate
        dicts = [m for _, m in models]
        # every staged slot must have landed before anything reads it, on
        # every path below (a list can mix staged uploads with stale ones
        # that were buffered as plain dicts).  type() identity, not
        # isinstance: StagedUpdate is a Mapping, whose ABC isinstance check
        # costs ~0.5 us per dict
        staged = [d for d in dicts if type(d) is StagedUpdate]
        for ing in {id(d.ingress): d.ingress for d in staged}.values():
            ing.sync()
        if staged and len(staged) == len(dicts):
            ing = dicts[0].ingress
            # keys of other dtypes (typed side copies) are reduced per key
            # by _weighted_avg_device; the robust rules cast every key to
            # float and take the general path below
            if all(d.ingress is ing for d in dicts) and \
                    (not ing.layout.other or not as_float):
                if require_all:
                    for i, d in enumerate(dicts):
                        if len(d) != len(ing.layout.keys):
                            raise KeyError('client %d lacks keys' % i)
                slots = [d.slot for d in dicts]
                return StagedSet(ing.layout, ops.RowSet.from_stack(
                    ing.stack, slots, ephemeral=True), ing.stack, slots)
        # device-resident fp32 dicts: read in place through a key table
        d0 = dicts[0]
        fk = (tuple(d0.keys()), bool(as_float))
        layout = self._fast_layouts.get(fk)
        if layout is None:
            layout = self._layout(d0, as_float=as_float)
            self._fast_layouts[fk] = layout
        if not layout.other:
            kt = self._key_table(layout, dicts, virtual=True)
            if kt is not None and kt[1]:
                virt, _, nmiss, uniform = kt
                gone = 0
                if nmiss:        # absent keys (an empty key never counts)
                    absent = ops.absent(layout, virt.T)
                    if require_all and absent.any():
                        i, s = [int(x[0]) for x in absent.nonzero()]
                        raise KeyError('client %d lacks key %r' %
                                       (i, layout.keys[s]))
                    gone = int(absent.sum())
                return StagedSet(layout, ops.RowSet.from_virtual(
                    layout, virt, self.compute_device, keepalive=(dicts, ),
                    missing=gone, uniform=uniform, ephemeral=True))
        # staged through a device stack
        layout = self._layout(d0, as_float=as_float)
        present = [[k in d for k in layout.keys] for d in dicts]
        if require_all:
            for i, row in enumerate(present):
                for k, ok in zip(layout.keys, row):
                    if not ok:
                        raise KeyError('client %d lacks key %r' % (i, k))
        if not whole:
            return StagedSet(layout, slots=present,
                             pieces=[(0, 0, 0, _NoRows(len(dicts)))])
        stack = self._stack(layout, dicts, as_float=as_float)
        slots = list(range(len(dicts)))
        return StagedSet(layout, ops.RowSet.from_stack(stack, slots,
                                                       present=present,
                                                       ephemeral=True),
                         stack, slots)

    def _stage_all(self, models, as_float=True):
        """Pack every client (robust rules need all keys in all clients)."""
        return self._staged(models, as_float=as_float, require_all=True)


_HOST = []


def _host_ext():
    """The _fsagg_host extension, or None when it was not built (looked up
    once): the key-table fast path is then skipped and client dicts are
    staged through a device stack — the kernels themselves still need
    libfsagg.so."""
    if not _HOST:
        from ... import _lib
        try:
            _HOST.append(_lib.host())
        except (_lib.FsaggError, ImportError, OSError):
            _HOST.append(None)
    return _HOST[0]


# fsagg_pairgram_finish_f32's flagging threshold: +inf, only non-finite
# pairs are recomputed pair by pair — the Krum selection is certified with the
# per-pair bounds instead
_GRAM_TOL = float('inf')


def certified_selection(D, B, f, m, order, ordered=True):
    """Whether the Krum selection of the first ``m`` clients of ``order`` is
    the one exact distances give, from D (host fp32 [n][n]) and per-pair
    bounds B on |D − the exact distances' sum| (host fp64, D's own fp32
    formation included).  Krum's score, the sum of a client's n − f − 2
    smallest distances, is monotone in every distance: the exact score lies
    in [lo, hi], the same sums over D − B and D + B.  The selected set holds
    when the largest hi among the first m is below the smallest lo after
    them; with ``ordered`` (a multi-Krum average sums its clients in that
    order) every position i < m must clear every client after it."""
    amb = ambiguous_clients(D, B, f, m, order, ordered)
    return amb is not None and not amb


def ambiguous_clients(D, B, f, m, order, ordered=True):
    """The clients whose score intervals keep :func:`certified_selection`
    from holding — an empty list when it holds; None when no interval
    argument applies (no distances in a score: n − f − 2 <= 0).  Unordered: the first m whose hi reaches the smallest lo
    after them, and the others whose lo reaches the largest hi among the
    first m.  Ordered: every position i < m whose hi reaches a lo after it,
    with the clients after it whose lo it reaches."""
    import numpy as np
    D = np.asarray(D, dtype=np.float64)
    n = D.shape[0]
    k = n - f - 2
    if k <= 0:
        return None
    if m <= 0:
        return []
    B = np.asarray(B, dtype=np.float64)
    lo = np.sort(np.maximum(D - B, 0.0), 1)[:, :k].sum(1) * (1 - 1e-12)
    hi = np.sort(D + B, 1)[:, :k].sum(1) * (1 + 1e-12)
    o = np.asarray(order)
    lo_o, hi_o = lo[o], hi[o]
    if m >= n:
        if not ordered:
            return []
        m = n - 1
    suf = np.minimum.accumulate(lo_o[::-1])[::-1]
    amb = set()
    if not ordered:
        top = hi_o[:m].max()
        if top < suf[m]:
            return []
        amb.update(o[:m][hi_o[:m] >= suf[m]].tolist())
        amb.update(o[m:][lo_o[m:] <= top].tolist())
        return sorted(amb)
    for i in range(m):
        if hi_o[i] >= suf[i + 1]:
            amb.add(int(o[i]))
            amb.update(o[i + 1:][lo_o[i + 1:] <= hi_o[i]].tolist())
    return sorted(amb)


def refine_selection(D, B, f, m, ordered, amb, exact_rows, rel, max_rows):
    """A Krum selection from D (host [n][n]: the Gram path's fp64 sums) and
    its bounds B with the ambiguous clients' rows recomputed: ``exact_rows(sel)`` returns their
    rows of D (fp64 host [len(sel)][n], +inf at their own column) within
    ``rel``·D of the exact distances.  Those clients' scores — sums over
    their own rows — become near points, the others keep their intervals
    (their entries against the recomputed clients tightened too).  Two
    rounds at most (a round's points may overlap clients the first left
    alone), at most ``max_rows`` rows in all.  Returns (fp64 scores, order,
    rows recomputed), or None when the selection stays uncertified or a
    recomputed distance is not finite (the caller recomputes all of D)."""
    import numpy as np
    n = D.shape[0]
    k = n - f - 2
    if amb is None or k <= 0:
        return None
    Dx = np.asarray(D, dtype=np.float64).copy()
    Bx = np.asarray(B, dtype=np.float64).copy()
    done = set()
    for _ in range(2):
        new = sorted(set(int(i) for i in amb) - done)
        if not new or len(done) + len(new) > max_rows:
            return None
        rows = np.asarray(exact_rows(new), dtype=np.float64)
        own = np.zeros(rows.shape, dtype=bool)
        own[np.arange(len(new)), new] = True
        if not np.isfinite(rows[~own]).all():
            return None
        Dx[new, :] = rows
        Dx[:, new] = rows.T
        bnd = rel * np.where(own, 0.0, rows)
        Bx[new, :] = bnd
        Bx[:, new] = bnd.T
        done.update(new)
        sc = np.sort(Dx, 1)[:, :k].sum(1)
        order = np.argsort(sc, kind='stable')
        amb = ambiguous_clients(Dx, Bx, f, m, order, ordered)
        if amb is None:
            return None
        if not amb:
            return sc, order, len(done)
    return None


class _PairInfo:
    """The Gram path's per-pair data behind the last distance matrix, on
    the host, built on demand from the finish buffer's host copy
    (ops._gram_buf): ``cert()`` = (D64, B64), the fp64 key sums and the
    kernel's bounds on them — what the selection is certified with (D's
    fp32 rounding, about half of the full bound on i.i.d. data, is no part
    of the exact distances); ``bound()`` = the bounds on the fp32 D (B64
    plus D's own fp32 formation).  ``raw``: no pair was recomputed, so the
    native certificate (_fsagg_host.gram_select) reads the buffer as is."""

    def __init__(self, host, nseg, cert=None, bound=None):
        self.host, self.nseg = host, nseg
        self._cert, self._bound = cert, bound
        self.raw = cert is None

    def cert(self):
        if self._cert is None:
            import numpy as np
            _, _, Bf, D64 = ops.gram_views(self.host)
            D64 = D64.numpy().copy()
            Bf = Bf.numpy().astype(np.float64)
            # D64's own fp64 sum over the keys (relative 2^-53 per add)
            self._cert = (D64, np.maximum(Bf, Bf.T) + (self.nseg + 2) *
                          2.0 ** -52 * np.where(np.isfinite(D64), D64, 0.0))
        return self._cert

    def bound(self):
        if self._bound is None:
            import numpy as np
            D = ops.gram_views(self.host)[0].numpy().astype(np.float64)
            # D is the fp32 formation of the fp64 per-key distances (a
            # rounded sqrt and an fp32 add per key)
            self._bound = self.cert()[1] + (2 * self.nseg + 2) * \
                2.0 ** -24 * np.where(np.isfinite(D), D, 0.0)
        return self._bound


class _PendingD:
    """Krum's distance matrix while its kernels run (``_pairdist``):
    ``cpu()`` copies D (and the Gram path's flags, bounds and fp64 sums) to
    the host, recomputes the flagged (non-finite) pairs exactly and returns
    the host fp32 [n][n] matrix; the per-pair data go to the engine's
    ``_pair_info`` (:class:`_PairInfo`: ``last_pair_bound``,
    ``last_pair_cert``)."""

    def __init__(self, eng, st, buf=None, D=None, tab=None):
        self._eng, self._st, self._buf, self._D = eng, st, buf, D
        # the Gram chain's device copy of the row table (ops.krum_select)
        self._tab = tab

    def cpu(self):
        if self._D is not None:
            return self._D.cpu()
        import numpy as np
        eng, st = self._eng, self._st
        host = self._buf.cpu()
        nseg = max(1, len(st.layout.keys))
        D, flags, _, _ = ops.gram_views(host)
        eng.last_pairdist_path = 'mfma'
        flags = flags.numpy()
        if not flags.any():
            eng._pair_info = _PairInfo(host, nseg)
            return D
        info = _PairInfo(host, nseg)
        D64, B64 = (a.copy() for a in info.cert())
        B = info.bound().copy()
        D = D.clone()
        flags = (flags + flags.T) > 0
        # the flagged pairs exactly: the VALU kernel over the clients
        # involved (every pair among them)
        sel = sorted(set(np.nonzero(flags)[0].tolist()))
        exact = eng._sum_pieces(
            st.subset(sel), lambda rs, lo, hi: ops.pairdist_rows_segsq(
                rs, lo, hi))
        sub = ops.pairdist_finish(exact).cpu()
        idx = torch.tensor(sel)
        D[idx[:, None], idx[None, :]] = sub
        # the VALU kernel's sums: every fp32 per-chunk partial adds at most
        # m = chunk + 256 non-negative terms (a k-slice's squares, then the
        # slices), relative error <= (1 + u)^m − 1; the fp64 chunk sums add
        # (chunks + 64)·2^-53 more (counted as 64·u); sqrt maps a relative
        # δ to <= δ / (2(1 − δ)); then D's own fp32 formation (a rounded
        # sqrt and an fp32 add per key)
        import math
        u = 2.0 ** -24
        ext = max([hi - lo for _, lo, hi, _ in st.pieces] + [1])
        chl = int(ops.L.load().fsagg_pairdist_chunk_elems(len(sel), ext,
                                                           nseg))
        acc = math.expm1((chl + 256) * math.log1p(u)) + 64 * u
        rel = acc / (2.0 * (1.0 - acc)) if acc < 1.0 else math.inf
        s = sub.numpy().astype(np.float64)
        fin = np.where(np.isfinite(s), s, 0.0)
        form = (rel + (2 * nseg + 2) * u) * fin
        B[np.ix_(sel, sel)] = form
        D64[np.ix_(sel, sel)] = s
        B64[np.ix_(sel, sel)] = form
        eng.last_pairdist_path = 'mfma + exact %d of %d clients' % (
            len(sel), st.n)
        eng._pair_info = _PairInfo(host, nseg, cert=(D64, B64), bound=B)
        return D


class _NoRows:
    """Placeholder rows of a not-yet-staged client set (client count)."""

    def __init__(self, n):
        self.n = n


def _as_float_proto(v):
    t = param_meta(v)
    if not isinstance(t, torch.Tensor):
        import numpy as np
        t = torch.as_tensor(np.asarray(t))
    if t.dtype != torch.float32:
        return torch.empty(t.shape, dtype=torch.float32)
    return t
