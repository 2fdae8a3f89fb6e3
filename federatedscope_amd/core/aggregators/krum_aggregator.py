"""Krum / multi-Krum (federatedscope/core/aggregators/krum_aggregator.py:6-90).

Device path: the client updates are read where they lie (a row set: the
clients' own device tensors, or their staged stack rows).  The n×n distance
matrix (the per-key L2 distances summed over keys, +inf diagonal, :58-73):

* up to 256 clients on the matrix cores (fsagg_pairgram_rows_f32: the Gram of
  the rows centred on a central client, fp32 split exactly into three bf16
  limbs, fp64 accumulation), with a worst-case error bound per pair — the
  selection below is certified against those bounds, and recomputed from
  the VALU kernel's matrix when the score gaps do not clear them
  (_engine._certified_order);
* above 256 clients on the VALU kernel (fsagg_pairdist_rows_segsq_f32 +
  fsagg_pairdist_finish_f64: direct differences).

On the Gram path the scores, their stable order and the selection's
certificate are computed on the device from the fp64 key sums and their
bounds (fsagg_krum_select_f32), which also writes the selected clients' row
table and weights; their average (init + avg fused, ascending-score order,
fsagg_weighted_sum_rows_f32) is launched right behind it and the host reads
back one flag and the order.  An uncertified selection, and the VALU path,
take the host route: the matrix comes back, the certificate runs natively
(or the ambiguous rows are recomputed, :75-87), then the average.
"""
import torch

from ... import ops
from ._engine import _first_device, fedavg_weights
from .clients_avg_aggregator import ClientsAvgAggregator


def krum_scores(D, byzantine_node_num):
    """_calculate_score's tail (krum_aggregator.py:75-77), on the host."""
    model_num = D.shape[0]
    closest_num = model_num - byzantine_node_num - 2
    sorted_distance = torch.sort(D)[0]
    return torch.sum(sorted_distance[:, :closest_num], axis=-1)


class KrumAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)
        self.byzantine_node_num = config.aggregator.byzantine_node_num
        self.krum_agg_num = config.aggregator.BFT_args.krum_agg_num
        assert 2 * self.byzantine_node_num + 2 < config.federate.client_num, \
            "it should be satisfied that 2*byzantine_node_num + 2 < client_num"

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        out_dev = _first_device(models[0][1])
        layout, flat, keys = self._krum_device(models, self.krum_agg_num)
        return self._emit(layout, flat, keys, out_dev)

    def distance_matrix(self, models):
        """D (host fp32 [n, n]) as _calculate_score fills it (:58-73)."""
        st = self._stage_all(models)
        return self._pairdist(st).cpu(), st

    def _calculate_score(self, models):
        D, _ = self.distance_matrix([(0, m) for m in models])
        return krum_scores(D, self.byzantine_node_num)

    def _krum_device(self, models, agg_num):
        st = self._stage_all(models)
        layout = st.layout
        D = self._pairdist(st)
        # host work that does not need the selection runs while the
        # distance kernels do (the .cpu() below waits for them)
        base = self._base(layout, self.model.state_dict(), as_float=True)
        out = self._select_on_device(st, D, models, agg_num, base)
        if out is not None:
            return layout, out, list(models[0][1].keys())
        _, _, index_order = self._certified_order(
            st, D.cpu(), self.byzantine_node_num, agg_num, ordered=True)
        sel = [int(i) for i in index_order[:agg_num]]
        self.last_selection = sel
        sizes = [models[i][0] for i in sel]
        weights = fedavg_weights(sizes, self.cfg.federate.ignore_weight)
        out = self._run_pieces(
            st.subset(sel), lambda rs, o, lo, hi: ops.weighted_sum_rows(
                rs, weights, o, base=base, lo=lo, hi=hi),
            bcast=lambda rs, o, peers, lo, hi: ops.weighted_sum_rows_bcast(
                rs, weights, o, peers, base=base, lo=lo, hi=hi))
        return layout, out, list(models[0][1].keys())

    def _select_on_device(self, st, D, models, agg_num, base):
        """The multi-Krum average with its selection certified on the
        device (ops.krum_select: the scores, order and certificate of
        _certified_order's native path, from the Gram finish buffer) and the
        selected clients' average launched right behind it — the host reads
        back one flag and the order instead of the n x n buffer, and
        certifies, gathers and uploads nothing in between.  None (nothing
        launched that the caller needs) when the path does not apply or the
        selection is not certified: the host path then runs as before."""
        import numbers

        import numpy as np
        from ... import _lib
        from ._engine import _PairInfo
        tab = getattr(D, '_tab', None)
        buf = getattr(D, '_buf', None)
        n = st.n
        if tab is None or buf is None or st.plan is not None or \
                n > _lib.FSAGG_KRUMSEL_MAX_CLIENTS or agg_num < 1:
            return None
        sizes = []
        for s, _ in models:
            if isinstance(s, bool) or not isinstance(s, numbers.Real):
                return None
            v = float(s)
            # fedavg_weights' Python arithmetic, exactly, in fp64
            if not np.isfinite(v) or v != s or v <= 0.0 or abs(v) >= 2**53:
                return None
            sizes.append(v)
        layout = st.layout
        nseg = max(1, len(layout.keys))
        rs = st.rows()
        bh = None
        if base is not None:
            if base.host is None or nseg > _lib.FSAGG_KRUMSEL_MAX_SEGS:
                return None
            bh = list(base.host) if base.bss else [base.host[0]] * nseg
        msel = min(int(agg_num), n)
        sel, sub_tab, sub_w, sub_base = ops.krum_select(
            buf, nseg, self.byzantine_node_num, agg_num, True, sizes,
            self.cfg.federate.ignore_weight, tab, rs.ss,
            nseg if rs.ss else 1, bh)
        # the flag, order and finish buffer go to the host on a side stream
        # while the average runs on this one
        dev = self.compute_device
        cur = torch.cuda.current_stream(dev)
        side = self.__dict__.get('_ksel_stream')
        if side is None or side.device != dev:
            side = self._ksel_stream = torch.cuda.Stream(device=dev)
        pins = self.__dict__.setdefault('_ksel_pinned', {})
        hb = pins.get(n)
        if hb is None:
            hb = pins[n] = (torch.empty(2 + n, dtype=torch.int32,
                                        pin_memory=True),
                            torch.empty(tuple(buf.shape), dtype=torch.int32,
                                        pin_memory=True))
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            hb[0].copy_(sel, non_blocking=True)
            hb[1].copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        sel.record_stream(side)
        out = torch.empty(layout.numel, dtype=torch.float32, device=dev)
        ops.weighted_sum_rows_devtab(layout, sub_tab, msel if rs.ss else 0,
                                     msel, sub_w, out, base=sub_base)
        ev.synchronize()
        got = hb[0].numpy()
        if not got[0]:
            return None
        self.last_selection = [int(i) for i in got[2:2 + msel]]
        self.last_pairdist_path = 'mfma'
        self._pair_info = _PairInfo(hb[1].clone(), nseg)
        return out
