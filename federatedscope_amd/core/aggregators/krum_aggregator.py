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

The matrix (≤ 200² floats) comes back to the host where the score/sort/select
logic runs with the same torch CPU ops as the reference (:75-87); the
selected clients are then averaged in ascending-score order with init + avg
fused into the kernel (fsagg_weighted_sum_rows_f32).
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
