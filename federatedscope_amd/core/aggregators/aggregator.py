"""Aggregator interface (federatedscope/core/aggregators/aggregator.py:6-64)."""
import os
from abc import ABC, abstractmethod

import torch


class Aggregator(ABC):
    """Abstract aggregator: ``aggregate(agg_info) -> state_dict``.

    ``agg_info`` carries ``'client_feedback'`` (list of
    ``(sample_size, model_para)``), ``'recover_fun'`` and ``'staleness'``
    exactly as Server._perform_federated_aggregation builds it
    (federatedscope/core/workers/server.py:479-483)."""
    def __init__(self):
        pass

    @abstractmethod
    def aggregate(self, agg_info):
        pass


class _ModelIO:
    """update / save_model / load_model shared by every drop-in
    (clients_avg_aggregator.py:37-58)."""
    def update(self, model_parameters):
        self.model.load_state_dict(model_parameters, strict=False)

    def save_model(self, path, cur_round=-1):
        assert self.model is not None
        ckpt = {'cur_round': cur_round, 'model': self.model.state_dict()}
        torch.save(ckpt, path)

    def load_model(self, path):
        assert self.model is not None
        if os.path.exists(path):
            ckpt = torch.load(path, map_location=self.device,
                              weights_only=True)
            self.model.load_state_dict(ckpt['model'])
            return ckpt['cur_round']
        raise ValueError("The file {} does NOT exist".format(path))


class NoCommunicationAggregator(_ModelIO, Aggregator):
    """Clients train locally; nothing is aggregated (aggregator.py:24-64)."""
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__()
        self.model = model
        self.device = device
        self.cfg = config

    def aggregate(self, agg_info):
        return {}
