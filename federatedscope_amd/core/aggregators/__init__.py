"""MI355X drop-ins for federatedscope.core.aggregators (same names, same
constructor signatures and aggregate(agg_info) contract)."""
from .aggregator import Aggregator, NoCommunicationAggregator
from .clients_avg_aggregator import ClientsAvgAggregator, \
    OnlineClientsAvgAggregator
from .asyn_clients_avg_aggregator import AsynClientsAvgAggregator
from .server_clients_interpolate_aggregator import \
    ServerClientsInterpolateAggregator
from .fedopt_aggregator import FedOptAggregator
from .krum_aggregator import KrumAggregator
from .median_aggregator import MedianAggregator
from .trimmedmean_aggregator import TrimmedmeanAggregator
from .bulyan_aggregator import BulyanAggregator
from .normbounding_aggregator import NormboundingAggregator

__all__ = [
    'Aggregator',
    'NoCommunicationAggregator',
    'ClientsAvgAggregator',
    'OnlineClientsAvgAggregator',
    'AsynClientsAvgAggregator',
    'ServerClientsInterpolateAggregator',
    'FedOptAggregator',
    'KrumAggregator',
    'MedianAggregator',
    'TrimmedmeanAggregator',
    'BulyanAggregator',
    'NormboundingAggregator',
]
