"""get_aggregator (federatedscope/core/auxiliaries/aggregator_builder.py:7-124)
returning the MI355X drop-ins.  Same selection logic; the TensorFlow backend
and the NLP ATC aggregator are outside this engine and raise."""
import logging

logger = logging.getLogger(__name__)

# federatedscope/core/configs/constants.py:11-24
AGGREGATOR_TYPE = {
    "local": "no_communication",
    "global": "no_communication",
    "fedavg": "clients_avg",
    "pfedme": "server_clients_interpolation",
    "ditto": "clients_avg",
    "fedsageplus": "clients_avg",
    "gcflplus": "clients_avg",
    "fedgc": "clients_avg",
    "fedopt": "fedopt",
}


def get_aggregator(method, model=None, device=None, online=False,
                   config=None):
    from federatedscope_amd.core.aggregators import (
        ClientsAvgAggregator, OnlineClientsAvgAggregator,
        ServerClientsInterpolateAggregator, FedOptAggregator,
        NoCommunicationAggregator, AsynClientsAvgAggregator, KrumAggregator,
        MedianAggregator, TrimmedmeanAggregator, BulyanAggregator,
        NormboundingAggregator)

    if getattr(config, 'backend', 'torch') == 'tensorflow':
        raise NotImplementedError('the TensorFlow backend is not served by '
                                  'the MI355X engine')

    STR2AGG = {
        'fedavg': ClientsAvgAggregator,
        'krum': KrumAggregator,
        'median': MedianAggregator,
        'bulyan': BulyanAggregator,
        'trimmedmean': TrimmedmeanAggregator,
        'normbounding': NormboundingAggregator
    }

    if method.lower() in AGGREGATOR_TYPE:
        aggregator_type = AGGREGATOR_TYPE[method.lower()]
    else:
        aggregator_type = "clients_avg"
        logger.warning(
            'Aggregator for method {} is not implemented. Will use default one'
            .format(method))

    data_type = getattr(getattr(config, 'data', None), 'type', '')
    if str(data_type).lower() == 'hetero_nlp_tasks' and \
            not config.federate.atc_vanilla:
        raise NotImplementedError('ATCAggregator is not served by the MI355X '
                                  'engine')

    if config.fedopt.use or aggregator_type == 'fedopt':
        return FedOptAggregator(config=config, model=model, device=device)
    elif aggregator_type == 'clients_avg':
        if online:
            return OnlineClientsAvgAggregator(
                model=model,
                device=device,
                config=config,
                src_device=device
                if config.federate.share_local_model else 'cpu')
        elif config.asyn.use:
            return AsynClientsAvgAggregator(model=model,
                                            device=device,
                                            config=config)
        else:
            if config.aggregator.robust_rule not in STR2AGG:
                logger.warning(
                    f'The specified {config.aggregator.robust_rule} '
                    'aggregtion rule has not been supported, the vanilla '
                    'fedavg algorithm will be used instead.')
            return STR2AGG.get(config.aggregator.robust_rule,
                               ClientsAvgAggregator)(model=model,
                                                     device=device,
                                                     config=config)
    elif aggregator_type == 'server_clients_interpolation':
        return ServerClientsInterpolateAggregator(
            model=model,
            device=device,
            config=config,
            beta=config.personalization.beta)
    elif aggregator_type == 'no_communication':
        return NoCommunicationAggregator(model=model,
                                         device=device,
                                         config=config)
    else:
        raise NotImplementedError(
            "Aggregator {} is not implemented.".format(aggregator_type))
