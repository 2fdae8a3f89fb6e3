from .metric_calculator import calc_blocal_dissim, calc_l2_dissim

__all__ = ['calc_blocal_dissim', 'calc_l2_dissim']
