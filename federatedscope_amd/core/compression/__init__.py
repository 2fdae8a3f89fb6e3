from .utils import symmetric_uniform_dequantization
from .wire import QuantPlan, WireStager

__all__ = ['symmetric_uniform_dequantization', 'QuantPlan', 'WireStager']
