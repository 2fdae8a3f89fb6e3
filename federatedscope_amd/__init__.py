"""federatedscope_amd — MI355X-native server-side aggregation engine.

Drop-in replacements for federatedscope.core.aggregators (FedAvg, async,
online, Krum/multi-Krum, median, trimmed mean, Bulyan, norm bounding,
server/client interpolation) whose reductions run as hand-written HIP
kernels for gfx950 (libfsagg.so, C ABI in include/fsagg.h).
"""
__version__ = '0.1.0'
