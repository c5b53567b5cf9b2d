"""shadow_amd -- MI355X-native engine for Shadow's routing build and per-round packet relay.

The product path is the native library ``libshd_accel.so`` (hand-written gfx950 HIP kernels
behind the C ABI in ``include/shd_accel.h``); this package is its Python host layer:
``routing`` (NetworkGraph / RoutingInfo mirror), ``relay`` (send_packet batched per round),
``synth`` (synthetic workloads of BASELINE.json's configs) and ``dist`` (multi-GPU sharding
over torch.distributed / RCCL).
"""
from ._native import ShdError  # noqa: F401

__all__ = ["ShdError"]
