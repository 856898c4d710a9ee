"""retina_amd -- MI355X-native flow-aggregation engine for Retina's enricher +
advanced-metrics path.  The compute path is ``libgpuagg.so``
(hand-written gfx950 HIP kernels behind the C ABI in ``include/gpuagg.h``)."""

from .engine import ContextOptions, Endpoint, GpuAgg, GpuAggError, HostBatch, RawFeed  # noqa: F401

__all__ = ["ContextOptions", "Endpoint", "GpuAgg", "GpuAggError", "HostBatch", "RawFeed"]
