"""mipipe: an MI355X-native pipeline-parallel training engine.

Same capabilities as the reference ``aa5490/Distributed-Training-with-Pipeline-Parallelism``
(GPipe / 1F1B / Interleaved-1F1B pipeline schedules, manual layer splitting,
throughput benchmarking), re-designed for AMD MI355X (gfx950): hand-written
CDNA4 HIP kernels for the transformer hot path, RCCL point-to-point over xGMI
between pipeline stages, explicit per-layer backward with a static activation
stash, and DP x PP gradient all-reduce overlapped with the pipeline flush.
"""
__version__ = "0.1.0"

from . import parallel  # noqa: F401
