"""Hot-path ops: hand-written gfx950 HIP kernels with PyTorch reference implementations.

Every op takes and returns plain tensors (outputs may be passed in to reuse static
buffers).  On a GPU tensor the HIP kernel from ``_C.so`` runs; if the extension is not
built the call fails loudly (no silent eager fallback on the GPU).  On CPU tensors the
same math runs in PyTorch (f32) so the explicit-backward models are testable without a
GPU; those CPU versions double as the numerics oracle for the kernel tests.
"""
from .kernels import *  # noqa: F401,F403
from .kernels import ext_available, load_ext  # noqa: F401
