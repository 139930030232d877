"""Loader for the in-tree native extension ``_vep`` (built by ``csrc/build.py``).

The native module is mandatory: there is no silent Python fallback for the data plane. When it
is missing, importing fails loudly with the build command to run.
"""
from __future__ import annotations

import functools

# PyTorch-ROCm ships its own HIP/HSA runtime next to the /opt/rocm one the extension links. When
# the extension's runtime initialises the GPU first, torch's later initialisation finds no device
# ("No HIP GPUs are available", seen on the MI355X boxes); loading torch first keeps both working
# (consumer tensors, RCCL) in every import order.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch-less deployments still get the data plane
    pass

try:
    from . import _vep as native  # type: ignore[attr-defined]
except ImportError as e:  # pragma: no cover - exercised only on a broken checkout
    raise ImportError(
        "video_edge_ai_proxy_amd._vep is not built; run `python csrc/build.py` "
        f"(hipcc --offload-arch=gfx950). Original error: {e}"
    ) from e


@functools.lru_cache(maxsize=1)
def gpu_count() -> int:
    """Number of visible HIP devices (0 on a CPU-only host)."""
    return int(native.device_count())


def require_gpu() -> None:
    if gpu_count() == 0:
        raise RuntimeError("no HIP device visible: the gfx950 data plane needs an MI355X")
