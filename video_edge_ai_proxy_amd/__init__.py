"""vep — MI355X-native multi-camera RTSP ingest and frame-serving hub.

Capabilities of tangtang888/video-edge-ai-proxy (camera registry + supervision, latest-frame
gRPC serving, REST/portal API, lazy/keyframe-only decode, RTMP pass-through, cloud storage
toggle, batched annotation upload, per-GOP MP4 archive) re-designed for AMD MI355X (gfx950):
native C++ ingest/bitstream layer, batched CDNA4 HIP decode/convert kernels, per-camera HBM
frame rings and camera-data-parallel sharding over RCCL/xGMI.
"""

__version__ = "0.1.0"

import os as _os

# A GPU worker runs a serving stream plus, per decode lane, a kernel stream and a copy stream
# (7 for the default 3 lanes): 8 hardware queues instead of HIP's 4, so none of them shares a
# queue with another. Read once when HIP initialises, so it must be set before that.
_os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

from ._native import gpu_count, native  # noqa: F401
