"""vep — MI355X-native multi-camera RTSP ingest and frame-serving hub.

Capabilities of tangtang888/video-edge-ai-proxy (camera registry + supervision, latest-frame
gRPC serving, REST/portal API, lazy/keyframe-only decode, RTMP pass-through, cloud storage
toggle, batched annotation upload, per-GOP MP4 archive) re-designed for AMD MI355X (gfx950):
native C++ ingest/bitstream layer, batched CDNA4 HIP decode/convert kernels, per-camera HBM
frame rings and camera-data-parallel sharding over RCCL/xGMI.
"""

__version__ = "0.1.0"

from ._native import gpu_count, native  # noqa: F401
