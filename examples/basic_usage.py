"""List streams and print one frame's metadata (reference: examples/basic_usage.py).

    python examples/basic_usage.py --list
    python examples/basic_usage.py --device front_door
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from video_edge_ai_proxy_amd.proto import pb  # noqa: E402
from video_edge_ai_proxy_amd.server.grpc_server import ImageClient  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="vep basic example")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--device", default=None)
    ap.add_argument("--addr", default="127.0.0.1:50001")
    a = ap.parse_args()
    stub = ImageClient(a.addr)  # max message size raised: 1080p frames are 6.2 MB
    if a.list:
        for s in stub.ListStreams(pb.ListStreamRequest()):
            print(s)
    if a.device:
        req = iter([pb.VideoFrameRequest(device_id=a.device, key_frame_only=False)])
        for frame in stub.VideoLatestImage(req):
            print("is keyframe: ", frame.is_keyframe)
            print("frame type: ", frame.frame_type)
            print("frame shape: ", frame.shape)
