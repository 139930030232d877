"""Enable/disable cloud storage of a camera's RTMP stream (reference: examples/storage_onoff.py).

    python examples/storage_onoff.py --device front_door --on true
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from video_edge_ai_proxy_amd.proto import pb  # noqa: E402
from video_edge_ai_proxy_amd.server.grpc_server import ImageClient  # noqa: E402


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", required=True)
    ap.add_argument("--on", type=str2bool, required=True)
    ap.add_argument("--addr", default="127.0.0.1:50001")
    a = ap.parse_args()
    print(ImageClient(a.addr).Storage(pb.StorageRequest(device_id=a.device, start=a.on)))
