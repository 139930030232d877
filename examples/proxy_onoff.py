"""Start/stop RTMP pass-through of a camera (the reference had the RPC but no example).

    python examples/proxy_onoff.py --device front_door --on true
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from video_edge_ai_proxy_amd.proto import pb  # noqa: E402
from video_edge_ai_proxy_amd.server.grpc_server import ImageClient  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", required=True)
    ap.add_argument("--on", choices=["true", "false"], required=True)
    ap.add_argument("--addr", default="127.0.0.1:50001")
    a = ap.parse_args()
    print(ImageClient(a.addr).Proxy(pb.ProxyRequest(device_id=a.device, passthrough=a.on == "true")))
