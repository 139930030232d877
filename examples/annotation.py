"""Send an annotation event (reference: examples/annotation.py).

    python examples/annotation.py --device front_door --type moving
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from video_edge_ai_proxy_amd.proto import pb  # noqa: E402
from video_edge_ai_proxy_amd.server.grpc_server import ImageClient  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", required=True)
    ap.add_argument("--type", required=True)
    ap.add_argument("--addr", default="127.0.0.1:50001")
    a = ap.parse_args()
    now = int(time.time() * 1000)
    req = pb.AnnotateRequest(device_name=a.device, type=a.type, start_timestamp=now,
                             end_timestamp=now + 500, object_type="person", object_id="1",
                             confidence=0.93, ml_model="example", ml_model_version="1.0",
                             object_bouding_box=pb.BoudingBox(top=20, left=30, width=120, height=240),
                             location=pb.Location(lat=46.05, lon=14.5))
    print(ImageClient(a.addr).Annotate(req))
