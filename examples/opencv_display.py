"""Continuously fetch the latest frame of a camera (reference: examples/opencv_display.py).

Shows the frames with OpenCV when it is installed; otherwise writes ``<device>.ppm`` each frame.

    python examples/opencv_display.py --device front_door [--keyframe]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from video_edge_ai_proxy_amd.proto import pb  # noqa: E402
from video_edge_ai_proxy_amd.server.grpc_server import ImageClient  # noqa: E402

try:
    import cv2  # type: ignore
except ImportError:
    cv2 = None

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", required=True)
    ap.add_argument("--keyframe", action="store_true")
    ap.add_argument("--addr", default="127.0.0.1:50001")
    ap.add_argument("--frames", type=int, default=0, help="stop after N frames (0 = forever)")
    a = ap.parse_args()
    stub = ImageClient(a.addr)
    n = 0
    t0 = time.time()
    while a.frames == 0 or n < a.frames:
        req = iter([pb.VideoFrameRequest(device_id=a.device, key_frame_only=a.keyframe)])
        for frame in stub.VideoLatestImage(req):
            if not frame.width:
                continue
            img = np.frombuffer(frame.data, np.uint8).reshape([d.size for d in frame.shape.dim])
            n += 1
            if cv2 is not None:
                cv2.imshow("vep", img)
                if cv2.waitKey(1) & 0xFF == ord("q"):
                    sys.exit(0)
            else:
                with open(f"{a.device}.ppm", "wb") as f:
                    f.write(f"P6 {img.shape[1]} {img.shape[0]} 255\n".encode() + img[:, :, ::-1].tobytes())
    print(f"{n} frames in {time.time() - t0:.2f} s")
