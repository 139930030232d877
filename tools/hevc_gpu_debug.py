"""Decode a small H.265 coverage stream on GPU 0 in both intra-TU scheduling modes (one queue
launch vs one launch per level) and report published / differing frames and the camera's logs."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from video_edge_ai_proxy_amd import native  # noqa: E402
from test_hevc_camera import synth_hevc  # noqa: E402


def run(mode, w=200, h=120, n=14, **kw):
    os.environ["VEP_HEVC_TU_QUEUE"] = mode
    s = synth_hevc(native, w, h, **kw)
    wk = native.Worker(device=0)
    cam = wk.add_camera("hevc", 4)
    want, pub, bad, seq = {}, 0, 0, 0
    for _ in range(n):
        au = s.next()
        y, uv = s.picture()
        want[s.last_pts] = native.nv12_to_bgr_cpu(y, uv, 0, 0, w, h)
        wk.decode_now(cam, au)
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, got = r
        seq = meta["seq"]
        pub += 1
        bad += int(not np.array_equal(got, want[meta["pts"]]))
    print(f"mode={mode} published={pub} differing={bad} stats={ {k: v for k, v in wk.stats(cam).items() if k in ('decoded', 'errors', 'skipped')} }")
    print("  err log:", wk.logs(cam, True, 5)[-600:])


if __name__ == "__main__":
    for mode in ("0", "1"):
        run(mode, coverage=True, bframes=1, slices=2)
