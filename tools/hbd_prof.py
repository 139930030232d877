"""avc_hbd_kernel phase clocks on one H.264 High 10 / 4:2:2 camera (VEP_AVC_PROF=1): cycles per
picture of the intra pass, the loop-filter pass and the barriers between diagonal steps.
Usage: VEP_AVC_PROF=1 python tools/hbd_prof.py [width height bit_depth chroma_format frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from video_edge_ai_proxy_amd import native as vep  # noqa: E402


def main():
    w, h, bd, cf, n = (int(x) for x in (sys.argv[1:6] + ["1920", "1080", "10", "1", "24"][len(sys.argv[1:6]):]))
    c = vep.SynthConfig()
    c.width, c.height, c.gop, c.codec, c.compressed, c.profile = w, h, 12, "h264", True, "high"
    c.bframes, c.qp, c.temporal_noise, c.bit_depth, c.chroma_format = 2, 24, 2.0, bd, cf
    s = vep.SynthH264(c)
    aus = [s.next() for _ in range(n)]
    wk = vep.Worker(device=0)
    cam = wk.add_camera("p", 4)
    t0 = time.perf_counter()
    for au in aus:
        wk.decode_now(cam, au)
    dt = time.perf_counter() - t0
    pr = wk.avc_profile()
    pics = max(1, pr["hbd_pictures"])
    mbs = max(1, pr["hbd_dbk_mbs"])
    print({"pictures": pr["hbd_pictures"], "ms_per_picture_wall": round(dt * 1e3 / n, 3),
           **{k: round(pr[k] / pics) for k in ("hbd_intra", "hbd_dbk", "hbd_barrier")},
           "dbk_cycles_per_mb": {k[8:]: round(pr[k] / mbs) for k in ("hbd_dbk_load", "hbd_dbk_edges", "hbd_dbk_store")}})


if __name__ == "__main__":
    main()
