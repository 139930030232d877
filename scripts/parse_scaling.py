"""Host H.264 parse throughput (PROFILE=baseline|main|high) vs thread count (no GPU work): the replay bench's parse stage
alone, on synthetic 1080p camera streams. Usage: python scripts/parse_scaling.py [cams] [threads...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from video_edge_ai_proxy_amd import native as vep  # noqa: E402


def main():
    cams = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    threads = [int(t) for t in sys.argv[2:]] or [1, 4, 8, 14]
    cfg = vep.SynthConfig()
    cfg.width, cfg.height, cfg.fps, cfg.gop = 1920, 1080, 30, 30
    cfg.compressed = True
    profile = os.environ.get("PROFILE", "baseline")
    if profile == "baseline":
        cfg.qp, cfg.noise, cfg.temporal_noise, cfg.refs = 27, 8.0, 1.0, 1
    else:  # bench.py's default High CABAC IBBP streams
        cfg.qp, cfg.noise, cfg.temporal_noise, cfg.refs = 25, 8.0, 1.5, 1
        cfg.profile, cfg.bframes, cfg.cabac = profile, 2, True
    w = vep.Worker(device=-1, max_cameras=cams * len(threads))
    for th in threads:
        rb = vep.ReplayBench(w, cams, cfg, cached_frames=30, threads=th, ring_slots=2,
                             prefix=f"t{th}_")
        ms = min(rb.parse_only_ms(30) for _ in range(3))
        print(f"threads={th:2d}: {ms:7.2f} ms/tick ({cams} cams)  {ms * th / cams:5.2f} thread-ms/frame",
              flush=True)
        del rb


if __name__ == "__main__":
    main()
