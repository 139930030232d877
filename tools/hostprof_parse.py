"""In-situ host profile of the replay bench's parse pool (no GPU work): N threads parsing the
bench's 32 camera streams while the extension's SIGPROF sampler runs.
Usage: PROFILE=high python tools/hostprof_parse.py OUT.txt [threads] [cams] [ticks]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from video_edge_ai_proxy_amd import native as vep  # noqa: E402


def main():
    out = sys.argv[1]
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    cams = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    ticks = int(sys.argv[4]) if len(sys.argv) > 4 else 300
    cfg = vep.SynthConfig()
    cfg.width, cfg.height, cfg.fps, cfg.gop = 1920, 1080, 30, 30
    cfg.compressed = True
    cfg.qp, cfg.noise, cfg.temporal_noise, cfg.refs = 25, 8.0, 1.5, 1
    cfg.profile, cfg.bframes, cfg.cabac = os.environ.get("PROFILE", "high"), 2, True
    w = vep.Worker(device=-1, max_cameras=cams)
    rb = vep.ReplayBench(w, cams, cfg, cached_frames=30, threads=threads, ring_slots=2, prefix="p_")
    rb.parse_only_ms(30)  # warm
    vep.hostprof_start(500)
    ms = rb.parse_only_ms(ticks)
    n = vep.hostprof_stop(out)
    print(f"threads={threads}: {ms:.2f} ms/tick, {ms * threads / cams:.2f} thread-ms/frame, {n} samples -> {out}")


if __name__ == "__main__":
    main()
