"""Single-thread host parse throughput of the bench's H.264 High streams (replay, parse only),
optionally with another build of the extension (A/B of parser changes on one machine):
  python tools/parse_ab.py [--so path/to/_vep...so] [--reps 5] [--codec h265] [--threads N --cams 32]
Prints the best and median ms per tick over `reps` measurements of 60 ticks, the CABAC bins per
picture and the time-stamp-counter cycles per bin (per parse thread)."""
import argparse
import importlib.machinery
import importlib.util
import os
import statistics
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default="")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cams", type=int, default=4)
    ap.add_argument("--codec", default="h264")
    ap.add_argument("--threads", type=int, default=1, help="parse pool threads (multi-thread throughput)")
    a, rest = ap.parse_known_args()
    if a.so:  # load the other build under the package's module name before anything imports it
        name = "video_edge_ai_proxy_amd._vep"
        spec = importlib.util.spec_from_file_location(name, a.so)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
    sys.argv = ["bench.py", "--cpu", "--source", "replay", "--codec", a.codec] + rest
    import bench
    from video_edge_ai_proxy_amd import native as vep

    b = bench.parse_args()
    w = vep.Worker(device=-1, letterbox_size=0, max_cameras=a.cams)
    cfg = bench.make_cfg(vep, b, 0, True)
    rb = vep.ReplayBench(w, a.cams, cfg, cached_frames=b.gop * b.cache_gops, threads=a.threads, prefix="p")
    import time

    rb.parse_only_ms(30)
    b0, c0, t0 = vep.cabac_bins_decoded(), vep.tsc_now(), time.perf_counter()
    ms = [rb.parse_only_ms(60) for _ in range(a.reps)]
    b1, c1, t1 = vep.cabac_bins_decoded(), vep.tsc_now(), time.perf_counter()
    pics = a.cams * 60 * a.reps
    bins_per_pic = (b1 - b0) / pics
    tsc_ghz = (c1 - c0) / (t1 - t0) / 1e9
    cyc_per_bin = (t1 - t0) * a.threads * tsc_ghz * 1e9 / max(1, b1 - b0)
    print(f"{a.so or 'tree'}: best {min(ms):.3f} median {statistics.median(ms):.3f} ms/tick "
          f"-> {a.cams / min(ms) * 1000 / a.threads:.1f} fps/thread (best), {a.cams / min(ms) * 1000:.0f} fps "
          f"with {a.threads} threads; {bins_per_pic:.0f} CABAC bins/picture, {cyc_per_bin:.1f} TSC cycles/bin "
          f"per thread (TSC {tsc_ghz:.2f} GHz)", flush=True)


if __name__ == "__main__":
    main()
