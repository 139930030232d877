"""Host CPU topology and load snapshot (what the parse threads share): cgroup quota, affinity,
SMT siblings, and per-CPU busy fraction over a short window (other tenants' load).
    python tools/cpu_load.py [--seconds 1.0]"""
import argparse
import os
import time


def stat():
    out = {}
    with open("/proc/stat") as f:
        for line in f:
            if line.startswith("cpu") and line[3].isdigit():
                p = line.split()
                v = [int(x) for x in p[1:]]
                out[int(p[0][3:])] = (sum(v), v[3] + v[4])  # total, idle + iowait
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.0)
    a = ap.parse_args()
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective", "/proc/loadavg"):
        try:
            print(path, open(path).read().strip())
        except OSError:
            print(path, "n/a")
    aff = sorted(os.sched_getaffinity(0))
    print("affinity", len(aff), "cpus; os.cpu_count", os.cpu_count())
    for c in (aff[0], aff[min(len(aff) - 1, 15)]):
        try:
            print(f"cpu{c} siblings", open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip())
        except OSError:
            pass
    s0 = stat()
    time.sleep(a.seconds)
    s1 = stat()
    busy = {c: 1 - (s1[c][1] - s0[c][1]) / max(1, s1[c][0] - s0[c][0]) for c in s1 if c in aff}
    hot = [c for c, b in busy.items() if b > 0.5]
    print(f"busy > 50% on {len(hot)} of {len(busy)} allowed CPUs: {hot[:64]}")
    print("mean busy of allowed CPUs: %.3f" % (sum(busy.values()) / max(1, len(busy))))


if __name__ == "__main__":
    main()
