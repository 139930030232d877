"""Clock of this process's busy CPUs: /proc/cpuinfo 'cpu MHz' of the CPUs that were >50% busy over
the last 0.5 s (with the whole machine's median for comparison). Run while a load runs."""
import statistics
import time


def busy():
    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    p = line.split()
                    v = [int(x) for x in p[1:]]
                    out[int(p[0][3:])] = (sum(v), v[3] + v[4])
        return out

    a = snap()
    time.sleep(0.5)
    b = snap()
    return {c for c in b if 1 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) > 0.5}


def mhz():
    out, cur = {}, None
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("processor"):
                cur = int(line.split(":")[1])
            elif line.startswith("cpu MHz") and cur is not None:
                out[cur] = float(line.split(":")[1])
    return out


if __name__ == "__main__":
    hot = busy()
    m = mhz()
    hv = [m[c] for c in hot if c in m]
    print(f"busy CPUs: {len(hot)}; their MHz median {statistics.median(hv) if hv else 0:.0f} "
          f"(min {min(hv) if hv else 0:.0f}, max {max(hv) if hv else 0:.0f}); all CPUs median {statistics.median(m.values()) if m else 0:.0f}")
