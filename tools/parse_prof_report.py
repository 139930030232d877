"""Symbolise a host sampling profile and print per-function and per-source-line shares
(inlined frames resolved by llvm-symbolizer; each enclosing function counted once).

Two input formats:
  * parse_bench / hevc_bench (`PROF=<s>`): "count 0xaddr" lines, absolute addresses of BIN
    (built -no-pie): python tools/parse_prof_report.py BIN [parse_prof.txt]
  * the extension's hostprof (vep.native.hostprof_stop): "count object 0xoffset symbol" lines;
    offsets inside our extension are symbolised, other objects are reported by dynamic symbol:
    python tools/parse_prof_report.py --hostprof PROF.txt
"""
import collections
import os
import subprocess
import sys

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def symbolize(obj, addrs):
    out = subprocess.run([SYM, "--obj", obj, "-i", "-C"], input="\n".join(addrs) + "\n",
                         capture_output=True, text=True).stdout
    res = []
    for b in out.strip("\n").split("\n\n"):
        ls = b.replace("(anonymous namespace)", "anon").split("\n")
        res.append([(ls[i], ls[i + 1]) for i in range(0, len(ls) - 1, 2)])
    return res


def fname(f):
    return f.split("(")[0][-80:]


def report(samples, top=30):
    """samples: list of (count, frames) with frames = [(function, file:line:col), ...] innermost first."""
    total = sum(c for c, _ in samples) or 1
    by_line, self_, incl = collections.Counter(), collections.Counter(), collections.Counter()
    for c, frames in samples:
        if not frames:
            continue
        fn0, loc0 = frames[0]
        by_line[(fname(fn0)[-60:], loc0.split("/")[-1])] += c
        self_[fname(fn0)] += c
        for fn in {fname(f) for f, _ in frames}:
            incl[fn] += c
    print(f"{total} samples")
    for title, ctr in (("self (innermost inlined frame)", self_), ("inclusive", incl)):
        print(f"\n-- {title} --")
        for fn, c in ctr.most_common(top):
            print(f"{100 * c / total:6.2f}%  {fn}")
    print("\n-- lines --")
    for (fn, loc), c in by_line.most_common(top + 10):
        print(f"{100 * c / total:6.2f}%  {loc:28s} {fn}")


def main():
    if sys.argv[1] == "--hostprof":
        rows = [l.split(maxsplit=3) for l in open(sys.argv[2]) if l.strip()]
        by_obj = collections.defaultdict(list)
        for c, obj, off, sym in rows:
            by_obj[obj].append((int(c), off, sym))
        samples = []
        objs = collections.Counter()
        for obj, items in by_obj.items():
            objs[os.path.basename(obj)] += sum(c for c, _, _ in items)
            local = obj if os.path.exists(obj) else os.path.join(
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video_edge_ai_proxy_amd",
                os.path.basename(obj))  # a profile taken on the GPU box: the same .so in this tree
            if "_vep" in os.path.basename(obj) and os.path.exists(local):
                for (c, _, _), frames in zip(items, symbolize(local, [o for _, o, _ in items])):
                    samples.append((c, frames))
            else:
                for c, off, sym in items:
                    samples.append((c, [(f"{os.path.basename(obj)}:{sym}", "?")]))
        total = sum(objs.values()) or 1
        print("-- objects --")
        for o, c in objs.most_common(12):
            print(f"{100 * c / total:6.2f}%  {o}")
        report(samples)
        return
    binp = sys.argv[1]
    prof = sys.argv[2] if len(sys.argv) > 2 else "parse_prof.txt"
    rows = [l.split() for l in open(prof) if l.strip()]
    frames = symbolize(binp, [a for _, a in rows])
    report([(int(c), f) for (c, _), f in zip(rows, frames)])


if __name__ == "__main__":
    main()
