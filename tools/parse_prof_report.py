"""Symbolise parse_bench's sampling profile (PROF=<s> ./parse_bench ... -> parse_prof.txt):
per-function and per-source-line sample shares, inlined frames resolved to the innermost line
and attributed to each enclosing function once. Usage: python tools/parse_prof_report.py BIN [prof.txt]"""
import collections
import subprocess
import sys

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def main():
    binp = sys.argv[1]
    prof = sys.argv[2] if len(sys.argv) > 2 else "parse_prof.txt"
    rows = [l.split() for l in open(prof) if l.strip()]
    counts = [int(c) for c, _ in rows]
    addrs = [a for _, a in rows]
    out = subprocess.run([SYM, "--obj", binp, "--inlining", "--demangle", "--no-untag-addresses"] if False else
                         [SYM, "--obj", binp, "-i", "-C"], input="\n".join(addrs) + "\n",
                         capture_output=True, text=True).stdout
    blocks = out.strip("\n").split("\n\n")
    total = sum(counts)
    by_line = collections.Counter()
    by_fn_self = collections.Counter()
    by_fn_incl = collections.Counter()
    for c, b in zip(counts, blocks):
        ls = b.replace("(anonymous namespace)", "anon").split("\n")
        frames = [(ls[i], ls[i + 1]) for i in range(0, len(ls) - 1, 2)]
        if not frames:
            continue
        fn0, loc0 = frames[0]
        by_line[(fn0.split("(")[0][-60:], loc0.split("/")[-1])] += c
        by_fn_self[fn0.split("(")[0][-80:]] += c
        for fn in {f.split("(")[0][-80:] for f, _ in frames}:
            by_fn_incl[fn] += c
    print(f"{total} samples")
    print("\n-- self (innermost inlined frame) --")
    for fn, c in by_fn_self.most_common(25):
        print(f"{100 * c / total:6.2f}%  {fn}")
    print("\n-- inclusive --")
    for fn, c in by_fn_incl.most_common(30):
        print(f"{100 * c / total:6.2f}%  {fn}")
    print("\n-- lines --")
    for (fn, loc), c in by_line.most_common(40):
        print(f"{100 * c / total:6.2f}%  {loc:28s} {fn}")


if __name__ == "__main__":
    main()
