"""Summarise rocprofv3 --pmc databases: per kernel, the sum of every counter over its dispatches,
then the derived ratios whose counters were collected (each pass holds only a few: see
scripts/gpu_r5_pmc.sh), and the achieved HBM traffic (FETCH_SIZE / WRITE_SIZE, KB) against the
kernel time and the MI355X peak. A ratio whose counters are missing is not printed as 0 or nan:
it is listed as missing, and the tool exits 2 when a --require'd ratio cannot be computed (or
nothing at all can). Usage:

  python tools/rocpd_pmc_summary.py [--require NAME[,NAME]] <pass1/results.db> [...more passes]
"""
import argparse
import collections
import re
import sqlite3
import sys

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, ~8 TB/s

# name -> (numerator counters, denominator counter or None, description)
RATIOS = {
    "valu_per_wave_cycle": (["SQ_ACTIVE_INST_VALU"], "SQ_WAVE_CYCLES", "VALU issue cycles / wave cycles"),
    "lds_per_wave_cycle": (["SQ_ACTIVE_INST_LDS"], "SQ_WAVE_CYCLES", "LDS issue cycles / wave cycles"),
    "any_per_wave_cycle": (["SQ_ACTIVE_INST_ANY"], "SQ_WAVE_CYCLES", "any-instruction issue / wave cycles"),
    "wait_per_wave_cycle": (["SQ_WAIT_ANY"], "SQ_WAVE_CYCLES", "waiting (dependency / memory) / wave cycles"),
    "valu_insts_per_wave": (["SQ_INSTS_VALU"], "SQ_WAVES", "VALU instructions per wave"),
    "lds_bank_conflicts_per_lds_inst": (["SQ_LDS_BANK_CONFLICT"], "SQ_INSTS_LDS", "LDS bank conflict cycles per LDS inst"),
    "l2_hit_rate": (["TCC_HIT_sum"], None, "TCC hits / (hits + misses)"),
}


def short(k):
    m = re.search(r"(avc_\w+_kernel|hevc_\w+_kernel|decode_convert_kernel|letterbox\w*_kernel|nv12_\w+_kernel|"
                  r"gather_kernel|narrow\w*_kernel|weave_kernel|__amd_rocclr_\w+)", k)
    return m.group(1) if m else k[:40]


def load(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)  # kernel -> {(pass, dispatch): ns}
    passes = collections.defaultdict(set)  # counter -> passes it came from
    for p in paths:
        db = sqlite3.connect(p)
        for kname, did, cname, val, d in db.execute(
                "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
            k = short(kname)
            tot[k][cname] += float(val)
            dur[k][(p, did)] = float(d)
            passes[cname].add(p)
    return tot, dur, passes


def ratio(name, t):
    num, den, _ = RATIOS[name]
    if name == "l2_hit_rate":
        if "TCC_HIT_sum" not in t or "TCC_MISS_sum" not in t:
            return None
        h, m = t["TCC_HIT_sum"], t["TCC_MISS_sum"]
        return h / (h + m) if h + m else None
    if any(c not in t for c in num) or den not in t or not t[den]:
        return None
    return sum(t[c] for c in num) / t[den]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--require", default="", help="comma-separated ratio names that must be computable")
    ap.add_argument("dbs", nargs="+")
    a = ap.parse_args()
    tot, dur, passes = load(a.dbs)
    if not tot:
        print("no counter records in the given databases", file=sys.stderr)
        return 2
    names = sorted({c for k in tot for c in tot[k]})
    print("# counters (sum over dispatches)")
    print("kernel," + ",".join(names))
    for k in sorted(tot):
        print(k + "," + ",".join(f"{tot[k][c]:.0f}" if c in tot[k] else "" for c in names))
    print()
    computable = [r for r in RATIOS if any(ratio(r, tot[k]) is not None for k in tot)]
    missing = [r for r in RATIOS if r not in computable]
    print("# derived ratios (only those whose counters were collected)")
    print("kernel," + ",".join(computable))
    for k in sorted(tot):
        vals = [ratio(r, tot[k]) for r in computable]
        print(k + "," + ",".join("" if v is None else f"{v:.3f}" for v in vals))
    if missing:
        print("# not collected: " + ", ".join(f"{r} ({'+'.join(RATIOS[r][0] + ([RATIOS[r][1]] if RATIOS[r][1] else []))})"
                                             for r in missing))
    print()
    # HBM traffic: FETCH_SIZE / WRITE_SIZE are KB per dispatch; kernel time from the same pass
    if any("FETCH_SIZE" in t or "WRITE_SIZE" in t for t in tot.values()):
        print("# HBM traffic (achieved over the kernels' own time; MI355X peak ~8 TB/s)")
        print("kernel,dispatches,kernel_ms,read_MB,write_MB,read_GBps,write_GBps,total_GBps,pct_of_peak")
        for k in sorted(tot):
            t = tot[k]
            if "FETCH_SIZE" not in t and "WRITE_SIZE" not in t:
                continue
            # (the duration of the dispatches of the passes that carried the byte counters)
            ps = passes.get("FETCH_SIZE", set()) | passes.get("WRITE_SIZE", set())
            ds = [v for (p, _), v in dur[k].items() if p in ps]
            ms = sum(ds) / 1e6 / max(1, len(ps))
            rd, wr = t.get("FETCH_SIZE", 0) * 1024 / len(passes.get("FETCH_SIZE", {1})), \
                t.get("WRITE_SIZE", 0) * 1024 / len(passes.get("WRITE_SIZE", {1}))
            gr, gw = (rd / (ms * 1e6) if ms else 0), (wr / (ms * 1e6) if ms else 0)
            print(f"{k},{len(ds) // max(1, len(ps))},{ms:.3f},{rd / 1e6:.1f},{wr / 1e6:.1f},{gr:.1f},{gw:.1f},"
                  f"{gr + gw:.1f},{100 * (gr + gw) / HBM_PEAK_GBS:.2f}")
    req = [r for r in a.require.split(",") if r]
    bad = [r for r in req if r not in computable]
    if bad or not computable:
        print(f"missing required ratios: {bad or list(RATIOS)}", file=sys.stderr)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
