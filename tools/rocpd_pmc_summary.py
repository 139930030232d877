"""Summarise rocprofv3 --pmc databases: per kernel, the sum of every counter over its dispatches,
plus derived ratios when the counters are present. Usage:
  python tools/rocpd_pmc_summary.py <pmc_results.db> [...more passes]"""
import collections
import re
import sqlite3
import sys


def short(k):
    m = re.search(r"(avc_\w+_kernel|hevc_\w+_kernel|decode_convert_kernel|letterbox\w*_kernel|nv12_\w+_kernel|__amd_rocclr_\w+)", k)
    return m.group(1) if m else k[:40]


def load(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for p in paths:
        db = sqlite3.connect(p)
        for kname, did, cname, val, d in db.execute(
                "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
            k = short(kname)
            tot[k][cname] += float(val)
            disp[(k, p)].add(did)
            dur[(k, p)][did] = d
    return tot, disp


def main():
    tot, disp = load(sys.argv[1:])
    names = sorted({c for k in tot for c in tot[k]})
    print("kernel," + ",".join(names))
    for k in sorted(tot):
        print(k + "," + ",".join(f"{tot[k].get(c, 0):.0f}" for c in names))
    print()
    print("kernel,VALU/wave-cycle,LDS-issue/wave-cycle,any-issue/wave-cycle,waiting/wave-cycle,"
          "LDS bank conflicts per LDS inst,VALU insts per wave,L2 hit rate")
    for k in sorted(tot):
        t = tot[k]
        wc = t.get("SQ_WAVE_CYCLES", 0)
        f = lambda a: (t.get(a, 0) / wc) if wc else float("nan")
        lds = t.get("SQ_INSTS_LDS", 0)
        bc = (t.get("SQ_LDS_BANK_CONFLICT", 0) / lds) if lds else float("nan")
        waves = t.get("SQ_WAVES", 0)
        vpw = t.get("SQ_INSTS_VALU", 0) / waves if waves else float("nan")
        h, m = t.get("TCC_HIT_sum", 0), t.get("TCC_MISS_sum", 0)
        hit = h / (h + m) if h + m else float("nan")
        print(f"{k},{f('SQ_ACTIVE_INST_VALU'):.3f},{f('SQ_ACTIVE_INST_LDS'):.3f},{f('SQ_ACTIVE_INST_ANY'):.3f},"
              f"{f('SQ_WAIT_ANY'):.3f},{bc:.3f},{vpw:.0f},{hit:.3f}")


if __name__ == "__main__":
    main()
