#!/usr/bin/env python3
"""Per-kernel summary (calls, total / mean / max us, share) from a rocprofv3 rocpd SQLite
database (`rocprofv3 --kernel-trace -d DIR -o NAME` writes DIR/.../NAME_results.db)."""
import glob
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = con.execute(
        f"select s.kernel_name, count(*), sum(d.end - d.start), max(d.end - d.start) "
        f"from {kd} d join {ks} s on d.kernel_id = s.id group by s.kernel_name").fetchall()
    total = sum(r[2] for r in rows) or 1
    rows.sort(key=lambda r: -r[2])
    out = ["kernel,calls,total_us,mean_us,max_us,percent"]
    for name, n, tot, mx in rows:
        short = name.split("(")[0]
        out.append(f"{short},{n},{tot / 1e3:.1f},{tot / 1e3 / n:.2f},{mx / 1e3:.2f},{100.0 * tot / total:.1f}")
    return "\n".join(out)


if __name__ == "__main__":
    for path in sys.argv[1:]:
        for db in glob.glob(path if path.endswith(".db") else path + "/**/*.db", recursive=True):
            print(f"# {db}")
            print(stats(db))
