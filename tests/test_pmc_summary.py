"""tools/rocpd_pmc_summary.py: ratios only from collected counters, a failing exit code when a
required ratio's counters are missing (round 4's summary printed 0.000 / nan instead), and the
achieved HBM bandwidth from FETCH_SIZE / WRITE_SIZE against the kernels' own time."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "rocpd_pmc_summary.py")


def _db(path, rows):
    db = sqlite3.connect(path)
    db.execute("create table counters_collection (kernel_name text, dispatch_id int, counter_name text, "
               "value real, duration real)")
    db.executemany("insert into counters_collection values (?,?,?,?,?)", rows)
    db.commit()
    db.close()


def _run(*args):
    return subprocess.run([sys.executable, TOOL, *args], capture_output=True, text=True)


def test_pmc_summary_ratios_and_bandwidth(tmp_path):
    k = "vep::gpu::decode_convert_kernel(vep::gpu::DecodeDesc const*, int)"
    a, b = str(tmp_path / "a.db"), str(tmp_path / "b.db")
    _db(a, [(k, 1, "SQ_WAVE_CYCLES", 1000, 10000), (k, 1, "SQ_ACTIVE_INST_VALU", 250, 10000),
            (k, 1, "SQ_WAVES", 10, 10000), (k, 1, "SQ_INSTS_VALU", 500, 10000)])
    # 4 MB read + 2 MB written in 1 ms -> 6 GB/s... per 1e6 ns: (4096 KB + 2048 KB) * 1024 B / 1 ms
    _db(b, [(k, 1, "FETCH_SIZE", 4096, 1_000_000), (k, 1, "WRITE_SIZE", 2048, 1_000_000)])
    r = _run("--require", "valu_per_wave_cycle", a, b)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "decode_convert_kernel,0.250" in out.replace(" ", "")  # VALU / wave-cycle
    assert "not collected:" in out and "lds_bank_conflicts_per_lds_inst" in out
    line = [l for l in out.splitlines() if l.startswith("decode_convert_kernel,1,")][0].split(",")
    assert abs(float(line[5]) - 4.2) < 0.05 and abs(float(line[6]) - 2.1) < 0.05  # GB/s


def test_pmc_summary_fails_when_required_counters_missing(tmp_path):
    a = str(tmp_path / "a.db")
    _db(a, [("avc_deblock_kernel", 1, "SQ_WAVES", 10, 5)])
    r = _run("--require", "wait_per_wave_cycle", a)
    assert r.returncode == 2 and "wait_per_wave_cycle" in r.stderr
    r = _run(a)  # nothing computable at all
    assert r.returncode == 2
