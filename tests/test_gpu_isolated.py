"""The process-isolated hub on the GPU (``gpu.isolation: process``): a front-end program that
never touches the GPU supervises a worker process on device 0 (vep_bench/isolated_check.py). Checks
frames served through page-locked shared memory against the ring, the RCCL-group consumer batch
against the fp32 letterbox reference, and a SIGKILLed GPU worker's restart + group re-formation.
Started as a child program with its own time limit (this pytest process holds a GPU context, so
the front-end must be a separate process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_isolated_hub_on_gpu():
    cmd = [sys.executable, "-m", "vep_bench.isolated_check", "--devices=0", "--cams", "2",
           "--width", "1920", "--height", "1080", "--letterbox", "640", "--samples", "30", "--kill"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stderr[-3000:]
    d = json.loads(lines[-1])
    assert r.returncode == 0 and d["ok"], (d, r.stderr[-2000:])
    assert d["shm_pinned"] and d["frame_equal"] and d["batch_max_abs_err"] <= 1
    assert d["group"][0]["backend"] == "nccl" and d["restarted"]
