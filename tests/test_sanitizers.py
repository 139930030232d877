"""ThreadSanitizer / AddressSanitizer runs of the native stress driver (csrc/tests/native_stress.cpp).

Host-code sanitizers only (`-Xarch_host -fsanitize=...`; GPU sanitizers are unavailable), CPU
backend. Building takes about a minute per sanitizer, so the test runs when VEP_SANITIZERS=1
(`make tsan asan` runs the same thing; the last logs are kept in profiles/).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(os.environ.get("VEP_SANITIZERS") != "1", reason="set VEP_SANITIZERS=1")
@pytest.mark.parametrize("target", ["tsan", "asan"])
def test_native_stress_under_sanitizer(target):
    r = subprocess.run(["make", "-C", ROOT, target], capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "native_stress ok" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out


def test_sanitizer_target_links():
    """The sanitizer binaries' source set links (every csrc/vep/*.cpp + *.hip): a cheap check
    that runs in the default CPU suite, so a missing kernel file breaks here, not only under
    VEP_SANITIZERS=1."""
    r = subprocess.run(["make", "-C", ROOT, "link-check"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert os.path.exists(os.path.join(ROOT, "build", "linkcheck", "native_stress"))
