"""Host sanitizers ("host ASan/UBSan on the CPU restatement").

* the oracle's C restatement under ASan/UBSan (oracle/sanitize_driver.c:
  pcg64 known answers, the P-rank sort against an independent merge sort,
  checkSorted);
* the C ABI's host code under ASan/UBSan with leak detection
  (tools/host_asan.cpp: the host planner on random / skewed / empty count
  matrices with a permutation check of every placement, every argument
  check, and context teardown after a failed device allocation).
Device code is not instrumented (GPU sanitizers are not available here).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make(target_dir, target):
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, target_dir), target],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_under_asan_ubsan():
    assert "oracle sanitizer driver: ok" in _make("oracle", "sanitize")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_host_abi_under_asan_ubsan():
    assert "host ABI sanitizer driver: ok" in _make("distributed-lsb_amd", "asan")
