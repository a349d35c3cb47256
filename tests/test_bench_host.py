"""bench.py's host-side legs on CPU: the core count it reports and the CPU
baseline (the reference's own mpi_lsbsort, oracle/_ref, timed by its own
sort-only window, mpi/mpi_lsbsort.cpp:688-699), on a small n."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_host_cores_fields():
    c = bench.host_cores()
    assert c["nproc"] >= 1 and 1 <= c["share"] <= c["nproc"]
    assert c["physical"] is None or 1 <= c["physical"] <= c["nproc"]


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "mpi_lsbsort")) or
                    not (shutil.which("mpirun") or os.path.exists("/opt/conda/bin/mpirun")),
                    reason="reference binary (make -C oracle ref) or mpirun absent")
def test_cpu_baseline_times_the_reference():
    r = bench.cpu_baseline(1 << 20, cpu_n=1 << 20, runs=1)
    assert r is not None
    assert r["kind"] == "reference" and r["n"] == 1 << 20 and r["n_basis"] == "requested"
    assert r["ranks"] >= 5 and r["cores_used"] == r["ranks"]  # >= 5 ranks
    assert len(r["runs"]) == 1 and r["value"] == r["median"] > 0
