"""The drop-in at the reference's own seam.

oracle/_ref/mpi_lsbsort_hip is the reference's mpi/mpi_lsbsort.cpp with ONLY
its mySort (:580-585) replaced by the stub oracle/dropin/lsb_mysort.inc
(built by `make -C oracle dropin`; the reference text is streamed into the
compiler, never stored).  Everything else is the reference's: MPI_Init, the
CLI, the pcg64 input, the timed window, --print and its verify -- the
gather to rank 0, std::stable_sort and the element-wise == whose failure
aborts (:710-738).  So each case below is the reference program itself
sorting on the MI355X through the C ABI, one MPI rank per RCCL rank; with
more ranks than GPUs every rank is its own RCCL host (socket transport).

Checks: exit 0 (the reference's assert did not fire), no "did not match"
line, and the lines it prints with --print equal what the unmodified
reference printed for the same (n, P) (tests/golden/ref_print_vectors.json,
made by tests/golden/make_golden.py from oracle/_ref/mpi_lsbsort).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "mpi_lsbsort_hip")
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"

pytestmark = [
    pytest.mark.gpu,
    pytest.mark.skipif(not os.path.exists(DROPIN) or not os.path.exists(MPIRUN),
                       reason="drop-in binary (make -C oracle dropin) or mpirun absent"),
]


def _run(n, P, radix=None, timeout=240):
    env = dict(os.environ)
    if radix:
        env["LSB_DROPIN_RADIX_BITS"] = str(radix)
    return subprocess.run([MPIRUN, "-n", str(P), DROPIN, "--n", str(n), "--print", "--verify"],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd="/tmp")


@pytest.mark.parametrize("n,P,radix", [
    (1048576, 1, None), (1000000, 2, None), (1000003, 4, None), (100003, 4, 8), (1000, 3, 64),
    (7, 2, None), (3, 4, None), (0, 2, None),
])
def test_reference_program_sorts_through_the_stub(lsb_built, ref_vectors, n, P, radix):
    r = _run(n, P, radix)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = r.stdout.splitlines()
    assert f"Total number of MPI ranks: {P}" in lines and f"Problem size: {n}" in lines
    assert any(l.startswith(f"Sorted {n} values in ") for l in lines)
    assert any(l.startswith("That's ") and l.endswith(" M elements sorted / s") for l in lines)
    assert "Verifying" in lines and not any("did not match" in l for l in lines)
    # the A[i] lines before and after "Sorting", by index (ranks print in turn)
    case = next(c for c in ref_vectors["cases"] if c["n"] == n and c["P"] == P)
    before, after, seen = {}, {}, False
    for l in lines:
        if l.startswith("Sorting"):
            seen = True
        m = re.match(r"^A\[(\d+)\] = \(([0-9a-f]{16}),(\d+)\)$", l.strip())
        if m:
            (after if seen else before)[int(m.group(1))] = [m.group(2), int(m.group(3))]
    assert before == {i: [k, v] for i, k, v in case["input"]}
    assert after == {i: [k, v] for i, k, v in case["output"]}
