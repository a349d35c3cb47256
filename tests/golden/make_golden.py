#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs the reference's own ``mpi/mpi_lsbsort.cpp`` (compiled in place by
``make -C oracle ref`` into ``oracle/_ref/mpi_lsbsort``; never copied into
the repo) under MPICH's ``mpirun`` and records what it prints with
``--print``:

  * ``ref_print_vectors.json`` — for each (n, P): every ``A[i] = (key,val)``
    line the reference prints before and after sorting.  When every rank
    holds <= 10 elements this is the whole input and output array; otherwise
    it is the first 10 elements of every rank (mpi/mpi_lsbsort.cpp:171-200).
    The reference's built-in verify (stable_sort + ``==``,
    mpi/mpi_lsbsort.cpp:710-738) runs too; a failure aborts this script.

``digests.json`` is NOT produced here: its SHA-256 rows were recorded from
the same reference binary during the survey and are kept
verbatim.  tests/test_oracle.py re-derives them from the oracle.

Usage:  python tests/golden/make_golden.py   (needs /root/reference + MPICH)
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "mpi_lsbsort")
MPIRUN = "/opt/conda/bin/mpirun"

# (n, P): small enough that every element prints, plus larger ones where the
# first 10 per rank print.  Ragged n % P, n < P and n == 0 are included.
CASES = [
    (0, 1), (0, 2), (1, 1), (1, 3), (3, 4), (7, 2), (10, 1), (17, 8), (20, 2),
    (30, 3), (40, 4), (80, 8), (5, 8),
    (1000, 3), (100003, 4), (1000000, 2), (1000003, 4), (1 << 20, 1), (1 << 20, 8),
]

LINE = re.compile(r"^A\[(\d+)\] = \(([0-9a-f]{16}),(\d+)\)$")


def run_case(n, P):
    cmd = [MPIRUN, "-n", str(P), REF_BIN, "--n", str(n), "--print", "--verify"]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    before, after = {}, {}
    seen_sorting = False
    for line in out.splitlines():
        if line.startswith("Sorting"):
            seen_sorting = True
            continue
        m = LINE.match(line.strip())
        if m:
            idx, key, val = int(m.group(1)), m.group(2), int(m.group(3))
            (after if seen_sorting else before)[idx] = [key, val]
    if "Verifying" not in out and n < 128 * 1024 * 1024:
        raise RuntimeError(f"reference did not verify for n={n} P={P}:\n{out}")
    full = all(min(10, max(0, min(-(-n // P), n - r * (-(-n // P))))) ==
               max(0, min(-(-n // P), n - r * (-(-n // P)))) for r in range(P)) if n else True
    return {
        "n": n, "P": P, "complete": bool(full),
        "input": [[i] + before[i] for i in sorted(before)],
        "output": [[i] + after[i] for i in sorted(after)],
    }


def main():
    if not os.path.exists(REF_BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    cases = []
    for n, P in CASES:
        c = run_case(n, P)
        print(f"n={n} P={P} complete={c['complete']} printed={len(c['input'])}", file=sys.stderr)
        cases.append(c)
    doc = {
        "source": "oracle/_ref/mpi_lsbsort (reference mpi/mpi_lsbsort.cpp) under MPICH 3.3.2 mpirun",
        "format": "rows are [global_index, key_hex16, val]",
        "cases": cases,
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_print_vectors.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=0)
    print(path)


if __name__ == "__main__":
    main()
