#!/usr/bin/env python3
"""Print the reference's mpi/mpi_lsbsort.cpp with ONLY its mySort definition
(mpi/mpi_lsbsort.cpp:580-585) replaced by `#include "lsb_mysort.inc"`, the
drop-in stub of INTEGRATION.md section 2 (oracle/dropin/lsb_mysort.inc).

The output goes to stdout and straight into the compiler (oracle/Makefile
target `dropin`): no reference text is written to disk or committed.  The
rest of the program -- MPI_Init, the CLI, the pcg64 input, the timed window,
--print and the gather + std::stable_sort verify (:587-743) -- is the
reference's own, unchanged.

Usage: python3 oracle/dropin/splice.py /root/reference/mpi/mpi_lsbsort.cpp
"""
import re
import sys

MYSORT = re.compile(r"void mySort\(DistributedArray<SortElement>& A,\s*DistributedArray<SortElement>& B\)\s*\{"
                    r".*?\n\}\n", re.S)


def splice(text):
    found = MYSORT.findall(text)
    if len(found) != 1:
        raise SystemExit(f"splice.py: expected one mySort definition, found {len(found)}")
    if "globalShuffle(A, B, digit)" not in found[0]:
        raise SystemExit("splice.py: mySort does not look like the reference's digit loop")
    return MYSORT.sub('#include "lsb_mysort.inc"\n', text)


if __name__ == "__main__":
    sys.stdout.write(splice(open(sys.argv[1]).read()))
