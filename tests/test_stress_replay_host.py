"""tools/stress_replay.py on the CPU: the r05_v12 stress fault's configuration
comes back from the seed alone.  The round-5 stress
(seed 7, before the placement-probe draw was added) faulted at its 657th
sort; iteration 656 is that sort and 655 the context destroyed before it."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_seed7_iterations_655_656():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stress_replay.py"), "--seed", "7",
                        "--draws", "r05v12", "--list", "655:657"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert [r["iter"] for r in rows] == [655, 656]
    before, fault = rows
    # the context destroyed just before the fault: one rank, no exchange
    assert (before["n"], before["P"], before["bits"], before["dist"], before["hybrid"], before["vmm"]) == \
        (109863384, 1, 16, "zipf", 1, 64)
    # the faulting sort: P = 8 loopback, 16-bit digits, gathered exchanges, 64 MiB VMM pieces
    assert (fault["n"], fault["P"], fault["bits"], fault["dist"], fault["gather"], fault["vmm"]) == \
        (88599894, 8, 16, "uniform", 1, 64)
