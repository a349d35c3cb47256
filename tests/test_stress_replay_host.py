"""tools/stress_replay.py on the CPU: the r05_v12 stress fault's configuration
comes back from the seed alone.  The round-5 stress
(seed 7, before the placement-probe draw was added) faulted at its 657th
sort; iteration 656 is that sort and 655 the context destroyed before it."""
import json
import os
import subprocess
import sys

import pytest

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


def _logged(path, hi):
    """(iteration, configuration fields) of the sorts a stress_mix log names."""
    import re
    out = {}
    with open(path) as f:
        for line in f:
            m = re.match(r"iter (\d+): (.*?) first_pass=", line)
            if m and int(m.group(1)) < hi:
                out[int(m.group(1))] = dict(kv.split("=") for kv in m.group(2).split())
    return out


@pytest.mark.parametrize("log,seed,draws", [("stress/stress_mix_seed61.log", 61, "current"),
                                            ("g10/replay_r05v12.log", 7, "r05v12")])
def test_replay_matches_the_round6_stress_logs(log, seed, draws):
    """stress_mix.py and stress_replay.py share one draw function: the replay
    names the same configurations, iteration by iteration, as the round-6
    runs on the GPU logged: the stress of seed 61 (profiles/r06/stress/) and
    the debug-build run of round 5's seed-7 sequence (profiles/r06/g10/)."""
    want = _logged(os.path.join(ROOT, "profiles", "r06", log), 300)
    assert len(want) == 300
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stress_replay.py"), "--seed", str(seed),
                        "--draws", draws, "--list", "0:300"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(rows) == 300
    for r in rows:
        w = want[r["iter"]]
        got = {k: str(r[k]) for k in ("n", "P", "bits", "dist", "split", "hybrid", "gather", "vmm", "region_min",
                                      "probe", "chunks")}
        assert got == w, (r["iter"], got, w)
