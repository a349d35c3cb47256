"""Teardown and error-return paths that leave a context, or its buffers, in a
state the next call must survive (advisor r05).

* A loopback context of 8 ranks on VMM pieces destroyed right after its sort,
  and right after a sort that failed with the ranks' streams busy; a fresh
  context then sorts and verifies.  Run in this process (the shipped library)
  and in a child process with the debug build, whose teardown_check reports
  any stream still busy when a record buffer is freed: none may be.
* Peer stores on a world-of-one RCCL context swap its VMM buffers for
  hipMalloc'd ones; those must hold r.cap records, since a later sort with the
  exchange off starts with the regional first pass (advisor r05, medium).
* A regional LSD sort whose layout-reading pass fails to launch leaves the
  input in A (advisor r05, medium).

The reference frees nothing mid-run (mpi/mpi_lsbsort.cpp:511-516, :741).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-lsb_amd")
DEBUG_LIB = os.path.join(PKG, "build", "debug", "liblsb.so")
PROBE = os.path.join(ROOT, "tools", "teardown_probe.py")


def _fresh_sort(L, n, P, bits):
    with L.World(n, ranks=P, radix_bits=bits) as w:
        w.set_option(L.OPT_EXCHANGE_GATHER, 1)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        assert w.check_sorted()


def test_loopback_vmm_destroyed_right_after_sort(lsb_built, monkeypatch):
    L = lsb_built
    monkeypatch.setenv("LSB_VMM_CHUNK_MIB", "2")
    n = 8 * (1 << 21) + 12345
    w = L.World(n, ranks=8, radix_bits=16)
    w.set_option(L.OPT_EXCHANGE_GATHER, 1)
    w.set_option(L.OPT_FORCE_EXCHANGE, 1)
    w.generate()
    w.my_sort()
    w.close()  # no sync in between
    _fresh_sort(L, n, 8, 16)


def test_loopback_vmm_destroyed_after_failed_sort(lsb_built, monkeypatch):
    L = lsb_built
    monkeypatch.setenv("LSB_VMM_CHUNK_MIB", "2")
    n = 8 * (1 << 21)
    w = L.World(n, ranks=8, radix_bits=16)
    w.set_option(L.OPT_EXCHANGE_GATHER, 1)
    w.generate()
    w.set_option(L.OPT_FAIL_ONESWEEP, 11)  # ranks 0-7 queued pass 0, ranks 0-2 pass 1
    with pytest.raises(L.LsbError):
        w.my_sort()
    w.close()
    _fresh_sort(L, n, 8, 16)


def test_debug_build_teardown_check_stays_quiet(lsb_built):
    """The same sequences under the debug build: teardown_check finds every
    stream idle before any record buffer is freed."""
    assert os.path.exists(DEBUG_LIB), "make -C distributed-lsb_amd debug"
    env = dict(os.environ, LSB_LIBRARY=DEBUG_LIB)
    env.pop("LSB_TEARDOWN_LEGACY", None)
    p = subprocess.run([sys.executable, "-u", PROBE, "--per", str(1 << 21)], capture_output=True, text=True,
                       timeout=180, cwd=ROOT, env=env)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert lines, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    r = json.loads(lines[-1])
    assert r["library"].endswith("debug/liblsb.so")
    assert r["sorted_then_fresh_ok"] and r["failed_sort_raised"] and r["failed_then_fresh_ok"], r
    assert "teardown check" not in p.stderr, p.stderr[-3000:]
    assert p.returncode == 0


def test_peer_world_of_one_then_regional_sort(lsb_built, oracle_mod, monkeypatch):
    """Advisor r05: peer_setup's hipMalloc'd replacements of VMM buffers hold
    r.cap records, so the regional first pass of a later sort stays inside."""
    L = lsb_built
    monkeypatch.setenv("LSB_VMM_CHUNK_MIB", "2")
    monkeypatch.setenv("LSB_REGION_MIN", str(1 << 16))
    n = (1 << 20) + 77
    w = L.World.rank(n, 1, 0, 0, L.get_unique_id(), radix_bits=16)
    try:
        w.set_option(L.OPT_FORCE_EXCHANGE, 1)
        w.set_option(L.OPT_EXCHANGE_PEER, 1)
        w.generate()
        inp = w.copy_out(0)
        w.my_sort()
        w.sync()
        assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(inp))
        w.set_option(L.OPT_FORCE_EXCHANGE, 0)
        w.set_option(L.OPT_EXCHANGE_PEER, 0)
        for _ in range(2):
            w.generate()
            w.my_sort()
            assert w.first_pass() == L.FIRST_REGIONAL
            assert w.verify() == (True, -1)
    finally:
        w.close()


def test_failed_layout_pass_keeps_the_input(lsb_built, oracle_mod, monkeypatch):
    """Advisor r05: the regional first pass ran, the pass that reads its layout
    fails to launch (LSB_OPT_FAIL_ONESWEEP = 2): A holds the input again, and
    the next sort on the context sorts it exactly."""
    L = lsb_built
    monkeypatch.setenv("LSB_REGION_MIN", str(1 << 16))
    n = (1 << 20) + 4097
    with L.World(n, ranks=1) as w:
        w.generate()
        inp = w.copy_out(0)
        w.set_option(L.OPT_FAIL_ONESWEEP, 2)
        with pytest.raises(L.LsbError):
            w.my_sort()
        assert np.array_equal(w.copy_out(0), inp)
        w.my_sort()
        assert w.first_pass() == L.FIRST_REGIONAL
        assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(inp))
        assert w.verify() == (True, -1)
