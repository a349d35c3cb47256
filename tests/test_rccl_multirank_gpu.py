"""The multi-GPU data path between REAL RCCL ranks, on the one GPU we have.

RCCL refuses two ranks of one host on one device, but it decides "one host"
by NCCL_HOSTID when that is set.  tools/rccl_two_ranks.py starts P processes
on the GPU, each with its own NCCL_HOSTID, so RCCL connects them with its
socket transport over loopback.  Every collective of the N > 1 path then runs
between real ranks with non-empty peer segments: the counts ncclAllGather,
the sliced ncclAllToAllv or grouped ncclSend/ncclRecv of the records
(mpi/mpi_lsbsort.cpp:316-324, :563), the span all-gather, the whole-key
form's splitter-search all-gathers, verify's all-reduce.  The output must be
the reference's golden digest for `mpirun -n P mpi_lsbsort --n n`.

The wire here is a socket, not xGMI, so nothing is timed.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "rccl_two_ranks.py")


def _run(bits, n, world, exchange="alltoallv", slices=0, dist="uniform", dump="", env=None):
    p = subprocess.run([sys.executable, "-u", TOOL, str(bits), str(n), str(world), exchange, str(slices),
                        dist, dump],
                       capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, **(env or {})))
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert lines, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    return p.returncode, json.loads(lines[-1])


@pytest.mark.parametrize("bits,n,world,exchange,slices", [
    (8, 1_000_000, 2, "alltoallv", 0),
    (16, 1_000_000, 2, "p2p", 1),
    (16, 1_000_003, 4, "alltoallv", 7),
    (64, 1_000_003, 4, "p2p", 0),
    (16, 1_048_576, 8, "alltoallv", 0),
    (64, 1_048_576, 8, "alltoallv", 0),
])
def test_real_rccl_ranks_golden(lsb_built, bits, n, world, exchange, slices):
    rc, r = _run(bits, n, world, exchange, slices)
    assert r["status"] == "ok", r
    assert r["golden_match"] is True, r
    assert all(r["verify"]) and all(r["check_sorted"]), r
    # every rank handed records to RCCL (its peers' segments are non-empty)
    assert all(b > 0 for b in r["rccl_bytes"]), r
    assert rc == 0


@pytest.mark.parametrize("bits,n,world,exchange", [
    (16, 1_000_003, 4, "alltoallv"),
    (64, 1_000_003, 4, "p2p"),
    (16, 1_048_576, 8, "alltoallv"),
    (64, 1_048_576, 8, "alltoallv"),
])
def test_real_rccl_ranks_zipf(lsb_built, oracle_mod, tmp_path, bits, n, world, exchange):
    """configs[3]'s skew through real RCCL ranks: Zipf (s = 1.1) keys make
    per-pair exchange volumes uneven and duplicate keys test stability across
    ranks (the reference's exchange, mpi/mpi_lsbsort.cpp:527-576).  The
    reference has no Zipf input, so the check is the oracle's stable sort of
    the gathered input, bit for bit, plus lsb_verify on every rank."""
    import numpy as np
    rc, r = _run(bits, n, world, exchange, 0, "zipf", str(tmp_path))
    assert r["status"] == "ok", r
    assert all(r["verify"]) and all(r["check_sorted"]), r
    assert all(b > 0 for b in r["rccl_bytes"]), r
    assert rc == 0
    inp = np.concatenate([np.load(tmp_path / f"in_{q}.npy") for q in range(world)])
    out = np.concatenate([np.load(tmp_path / f"out_{q}.npy") for q in range(world)])
    assert inp.size == n and np.unique(inp["key"]).size < n // 2  # heavy duplicates
    assert np.array_equal(out, oracle_mod.stable_sort(inp))


@pytest.mark.parametrize("bits,n,world,exchange", [
    (16, 1_000_003, 4, "alltoallv"),
    (64, 1_000_000, 2, "p2p"),
])
def test_real_rccl_ranks_vmm_pieces(lsb_built, bits, n, world, exchange):
    """Record buffers built from 2 MiB VMM pieces (LSB_VMM_CHUNK_MIB=2; at
    2^30 records per rank they are 1 GiB pieces) as RCCL's send and receive
    buffers between real ranks: the golden digest, every rank verified."""
    rc, r = _run(bits, n, world, exchange, env={"LSB_VMM_CHUNK_MIB": "2"})
    assert r["status"] == "ok", r
    assert r["golden_match"] is True, r
    assert all(r["verify"]) and all(r["check_sorted"]), r
    assert all(b > 0 for b in r["rccl_bytes"]), r
    assert rc == 0


def test_real_rccl_ranks_two_gib_segments(lsb_built):
    """Two real ranks of 2^28 records each, one slice per exchange: each
    rank's segment to its peer is ~2 GiB per call, which RCCL moves wrongly in
    one piece; the runtime cuts it into calls of at most 1 GiB per peer
    (coll_alltoallv_u64).  Verified on device on both ranks."""
    rc, r = _run(16, 1 << 29, 2, "alltoallv", 1)
    assert r["status"] == "ok", r
    assert all(r["verify"]) and all(r["check_sorted"]), r
    assert all(b >= (1 << 31) for b in r["rccl_bytes"]), r  # >= 2 GiB handed to RCCL per rank
    assert rc == 0


@pytest.mark.parametrize("bits,n,world,exchange", [
    (16, 1_000_000, 2, "alltoallv"),
    (16, 1_048_576, 8, "p2p"),
    (64, 1_000_003, 4, "alltoallv"),
])
def test_real_rccl_ranks_cut_calls(lsb_built, bits, n, world, exchange):
    """The cut of RCCL calls between real ranks (advisor r05): with the per-peer
    call bound lowered to 4096 u64 (LSB_RCCL_CALL_U64; 2^27 by default) every
    slice goes as several calls, and at P > 1 the per-digit exchange agrees on
    the cut through its all-reduce of the largest peer segment.  The golden
    digest, every rank verified, and no call above the bound."""
    bound = 4096
    rc, r = _run(bits, n, world, exchange, env={"LSB_RCCL_CALL_U64": str(bound)})
    assert r["status"] == "ok", r
    assert r["golden_match"] is True, r
    assert all(r["verify"]) and all(r["check_sorted"]), r
    assert all(b > 0 for b in r["rccl_bytes"]), r
    assert all(m <= world * bound * 8 for m in r["rccl_max_call_bytes"]), r
    assert rc == 0
