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


# ---- the N > 1 launch (no GPU: --dry-rank runs the plumbing only) ----------
# `python bench.py --gpus N` without a launcher starts the N rank processes
# itself, as `mpirun -n N` starts the reference's ranks (mpi/README.md:24-28);
# under torch.distributed.run the launcher's processes are the ranks.  Either
# way the whole-key extra runs in fresh processes after the headline.
def _bench(args, env=None, timeout=240):
    import subprocess
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT, env=env)


def _line(stdout):
    import json
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_self_launch_relays_rank0_line():
    r = _bench(["--gpus", "3", "--dry-rank", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 3 and out["max_rank"] == 2.0  # all three ranks joined one group
    assert out["launcher"].startswith("bench.py started 3 rank processes")
    # the whole-key extra ran in its own rank processes, with the 64-bit digit
    assert out["whole_key_melem_s"] == 3 * 64 and out["whole_key_verified"] is True
    # so did the peer-store extra, with the headline's 16-bit digits
    assert out["peer_melem_s"] == 3 * 16 and out["peer_verified"] is True
    assert out["peer_exchange_roofline"]["bound"] == "xgmi"
    assert out["cpu_baseline"] is None


def test_exchange_roofline_keys():
    """N > 1: the line carries the exchange side of SURVEY 8(d) (bench.py
    exchange_roofline, here from dry_stats' made-up per-rank bytes: rank r
    sends (r + 1) MiB per peer per exchange, 4 exchanges per sort)."""
    r = _bench(["--gpus", "3", "--dry-rank", "--no-cpu-baseline", "--no-extras", "--steps", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    x = _line(r.stdout)["exchange_roofline"]
    assert x["bound"] == "xgmi" and x["unit"] == "GB/s" and x["peak"] == 153.0 and "spec" in x["peak_source"]
    assert x["exchanges_per_sort"] == 4
    mib = 1 << 20
    assert x["link_bytes_per_exchange"] == {"max": 3 * mib, "min": mib}
    assert x["link_bytes_per_sort"]["max_link"][0] == 2 and x["link_bytes_per_sort"]["min_link"][0] == 0
    assert x["link_bytes_per_sort"]["max_over_min"] == 3.0
    assert x["rank_bytes_per_sort"] == {"max": 2 * 4 * 3 * mib, "min": 2 * 4 * mib}
    # wire: 1 ms per exchange -> the busiest link moved 12 MiB in 4 ms
    assert x["wire_ms_per_sort"]["max"] == 4.0
    assert x["achieved"] == round(12 * mib / 4e-3 / 1e9, 2)
    assert x["frac"] == round(x["achieved"] / 153.0, 4)
    assert x["link_bound_ms_per_sort"] == round(12 * mib / 153e9 * 1e3, 3)
    p = x["place"]
    assert p["tail_ms_per_sort"] == 0.5 and p["ms_per_sort"] == 2.0 and p["overlapped_frac"] == 0.75
    assert p["placed_records_per_sort"] == 1000 and p["counted_records_per_sort"] == 3000


def test_peer_failure_keeps_the_headline():
    r = _bench(["--gpus", "2", "--dry-rank", "--dry-fail-peer", "1", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["value"] == 2 * 16 and out["whole_key_melem_s"] == 2 * 64
    assert "peer_melem_s" not in out and "rank exit codes" in out["peer_error"]


def test_self_launch_fails_with_the_failing_rank():
    r = _bench(["--gpus", "2", "--dry-rank", "--dry-fail", "1", "--no-cpu-baseline"])
    assert r.returncode == 1
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "rank exit codes" in r.stderr and "rank 1" in r.stderr


def test_whole_key_failure_keeps_the_headline():
    r = _bench(["--gpus", "2", "--dry-rank", "--dry-fail-whole-key", "0", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["value"] == 2 * 16 and "whole_key_melem_s" not in out
    assert "whole_key_error" in out and "rank exit codes" in out["whole_key_error"]
    assert out["peer_melem_s"] == 2 * 16


@pytest.mark.parametrize("fail_extra", [False, True])
def test_torchrun_ranks_run_the_extra_in_child_processes(fail_extra):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dry-rank", "--no-cpu-baseline"]
    if fail_extra:
        cmd += ["--dry-fail-whole-key", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 2 and out["value"] == 32.0
    if fail_extra:  # every rank agreed the extra failed; the headline stands
        assert "whole_key_error" in out and "whole_key_melem_s" not in out
    else:
        assert out["whole_key_melem_s"] == 128.0
    assert out["peer_melem_s"] == 32.0 and out["exchange_roofline"]["exchanges_per_sort"] == 4


def test_eight_rank_dry_launch():
    """The driver's largest scaling case (N = 8, `python bench.py --gpus 8`)
    through the whole host path: eight rank processes, the all-gathered
    exchange stats of eight ranks (7 peers each), both extras in fresh
    processes, one line from rank 0."""
    r = _bench(["--gpus", "8", "--dry-rank", "--no-cpu-baseline", "--steps", "2", "--warmup", "1"],
               timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 8 and out["max_rank"] == 7.0 and out["value"] == 8 * 16
    assert out["whole_key_melem_s"] == 8 * 64 and out["whole_key_verified"] is True
    assert out["peer_melem_s"] == 8 * 16 and out["peer_verified"] is True
    x = out["exchange_roofline"]
    mib = 1 << 20
    # dry_stats: rank r sends (r + 1) MiB to each of its 7 peers per exchange
    assert x["link_bytes_per_exchange"] == {"max": 8 * mib, "min": mib}
    assert x["rank_bytes_per_sort"] == {"max": 7 * 4 * 8 * mib, "min": 7 * 4 * mib}
    assert x["link_bytes_per_sort"]["max_link"][0] == 7 and x["link_bytes_per_sort"]["max_over_min"] == 8.0


# ---- N = 1: the extras after the headline -------------
def test_one_gpu_line_carries_hybrid_x16_and_c5_keys():
    """N = 1 runs two extras in fresh processes: the hybrid local sort and
    x16, the reference's 16-bit digit (BASELINE configs[4]) with its exchange
    path forced through a world-of-one RCCL communicator (--force-exchange);
    both are priced against SURVEY 8(d)'s C5 denominator (192 B per record)."""
    r = _bench(["--dry-rank", "--no-cpu-baseline", "--steps", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 1 and out["value"] == 8.0 and out["verified"] is True
    assert out["hybrid_melem_s"] == 8.0 and out["hybrid_verified"] is True
    assert out["x16_melem_s"] == 16.0 and out["x16_verified"] is True  # --radix-bits 16
    x = out["x16_exchange_roofline"]
    assert x["bound"] == "self" and x["peak"] is None and x["frac"] is None
    mib = 1 << 20
    assert x["link_bytes_per_exchange"] == {"max": mib, "min": mib} and x["exchanges_per_sort"] == 4
    assert x["place"]["tail_ms_per_sort"] == 0.5 and x["place"]["ms_per_sort"] == 2.0
    assert out["x16_per_pass"][0]["place_tail_ms"] == 0.125
    frac = round(192 * (1 << 30) / 1e-3 / 8e12, 4)  # dry lines report 1 ms per step
    assert out["hybrid_c5_survey_frac"] == frac and out["x16_c5_survey_frac"] == frac
    assert "two stable 8-bit passes" in out["c5_basis"]


def test_x16_failure_keeps_the_headline():
    r = _bench(["--dry-rank", "--no-cpu-baseline", "--steps", "2", "--dry-fail-x16", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["value"] == 8.0 and out["hybrid_melem_s"] == 8.0
    assert "x16_melem_s" not in out and "rank exit codes" in out["x16_error"]


@pytest.mark.parametrize("form", ["x16", "hybrid"])
def test_wrong_extra_output_fails_the_run(form):
    """An extra whose output fails lsb_verify fails the run (exit 1), as the
    headline does, but its line is still printed (advisor r04)."""
    r = _bench(["--dry-rank", "--no-cpu-baseline", "--steps", "2", "--dry-unverified", form])
    assert r.returncode == 1
    out = _line(r.stdout)
    assert out["verified"] is True and out[f"{form}_verified"] is False


def test_wrong_peer_output_fails_the_run():
    r = _bench(["--gpus", "2", "--dry-rank", "--no-cpu-baseline", "--steps", "2", "--dry-unverified", "peer"])
    assert r.returncode == 1
    out = _line(r.stdout)
    assert out["verified"] is True and out["peer_verified"] is False and out["whole_key_verified"] is True


@pytest.mark.parametrize("candidates", [None, "8"])
def test_eight_rank_memory_fits_the_device(candidates):
    """at the driver's N = 8 (2^30 records per GPU) one
    rank's A, B, R, look-back rows and tables fit one MI355X (288 GB, the
    dry run's stand-in for lsb_device_memory), with the placement probe's
    default 4 candidates and with 8 (LSB_PLACEMENT_CANDIDATES=8), and a
    failing peer extra keeps the headline line."""
    env = dict(os.environ)
    env.pop("LSB_PLACEMENT_CANDIDATES", None)
    if candidates:
        env["LSB_PLACEMENT_CANDIDATES"] = candidates
    r = _bench(["--gpus", "8", "--dry-rank", "--no-cpu-baseline", "--steps", "2", "--warmup", "1",
                "--dry-fail-peer", "5", "--no-whole-key"], env=env, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["value"] == 8 * 16 and "rank exit codes" in out["peer_error"]
    m = out["device_memory"]
    gib = 1 << 30
    assert 48 * gib <= m["bytes"] < 49 * gib  # A, B, R of 16 GiB each + 1/64 look-back rows
    assert m["probe_bytes"] == 16 * gib  # one candidate beside A and B at a time, whatever K
    assert m["device_bytes"] == 288 * 10**9 and m["fits"] and m["peak_frac"] < 0.9


def test_chunked_extra_at_n2():
    """N > 1 with 16-bit digits: the chunked exchange (LSB_OPT_EXCHANGE_CHUNKS =
    8) is timed as the chunked_* extra beside the headline, verified like the
    others; a wrong chunked output fails the run."""
    r = _bench(["--gpus", "2", "--dry-rank", "--no-cpu-baseline", "--steps", "2", "--no-whole-key", "--no-peer"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["chunked_melem_s"] == 2 * 16 and out["chunked_verified"] is True
    r = _bench(["--gpus", "2", "--dry-rank", "--no-cpu-baseline", "--steps", "2", "--no-whole-key", "--no-peer",
                "--dry-unverified", "chunked"])
    assert r.returncode == 1
    assert _line(r.stdout)["chunked_verified"] is False
