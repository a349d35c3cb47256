#!/usr/bin/env python3
"""Benchmark of the MI355X LSD radix sort (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step is one full sort (mySort: 8 local passes of 8-bit digits over 64-bit
keys) of 2^30 16-byte records per GPU (weak scaling: n = N * 2^30), generated on
device with the reference's PCG64 input (seed = rank, val = global index;
mpi/mpi_lsbsort.cpp:650-656) before every step, outside the timed window —
the reference times the sort only (mpi/mpi_lsbsort.cpp:688-699).  Each step
is bracketed by a barrier + device synchronize on both sides; the time is
the max over ranks.  The result of the last step is verified on device
(bit-exact stable-sort invariant, lsb_verify).

Multi-GPU: one process per GPU (RANK / WORLD_SIZE / LOCAL_RANK from the
environment).  torch.distributed (gloo, CPU) only ships the RCCL unique id
and reduces timings; the data path is the library's own RCCL communicator.
`python bench.py --gpus N` with no launcher starts the N rank processes
itself (the way `mpirun -n N` starts the reference's ranks,
mpi/README.md:24-28): this parent never touches HIP; it relays rank 0's line
and fails with the failing rank's stderr tail.  Under torch.distributed.run
the ranks are the launcher's processes.  Either way the whole-key extra runs
in fresh rank processes of its own after the headline is measured, so a
failure there costs only its own keys.
At N > 1 the headline is the reference's own structure (BASELINE configs[2],
configs[3]): per 16-bit digit (the reference's RADIX 16) an RCCL AllGather
of the counts and an RCCL AllToAllv of the records (--radix-bits 16;
--radix-bits 8 exchanges per 8-bit digit).  The whole-key exchange (local
sort, one sliced all-to-all, merge) is timed after it and
reported as an extra key (whole_key_melem_s), not as `value`.

The JSON line carries the roofline of the dominant kernel (k_onesweep, or
k_scatter: 32 algorithmic bytes per record per launch, timed with HIP events
on the library's stream), its HBM traffic measured in this run (N = 1: two
rocprofv3 --pmc passes, FETCH_SIZE and WRITE_SIZE, over one sort of the same
workload), and, on rank 0, a CPU baseline: the reference's own mpi_lsbsort
(oracle/_ref, built from /root/reference) on the host's cores, median of 3.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))

import lsbsort  # noqa: E402

METRIC = "Melem/s (16-byte elems) at 1/2/4/8 GPUs; per-pass HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
SCATTER_BYTES_PER_ELEM = 32     # 16 B read + 16 B written per record per pass
COUNT_BYTES_PER_ELEM = 16       # histogram read of the keys' lines
SAMPLE_RECORDS = 1 << 20        # the regional first pass's sample (256 tiles of 4096 records)
REF_MPI_MELEMS = 830.0          # mpi_lsbsort, 64 nodes x 128 cores, n = 2^36
XGMI_LINK_GBS = 153.0           # per xGMI link of an MI355X (spec figure, see XGMI_PEAK_SOURCE)
XGMI_PEAK_SOURCE = ("spec figure, not measured here: MI355X, 7 xGMI links x ~153 GB/s per GPU, one direct link "
                    "per GPU pair on an 8-GPU node (task brief; SURVEY.md 5 and 8(d), which prices the per-pass "
                    "exchange as 16*m/P bytes per link at 153 GB/s); frac = the busiest link's bytes in one "
                    "direction / its sender's wire time / 153 GB/s")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n-per-gpu", type=int, default=1 << 30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-n", type=int, default=0,
                    help="records the CPU baseline sorts (default: the GPU run's n, capped by host "
                         "memory and a ~20 s per-run budget, as a power of two)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 --pmc passes that measure the dominant kernel's HBM bytes")
    ap.add_argument("--no-whole-key", action="store_true",
                    help="N > 1: skip the extra whole-key exchange timing")
    ap.add_argument("--no-peer", action="store_true",
                    help="N > 1: skip the extra peer-store exchange timing (LSB_OPT_EXCHANGE_PEER)")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-rank", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail-whole-key", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail-peer", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail-x16", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-unverified", default="", help=argparse.SUPPRESS)
    ap.add_argument("--rank-timeout", type=int, default=1500,
                    help="self-launched rank processes: seconds before they are stopped")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--radix-bits", type=int, default=0, choices=(0, 8, 16, 64),
                    help="exchange digit width: 8 or 16 (one all-to-all per digit), or 64 (the "
                         "whole key: local sort, ONE all-to-all, merge); default 8 on 1 GPU, 16 on "
                         ">1 GPU; local passes are 8-bit either way")
    ap.add_argument("--dist", choices=("uniform", "zipf"), default="uniform")
    ap.add_argument("--transport", choices=("rccl", "rccl-sockets", "gloo"), default="rccl",
                    help="N > 1 collectives: RCCL over xGMI (the measurement); RCCL between ranks "
                         "that share GPUs, one NCCL_HOSTID per rank so RCCL links them by its socket "
                         "transport (a rehearsal of the RCCL path on fewer GPUs); or gloo host "
                         "callbacks (lsb_create_rank_ops)")
    ap.add_argument("--exchange", choices=("alltoallv", "p2p", "peer"), default="alltoallv",
                    help="N > 1 element exchange: RCCL AllToAllv in slices (default), grouped "
                         "ncclSend/ncclRecv, or direct peer stores into the owners' buffers")
    ap.add_argument("--exchange-chunks", type=int, choices=(0, 2, 4, 8), default=0,
                    help="16-bit exchange digits sent in C chunks while the high-byte pass runs chunk by "
                         "chunk (LSB_OPT_EXCHANGE_CHUNKS; 0: after the whole pass).  N > 1 reports C = 8 "
                         "as the chunked_* extra")
    ap.add_argument("--zipf-s", type=float, default=1.1)
    ap.add_argument("--passes", choices=("onesweep", "reduce-scan", "hybrid"), default="onesweep",
                    help="local pass form: single-read (look-back), count + scan + scatter, or the "
                         "hybrid (single-read passes on the top bytes, then one segmented local sort; "
                         "LSB_OPT_HYBRID, P = 1 and the whole-key form's local sorts)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra forms timed after the headline (hybrid and x16 at N = 1, whole key, "
                         "peer and chunked at N > 1)")
    ap.add_argument("--force-exchange", action="store_true",
                    help="N = 1: run the exchange path anyway, over a world-of-one RCCL communicator that "
                         "carries every record through ncclAllToAllv (LSB_OPT_FORCE_EXCHANGE + "
                         "LSB_OPT_EXCHANGE_SELF); the x16 extra is this with --radix-bits 16")
    return ap.parse_args()


class Dist:
    """Rank bookkeeping: torch.distributed (gloo) when WORLD_SIZE > 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def bcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        return self.max_list([x])[0]

    def max_list(self, xs):
        """Element-wise max over ranks."""
        if not self.dist:
            return list(xs)
        import torch
        t = torch.tensor(list(xs), dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return [float(v) for v in t.tolist()]

    def all_gather_obj(self, obj):
        """[obj of rank 0, obj of rank 1, ...] on every rank."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def all_true(self, ok):
        if not self.dist:
            return ok
        import torch
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return bool(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


class GlooComm:
    """lsb_comm_ops_t over torch.distributed gloo, on host byte buffers.

    For `--transport gloo` (rehearsing the N > 1 flow where RCCL is not
    available, e.g. several ranks on one GPU) and the multi-process tests.
    """

    def __init__(self, dist, world, rank):
        import torch
        self.torch, self.dist, self.world, self.rank = torch, dist, world, rank

    def allgather(self, send):
        t = self.torch.from_numpy(send)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return self.torch.cat(out).numpy()

    def alltoallv(self, send, sc, sd, recv, rc, rd):
        reqs, bufs = [], []
        for q in range(self.world):
            if q == self.rank:
                if sc[q]:
                    recv[rd[q]:rd[q] + rc[q]] = send[sd[q]:sd[q] + sc[q]]
                continue
            if sc[q]:
                reqs.append(self.dist.isend(self.torch.from_numpy(send[sd[q]:sd[q] + sc[q]].copy()), q))
            if rc[q]:
                buf = self.torch.empty(rc[q], dtype=self.torch.uint8)
                reqs.append(self.dist.irecv(buf, q))
                bufs.append((buf, rd[q]))
        for r in reqs:
            r.wait()
        for buf, off in bufs:
            recv[off:off + buf.numel()] = buf.numpy()

    def allreduce_min(self, v):
        t = self.torch.tensor([v], dtype=self.torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return int(t[0])

    def barrier(self):
        self.dist.barrier()


def visible_devices():
    """HIP devices this process can see (device_count does not initialize HIP)."""
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 1


_TORCH_DEV = None


def bind_device(local_rank):
    """Point torch at this rank's GPU so its synchronize() waits on that device."""
    global _TORCH_DEV
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank)
            _TORCH_DEV = local_rank
    except Exception:
        _TORCH_DEV = None


def device_sync():
    if _TORCH_DEV is None:
        return
    import torch
    torch.cuda.synchronize(_TORCH_DEV)


def measure_traffic(a, kernel, elems):
    """HBM bytes per launch of `kernel`, measured now: two rocprofv3 --pmc
    passes (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass) over one
    sort of the same workload (this script with --probe), combined as
    MI355X_MICROARCH.md §HBM prescribes for gfx950: 2 * FETCH_SIZE (it counts
    half of a 16 B/lane stream) + WRITE_SIZE, in KB.  None when rocprofv3 is
    absent or a pass fails."""
    import collections
    import csv
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    probe = [sys.executable, os.path.abspath(__file__), "--probe", "--n-per-gpu", str(a.n_per_gpu),
             "--dist", a.dist, "--zipf-s", str(a.zipf_s), "--passes", a.passes,
             "--radix-bits", str(a.radix_bits or 8)]
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", "120", prof, "--kernel-trace", "--pmc", counter,
                   "--kernel-include-regex", kernel, "--output-format", "csv", "-d", out, "-o", "run",
                   "--"] + probe
            try:
                subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, timeout=150, check=True)
            except (subprocess.SubprocessError, OSError) as e:
                return None, f"rocprofv3 --pmc {counter} failed: {type(e).__name__}"
            per = collections.defaultdict(list)
            for root, _, files in os.walk(out):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        for r in csv.DictReader(open(os.path.join(root, f))):
                            name = r["Kernel_Name"]
                            # the placement probe's passes at context creation
                            # run as k_onesweep_probe: not the sort's launches
                            if r["Counter_Name"] == counter and kernel in name and "_probe" not in name:
                                per[r.get("Dispatch_Id", len(per))].append(float(r["Counter_Value"]))
            if not per:
                return None, f"no {counter} rows for {kernel}"
            vals[counter] = sum(sum(v) for v in per.values()) / len(per)
    hbm = (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024
    return hbm, (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes in this run, one sort, {kernel} "
                 f"launches averaged; hbm = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 "
                 f"(algorithmic {SCATTER_BYTES_PER_ELEM * elems:.4g} B per launch)")


def host_cores():
    """Core counts of this host: nproc, lscpu's physical cores, and this
    job's CPU share (OMP_NUM_THREADS as the GPU pool sets it per job, else the
    cgroup quota, else the affinity mask)."""
    total = os.cpu_count() or 1
    try:
        rows = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True,
                              timeout=10).stdout.splitlines()
        physical = len({r for r in rows if r and not r.startswith("#")}) or None
    except (subprocess.SubprocessError, OSError):
        physical = None
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = total
    share, basis = affinity, "affinity mask"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            share, basis = min(share, max(1, int(int(q) / int(per)))), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0 and int(omp) < share:
        share, basis = int(omp), "OMP_NUM_THREADS (the job's CPU share)"
    return {"nproc": total, "physical": physical, "affinity": affinity, "share": share,
            "share_basis": basis}


def cpu_baseline(gpu_n, cpu_n=0, runs=3):
    """The reference's own MPI sort (mpi/mpi_lsbsort.cpp, oracle/_ref) on this
    host, per BASELINE.md §4: one rank per core of the job's CPU share (at
    least 5 ranks), n = the GPU run's n or the largest power of two that fits
    ~80 B per record of host memory and a ~20 s per-run budget, the median of
    `runs` runs of its sort-only window (mpi/mpi_lsbsort.cpp:688-699)."""
    cores = host_cores()
    ranks = max(5, cores["share"])
    ref = os.path.join(ROOT, "oracle", "_ref", "mpi_lsbsort")
    mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
    if not (os.path.exists(ref) and os.path.exists(mpirun)):
        return None
    try:
        import psutil
        avail = psutil.virtual_memory().available
    except Exception:
        avail = 32 << 30
    if cpu_n:
        n, why = cpu_n, "requested"
    else:
        mem_cap = min(avail * 0.6, 200 << 30) / 80
        time_cap = 20 * 4e6 * ranks  # the reference sorts ~4-6 M records/s per rank
        n, why = gpu_n, "the GPU run's n"
        if n > mem_cap or n > time_cap:
            n = 1 << int(min(mem_cap, time_cap, gpu_n)).bit_length() - 1
            why = ("largest power of two within " +
                   ("host memory (80 B/record)" if mem_cap < time_cap else "a ~20 s per-run budget"))
    vals = []
    cmd = [mpirun, "-n", str(ranks), ref, "--n", str(n), "--no-verify"]
    for _ in range(runs):
        try:
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True).stdout
        except (subprocess.SubprocessError, OSError):
            break
        m = re.search(r"That's ([0-9.eE+-]+) M elements sorted / s", out)
        if not m:
            break
        vals.append(float(m.group(1)))
    if not vals:
        return None
    med = sorted(vals)[len(vals) // 2]
    return {"value": med, "unit": "Melem/s", "cores": ranks, "kind": "reference",
            "n": n, "n_basis": why, "ranks": ranks, "runs": vals, "median": med,
            "cores_total": cores["nproc"], "cores_physical": cores["physical"],
            "cores_share": cores["share"], "cores_share_basis": cores["share_basis"],
            "cores_used": ranks,
            "sample": f"mpirun -n {ranks} oracle/_ref/mpi_lsbsort --n {n} --no-verify (the reference "
                      f"mpi/mpi_lsbsort.cpp, 16-bit digits, its sort-only window), median of {len(vals)}"}


def parallelism(N, radix, a):
    if N == 1:
        return "1 GPU, no exchange"
    if a.transport == "gloo":
        return f"{N} ranks, gloo host collectives (rehearsal, not a measurement)"
    if a.transport == "rccl-sockets":
        return (f"{N} ranks, RCCL between ranks sharing GPUs over its socket transport "
                f"(rehearsal of the RCCL path, not a measurement)")
    if radix == 64:
        return (f"block partition over {N} GPUs; local sort per GPU" +
                (" (hybrid)" if a.passes == "hybrid" else "") + ", splitter search (8 RCCL AllGathers "
                f"of candidate counts), one RCCL " + ("AllToAllv" if a.exchange == "alltoallv" else
                                                       "grouped Send/Recv") +
                ", stable merge tree of the P runs")
    return (f"block partition over {N} GPUs; per exchange digit RCCL AllGather of counts + " +
            {"alltoallv": "AllToAllv in 5 halving slices", "p2p": "grouped Send/Recv in 5 halving slices",
             "peer": "direct peer stores (IPC)"}[a.exchange])


def make_world(a, d, N, n_total, radix):
    """The sort context of this process: one rank of an RCCL world (N > 1),
    one rank over gloo host collectives (--transport gloo), or one GPU."""
    if d.world > 1 and a.transport == "gloo":
        # Rehearsal: ranks may share GPUs; collectives go through gloo on the host.
        device = d.local_rank % max(1, visible_devices())
        w = lsbsort.World.rank_ops(n_total, N, d.rank, device, GlooComm(d.dist, d.world, d.rank),
                                   radix_bits=radix)
    elif d.world > 1:
        # One GPU per rank; the modulo keeps a launcher that narrows each
        # rank's visible devices (HIP_VISIBLE_DEVICES) on that rank's GPU.
        device = d.local_rank % max(1, visible_devices())
        if a.transport == "rccl-sockets":
            # Ranks may share a GPU: RCCL accepts that only across "hosts",
            # so each rank is its own host and the wire is a loopback socket.
            os.environ["NCCL_HOSTID"] = f"lsb-bench-rank-{d.rank}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")
            device = d.local_rank % max(1, visible_devices())
        uid = lsbsort.get_unique_id() if d.rank == 0 else None
        uid = d.bcast_bytes(uid)
        w = lsbsort.World.rank(n_total, N, d.rank, device, uid, radix_bits=radix)
    elif a.force_exchange:
        # One rank of a world of one: the exchange path with the rank's own
        # records through RCCL (BASELINE configs[4]'s exchange structure).
        if N != 1:
            raise SystemExit("--force-exchange is a one-GPU form")
        device = 0
        w = lsbsort.World.rank(n_total, 1, 0, device, lsbsort.get_unique_id(), radix_bits=radix)
        w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
        w.set_option(lsbsort.OPT_EXCHANGE_SELF, 1)
    else:
        if N != 1:
            raise SystemExit("multi-GPU runs are launched one process per GPU (torch.distributed.run)")
        device = 0
        w = lsbsort.World(n_total, ranks=1, radix_bits=radix)
    if a.exchange == "p2p":
        w.set_option(lsbsort.OPT_EXCHANGE_P2P, 1)
    elif a.exchange == "peer" and radix != 64:
        w.set_option(lsbsort.OPT_EXCHANGE_PEER, 1)
    w.set_option(lsbsort.OPT_ONESWEEP, 0 if a.passes == "reduce-scan" else 1)
    w.set_option(lsbsort.OPT_HYBRID, 1 if a.passes == "hybrid" else 0)
    if a.exchange_chunks:
        w.set_option(lsbsort.OPT_EXCHANGE_CHUNKS, a.exchange_chunks)
    return w, device


def timed_sorts(w, d, a, steps, warmup):
    """`warmup` untimed sorts, then `steps` timed ones; each step regenerates
    the input (untimed) and times the sort between barrier + synchronize
    brackets.  Returns (max-over-ranks total seconds, verified or None,
    per-step max-over-ranks seconds)."""
    def step():
        w.generate(a.dist, a.zipf_s)
        w.barrier()
        device_sync()
        d.barrier()
        t0 = time.perf_counter()
        w.my_sort()
        w.barrier()
        device_sync()
        d.barrier()
        return time.perf_counter() - t0

    for _ in range(warmup):
        step()
    w.reset_kernel_stats()
    w.set_timing(True)
    times = [step() for _ in range(steps)]
    w.set_timing(False)
    verified = None
    if not a.no_verify:
        ok, _ = w.verify()
        verified = d.all_true(ok)
    return d.max(sum(times)), verified, d.max_list(times)


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_env(rank, world, local_rank, port, master="127.0.0.1"):
    """Environment of one rank process, as torch.distributed.run sets it.  A
    launcher's own agent-store variables are dropped: the child forms a new
    group on its own port (TORCHELASTIC_USE_AGENT_STORE would make every
    child a client of a store nobody serves)."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local_rank),
               LOCAL_WORLD_SIZE=str(world), MASTER_ADDR=master, MASTER_PORT=str(port))
    return env


def spawn_ranks(argv, ranks, timeout, label):
    """Run this script once per (rank, env) in `ranks` as fresh processes and
    wait.  Returns (ok, stdout of the first process, failure report).  When a
    process fails, the others get 60 s (they may be waiting in a collective
    the failed rank never joins) and are then stopped."""
    import tempfile
    tmp = tempfile.mkdtemp(prefix="lsb-bench-")
    procs = []
    for i, env in enumerate(ranks):
        out = open(os.path.join(tmp, f"{i}.out"), "w+")
        err = open(os.path.join(tmp, f"{i}.err"), "w+")
        p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                             stdout=out, stderr=err, start_new_session=True)
        procs.append((p, out, err))
    t0 = time.time()
    first_fail = None
    beat = t0
    while any(p.poll() is None for p, _, _ in procs):
        time.sleep(0.5)
        now = time.time()
        if first_fail is None and any(p.poll() not in (None, 0) for p, _, _ in procs):
            first_fail = now
        late = (first_fail is not None and now - first_fail > 60) or now - t0 > timeout
        if late:
            for p, _, _ in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, 9)  # the process group this call started
                    except OSError:
                        pass
            for p, _, _ in procs:
                p.wait()
            break
        if now - beat > 30:
            beat = now
            print(f"[bench] {label}: {len(procs)} rank processes running, {now - t0:.0f} s",
                  file=sys.stderr, flush=True)
    codes = [p.returncode for p, _, _ in procs]
    texts = []
    for _, out, err in procs:
        out.seek(0)
        err.seek(0)
        texts.append((out.read(), err.read()))
        out.close()
        err.close()
    shutil.rmtree(tmp, ignore_errors=True)
    ok = all(c == 0 for c in codes)
    report = ""
    if not ok:
        bad = [i for i, c in enumerate(codes) if c != 0]
        report = f"{label}: rank exit codes {codes}; " + " | ".join(
            f"rank {i} stderr tail: {texts[i][1][-1500:]}" for i in bad[:2])
    return ok, texts[0][0], report


def last_json(text):
    lines = [l for l in text.splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def extra_argv(a, flags, steps=3):
    """The command line of an extra form: this run's flags plus `flags`,
    fewer steps, no extras or CPU baseline of its own."""
    return sys.argv[1:] + flags + ["--steps", str(min(a.steps, steps)), "--warmup", "1",
                                   "--no-cpu-baseline", "--no-extras", "--no-traffic"]


def whole_key_argv(a):
    """The whole-key extra: the 64-bit exchange digit (a per-digit --exchange
    peer becomes AllToAllv), each rank's local sort by the hybrid (the
    fastest local sort; same output) unless --passes chose another form."""
    return extra_argv(a, ["--radix-bits", "64"] + (["--exchange", "alltoallv"] if a.exchange == "peer" else []) +
                      (["--passes", "hybrid"] if a.passes == "onesweep" else []))


def peer_argv(a):
    """The peer-store extra: the headline's per-digit exchange with direct
    stores into the owners' buffers (LSB_OPT_EXCHANGE_PEER; the reference's
    shmem_putmem / MPI_Put form, shmem/shmem_lsbsort.cpp:441-456,
    mpi/mpi_lsbsort_onesided.cpp:487-509), verified by lsb_verify."""
    return extra_argv(a, ["--exchange", "peer", "--radix-bits", str(a.radix_bits or 16)])


def extra_timeout(a):
    """Seconds an extra form's processes get (a few sorts of the workload):
    a hung extra costs its keys and this much of the run, not the headline."""
    return min(a.rank_timeout, 420)


def extras_at(a, N):
    """The extra forms timed after the headline, in fresh processes: (name,
    argv).  N > 1: the whole-key exchange, the chunked 16-bit exchange and
    the peer-store exchange (unless the headline already is that form);
    N = 1: the hybrid local sort and the forced 16-bit exchange (x16)."""
    if a.no_extras:
        return []
    radix = a.radix_bits or (8 if N == 1 else 16)
    if N == 1:
        if a.passes != "onesweep" or a.force_exchange:
            return []
        # the hybrid local sort, and the forced 16-bit exchange (x16): the
        # reference's own digit (configs[4]) with its exchange path run
        return [("hybrid", extra_argv(a, ["--passes", "hybrid"])),
                ("x16", extra_argv(a, ["--force-exchange", "--radix-bits", "16"]))]
    out = []
    if radix != 64 and not a.no_whole_key:
        out.append(("whole_key", whole_key_argv(a)))
    # the 16-bit exchange in chunks (LSB_OPT_EXCHANGE_CHUNKS = 8): each chunk's
    # records on the wire while the next chunk's high-byte pass runs
    if radix == 16 and a.exchange == "alltoallv" and not a.exchange_chunks and a.transport != "gloo":
        out.append(("chunked", extra_argv(a, ["--exchange-chunks", "8"])))
    # last: the only form whose kernels store into another GPU's memory (IPC
    # mappings), never run across devices before; whatever it does to the
    # node, the other forms have been measured
    if radix != 64 and a.exchange != "peer" and not a.no_peer and a.transport != "gloo":
        out.append(("peer", peer_argv(a)))
    return out


MI355X_HBM_BYTES = 288 * 10**9  # device memory of one MI355X (spec); --dry-rank's stand-in for lsb_device_memory


def memory_keys(a, N, radix, device_total, ranks_per_device=1):
    """Device memory of one rank (lsb_rank_footprint, host arithmetic) against
    the device's: A, B, R, look-back rows and tables, plus the optional
    placement probe's transient (LSB_PLACEMENT_CANDIDATES) while it runs."""
    with_recv = N > 1 or a.force_exchange or a.passes == "hybrid"
    fp = lsbsort.rank_footprint(a.n_per_gpu * N, N, radix, with_recv)
    peak = ranks_per_device * (fp["bytes"] + fp["probe_bytes"])
    return {"bytes": fp["bytes"], "probe_bytes": fp["probe_bytes"], "ranks_per_device": ranks_per_device,
            "device_bytes": device_total, "peak_frac": round(peak / device_total, 4) if device_total else None,
            "fits": bool(device_total) and peak <= device_total,
            "basis": "lsb_rank_footprint: A, B" + (", R" if with_recv else "") + ", look-back rows, tables; "
                     "probe_bytes = the placement probe's candidates beyond A and B (0: no probe)"}


def any_unverified(out):
    """The headline or any extra form produced output that failed lsb_verify
    (an extra that failed to run is `<name>_error`, not a wrong answer)."""
    return out.get("verified") is False or any(
        k.endswith("_verified") and v is False for k, v in out.items())


C5_BYTES_PER_ELEM = 192  # configs[4], 48 B per record per pass, 4 passes


def c5_keys(out, n):
    """N = 1: BASELINE configs[4] (the reference's 16-bit digits, 4 passes)
    against SURVEY 8(d)'s C5 denominator (192 B per record).  At P = 1 a
    16-bit digit runs as two stable 8-bit passes, so `--radix-bits 16`
    alone is the headline's work; the forms that are C5's own answer are the
    hybrid (4 byte passes over HBM plus one segmented sort) and the x16 extra
    (the 16-bit exchange path run through RCCL)."""
    for name in ("hybrid", "x16"):
        ms = out.get(f"{name}_ms_per_step")
        if ms:
            out[f"{name}_c5_survey_frac"] = round(C5_BYTES_PER_ELEM * n / (ms / 1e3) / (HBM_PEAK_GBS * 1e9), 4)
    out["c5_basis"] = ("SURVEY.md 8(d) C5: 192 B per record (48 B x 4 passes of 16-bit digits) / sort time / "
                       "8 TB/s; at P = 1 a 16-bit digit runs as two stable 8-bit passes (a 65536-bucket "
                       "pass is write-bound, DESIGN.md 5.15), so C5's answers are hybrid_* (4 byte passes + "
                       "one segmented sort, same output) and x16_* (the 16-bit exchange path through RCCL)")


def merge_extra(out, name, ok, text, report):
    """An extra form's keys into the headline line: <name>_melem_s,
    _ms_per_step, _verified (and its per-pass rows and dominant-kernel
    roofline when it has them), or <name>_error."""
    r = last_json(text)
    if r is not None and not ok and r.get("verified") is not False:
        r = None  # a failed form's line counts only to say its output was wrong
    if r is None:
        out[f"{name}_error"] = report or "no result line"
        return
    if not ok:
        out[f"{name}_error"] = report or "failed"
    out[f"{name}_melem_s"] = r["value"]
    out[f"{name}_ms_per_step"] = r["ms_per_step"]
    out[f"{name}_verified"] = r["verified"]
    for k in ("per_pass", "kernel_ms_per_step", "roofline", "exchange_roofline"):
        if r.get(k) is not None:
            out[f"{name}_{k}"] = r[k]


def rank_extra(a, d, out, name, argv):
    """Launcher-started ranks (torch.distributed.run): an extra form, same
    input, fewer steps, in one fresh process per rank (this rank's context is
    closed by now), so a failure there costs only its own keys.  Every rank
    takes the same branch: the children's success is agreed on before rank 0
    reads its child's line."""
    port = d.bcast_bytes(free_port() if d.rank == 0 else None)
    env = rank_env(d.rank, d.world, d.local_rank, port, os.environ.get("MASTER_ADDR", "127.0.0.1"))
    ok, text, report = spawn_ranks(argv, [env], extra_timeout(a), f"{name} extra")
    ok = d.all_true(ok)
    if d.rank == 0:
        merge_extra(out, name, ok, text, report or ("" if ok else "another rank's process failed"))


def dry_stats(rank, P, steps):
    """Exchange stats of the shape lsb_get_exchange_stats reports, made up
    for --dry-rank (rank r sends (r + 1) MB to every peer per exchange)."""
    per = [0 if q == rank and P > 1 else (rank + 1) << 20 for q in range(P)]  # P = 1: to itself
    ex = 4 * steps
    return {"exchanges": ex, "calls": 4 * ex, "sent_bytes": [b * ex for b in per],
            "recv_bytes": [0 if q == rank and P > 1 else ((q + 1) << 20) * ex for q in range(P)],
            "wire_ms": 1.0 * ex, "plan_ms": 0.1 * ex, "place_ms": 0.5 * ex, "place_tail_ms": 0.125 * ex,
            "place_bytes": 32 * 1000 * ex, "placed_records": 1000 * steps, "counted_records": 3000 * steps}


def dry_run(a):
    """--dry-rank (tests, CPU): the launch plumbing without a GPU.  Each rank
    joins the gloo group and max-reduces its rank; rank 0 prints a line of
    the bench's shape (with an exchange roofline from made-up stats at
    N > 1); --dry-fail R makes rank R exit with status 3 (and
    --dry-fail-whole-key / --dry-fail-peer R rank R of that extra)."""
    d = Dist()
    radix = a.radix_bits or (8 if d.world == 1 else 16)
    fail = (a.dry_fail_whole_key if radix == 64 else a.dry_fail_peer if a.exchange == "peer" else
            a.dry_fail_x16 if a.force_exchange else a.dry_fail)
    if d.rank == fail:
        sys.exit(3)
    top = d.max(float(d.rank))
    form = ("x16" if a.force_exchange else "whole_key" if radix == 64 and d.world > 1 else
            "peer" if a.exchange == "peer" else "hybrid" if a.passes == "hybrid" else
            "chunked" if a.exchange_chunks else "headline")
    out = {"metric": METRIC, "value": float(d.world * radix), "ms_per_step": 1.0,
           "verified": form != a.dry_unverified,
           "n_gpus": d.world, "max_rank": top, "radix_bits": radix, "exchange": a.exchange,
           "config": {"n_total": a.n_per_gpu * d.world},
           "device_memory": memory_keys(a, d.world, radix, MI355X_HBM_BYTES)}
    if d.world > 1 or a.force_exchange:
        out["exchange_roofline"] = exchange_roofline(
            d.all_gather_obj({"stats": dry_stats(d.rank, d.world, a.steps)}), a.steps)
        out["per_pass"] = [{"pass": 0, "shift": 0, "kernel": "k_onesweep", "ms": 1.0, "exchange_ms": 0.5,
                            "place_ms": 0.25, "wire_ms": 0.5, "place_tail_ms": 0.125}]
    if d.world > 1:
        for name, argv in extras_at(a, d.world):
            rank_extra(a, d, out, name, argv)
    else:
        for name, argv in extras_at(a, 1):
            merge_extra(out, name, *spawn_ranks(argv, [dict(os.environ)], extra_timeout(a), f"{name} extra"))
        c5_keys(out, a.n_per_gpu)
    d.barrier()
    d.close()
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    if any_unverified(out):
        sys.exit(1)


def launch(a):
    """`bench.py --gpus N` without a launcher: start the N rank processes
    here (one per GPU, RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* set as
    torch.distributed.run would), relay rank 0's line.  Nothing in this
    process initialises HIP."""
    N = a.gpus
    argv = sys.argv[1:] + ["--no-cpu-baseline", "--no-extras"]
    port = free_port()
    ok, text, report = spawn_ranks(argv, [rank_env(r, N, r, port) for r in range(N)], a.rank_timeout,
                                   "headline")
    out = last_json(text) if ok else None
    if out is None:
        print(f"bench.py: {report or 'rank 0 printed no result line'}", file=sys.stderr, flush=True)
        sys.exit(1)
    out["launcher"] = f"bench.py started {N} rank processes (one per GPU)"
    for name, xargv in extras_at(a, N):
        port = free_port()
        merge_extra(out, name, *spawn_ranks(xargv, [rank_env(r, N, r, port) for r in range(N)],
                                            extra_timeout(a), f"{name} extra"))
    out["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline(out["config"]["n_total"], a.cpu_n)
    print(json.dumps(out), flush=True)
    if any_unverified(out):
        sys.exit(1)


def probe(a):
    """One sort of the workload, nothing printed: the program rocprofv3's
    --pmc passes run (measure_traffic)."""
    w = lsbsort.World(a.n_per_gpu, ranks=1, radix_bits=a.radix_bits or 8)
    w.set_option(lsbsort.OPT_ONESWEEP, 0 if a.passes == "reduce-scan" else 1)
    w.set_option(lsbsort.OPT_HYBRID, 1 if a.passes == "hybrid" else 0)
    w.generate(a.dist, a.zipf_s)
    w.my_sort()
    w.sync()
    w.close()


def exchange_roofline(ranks, steps):
    """The exchange side of a sort at N > 1 ("the k_place
    bytes" and "the xGMI bound: each GPU sends 16*m/P B to each of its P-1
    peers per pass"), from every rank's lsb_get_exchange_stats (`ranks[r]
    ["stats"]`, summed over `steps` sorts).  Per sort: the payload each rank
    handed RCCL and per directed link (busiest / least busy pair: the skew of
    Zipf keys shows here), the all-to-all's wire time on the ranks' streams
    (plan and placement excluded), the busiest link's achieved GB/s and its
    fraction of the per-link xGMI figure, each GPU's send rate, and the
    placement (k_place / merge) bytes, time and the part of it left after the
    last slice arrived (not overlapped with the wire)."""
    P = len(ranks)
    st = [r["stats"] for r in ranks]
    S = [[st[s]["sent_bytes"][q] / steps for q in range(P)] for s in range(P)]
    # P = 1 (--force-exchange): the one "link" is the rank to itself through RCCL
    links = sorted((S[s][q], s, q) for s in range(P) for q in range(P) if q != s or P == 1)
    wire = [x["wire_ms"] / steps for x in st]
    ex = st[0]["exchanges"] / steps

    def gbs(b, ms):
        return round(b / (ms / 1e3) / 1e9, 2) if ms > 0 else None

    hi, lo = links[-1], links[0]
    link_gbs = gbs(hi[0], wire[hi[1]])
    sent = [sum(S[s][q] for q in range(P) if q != s or P == 1) for s in range(P)]
    gpu = [g for g in (gbs(sent[s], wire[s]) for s in range(P)) if g is not None]
    place_ms = [x["place_ms"] / steps for x in st]
    tail = [x["place_tail_ms"] / steps for x in st]
    pbytes = [x["place_bytes"] / steps for x in st]
    busy = max(range(P), key=lambda r: place_ms[r])
    self_only = P == 1
    return {
        "bound": "self" if self_only else "xgmi", "unit": "GB/s",
        "peak": None if self_only else XGMI_LINK_GBS,
        "peak_source": ("one GPU: the rank's records go through RCCL to itself (a device copy, no link); "
                        "no xGMI figure applies") if self_only else XGMI_PEAK_SOURCE,
        "achieved": link_gbs,
        "frac": round(link_gbs / XGMI_LINK_GBS, 4) if link_gbs and not self_only else None,
        "exchanges_per_sort": ex, "calls_per_sort": st[0]["calls"] / steps,
        "rank_bytes_per_sort": {"max": int(max(sent)), "min": int(min(sent))},
        "link_bytes_per_sort": {"max": int(hi[0]), "max_link": [hi[1], hi[2]],
                                "min": int(lo[0]), "min_link": [lo[1], lo[2]],
                                "max_over_min": round(hi[0] / lo[0], 3) if lo[0] else None},
        "link_bytes_per_exchange": {"max": int(hi[0] / ex) if ex else None,
                                    "min": int(lo[0] / ex) if ex else None},
        "wire_ms_per_sort": {"max": round(max(wire), 3), "min": round(min(wire), 3)},
        "gpu_send_gbs": {"max": max(gpu), "min": min(gpu)} if gpu else None,
        "link_bound_ms_per_sort": round(hi[0] / (XGMI_LINK_GBS * 1e9) * 1e3, 3),
        "plan_ms_per_sort": round(max(x["plan_ms"] / steps for x in st), 3),
        "place": {"bytes_per_sort": int(pbytes[busy]), "ms_per_sort": round(place_ms[busy], 3),
                  "gbs": gbs(pbytes[busy], place_ms[busy]), "tail_ms_per_sort": round(max(tail), 3),
                  "overlapped_frac": round(min(1 - t / m for t, m in zip(tail, place_ms) if m > 0), 4)
                  if any(m > 0 for m in place_ms) else None,
                  "placed_records_per_sort": int(st[busy]["placed_records"] / steps),
                  "counted_records_per_sort": int(st[busy]["counted_records"] / steps),
                  "basis": "rank with the longest placement; 32 B per placed record, 16 B per "
                           "counted one, 32 B per merge level"},
    }


def per_pass_rows(passes, steps, kernel, N):
    """Per local pass, per step (lsb_get_pass_stats): the scatter kernel's
    time, its HBM rate (32 algorithmic bytes per record) and its fraction of
    the peak, plus the pass's count, exchange and placement time; with an
    exchange after the pass, its all-to-all payload, wire time and rate
    (this rank's) and the placement tail."""
    rows = []
    for p in passes:
        if not p["launches"]:
            continue
        avg = p["ms_scatter"] / p["launches"]
        gbs = SCATTER_BYTES_PER_ELEM * (p["elems"] / p["launches"]) / (avg / 1e3) / 1e9 if avg > 0 else 0.0
        row = {"pass": p["pass"], "shift": p["shift"], "kernel": "k_segsort" if p["shift"] == 64 else kernel,
               "ms": round(p["ms_scatter"] / steps, 4), "gbs": round(gbs, 1),
               "frac": round(gbs / HBM_PEAK_GBS, 4)}
        if p["ms_count"]:
            row["count_ms"] = round(p["ms_count"] / steps, 4)
        if N > 1 or p["ms_exchange"] or p["ms_place"]:
            row["exchange_ms"] = round(p["ms_exchange"] / steps, 4)
            row["place_ms"] = round(p["ms_place"] / steps, 4)
        if p.get("ms_wire"):
            row["exchange_bytes"] = int(p["exchange_bytes"] / steps)
            row["wire_ms"] = round(p["ms_wire"] / steps, 4)
            row["exchange_gbs"] = round(p["exchange_bytes"] / (p["ms_wire"] / 1e3) / 1e9, 2)
            row["place_tail_ms"] = round(p["ms_place_tail"] / steps, 4)
        rows.append(row)
    return rows


def main():
    a = parse()
    if a.probe:
        return probe(a)
    if a.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return launch(a)
    if a.dry_rank:
        return dry_run(a)
    d = Dist()
    N = d.world if d.world > 1 else a.gpus
    n_total = a.n_per_gpu * N
    radix = a.radix_bits or (8 if N == 1 else 16)
    if radix == 64 and a.exchange == "peer":
        raise SystemExit("--exchange peer is a per-digit exchange form; use --radix-bits 8 or 16")
    w, device = make_world(a, d, N, n_total, radix)
    bind_device(device)
    # Dominant kernel: the local pass.  Single-read passes (k_onesweep) in
    # every form: P = 1, the per-digit exchange (the exchange's placement
    # counts the next pass's histogram) and each rank of the whole-key form.
    kernel = "k_scatter" if a.passes == "reduce-scan" else "k_onesweep"

    total, verified, step_s = timed_sorts(w, d, a, a.steps, a.warmup)
    stats = w.kernel_stats()
    passes = w.pass_stats()
    scatter_elems = w.scatter_elems()
    xcalls, xbytes, _ = w.exchange_bytes()
    xstats = w.exchange_stats()
    placement = w.placement()
    last = w.last_sort()
    first = w.first_pass()  # the regional first pass (no count read) or a count read
    w.close()
    mem = memory_keys(a, N, radix, lsbsort.device_memory(device)[1],
                      max(1, N // max(1, visible_devices())) if N > 1 else 1)
    xroof = exchange_roofline(d.all_gather_obj({"stats": xstats}), a.steps) if N > 1 or a.force_exchange else None

    ms_per_step = total / a.steps * 1e3
    value = n_total * a.steps / total / 1e6
    launches, scatter_ms = stats["scatter"]
    m = a.n_per_gpu
    size = f"2^{m.bit_length() - 1}" if m > 0 and m & (m - 1) == 0 else str(m)
    if N == 1:
        cfg = "configs[1]" if radix == 8 else "configs[4]"
        workload = (f"{cfg}: sort of {size} 16-byte records per GPU, {radix}-bit digits, "
                    f"{64 // radix} passes, {N} GPU(s)")
        if radix == 16 and a.force_exchange:
            workload += (" (each digit as two stable 8-bit sub-passes, then the digit's exchange: counts "
                         "all-gather, plan, RCCL AllToAllv of every record to this rank itself, placement)")
        elif radix == 16:
            workload += " (each digit as two stable 8-bit sub-passes; no exchange)"
    else:
        cfg = "configs[2]" if a.dist == "uniform" else "configs[3]"
        workload = (f"{cfg}: sort of {N} x {size} 16-byte records block-partitioned over {N} GPUs, "
                    f"8-bit local passes, " +
                    (f"RCCL AllToAllv per {radix}-bit digit ({64 // radix} exchanges)" if radix != 64 else
                     "whole-key exchange digit (local sort, 1 all-to-all, merge of the P runs)"))
    if a.passes == "hybrid":
        workload += (" (hybrid local sort: single-read passes on the top varying bytes, then one "
                     "segmented local sort; the same stable order)")
    if a.dist != "uniform":
        workload += f", zipf s={a.zipf_s} keys"
    if m != 1 << 30:
        workload = "custom size, " + workload
    roof = None
    if launches and scatter_ms > 0:
        elems_per_launch = scatter_elems / launches
        avg_s = scatter_ms / launches / 1e3
        achieved = SCATTER_BYTES_PER_ELEM * elems_per_launch / avg_s / 1e9
        traffic, traffic_src = None, "not measured at N > 1 (rocprofv3 passes run at N = 1)"
        if N == 1 and not a.no_traffic:
            traffic, traffic_src = measure_traffic(a, kernel, elems_per_launch)
        elif a.no_traffic:
            traffic_src = "skipped (--no-traffic)"
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_ratio": round(traffic / (SCATTER_BYTES_PER_ELEM * elems_per_launch), 4)
                if traffic else None, "traffic_source": traffic_src,
                "kernel": kernel, "bytes_per_launch": int(SCATTER_BYTES_PER_ELEM * elems_per_launch),
                "avg_launch_ms": round(scatter_ms / launches, 4)}
    # Algorithmic bytes of a sort: 32 B per record per scatter launch, 16 B
    # per count read (one per pass for reduce-then-scan, one per sort for
    # single-read passes; none when the sort starts with the regional first
    # pass, whose count launch is a sample of 2^20 records).
    count_elem = (COUNT_BYTES_PER_ELEM * min(1.0, SAMPLE_RECORDS / max(1, n_total / N))
                  if first == lsbsort.FIRST_REGIONAL else COUNT_BYTES_PER_ELEM)
    per_elem = (SCATTER_BYTES_PER_ELEM * launches + count_elem * stats["upsweep"][0]) / a.steps
    sort_gbs = per_elem * (n_total / N) / (ms_per_step / 1e3) / 1e9
    # SURVEY.md §8(d)'s sort-level figure: 48 B per record per digit pass
    # (16 B histogram read + 32 B scatter) over D = 64 / radix_bits passes,
    # a fixed denominator whatever the design moves (measured bytes: roofline).
    D = 64 // radix if radix != 64 else 8
    med_s = sorted(step_s)[len(step_s) // 2]
    survey_frac = 48 * D * (n_total / N) / med_s / (HBM_PEAK_GBS * 1e9)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Melem/s",
        "n_gpus": N,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / REF_MPI_MELEMS, 3),
        "dtype": "u64",
        "data": ("synthetic: pcg64(rank) keys, val = global index (mpi_lsbsort.cpp:650-656), regenerated on device before every step"
                 if a.dist == "uniform" else
                 f"synthetic: zipf(s={a.zipf_s}) keys drawn from the pcg64(rank) stream (build-defined, SURVEY 8d C4)"),
        "config": {"workload": workload, "n_total": n_total, "n_per_gpu": a.n_per_gpu,
                   "local_digit_bits": 8, "local_passes": last[0], "exchanges": last[1],
                   "pass_form": ("hybrid (k_subhist, k_onesweep on the top varying bytes, then one "
                                 "k_segsort of the runs equal on them)" if a.passes == "hybrid" else
                                 ("single-read (" + ("a 2^20-record sample, then the regional first pass "
                                                     "(no count read; DESIGN.md 4), k_onesweep per pass"
                                                     if first == lsbsort.FIRST_REGIONAL else
                                                     "k_subhist once, k_onesweep per pass") +
                                  ("; k_place counts the next pass's histogram)" if N > 1 and radix != 64
                                   else ")")) if kernel == "k_onesweep"
                                 else "reduce-then-scan (k_upsweep, k_scan, k_scatter per pass)"),
                   "first_pass": {0: "count read", 1: "regional", 2: "regional, overflowed: redone"}.get(first),
                   "exchange_digit_bits": radix if N > 1 else None,
                   "record_bytes": 16, "dist": a.dist,
                   "parallelism": parallelism(N, radix, a)},
        "roofline": roof,
        "sort_hbm_frac": round(sort_gbs / HBM_PEAK_GBS, 4),
        "step_ms": [round(t * 1e3, 3) for t in step_s],
        "median_melem_s": round(n_total / med_s / 1e6, 2),
        "survey_roofline": {"frac": round(survey_frac, 4), "bytes_per_elem": 48 * D, "passes": D,
                            "basis": "SURVEY.md 8(d): 48*D*n / (t_sort * P * 8e12), fixed denominator, "
                                     "median step"},
        "kernel_ms_per_step": {k: round(v[1] / a.steps, 3) for k, v in stats.items()},
        "per_pass": per_pass_rows(passes, a.steps, kernel, N),
        "kernel_ms_per_step_legend": {
            "upsweep": "count read (k_subhist once per sort, or k_upsweep per pass; with the regional "
                       "first pass: the 2^20-record sample)",
            "scan": "chunk scan (k_scan, reduce-then-scan only)",
            "scatter": "local passes (k_onesweep, or k_scatter)",
            "exchange": "exchange on the rank's stream: splitter search + all-to-all (whole key) "
                        "or counts all-gather + plan + all-to-all (per digit); includes wire time",
            "place": "placement stream: merge of the received runs (whole key) or k_place",
            "sort": "the whole sort, per rank"},
        "exchange_bytes_per_step": xbytes // a.steps if N > 1 or a.force_exchange else 0,
        "exchange_roofline": xroof,
        "placement": dict(placement, record_alloc=os.environ.get("LSB_RECORD_ALLOC", "vmm 1 GiB pieces"),
                          basis="rank 0's A and B: built from 1 GiB VMM pieces, chosen at context creation "
                                "among K candidate buffers (by default 4 for buffers of >= 4 GiB; "
                                "LSB_PLACEMENT_CANDIDATES = K; candidates 0: no probe), each timed once "
                                "as the destination of a k_onesweep pass (one chain of passes, losers "
                                "freed at once); ms per pass as a destination: the kept two (mean), "
                                "the first two allocated (mean), the slowest (lsb_get_placement; "
                                "DESIGN.md 0, 4)"),
        "device_memory": mem,
        "verified": verified,
        "vs_baseline_basis": "MPI mpi_lsbsort 830 M elem/s (64 nodes x 128 cores, n=2^36; BASELINE.md §1)",
        "library": lsbsort.build_info(),
    }
    # The extra forms, in fresh processes after the headline: N > 1 the
    # whole-key and peer-store exchanges, N = 1 the hybrid local sort.
    for name, xargv in extras_at(a, N):
        if N > 1:
            rank_extra(a, d, out, name, xargv)
        else:
            merge_extra(out, name, *spawn_ranks(xargv, [dict(os.environ)], extra_timeout(a), f"{name} extra"))
    if N == 1:
        c5_keys(out, n_total)
    if d.rank == 0 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n_total, a.cpu_n)
    elif d.rank == 0:
        out["cpu_baseline"] = None
    d.barrier()
    d.close()
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    if any_unverified(out):
        sys.exit(1)


if __name__ == "__main__":
    main()
