#!/usr/bin/env python3
"""P real RCCL ranks in P processes on ONE GPU (development check).

RCCL refuses two ranks of one host on one device ("Duplicate GPU detected"),
but it keys "one host" on NCCL_HOSTID when that is set.  Each rank here gets
its own NCCL_HOSTID, so RCCL sees P single-GPU hosts and connects them with
its socket transport over loopback (NCCL_SOCKET_IFNAME=lo): slow, but every
collective of the multi-GPU path runs through RCCL between real ranks with
non-empty peer segments -- the counts ncclAllGather, the sliced
ncclAllToAllv / grouped ncclSend-ncclRecv of records, the span all-gather,
the whole-key form's splitter-search all-gathers, verify's all-reduce.

Output: the reference's golden digest for `mpirun -n P mpi_lsbsort --n n`
where one exists (tests/golden/digests.json), plus the on-device verify and
checkSorted of every rank.

    python tools/rccl_two_ranks.py [radix_bits] [n] [world] [exchange] [slices] [dist] [dump_dir]
      exchange: alltoallv (default) | p2p
      dist:     uniform (default) | zipf (s = 1.1)
      dump_dir: each rank writes its input and sorted output there as
                in_<r>.npy / out_<r>.npy (the tests compare them with the
                oracle's stable sort: Zipf input has no reference digest)
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))


def worker(rank, world, n, bits, exchange, slices, dist, dump, q_uid, q_out):
    # One "host" per rank, before anything touches RCCL.
    os.environ["NCCL_HOSTID"] = f"lsb-rank-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    import lsbsort
    if rank == 0:
        uid = lsbsort.get_unique_id()
        for _ in range(world - 1):
            q_uid.put(uid)
    else:
        uid = q_uid.get(timeout=60)
    try:
        dev = rank % int(os.environ.get("LSB_NUM_GPUS", "1"))
        w = lsbsort.World.rank(n, world, rank, dev, uid, radix_bits=bits)
        if exchange == "p2p":
            w.set_option(lsbsort.OPT_EXCHANGE_P2P, 1)
        if slices:
            w.set_option(lsbsort.OPT_EXCHANGE_SLICES, slices)
        w.generate(dist)
        if dump:
            import numpy as np
            np.save(os.path.join(dump, f"in_{rank}.npy"), w.copy_out(rank))
        w.barrier()
        w.my_sort()
        w.barrier()
        ok, bad = w.verify()
        sorted_ = w.check_sorted()
        _, xbytes, xmax = w.exchange_bytes()
        # large blocks are checked on device only (lsb_verify), not digested
        out = w.copy_out(rank) if n <= (1 << 26) or dump else None
        if dump:
            import numpy as np
            np.save(os.path.join(dump, f"out_{rank}.npy"), out)
        w.close()
        q_out.put((rank, "ok", ok, bad, sorted_, out.tobytes() if out is not None else b"", xbytes, xmax))
    except Exception as e:  # report, never hang the parent
        q_out.put((rank, "error", repr(e), None, None, b"", 0, 0))


def main():
    bits = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    world = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    exchange = sys.argv[4] if len(sys.argv) > 4 else "alltoallv"
    slices = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    dist = sys.argv[6] if len(sys.argv) > 6 else "uniform"
    dump = sys.argv[7] if len(sys.argv) > 7 else ""
    ctx = mp.get_context("spawn")
    q_uid, q_out = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, n, bits, exchange, slices, dist, dump, q_uid, q_out))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q_out.get(timeout=300)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    errors = {r: v[2] for r, v in res.items() if v[1] != "ok"}
    if errors:
        print(json.dumps({"status": "error", "errors": errors}))
        sys.exit(1)
    digest = hashlib.sha256(b"".join(res[r][5] for r in range(world))).hexdigest() if n <= (1 << 26) else None
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    want = None if dist != "uniform" else next(
        (g["output"] for g in golden["rows"] if g["n"] == n and g["P"] == world), None)
    verify = [res[r][2] for r in range(world)]
    sorted_ = [res[r][4] for r in range(world)]
    good = all(verify) and all(sorted_) and (want is None or digest == want)
    print(json.dumps({"status": "ok" if good else "mismatch", "radix_bits": bits, "n": n, "world": world,
                      "dist": dist,
                      "exchange": exchange, "slices": slices or "default", "verify": verify,
                      "check_sorted": sorted_, "rccl_bytes": [res[r][6] for r in range(world)],
                      "rccl_max_call_bytes": [res[r][7] for r in range(world)], "digest": digest,
                      "golden_match": (digest == want) if want else None}), flush=True)
    sys.exit(0 if good else 1)


if __name__ == "__main__":
    main()
