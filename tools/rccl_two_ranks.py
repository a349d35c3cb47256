#!/usr/bin/env python3
"""Two RCCL ranks in two processes on ONE GPU (development check).

Exercises the real multi-process path of the runtime (lsb_create_rank:
ncclCommInitRank, ncclAllGather of counts, grouped ncclSend/ncclRecv,
k_place) where only one GPU exists, if RCCL accepts two ranks on one
device.  Compares against the reference's golden digest for
`mpirun -n 2 mpi_lsbsort --n 1000000`.

    python tools/rccl_two_ranks.py [radix_bits] [n]
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))


def worker(rank, world, n, bits, q_uid, q_out):
    import lsbsort
    if rank == 0:
        uid = lsbsort.get_unique_id()
        for _ in range(world - 1):
            q_uid.put(uid)
    else:
        uid = q_uid.get(timeout=60)
    try:
        # On a 1-GPU box both ranks share device 0, which RCCL 2.27 rejects
        # ("Duplicate GPU detected"): this check needs LSB_NUM_GPUS >= 2.
        dev = rank % int(os.environ.get("LSB_NUM_GPUS", "1"))
        w = lsbsort.World.rank(n, world, rank, dev, uid, radix_bits=bits)
        w.generate()
        w.barrier()
        w.my_sort()
        w.barrier()
        ok, bad = w.verify()
        sorted_ = w.check_sorted()
        out = w.copy_out(rank)
        w.close()
        q_out.put((rank, "ok", ok, bad, sorted_, out.tobytes()))
    except Exception as e:  # report, never hang the parent
        q_out.put((rank, "error", repr(e), None, None, b""))


def main():
    bits = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    world = 2
    ctx = mp.get_context("spawn")
    q_uid, q_out = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, n, bits, q_uid, q_out)) for r in range(world)]
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
    digest = hashlib.sha256(b"".join(res[r][5] for r in range(world))).hexdigest()
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    want = next((g["output"] for g in golden["rows"] if g["n"] == n and g["P"] == world), None)
    print(json.dumps({"status": "ok", "radix_bits": bits, "n": n, "verify": [res[r][2] for r in range(world)],
                      "check_sorted": [res[r][4] for r in range(world)], "digest": digest,
                      "golden_match": (digest == want) if want else None}))
    sys.exit(0 if (want is None or digest == want) else 1)


if __name__ == "__main__":
    main()
