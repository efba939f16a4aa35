#!/usr/bin/env python3
"""Probe (not part of the product or the test suite): can the RCCL branch of
qe_allreduce_stats run with nranks = 2 on a one-GPU box?  Two processes on
cuda:0 build one communicator through the C ABI (qe_comm_unique_id ->
qe_comm_init) and all-reduce a uint64 vector; each rank checks the sum.
RCCL may refuse two ranks on one device; the script then reports the error
status instead of a sum.  Run under `timeout`."""
import ctypes as C
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, idpath, q):
    sys.path.insert(0, ROOT)
    import torch

    from etcd_amd import engine
    L = engine._lib.lib()
    n = L.qe_comm_id_bytes()
    if rank == 0:
        idb = (C.c_uint8 * n)()
        engine.check("qe_comm_unique_id", L.qe_comm_unique_id(idb))
        with open(idpath + ".tmp", "wb") as f:
            f.write(bytes(idb))
        os.replace(idpath + ".tmp", idpath)
    else:
        t0 = time.time()
        while not os.path.exists(idpath):
            if time.time() - t0 > 60:
                q.put((rank, "no id", None))
                return
            time.sleep(0.05)
        with open(idpath, "rb") as f:
            idb = (C.c_uint8 * n).from_buffer_copy(f.read())
    comm = C.c_void_p()
    rc = L.qe_comm_init(C.byref(comm), 2, rank, idb, 0)
    if rc != 0:
        q.put((rank, f"qe_comm_init {rc} {L.qe_strerror(rc).decode()}", None))
        return
    x = torch.tensor([(rank + 1) * (k + 1) for k in range(16)], dtype=torch.int64, device="cuda:0")
    x[15] = -1 - rank  # uint64 wraparound: (2^64-1) + (2^64-2) mod 2^64
    rc = L.qe_allreduce_stats(engine._ptr(x), 16, comm, engine._stream(x.device))
    torch.cuda.synchronize()
    got = x.cpu().tolist()
    L.qe_comm_destroy(comm)
    want = [3 * (k + 1) for k in range(15)] + [-3]
    q.put((rank, f"allreduce rc {rc}", got == want))


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        idpath = os.path.join(d, "rccl.id")
        ps = [ctx.Process(target=rank_main, args=(r, idpath, q)) for r in range(2)]
        for p in ps:
            p.start()
        res = []
        t0 = time.time()
        while len(res) < 2 and time.time() - t0 < 150:
            try:
                res.append(q.get(timeout=5))
            except Exception:
                pass
        for p in ps:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    print("rccl two ranks on one GPU:", sorted(res, key=lambda r: r[0]))
    ok = len(res) == 2 and all(r[2] for r in res)
    print("RESULT", "sum correct on both ranks" if ok else "not run / failed")


if __name__ == "__main__":
    main()
