#!/usr/bin/env python3
"""Collective / transport microbenchmark for the exchange engines (SURVEY.md §7.2 comm_bench).

Times, for message sizes typical of gradient buckets (1 MB .. 256 MB of bf16), every data path
hipps moves gradients or parameters over:

  * torch.distributed all-gather / gather / broadcast (backend nccl = RCCL over xGMI; the sync
    engines' default transport),
  * hipps' own RCCL communicator (``transport='rccl'``): all-gather, ncclGather, broadcast,
  * the async PS's one-sided paths: a worker's stream-ordered copy into the PS rank's HIP-IPC
    mailbox (gradient push) and a copy kernel reading the PS rank's publish buffer (pull).

Bus bandwidth follows the usual convention: all-gather moves (W-1)/W of the output per rank,
gather / broadcast the message once per non-root rank.  Launch::

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port 29500 bench/comm_bench.py [--sizes-mb 1,16,64,256] [--out f.json]

At N = 1 only the local copy rows are meaningful (the collectives are copies).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    mx = torch.tensor([dt], device="cuda")
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    return float(mx.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,16,64,256")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-rccl", action="store_true", help="skip hipps' native RCCL communicator rows")
    a = ap.parse_args()
    from hipps.parallel import dist as hdist

    world = hdist.init_from_env()
    if not dist.is_initialized():  # plain `python bench/comm_bench.py`: a one-rank RCCL group
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        world = hdist.current()
    W, rank = world.size, world.rank
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    rc = None
    if not a.no_rccl and W > 1:
        from hipps.parallel.rccl import RcclGroup

        rc = RcclGroup(world, dev)
    rows = []
    from hipps.ops._native import native

    C = native()
    max_n = int(max(float(s) for s in a.sizes_mb.split(",")) * (1 << 20)) // 2
    # rank 0's HIP-IPC mailbox, one slot per rank (the async PS's gradient mailboxes / publish
    # buffer), mapped by every rank through the exported handle
    box = C.DeviceMailbox(W * max_n * 2) if rank == 0 else None
    h = [box.handle() if rank == 0 else None]
    dist.broadcast_object_list(h, src=0)
    if rank != 0:
        box = C.DeviceMailbox(h[0], W * max_n * 2)
    mem = box.tensor()
    sel = torch.zeros(3, dtype=torch.int64, device=dev)  # "version 0" for the pull copy kernel

    def emit(op, mb, dt, bus_bytes):
        row = {"op": op, "world": W, "msg_MB": mb, "us": round(dt * 1e6, 1),
               "busbw_GBps": round(bus_bytes / dt / 1e9, 1) if dt > 0 else None}
        rows.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)

    for mb in [float(s) for s in a.sizes_mb.split(",")]:
        n = int(mb * (1 << 20)) // 2
        x = torch.randn(n, device=dev).to(torch.bfloat16)
        out = torch.empty(n * W, dtype=torch.bfloat16, device=dev)
        nbytes = n * 2
        emit("torch.all_gather", mb, _time(lambda: dist.all_gather_into_tensor(out, x), a.iters),
             nbytes * (W - 1))
        if W > 1:
            gl = [torch.empty_like(x) for _ in range(W)] if rank == 0 else None
            emit("torch.gather", mb, _time(lambda: dist.gather(x, gl, dst=0), a.iters), nbytes * (W - 1))
        emit("torch.broadcast", mb, _time(lambda: dist.broadcast(x, 0), a.iters), nbytes * max(W - 1, 1))
        if rc is not None:
            emit("rccl.all_gather", mb, _time(lambda: rc.all_gather_into(out, x), a.iters), nbytes * (W - 1))
            go = out if rank == 0 else None
            emit("rccl.gather", mb, _time(lambda: rc.gather_into(go, x, 0), a.iters), nbytes * (W - 1))
            emit("rccl.broadcast", mb, _time(lambda: rc.broadcast(x, 0), a.iters), nbytes * (W - 1))
        # async PS paths: every rank pushes its message into its own slot of rank 0's mailbox
        # (stream-ordered copy over xGMI; local on rank 0), and pulls rank 0's "publish buffer"
        # (slot 0) with the GPU-time pull's copy kernel (bf16 -> f32, as at param_wire='bf16')
        slot = mem[rank * max_n * 2: rank * max_n * 2 + nbytes].view(torch.bfloat16)
        emit("ipc.push", mb, _time(lambda: slot.copy_(x), a.iters), nbytes)
        pub = mem[: max_n * 2]
        dst = torch.empty(n, dtype=torch.float32, device=dev)
        emit("ipc.pull_kernel", mb, _time(lambda: C.pull_copy(sel, pub, max_n * 2, 1, True, dst, 0, n), a.iters),
             nbytes)
        y = torch.empty_like(x)
        emit("local.copy", mb, _time(lambda: y.copy_(x), a.iters), 2 * nbytes)
    if rank == 0 and a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    if rc is not None:
        rc.close()
    dist.barrier()
    box.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
