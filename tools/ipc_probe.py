"""How long does mapping the PS mailbox take?  Rank 0 allocates a DeviceMailbox of each size and
exports it; every other rank maps it with hipIpcOpenMemHandle (dmabuf IPC) and times the call.
Run under torch.distributed.run with the gloo backend (ranks may share one GPU).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/ipc_probe.py 256 1024 4096
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    from hipps.ops import _native

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    C = _native.native()
    for mb in [int(a) for a in sys.argv[1:]]:
        n = mb << 20
        t0 = time.perf_counter()
        mbx = C.DeviceMailbox(n) if rank == 0 else None
        meta = [mbx.handle() if rank == 0 else None]
        t_alloc = time.perf_counter() - t0
        dist.broadcast_object_list(meta, src=0)
        t0 = time.perf_counter()
        if rank != 0:
            mbx = C.DeviceMailbox(meta[0], n)
            mbx.tensor()[:16].fill_(rank)  # touch it
            torch.cuda.synchronize()
        t_open = time.perf_counter() - t0
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, round(t_open, 3))
        if rank == 0:
            print(f"mailbox {mb} MB: alloc+export {t_alloc:.3f} s, open per rank {out[1:]} s", flush=True)
        dist.barrier()
        mbx.close()
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
