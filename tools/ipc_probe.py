"""How long does importing a PS mailbox take, and where does a stuck import sit?

Rank 0 allocates a DeviceMailbox of each size (or, with --chunk-mb, the same bytes as several
allocations), stamps each allocation, and exports it; every other rank imports it with
hipIpcOpenMemHandle (dmabuf IPC), one rank at a time, each import bounded
(hipps.parallel.ps_async._bounded_open), and checks the stamps.  A timed-out
import prints the stuck thread's /proc state sampled over a few seconds (wait channel, syscall,
user / system CPU ticks: a thread burning CPU in user space is a runtime loop, one parked in a
syscall is the kernel driver) and ends the probe (the thread cannot be cancelled).
Run under torch.distributed.run with the gloo backend (ranks may share one GPU).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/ipc_probe.py \
        --sizes 256,1024,4096,8192 [--chunk-mb 512] [--limit 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _cpu_ticks(tid):
    try:
        with open(f"/proc/self/task/{tid}/stat") as f:
            parts = f.read().rsplit(")", 1)[1].split()
        return int(parts[11]), int(parts[12])  # utime, stime (fields 14, 15)
    except OSError:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,1024,2048,4096,8192")
    ap.add_argument("--chunk-mb", type=int, default=0, help="split every region into allocations of this size")
    ap.add_argument("--limit", type=float, default=20.0)
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from hipps.ops import _native
    from hipps.parallel.ps_async import IPCOpenTimeout, _bounded_open, _thread_diag

    dist.init_process_group("gloo")
    rank, W = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    C = _native.native()
    for rep in range(a.repeat):
        for mb in [int(s) for s in a.sizes.split(",")]:
            parts = [mb] if not a.chunk_mb else [min(a.chunk_mb, mb - o) for o in range(0, mb, a.chunk_mb)]
            t0 = time.perf_counter()
            mine = [C.DeviceMailbox(p << 20) for p in parts] if rank == 0 else []
            for c, m in enumerate(mine):  # stamp every allocation (checked by the importers)
                m.tensor()[0] = (c % 200) + 1
            torch.cuda.synchronize()
            meta = [[m.handle() for m in mine] if rank == 0 else None]
            t_alloc = time.perf_counter() - t0
            dist.broadcast_object_list(meta, src=0)
            res = None
            for r in range(1, W):  # one importer at a time
                if rank == r:
                    t1 = time.perf_counter()
                    try:
                        for c, (h, p) in enumerate(zip(meta[0], parts)):
                            mbx, _ = _bounded_open(lambda h=h, p=p: C.DeviceMailbox(h, p << 20), f"{p} MB", rank,
                                                   torch.cuda.current_device(), a.limit)
                            mine.append(mbx)
                            got = int(mbx.tensor()[0])
                            if got != (c % 200) + 1:
                                raise IPCOpenTimeout(f"STALE rank {rank}: allocation {c} reads {got}")
                        torch.cuda.synchronize()
                        res = round(time.perf_counter() - t1, 4)
                    except IPCOpenTimeout as e:
                        res = f"TIMEOUT {e}"
                dist.barrier()
            out = [None] * W
            dist.all_gather_object(out, res)
            if rank == 0:
                print(f"rep {rep} region {mb} MB as {len(parts)} allocation(s): "
                      f"alloc+export {t_alloc:.3f} s, "
                      f"import per rank {out[1:]}", flush=True)
            if any(isinstance(o, str) for o in out):
                if isinstance(res, str):  # sample the stuck thread a few more times, then leave
                    import threading
                    tids = [t.native_id for t in threading.enumerate() if t.name == "hipps-ipc-open"]
                    for k in range(4):
                        time.sleep(1.0)
                        print(f"  rank {rank} t+{k + 1}s: " + "; ".join(
                            f"{_thread_diag(t)} cpu(utime,stime)={_cpu_ticks(t)}" for t in tids), flush=True)
                sys.stdout.flush()
                os._exit(4)
            dist.barrier()
            for m in mine:
                m.close()
            dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
