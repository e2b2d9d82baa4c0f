"""Spawn a local gloo world (127.0.0.1) and run fn(rank, world_size, *args) in each rank."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pack(o):
    import torch

    if isinstance(o, torch.Tensor):
        return ("__t__", o.detach().cpu().numpy(), str(o.dtype))
    if isinstance(o, (list, tuple)):
        return type(o)(_pack(x) for x in o)
    if isinstance(o, dict):
        return {k: _pack(v) for k, v in o.items()}
    return o


def _unpack(o):
    import torch

    if isinstance(o, tuple) and len(o) == 3 and o[0] == "__t__":
        return torch.from_numpy(o[1])
    if isinstance(o, (list, tuple)):
        return type(o)(_unpack(x) for x in o)
    if isinstance(o, dict):
        return {k: _unpack(v) for k, v in o.items()}
    return o


def _entry(rank, world_size, port, fn, args, q, backend="gloo"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from hipps.parallel import dist as hdist

        hdist.init_from_env(backend=backend)
        out = fn(rank, world_size, *args)
        q.put((rank, "ok", _pack(out)))
    except BaseException:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def run_world(fn, world_size=2, *args, timeout=240, backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world_size, port, fn, args, q, backend)) for r in range(world_size)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world_size):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            results[rank] = _unpack(out)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world_size)]
