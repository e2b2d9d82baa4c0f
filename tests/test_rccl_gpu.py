"""hipps' native RCCL communicator (hipps/csrc/runtime/rccl.cpp) on one GPU (nranks = 1: every
collective is a local copy through RCCL's own kernels; send/recv to self exercises the grouped
point-to-point path), and the sync engines on ``transport='rccl'``.  Multi-rank RCCL needs one GPU
per rank: tests/test_multigpu.py covers it on >= 2 devices."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def comm():
    from hipps.ops._native import native

    C = native()
    c = C.RcclComm(C.RcclComm.unique_id(), 1, 0)
    yield c
    c.destroy()


def test_collectives_single_rank(comm):
    s = torch.cuda.current_stream().cuda_stream
    x = torch.randn(1000, device=DEV)
    out = torch.empty(1000, device=DEV)
    comm.all_gather(x, out, s)
    g = torch.empty(1000, device=DEV)
    comm.gather(x, g, 0, s)
    b = x.clone()
    comm.broadcast(b, 0, s)
    v = torch.zeros(1500, device=DEV)
    comm.all_gather_v(x, v, [1000], [300], s)
    r = x.clone()
    comm.all_reduce_sum(r, s)
    torch.cuda.synchronize()
    for t in (out, g, b, r):
        assert torch.equal(t, x)
    assert torch.equal(v[300:1300], x) and v[:300].abs().sum() == 0
    assert comm.async_error() == 0 and comm.rank == 0 and comm.size == 1


def test_send_recv_to_self_grouped(comm):
    from hipps.ops._native import native

    C = native()
    s = torch.cuda.current_stream().cuda_stream
    x = torch.arange(4096, device=DEV, dtype=torch.int32)
    y = torch.empty_like(x)
    C.RcclComm.group_start()
    comm.send(x, 0, s)
    comm.recv(y, 0, s)
    C.RcclComm.group_end()
    torch.cuda.synchronize()
    assert torch.equal(x, y)


def test_split_and_abort():
    from hipps.ops._native import native

    C = native()
    c = C.RcclComm(C.RcclComm.unique_id(), 1, 0)
    sub = c.split(0, 0)
    assert sub is not None and sub.size == 1
    assert c.split(-1, 0) is None  # NCCL_SPLIT_NOCOLOR
    sub.destroy()
    c.abort()
    assert not c.alive
    with pytest.raises(RuntimeError, match="aborted"):
        c.broadcast(torch.zeros(4, device=DEV), 0, torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("mode", ["allgather", "ps_sync"])
def test_sync_engine_on_native_rccl_matches_local(mode):
    import hipps

    res = []
    for kw in ({"mode": "local"}, {"mode": mode, "transport": "rccl"}):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, 10)).to(DEV)
        opt = hipps.SGD(m.named_parameters(), lr=0.1, momentum=0.9, code="fp32", **kw)
        g = torch.Generator().manual_seed(1)
        for _ in range(4):
            x, y = torch.randn(32, 64, generator=g).to(DEV), torch.randint(0, 10, (32,), generator=g).to(DEV)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
        torch.cuda.synchronize()
        if kw.get("transport"):
            assert opt.engine.rccl is not None
        opt.close()
        res.append([p.detach().clone() for p in m.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_comm_bench_single_rank(tmp_path):
    """bench/comm_bench.py at N = 1 (one-rank RCCL group, IPC mailbox, pull kernel) runs and
    reports every row."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "comm.json"
    r = subprocess.run([sys.executable, os.path.join(root, "bench", "comm_bench.py"), "--sizes-mb", "1,4", "--iters",
                        "3", "--out", str(out)], cwd=root, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    ops = {row["op"] for row in json.load(open(out))}
    assert {"torch.all_gather", "torch.broadcast", "ipc.push", "ipc.pull_kernel", "local.copy"} <= ops
