"""Host-side cost per call of the ResNet-50 fc GEMMs (bs256: [256, 2048] x [1000, 2048]^T) through
PyTorch's BLAS dispatch, hipBLASLt vs rocBLAS: the 200 us host gap before the fc backward GEMM in
the steady table (profiles/r5/final/steady.txt) sits exactly there.  Host time per call is the
enqueue time with the GPU kept busy (no sync inside the loop).

    python tools/diag/blas_host_cost.py
"""
import time

import torch


def host_us(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    # keep the GPU busy so enqueue never waits
    big = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    for _ in range(20):
        big.fill_(1)
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    dt = (time.perf_counter() - t) / iters * 1e6
    torch.cuda.synchronize()
    return dt


def main():
    dev = "cuda"
    x = torch.randn(256, 2048, device=dev).bfloat16()
    w = torch.randn(1000, 2048, device=dev).bfloat16()
    dy = torch.randn(256, 1000, device=dev).bfloat16()
    b = torch.randn(1000, device=dev).bfloat16()
    dw = torch.empty(1000, 2048, device=dev)
    y = torch.empty(256, 1000, device=dev, dtype=torch.bfloat16)
    cases = {
        "fwd addmm bias": lambda: torch.addmm(b, x, w.t(), out=y),
        "bwd dx mm": lambda: torch.mm(dy, w),
        "bwd dw mm fp32 out": lambda: torch.ops.aten.mm.dtype_out(dy.t(), x, torch.float32, out=dw),
        "bwd dw mm bf16": lambda: torch.mm(dy.t(), x),
        "empty launch (fill_)": lambda: y.fill_(0),
    }
    for lib in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:  # noqa: BLE001
            print(f"{lib}: {e}")
            continue
        for name, fn in cases.items():
            print(f"{lib:9s} {name:22s} {host_us(fn):8.1f} us/call host", flush=True)


if __name__ == "__main__":
    main()
