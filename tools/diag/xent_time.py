"""Time the fused cross-entropy forward / backward (csrc/xent.hip) on a BERT-sized logits matrix.

    python tools/diag/xent_time.py [rows] [vocab]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hipps.ops.nn as hnn  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    vocab = int(sys.argv[2]) if len(sys.argv) > 2 else 30522
    x = torch.randn(rows, vocab, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, vocab, (rows,), device="cuda")
    for _ in range(3):
        hnn.cross_entropy(x, y).backward()
    torch.cuda.synchronize()
    f, b = [], []
    for _ in range(10):
        e0, e1, e2 = (torch.cuda.Event(True) for _ in range(3))
        e0.record()
        loss = hnn.cross_entropy(x, y)
        e1.record()
        loss.backward()
        e2.record()
        torch.cuda.synchronize()
        f.append(e0.elapsed_time(e1))
        b.append(e1.elapsed_time(e2))
    gb = rows * vocab * 2 / 1e9
    fm, bm = sorted(f)[5], sorted(b)[5]
    print(f"xent {rows}x{vocab}: forward {fm * 1e3:.1f} us ({gb / fm:.2f} TB/s), "
          f"backward {bm * 1e3:.1f} us ({2 * gb / bm:.2f} TB/s incl. the grad write)")


if __name__ == "__main__":
    main()
