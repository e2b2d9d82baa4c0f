"""Host-side cProfile of steady training steps only (setup and warmup excluded): where the Python
side of forward / backward / opt.step() spends its time.

    python tools/diag/step_prof.py --model bert-base --batch 32 --seq 512 [--steps 10]
"""
import argparse
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import hipps
    from hipps.models.transformer import build

    torch.manual_seed(0)
    m = build(a.model).cuda()
    opt = hipps.SGD(m.named_parameters(), lr=1e-4, momentum=0.9, mode="ps_async", code="bf16", average=True)
    ids = torch.randint(0, m.c.vocab, (a.batch, a.seq), device="cuda")

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(ids, ids)
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)
    if a.out:
        st.dump_stats(a.out)
    opt.close()


if __name__ == "__main__":
    main()
