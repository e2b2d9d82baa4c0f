#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 synthetic-ImageNet async parameter server (AsySG-InCon), bf16.

BASELINE.json metric "samples/sec (node) ResNet-50 async PS at 1/2/4/8 MI355X; grad bytes/step".
One process per GPU; rank 0 is the PS (and also trains, as worker 0); every rank trains
ResNet-50 (random init, 224x224 synthetic images, 1000 classes) with autocast-bf16 compute and
fp32 parameters; gradients go to the PS through the bf16 wire codec; the PS applies SGD-momentum
to an fp32 master with the fused HIP kernel and publishes new parameters that workers pull
one-sidedly (HIP-IPC over xGMI).

    python bench.py                                   # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Timing: W warmup steps, then barrier + synchronize, K timed steps, barrier + synchronize; the
per-rank elapsed time is max-reduced; rank 0 prints one JSON line.  value = whole-job samples/s
(N x per-GPU batch x K / max elapsed).  Weak scaling: per-GPU batch fixed as N grows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "samples/sec (node) ResNet-50 async PS at 1/2/4/8 MI355X; grad bytes/step"
TIMED_HOOKS: list = []  # callables(bool): True right before the timed steps, False right after (tools/)
TRANSFORMERS = ("bert-base", "bert-tiny", "llama3-8b", "llama3-1b", "llama-tiny")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--mode", default="ps_async", choices=["ps_async", "ps_sync", "allgather", "local"])
    ap.add_argument("--codec", default="bf16")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--accumulate", type=int, default=0, help="PS update every M grads (0 = world size)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--seq", type=int, default=512, help="sequence length (transformer configs)")
    ap.add_argument("--param-wire", default="auto", choices=["auto", "fp32", "bf16"],
                    help="published-parameter dtype: auto = fp32 at N=1 (local pull), bf16 at N>1 (halves the "
                         "xGMI pull; the PS keeps the fp32 master, workers compute in bf16 anyway)")
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--optim", default="sgd", choices=["sgd", "adam"],
                    help="the PS optimizer: the reference's SGD (ps.py:195-214) or Adam (ps.py:217-261)")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="bucket size in MB (default: the library's, PSConfig.bucket_mb)")
    ap.add_argument("--granularity", default=None, choices=["model", "bucket", "auto"],
                    help="ps_async update/publication granularity (default: the library's, PSConfig.ps_granularity)")
    ap.add_argument("--lookahead", type=float, default=None,
                    help="ps_async look-ahead publish tau (default: the library's, PSConfig.stale_lookahead = 0: "
                         "plain AsySG-InCon, the reference's algorithm; -1 = auto delay compensation)")
    ap.add_argument("--mailbox-slots", type=int, default=0,
                    help="ps_async: bucket messages in flight per worker (0 = the library's auto)")
    ap.add_argument("--no-defer-wgrad-join", action="store_true",
                    help="join the weight-gradient side stream at the end of every backward (the library "
                         "default); the bench's loop reads no param.grad between backward and step, so by "
                         "default it lets the async PS order its gradient reads itself (defer_wgrad_join)")
    ap.add_argument("--gc", default=os.environ.get("BENCH_GC", "freeze"), choices=["freeze", "default", "off"],
                    help="Python garbage collector during the timed steps: 'freeze' (default) moves every object "
                         "alive after warmup (model, optimizer, autograd machinery) out of the collector's "
                         "generations, so periodic full collections no longer stall the host at step boundaries; "
                         "'off' disables it for the timed steps; 'default' leaves it alone")
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--nondeterministic", action="store_true",
                    help="let MIOpen use its non-deterministic convolution algorithms (default: "
                         "hipps.set_deterministic, bit-for-bit repeatable steps at no measured cost)")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--no-fallback", action="store_true",
                    help="fail if the ps_async IPC transport refuses to initialise (default: when the driver call "
                         "returned an error, run the SAME async PS over its p2p transport -- RCCL pair send/recv -- "
                         "and record that in the JSON line; a TIMED-OUT import always exits non-zero)")
    ap.add_argument("--allow-fallback", action="store_true", help=argparse.SUPPRESS)  # round-1 flag, now the default
    ap.add_argument("--async-transport", default="ipc", choices=["ipc", "p2p"])
    ap.add_argument("--no-pull-overlap", action="store_true",
                    help="ps_async: one GPU-time pull of all params before the forward (A/B)")
    ap.add_argument("--ps-dedicated", action="store_true",
                    help="reference topology (README.md:64-75): rank 0 only serves, ranks 1..N-1 train; the value "
                         "counts the N-1 workers' samples")
    ap.add_argument("--emulate-workers", type=int, default=0,
                    help="rehearse the N=8 PS load on ONE GPU: launch 1+E ranks (HIPPS_BACKEND=gloo); rank 0 trains "
                         "as worker 0 + PS, ranks 1..E push real bucket messages and pull parameters in lockstep "
                         "with worker 0 without computing (the PS-side load of E remote workers)")
    ap.add_argument("--emulate-remote", type=int, default=0,
                    help="N=1 rehearsal of the co-located PS at N=1+E: the PS also accumulates E emulated remote "
                         "messages per step and sweeps their push / pull bytes (PSConfig.emulate_remote)")
    return ap.parse_args()


def main():
    a = parse()
    if os.environ.get("BENCH_HANG_DUMP"):
        # diagnosis of a hung run: every rank prints all its threads' Python stacks after this
        # many seconds and exits
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["BENCH_HANG_DUMP"]), exit=True)
    from hipps.parallel import dist as hdist

    world = hdist.init_from_env()
    if world.size != a.gpus and world.rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world.size}; using WORLD_SIZE", file=sys.stderr)
    N = world.size
    dev = torch.device("cuda", torch.cuda.current_device())
    if os.environ.get("BENCH_HIPRIO") == "1":
        # the training step on a high-priority stream (the weight-gradient side stream and the
        # bucket comm stream stay at the default priority): A/B of CU arbitration between the
        # input-gradient chain and the work beside it
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    torch.backends.cudnn.benchmark = True

    import hipps
    import hipps.ops.nn as hnn
    from hipps.models import build_model

    hipps.set_deterministic(not a.nondeterministic)

    torch.manual_seed(1234 + world.rank)
    is_tf = a.model in TRANSFORMERS
    model = build_model(a.model).to(dev)
    cl = not a.no_channels_last and not is_tf
    if cl:
        model = model.to(memory_format=torch.channels_last)
    if is_tf:
        vocab = model.c.vocab
        x = torch.randint(0, vocab, (a.batch, a.seq), device=dev)
        y = torch.randint(0, vocab, (a.batch, a.seq), device=dev)
    else:
        x = torch.randn(a.batch, 3, a.image, a.image, device=dev)
        if cl:
            x = x.contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (a.batch,), device=dev)

    emulated = a.emulate_workers > 0 and world.rank > 0
    if a.emulate_workers and N != a.emulate_workers + 1:
        raise SystemExit(f"--emulate-workers {a.emulate_workers} needs WORLD_SIZE={a.emulate_workers + 1}")
    if emulated:  # tiny batch: only the gradients' shapes matter, the messages are real bucket images
        x, y = x[:2, :, :64, :64].contiguous(memory_format=torch.channels_last), y[:2]
    mode = a.mode if N > 1 or a.mode in ("ps_async", "local") else "local"
    if a.param_wire == "auto":
        a.param_wire = "bf16" if N > 1 else "fp32"
    note = None
    dedicated = bool(a.ps_dedicated and mode == "ps_async" and N > 1)
    from hipps.config import PSConfig

    dflt = PSConfig()
    dflt.apply_env()  # HIPPS_<FIELD> overrides count as the defaults (and are recorded below)
    if a.granularity is None:
        a.granularity = dflt.ps_granularity
    if a.lookahead is None:
        a.lookahead = dflt.stale_lookahead
    if a.bucket_mb is None:
        a.bucket_mb = dflt.bucket_mb
    kw = dict(lr=a.lr, momentum=a.momentum, weight_decay=5e-5, mode=mode, code=a.codec,
              accumulate=a.accumulate or None, average=True, param_wire=a.param_wire, bucket_mb=a.bucket_mb,
              mailbox_slots=a.mailbox_slots, ps_granularity=a.granularity, stale_lookahead=a.lookahead,
              async_transport=a.async_transport, ps_dedicated=dedicated)
    if mode == "ps_async":
        kw["defer_wgrad_join"] = not a.no_defer_wgrad_join
    if a.emulate_remote and N == 1:
        kw["emulate_remote"] = a.emulate_remote
    from hipps.parallel.ps_async import IPCOpenTimeout

    ocls = hipps.SGD
    if a.optim == "adam":  # (betas / eps: the reference's defaults; no momentum argument)
        ocls = hipps.Adam
        kw.pop("momentum")
    try:
        opt = ocls(model.named_parameters(), **kw)
    except IPCOpenTimeout as e:
        # a mailbox import is stuck inside the HIP driver on some rank (every rank learnt it
        # through the setup agreement): no other engine is built in this process -- report the
        # stuck thread's diagnostic and exit non-zero without interpreter teardown (which could
        # block on that thread)
        print(f"[bench] rank {world.rank}: FATAL ps_async mailbox import timed out: {e}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(3)
    except Exception as e:
        # a clean refusal (the driver call returned an error: no thread is left inside it): the
        # same async PS algorithm over its two-sided (RCCL pair send/recv) transport, recorded in
        # the JSON line; never a different mode under the async-PS metric
        if mode != "ps_async" or N == 1 or a.no_fallback or a.async_transport == "p2p":
            raise
        note = f"ps_async ipc transport failed ({type(e).__name__}: {e}); fell back to the p2p transport"
        print("[bench] " + note, file=sys.stderr)
        kw["async_transport"] = "p2p"
        kw["ps_granularity"] = "model"  # per-bucket publication needs the ipc transport
        opt = ocls(model.named_parameters(), **kw)
    if mode == "ps_async" and N > 1:
        eng0 = opt.engine
        print(f"[bench] rank {world.rank}: mailbox mapped {getattr(eng0, 'mapped_bytes', 0) / 2**20:.1f} MiB "
              f"(ring {eng0.ring_bytes / 2**20:.1f} MiB + publish {eng0.NPUB} x {eng0.pub_bytes / 2**20:.1f} MiB) "
              f"in {getattr(eng0, 'open_s', 0.0):.3f} s", file=sys.stderr, flush=True)
    # N > 1: pull the last stage's parameters (ResNet layer4 + fc: 2/3 of the model) over xGMI on a
    # side stream, overlapped with the forward of layers 1-3.  At N = 1 the pull is a local
    # 0.1 ms copy and the split costs more than it hides (A/B: 10099 vs 10170 img/s)
    pull_overlap = bool(N > 1 and not a.no_pull_overlap and hasattr(model, "layer4")
                        and opt.overlap_pull(model.layer4))

    host_t = [0.0] * 7 if os.environ.get("HIPPS_HOST_TIMING") else None  # diagnostics: host s per phase

    def step():
        if host_t is not None:
            t = [time.perf_counter()]
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            # (the fused bf16 cross-entropy, csrc/xent.hip: one read of the logits forward, one
            # read + gradient write backward, instead of PyTorch's log-softmax / nll kernels)
            loss = model(x, y) if is_tf else hnn.cross_entropy(model(x), y)
        if host_t is not None:
            t.append(time.perf_counter())
        loss.backward()
        if host_t is not None:
            t.append(time.perf_counter())
        _, data = opt.step()
        if host_t is not None:
            t.append(time.perf_counter())
            for i in range(3):
                host_t[i] += t[i + 1] - t[i]
            host_t[3] += 1
            for i, k in enumerate(("slot_wait", "code_wait", "comm_wait")):
                host_t[4 + i] += float(data.get(k, 0.0))
        return loss, data

    ps_only = bool(getattr(opt, "ps_only", False))
    if emulated:
        # gradients once; every step re-encodes and pushes them (real bucket images through the
        # real mailbox / doorbells) and pulls the newest parameters -- paced so that message k is
        # pushed after worker 0 pushed its step k, as identical GPUs would
        with torch.autocast("cuda", dtype=torch.bfloat16):  # zero gradients: load without perturbing training
            (0.0 * F.cross_entropy(model(x), y)).backward()
        eng = opt.engine
        nb = len(eng.plan.buckets)
        k = [0]

        def step():  # noqa: F811
            k[0] += 1
            eng.ctl.wait_ge(eng.C.F_PUSH_SEQ, 0, (k[0] - 1) * nb + 1, 600 * 1000000)
            _, data = opt.step()
            return None, data
    elif ps_only:
        def step():  # noqa: F811  -- the PS thread serves; rank 0's main thread only times
            return None, {}

    first_loss = None
    losses = []  # device scalars; read after the timed region (no host sync inside it)
    for _ in range(a.warmup):
        loss, _ = step()
        if loss is not None:
            losses.append(loss.detach())
            if first_loss is None:
                first_loss = float(loss.float().item())
    tr = opt.engine.tracer  # HIPPS_TRACE=1: per-phase device ms (HIP events), excluded from warmup
    if tr.enabled:
        torch.cuda.synchronize()
        tr.flush()
        tr.totals.clear()
    import gc

    if a.gc != "default":
        gc.collect()
        gc.freeze()  # long-lived objects leave the collector's generations (Python >= 3.7)
        if a.gc == "off":
            gc.disable()
    hdist.barrier(world)
    torch.cuda.synchronize()
    if host_t is not None:
        host_t[:] = [0.0] * 7
        ms0 = torch.cuda.memory_stats(dev)
        seq0 = getattr(opt.engine, "seq", 0)
    for hook in TIMED_HOOKS:
        hook(True)
    t0 = time.perf_counter()
    last = None
    for _ in range(a.steps):
        loss, last = step()
        if loss is not None:
            losses.append(loss.detach())
    for hook in TIMED_HOOKS:
        hook(False)
    torch.cuda.synchronize()
    hdist.barrier(world)
    t1 = time.perf_counter()
    if a.gc == "off":
        gc.enable()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev if world.backend == "nccl" else "cpu")
    if N > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    if host_t is not None and host_t[3]:
        print("[bench] host ms/step: forward %.2f backward %.2f step %.2f (wall %.2f); waits: slot %.2f "
              "encode %.2f pull %.2f" % tuple([1e3 * v / host_t[3] for v in host_t[:3]] + [1e3 * elapsed / a.steps]
                                              + [1e3 * v / host_t[3] for v in host_t[4:]]), file=sys.stderr)
        if hasattr(opt.engine, "wait_summary"):
            print("[bench] mailbox waits (timed steps): " + opt.engine.wait_summary(seq0), file=sys.stderr)
        ms1 = torch.cuda.memory_stats(dev)
        print("[bench] allocator during timed steps: " + " ".join(
            f"{k}+{ms1.get(k, 0) - ms0.get(k, 0)}" for k in ("num_alloc_retries", "num_device_alloc", "num_device_free",
                                                              "num_sync_all_streams", "segment.all.allocated"))
              + f" reserved={ms1.get('reserved_bytes.all.current', 0) / 2**30:.1f} GiB", file=sys.stderr)
    if dedicated and N > 1:  # the losses live on the workers: rank 1 reports them
        box = [(first_loss, [float(v.float()) for v in losses], last)]
        allb = [None] * N
        dist.all_gather_object(allb, box[0])
        if world.rank == 0:
            first_loss, lvals, last = allb[1]
            losses = [torch.tensor(v) for v in lvals]
            loss = losses[-1]
    final_loss = float(loss.float().item()) if loss is not None else float("nan")
    grad_bytes = int(last.get("grad_bytes_sent", 0)) if last else 0
    # bytes that carry information in the last step's messages (reads the device count header of
    # variable-size codecs; outside the timed region)
    grad_used = opt.engine.wire_bytes_used() if not opt.engine.is_object else grad_bytes
    trace = None
    if tr.enabled:
        tr.flush()
        trace = {k: round(v / a.steps, 4) for k, v in tr.totals.items()}
    nbuckets = len(opt.engine.plan.buckets)
    gran_eff = getattr(opt.engine, "granularity", None)
    ti = opt.engine.transport_info() if hasattr(opt.engine, "transport_info") else {}
    nparams = sum(p.numel() for p in model.parameters())
    opt.close()
    stats = {}
    if hasattr(opt, "_last_engine_stats"):
        stats = opt._last_engine_stats
    per_sample = a.seq if is_tf else 1
    trainers = N - 1 if dedicated else (1 if a.emulate_workers else N)
    value = trainers * a.batch * per_sample * a.steps / elapsed
    if world.rank == 0:
        metric = METRIC if a.model == "resnet50" else (
            f"{'tokens' if is_tf else 'samples'}/sec (node) {a.model} {mode} (secondary BASELINE config)")
        if a.emulate_remote and N == 1:
            metric = (f"worker-0 samples/sec with the co-located PS carrying {a.emulate_remote} emulated remote "
                      "workers (one GPU; rehearsal, not the headline)")
        if a.emulate_workers:
            metric = (f"worker-0 samples/sec under an emulated {a.emulate_workers}-worker async PS load on one GPU "
                      "(rehearsal, not the headline)")
        rec = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "tokens/s" if is_tf else "samples/s",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("synthetic (random tokens, random-init weights)" if is_tf else
                     "synthetic (random 224x224 images / labels, random-init weights)"),
            "config": {
                "model": a.model,
                "per_gpu_batch": a.batch,
                "seq_len": a.seq if is_tf else None,
                "image": None if is_tf else a.image,
                "parallelism": (f"dp{N - 1} {mode} (rank0 = dedicated PS, ranks 1..{N - 1} = workers)" if dedicated
                                else f"dp{N} {mode} (rank0 = PS + worker)" if not a.emulate_workers
                                else f"1 worker + PS, {a.emulate_workers} emulated workers on the same GPU"),
                "global_batch": a.batch * trainers,
                "codec": a.codec,
                "optimizer": a.optim if a.optim == "adam" else f"sgd(momentum={a.momentum})",
                "accumulate": a.accumulate or N,
                "grad_bytes_per_step_per_worker": grad_bytes,
                "grad_bytes_per_step_used": int(grad_used),
                "param_wire": a.param_wire, "pull_overlap": pull_overlap,
                "async_transport": kw.get("async_transport") if mode == "ps_async" else None,
                # which algorithm ran: AsySG-InCon (README.md:56-81) reads the PS's parameters as
                # published (stale_lookahead 0); > 0 / -1 = delay-compensated (look-ahead) publish
                "algorithm": ("AsySG-InCon" + ("" if kw.get("stale_lookahead", 0) == 0 else
                                               " + look-ahead publish (delay compensation)"))
                if mode == "ps_async" else mode,
                "ps_granularity": gran_eff if mode == "ps_async" else None,
                "stale_lookahead": kw.get("stale_lookahead") if mode == "ps_async" else None,
                "bucket_mb": a.bucket_mb,
                "mailbox": ({"ring_mb_per_worker": round(ti.get("ring_bytes", 0) / 2**20, 1),
                             "message_slots": ti.get("mailbox_slots"), "direct_push": ti.get("direct_push"),
                             "npub": ti.get("npub"),
                             "rank0_budget_gb": ti.get("budget_gb")}
                            if mode == "ps_async" else None),
                "python_gc": a.gc,
                "deterministic": not a.nondeterministic,
                "wgrad_join": ("deferred" if mode == "ps_async" and not a.no_defer_wgrad_join else "end of backward"),
                "num_params": nparams,
                "buckets": nbuckets,
            },
            "first_loss": None if first_loss is None else round(first_loss, 4),
            "final_loss": round(final_loss, 4),
            # every 5th step's loss (warmup included), read back after timing
            "loss_every5": [round(float(v.float()), 4) for v in losses[::5]],
            "staleness_last": last.get("staleness") if last else None,
            "ps": {k: (int(v) if isinstance(v, (int, float)) else v) for k, v in stats.items()},
            "ps_staleness_mean": (round(stats["staleness_sum"] / stats["accumulated"], 3)
                                  if stats.get("accumulated") else None),
        }
        if trace:
            rec["trace_device_ms_per_step"] = trace
        if note:
            rec["note"] = note
        line = json.dumps(rec)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    if N > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
