"""PSConfig: every engine knob in one place.

The reference has only constructor kwargs (ps.py:54-59) and hard-coded constants (pool size
200 ps.py:85, blosc level 0 mpi_comms.py:18, 32-byte sentinel mpi_comms.py:80, 15 KiB slot floor
mpi_comms.py:82-83, accumulate count 32 README.md:69).  Here they are fields, filled from
kwargs, then overridden by ``HIPPS_<FIELD>`` environment variables (e.g. ``HIPPS_MODE=ps_async``,
``HIPPS_CODEC=topk:0.01``, ``HIPPS_ACCUMULATE=8``).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, fields
from typing import Optional

MODES = ("auto", "local", "allgather", "ps_sync", "ps_async")


@dataclass
class PSConfig:
    # local | allgather (reference ps.py semantics) | ps_sync | ps_async (AsySG-InCon)
    mode: str = "auto"
    # codec spec or object; see hipps.codecs.get_codec
    codec: object = None
    # async PS: gradients summed per update (README.md:69 uses 32); 0 -> world size
    accumulate: int = 0
    # async PS: drop gradients computed on params older than (version - staleness); -1 = never
    staleness: int = -1
    # async PS: a worker blocks in irequest_params() until the published params include all but
    # its newest `max_delay` gradients (SSP-style bound; 0 = synchronous per worker; -1 = unbounded)
    max_delay: int = -1
    # async PS: pull the newest published params at the end of every step() (AsySG-InCon read)
    auto_pull: bool = True
    # async PS parameter pull on a GPU: 'device' (the GPU picks the newest published version when
    # it reaches the pull, right before the next forward, and copies it in stream order; needs
    # GPU-rung doorbells) | 'prefetch' (host-chosen version, side-stream copy adopted at the next
    # step) | 'direct' (host-chosen, copy on the compute stream)
    pull: str = "device"
    # async PS data path: 'ipc' (workers map the PS's mailbox and copy one-sidedly over xGMI, GPU
    # doorbells) | 'p2p' (two-sided send/recv: RCCL pair communicators through torch.distributed on
    # GPU, gloo on CPU -- the fallback when IPC memory cannot be mapped)
    async_transport: str = "ipc"
    # async PS topology: False = rank 0 is the PS *and* worker 0 (default: N GPUs train); True =
    # the reference's topology (README.md:64-75): rank 0 only receives, sums, steps and publishes,
    # ranks 1..N-1 are the workers (rank 0 calls opt.serve() instead of training)
    ps_dedicated: bool = False
    # async PS update/publication granularity: 'model' (one version for the whole model: the PS
    # steps once M complete worker steps arrived) | 'bucket' (README.md:64-76, the reference PS
    # steps and broadcasts each parameter on its own: every bucket is updated and published as soon
    # as M messages for it arrived, workers adopt the newest version of each bucket -- reads may
    # mix versions across buckets; ipc transport only) | 'auto' (bucket where it applies -- ipc
    # transport, device codecs -- model otherwise; the default: on the headline config plain
    # AsySG-InCon converges like local SGD with it and oscillates with whole-model versions,
    # profiles/r4/traj_headline.json)
    ps_granularity: str = "auto"
    # async PS: push each bucket's message from its backward hook as soon as it is encoded
    # ('auto' = on for the ipc transport), instead of all messages at step(): the PS accumulates
    # (and with ps_granularity='bucket' updates and publishes) the last layers' buckets while the
    # worker still runs backward.  A gradient arriving later for a pushed bucket (backward()
    # twice before step() without opt.no_sync()) is an error.  'auto' | 'on' | 'off'
    push_early: str = "auto"
    # async PS: scale a kept gradient by 1/max(1, staleness) (staleness-aware async SGD)
    staleness_lr: bool = False
    # async PS look-ahead publish (delay-compensated momentum, DANA-style; NOT part of the
    # reference's AsySG-InCon, README.md:56-81, which reads the PS's parameters as they are):
    # workers read the parameters extrapolated by the momentum of the next tau updates, the tau
    # updates their gradient will arrive late by; the PS master is unchanged.  0 = off (default:
    # the reference's algorithm), -1 = auto (tau = mean measured staleness of the recent accumulated
    # steps; off when max_delay == 0), > 0 = fixed tau
    stale_lookahead: float = 0.0
    # rehearsal knob (one process, one GPU): the co-located PS also carries the load of this many
    # emulated remote workers -- every message of worker 0 is accumulated 1 + E times (one launch
    # each; the update scales by 1/(1+E), so the math is unchanged) and every update is followed by
    # E write sweeps of the step's wire bytes (their pushes landing in HBM) and E read sweeps of the
    # published parameters (their pulls), from 8 workgroups on the PS stream (on a real node that
    # traffic moves over xGMI without running on this GPU's CUs)
    emulate_remote: int = 0
    # ps_async on GPUs: no end-of-backward join of the weight-gradient side stream into the caller's
    # stream -- every gradient the engine reads is ordered after that stream by its per-bucket
    # encode, so the next step's pull and forward run beside the last weight gradients (ResNet-50:
    # the stem and layer 1, +0.7 %, profiles/r5/defer/).  Only for loops that do not read
    # param.grad between backward() and step() (gradient clipping, logging): call
    # opt.join_grads() before such a read
    defer_wgrad_join: bool = False
    # samples per worker step (e.g. the batch size): adds samples_per_sec to step() data
    samples_per_step: int = 0
    # async PS failure detection: a worker silent for this long (no heartbeat, no STOP) is dead
    dead_after_s: float = 60.0
    # async PS mailbox: bucket messages in flight per worker (0 = auto: min(2*buckets, mailbox_mb))
    mailbox_slots: int = 0
    mailbox_mb: float = 4096.0
    # async PS rotating published-parameter buffers (0 = auto: 4, lowered to 2 -- and the mailbox
    # rings shrunk toward two of the largest message -- when rank 0's HBM budget needs it,
    # ps_async.plan_geometry)
    npub: int = 0
    # bucket size for hook-driven encode overlap (also the async PS message / version granularity:
    # ResNet-50 is 7 buckets at 16 MB)
    bucket_mb: float = 16.0
    # scale the rank-summed gradient by 1/accumulate (reference sums: ps.py:176)
    average: bool = False
    # encode buckets from post-accumulate-grad hooks on a side stream during backward
    overlap: bool = True
    # GPU distributed modes: gather autograd-owned grads per bucket with one multi-tensor kernel
    # instead of accumulating into preset flat-buffer views (161 fewer kernels for ResNet-50)
    grad_gather: bool = True
    # published-parameter wire dtype for PS modes: 'fp32' | 'bf16' | 'auto' (bf16 for ps_async with
    # more than one GPU rank, fp32 otherwise -- ps_sync 'bf16' halves the broadcast but leaves the
    # non-PS replicas on bf16-rounded copies of the PS's fp32 parameters)
    param_wire: str = "auto"
    # bf16 weight shadow: one flat bf16 copy of the fp32 params, refreshed by one cast kernel after
    # every step()/irequest_params(), read by the hipps conv kernels instead of one autocast cast
    # per layer per forward.  'auto' = on for ps_async on a GPU for models with conv or Linear
    # weights (hipps.ops.nn.Linear reads it too; the engine owns the params there:
    # any out-of-band edit is overwritten by the next adoption anyway); 'on' | 'off' otherwise.
    # With 'on', call opt.refresh_bf16_weights() after editing params outside step().
    bf16_weights: str = "auto"
    # parameters that produced no gradient this step are left untouched -- no weight decay, no
    # momentum step (ps.py:178-179 `if p.grad is None: continue`); the sync modes OR the
    # per-rank presence so replicas stay identical, the async PS ORs the accumulated messages'
    skip_missing_grads: bool = True
    # raise ValueError when a parameter produced no gradient (the reference's ps.py:118-119 check)
    require_all_grads: bool = False
    # sync-mode collectives: 'torch' (torch.distributed: RCCL process group / gloo) | 'rccl'
    # (hipps' native RCCL communicator, hipps/csrc/runtime/rccl.cpp: ncclGather for the PS
    # gather, ncclCommGetAsyncError polling every step, ncclCommAbort from the watchdog)
    transport: str = "torch"
    # collective / transport timeout: the process-group timeout for the sync modes and the
    # async PS's waits; a watchdog thread aborts the process (exit code 3) if one step's
    # exchange exceeds it, instead of hanging on a dead peer
    comm_timeout_s: float = 600.0
    # ObjectCodec (reference encode/decode/.codes objects): max serialized bytes per rank per
    # step in the async PS mailbox (0 = auto: 2x the fp32 model + 1 MiB)
    object_slot_mb: float = 0.0
    # host pickle slow path compression level (mpi_comms.py:18; 0 = framing only)
    compress_level: int = 0
    # Adam eps placement: 'reference' (ps.py:255) or 'torch'
    adam_variant: str = "reference"
    # all-gather a hash of the posting sequence each step and assert equality (race detector)
    debug_check_order: bool = False
    # write a 16-byte 0x29 canary after every bucket message (the device analogue of the reference
    # sentinel, mpi_comms.py:80,101-103) and verify it after encode and after every transfer
    debug_canary: bool = False
    # device phase timing with HIP events + roctx ranges (encode_ms / comm_ms / update_ms keys)
    trace: bool = False
    # metrics JSONL path (per rank; '{rank}' is substituted)
    metrics_path: Optional[str] = None

    @classmethod
    def from_kwargs(cls, **kw) -> "PSConfig":
        names = {f.name for f in fields(cls)}
        cfg = cls(**{k: v for k, v in kw.items() if k in names and v is not None})
        cfg.apply_env()
        cfg.validate()
        return cfg

    def apply_env(self):
        for f in fields(self):
            v = os.environ.get("HIPPS_" + f.name.upper())
            if v is None:
                continue
            cur = getattr(self, f.name)
            if isinstance(cur, bool) or f.type in ("bool",):
                val = v.lower() in ("1", "true", "yes", "on")
            elif isinstance(cur, int) and not isinstance(cur, bool):
                val = int(v)
            elif isinstance(cur, float):
                val = float(v)
            else:
                val = v
            setattr(self, f.name, val)

    def validate(self):
        if self.mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}, got {self.mode!r}")
        if self.pull not in ("device", "prefetch", "direct"):
            raise ValueError("pull must be 'device', 'prefetch' or 'direct'")
        if self.param_wire not in ("fp32", "bf16", "auto"):
            raise ValueError("param_wire must be 'fp32', 'bf16' or 'auto'")
        if self.bf16_weights not in ("auto", "on", "off"):
            raise ValueError("bf16_weights must be 'auto', 'on' or 'off'")
        if self.async_transport not in ("ipc", "p2p"):
            raise ValueError("async_transport must be 'ipc' or 'p2p'")
        if self.transport not in ("torch", "rccl"):
            raise ValueError("transport must be 'torch' or 'rccl'")
        if self.push_early not in ("auto", "on", "off"):
            raise ValueError("push_early must be 'auto', 'on' or 'off'")
        if self.ps_granularity not in ("model", "bucket", "auto"):
            raise ValueError("ps_granularity must be 'model', 'bucket' or 'auto'")
        if self.adam_variant not in ("reference", "torch"):
            raise ValueError("adam_variant must be 'reference' or 'torch'")

    def replace(self, **kw) -> "PSConfig":
        return dataclasses.replace(self, **kw)
