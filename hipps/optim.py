"""Reference-compatible optimizer API: ``MPI_PS``, ``SGD``, ``Adam`` (ps.py:53-261).

Constructor parity with the reference (ps.py:54-59)::

    opt = SGD(model.named_parameters(), model.parameters(), lr=0.1, momentum=0.9,
              code=codec, cuda=True)
    loss, data = opt.step()            # (loss, metrics) like ps.py:193

``named_params`` feeds the gradient hooks and names; ``*args`` goes to ``torch.optim`` exactly as
in the reference MRO (``SGD(MPI_PS, torch.optim.SGD)``).  If ``*args`` is omitted the params are
taken from ``named_params``.  ``optim`` ('sgd'/'adam') is inferred from the class.

What changed underneath (MI355X design):
  * parameters/gradients live in one flat fp32 buffer (hipps/parallel/flat.py); ``param.name``
    is not set (it is read-only on torch >= 2, ps.py:64) -- names are kept in a dict;
  * the update is ONE fused HIP kernel per param group (decode + sum_W + wd + momentum/Adam +
    optional publish cast) instead of ~6 eager ops per tensor (ps.py:197-261);
  * the exchange strategy is a config knob (``mode``): 'allgather' reproduces ps.py:140-190,
    'ps_sync' and 'ps_async' are the centralized PS of README.md:56-81.
"""
from __future__ import annotations

import time
from typing import Dict, Iterable, List, Optional, Tuple

import torch

from . import ops
from .codecs import get_codec
from .config import PSConfig
from .parallel import dist as hdist
from .parallel.flat import FlatStore


class _HyperGroup(dict):
    """A param group (dict) that calls ``notify()`` when a hyper-parameter changes value."""

    _KEYS = frozenset(("lr", "weight_decay", "momentum", "dampening", "nesterov", "betas", "eps", "amsgrad"))

    def __init__(self, d, notify):
        super().__init__(d)
        self._notify = notify

    def __setitem__(self, k, v):
        changed = k in self._KEYS and (k not in self or self[k] != v)
        super().__setitem__(k, v)
        if changed:
            self._notify()

    def __reduce__(self):  # (pickles / deep-copies as the plain dict torch expects)
        return (dict, (dict(self),))


class MPI_PS(torch.optim.Optimizer):
    """Base PS optimizer (ps.py:53).  Subclasses provide ``_update_group``."""

    optim = "base"

    def __new__(cls, *args, optim=None, **kwargs):
        # MPI_PS(..., optim='sgd' | 'adam') builds the matching subclass (the reference's MPI_PS
        # selects its update rule from ``optim``, ps.py:56, 182-190)
        if cls is MPI_PS:
            key = (optim or "sgd").lower()
            sub = {c.optim: c for c in MPI_PS.__subclasses__()}.get(key)
            if sub is None:
                raise ValueError(f"optim must be one of {sorted(c.optim for c in MPI_PS.__subclasses__())}")
            cls = sub
        return super().__new__(cls)

    def __init__(self, named_params, *args, names=(), optim=None, code=None, use_mpi=True, cuda=None,
                 config: Optional[PSConfig] = None, **kwargs):
        """``named_params, *args, names, optim, code, use_mpi, cuda`` as in ps.py:54-59; any
        :class:`PSConfig` field (mode, accumulate, staleness, max_delay, average, bucket_mb, ...)
        may be passed as a keyword; the rest goes to ``torch.optim`` (lr, momentum, betas, ...)."""
        import dataclasses

        named_params = list(named_params)
        if named_params and not isinstance(named_params[0], (tuple, list)):
            named_params = [(f"param{i}", p) for i, p in enumerate(named_params)]
        cfg_fields = {f.name for f in dataclasses.fields(PSConfig)}
        over = {k: kwargs.pop(k) for k in list(kwargs) if k in cfg_fields}
        over = {k: v for k, v in over.items() if v is not None}
        if code is not None:
            over["codec"] = code
        if not args:
            args = ([p for _, p in named_params],)
        super().__init__(*args, **kwargs)
        if optim is not None and optim != self.optim and self.optim != "base":
            raise ValueError(f"optim={optim!r} does not match optimizer class {type(self).__name__}")
        self.code = code
        self.use_mpi = use_mpi
        self.cuda = cuda
        self.names = list(names)
        self.cfg = (config or PSConfig()).replace(**over)
        self.cfg.apply_env()
        self.cfg.validate()
        self.codec = get_codec(self.cfg.codec)
        if self.code is None:
            self.code = self.codec
        # names: named_params order (the reference sets param.name, ps.py:63-64)
        self.param_names: Dict[int, str] = {id(p): n for n, p in named_params}
        seen = {id(p) for g in self.param_groups for p in g["params"]}
        missing = [n for n, p in named_params if id(p) not in seen]
        if missing:
            raise ValueError(f"named parameters not in the optimizer's param groups: {missing[:5]}")
        names = [self.param_names.get(id(p)) for g in self.param_groups for p in g["params"]]
        names = [n for n in names if n is not None]
        if len(names) != len(set(names)):  # ps.py:150-153
            repeated = sorted({x for x in names if names.count(x) > 1})
            raise ValueError(f"names not unique. Repeated names = {repeated}")
        # frozen parameters (requires_grad=False) are neither hooked, exchanged nor updated; they
        # keep their own storage (torch.optim skips them the same way: their .grad stays None)
        groups = [[p for p in g["params"] if p.requires_grad] for g in self.param_groups]
        self.frozen = [p for g in self.param_groups for p in g["params"] if not p.requires_grad]
        if not any(groups):
            raise ValueError("no trainable parameters (every parameter has requires_grad=False)")
        dev = next(p for g in groups for p in g).device
        self.world = hdist.current()
        self.store = FlatStore(groups, self.param_names, device=dev)
        self._init_state()
        self.steps = 0
        self.engine = self._make_engine()
        self._watch_hyper()
        bw = self.cfg.bf16_weights
        # auto: where a reader exists -- the hipps conv kernels (4-D weights) and hipps.ops.nn.Linear
        # (parameters tagged reads_bf16_shadow, _ShadowLinear) read the shadow instead of autocast casting every weight in
        # every forward; for Llama-3-8B the 16 GB shadow replaces the same 16 GB of per-forward
        # autocast copies held until backward
        has_reader = any(s.param.dim() == 4 or getattr(s.param, "reads_bf16_shadow", False) for s in self.store.slots)
        if bw == "on" or (bw == "auto" and self.mode == "ps_async" and self.store.device.type == "cuda" and has_reader):
            self.store.enable_bf16_shadow()
        self._metrics = None
        if self.cfg.metrics_path:
            from .utils.metrics import MetricsWriter

            self._metrics = MetricsWriter(self.cfg.metrics_path, self.world.rank)

    # ------------------------------------------------------------------ engine
    def _make_engine(self):
        from .parallel.engine import AllGatherEngine, LocalEngine, PSSyncEngine

        mode = self.cfg.mode
        if mode == "auto":
            mode = "allgather" if self.world.size > 1 else "local"
        self.mode = mode
        if self.cfg.param_wire == "auto":
            # (self.cfg is this optimizer's own copy: PSConfig.replace in __init__)
            # the async PS moves whole-model parameter versions every step: at W > 1 on GPUs they go
            # as bf16 (workers compute under bf16 autocast anyway; the fp32 master stays on the PS).
            # ps_sync keeps the reference's full-precision broadcast (README.md:76), so its replicas
            # stay bitwise identical to the PS's parameters
            multi = self.world.size > 1 and self.store.device.type == "cuda"
            self.cfg.param_wire = "bf16" if multi and mode == "ps_async" else "fp32"
        if mode == "local":
            if self.world.size > 1:
                raise ValueError("mode='local' with world size > 1")
            return LocalEngine(self, self.cfg, self.store, self.codec, self.world)
        if mode == "allgather":
            return AllGatherEngine(self, self.cfg, self.store, self.codec, self.world)
        if mode == "ps_sync":
            return PSSyncEngine(self, self.cfg, self.store, self.codec, self.world)
        if mode == "ps_async":
            from .parallel.ps_async import PSAsyncEngine

            return PSAsyncEngine(self, self.cfg, self.store, self.codec, self.world)
        raise ValueError(mode)

    # ------------------------------------------------------------------ state
    def _init_state(self):
        """Flat optimizer state; per-param torch-compatible views in self.state."""
        self.flat_state: Dict[str, torch.Tensor] = {}
        self._group_steps = [0] * len(self.param_groups)
        # per-16-element-chunk update counts (int32; a chunk never straddles two parameters): the
        # reference's per-parameter optimizer state -- momentum buffer created on a parameter's
        # first gradient (ps.py:202-205), Adam state['step'] advanced only when the parameter has
        # a gradient (ps.py:178-179, 241).  The fused kernels read and advance them under the
        # chunk mask, so a parameter that starts late gets its own first step.
        self.chunk_steps: Optional[torch.Tensor] = None

    def _csteps(self) -> Optional[torch.Tensor]:
        if self.chunk_steps is None and self._needs_csteps():
            self.chunk_steps = torch.zeros(self.store.nchunks, dtype=torch.int32, device=self.store.device)
        return self.chunk_steps

    def _needs_csteps(self) -> bool:
        return True

    def state_floats(self) -> int:
        """fp32 optimizer-state words per parameter (PS memory budget)."""
        return 0

    def _ensure_state(self, key: str) -> torch.Tensor:
        if key not in self.flat_state:
            buf = self.store.new_buffer()
            self.flat_state[key] = buf
            for i, s in enumerate(self.store.slots):
                self.state[s.param][key] = self.store.param_view(buf, i)
        return self.flat_state[key]

    def _update_flat(self, sources: List[torch.Tensor], target: torch.Tensor, gscale: float, zero_src: bool = False,
                     pub: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None, lookahead: float = 0.0):
        """Apply the optimizer to flat ``target`` from flat gradient ``sources`` (summed).
        ``mask`` (uint8 per 16-element chunk, FlatStore.chunk_mask) skips the parameters that
        produced no gradient this step, like ``if p.grad is None: continue`` (ps.py:178-179).
        ``lookahead`` tau > 0 (async PS): ``pub`` receives the parameters extrapolated by the
        momentum of the next tau updates (optimizers without momentum ignore it)."""
        self._begin_update()
        self._update_range(sources, target, 0, self.store.numel, gscale, zero_src, pub, mask, lookahead=lookahead)

    def _begin_update(self):
        """Start one optimizer step: advance every non-empty group's step counter once (the
        update itself may then run as several flat ranges, e.g. one per bucket as its gradient
        exchange lands)."""
        for gi in range(len(self.param_groups)):
            a, b = self.store.group_ranges[gi]
            if b > a:
                self._group_steps[gi] += 1

    def _update_range(self, sources: List[torch.Tensor], target: torch.Tensor, lo: int, hi: int, gscale: float,
                      zero_src: bool = False, pub: Optional[torch.Tensor] = None,
                      mask: Optional[torch.Tensor] = None, src_lo: int = 0, lookahead: float = 0.0,
                      pub_lo: int = 0):
        """Update flat elements [lo, hi) (16-aligned).  ``target``/``mask`` index the whole flat
        space; ``sources`` start at flat element ``src_lo`` (e.g. one bucket's images), ``pub`` at
        ``pub_lo`` (one chunk of a publish buffer split over several IPC allocations)."""
        for gi, group in enumerate(self.param_groups):
            a, b = self.store.group_ranges[gi]
            a, b = max(a, lo), min(b, hi)
            if b <= a:
                continue
            cs = self._csteps()
            self._update_group(gi, group, [s[a - src_lo:b - src_lo] for s in sources], target[a:b], gscale,
                               zero_src, None if pub is None else pub[a - pub_lo:b - pub_lo],
                               None if mask is None else mask[a // 16:b // 16], a, b,
                               None if cs is None else cs[a // 16:b // 16], lookahead)

    def _update_group(self, gi, group, srcs, target, gscale, zero_src, pub, mask=None, lo=None, hi=None,
                      csteps=None, lookahead=0.0):
        raise NotImplementedError

    def param_steps(self) -> Dict[int, int]:
        """slot index -> number of updates that parameter has received (host read)."""
        if self.chunk_steps is None:
            return {i: self._group_steps[s.group] for i, s in enumerate(self.store.slots)}
        cs = self.chunk_steps.cpu()
        return {i: int(cs[s.offset // 16]) for i, s in enumerate(self.store.slots)}

    # ------------------------------------------------------------------ public API
    @torch.no_grad()
    def step(self, closure=None):
        """One exchange + update.  Returns ``(loss, data)`` like the reference (ps.py:193)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.steps += 1
        t0 = time.perf_counter()
        if self.store.device.type == "cuda":
            from .ops import nn as hnn

            # gradients computed on the weight-gradient side stream: every backward already ends by
            # joining it into the caller's stream (an autograd final callback, ops.nn._join_wgrad),
            # so only a side-stream use outside a backward pass needs the join here (one event
            # record less on the host at every step boundary)
            if (hnn.wgrad_stream(self.store.device) is not None and hnn.wgrad_join_pending(self.store.device)
                    and not hnn.wgrad_join_deferred(self.store.device)):
                hnn.join_wgrad_stream(self.store.device)
        data = self.engine.step()
        self._refresh_shadow()
        now = time.perf_counter()
        data["step_time"] = now - t0
        if self.cfg.samples_per_step > 0:  # host wall time between consecutive step() calls
            last = getattr(self, "_last_step_t", None)
            if last is not None and now > last:
                data["samples_per_sec"] = self.cfg.samples_per_step / (now - last)
            self._last_step_t = now
        if self._metrics is not None:
            self._metrics.write(self.steps, data)
        return loss, data

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics: ``p.grad = None`` by default; a parameter whose gradient is still None
        at step() is skipped (ps.py:178-179).  ``set_to_none=False`` zero-fills the flat gradient
        views instead (every parameter then counts as having a gradient)."""
        if getattr(self, "engine", None) is not None and hasattr(self.engine, "before_zero_grad"):
            self.engine.before_zero_grad()
        self.store.zero_grad(set_to_none)

    def no_sync(self):
        """Gradient accumulation over several backward() calls (like DDP's ``no_sync``): inside
        the context the hooks only record which parameters got a gradient; the encode and the
        exchange run for the summed gradients at the next backward() outside it / at step()."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            eng = self.engine
            prev = eng.accumulating
            eng.accumulating = True
            try:
                yield
            finally:
                eng.accumulating = prev

        return ctx()

    @property
    def ps_only(self) -> bool:
        """True on rank 0 of a dedicated async parameter server (``ps_dedicated=True``)."""
        return bool(getattr(self.engine, "ps_only", False))

    def serve(self, timeout_s: Optional[float] = None) -> dict:
        """Dedicated PS rank: receive, sum, step and publish until the workers stop; returns the
        PS statistics (the reference's ``if rank == 0`` loop, README.md:64-73)."""
        stats = self.engine.serve(timeout_s)
        self._last_engine_stats = stats
        self.close()
        return stats

    def irequest_params(self, **kw):
        """AsySG-InCon parameter refresh (README.md:63): adopt the newest published params that
        have arrived, without waiting for the rest (inconsistent read).  No-op in sync modes."""
        r = self.engine.irequest_params(**kw)
        self._refresh_shadow()
        return r

    def _refresh_shadow(self):
        eng = self.engine
        if hasattr(eng, "take_shadow_done"):
            if eng.take_shadow_done():  # a split pull refreshed each half on its own stream
                return
            eng.join_pull()
        self.store.refresh_shadow()

    def overlap_pull(self, module: torch.nn.Module) -> bool:
        """ps_async with the GPU-time pull: copy the parameters of ``module`` and of everything
        after it in parameter order on a side stream, overlapped with the forward of the earlier
        layers; ``module``'s forward waits for them.  Use it only when no parameter from ``module``
        on is read before ``module`` runs (ResNet: ``model.layer4``).  Code that reads parameters
        outside the model's forward (evaluation copies, logging) calls ``join_pull()`` first;
        checkpoints and the next pull do.  Returns False (no-op) in other modes or when the module
        has no managed parameters."""
        eng = self.engine
        if not hasattr(eng, "set_pull_overlap"):
            return False
        offs = [s.offset for s in self.store.slots if any(s.param is p for p in module.parameters())]
        if not offs:
            return False
        return eng.set_pull_overlap(min(offs), module)

    def join_pull(self):
        """Order the current stream after any parameter copy still in flight (split pull)."""
        if hasattr(self.engine, "join_pull"):
            self.engine.join_pull()

    def join_grads(self):
        """Order the current stream after every gradient still being computed on the
        weight-gradient side stream (needed before reading ``param.grad`` between ``backward()``
        and ``step()`` when ``defer_wgrad_join`` is on; a no-op otherwise)."""
        if self.store.device.type == "cuda":
            from .ops import nn as hnn

            hnn.join_wgrad_stream(self.store.device)

    def refresh_bf16_weights(self):
        """Re-cast the bf16 weight shadow after editing parameters outside ``step()``."""
        if hasattr(self.engine, "join_pull"):
            self.engine.join_pull()
        self.store.refresh_shadow()

    def watch_module(self, module: torch.nn.Module):
        """Refresh the bf16 weight shadow whenever ``module.load_state_dict`` writes parameters
        this optimizer manages (a post-hook: the shadow-reading conv / Linear kernels would
        otherwise keep reading the pre-load weights until the next step).  ``load_state_dict`` of
        the optimizer itself and ``hipps.utils.checkpoint.load`` refresh it already."""
        return module.register_load_state_dict_post_hook(lambda _m, _keys: self.refresh_bf16_weights())

    def close(self):
        if getattr(self, "engine", None) is not None:
            self.engine.close()
            if hasattr(self.engine, "ps_stats"):
                self._last_engine_stats = self.engine.ps_stats()  # drained totals after close
            self.engine = None
        if getattr(self, "store", None) is not None:
            self.store.disable_bf16_shadow()
        if self._metrics is not None:
            self._metrics.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def state_dict(self):
        """torch-compatible state dict.  In ps_async mode the PS thread advances the optimizer
        state on its own stream, so the snapshot is taken with that thread held between messages
        (engine.quiesced(), as checkpoint.save does) and the tensors are copied out before it
        resumes: per-parameter 'step' counts, moments and chunk counts belong to one PS state."""
        import contextlib

        eng = getattr(self, "engine", None)
        q = getattr(eng, "quiesced", None) if eng is not None else None
        with (q() if q is not None else contextlib.nullcontext()):
            self._sync_param_state()
            sd = super().state_dict()
            if q is not None:  # detach from the live flat buffers the PS keeps updating
                sd["state"] = {k: {n: (v.detach().clone() if torch.is_tensor(v) else v) for n, v in st.items()}
                               for k, st in sd["state"].items()}
            sd["hipps"] = {"steps": self.steps, "group_steps": list(self._group_steps), "mode": self.mode,
                           "codec": self.codec.name}
            if self.chunk_steps is not None:
                sd["hipps"]["chunk_steps"] = self.chunk_steps.detach().cpu()
        return sd

    def _watch_hyper(self):
        """Make every param group notify the engine when a hyper-parameter is written (an LR
        scheduler's ``group['lr'] = ...``): the native PS loop (ps_async, C++ without the GIL)
        cannot read ``param_groups`` at each update the way the Python loop does, so the new value
        is pushed into it at once -- both loops then use the same lr from the same moment on
        (ADVICE r5)."""
        if getattr(self.engine, "_push_hyper", None) is None:
            return

        def push():
            eng = getattr(self, "engine", None)
            if eng is not None and hasattr(eng, "_push_hyper"):
                eng._push_hyper()

        for i, g in enumerate(self.param_groups):
            if not isinstance(g, _HyperGroup):
                self.param_groups[i] = _HyperGroup(g, push)

    def _sync_param_state(self):
        """Refresh host-side per-parameter state entries derived from device state."""

    def load_state_dict(self, state_dict):
        extra = state_dict.get("hipps", {})
        sd = {k: v for k, v in state_dict.items() if k != "hipps"}
        # torch's loader replaces per-param tensors; copy them back into our flat buffers
        super().load_state_dict(sd)
        keys = {k for st in self.state.values() for k, v in st.items() if torch.is_tensor(v) and v.dim() > 0}
        for key in sorted(keys):
            buf = self._ensure_state_nocopy(key)
            for i, s in enumerate(self.store.slots):
                t = self.state[s.param].get(key)
                v = self.store.param_view(buf, i)
                if t is not None and t.data_ptr() != v.data_ptr():
                    v.copy_(t)
                self.state[s.param][key] = v
        self.steps = extra.get("steps", self.steps)
        if "group_steps" in extra:
            self._group_steps = list(extra["group_steps"])
        cs = self._csteps()
        if cs is not None:
            if "chunk_steps" in extra:
                cs.copy_(extra["chunk_steps"].to(cs.device))
            else:  # a plain torch state dict: per-parameter counts from its own entries
                self._csteps_from_state(cs)
        # torch rebuilt param_groups as plain dicts: watch them again, and hand the loaded
        # hyper-parameters and group step counts to a native PS loop
        self._watch_hyper()
        eng = getattr(self, "engine", None)
        if eng is not None and hasattr(eng, "reload_hyper"):
            eng.reload_hyper()
        self.store.refresh_shadow()

    def _csteps_from_state(self, cs: torch.Tensor):
        for s in self.store.slots:
            n = self._state_count(self.state.get(s.param, {}), s.group)
            a = s.offset // 16
            cs[a:a + (s.numel + 15) // 16].fill_(n)

    def _state_count(self, st: dict, gi: int) -> int:
        return self._group_steps[gi]

    def csteps_from_groups(self, cs: torch.Tensor, started=None):
        """Per-chunk counts for a checkpoint written before chunk_steps existed (it stored only
        per-group step counts, and for SGD the groups whose momentum had started,
        ``mom_started``): every parameter of a group took that group's steps."""
        for s in self.store.slots:
            a = s.offset // 16
            cs[a:a + (s.numel + 15) // 16].fill_(self._group_count(s.group, started))

    def _group_count(self, gi: int, started=None) -> int:
        return self._group_steps[gi]

    def _ensure_state_nocopy(self, key):
        if key not in self.flat_state:
            self.flat_state[key] = self.store.new_buffer()
        return self.flat_state[key]


class SGD(MPI_PS, torch.optim.SGD):
    """Reference SGD (ps.py:195-214): wd, momentum (buf = d_p on first step), dampening,
    nesterov, p -= lr*d_p.  Fused into one kernel per param group."""

    optim = "sgd"

    def _needs_csteps(self) -> bool:
        return any(g.get("momentum", 0) for g in self.param_groups)

    def state_floats(self) -> int:
        return 1 if any(g.get("momentum", 0) for g in self.param_groups) else 0

    def _update_group(self, gi, group, srcs, target, gscale, zero_src, pub, mask=None, lo=None, hi=None,
                      csteps=None, lookahead=0.0):
        mom = group.get("momentum", 0) or 0
        a, b = (lo, hi) if lo is not None else self.store.group_ranges[gi]
        buf = self._ensure_state("momentum_buffer")[a:b] if mom else None
        # buf = d_p on each parameter's own first step (ps.py:203-205): the kernel reads the
        # chunk's update count, so masked steps and late-starting parameters follow the reference
        ops.sgd_step(srcs, target, buf, pub, zero_src, gscale, lr=group["lr"],
                     weight_decay=group.get("weight_decay", 0) or 0, momentum=mom,
                     dampening=group.get("dampening", 0) or 0, nesterov=bool(group.get("nesterov", False)),
                     first=False, mask=mask, csteps=csteps if mom else None,
                     lookahead=self.lookahead_coef(group, lookahead) if pub is not None else 0.0)

    @staticmethod
    def lookahead_coef(group, tau: float) -> float:
        """lr * (mu + mu^2 + ... + mu^tau): the momentum displacement of the next tau updates
        (fractional tau interpolates the geometric sum)."""
        mom = group.get("momentum", 0) or 0
        if tau <= 0 or not mom or group.get("nesterov", False):
            return 0.0
        geo = mom * (1 - mom ** tau) / (1 - mom) if mom < 1 else tau
        return float(group["lr"]) * geo

    def _state_count(self, st: dict, gi: int) -> int:
        return max(1, self._group_steps[gi]) if "momentum_buffer" in st else 0

    def _group_count(self, gi: int, started=None) -> int:
        if started is not None:
            has = gi in set(started)
        else:
            has = "momentum_buffer" in self.flat_state and self._group_steps[gi] > 0
        return max(1, self._group_steps[gi]) if has else 0


class Adam(MPI_PS, torch.optim.Adam):
    """Reference Adam (ps.py:217-261): eps added to the un-corrected sqrt(v) unless
    ``adam_variant='torch'``; amsgrad honoured (the reference never passes it, ps.py:185-186)."""

    optim = "adam"

    def state_floats(self) -> int:
        return 3 if any(g.get("amsgrad", False) for g in self.param_groups) else 2

    def _sync_param_state(self):
        for i, n in self.param_steps().items():  # torch-compatible per-parameter step (ps.py:241)
            self.state[self.store.slots[i].param]["step"] = n

    def _state_count(self, st: dict, gi: int) -> int:
        return int(st.get("step", 0))

    def _update_group(self, gi, group, srcs, target, gscale, zero_src, pub, mask=None, lo=None, hi=None,
                      csteps=None, lookahead=0.0):
        a, b = (lo, hi) if lo is not None else self.store.group_ranges[gi]
        m = self._ensure_state("exp_avg")[a:b]
        v = self._ensure_state("exp_avg_sq")[a:b]
        ams = bool(group.get("amsgrad", False))
        vm = self._ensure_state("max_exp_avg_sq")[a:b] if ams else None
        step = self._group_steps[gi]
        ops.adam_step(srcs, target, m, v, vm, pub, zero_src, gscale, lr=group["lr"], betas=group["betas"],
                      eps=group["eps"], weight_decay=group.get("weight_decay", 0) or 0, step=step, amsgrad=ams,
                      torch_mode=self.cfg.adam_variant == "torch", mask=mask, csteps=csteps)
