"""FusedAdam — torch.optim.Adam's update for every parameter tensor in one HIP launch.

The reference optimises each model with ``torch.optim.Adam(model.parameters(), lr=...,
weight_decay=...)`` (train/loop_utils.py:45-61) and steps it after every accepted batch
(train/multimodal.py:141-143).  ``FusedAdam`` is a drop-in ``torch.optim.Optimizer``: same
constructor arguments (amsgrad / maximize / capturable are not on the path and are rejected),
same ``param_groups`` (so ``StepLR`` drives ``lr``), and the same per-parameter state keys
``step`` / ``exp_avg`` / ``exp_avg_sq`` — its ``state_dict()`` loads into torch.optim.Adam and
back.  The step is one ``mauv_adam_step`` launch per parameter group over a device table of
(param, grad, exp_avg, exp_avg_sq, numel) rows; the table is rebuilt only when a pointer
changes.  Parameters whose ``.grad`` is None are skipped, like torch.

``step_gated(gate)`` is the training loop's form (mauv.train.mc_train_step): the decision of
multimodal.py:133-145 — skip on a non-finite loss, skip the step and the zero_grad on
non-finite gradients — is read from a device ``MauvStepGate`` by the kernel, and the Adam
step count lives in that gate, so a training step never waits on the host.
"""
import numpy as np
import torch

from . import ops  # noqa: F401  (loads the library)
from ._lib import lib, check

GATE_WORDS = 16          # sizeof(MauvStepGate) / 4 (include/mauv.h)
G_OK_LOSS, G_NONFINITE, G_POISONED, G_MODE, G_STEP, G_STEPPED, G_SKIP_LOSS, G_SKIP_GRAD = range(8)
G_SCRATCH = 15           # a reserved word the training step counts non-finite inputs in


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, maximize=False, **unsupported):
        if amsgrad or maximize:
            raise ValueError("FusedAdam: amsgrad / maximize are not supported")
        for k, v in unsupported.items():
            if v not in (None, False):
                raise ValueError(f"FusedAdam: unsupported option {k}={v}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=False))
        self._tables = {}
        # per group: the tensors of the last step when every live parameter shared one step
        # count — the next step with the same tensors skips the per-parameter Python work
        # (checks, one .item() per step counter, table key).  The entry holds strong references
        # to the moment tensors the device table points at, and is used only while the state
        # still holds exactly those tensors (a cleared / replaced state drops to the slow path
        # instead of writing through stale pointers).
        self._fast = {}
        self._gate = None          # device MauvStepGate (int32[16]) of the gated form
        self._gate_dirty = False   # the gate's step count is ahead of state["step"]
        self._gate_params = None

    def _table(self, gi, live):
        key = tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                     self.state[p]["exp_avg_sq"].data_ptr()) for p in live)
        cached = self._tables.get(gi)
        if cached is not None and cached[0] == key:
            return cached[1]
        rows = np.zeros((len(live), 5), dtype=np.int64)
        for i, p in enumerate(live):
            st = self.state[p]
            rows[i] = (p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                       st["exp_avg_sq"].data_ptr(), p.numel())
        tab = torch.from_numpy(rows).to(live[0].device)
        self._tables[gi] = (key, tab)
        return tab

    def _fast_entry(self, gi, live):
        """The cached (t, table, step buffer) of group ``gi`` if it is still valid for ``live``."""
        fast = self._fast.get(gi)
        if fast is None:
            return None
        ptrs, gptrs, moments, state_id, t, tab, steps = fast
        if state_id != id(self.state) or len(ptrs) != len(live):
            return None
        if [p.data_ptr() for p in live] != ptrs or [p.grad.data_ptr() for p in live] != gptrs:
            return None
        try:
            for p, (m, v) in zip(live, moments):
                st = self.state[p]
                if st["exp_avg"] is not m or st["exp_avg_sq"] is not v:
                    return None
        except KeyError:
            return None
        return fast

    def _prepare(self, gi, group, live):
        """Slow path: create / bump the per-parameter state, launch per shared step count."""
        self._fast.pop(gi, None)
        for p in live:
            if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous() \
                    or p.grad.is_sparse:
                raise TypeError("FusedAdam: dense contiguous fp32 ROCm parameters only")
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)

    def _remember(self, gi, live, t, tab):
        # re-home the step counters as 0-dim views of one CPU tensor (still float tensors,
        # torch.optim.Adam-compatible): the fast path bumps them in one op
        buf = torch.full((len(live),), float(t))
        for i, p in enumerate(live):
            self.state[p]["step"] = buf[i]
        moments = [(self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"]) for p in live]
        self._fast[gi] = ([p.data_ptr() for p in live], [p.grad.data_ptr() for p in live],
                          moments, id(self.state), t, tab, buf)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._sync_gate()
        self._gate = None   # an ungated step moves the count on the host: re-read it next time
        for gi, group in enumerate(self.param_groups):
            live = [p for p in group["params"] if p.grad is not None]
            if not live:
                continue
            b1, b2 = group["betas"]
            fast = self._fast_entry(gi, live)
            if fast is not None:
                ptrs, gptrs, moments, sid, t, tab, steps = fast
                t += 1
                steps.add_(1.0)   # every live parameter's state["step"] is a view of it
                check(lib.mauv_adam_step(tab.data_ptr(), len(live), group["lr"], b1, b2,
                                         group["eps"], group["weight_decay"], t,
                                         ops.stream()), "adam_step")
                self._fast[gi] = (ptrs, gptrs, moments, sid, t, tab, steps)
                continue
            self._prepare(gi, group, live)
            for p in live:
                self.state[p]["step"] += 1
            # one bias-correction step per group (params of a group step together; a param that
            # missed steps because its grad was None keeps its own count like torch — split it)
            steps = {}
            for p in live:
                steps.setdefault(int(self.state[p]["step"].item()), []).append(p)
            for t, ps in steps.items():
                tab = self._table((gi, t) if len(steps) > 1 else gi, ps)
                check(lib.mauv_adam_step(tab.data_ptr(), len(ps), group["lr"], b1, b2,
                                         group["eps"], group["weight_decay"], t,
                                         ops.stream()), "adam_step")
                if len(steps) == 1:
                    self._remember(gi, ps, t, tab)
        return loss

    # ---- the device-gated form ---------------------------------------------------------------
    def gate(self, params, device):
        """The device MauvStepGate for a training loop over ``params`` (the model's parameters),
        or None when the gated form does not apply: one parameter group holding exactly those
        tensors, all sharing one step count."""
        if self._gate is not None and self._gate_params is params and \
                self._gate.device == torch.device(device):
            return self._gate
        if len(self.param_groups) != 1:
            return None
        gp = self.param_groups[0]["params"]
        if len(gp) != len(params) or {id(p) for p in gp} != {id(p) for p in params}:
            return None
        if self._gate is None or self._gate.device != torch.device(device):
            counts = {int(self.state[p]["step"].item()) if "step" in self.state[p] else 0
                      for p in gp}
            if len(counts) != 1:
                return None
            # the gate takes a skipped batch's gradients back out by zeroing a clean arena, so it
            # starts from what the arena holds: non-finite values (an ungated step skipped on
            # them: "poisoned", kept as the reference keeps them) or nothing.  Finite leftovers
            # (a backward outside the loop) would be lost by that zeroing: such a step takes the
            # host-decided path, whose skip runs no backward (multimodal.py:133-135)
            grads = [p.grad for p in gp if p.grad is not None]
            poisoned = 0
            if grads:
                top = torch.stack(torch._foreach_norm(grads, float("inf")))
                if not bool(torch.isfinite(top).all()):
                    poisoned = 1
                elif bool((top != 0).any()):
                    return None
            g = torch.zeros(GATE_WORDS, dtype=torch.int32)
            g[G_STEP] = counts.pop()
            g[G_POISONED] = poisoned
            self._gate = g.to(device)
            self._gate_dirty = False
        self._gate_params = params
        return self._gate

    @torch.no_grad()
    def step_gated(self, gate):
        """One step whose execution (step + zero_grad, restore, or nothing) the kernel reads
        from ``gate`` — no host synchronisation.  Every parameter of the group must hold a
        gradient (the model's arena views)."""
        assert gate is self._gate, "step_gated: use the gate returned by FusedAdam.gate()"
        group = self.param_groups[0]
        live = group["params"]
        if any(p.grad is None for p in live):
            raise RuntimeError("step_gated: every parameter needs a gradient tensor")
        b1, b2 = group["betas"]
        fast = self._fast_entry(0, live)
        if fast is None:
            self._prepare(0, group, live)
            tab = self._table(0, live)
            t = int(self._gate_step_host())
            self._remember(0, live, t, tab)
            fast = self._fast[0]
        tab = fast[5]
        from torch.optim import optimizer as _topt
        for hook in list(_topt._global_optimizer_pre_hooks.values()) + \
                list(self._optimizer_step_pre_hooks.values()):
            hook(self, (self,), {})
        check(lib.mauv_adam_step_gated(tab.data_ptr(), len(live), group["lr"], b1, b2,
                                       group["eps"], group["weight_decay"], gate.data_ptr(),
                                       ops.stream()), "adam_step_gated")
        self._gate_dirty = True
        # what torch.optim.Optimizer.step's wrapper records: an LR scheduler stepped after this
        # does not warn "lr_scheduler.step() before optimizer.step()"; step hooks still run
        self._opt_called = True
        for hook in list(self._optimizer_step_post_hooks.values()) + \
                list(_topt._global_optimizer_post_hooks.values()):
            hook(self, (self,), {})

    def _gate_step_host(self):
        """Step count held by the gate (one device read; only on a cache rebuild)."""
        return int(self._gate[G_STEP].item()) if self._gate is not None else 0

    def _sync_gate(self):
        """After gated steps, bring state["step"] up to the device count (before an ungated
        step or a state_dict)."""
        if self._gate is None or not self._gate_dirty:
            return
        t = self._gate_step_host()
        for p in self.param_groups[0]["params"]:
            if "step" in self.state[p]:
                self.state[p]["step"].fill_(float(t))
        fast = self._fast.get(0)
        if fast is not None:
            self._fast[0] = fast[:4] + (t,) + fast[5:]
        self._gate_dirty = False

    def state_dict(self):
        self._sync_gate()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """torch's load (new state tensors, step counts): the cached tables are dropped."""
        super().load_state_dict(state_dict)
        self._tables.clear()
        self._fast.clear()
        self._gate = None
        self._gate_dirty = False
