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
"""
import numpy as np
import torch

from . import ops  # noqa: F401  (loads the library)
from ._lib import lib, check


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
        # per group: (param ptrs, grad ptrs, step t, table, step buffer) of the last step when
        # every live parameter shared one step count — the next step with the same tensors skips
        # the per-parameter Python work (checks, one .item() per step counter, table key): on a
        # 696-tensor model that work was ~2.4 ms of host time with the GPU idle before the launch
        self._fast = {}

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

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            live = [p for p in group["params"] if p.grad is not None]
            if not live:
                continue
            b1, b2 = group["betas"]
            ptrs = [p.data_ptr() for p in live]
            gptrs = [p.grad.data_ptr() for p in live]
            fast = self._fast.get(gi)
            if fast is not None and fast[0] == ptrs and fast[1] == gptrs:
                _, _, t, tab, steps = fast
                t += 1
                steps.add_(1.0)   # every live parameter's state["step"] is a view of it
                check(lib.mauv_adam_step(tab.data_ptr(), len(live), group["lr"], b1, b2,
                                         group["eps"], group["weight_decay"], t,
                                         ops.stream()), "adam_step")
                self._fast[gi] = (ptrs, gptrs, t, tab, steps)
                continue
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
                st["step"] += 1
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
                    # re-home the step counters as 0-dim views of one CPU tensor (still float
                    # tensors, torch.optim.Adam-compatible): the fast path bumps them in one op
                    buf = torch.full((len(ps),), float(t))
                    for i, p in enumerate(ps):
                        self.state[p]["step"] = buf[i]
                    self._fast[gi] = (ptrs, gptrs, t, tab, buf)
        return loss

    def load_state_dict(self, state_dict):
        """torch's load (new state tensors, step counts): the cached tables are dropped."""
        super().load_state_dict(state_dict)
        self._tables.clear()
        self._fast.clear()
