"""FusedAdam — ``torch.optim.Adam`` semantics over a parameter arena, one HIP launch per step.

The reference builds ``partial(Adam, lr=lr, betas=betas)`` (experiments/basic_conf.py:55,67;
gradient_penalty_conf.py:9-10) and calls ``optimizer.step()`` once per update
(Trainer.py:135,157).  Here every parameter, gradient and moment of a module lives in one flat
``Arena`` (cgan3d_amd.engine), so the whole update is a single elementwise kernel
(``cgan3d_adam``).  It is a real ``torch.optim.Optimizer``: ``param_groups`` drive the learning
rate (so ``MultiStepLR`` works unchanged) and ``state_dict`` carries torch-Adam-shaped state
(``step``, ``exp_avg``, ``exp_avg_sq`` per parameter) for checkpoint interchange.
"""
from __future__ import annotations

from functools import partial

import torch

from .. import ops
from ..engine import Arena


def adam_hyper_from_partial(optim_class) -> dict:
    """lr / betas / eps of a ``partial(torch.optim.Adam, ...)`` config entry."""
    func = optim_class.func if isinstance(optim_class, partial) else optim_class
    if func is not torch.optim.Adam:
        raise NotImplementedError(f"the HIP step implements Adam only (got {getattr(func, '__name__', func)})")
    kw = dict(optim_class.keywords) if isinstance(optim_class, partial) else {}
    for bad in ("weight_decay", "amsgrad", "maximize"):
        if kw.get(bad):
            raise NotImplementedError(f"Adam({bad}=...) is not used by the reference configs")
    betas = kw.get("betas", (0.9, 0.999))
    return {"lr": float(kw.get("lr", 1e-3)), "betas": (float(betas[0]), float(betas[1])),
            "eps": float(kw.get("eps", 1e-8))}


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, arena: Arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_clip=None):
        super().__init__(arena.params, dict(lr=lr, betas=betas, eps=eps))
        self.arena = arena
        dev = arena.flat.device
        # device-resident [lr, beta1, beta2, eps, step, clip] so a captured step replays correctly
        self.hyper = torch.tensor([lr, betas[0], betas[1], eps, 0.0, weight_clip or 0.0], device=dev,
                                  dtype=torch.float32)
        self.ticket = ops.tickets(1, dev)[0]  # launch ticket of the fused update + repack
        self._host_step = 0
        self._host_lr = lr
        for p, name in zip(arena.params, arena.names):
            off = self._offset(p)
            n = p.numel()
            self.state[p] = {"exp_avg": arena.exp_avg[off:off + n].view_as(p),
                             "exp_avg_sq": arena.exp_avg_sq[off:off + n].view_as(p)}

    def _offset(self, p):
        return (p.data_ptr() - self.arena.flat.data_ptr()) // 4

    def sync_hyper(self):
        """Push a changed learning rate (LR scheduler) to the device scalar."""
        lr = float(self.param_groups[0]["lr"])
        if lr != self._host_lr:
            self.hyper[0].fill_(lr)
            self._host_lr = lr

    def launch(self, packs=None):
        """Enqueue one update (step counter advanced on the device); no host sync.  One launch
        (cgan3d_adam_pack: the step tick rides on the Adam kernel, its last block out advances it).
        With ``packs`` (an ops.PackSet over this arena's weights) the packed copies are refreshed in
        the same launch — each updated parameter written straight into its packed positions; those
        are scattered 2-byte stores, measured slower than a separate coalesced repack launch for the
        generator (37 us against 11 + 11), so the engine repacks separately."""
        a = self.arena
        ops.adam_pack(a.flat, a.grad, a.exp_avg, a.exp_avg_sq, self.hyper, self.ticket, packs)
        self._opt_called = True  # what torch's LR schedulers check optimizer.step() for
        if not ops.recording():  # a recorded plan counts its steps when it runs (note_step)
            self._host_step += 1

    def note_step(self):
        """Count one update issued by a replayed launch plan (the device counter ticks itself)."""
        self._opt_called = True
        self._host_step += 1

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.sync_hyper()
        self.launch()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        self.arena.grad.zero_()
        self.arena.rebind_grads()

    def state_dict(self):
        step = float(self.hyper[4].item())  # device counter (correct under graph replay too)
        for p in self.arena.params:
            self.state[p]["step"] = torch.tensor(step)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        views = {p: (self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"]) for p in self.arena.params}
        super().load_state_dict(state_dict)
        step = 0
        for p in self.arena.params:
            st = self.state[p]
            m, v = views[p]
            m.copy_(st["exp_avg"])
            v.copy_(st["exp_avg_sq"])
            st["exp_avg"], st["exp_avg_sq"] = m, v
            step = int(st.get("step", torch.tensor(0.0)).item())
        self._host_step = step
        self.hyper[4].fill_(float(step))
        self._host_lr = None
        self.sync_hyper()
