"""Trainer — drop-in for ``contrast_gan_3D/trainer/Trainer.py:34-363`` on the HIP step engine.

Same constructor (positional order of ``train.py:154-176``), same methods and ``log_dict`` keys
(``"D"``, ``"G"``, ``"G-full"``, ``"sim"``, ``"HU"``), same checkpoint layout.  ``train_step``
runs ``cgan3d_amd.engine.StepEngine``: the generator forward once, the critic update with the
gradient penalty and the generator update as explicit HIP launches over resident buffers, Adam
fused over a parameter arena.  Loss values stay on the device and are read only on logging
iterations (as in the reference, ``Trainer.py:187-190``).

Differences from the reference, all deliberate and documented in DESIGN.md:
* the critic weights are checkpointed under ``"critic"`` (the reference lists the non-existent
  attribute ``"discriminator"``, Trainer.py:316, so its critic is never saved); the
  ``"discriminator": None`` entry is kept so either kind of checkpoint loads;
* ``train_critic`` / ``train_generator`` act on the engine's resident batch (``train_step``
  loads it); they keep the reference signatures for callers that drive them directly.
"""
from __future__ import annotations

import os
from functools import partial
from pathlib import Path
from typing import Dict, List, Optional, Union

import numpy as np
import torch
from torch import Tensor, nn

from .. import _lib as L
from .. import ops
from ..engine import Arena, StepEngine, _planar_dims
from ..model.loss import WassersteinLoss, ZNCCLoss
from .optim import FusedAdam, adam_hyper_from_partial

try:  # tqdm is what the reference uses for progress; optional here
    from tqdm.auto import trange
except Exception:  # pragma: no cover
    trange = range

import logging

logger = logging.getLogger(__name__)

ScanTypes = (0, -1, 1)  # ScanType.OPT, LOW, HIGH (contrast_gan_3D/alias.py:24-27)


class Trainer:
    def __init__(self, train_iterations: int, val_iterations: int, validate_every: int, train_generator_every: int,
                 train_critic_every: int, log_every: int, log_images_every: int, generator_class: partial,
                 critic_class: partial, generator_optim_class: partial, critic_optim_class: partial,
                 hu_loss_instance: nn.Module, logger_interface, device: torch.device, debug: bool = False,
                 checkpoint_dir: Optional[Union[str, Path]] = None, weight_clip: Optional[float] = None,
                 generator_lr_scheduler_class: Optional[partial] = None,
                 critic_lr_scheduler_class: Optional[partial] = None, hu_loss_weight: float = 1.0,
                 sim_loss_weight: float = 1.0, gan_loss_weight: float = 1.0, gp_weight: float = 10,
                 checkpoint_every: Optional[int] = 1000, rng: Optional[np.random.Generator] = None,
                 precision: str = "f32"):
        self.rng = rng
        self.precision = precision  # "f32" (the reference's arithmetic) or "bf16" MFMA convolutions
        self.device = torch.device(device)
        self.debug = debug
        self.train_log_sample_size, self.val_log_sample_size = None, None
        self.train_iterations, self.val_iterations = train_iterations, val_iterations
        self.val_every = validate_every
        self.train_generator_every, self.train_critic_every = train_generator_every, train_critic_every
        self.log_every, self.log_images_every = log_every, log_images_every
        self.hu_loss_w, self.sim_loss_w, self.gan_loss_w = hu_loss_weight, sim_loss_weight, gan_loss_weight
        self.gp_w, self.weight_clip = gp_weight, weight_clip

        self.generator: nn.Module = generator_class().to(self.device)
        g_h = adam_hyper_from_partial(generator_optim_class)
        self.optimizer_G = FusedAdam(Arena(self.generator, self.device), **g_h)
        self.lr_scheduler_G = generator_lr_scheduler_class(self.optimizer_G) if generator_lr_scheduler_class else None

        self.critic: nn.Module = critic_class().to(self.device)
        d_h = adam_hyper_from_partial(critic_optim_class)
        # weight clipping (Trainer.py:136-138) is applied by the critic's Adam kernel after the update
        self.optimizer_D = FusedAdam(Arena(self.critic, self.device), **d_h, weight_clip=weight_clip)
        self.lr_scheduler_D = critic_lr_scheduler_class(self.optimizer_D) if critic_lr_scheduler_class else None

        self.loss_GAN = WassersteinLoss()
        self.loss_similarity = ZNCCLoss()
        self.loss_HU = hu_loss_instance
        self.logger_interface = logger_interface
        self.engine: Optional[StepEngine] = None
        # launch plans per (engine, do_critic, do_generator) (_replay); CGAN3D_TRAINER_PLANS=0: eager
        self.use_plans = os.environ.get("CGAN3D_TRAINER_PLANS", "1") == "1"
        self._plans: Dict[tuple, object] = {}

        self.iteration = 0
        self.checkpoint_every = checkpoint_every
        self.checkpoint_dir = checkpoint_dir
        if self.checkpoint_dir is not None:
            self.checkpoint_dir = Path(self.checkpoint_dir)
            self.checkpoint_dir.mkdir(exist_ok=True, parents=True)
            self.load_checkpoint(_find_latest_checkpoint(self.checkpoint_dir))

    # ------------------------------------------------------------------------------------------
    def _engine_for(self, b_opt: int, b_sub: int, dims) -> StepEngine:
        e = self.engine
        dims = _planar_dims(dims, bool(getattr(self.generator.config, "is_2D", False)))  # 2-D: (1, H, W)
        if e is None or (e.b_opt, e.b_sub, e.dims) != (b_opt, b_sub, tuple(dims)):
            lo, hi = _hu_bounds(self.loss_HU)
            self.engine = StepEngine(self.generator, self.critic, self.generator.config, self.critic.config, b_opt,
                                     b_sub, tuple(dims), gp_weight=float(self.gp_w), hu_bounds=(lo, hi),
                                     gan_w=self.gan_loss_w, sim_w=self.sim_loss_w, hu_w=self.hu_loss_w,
                                     device=self.device, g_optim=self.optimizer_G, d_optim=self.optimizer_D,
                                     precision=self.precision, weight_clip=self.weight_clip)
            self._plans.clear()  # plans refer to the old engine's buffers
        return self.engine

    def _losses(self, keys) -> Dict[str, Tensor]:
        slots = {"D": L.L_D, "G": L.L_G, "G-full": L.L_GFULL, "sim": L.L_SIM, "HU": L.L_HU}
        return {k: self.engine.losses[slots[k]] for k in keys}

    @staticmethod
    def _same(t: Optional[Tensor], slot: Tensor) -> bool:
        """``t`` is None (the engine's resident operand), that operand itself, or equal to it."""
        if t is None:
            return True
        if t.numel() != slot.numel():
            return False
        if t.device == slot.device and t.data_ptr() == slot.data_ptr():
            return True
        return bool(torch.equal(t.detach().reshape(-1).to(slot.device, slot.dtype), slot.reshape(-1)))

    def _need_engine(self, who: str) -> StepEngine:
        if self.engine is None:
            raise RuntimeError(f"Trainer.{who}: no step engine yet (Trainer.train_step builds it from the first batch)")
        return self.engine

    def train_critic(self, real: Tensor, reconstructions: Tensor, retain_graph: bool) -> Dict[str, Tensor]:
        """Critic update (Trainer.py:108-142) on ``real`` and ``reconstructions`` (treated as data, as the
        reference's ``reconstructions.detach()``): tensors other than the engine's resident batch are
        copied into its slots first (same shapes required); None = the resident batch."""
        eng = self._need_engine("train_critic")
        for t, slot, name in ((real, eng.xc[:eng.b_opt], "real"), (reconstructions, eng.opt_hat, "reconstructions")):
            if t is not None and not (t.device == slot.device and t.data_ptr() == slot.data_ptr()):
                if t.numel() != slot.numel():
                    raise ValueError(f"train_critic: {name} has {t.numel()} elements, the engine's batch "
                                     f"{slot.numel()} (batch and patch size are fixed per engine)")
                slot.view(-1).copy_(t.detach().reshape(-1), non_blocking=True)
                if name == "reconstructions":
                    # the slot no longer holds the generator forward's output: train_generator refuses
                    # to backprop through it until the next generator forward
                    eng.opt_hat_foreign = True
        self.optimizer_D.sync_hyper()
        eng.critic_update()
        if self.lr_scheduler_D is not None:
            self.lr_scheduler_D.step()
        return self._losses(["D"])

    def train_generator(self, inputs: Tensor, reconstructions: Tensor, centerlines_masks: Tensor
                        ) -> Dict[str, Tensor]:
        """Generator update (Trainer.py:144-161).  The backward runs through the activations of the
        engine's last generator forward, so ``reconstructions`` must be that forward's output and
        ``inputs`` / ``centerlines_masks`` its batch (None = the resident ones); anything else raises
        ValueError rather than silently training on another batch."""
        eng = self._need_engine("train_generator")
        if getattr(eng, "opt_hat_foreign", False):
            raise ValueError("train_generator: train_critic replaced the generator output with other reconstructions "
                             "since the last generator forward (Trainer.train_step runs that forward)")
        for t, slot, name in ((inputs, eng.subopt, "inputs"), (reconstructions, eng.opt_hat, "reconstructions"),
                              (centerlines_masks, eng.mask, "centerlines_masks")):
            if not self._same(t, slot):
                raise ValueError(f"train_generator: {name} is not the batch of the engine's last generator forward "
                                 "(Trainer.train_step loads the batch and runs that forward)")
        self.optimizer_G.sync_hyper()
        eng.generator_update()
        if self.lr_scheduler_G is not None:
            self.lr_scheduler_G.step()
        return self._losses(["G", "G-full", "sim", "HU"])

    def train_step(self, patches: List[dict], iteration: int):
        opt, low, high = patches
        b_opt, b_sub = len(opt["data"]), len(low["data"]) + len(high["data"])
        dims = tuple(opt["data"].shape[2:])
        eng = self._engine_for(b_opt, b_sub, dims)
        # host -> HBM into the resident slots (Trainer.py:165-167,182-183)
        nl = low["data"].numel()
        do_g = iteration % self.train_generator_every == 0
        pairs = [(opt["data"], eng.xc[:b_opt].view(-1)), (low["data"], eng.subopt.view(-1)[:nl]),
                 (high["data"], eng.subopt.view(-1)[nl:])]
        if do_g:
            ml = low["seg"].numel()
            pairs += [(low["seg"], eng.mask.view(-1)[:ml]), (high["seg"], eng.mask.view(-1)[ml:])]
        if all(s.is_cuda and s.is_contiguous() and s.data_ptr() % 16 == 0 and d.data_ptr() % 16 == 0
               and s.numel() == d.numel() and s.element_size() == d.element_size() and s.dtype != torch.float64
               and (s.dtype == torch.float32) == (d.dtype == torch.float32) for s, d in pairs):
            # one launch for the batch (the loader's batches are in HBM already): fewer host calls per
            # step — the replayed plan's host enqueue is close to the step's GPU time
            ops.copy_multi([(s.reshape(-1), d) for s, d in pairs])
        else:
            for s, d in pairs:
                d.copy_(s.reshape(-1), non_blocking=True)
        # |OPT| != |LOW|+|HIGH|: the penalty's rows resampled on the host (model/utils.py:21-25, rng=self.rng)
        if eng.gp_idx is not None:
            if self.rng is None:
                self.rng = np.random.default_rng()
            eng.draw_gp_indices(self.rng)
        # eps ~ U[0,1) per interpolated sample, drawn on the device (model/utils.py:26)
        eng.eps.uniform_(0.0, 1.0)
        do_c = iteration % self.train_critic_every == 0
        log_dict = {}
        eng.opt_hat_foreign = False  # the step's own generator forward (replayed or eager) writes opt_hat
        if self._replay(eng, do_c, do_g):
            if do_c:
                log_dict = self._losses(["D"])
            if do_g:
                log_dict |= self._losses(["G", "G-full", "sim", "HU"])
        else:
            eng.generator_forward()
            if do_c:
                log_dict = self.train_critic(None, None, do_g)
            if do_g:
                log_dict |= self.train_generator(None, None, None)

        if iteration % self.log_every == 0:
            self.logger_interface.logger.log_loss({k: v.mean() for k, v in log_dict.items()}, iteration, "train")
        if iteration % self.log_images_every == 0:
            self.maybe_set_log_images_sample_size("train", patches[0]["data"].shape)
            cut = len(low["data"])
            opt_hat = eng.opt_hat.view(b_sub, 1, *dims)
            att = eng.G.att.view(b_sub, 1, *dims)
            self.logger_interface(patches, [None, opt_hat[:cut], opt_hat[cut:]], [None, att[:cut], att[cut:]],
                                  _scan_types(), iteration, "train", self.train_log_sample_size)
        return log_dict

    def _replay(self, eng: StepEngine, do_c: bool, do_g: bool) -> bool:
        """Run this iteration's generator forward + updates from a recorded launch plan
        (engine.record / run_plan, cgan3d_plan_*): one plan per (engine, schedule) combination,
        recorded on the combination's second iteration (the first runs eagerly: kernel code objects
        load lazily) and re-issued from C++ afterwards.  Learning rates reach the plan through the
        optimisers' device scalars (sync_hyper), the LR schedulers step on the host as in the eager
        path.  Returns False when the eager path must run (first sighting, debug mode, no plans)."""
        if not self.use_plans or self.debug:
            return False
        key = (id(eng), do_c, do_g)
        plan = self._plans.get(key)
        if plan is None:
            if key not in self._plans:
                self._plans[key] = None  # seen once: eager this time, record next time
                return False
            host = (self.optimizer_D._host_step, self.optimizer_G._host_step)
            plan = self._plans[key] = eng.record(do_c, do_g)
            assert (self.optimizer_D._host_step, self.optimizer_G._host_step) == host
        if do_c:
            self.optimizer_D.sync_hyper()
        if do_g:
            self.optimizer_G.sync_hyper()
        plan.run()
        if do_c:
            self.optimizer_D.note_step()
            if self.lr_scheduler_D is not None:
                self.lr_scheduler_D.step()
        if do_g:
            self.optimizer_G.note_step()
            if self.lr_scheduler_G is not None:
                self.lr_scheduler_G.step()
        return True

    def fit(self, train_loaders, val_loaders, profiler=None):
        self.generator.train()
        self.critic.train()
        augmenters = {"train": train_loaders, "val": val_loaders}
        self._manage_augmenters(augmenters, "start")
        for iteration in trange(self.iteration, self.train_iterations):
            patches = [next(train_loaders[st]) for st in ScanTypes]
            self.train_step(patches, iteration)
            if self.val_every is not None and iteration != 0 and iteration % self.val_every == 0:
                self.validate(val_loaders, iteration)
            if self.checkpoint_every is not None and iteration != 0 and iteration % self.checkpoint_every == 0:
                self.save_checkpoint(iteration)
            if profiler:
                profiler.step()
        if profiler:
            profiler.stop()
        if self.checkpoint_every is not None:
            self.save_checkpoint(self.train_iterations)
        self._manage_augmenters(augmenters, "end")
        self.logger_interface.end_hook()

    @torch.no_grad()
    def validate(self, val_loaders, train_iteration: int):
        """Eval-mode pass (Trainer.py:247-308): running-stat BN, no gradients."""
        if self.engine is not None:
            self.engine.sync_bn_buffers()  # data parallelism: rank 0's running statistics (engine docstring)
        self.critic.eval()
        self.generator.eval()
        z = torch.zeros(4, dtype=torch.float32, device=self.device)
        loss_sim, loss_G, loss_real_C, loss_fake_C = z.chunk(4)
        loggable = []
        for i in range(self.val_iterations):
            for st in ScanTypes:
                batch = next(val_loaders[st])
                sample = batch["data"].to(self.device, non_blocking=True)
                if st == 0:
                    loss_real_C -= self.loss_GAN(self.critic(sample))
                else:
                    attenuation = self.generator(sample)
                    sample_hat = sample - attenuation
                    loss_fake = self.loss_GAN(self.critic(sample_hat))
                    loss_fake_C += loss_fake
                    loss_G -= loss_fake
                    loss_sim += self.loss_similarity(sample_hat, sample)
                    if i == 0 and loggable is not None:
                        loggable.append([batch, sample_hat, attenuation])
                        if len(loggable) == 2:
                            patches, recs, atts = list(zip(*loggable))
                            self.maybe_set_log_images_sample_size("val", patches[0]["data"].shape)
                            self.logger_interface(patches, list(recs), list(atts), _scan_types()[1:],
                                                  train_iteration, "validation", self.val_log_sample_size)
                            loggable = None
        self.critic.train()
        self.generator.train()
        val_loss = {"D": (loss_real_C + loss_fake_C) / self.val_iterations,
                    "G": loss_G / (self.val_iterations * 2), "sim": loss_sim / (self.val_iterations * 2)}
        self.logger_interface.logger.log_loss(val_loss, train_iteration, "validation")
        return val_loss

    @property
    def model_torch_attrs(self) -> List[str]:
        return ["generator", "optimizer_G", "lr_scheduler_G", "discriminator", "critic", "optimizer_D",
                "lr_scheduler_D"]

    def save_checkpoint(self, iteration: int):
        if self.engine is not None:
            self.engine.sync_bn_buffers()
        state = {"iteration": iteration}
        for attr in self.model_torch_attrs:
            el = getattr(self, attr, None)
            state[attr] = el if el is None else el.state_dict()
        torch.save(state, self.checkpoint_dir / f"{iteration}.pt")
        logger.info("Checkpoint iteration %d", iteration)

    def load_checkpoint(self, ckpt_path: Optional[Path]):
        if ckpt_path is not None and Path(ckpt_path).is_file():
            logger.info("Resuming run from '%s'", str(ckpt_path))
            checkpoint: dict = torch.load(ckpt_path, map_location="cpu", weights_only=True)
            for k, v in checkpoint.items():
                if k in self.model_torch_attrs:
                    if v is not None and getattr(self, k, None) is not None:
                        getattr(self, k).load_state_dict(v)
                else:
                    setattr(self, k, v)
        logger.info("Starting from iteration %d", self.iteration)

    def _manage_augmenters(self, augmenters, event: str):
        assert event in ["start", "end"], f"Unknown event {event!r}"
        for mode, d in augmenters.items():
            if mode == "val" and self.val_every is None:
                continue
            for aug in d.values():
                if event == "start" and hasattr(aug, "restart"):
                    aug.restart()
                elif hasattr(aug, "_finish"):
                    aug._finish()

    def maybe_set_log_images_sample_size(self, mode: str, batch_shape):
        attr = f"{mode}_log_sample_size"
        if getattr(self, attr) is None:
            bs = batch_shape[-1 if len(batch_shape) == 5 else 0]
            setattr(self, attr, min(bs, 64))


def _hu_bounds(hu_loss) -> tuple:
    if hasattr(hu_loss, "lo"):
        return float(hu_loss.lo), float(hu_loss.hi)
    if hasattr(hu_loss, "min_HU"):  # the reference's HULoss stores full constant tensors (loss.py:51-56)
        return float(hu_loss.min_HU.reshape(-1)[0]), float(hu_loss.max_HU.reshape(-1)[0])
    raise TypeError("hu_loss_instance must be a HULoss")


def _scan_types():
    try:
        from contrast_gan_3D.alias import ScanType  # the caller's enum when running under train.py
        return list(ScanType)
    except Exception:
        return list(ScanTypes)


def _find_latest_checkpoint(d: Path) -> Optional[Path]:
    """``<int>.pt`` with the largest iteration (trainer/utils.py:26-34)."""
    cands = [p for p in Path(d).glob("*.pt") if p.stem.isdigit()]
    return max(cands, key=lambda p: int(p.stem)) if cands else None
