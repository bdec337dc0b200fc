"""Diffusion schedulers (the reference uses candle's DDIM and Euler-ancestral,
cake-core/src/models/sd/sd.rs:429-431,442,476,504).

Both operate on f32 latents with host-side coefficients.  The device path
(``step_coefs`` + sd_small.hip ``sched_step``) writes every step's update as
``prev = A x + B eps + N z`` with the next step's input scale S, so the
CFG combine, the update and the next UNet input are one kernel whose
coefficients come from a device table (the denoise step replays as a graph);
the torch methods below are the CPU path and the reference math.
"""
from __future__ import annotations

import math

import torch

from .config import SchedulerConfig


def _alphas_cumprod(cfg: SchedulerConfig) -> torch.Tensor:
    betas = torch.linspace(math.sqrt(cfg.beta_start), math.sqrt(cfg.beta_end),
                           cfg.train_timesteps, dtype=torch.float64) ** 2  # scaled_linear
    return torch.cumprod(1.0 - betas, 0)


class DDIMScheduler:
    """DDIM, eta = 0; epsilon or v-prediction; 'leading' spacing + steps_offset."""

    def __init__(self, cfg: SchedulerConfig, steps: int):
        self.cfg = cfg
        self.n_steps = steps
        self.acp = _alphas_cumprod(cfg)
        self.step_ratio = cfg.train_timesteps // steps
        self._timesteps = [s * self.step_ratio + cfg.steps_offset for s in range(steps)][::-1]
        self.final_acp = float(self.acp[0])
        self.init_noise_sigma = 1.0

    def timesteps(self) -> list[int]:
        return list(self._timesteps)

    def scale_model_input(self, sample: torch.Tensor, timestep: int) -> torch.Tensor:
        return sample

    def step(self, model_output: torch.Tensor, timestep: int, sample: torch.Tensor,
             generator: torch.Generator | None = None) -> torch.Tensor:
        t = timestep if timestep < len(self.acp) else timestep - 1
        prev = t - self.step_ratio
        a_t = float(self.acp[t])
        a_prev = float(self.acp[prev]) if prev >= 0 else self.final_acp
        b_t = 1.0 - a_t
        x = sample.float()
        e = model_output.float()
        if self.cfg.prediction_type == "epsilon":
            x0 = (x - math.sqrt(b_t) * e) / math.sqrt(a_t)
            eps = e
        else:  # v_prediction
            x0 = math.sqrt(a_t) * x - math.sqrt(b_t) * e
            eps = math.sqrt(a_t) * e + math.sqrt(b_t) * x
        return math.sqrt(a_prev) * x0 + math.sqrt(1.0 - a_prev) * eps

    def add_noise(self, original: torch.Tensor, noise: torch.Tensor, timestep: int) -> torch.Tensor:
        t = timestep if timestep < len(self.acp) else timestep - 1
        a = float(self.acp[t])
        return math.sqrt(a) * original.float() + math.sqrt(1.0 - a) * noise.float()

    def input_scale(self, timestep: int) -> float:
        return 1.0

    def step_coefs(self, timestep: int, next_timestep: int | None) -> tuple:
        """(A, B, N, S_next): prev = A x + B eps (+ N z); S_next scales the next input."""
        t = timestep if timestep < len(self.acp) else timestep - 1
        prev = t - self.step_ratio
        a_t = float(self.acp[t])
        a_p = float(self.acp[prev]) if prev >= 0 else self.final_acp
        if self.cfg.prediction_type == "epsilon":
            A = math.sqrt(a_p / a_t)
            B = math.sqrt(1.0 - a_p) - math.sqrt(a_p * (1.0 - a_t) / a_t)
        else:  # v_prediction
            A = math.sqrt(a_p * a_t) + math.sqrt((1.0 - a_p) * (1.0 - a_t))
            B = math.sqrt((1.0 - a_p) * a_t) - math.sqrt(a_p * (1.0 - a_t))
        return (A, B, 0.0, 1.0)


class EulerAncestralScheduler:
    """Euler-ancestral (SDXL-Turbo), epsilon prediction."""

    def __init__(self, cfg: SchedulerConfig, steps: int):
        self.cfg = cfg
        self.n_steps = steps
        acp = _alphas_cumprod(cfg)
        sig = ((1 - acp) / acp).sqrt()
        T = cfg.train_timesteps
        if cfg.timestep_spacing == "trailing":
            ts = torch.arange(T, 0, -T / steps, dtype=torch.float64).round() - 1
        elif cfg.timestep_spacing == "leading":
            ratio = T // steps
            ts = (torch.arange(0, steps, dtype=torch.float64) * ratio).round().flip(0) + cfg.steps_offset
        else:
            ts = torch.linspace(0, T - 1, steps, dtype=torch.float64).flip(0)
        idx = torch.arange(T, dtype=torch.float64)
        sig_t = torch.from_numpy(__import__("numpy").interp(ts.numpy(), idx.numpy(), sig.numpy()))
        self.sigmas = torch.cat([sig_t, torch.zeros(1, dtype=torch.float64)])
        self._timesteps = [int(t) for t in ts.tolist()]
        self.init_noise_sigma = float(math.sqrt(float(self.sigmas.max()) ** 2 + 1))
        self._index = {t: i for i, t in enumerate(self._timesteps)}

    def timesteps(self) -> list[int]:
        return list(self._timesteps)

    def scale_model_input(self, sample: torch.Tensor, timestep: int) -> torch.Tensor:
        s = float(self.sigmas[self._index[timestep]])
        return sample / math.sqrt(s * s + 1)

    def step(self, model_output: torch.Tensor, timestep: int, sample: torch.Tensor,
             generator: torch.Generator | None = None) -> torch.Tensor:
        i = self._index[timestep]
        s_from, s_to = float(self.sigmas[i]), float(self.sigmas[i + 1])
        x = sample.float()
        x0 = x - s_from * model_output.float()
        s_up = math.sqrt(max(0.0, s_to ** 2 * (s_from ** 2 - s_to ** 2) / s_from ** 2))
        s_down = math.sqrt(max(0.0, s_to ** 2 - s_up ** 2))
        d = (x - x0) / s_from
        prev = x + d * (s_down - s_from)
        if s_up > 0:
            noise = torch.randn(x.shape, generator=generator, device="cpu").to(x.device)
            prev = prev + noise * s_up
        return prev

    def add_noise(self, original: torch.Tensor, noise: torch.Tensor, timestep: int) -> torch.Tensor:
        s = float(self.sigmas[self._index.get(timestep, 0)])
        return original.float() + noise.float() * s

    def input_scale(self, timestep: int) -> float:
        s = float(self.sigmas[self._index[timestep]])
        return 1.0 / math.sqrt(s * s + 1)

    def step_coefs(self, timestep: int, next_timestep: int | None) -> tuple:
        i = self._index[timestep]
        s_from, s_to = float(self.sigmas[i]), float(self.sigmas[i + 1])
        s_up = math.sqrt(max(0.0, s_to ** 2 * (s_from ** 2 - s_to ** 2) / s_from ** 2))
        s_down = math.sqrt(max(0.0, s_to ** 2 - s_up ** 2))
        S = self.input_scale(next_timestep) if next_timestep is not None else 1.0
        return (1.0, s_down - s_from, s_up, S)


def build_scheduler(cfg: SchedulerConfig, steps: int):
    if cfg.kind == "ddim":
        return DDIMScheduler(cfg, steps)
    if cfg.kind == "euler_ancestral":
        return EulerAncestralScheduler(cfg, steps)
    raise ValueError(cfg.kind)
