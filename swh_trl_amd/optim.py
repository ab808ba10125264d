"""Flat-buffer AdamW with on-device global-norm clipping (HIP kernels).

Replaces torch.optim.AdamW (+ clip_grad_norm_) that transformers' Trainer
builds for the reference.  Every trainable weight is a
view into one flat buffer, so one kernel updates all of them and the clip
coefficient is consumed on device (no host sync).  Master weights and both
moments are fp32; the bf16 model copy is refreshed in the same pass.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib, profiling
from ._lib import call
from .ops import _dtype_code, _p, _stream


class FlatAdamW:
    def __init__(self, numel: int, device, lr: float = 1e-6, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: Optional[float] = 1.0, no_decay_ranges=()):
        self.numel = int(numel)
        self.lr = float(lr)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.master = torch.zeros(self.numel, device=device, dtype=torch.float32)
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self._partials = torch.empty(_lib.load().swh_sqnorm_partials(self.numel), device=device,
                                     dtype=torch.float32)
        self.clip_out = torch.empty(2, device=device, dtype=torch.float32)  # {total_norm, coef}
        # [start, end) element ranges without weight decay (biases / norm weights), merged,
        # each start/end a multiple of 4 (the model layout aligns every view to 64)
        merged = []
        for s, e in sorted(no_decay_ranges):
            if merged and s <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], e)
            else:
                merged.append([s, e])
        if any(s % 4 or (e % 4 and e != self.numel) for s, e in merged):
            raise ValueError("no_decay_ranges must start and end on multiples of 4 elements")
        self.no_decay = (torch.tensor(merged, dtype=torch.int64, device=device).reshape(-1)
                         if merged else None)

    def grad_norm(self, grad: torch.Tensor) -> torch.Tensor:
        call("swh_grad_sqnorm", grad.data_ptr(), _dtype_code(grad, "grad_norm"), self.numel, self._partials.data_ptr(),
             _stream())
        mn = float(self.max_grad_norm) if self.max_grad_norm else 0.0
        call("swh_finalize_clip", self._partials.data_ptr(), self._partials.numel(), mn, self.clip_out.data_ptr(),
             _stream())
        return self.clip_out[0]

    def step(self, grad: torch.Tensor, model_out: Optional[torch.Tensor] = None, lr: Optional[float] = None):
        """Clip (if max_grad_norm) and update; returns the pre-clip total norm (device)."""
        if grad.numel() != self.numel:
            raise ValueError("flat gradient size mismatch")
        norm = self.grad_norm(grad)
        self.step_count += 1
        lr = self.lr if lr is None else float(lr)
        clip = self.clip_out if self.max_grad_norm else None
        nbytes = self.numel * (24 + grad.element_size() + (model_out.element_size() if model_out is not None else 0))
        nd = self.no_decay
        with profiling.kernel("adamw", nbytes):
            call("swh_adamw", self.master.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                 grad.data_ptr(), _dtype_code(grad, "adamw"), _p(model_out),
                 _dtype_code(model_out, "adamw") if model_out is not None else 0, self.numel, lr, self.betas[0],
                 self.betas[1], self.eps, self.weight_decay, self.step_count, _p(clip), _p(nd),
                 0 if nd is None else nd.numel() // 2, _stream())
        return norm

    def state_dict(self):
        return {"master": self.master, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "step": self.step_count, "lr": self.lr}

    def load_state_dict(self, sd):
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
        self.lr = float(sd.get("lr", self.lr))


def sync_ref_model(ref_flat: torch.Tensor, policy_flat: torch.Tensor, alpha: float) -> None:
    """TR-DPO mixup (callbacks.py:106-131): ref = ref * (1 - alpha) + alpha * policy,
    one streaming kernel over the flat parameter buffers."""
    if ref_flat.shape != policy_flat.shape or ref_flat.dtype != policy_flat.dtype:
        raise ValueError("sync_ref_model: reference and policy buffers must match in size and dtype")
    call("swh_ema_mix", ref_flat.data_ptr(), policy_flat.data_ptr(), _dtype_code(ref_flat, "sync_ref_model"),
         ref_flat.numel(), 1.0 - float(alpha), float(alpha), _stream())
