"""Learning-rate schedules of the transformers Trainer that the reference's
GRPOTrainer / PPOTrainer inherit (`lr_scheduler_type`, `lr_scheduler_kwargs`,
`warmup_steps` / `warmup_ratio`; transformers optimization.py `get_scheduler`).

The fused AdamW takes the learning rate as a launch argument, so a schedule is
just the LambdaLR multiplier: `multiplier(step)` is the factor for the
optimizer step that follows `step` completed steps (the Trainer calls
`optimizer.step()` then `lr_scheduler.step()`, so step 0 uses lambda(0)).
Each lambda restates transformers' `_get_*_lr_lambda` of the same name.
Schedules that need evaluation metrics or per-parameter state
(reduce_lr_on_plateau, greedy) and warmup_stable_decay raise.
"""
from __future__ import annotations

import functools
import math
from typing import Callable, Optional


def _warm(step: int, warmup: int) -> float:
    return float(step) / float(max(1, warmup))


def _linear(step: int, *, warmup: int, total: int) -> float:
    if step < warmup:
        return _warm(step, warmup)
    return max(0.0, float(total - step) / float(max(1, total - warmup)))


def _cosine(step: int, *, warmup: int, total: int, num_cycles: float = 0.5, min_lr_rate: float = 0.0) -> float:
    if step < warmup:
        return _warm(step, warmup)
    progress = float(step - warmup) / float(max(1, total - warmup))
    factor = 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress))
    return max(0, factor * (1 - min_lr_rate) + min_lr_rate)


def _cosine_restarts(step: int, *, warmup: int, total: int, num_cycles: int = 1) -> float:
    if step < warmup:
        return _warm(step, warmup)
    progress = float(step - warmup) / float(max(1, total - warmup))
    if progress >= 1.0:
        return 0.0
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * ((float(num_cycles) * progress) % 1.0))))


def _polynomial(step: int, *, warmup: int, total: int, lr_end: float, power: float, lr_init: float) -> float:
    if step < warmup:
        return _warm(step, warmup)
    if step > total:
        return lr_end / lr_init
    pct_remaining = 1 - (step - warmup) / (total - warmup)
    return ((lr_init - lr_end) * pct_remaining ** power + lr_end) / lr_init


def _constant(step: int) -> float:
    return 1.0


def _constant_warmup(step: int, *, warmup: int) -> float:
    if step < warmup:
        return float(step) / float(max(1.0, warmup))
    return 1.0


def _inverse_sqrt(step: int, *, warmup: int, timescale: int) -> float:
    if step < warmup:
        return _warm(step, warmup)
    return 1.0 / math.sqrt((step + timescale - warmup) / timescale)


def _cosine_warmup_min_lr(step: int, *, warmup: int, total: int, num_cycles: float = 0.5, min_lr_rate: float = 0.0,
                          warmup_lr_rate: Optional[float] = None) -> float:
    s, w, t = float(step), float(warmup), float(total)
    if s < w:
        if warmup_lr_rate is None:
            return (s + 1.0) / max(1.0, w)
        return float(warmup_lr_rate) + (1.0 - float(warmup_lr_rate)) * s / max(1, w - 1)
    progress = (s - w + 1.0) / max(1.0, t - w)
    factor = 0.5 * (1.0 + math.cos(math.pi * num_cycles * 2.0 * progress))
    return max(0, factor * (1 - min_lr_rate) + min_lr_rate)


def _min_lr_rate(kw: dict, lr: float) -> float:
    min_lr, rate = kw.pop("min_lr", None), kw.pop("min_lr_rate", None)
    if min_lr is not None and rate is not None:
        raise ValueError("Only one of min_lr or min_lr_rate should be set")
    if min_lr is not None:
        return min_lr / lr
    if rate is None:
        raise ValueError("One of min_lr or min_lr_rate should be set through the `lr_scheduler_kwargs`")
    return rate


def warmup_steps(args, total: int) -> int:
    """TrainingArguments.get_warmup_steps: `warmup_steps` when >= 1 (a float
    below 1 is a ratio in transformers >= 5), else ceil(total * warmup_ratio)."""
    ws = getattr(args, "warmup_steps", 0) or 0
    if ws >= 1:
        return int(ws)
    if ws > 0:
        return math.ceil(total * ws)
    return math.ceil(total * (getattr(args, "warmup_ratio", 0.0) or 0.0))


def multiplier(kind: str, total: int, warmup: int, lr: float, kwargs: Optional[dict] = None) -> Callable[[int], float]:
    """The LambdaLR lambda of transformers `get_scheduler(kind, ...)` (a
    picklable functools.partial of a module-level function, as transformers')."""
    kind = getattr(kind, "value", kind)
    kw = dict(kwargs or {})
    if kind == "linear":
        return functools.partial(_linear, warmup=warmup, total=total)
    if kind == "cosine":
        return functools.partial(_cosine, warmup=warmup, total=total, **kw)
    if kind == "cosine_with_restarts":
        return functools.partial(_cosine_restarts, warmup=warmup, total=total, **kw)
    if kind == "polynomial":
        lr_end, power = kw.pop("lr_end", 1e-7), kw.pop("power", 1.0)
        if kw:
            raise TypeError(f"polynomial schedule: unexpected kwargs {sorted(kw)}")
        if not lr > lr_end:
            raise ValueError(f"lr_end ({lr_end}) must be smaller than initial lr ({lr})")
        return functools.partial(_polynomial, warmup=warmup, total=total, lr_end=lr_end, power=power, lr_init=lr)
    if kind == "constant":
        return _constant
    if kind == "constant_with_warmup":
        return functools.partial(_constant_warmup, warmup=warmup)
    if kind == "inverse_sqrt":
        ts = kw.pop("timescale", None)
        return functools.partial(_inverse_sqrt, warmup=warmup, timescale=ts if ts is not None else (warmup or 10_000))
    if kind == "cosine_with_min_lr":
        rate = _min_lr_rate(kw, lr)
        return functools.partial(_cosine, warmup=warmup, total=total, min_lr_rate=rate, **kw)
    if kind == "cosine_warmup_with_min_lr":
        rate = _min_lr_rate(kw, lr)
        return functools.partial(_cosine_warmup_min_lr, warmup=warmup, total=total, min_lr_rate=rate, **kw)
    raise ValueError(f"lr_scheduler_type {kind!r} is not supported by the MI355X trainers (supported: linear, cosine, "
                     "cosine_with_restarts, polynomial, constant, constant_with_warmup, inverse_sqrt, "
                     "cosine_with_min_lr, cosine_warmup_with_min_lr)")


def for_args(args, total: int) -> Callable[[int], float]:
    """The multiplier a TrainingArguments-like config asks for over `total` steps."""
    return multiplier(args.lr_scheduler_type, total, warmup_steps(args, total), args.learning_rate,
                      getattr(args, "lr_scheduler_kwargs", None))
