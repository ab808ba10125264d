"""CPU restatement of the reference's RL math helpers (test oracle only).

Every function restates one reference symbol; the docstring cites the
reference lines it follows.  Written independently in plain torch-CPU /
Python so it can be read against the reference line by line; it is not a
copy of the reference source.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

# ---------------------------------------------------------------------------
# trl/core.py
# ---------------------------------------------------------------------------


def masked_mean(values: torch.Tensor, mask: torch.Tensor, axis=None) -> torch.Tensor:
    """trl/core.py:43-48 — sum(values*mask)/sum(mask), optionally along `axis`."""
    prod = values * mask
    if axis is None:
        return prod.sum() / mask.sum()
    return prod.sum(axis) / mask.sum(axis)


def masked_var(values: torch.Tensor, mask: torch.Tensor, unbiased: bool = True) -> torch.Tensor:
    """trl/core.py:51-67 — masked variance about the masked mean; Bessel n/(n-1).

    Raises ValueError when the mask sums to zero (core.py:59-63).
    """
    mu = masked_mean(values, mask)
    var = masked_mean((values - mu) ** 2, mask)
    if unbiased:
        n = mask.sum()
        if n == 0:
            raise ValueError("The sum of the mask is zero")
        var = var * (n / (n - 1))
    return var


def masked_whiten(values: torch.Tensor, mask: torch.Tensor, shift_mean: bool = True) -> torch.Tensor:
    """trl/core.py:70-76 — (x-mu)*rsqrt(var+1e-8) (+mu back if not shift_mean)."""
    mu = masked_mean(values, mask)
    var = masked_var(values, mask)
    out = (values - mu) * torch.rsqrt(var + 1e-8)
    if not shift_mean:
        out = out + mu
    return out


# ---------------------------------------------------------------------------
# trl/trainer/utils.py
# ---------------------------------------------------------------------------


def selective_log_softmax(logits: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """trl/trainer/utils.py:1430-1462.

    fp32/fp64: gather(logits) - logsumexp(logits) (:1449-1453).
    fp16/bf16: log_softmax per row in the input dtype, then gather
    (:1454-1461) — output keeps the input dtype.
    """
    if logits.dtype in (torch.float32, torch.float64):
        picked = logits.gather(-1, index.unsqueeze(-1)).squeeze(-1)
        return picked - torch.logsumexp(logits, dim=-1)
    out = torch.log_softmax(logits, dim=-1)
    return out.gather(-1, index.unsqueeze(-1)).squeeze(-1)


def entropy_from_logits(logits: torch.Tensor, chunk_size: int = 1) -> torch.Tensor:
    """trl/trainer/utils.py:1465-1490 — -sum(exp(logp)*logp) over the last axis.

    The chunking only bounds peak memory; it does not change the value.
    """
    del chunk_size
    lp = torch.log_softmax(logits, dim=-1)
    return -(lp.exp() * lp).sum(-1)


def first_true_indices(bools: torch.Tensor, dtype=torch.long) -> torch.Tensor:
    """trl/trainer/utils.py:877-897 — index of first True per row, row length if none."""
    n = bools.size(-1)
    pos = torch.arange(n, dtype=dtype).expand_as(bools)
    cand = torch.where(bools, pos, torch.full_like(pos, n))
    return cand.min(dim=-1).values


def truncate_response(stop_token_id: int, pad_token_id: int, responses: torch.Tensor) -> torch.Tensor:
    """trl/trainer/utils.py:1036-1056 — pad everything after the first stop token."""
    first = first_true_indices(responses == stop_token_id).unsqueeze(-1)
    pos = torch.arange(responses.shape[1]).view(1, -1)
    return responses.masked_fill(pos > first, pad_token_id)


def pad(tensors: Sequence[torch.Tensor], padding_value: int = 0, padding_side: str = "right",
        pad_to_multiple_of: Optional[int] = None) -> torch.Tensor:
    """trl/trainer/utils.py:245-308 — stack ragged tensors into one padded tensor:
    the output shape is the per-dim max (:284), the first dim rounded up to
    pad_to_multiple_of (:287-290); `padding_side` places each tensor along the
    FIRST dim only, the trailing dims always start at 0 (:296-305)."""
    shape = [max(t.shape[d] for t in tensors) for d in range(tensors[0].dim())]
    if pad_to_multiple_of is not None and shape[0] % pad_to_multiple_of:
        shape[0] += pad_to_multiple_of - shape[0] % pad_to_multiple_of
    out = torch.full([len(tensors)] + shape, padding_value, dtype=tensors[0].dtype)
    for i, t in enumerate(tensors):
        if padding_side == "left":
            start = shape[0] - t.shape[0]
        elif padding_side == "right":
            start = 0
        else:
            raise ValueError("padding_side must be 'left' or 'right'")
        sl = (slice(start, start + t.shape[0]),) + tuple(slice(0, s) for s in t.shape[1:])
        out[(i,) + sl] = t
    return out


# ---------------------------------------------------------------------------
# trl/trainer/grpo_trainer.py helpers
# ---------------------------------------------------------------------------


def repeat_sampler_indices(n: int, mini_repeat_count: int, batch_size: int = 1, repeat_count: int = 1,
                           shuffle: bool = True, seed: Optional[int] = None) -> list[int]:
    """grpo_trainer.py:97-192 (RepeatSampler.__iter__ :170-188).

    Permutation from a local torch.Generator seeded with `seed` (:165-168),
    chunks of `batch_size`, incomplete tail chunk dropped, each chunk emitted
    `repeat_count` times with every index repeated `mini_repeat_count` times.
    """
    if shuffle:
        g = torch.Generator()
        if seed is not None:
            g.manual_seed(seed)
        order = torch.randperm(n, generator=g).tolist()
    else:
        order = list(range(n))
    out: list[int] = []
    for c in range(n // batch_size):
        chunk = order[c * batch_size:(c + 1) * batch_size]
        for _ in range(repeat_count):
            for idx in chunk:
                out.extend([idx] * mini_repeat_count)
    return out


def nanstd(t: torch.Tensor) -> torch.Tensor:
    """grpo_trainer.py:196-211 — unbiased std ignoring NaNs (1-D)."""
    keep = t[~torch.isnan(t)]
    n = keep.numel()
    var = ((keep - keep.mean()) ** 2).mean() * (n / (n - 1))
    return torch.sqrt(var)


def split_tensor_dict(d: dict, num_chunks: int) -> list[dict]:
    """grpo_trainer.py:214-241 — equal split along dim 0 (None passes through)."""
    first = next(v for v in d.values() if v is not None)
    size = first.shape[0] // num_chunks
    return [{k: (None if v is None else v[i * size:(i + 1) * size]) for k, v in d.items()}
            for i in range(num_chunks)]


def permute_sequence_dict(d: dict, perm: torch.Tensor) -> dict:
    """grpo_trainer.py:244-271 with the permutation made explicit (the reference
    draws it from the global torch RNG, :259)."""
    def take(v):
        if v is None:
            return None
        if isinstance(v, torch.Tensor):
            return v[perm]
        return [v[int(i)] for i in perm]
    return {k: take(v) for k, v in d.items()}


def get_high_entropy_mask(entropies: torch.Tensor, mask: torch.Tensor, threshold: float) -> torch.Tensor:
    """grpo_trainer.py:341-364 — keep tokens with entropy >= quantile(non-pad, threshold)."""
    valid = entropies[mask.bool()].float()
    if valid.numel() == 0:
        return torch.zeros_like(entropies, dtype=torch.bool)
    thr = torch.quantile(valid, threshold)
    return ((entropies * mask.float()) >= thr) & mask.bool()


def truncate_with_protected_tokens(ids: torch.Tensor, mask: torch.Tensor, target_length: int,
                                   protected_tokens: list[int]):
    """grpo_trainer.py:367-421 — keep protected ids + the rightmost non-protected ones."""
    prot = set(int(x) for x in protected_tokens)
    rows_i, rows_m = [], []
    for r in range(ids.shape[0]):
        row = ids[r].tolist()
        is_p = [x in prot for x in row]
        need = target_length - sum(is_p)
        if need < 0:
            raise ValueError(f"target_length ({target_length}) is too small for the protected tokens")
        free_pos = [i for i, p in enumerate(is_p) if not p]
        keep_free = set(free_pos[len(free_pos) - need:]) if need > 0 else set()
        keep = [i for i in range(len(row)) if is_p[i] or i in keep_free]
        rows_i.append(ids[r][keep])
        rows_m.append(mask[r][keep])
    return torch.stack(rows_i), torch.stack(rows_m)


def completion_mask_from_eos(completion_ids: torch.Tensor, eos_token_id: int,
                             mask_truncated: bool = False):
    """grpo_trainer.py:1812-1831 — mask[t] = t <= first EOS (EOS included), int32;
    lengths = mask.sum(1); optionally zero rows that never emit EOS."""
    is_eos = completion_ids == eos_token_id
    C = completion_ids.shape[1]
    eos_idx = torch.full((completion_ids.shape[0],), C, dtype=torch.long)
    has = is_eos.any(1)
    eos_idx[has] = is_eos.int().argmax(1)[has]
    mask = (torch.arange(C).view(1, -1) <= eos_idx.view(-1, 1)).int()
    lengths = mask.sum(1)
    if mask_truncated:
        mask = mask * has.unsqueeze(1).int()
    return mask, lengths, is_eos


def group_advantages(rewards_per_func: torch.Tensor, weights: torch.Tensor, num_generations: int,
                     scale_rewards: bool = True):
    """grpo_trainer.py:1914-1930 — weighted nansum of rewards, per-group mean and
    UNBIASED std, A = r - mean (/(std + 1e-4) when scale_rewards).

    Parity unpinned by reference tests.
    Returns (advantages, rewards, group_mean, group_std, is_std_zero).
    """
    r = (rewards_per_func * weights.unsqueeze(0)).nansum(dim=1)
    g = r.view(-1, num_generations)
    mean = g.mean(dim=1)
    std = g.std(dim=1)
    zero = torch.isclose(std, torch.zeros_like(std))
    adv = r - mean.repeat_interleave(num_generations)
    if scale_rewards:
        adv = adv / (std.repeat_interleave(num_generations) + 1e-4)
    return adv, r, mean, std, zero


def grpo_loss(per_token_logps: torch.Tensor, advantages: torch.Tensor, completion_mask: torch.Tensor,
              old_per_token_logps: Optional[torch.Tensor] = None,
              ref_per_token_logps: Optional[torch.Tensor] = None,
              entropy_mask: Optional[torch.Tensor] = None,
              entropies: Optional[torch.Tensor] = None,
              beta: float = 0.0, epsilon_low: float = 0.2, epsilon_high: float = 0.2,
              delta: Optional[float] = None, loss_type: str = "bnpo",
              importance_sampling_level: str = "token", max_completion_length: int = 256):
    """grpo_trainer.py:2058-2175 (`_compute_loss`), from the log-probs onward.

    `per_token_logps` may require grad; the returned loss is differentiable so
    the test-suite can take d loss / d logps with autograd as the reference
    does.  Metrics mirror :2139-2174 (before the cross-rank gather).
    Parity unpinned by reference tests.
    """
    lp = per_token_logps
    m = completion_mask
    if beta != 0.0:
        d = ref_per_token_logps - lp
        kl = torch.exp(d) - d - 1  # :2085-2089
    old = lp.detach() if old_per_token_logps is None else old_per_token_logps  # :2097
    lr = lp - old
    if importance_sampling_level == "token":
        liw = lr
    elif importance_sampling_level == "sequence":
        liw = ((lr * m).sum(-1) / m.sum(-1).clamp(min=1.0)).unsqueeze(-1)  # :2102-2104
    else:
        raise ValueError(f"Unknown importance sampling level: {importance_sampling_level}")
    c1 = torch.exp(liw)
    c2 = torch.clamp(c1, 1 - epsilon_low, 1 + epsilon_high)
    if delta is not None:
        c1 = torch.clamp(c1, max=delta)  # :2116-2118
    a = advantages.unsqueeze(1)
    ptl = -torch.min(c1 * a, c2 * a)  # :2120-2122
    if entropy_mask is not None:
        ptl = ptl * entropy_mask
    if beta != 0.0:
        ptl = ptl + beta * kl
    if loss_type == "grpo":
        loss = ((ptl * m).sum(-1) / m.sum(-1).clamp(min=1.0)).mean()
    elif loss_type == "bnpo":
        loss = (ptl * m).sum() / m.sum().clamp(min=1.0)
    elif loss_type == "dr_grpo":
        loss = (ptl * m).sum() / (ptl.size(0) * max_completion_length)
    else:
        raise ValueError(f"Unknown loss type: {loss_type}")

    tok = m.sum().clamp(min=1.0)

    def bmean(x):
        return x.mean() if x.shape[1] == 1 else (x * m).sum() / tok

    metrics = {}
    with torch.no_grad():
        if beta != 0.0:
            metrics["kl"] = bmean(kl).item()
        if entropies is not None:
            metrics["entropy"] = bmean(entropies).item()
        low = ((c1 < 1 - epsilon_low) & (a < 0)).float()
        high = ((c1 > 1 + epsilon_high) & (a > 0)).float()
        metrics["clip_ratio/low_mean"] = bmean(low).item()
        metrics["clip_ratio/high_mean"] = bmean(high).item()
        metrics["clip_ratio/region_mean"] = bmean(torch.maximum(low, high)).item()
    return loss, metrics


# ---------------------------------------------------------------------------
# trl/trainer/ppo_trainer.py
# ---------------------------------------------------------------------------

INVALID_LOGPROB = 1.0  # ppo_trainer.py:81


def ppo_rewards(logprobs, ref_logprobs, scores, sequence_lengths, kl_coef: float, kl_estimator: str = "k1"):
    """ppo_trainer.py:500-516 — KL-shaped per-token rewards with the score added at
    min(seq_len+1, C-1).  Inputs already INVALID_LOGPROB-masked.
    Parity unpinned by reference tests."""
    logr = ref_logprobs - logprobs
    kl = -logr if kl_estimator == "k1" else (logr.exp() - 1) - logr
    non_score = -kl_coef * kl
    rewards = non_score.clone()
    C = rewards.size(1)
    sl1 = sequence_lengths + 1
    end = torch.where(sl1 < C, sl1, sequence_lengths)
    rewards[torch.arange(rewards.size(0)), end] += scores
    return rewards, kl, non_score


def gae(rewards: torch.Tensor, values: torch.Tensor, gamma: float, lam: float):
    """ppo_trainer.py:523-533 — reverse-time GAE recursion, returns = A + V.
    Parity unpinned by reference tests."""
    B, T = rewards.shape
    adv = torch.zeros_like(rewards)
    last = torch.zeros(B, dtype=rewards.dtype)
    for t in range(T - 1, -1, -1):
        nv = values[:, t + 1] if t < T - 1 else torch.zeros(B, dtype=rewards.dtype)
        d = rewards[:, t] + gamma * nv - values[:, t]
        last = d + gamma * lam * last
        adv[:, t] = last
    return adv, adv + values


def ppo_losses(new_logprobs, mb_logprobs, mb_advantage, vpred, mb_values, mb_return,
               padding_mask, padding_mask_p1, cliprange: float, cliprange_value: float, vf_coef: float,
               token_terms: bool = False):
    """ppo_trainer.py:557-605 — clipped value loss + clipped PG loss (inputs already
    INVALID_LOGPROB / zero masked as at :562-566).  Parity unpinned.
    token_terms: stats["tokens"] also holds each statistic's per-token terms
    (the elements its mean runs over), for error estimates in the tests."""
    vclip = torch.clamp(vpred, mb_values - cliprange_value, mb_values + cliprange_value)
    v1 = (vpred - mb_return) ** 2
    v2 = (vclip - mb_return) ** 2
    vf_loss = 0.5 * masked_mean(torch.max(v1, v2), ~padding_mask_p1)
    vf_clipfrac = masked_mean((v2 > v1).float(), ~padding_mask_p1)
    diff = new_logprobs - mb_logprobs
    ratio = torch.exp(diff)
    a = mb_advantage
    p1 = -a * ratio
    p2 = -a * torch.clamp(ratio, 1.0 - cliprange, 1.0 + cliprange)
    pg_loss = masked_mean(torch.max(p1, p2), ~padding_mask)
    loss = pg_loss + vf_coef * vf_loss
    with torch.no_grad():
        stats = dict(pg_clipfrac=masked_mean((p2 > p1).float(), ~padding_mask).item(),
                     vf_clipfrac=vf_clipfrac.item(), approxkl=(0.5 * (diff ** 2).mean()).item(),
                     ratio=ratio.mean().item())
        if token_terms:
            stats["tokens"] = dict(pg_loss=torch.max(p1, p2)[~padding_mask].float(),
                                   vf_loss=0.5 * torch.max(v1, v2)[~padding_mask_p1].float(),
                                   approxkl=0.5 * (diff ** 2).flatten().float(), ratio=ratio.flatten().float())
    return loss, pg_loss, vf_loss, stats


def value_head(hidden: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None):
    """trl/models/modeling_value_head.py:50-59 (eval: dropout is identity) — cast the
    hidden state to the head dtype, Linear(H, 1), squeeze."""
    h = hidden.to(weight.dtype)
    out = h @ weight.view(-1, 1)
    if bias is not None:
        out = out + bias
    return out.squeeze(-1)


# ---------------------------------------------------------------------------
# torch.optim.AdamW (third-party op the reference calls through transformers'
# Trainer.create_optimizer)
# ---------------------------------------------------------------------------


def adamw_step(p, g, m, v, step: int, lr: float, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
    """One decoupled-weight-decay Adam step in float64, the published AdamW update
    (Loshchilov & Hutter) as torch.optim.AdamW implements it:
        p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2
        p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
    """
    p = p * (1 - lr * weight_decay)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    p = p - (lr / bc1) * m / (torch.sqrt(v) / math.sqrt(bc2) + eps)
    return p, m, v


def clip_coef(grads: Sequence[torch.Tensor], max_norm: float):
    """torch.nn.utils.clip_grad_norm_ semantics: total L2 norm, coef = min(1, max/(norm+1e-6))."""
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads))
    return total, min(1.0, max_norm / (float(total) + 1e-6))
