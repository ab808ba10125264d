"""CPU restatement of the rollout sampler the reference drives (test oracle only).

The reference calls transformers' `GenerationMixin._sample` with a
`GenerationConfig(do_sample=True, temperature, top_p, top_k, min_p,
repetition_penalty)` built at trl/trainer/grpo_trainer.py:995-1014 (PPO:
ppo_trainer.py:369-375 with temperature+1e-7, top_k=0, top_p=1).  The
arithmetic lives in the third-party transformers package (installed 5.15.0;
the reference pins >=4.53.2, setup.cfg:44-47).  This module restates the
published processor algorithms in the order transformers applies them
(generation/utils.py `_get_logits_processor`: repetition penalty, min-new-
tokens EOS suppression, then the warpers temperature -> top-k -> top-p ->
min-p) and the final-token bookkeeping of `_sample` (pad after EOS).

The random draw is NOT the reference's `torch.multinomial` (whose stream no
device sampler can reproduce, SURVEY.md §7 "Sampling RNG"); parity for
sampled ids is therefore checked on identical logits with the product's own
Philox4x32-10 stream, restated in C in `oracle/c/philox_ref.c`.
"""
from __future__ import annotations

from typing import Optional

import torch

NEG_INF = float("-inf")


def repetition_penalty(scores: torch.Tensor, seen: torch.Tensor, penalty: float) -> torch.Tensor:
    """RepetitionPenaltyLogitsProcessor: for every token id already present in the
    row (prompt + generated), score<0 -> score*penalty, else score/penalty.
    `seen` is a bool [B, V] membership mask (duplicates collapse, as the
    gather/scatter in transformers does)."""
    if penalty == 1.0:
        return scores
    pen = torch.where(scores < 0, scores * penalty, scores / penalty)
    return torch.where(seen, pen, scores)


def suppress_eos(scores: torch.Tensor, eos_ids, active: bool) -> torch.Tensor:
    """MinNewTokensLengthLogitsProcessor: EOS ids -> -inf while fewer than
    min_new_tokens have been generated."""
    if not active or eos_ids is None:
        return scores
    out = scores.clone()
    for e in ([eos_ids] if isinstance(eos_ids, int) else eos_ids):
        out[:, e] = NEG_INF
    return out


def temperature(scores: torch.Tensor, t: float) -> torch.Tensor:
    """TemperatureLogitsWarper (skipped by transformers when t == 1.0)."""
    return scores if t == 1.0 else scores / t


def top_k(scores: torch.Tensor, k: Optional[int], min_tokens_to_keep: int = 1) -> torch.Tensor:
    """TopKLogitsWarper: drop scores strictly below the k-th largest (ties kept)."""
    if not k:
        return scores
    k = min(max(int(k), min_tokens_to_keep), scores.size(-1))
    kth = torch.topk(scores, k, dim=-1).values[..., -1:]
    return scores.masked_fill(scores < kth, NEG_INF)


def top_p(scores: torch.Tensor, p: float, min_tokens_to_keep: int = 1) -> torch.Tensor:
    """TopPLogitsWarper: sort ascending, cumulative softmax mass, remove entries whose
    cumulative mass (from the bottom) is <= 1-p, never the last min_tokens_to_keep."""
    if p >= 1.0:
        return scores
    srt, idx = torch.sort(scores, descending=False, dim=-1)
    cum = srt.softmax(dim=-1).cumsum(dim=-1)
    drop_sorted = cum <= (1 - p)
    drop_sorted[..., -min_tokens_to_keep:] = False
    drop = torch.zeros_like(drop_sorted).scatter(-1, idx, drop_sorted)
    return scores.masked_fill(drop, NEG_INF)


def min_p(scores: torch.Tensor, mp: Optional[float], min_tokens_to_keep: int = 1) -> torch.Tensor:
    """MinPLogitsWarper: drop tokens whose prob < min_p * max prob (keep the argmax)."""
    if mp is None:
        return scores
    probs = scores.softmax(dim=-1)
    thr = mp * probs.amax(dim=-1, keepdim=True)
    drop = probs < thr
    keep_idx = torch.topk(probs, min(min_tokens_to_keep, probs.size(-1)), dim=-1).indices
    drop.scatter_(-1, keep_idx, False)
    return scores.masked_fill(drop, NEG_INF)


def process_scores(logits: torch.Tensor, *, seen: Optional[torch.Tensor] = None, rep_penalty: float = 1.0,
                   eos_ids=None, suppress_eos_now: bool = False, t: float = 1.0, k: Optional[int] = None,
                   p: float = 1.0, mp: Optional[float] = None) -> torch.Tensor:
    """The full processor chain on fp32 scores (`_sample` takes `logits[:, -1].float()`)."""
    s = logits.float()
    if seen is not None:
        s = repetition_penalty(s, seen, rep_penalty)
    s = suppress_eos(s, eos_ids, suppress_eos_now)
    s = temperature(s, t)
    s = top_k(s, k)
    s = top_p(s, p)
    s = min_p(s, mp)
    return s


def gumbel_pick(scores: torch.Tensor, uniforms: torch.Tensor) -> torch.Tensor:
    """Exact categorical draw from softmax(scores) by the Gumbel-max identity,
    argmax_j(scores_j - log(-log u_j)), in float64.  -inf entries never win."""
    g = -torch.log(-torch.log(uniforms.double()))
    return torch.argmax(scores.double() + g, dim=-1)


def finish_tokens(next_tokens: torch.Tensor, unfinished: torch.Tensor, pad_token_id: int, eos_ids):
    """`_sample` bookkeeping: finished rows emit pad; a row finishes on EOS."""
    nt = next_tokens * unfinished + pad_token_id * (1 - unfinished)
    eos = torch.zeros_like(nt, dtype=torch.bool)
    for e in ([eos_ids] if isinstance(eos_ids, int) else eos_ids):
        eos |= nt == e
    return nt, unfinished & (~eos).long()
