"""Torch-facing operators over the HIP C-ABI (device tensors only).

Names, argument meaning and error behaviour mirror the reference helpers they
replace (trl/core.py, trl/trainer/utils.py, grpo_trainer.py, ppo_trainer.py);
every op runs on the swh_trl_amd HIP library and raises on CPU tensors.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib, profiling
from ._lib import GRPOLossParams, SampleParams, call



def _dev(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"swh_trl_amd.{name}: needs a ROCm device tensor (no CPU fallback)")


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


_dtype_code = _lib.dtype_code   # the one place a dtype code is made (from the tensor)


# ---------------------------------------------------------------------------
# log-probs / entropy (utils.py:1430-1490)
# ---------------------------------------------------------------------------

def _rows_view(logits: torch.Tensor):
    """(outer, inner, stride_outer, stride_inner, V) for a [..., V] tensor whose
    last dim is contiguous and whose leading dims collapse into <= 2 strides."""
    if logits.stride(-1) != 1:
        raise ValueError("logits must be contiguous in the vocabulary dimension")
    V = logits.shape[-1]
    lead = logits.shape[:-1]
    if len(lead) == 0:
        return 1, 1, V, V, V
    if len(lead) == 1:
        return 1, lead[0], 0, logits.stride(0), V
    if len(lead) == 2:
        return lead[0], lead[1], logits.stride(0), logits.stride(1), V
    flat = logits.reshape(-1, V)
    return 1, flat.shape[0], 0, flat.stride(0), V


def logp_entropy(logits: torch.Tensor, index: torch.Tensor, temperature: float = 1.0,
                 compute_entropy: bool = True, round_scaled: bool = False):
    """Fused `selective_log_softmax(logits / T, index)` + `entropy_from_logits`.

    Returns fp32 (logp, entropy or None, lse) of shape index.shape.
    """
    _dev(logits, "logp_entropy")
    if logits.dim() > 3:
        logits = logits.reshape(-1, logits.shape[-1])
        index = index.reshape(-1)
    o, i, so, si, V = _rows_view(logits)
    idx = index.reshape(-1).to(torch.int64).contiguous()
    n = o * i
    if idx.numel() != n:
        raise ValueError("index shape must match logits.shape[:-1]")
    logp = torch.empty(n, device=logits.device, dtype=torch.float32)
    lse = torch.empty_like(logp)
    ent = torch.empty_like(logp) if compute_entropy else None
    flags = _lib.SWH_LOGP_ROUND_SCALED if round_scaled else 0
    with profiling.kernel("logp_entropy_fwd", n * V * logits.element_size() + n * 20):
        call("swh_logp_entropy_fwd", logits.data_ptr(), _dtype_code(logits, "logp_entropy"), o, i, so, si, V,
             idx.data_ptr(), float(temperature), flags, logp.data_ptr(), _p(ent), lse.data_ptr(), _stream())
    shp = index.shape
    return logp.view(shp), (ent.view(shp) if ent is not None else None), lse.view(shp)


def logp_backward(logits: torch.Tensor, index: torch.Tensor, lse: torch.Tensor, dlogp: torch.Tensor,
                  temperature: float = 1.0, round_scaled: bool = False, out: Optional[torch.Tensor] = None):
    """d logp / d logits (fused softmax-minus-onehot), written in the logits dtype."""
    _dev(logits, "logp_backward")
    if logits.dim() > 3:
        logits = logits.reshape(-1, logits.shape[-1])
    o, i, so, si, V = _rows_view(logits)
    if out is None:
        out = torch.empty(logits.shape, device=logits.device, dtype=logits.dtype)
    do, di, dso, dsi, _ = _rows_view(out.view(logits.shape))
    idx = index.reshape(-1).to(torch.int64).contiguous()
    g = dlogp.reshape(-1).to(torch.float32).contiguous()
    flags = _lib.SWH_LOGP_ROUND_SCALED if round_scaled else 0
    with profiling.kernel("logp_bwd", 2 * o * i * V * logits.element_size() + o * i * 16):
        call("swh_logp_bwd", logits.data_ptr(), _dtype_code(logits, "logp_backward"), o, i, so, si, V,
             idx.data_ptr(), float(temperature), flags, lse.reshape(-1).contiguous().data_ptr(), g.data_ptr(),
             out.data_ptr(), dso, dsi, _stream())
    return out


class _LogpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, index, temperature, round_scaled, compute_entropy):
        logp, ent, lse = logp_entropy(logits, index, temperature, compute_entropy, round_scaled)
        ctx.save_for_backward(logits, index, lse)
        ctx.temperature, ctx.round_scaled = temperature, round_scaled
        if ent is not None:
            ctx.mark_non_differentiable(ent)
        return logp, ent

    @staticmethod
    def backward(ctx, dlogp, dent):
        logits, index, lse = ctx.saved_tensors
        grad = logp_backward(logits, index, lse, dlogp, ctx.temperature, ctx.round_scaled)
        return grad, None, None, None, None


def logp_entropy_autograd(logits, index, temperature: float = 1.0, compute_entropy: bool = True,
                          round_scaled: bool = False):
    """Differentiable fp32 log-probs (grad to logits) + no-grad entropies."""
    return _LogpFn.apply(logits, index, float(temperature), bool(round_scaled), bool(compute_entropy))


def selective_log_softmax(logits: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """trl/trainer/utils.py:1430 — log_softmax(logits).gather(index); output in the
    logits dtype like the reference.  bf16/fp16 rows of V <= 1024 take the
    exact-order kernel (bit-equal to torch's log_softmax, as the reference's
    test_utils.py:540-558 asks); wider half-precision rows and fp32/fp64 go
    through the fused fp32 kernel (wider bf16 rows: see DESIGN.md §8)."""
    _dev(logits, "selective_log_softmax")
    if logits.dtype in (torch.bfloat16, torch.float16) and 0 < logits.shape[-1] <= 1024:
        lg = logits.reshape(-1, logits.shape[-1]) if logits.dim() > 3 else logits
        o, i, so, si, V = _rows_view(lg)
        idx = index.reshape(-1).to(torch.int64).contiguous()
        if idx.numel() != o * i:
            raise ValueError("index shape must match logits.shape[:-1]")
        out = torch.empty(o * i, device=logits.device, dtype=logits.dtype)
        call("swh_log_softmax_gather_exact", lg.data_ptr(), _dtype_code(lg, "selective_log_softmax"), o, i, so, si,
             V, idx.data_ptr(), out.data_ptr(), _stream())
        return out.view(index.shape)
    logp, _, _ = logp_entropy(logits, index, 1.0, False)
    return logp.to(logits.dtype)


def entropy_from_logits(logits: torch.Tensor, chunk_size: int = 1) -> torch.Tensor:
    """trl/trainer/utils.py:1465 — per-row Shannon entropy (nats), logits dtype."""
    del chunk_size  # the fused kernel never materialises the softmax
    dummy = torch.zeros(logits.shape[:-1], dtype=torch.int64, device=logits.device)
    _, ent, _ = logp_entropy(logits, dummy, 1.0, True)
    return ent.to(logits.dtype)


# ---------------------------------------------------------------------------
# trl/core.py
# ---------------------------------------------------------------------------

_ZERO_MASK_MSG = ("The sum of the mask is zero, which can happen when `mini_batch_size=1`;"
                  "try increase the `mini_batch_size` or `gradient_accumulation_steps`")


def masked_whiten_stats(values: torch.Tensor, mask: torch.Tensor, shift_mean: bool = True):
    """Hot-path form of trl/core.py:70-76 with no host sync: returns (whitened,
    stats f32[3] = masked mean, unbiased masked variance, mask sum).  A zero
    mask yields NaNs here; `masked_whiten` raises for it as the reference."""
    _dev(values, "masked_whiten")
    v = values.reshape(-1).to(torch.float32).contiguous()
    m = mask.reshape(-1).to(torch.int32).contiguous()
    out = torch.empty_like(v)
    stats = torch.empty(3, device=v.device, dtype=torch.float32)
    call("swh_masked_whiten", v.data_ptr(), m.data_ptr(), v.numel(), int(shift_mean), out.data_ptr(),
         stats.data_ptr(), None, _stream())
    return out.view(values.shape).to(values.dtype), stats


def masked_whiten(values: torch.Tensor, mask: torch.Tensor, shift_mean: bool = True) -> torch.Tensor:
    """trl/core.py:70-76: `(values - mean) * rsqrt(var + 1e-8)` (+ mean back when
    shift_mean=False) over the masked entries, one device kernel.  Raises
    ValueError on an all-zero mask like the reference's `masked_var`
    (core.py:57-62), which checks `mask.sum() == 0` on the host too."""
    out, stats = masked_whiten_stats(values, mask, shift_mean)
    if float(stats[2]) == 0:
        raise ValueError(_ZERO_MASK_MSG)
    return out


def masked_mean(values: torch.Tensor, mask: torch.Tensor, axis=None) -> torch.Tensor:
    """trl/core.py:43-48 (reduction is tiny; kept in torch on the device)."""
    if axis is not None:
        return (values * mask).sum(axis=axis) / mask.sum(axis=axis)
    return (values * mask).sum() / mask.sum()


def masked_var(values: torch.Tensor, mask: torch.Tensor, unbiased: bool = True) -> torch.Tensor:
    """trl/core.py:51-67: the masked variance about the masked mean,
    Bessel-corrected when `unbiased` (the whitening kernel's statistics;
    raises ValueError on an all-zero mask, core.py:57-62).  unbiased=False is
    the plain masked mean of the squared deviations, as the reference forms it
    before its correction: 0 for a single unmasked element, NaN for none."""
    _, stats = masked_whiten_stats(values, mask)
    if unbiased:
        if float(stats[2]) == 0:
            raise ValueError(_ZERO_MASK_MSG)
        return stats[1]
    return masked_mean((values.to(torch.float32) - stats[0]) ** 2, mask.to(torch.float32))


# ---------------------------------------------------------------------------
# GRPO rollout scoring
# ---------------------------------------------------------------------------

def completion_mask(completion_ids: torch.Tensor, eos_token_id, mask_truncated: bool = False):
    """grpo_trainer.py:1812-1831 → (mask int32 [B,C], lengths int32 [B], has_eos int32 [B])."""
    _dev(completion_ids, "completion_mask")
    ids = completion_ids.to(torch.int64).contiguous()
    B, Cn = ids.shape
    eos = [eos_token_id] if isinstance(eos_token_id, int) else list(eos_token_id)
    eos_t = torch.tensor(eos, dtype=torch.int32, device=ids.device)
    mask = torch.empty(B, Cn, dtype=torch.int32, device=ids.device)
    lengths = torch.empty(B, dtype=torch.int32, device=ids.device)
    has = torch.empty(B, dtype=torch.int32, device=ids.device)
    call("swh_completion_mask", ids.data_ptr(), B, Cn, eos_t.data_ptr(), len(eos), int(mask_truncated),
         mask.data_ptr(), lengths.data_ptr(), has.data_ptr(), _stream())
    return mask, lengths, has


def group_advantages(rewards_per_func: torch.Tensor, weights: torch.Tensor, num_generations: int,
                     scale_rewards: bool = True):
    """grpo_trainer.py:1914-1930 → (advantages, rewards, group_mean, group_std, zero_std)."""
    _dev(rewards_per_func, "group_advantages")
    rpf = rewards_per_func.to(torch.float32).contiguous()
    N, F = rpf.shape
    if N % num_generations:
        raise ValueError("number of completions must be a multiple of num_generations")
    w = weights.to(device=rpf.device, dtype=torch.float32).contiguous()
    adv = torch.empty(N, device=rpf.device, dtype=torch.float32)
    rew = torch.empty_like(adv)
    ng = N // num_generations
    gm = torch.empty(ng, device=rpf.device, dtype=torch.float32)
    gs = torch.empty_like(gm)
    zs = torch.empty(ng, device=rpf.device, dtype=torch.int32)
    call("swh_group_advantage", rpf.data_ptr(), w.data_ptr(), N, F, num_generations, int(scale_rewards),
         adv.data_ptr(), rew.data_ptr(), gm.data_ptr(), gs.data_ptr(), zs.data_ptr(), _stream())
    return adv, rew, gm, gs, zs.bool()


def grpo_loss_fwd_bwd(per_token_logps: torch.Tensor, advantages: torch.Tensor, completion_mask: torch.Tensor, *,
                      old_per_token_logps=None, ref_per_token_logps=None, entropy_mask=None, entropies=None,
                      row_scale=None, segments=None, num_segments: int = 1, beta: float = 0.0,
                      epsilon_low: float = 0.2, epsilon_high: float = 0.2, delta: Optional[float] = None,
                      loss_type: str = "bnpo", importance_sampling_level: str = "token",
                      max_completion_length: int = 256, need_grad: bool = True, segment_metrics: bool = False):
    """grpo_trainer.py:2058-2175 fused: returns (loss[1], dlogp or None, metric sums[8]); with
    segment_metrics, metric sums [1 + num_segments, 8]: the totals, then one row per segment."""
    _dev(per_token_logps, "grpo_loss")
    if loss_type not in _lib.LOSS_TYPES:
        raise ValueError(f"Unknown loss type: {loss_type}")
    if importance_sampling_level not in _lib.IS_LEVELS:
        raise ValueError(f"Unknown importance sampling level: {importance_sampling_level}. Possible values are "
                         "'token' and 'sequence'.")
    lp = per_token_logps.detach().to(torch.float32).contiguous()
    R, T = lp.shape
    dev = lp.device

    def f32(x):
        return None if x is None else x.detach().to(device=dev, dtype=torch.float32).contiguous()

    old, ref, ent = f32(old_per_token_logps), f32(ref_per_token_logps), f32(entropies)
    if beta != 0.0 and ref is None:
        raise ValueError("beta != 0 needs ref_per_token_logps")
    adv = f32(advantages).reshape(-1)
    mask = completion_mask.to(device=dev, dtype=torch.int32).contiguous()
    em = None if entropy_mask is None else entropy_mask.to(device=dev, dtype=torch.uint8).contiguous()
    rs = f32(row_scale)
    seg = None if segments is None else segments.to(device=dev, dtype=torch.int32).contiguous()
    p = GRPOLossParams(float(beta), float(epsilon_low), float(epsilon_high), float(delta) if delta else 0.0,
                       _lib.LOSS_TYPES[loss_type], _lib.IS_LEVELS[importance_sampling_level],
                       int(max_completion_length), int(num_segments))
    loss = torch.empty(1, device=dev, dtype=torch.float32)
    dlogp = torch.empty_like(lp) if need_grad else None
    metrics = torch.empty((1 + num_segments) if segment_metrics else 1, 8, device=dev, dtype=torch.float32)
    ws = torch.empty(_lib.load().swh_grpo_loss_workspace_bytes(R) // 4 + 1, device=dev, dtype=torch.float32)
    call("swh_grpo_loss_fwd_bwd", lp.data_ptr(), _p(old), _p(ref), adv.data_ptr(), mask.data_ptr(), _p(em), _p(ent),
         _p(rs), _p(seg), R, T, p, loss.data_ptr(), _p(dlogp), metrics.data_ptr(),
         metrics[1:].data_ptr() if segment_metrics else None, ws.data_ptr(), _stream())
    return loss, dlogp, (metrics if segment_metrics else metrics[0])


class _GRPOLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, per_token_logps, kwargs):
        loss, dlogp, metrics = grpo_loss_fwd_bwd(per_token_logps, **kwargs)
        ctx.save_for_backward(dlogp)
        ctx.mark_non_differentiable(metrics)
        return loss[0], metrics

    @staticmethod
    def backward(ctx, gloss, gmetrics):
        (dlogp,) = ctx.saved_tensors
        return dlogp * gloss, None


def grpo_loss(per_token_logps, advantages, completion_mask, **kw):
    """Differentiable GRPO loss (the gradient comes from the fused kernel)."""
    kw = dict(kw, advantages=advantages, completion_mask=completion_mask)
    return _GRPOLossFn.apply(per_token_logps, kw)


# ---------------------------------------------------------------------------
# PPO (ppo_trainer.py)
# ---------------------------------------------------------------------------

def gae(rewards: torch.Tensor, values: torch.Tensor, gamma: float, lam: float):
    """ppo_trainer.py:523-533 → (advantages, returns) fp32."""
    _dev(rewards, "gae")
    r = rewards.to(torch.float32).contiguous()
    v = values.to(torch.float32).contiguous()
    B, T = r.shape
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    call("swh_gae_scan", r.data_ptr(), v.data_ptr(), B, T, float(gamma), float(lam), adv.data_ptr(), ret.data_ptr(),
         _stream())
    return adv, ret


def ppo_loss_fwd_bwd(new_logprobs, mb_logprobs, mb_advantage, vpred, mb_values, mb_return, padding_mask,
                     padding_mask_p1, cliprange: float, cliprange_value: float, vf_coef: float,
                     need_grad: bool = True):
    """ppo_trainer.py:557-605 → (loss[1], dnew_logp, dvpred, stats[8])."""
    _dev(new_logprobs, "ppo_loss")
    f = lambda x: x.detach().to(torch.float32).contiguous()  # noqa: E731
    nl, ol, a, vp, ov, rt = map(f, (new_logprobs, mb_logprobs, mb_advantage, vpred, mb_values, mb_return))
    if a.dim() == 1:
        a = a.unsqueeze(1).expand_as(nl).contiguous()
    pm = padding_mask.to(torch.uint8).contiguous()
    pm1 = padding_mask_p1.to(torch.uint8).contiguous()
    B, T = nl.shape
    loss = torch.empty(1, device=nl.device, dtype=torch.float32)
    dnl = torch.empty_like(nl) if need_grad else None
    dvp = torch.empty_like(nl) if need_grad else None
    stats = torch.empty(8, device=nl.device, dtype=torch.float32)
    call("swh_ppo_loss_fwd_bwd", nl.data_ptr(), ol.data_ptr(), a.data_ptr(), vp.data_ptr(), ov.data_ptr(),
         rt.data_ptr(), pm.data_ptr(), pm1.data_ptr(), B, T, float(cliprange), float(cliprange_value),
         float(vf_coef), loss.data_ptr(), _p(dnl), _p(dvp), stats.data_ptr(), None, _stream())
    return loss, dnl, dvp, stats


def ppo_truncate(responses: torch.Tensor, stop_token_id, pad_token_id: int):
    """utils.py:1036-1056 truncate_response + :877-897 first_true_indices in one
    launch: (postprocessed responses int64 [B, T], sequence_lengths int64 [B])."""
    _dev(responses, "ppo_truncate")
    r = responses.to(torch.int64).contiguous()
    B, T = r.shape
    post = torch.empty_like(r)
    seq = torch.empty(B, dtype=torch.int64, device=r.device)
    call("swh_ppo_truncate", r.data_ptr(), B, T, -1 if stop_token_id is None else int(stop_token_id), int(pad_token_id),
         post.data_ptr(), seq.data_ptr(), _stream())
    return post, seq


def ppo_rewards(post: torch.Tensor, sequence_lengths: torch.Tensor, logprobs: torch.Tensor,
                ref_logprobs: torch.Tensor, values: torch.Tensor, scores: torch.Tensor, *, eos_token_id,
                missing_eos_penalty, kl_coef: float, kl_estimator: str = "k1") -> dict:
    """ppo_trainer.py:490-516 in one launch: masks, INVALID_LOGPROB fill, value
    masking, missing-EOS penalty, KL (k1 / k3) and KL-shaped rewards with the
    score scattered at min(seq_len + 1, T - 1).  values / scores are the bf16
    outputs of the score heads, bf16 or fp32 (reference-precision mode), modified
    like the reference's tensors of that dtype."""
    _dev(post, "ppo_rewards")
    if kl_estimator not in ("k1", "k3"):
        raise ValueError(f"kl_estimator must be 'k1' or 'k3', got {kl_estimator!r}")
    if values.dtype != scores.dtype or values.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("ppo_rewards: values and scores are the score-head outputs (both bf16 or both fp32)")
    B, T = post.shape
    lp = logprobs.to(torch.float32).contiguous().clone()
    rf = ref_logprobs.to(torch.float32).contiguous().clone()
    v = values.contiguous().clone()
    s = scores.contiguous().clone()
    pm = torch.empty(B, T, dtype=torch.bool, device=post.device)
    pm1 = torch.empty_like(pm)
    kl, nsr, rew = torch.empty_like(lp), torch.empty_like(lp), torch.empty_like(lp)
    call("swh_ppo_rewards", post.contiguous().data_ptr(), sequence_lengths.to(torch.int64).contiguous().data_ptr(), B,
         T, -1 if eos_token_id is None else int(eos_token_id),
         0.0 if missing_eos_penalty is None else float(missing_eos_penalty), int(missing_eos_penalty is not None),
         float(kl_coef), int(kl_estimator == "k3"), lp.data_ptr(), rf.data_ptr(), v.data_ptr(), s.data_ptr(),
         _dtype_code(v, "ppo_rewards"), pm.data_ptr(), pm1.data_ptr(), kl.data_ptr(), nsr.data_ptr(), rew.data_ptr(), _stream())
    return {"logprobs": lp, "ref_logprobs": rf, "values": v, "scores": s, "padding_mask": pm,
            "padding_mask_p1": pm1, "kl": kl, "non_score_reward": nsr, "rewards": rew}


def value_head(hidden: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None):
    """modeling_value_head.py:50-59 (eval) → fp32 [*hidden.shape[:-1]]."""
    _dev(hidden, "value_head")
    H = hidden.shape[-1]
    h2 = hidden.reshape(-1, H)
    if h2.stride(-1) != 1:
        h2 = h2.contiguous()
    w = weight.reshape(-1).to(torch.float32).contiguous()
    b = None if bias is None else bias.reshape(-1).to(torch.float32).contiguous()
    out = torch.empty(h2.shape[0], device=hidden.device, dtype=torch.float32)
    call("swh_value_head_fwd", h2.data_ptr(), _dtype_code(h2, "value_head"), h2.shape[0], H, h2.stride(0),
         w.data_ptr(), _p(b), out.data_ptr(), _stream())
    return out.view(hidden.shape[:-1])


# ---------------------------------------------------------------------------
# sampling
# ---------------------------------------------------------------------------

def make_sample_params(temperature=1.0, top_p=1.0, top_k=None, min_p=None, repetition_penalty=1.0,
                       greedy=False, min_new_tokens=0, pad_token_id=-1, eos_token_ids=()) -> SampleParams:
    eos = list(eos_token_ids)[:4]
    p = SampleParams()
    p.temperature = float(temperature)
    p.top_p = float(top_p if top_p is not None else 1.0)
    p.min_p = float(min_p) if min_p is not None else 0.0
    p.repetition_penalty = float(repetition_penalty if repetition_penalty is not None else 1.0)
    p.top_k = int(top_k or 0)
    p.greedy = int(bool(greedy))
    p.min_new_tokens = int(min_new_tokens or 0)
    p.pad_token_id = int(pad_token_id if pad_token_id is not None else -1)
    p.n_eos = len(eos)
    for i, e in enumerate(eos):
        p.eos_ids[i] = int(e)
    return p


def sample_step(logits: torch.Tensor, params: SampleParams, rng: torch.Tensor, step: torch.Tensor,
                finished: torch.Tensor, out_tokens: torch.Tensor, cur_tokens: Optional[torch.Tensor] = None,
                seen: Optional[torch.Tensor] = None, out_logp: Optional[torch.Tensor] = None,
                scores_out: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None):
    """One device sampling step (all state on device; graph-capturable)."""
    _dev(logits, "sample_step")
    B, V = logits.shape
    if logits.stride(1) != 1:
        raise ValueError("logits rows must be contiguous")
    if workspace is None:
        workspace = torch.empty(_lib.load().swh_sample_workspace_bytes(B, V), dtype=torch.uint8,
                                device=logits.device)
    call("swh_sample_step", logits.data_ptr(), _dtype_code(logits, "sample_step"), B, V, logits.stride(0), params,
         rng.data_ptr(), step.data_ptr(), finished.data_ptr(), _p(seen), out_tokens.data_ptr(), out_tokens.stride(0),
         _p(cur_tokens), _p(out_logp), _p(scores_out), workspace.data_ptr(), _stream())


def seen_init(ids: torch.Tensor, mask: Optional[torch.Tensor], V: int, seen: torch.Tensor):
    B, L = ids.shape
    m = None if mask is None else mask.to(torch.int32).contiguous()
    call("swh_seen_init", ids.contiguous().data_ptr(), _p(m), B, L, V, seen.data_ptr(), _stream())


def step_advance(step: torch.Tensor):
    call("swh_step_advance", step.data_ptr(), _stream())
