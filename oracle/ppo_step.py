"""CPU restatement of the reference PPO rollout scoring and update — TEST ORACLE.

Follows trl/trainer/ppo_trainer.py:
  rollout scoring :389-535 (ref log-probs, truncation, value / reward-model
  scores through utils.py:900-979 `get_reward` / `forward`, missing-EOS
  penalty, INVALID_LOGPROB masking, KL-shaped rewards, reward whitening, GAE,
  advantage whitening),
  micro-batch loss :557-605 (clipped value loss, clipped PG loss, stats),
  update schedule :537-617 (epochs x mini-batches x accumulate(GA), loss / GA
  as accelerate's backward, one AdamW step per mini-batch, no clipping).
Models are the installed transformers Qwen2ForCausalLM /
Qwen2ForSequenceClassification (third-party: allowed as the oracle for
third-party ops); the reference itself is never imported.
Generation is not restated: sampled responses come from the engine under test
and their generation log-probs are checked against `generation_logprobs`.
"""
from __future__ import annotations

import torch

from . import trl_ref

INVALID_LOGPROB = 1.0  # ppo_trainer.py:81


def forward(model, query_responses: torch.Tensor, pad_token_id: int):
    """utils.py:950-979."""
    attention_mask = query_responses != pad_token_id
    position_ids = attention_mask.cumsum(1) - attention_mask.long()
    input_ids = torch.masked_fill(query_responses, ~attention_mask, 0)
    return model(input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids, return_dict=True,
                 output_hidden_states=True)


def get_reward(model, query_responses: torch.Tensor, pad_token_id: int, context_length: int):
    """utils.py:900-947: score head over the backbone's last hidden states, and
    the score at the last non-pad response token."""
    attention_mask = query_responses != pad_token_id
    position_ids = attention_mask.cumsum(1) - attention_mask.long()
    input_ids = torch.masked_fill(query_responses, ~attention_mask, 0)
    backbone = getattr(model, model.base_model_prefix)
    out = backbone(input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids, return_dict=True,
                   output_hidden_states=True, use_cache=False)
    reward_logits = model.score(out.hidden_states[-1])
    seq = trl_ref.first_true_indices(query_responses[:, context_length:] == pad_token_id) - 1 + context_length
    return reward_logits, reward_logits[torch.arange(reward_logits.size(0)), seq].squeeze(-1), seq


def generation_logprobs(policy, queries, responses, pad_token_id: int, temperature: float):
    """What `selective_log_softmax(logitss, response)` sees at :391: the fp32
    processed scores of generate (logits / (T + 1e-7)) at the drawn tokens —
    recomputed here by a full forward over query + response."""
    P = queries.shape[1]
    qr = torch.cat([queries, responses], 1)
    logits = forward(policy, qr, pad_token_id).logits[:, P - 1:-1].float() / (temperature + 1e-7)
    return trl_ref.selective_log_softmax(logits, responses)


def rollout_arith(logprobs, ref_logprobs, values, scores, postprocessed_responses, *, pad_token_id: int,
                  eos_token_id, kl_coef: float, kl_estimator: str, whiten_rewards: bool, missing_eos_penalty,
                  gamma: float, lam: float) -> dict:
    """ppo_trainer.py:480-535 on given log-probs / values / scores."""
    T = postprocessed_responses.shape[1]
    sequence_lengths = trl_ref.first_true_indices(postprocessed_responses == pad_token_id) - 1
    scores = scores.clone()
    if eos_token_id is not None:
        contain_eos = torch.any(postprocessed_responses == eos_token_id, dim=-1)
    else:
        contain_eos = torch.zeros(postprocessed_responses.shape[0], dtype=torch.bool)
    if missing_eos_penalty is not None:
        scores[~contain_eos] -= missing_eos_penalty
    idx = torch.arange(T).repeat(postprocessed_responses.shape[0], 1)
    padding_mask = idx > sequence_lengths.unsqueeze(1)
    logprobs = torch.masked_fill(logprobs, padding_mask, INVALID_LOGPROB)
    ref_logprobs = torch.masked_fill(ref_logprobs, padding_mask, INVALID_LOGPROB)
    padding_mask_p1 = idx > (sequence_lengths + 1).unsqueeze(1)
    values = torch.masked_fill(values, padding_mask_p1, 0)
    rewards, kl, non_score = trl_ref.ppo_rewards(logprobs, ref_logprobs, scores, sequence_lengths, kl_coef,
                                                 kl_estimator)
    if whiten_rewards:
        rewards = trl_ref.masked_whiten(rewards, ~padding_mask_p1, shift_mean=False)
        rewards = torch.masked_fill(rewards, padding_mask_p1, 0)
    adv, returns = trl_ref.gae(rewards, values.float(), gamma, lam)
    adv = trl_ref.masked_whiten(adv, ~padding_mask)
    adv = torch.masked_fill(adv, padding_mask, 0)
    return {"logprobs": logprobs, "ref_logprobs": ref_logprobs, "values": values, "scores": scores,
            "rewards": rewards, "advantages": adv, "returns": returns, "kl": kl, "non_score_reward": non_score,
            "padding_mask": padding_mask, "padding_mask_p1": padding_mask_p1, "sequence_lengths": sequence_lengths}


@torch.no_grad()
def rollout_scores(policy, ref_policy, value_model, reward_model, queries, responses, logprobs, *, pad_token_id,
                   stop_token_id, eos_token_id, temperature, kl_coef, kl_estimator="k1", whiten_rewards=False,
                   missing_eos_penalty=None, gamma=1.0, lam=0.95) -> dict:
    """ppo_trainer.py:389-535 for one rollout batch."""
    P = queries.shape[1]
    qr = torch.cat([queries, responses], 1)
    ref_logits = forward(ref_policy, qr, pad_token_id).logits[:, P - 1:-1]
    ref_logits = ref_logits / (temperature + 1e-7)
    ref_logprobs = trl_ref.selective_log_softmax(ref_logits, responses)
    post = responses
    if stop_token_id is not None:
        post = trl_ref.truncate_response(stop_token_id, pad_token_id, responses)
    full_value, _, _ = get_reward(value_model, qr, pad_token_id, P)
    values = full_value[:, P - 1:-1].squeeze(-1)
    _, score, _ = get_reward(reward_model, torch.cat([queries, post], 1), pad_token_id, P)
    out = rollout_arith(logprobs, ref_logprobs, values, score, post, pad_token_id=pad_token_id,
                        eos_token_id=eos_token_id, kl_coef=kl_coef, kl_estimator=kl_estimator,
                        whiten_rewards=whiten_rewards, missing_eos_penalty=missing_eos_penalty, gamma=gamma,
                        lam=lam)
    out.update(query_responses=qr, responses=responses, postprocessed_responses=post)
    return out


def micro_batch_loss(policy, value_model, ro: dict, inds, *, context_length: int, pad_token_id: int,
                     temperature: float, cliprange: float, cliprange_value: float, vf_coef: float,
                     token_terms: bool = False):
    """ppo_trainer.py:557-605 for one micro-batch (differentiable loss, stats;
    token_terms: stats["tokens"] = per-token terms of each statistic)."""
    qr = ro["query_responses"][inds]
    out = forward(policy, qr, pad_token_id)
    logits = out.logits[:, context_length - 1:-1] / (temperature + 1e-7)
    new_logprobs = trl_ref.selective_log_softmax(logits, ro["responses"][inds])
    new_logprobs = torch.masked_fill(new_logprobs, ro["padding_mask"][inds], INVALID_LOGPROB)
    full_value, _, _ = get_reward(value_model, qr, pad_token_id, context_length)
    vpred = full_value[:, context_length - 1:-1].squeeze(-1)
    vpred = torch.masked_fill(vpred, ro["padding_mask_p1"][inds], 0)
    loss, pg_loss, vf_loss, stats = trl_ref.ppo_losses(
        new_logprobs, ro["logprobs"][inds], ro["advantages"][inds], vpred, ro["values"][inds],
        ro["returns"][inds], ro["padding_mask"][inds], ro["padding_mask_p1"][inds], cliprange, cliprange_value,
        vf_coef, token_terms=token_terms)
    with torch.no_grad():
        prob = torch.softmax(logits.float(), -1)
        entropy = torch.logsumexp(logits.float(), -1) - (prob * logits.float()).sum(-1)
    stats = dict(stats, pg_loss=float(pg_loss.detach()), vf_loss=float(vf_loss.detach()),
                     entropy=float(entropy.mean()))
    if token_terms:
        stats["tokens"]["entropy"] = entropy.flatten()
    return loss, stats


def mini_batch_backward(policy, value_model, ro: dict, mini, *, per_device_train_batch_size: int,
                        gradient_accumulation_steps: int, **loss_kw):
    """ppo_trainer.py:551-605 for one mini-batch: its GA micro-batches, each
    loss / GA back-propagated into the accumulated gradients; returns the
    micro-batches' stats."""
    stats = []
    for u0 in range(0, len(mini), per_device_train_batch_size):
        loss, st = micro_batch_loss(policy, value_model, ro, mini[u0:u0 + per_device_train_batch_size], **loss_kw)
        (loss / gradient_accumulation_steps).backward()
        stats.append(st)
    return stats


def accelerate_sync(step: int, gradient_accumulation_steps: int, end_of_dataloader: bool):
    """accelerate 1.x `Accelerator._do_sync` (third-party, pinned accelerate >= 1.4 by
    setup.cfg:44-47; restated from the installed 1.14.0): entering
    `accelerator.accumulate(model)` at the last batch of a data epoch
    (DataLoaderShard flags end_of_dataloader one batch ahead) resets the counter and
    syncs; otherwise the counter increments and syncs every GA-th micro-batch.
    Returns (new step, sync)."""
    if end_of_dataloader:
        return 0, True
    step += 1
    return step, step % gradient_accumulation_steps == 0


def ppo_update(policy, value_model, optimizer, ro: dict, permutations, *, local_mini_batch_size: int,
               per_device_train_batch_size: int, gradient_accumulation_steps: int, on_step=None,
               accum_step: int = 0, end_of_dataloader: bool = False, **loss_kw):
    """ppo_trainer.py:537-617: for each epoch's permutation, mini-batches of
    micro-batches, each inside `accelerator.accumulate(model)`: loss / GA
    back-propagated (accelerator.backward), then optimizer.step() and
    zero_grad(), which the AcceleratedOptimizer performs only on a sync
    (accelerate_sync).  on_step(): called before each performed optimizer step
    (the accumulated gradients).  Returns (per-micro stats, accumulation counter)."""
    n = ro["responses"].shape[0]
    all_stats = []
    for perm in permutations:
        perm = torch.as_tensor(perm)
        for m0 in range(0, n, local_mini_batch_size):
            mini = perm[m0:m0 + local_mini_batch_size]
            for u0 in range(0, len(mini), per_device_train_batch_size):
                accum_step, sync = accelerate_sync(accum_step, gradient_accumulation_steps, end_of_dataloader)
                loss, st = micro_batch_loss(policy, value_model, ro, mini[u0:u0 + per_device_train_batch_size],
                                            **loss_kw)
                (loss / gradient_accumulation_steps).backward()
                all_stats.append(st)
                if sync:
                    if on_step is not None:
                        on_step()
                    optimizer.step()
                    optimizer.zero_grad()
    return all_stats, accum_step
