"""CPU restatement of one reference GRPO optimizer step — TEST ORACLE and the
timed CPU baseline (`bench.py` cpu_baseline, kind "port").

Follows trl/trainer/grpo_trainer.py:
  _generate_and_score_completions :1500-2003 (generate :1793-1810, EOS mask
  :1812-1831, rewards :1446-1498, advantages :1914-1930),
  _prepare_inputs :1411-1444 (shuffle + split into steps_per_generation),
  _get_per_token_logps_and_entropies :1205-1272, _compute_loss :2058-2175,
and the transformers Trainer around them (loss / GA, clip_grad_norm_(1.0),
AdamW step).  Generation and the model are the installed transformers
(third-party: allowed as the oracle for third-party ops); the
reference itself is never imported.
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import torch

from . import trl_ref


def hf_qwen2_from_config(cfg: dict, seed: int = 0, dtype=torch.float32):
    """Random-init transformers Qwen2ForCausalLM of the given architecture (no hub)."""
    from transformers import Qwen2Config, Qwen2ForCausalLM
    torch.manual_seed(seed)
    hc = Qwen2Config(vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden_size"],
                     intermediate_size=cfg["intermediate_size"], num_hidden_layers=cfg["num_hidden_layers"],
                     num_attention_heads=cfg["num_attention_heads"], num_key_value_heads=cfg["num_key_value_heads"],
                     rope_theta=cfg["rope_theta"], rms_norm_eps=cfg["rms_norm_eps"],
                     tie_word_embeddings=cfg["tie_word_embeddings"], max_position_embeddings=cfg.get(
                         "max_position_embeddings", 32768))
    hc._attn_implementation = "sdpa"
    m = Qwen2ForCausalLM(hc).to(dtype)
    m.eval()  # dropout-free (Qwen2 has none); generate() and the loss forward agree
    return m


def hf_gpt2_from_config(cfg: dict, seed: int = 0, dtype=torch.float32):
    """Random-init transformers GPT2LMHeadModel (BASELINE.json config 1), dropout
    off (`disable_dropout=True` in GRPOConfig terms: the engine has none)."""
    from transformers import GPT2Config, GPT2LMHeadModel
    torch.manual_seed(seed)
    H = cfg["hidden_size"]
    hc = GPT2Config(vocab_size=cfg["vocab_size"], n_embd=H, n_layer=cfg["num_hidden_layers"],
                    n_head=cfg["num_attention_heads"], n_positions=cfg["max_position_embeddings"],
                    n_inner=None if cfg["intermediate_size"] == 4 * H else cfg["intermediate_size"],
                    layer_norm_epsilon=cfg["rms_norm_eps"], resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0,
                    bos_token_id=None, eos_token_id=None)
    hc._attn_implementation = "sdpa"
    m = GPT2LMHeadModel(hc).to(dtype)
    m.eval()
    return m


def hf_from_config(cfg: dict, seed: int = 0, dtype=torch.float32):
    """The transformers model of cfg["model_type"] (GPT-2, or Qwen2 / Llama-style)."""
    if cfg.get("model_type") == "gpt2":
        return hf_gpt2_from_config(cfg, seed, dtype)
    return hf_qwen2_from_config(cfg, seed, dtype)


def generate(model, prompt_ids, prompt_mask, C: int, *, do_sample=True, temperature=1.0, top_p=1.0, top_k=None,
             min_p=None, repetition_penalty=1.0, min_new_tokens=0, pad_token_id=0, eos_token_id=None):
    """transformers generate with the GenerationConfig of grpo_trainer.py:995-1014."""
    from transformers import GenerationConfig
    gc = GenerationConfig(max_new_tokens=C, do_sample=do_sample, pad_token_id=pad_token_id,
                          eos_token_id=eos_token_id, bos_token_id=None, temperature=temperature, top_p=top_p,
                          top_k=top_k, min_p=min_p, repetition_penalty=repetition_penalty,
                          min_new_tokens=min_new_tokens, cache_implementation=None)
    with torch.no_grad():
        out = model.generate(input_ids=prompt_ids, attention_mask=prompt_mask, generation_config=gc)
    comp = out[:, prompt_ids.shape[1]:]
    if comp.shape[1] < C:  # generation stopped early: pad like a fixed-width buffer
        comp = torch.cat([comp, torch.full((comp.shape[0], C - comp.shape[1]), pad_token_id, dtype=comp.dtype)], 1)
    return comp


def per_token_logps(model, prompt_ids, prompt_mask, completion_ids, completion_mask, temperature=1.0,
                    compute_entropy=True):
    """grpo_trainer.py:1205-1272 (one batch)."""
    ids = torch.cat([prompt_ids, completion_ids], 1)
    am = torch.cat([prompt_mask, completion_mask], 1)
    C = completion_ids.shape[1]
    logits = model(input_ids=ids, attention_mask=am, logits_to_keep=C + 1).logits
    logits = logits[:, :-1][:, -C:] / temperature
    lp = trl_ref.selective_log_softmax(logits, completion_ids)
    ent = None
    if compute_entropy:
        with torch.no_grad():
            ent = trl_ref.entropy_from_logits(logits)
    return lp, ent


def grpo_step(model, optimizer, prompt_ids, prompt_mask, reward_fn: Callable, *, num_generations: int, C: int,
              per_device_train_batch_size: int, gradient_accumulation_steps: int, temperature=1.0,
              eos_token_id=None, pad_token_id=0, beta=0.0, epsilon=0.2, epsilon_high=None, loss_type="bnpo",
              importance_sampling_level="token", scale_rewards=True, max_grad_norm=1.0, do_sample=True,
              min_new_tokens=0, perm: Optional[torch.Tensor] = None, completion_ids=None, timings=None,
              ref_model=None, capture: bool = False):
    """One optimizer step; returns (mean loss, dict of intermediates).

    ref_model (beta != 0): the frozen reference scored on the whole batch
    before the shuffle (grpo_trainer.py:1871-1899).  capture=True adds the
    per-token log-probs of every micro-batch ("logps", permuted row order),
    the pre-clip gradients ("grads", name -> tensor) and the per-micro losses."""
    t0 = time.perf_counter()
    if completion_ids is None:
        completion_ids = generate(model, prompt_ids, prompt_mask, C, do_sample=do_sample, temperature=temperature,
                                  min_new_tokens=min_new_tokens, pad_token_id=pad_token_id,
                                  eos_token_id=eos_token_id)
    t1 = time.perf_counter()
    mask, lengths, _ = trl_ref.completion_mask_from_eos(completion_ids, eos_token_id if eos_token_id is not None
                                                        else -1)
    rewards = torch.tensor([float(x) for x in reward_fn(completion_ids, mask)], dtype=torch.float32).view(-1, 1)
    adv, _, _, _, _ = trl_ref.group_advantages(rewards, torch.ones(1), num_generations, scale_rewards)
    B = completion_ids.shape[0]
    ref_lp = None
    if beta != 0.0:
        if ref_model is None:
            raise ValueError("beta != 0 needs ref_model")
        with torch.no_grad():
            ref_lp, _ = per_token_logps(ref_model, prompt_ids, prompt_mask, completion_ids, mask, temperature,
                                        compute_entropy=False)
    perm = torch.arange(B) if perm is None else perm
    data = {"p": prompt_ids[perm], "pm": prompt_mask[perm], "c": completion_ids[perm], "cm": mask[perm],
            "a": adv[perm], "r": None if ref_lp is None else ref_lp[perm]}
    spg = B // per_device_train_batch_size
    GA = gradient_accumulation_steps
    losses = []
    grads_of_logps = []
    for j in range(min(spg, GA)):
        sl = slice(j * per_device_train_batch_size, (j + 1) * per_device_train_batch_size)
        lp, ent = per_token_logps(model, data["p"][sl], data["pm"][sl], data["c"][sl], data["cm"][sl], temperature)
        lp.retain_grad()
        loss, _ = trl_ref.grpo_loss(lp, data["a"][sl], data["cm"][sl],
                                    ref_per_token_logps=None if data["r"] is None else data["r"][sl],
                                    entropies=ent, beta=beta,
                                    epsilon_low=epsilon, epsilon_high=epsilon_high or epsilon, loss_type=loss_type,
                                    importance_sampling_level=importance_sampling_level, max_completion_length=C)
        (loss / GA).backward()
        losses.append(float(loss.detach()) / GA)
        grads_of_logps.append(lp.detach())
    grads = ({n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
             if capture else None)
    total = torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)
    optimizer.step()
    optimizer.zero_grad()
    t2 = time.perf_counter()
    if timings is not None:
        timings["generate_s"] = t1 - t0
        timings["update_s"] = t2 - t1
    out = {"completion_ids": completion_ids, "completion_mask": mask, "advantages": adv, "rewards": rewards,
           "grad_norm": float(total), "perm": perm}
    if capture:
        out.update(logps=torch.cat(grads_of_logps), grads=grads, losses=losses)
    return sum(losses), out
