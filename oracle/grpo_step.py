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


def hf_llama_from_config(cfg: dict, seed: int = 0, dtype=torch.float32):
    """Random-init transformers LlamaForCausalLM of the given architecture (the Llama-3
    family of BASELINE.json config 5: no q/k/v bias, untied head)."""
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(seed)
    hc = LlamaConfig(vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden_size"],
                     intermediate_size=cfg["intermediate_size"], num_hidden_layers=cfg["num_hidden_layers"],
                     num_attention_heads=cfg["num_attention_heads"], num_key_value_heads=cfg["num_key_value_heads"],
                     head_dim=cfg["head_dim"], rope_theta=cfg["rope_theta"], rms_norm_eps=cfg["rms_norm_eps"],
                     tie_word_embeddings=cfg["tie_word_embeddings"], attention_bias=cfg["attention_bias"],
                     max_position_embeddings=cfg.get("max_position_embeddings", 8192))
    hc._attn_implementation = "sdpa"
    m = LlamaForCausalLM(hc).to(dtype)
    m.eval()
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
    if cfg.get("model_type") == "llama":
        return hf_llama_from_config(cfg, seed, dtype)
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
    """grpo_trainer.py:1205-1272 (one batch), on the model's device."""
    dev = next(model.parameters()).device
    ids = torch.cat([prompt_ids, completion_ids], 1).to(dev)
    am = torch.cat([prompt_mask, completion_mask], 1).to(dev)
    completion_ids = completion_ids.to(dev)
    C = completion_ids.shape[1]
    logits = model(input_ids=ids, attention_mask=am, logits_to_keep=C + 1).logits
    logits = logits[:, :-1][:, -C:] / temperature
    lp = trl_ref.selective_log_softmax(logits, completion_ids)
    ent = None
    if compute_entropy:
        with torch.no_grad():
            ent = trl_ref.entropy_from_logits(logits)
    return lp, ent


def _rewards_per_func(reward_fn, ids, mask, reward_weights):
    """grpo_trainer.py:1446-1498 + :1918: one column per reward function (a function's
    None becomes NaN, :1485-1487), the weights of GRPOConfig.reward_weights (ones by
    default).  `reward_fn` is one callable (ids, mask) -> list of floats, or a list of
    them (several reward functions)."""
    fns = list(reward_fn) if isinstance(reward_fn, (list, tuple)) else [reward_fn]
    cols = [torch.tensor([float("nan") if x is None else float(x) for x in f(ids, mask)], dtype=torch.float32)
            for f in fns]
    w = torch.ones(len(fns)) if reward_weights is None else torch.tensor(reward_weights, dtype=torch.float32)
    if w.numel() != len(fns):
        raise ValueError("Number of reward weights must match number of reward functions")
    return torch.stack(cols, 1), w


def score_generation(model, g: dict, reward_fn: Callable, *, num_generations: int, temperature=1.0,
                     eos_token_id=None, scale_rewards=True, beta=0.0, ref_model=None, need_old: bool = False,
                     per_device_train_batch_size: Optional[int] = None, mask_truncated_completions: bool = False,
                     reward_weights=None):
    """The scoring half of _generate_and_score_completions (grpo_trainer.py:1812-1938) on a
    generation batch g = {prompt_ids, prompt_mask, completion_ids}: EOS mask, rewards,
    group advantages, the old-policy log-probs when the steps are not aligned with the
    generations (:1854-1869) and the frozen reference's (:1871-1899), both scored before
    the shuffle in micro-batches of per_device_train_batch_size rows (the reference's
    batch_size).

    Data parallel: g["world_completion_ids"] (every rank's completions in rank order, the
    accelerate gather of :1497) and g["rank"]: rewards and advantages are formed on the
    global batch and this rank keeps its slice (:1914-1938).

    mask_truncated_completions (:1829-1831): rows without EOS get an all-zero mask for
    scoring and training; the lengths (:1826) and the reward functions' completion ids
    (:1821-1823) are taken before that zeroing."""
    eos = eos_token_id if eos_token_id is not None else -1
    cids = g["completion_ids"]
    B = cids.shape[0]
    mask, lengths, _ = trl_ref.completion_mask_from_eos(cids, eos, mask_truncated_completions)
    all_ids = g.get("world_completion_ids")
    if all_ids is None:
        all_ids, r0 = cids, 0
    else:
        r0 = int(g["rank"]) * B
        assert torch.equal(all_ids[r0:r0 + B], cids)
    all_mask, _, _ = trl_ref.completion_mask_from_eos(all_ids, eos)
    rpf, w = _rewards_per_func(reward_fn, all_ids, all_mask, reward_weights)
    adv, rewards, _, _, _ = trl_ref.group_advantages(rpf, w, num_generations, scale_rewards)
    adv = adv[r0:r0 + B]
    bs = per_device_train_batch_size or B

    def scored(m):
        parts = []
        with torch.no_grad():
            for r0 in range(0, B, bs):
                sl = slice(r0, r0 + bs)
                lp, _ = per_token_logps(m, g["prompt_ids"][sl], g["prompt_mask"][sl], cids[sl], mask[sl],
                                        temperature, compute_entropy=False)
                parts.append(lp)
        return torch.cat(parts)
    old = scored(model).cpu() if need_old else None
    ref = None
    if beta != 0.0:
        if ref_model is None:
            raise ValueError("beta != 0 needs ref_model")
        ref = scored(ref_model).cpu()
    return {"p": g["prompt_ids"], "pm": g["prompt_mask"], "c": cids, "cm": mask, "a": adv, "old": old, "ref": ref,
            "rewards": rewards.view(-1, 1), "rewards_per_func": rpf, "lengths": lengths}


def grpo_train(model, optimizer, generations, reward_fn: Callable, *, num_generations: int, C: int,
               per_device_train_batch_size: int, gradient_accumulation_steps: int, n_steps: int,
               steps_per_generation: Optional[int] = None, num_iterations: int = 1, temperature=1.0,
               eos_token_id=None, beta=0.0, epsilon=0.2, epsilon_high=None, loss_type="bnpo",
               importance_sampling_level="token", scale_rewards=True, max_grad_norm=1.0, ref_model=None,
               delta=None, top_entropy_quantile: float = 1.0, mask_truncated_completions: bool = False,
               reward_weights=None, micro_steps_per_epoch: Optional[int] = None, capture: bool = False):
    """`n_steps` optimizer steps of the transformers Trainer around GRPOTrainer, with the
    reference's buffering (_prepare_inputs, grpo_trainer.py:1411-1444): a new generation
    every steps_per_generation * num_iterations micro-steps, shuffled (the permutation is
    given: g["perm"], the reference draws it from the global RNG, :259) and split into
    steps_per_generation micro-batches that are revisited num_iterations times; the old
    log-probs enter when GA is not a multiple of that period (:1854-1869).  Each micro-batch
    is a separate forward/backward of loss / GA (model_accepts_loss_kwargs False), then
    clip_grad_norm_ and the optimizer step.

    The GRPO knobs follow the reference where it applies them: epsilon_high and delta
    (two-sided clipping, :2110-2118), top_entropy_quantile (:2079-2082: the per-micro-
    batch quantile over the entropies that entropy_from_logits returns in the logits'
    dtype, utils.py:1465-1490, i.e. bf16 entropies for a bf16 model),
    mask_truncated_completions (:1829-1831), several reward functions with
    reward_weights and None -> NaN (:1485-1487, :1918), scale_rewards (:1929-1930).

    micro_steps_per_epoch (len of the train dataloader): the transformers Trainer ends an
    epoch whose micro-batches are not a multiple of GA with an update over the remainder,
    each micro loss divided by that remainder (trainer.py _run_epoch: `remainder`,
    current_gradient_accumulation_steps; training_step's loss / it).

    generations: iterable of {prompt_ids, prompt_mask, completion_ids, perm} consumed when a
    generation is due.  Returns one dict per optimizer step: loss (sum of the micro losses /
    GA), grad_norm, and with capture the micro-batch log-probs in training order ("logps"),
    the pre-clip gradients ("grads"), plus "gens": the scored generation batches."""
    GA = gradient_accumulation_steps
    spg = steps_per_generation or GA
    generate_every = spg * num_iterations
    need_old = GA % generate_every != 0
    it = iter(generations)
    buffered, micro_step, gens, out = None, 0, [], []
    for _ in range(n_steps):
        losses, lps, emasks = [], [], []
        n_acc = GA if not micro_steps_per_epoch else min(GA, micro_steps_per_epoch - micro_step % micro_steps_per_epoch)
        for _ in range(n_acc):
            if micro_step % generate_every == 0 or buffered is None:
                g = next(it)
                sc = score_generation(model, g, reward_fn, num_generations=num_generations,
                                      temperature=temperature, eos_token_id=eos_token_id,
                                      scale_rewards=scale_rewards, beta=beta, ref_model=ref_model,
                                      need_old=need_old, per_device_train_batch_size=per_device_train_batch_size,
                                      mask_truncated_completions=mask_truncated_completions,
                                      reward_weights=reward_weights)
                gens.append(sc)
                keys = ("p", "pm", "c", "cm", "a", "old", "ref")
                shuffled = trl_ref.permute_sequence_dict({k: sc[k] for k in keys}, g["perm"])
                buffered = trl_ref.split_tensor_dict(shuffled, spg)
            dev = next(model.parameters()).device
            mb = {k: (None if v is None else v.to(dev)) for k, v in buffered[micro_step % spg].items()}
            micro_step += 1
            lp, ent = per_token_logps(model, mb["p"], mb["pm"], mb["c"], mb["cm"], temperature)
            emask = None
            if top_entropy_quantile < 1.0:  # :2079-2082
                emask = trl_ref.get_high_entropy_mask(ent, mb["cm"], 1 - top_entropy_quantile)
                emasks.append(emask.cpu())
            loss, _ = trl_ref.grpo_loss(lp, mb["a"], mb["cm"], old_per_token_logps=mb["old"],
                                        ref_per_token_logps=mb["ref"], entropy_mask=emask, entropies=ent,
                                        beta=beta, delta=delta,
                                        epsilon_low=epsilon, epsilon_high=epsilon_high or epsilon,
                                        loss_type=loss_type, importance_sampling_level=importance_sampling_level,
                                        max_completion_length=C)
            (loss / n_acc).backward()
            losses.append(float(loss.detach()) / n_acc)
            lps.append(lp.detach().cpu())
        grads = ({n: p.grad.detach().cpu().clone() for n, p in model.named_parameters() if p.grad is not None}
                 if capture else None)
        total = torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)
        optimizer.step()
        optimizer.zero_grad()
        rec = {"loss": sum(losses), "grad_norm": float(total), "losses": losses}
        if capture:
            rec.update(logps=torch.cat(lps), grads=grads)
            if emasks:
                rec["entropy_mask"] = torch.cat(emasks)
        out.append(rec)
    if out:
        out[0]["gens"] = gens
    return out


def grpo_step(model, optimizer, prompt_ids, prompt_mask, reward_fn: Callable, *, num_generations: int, C: int,
              per_device_train_batch_size: int, gradient_accumulation_steps: int, temperature=1.0,
              eos_token_id=None, pad_token_id=0, beta=0.0, epsilon=0.2, epsilon_high=None, loss_type="bnpo",
              importance_sampling_level="token", scale_rewards=True, max_grad_norm=1.0, do_sample=True,
              min_new_tokens=0, perm: Optional[torch.Tensor] = None, completion_ids=None, timings=None,
              ref_model=None, capture: bool = False):
    """One optimizer step over one generation batch (steps_per_generation = rows /
    per_device_train_batch_size, as GRPOConfig derives it); returns (mean loss, dict of
    intermediates).

    completion_ids None: the completions come from transformers generate with the
    reference's GenerationConfig.  ref_model (beta != 0): the frozen reference scored on
    the whole batch before the shuffle (grpo_trainer.py:1871-1899).  capture=True adds
    the per-token log-probs of every micro-batch ("logps", permuted row order), the
    pre-clip gradients ("grads") and the per-micro losses."""
    t0 = time.perf_counter()
    if completion_ids is None:
        completion_ids = generate(model, prompt_ids, prompt_mask, C, do_sample=do_sample, temperature=temperature,
                                  min_new_tokens=min_new_tokens, pad_token_id=pad_token_id,
                                  eos_token_id=eos_token_id)
    t1 = time.perf_counter()
    B = completion_ids.shape[0]
    perm = torch.arange(B) if perm is None else perm
    spg = B // per_device_train_batch_size
    gen = {"prompt_ids": prompt_ids, "prompt_mask": prompt_mask, "completion_ids": completion_ids, "perm": perm}
    rec = grpo_train(model, optimizer, [gen], reward_fn, num_generations=num_generations, C=C,
                     per_device_train_batch_size=per_device_train_batch_size,
                     gradient_accumulation_steps=min(spg, gradient_accumulation_steps), n_steps=1,
                     steps_per_generation=spg, temperature=temperature, eos_token_id=eos_token_id, beta=beta,
                     epsilon=epsilon, epsilon_high=epsilon_high, loss_type=loss_type,
                     importance_sampling_level=importance_sampling_level, scale_rewards=scale_rewards,
                     max_grad_norm=max_grad_norm, ref_model=ref_model, capture=capture)[0]
    t2 = time.perf_counter()
    if timings is not None:
        timings["generate_s"] = t1 - t0
        timings["update_s"] = t2 - t1
    sc = rec["gens"][0]
    out = {"completion_ids": completion_ids, "completion_mask": sc["cm"], "advantages": sc["a"],
           "rewards": sc["rewards"], "grad_norm": rec["grad_norm"], "perm": perm}
    if capture:
        out.update(logps=rec["logps"], grads=rec["grads"], losses=rec["losses"])
    return rec["loss"], out
