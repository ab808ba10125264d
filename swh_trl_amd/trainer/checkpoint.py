"""Checkpoints in the transformers Trainer layout.

The reference saves through transformers `Trainer._save_checkpoint`, which
GRPOTrainer / PPOTrainer extend with a model card (grpo_trainer.py:2234-2241,
ppo_trainer.py:752-758; PPOTrainer.save_model keeps only the policy,
:332-346).  A checkpoint directory `output_dir/checkpoint-<step>/` holds:

  config.json, generation_config.json   transformers model config
  model.safetensors (+ index if sharded) the weights under the transformers
                                        names (tied lm_head omitted, as
                                        save_pretrained does)
  optimizer.pt                          torch AdamW state_dict: per-parameter
                                        exp_avg / exp_avg_sq / step in the
                                        model.named_parameters() order, split
                                        into the Trainer's decay / no-decay
                                        param groups
  scheduler.pt                          torch LambdaLR.state_dict() of the
                                        Trainer's schedule (loads into
                                        LambdaLR.load_state_dict)
  trainer_state.json                    transformers TrainerState fields
  README.md                             the trainer's model card

plus the engine's own exact-resume state, which a transformers checkpoint
does not carry: `swh_master.safetensors` (the fp32 master weights; the model
file holds the bf16 weights) and one `swh_trainer_state_<rank>.pt` per rank
(tensors only: data stream position, that rank's shuffle generator and
buffered rollouts — as transformers keeps one rng_state_<rank>.pth per process).
Loading reads safetensors / JSON, and torch.load(weights_only=True) only.
"""
from __future__ import annotations

import json
import math
import os
import re
from typing import Optional

import torch

from ..engine.config import DecoderConfig
from ..engine.model import CausalLM

SHARD_BYTES = 5 << 30  # transformers' default max_shard_size ("5GB")


def hf_config_dict(cfg: DecoderConfig, head: str = "lm", dtype: torch.dtype = torch.bfloat16,
                   eos_token_id=None, pad_token_id=None) -> dict:
    """transformers config.json for a Qwen2 / Llama / GPT-2 model (or its
    *ForSequenceClassification with one label for head="score")."""
    tdt = "float32" if dtype == torch.float32 else "bfloat16"
    if cfg.model_type == "gpt2":
        H = cfg.hidden_size
        d = {"architectures": ["GPT2LMHeadModel" if head == "lm" else "GPT2ForSequenceClassification"],
             "model_type": "gpt2", "vocab_size": cfg.vocab_size, "n_embd": H, "n_layer": cfg.num_hidden_layers,
             "n_head": cfg.num_attention_heads, "n_positions": cfg.max_position_embeddings,
             "n_inner": None if cfg.intermediate_size == 4 * H else cfg.intermediate_size,
             "layer_norm_epsilon": cfg.rms_norm_eps, "activation_function": "gelu_new", "resid_pdrop": 0.0,
             "embd_pdrop": 0.0, "attn_pdrop": 0.0, "scale_attn_weights": True, "tie_word_embeddings": True,
             "initializer_range": 0.02, "use_cache": True, "torch_dtype": tdt, "eos_token_id": eos_token_id,
             "pad_token_id": pad_token_id, "bos_token_id": None}
        if head == "score":
            d.update(num_labels=1, id2label={"0": "LABEL_0"}, label2id={"LABEL_0": 0})
        return d
    fam = "Qwen2" if cfg.model_type == "qwen2" else "Llama"
    arch = f"{fam}ForCausalLM" if head == "lm" else f"{fam}ForSequenceClassification"
    d = {
        "architectures": [arch], "model_type": cfg.model_type, "vocab_size": cfg.vocab_size,
        "hidden_size": cfg.hidden_size, "intermediate_size": cfg.intermediate_size,
        "num_hidden_layers": cfg.num_hidden_layers, "num_attention_heads": cfg.num_attention_heads,
        "num_key_value_heads": cfg.num_key_value_heads, "head_dim": cfg.head_dim, "hidden_act": "silu",
        "max_position_embeddings": cfg.max_position_embeddings, "rms_norm_eps": cfg.rms_norm_eps,
        "rope_theta": cfg.rope_theta, "rope_parameters": {"rope_theta": cfg.rope_theta, "rope_type": "default"},
        "tie_word_embeddings": cfg.tie_word_embeddings, "attention_dropout": 0.0, "initializer_range": 0.02,
        "use_cache": True, "torch_dtype": tdt,
        "eos_token_id": eos_token_id, "pad_token_id": pad_token_id, "bos_token_id": None,
    }
    if cfg.model_type == "llama":
        d.update(attention_bias=cfg.attention_bias, mlp_bias=False, pretraining_tp=1)
    else:
        d.update(use_sliding_window=False, sliding_window=None, max_window_layers=cfg.num_hidden_layers)
    if head == "score":
        d.update(num_labels=1, id2label={"0": "LABEL_0"}, label2id={"LABEL_0": 0})
    return d


def _state_for_save(model: CausalLM) -> dict:
    sd = model.hf_state_dict()
    if model.cfg.tie_word_embeddings and model.head == "lm":
        sd.pop("lm_head.weight", None)  # tied to the embedding: transformers drops it on save
    return sd


def save_pretrained(model: CausalLM, out_dir: str, eos_token_id=None, pad_token_id=None) -> None:
    """Write `model` so transformers' from_pretrained (and `load_model`) reads it."""
    from safetensors.torch import save_file
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(hf_config_dict(model.cfg, model.head, model.dtype, eos_token_id, pad_token_id), f, indent=2)
    if model.head == "lm":
        with open(os.path.join(out_dir, "generation_config.json"), "w") as f:
            json.dump({"eos_token_id": eos_token_id, "pad_token_id": pad_token_id, "bos_token_id": None}, f, indent=2)
    sd = _state_for_save(model)
    shards, cur, size = [], {}, 0
    for k, v in sd.items():  # in layout order; copies out of the flat buffer (no shared storage)
        nb = v.numel() * v.element_size()
        if cur and size + nb > SHARD_BYTES:
            shards.append(cur)
            cur, size = {}, 0
        cur[k] = v.detach().to("cpu").contiguous().clone()
        size += nb
    shards.append(cur)
    meta = {"format": "pt"}
    if len(shards) == 1:
        save_file(shards[0], os.path.join(out_dir, "model.safetensors"), metadata=meta)
        return
    wmap, total = {}, 0
    for i, sh in enumerate(shards):
        name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(out_dir, name), metadata=meta)
        for k, v in sh.items():
            wmap[k] = name
            total += v.numel() * v.element_size()
    with open(os.path.join(out_dir, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, f, indent=2)


def hf_param_order(model: CausalLM) -> list[str]:
    """model.named_parameters() order of the transformers module (tied lm_head
    is the embedding parameter and appears once)."""
    c = model.cfg
    if c.model_type == "gpt2":
        names = ["transformer.wte.weight", "transformer.wpe.weight"]
        for i in range(c.num_hidden_layers):
            pre = f"transformer.h.{i}."
            names += [pre + n for n in ("ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias",
                                        "attn.c_proj.weight", "attn.c_proj.bias", "ln_2.weight", "ln_2.bias",
                                        "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias")]
        names += ["transformer.ln_f.weight", "transformer.ln_f.bias"]
        if model.head == "score":
            names.append("score.weight")
        return names
    names = ["model.embed_tokens.weight"]
    for i in range(c.num_hidden_layers):
        pre = f"model.layers.{i}."
        for n in "qkv":
            names.append(pre + f"self_attn.{n}_proj.weight")
            if c.attention_bias:
                names.append(pre + f"self_attn.{n}_proj.bias")
        names += [pre + "self_attn.o_proj.weight", pre + "mlp.gate_proj.weight", pre + "mlp.up_proj.weight",
                  pre + "mlp.down_proj.weight", pre + "input_layernorm.weight", pre + "post_attention_layernorm.weight"]
    names.append("model.norm.weight")
    if model.head == "score":
        names.append("score.weight")
    elif not c.tie_word_embeddings:
        names.append("lm_head.weight")
    return names


def _no_decay_name(n: str) -> bool:
    """transformers Trainer.get_decay_parameter_names: biases and norm weights
    (GPT-2's LayerNorms are ln_1 / ln_2 / ln_f)."""
    return n.endswith(".bias") or "norm" in n or ".ln_" in n


def _flat_views(model: CausalLM, flat: torch.Tensor) -> dict:
    """Transformers-named views of another flat buffer with the model's layout."""
    saved = model.p
    try:
        model.p = {k: flat[o:o + math.prod(s)].view(s) for k, (o, s) in model.layout.items()}
        return model.hf_state_dict()
    finally:
        model.p = saved


def optimizer_state_dict(model: CausalLM, opt, weight_decay: float, parts=None) -> dict:
    """The flat AdamW state as torch.optim.AdamW.state_dict() of the Trainer's
    two param groups (decay, no decay) over the transformers parameters.
    parts: [(name prefix, model, flat optimizer), ...] for a module holding
    several models (PPO's PolicyAndValueWrapper: "policy.", "value_model.")."""
    parts = parts or [("", model, opt)]
    names, moments, steps = [], {}, {}
    for pre, mdl, o in parts:
        m, v = _flat_views(mdl, o.exp_avg), _flat_views(mdl, o.exp_avg_sq)
        for n in hf_param_order(mdl):
            names.append(pre + n)
            moments[pre + n] = (m[n], v[n])
            steps[pre + n] = o.step_count
    groups = [[n for n in names if not _no_decay_name(n)], [n for n in names if _no_decay_name(n)]]
    order = groups[0] + groups[1]
    state = {}
    for i, n in enumerate(order):
        state[i] = {"step": torch.tensor(float(steps[n])), "exp_avg": moments[n][0].detach().cpu().clone(),
                    "exp_avg_sq": moments[n][1].detach().cpu().clone()}
    base = {"lr": opt.lr, "betas": opt.betas, "eps": opt.eps, "amsgrad": False, "foreach": None, "maximize": False,
            "capturable": False, "differentiable": False, "fused": None, "initial_lr": opt.lr}
    pg = [dict(base, weight_decay=weight_decay, params=list(range(len(groups[0])))),
          dict(base, weight_decay=0.0, params=list(range(len(groups[0]), len(order))))]
    return {"state": state, "param_groups": pg, "swh_param_names": order}


def load_optimizer_state_dict(model: CausalLM, opt, sd: dict) -> None:
    names = sd.get("swh_param_names")
    if names is None:  # a transformers checkpoint: rebuild the Trainer grouping order
        allp = hf_param_order(model)
        names = [n for n in allp if not _no_decay_name(n)] + [n for n in allp if _no_decay_name(n)]
    m, v = _flat_views(model, opt.exp_avg), _flat_views(model, opt.exp_avg_sq)
    step = 0
    with torch.no_grad():
        for i, n in enumerate(names):
            st = sd["state"].get(i) if i in sd["state"] else sd["state"].get(str(i))
            if st is None:
                continue
            m[n].copy_(st["exp_avg"])
            v[n].copy_(st["exp_avg_sq"])
            step = int(float(st["step"]))
    opt.step_count = step
    opt.lr = float(sd["param_groups"][0].get("initial_lr", sd["param_groups"][0]["lr"]))


def trainer_state_json(state, args, train_batch_size: int) -> dict:
    """transformers TrainerState.save_to_json fields."""
    return {"best_global_step": None, "best_metric": None, "best_model_checkpoint": None, "epoch": state.epoch,
            "eval_steps": 500, "global_step": state.global_step, "is_hyper_param_search": False,
            "is_local_process_zero": True, "is_world_process_zero": True, "log_history": state.log_history,
            "logging_steps": args.logging_steps, "max_steps": state.max_steps,
            "num_input_tokens_seen": state.num_input_tokens_seen, "num_train_epochs": args.num_train_epochs,
            "save_steps": args.save_steps, "stateful_callbacks": {}, "total_flos": 0.0,
            "train_batch_size": train_batch_size, "trial_name": None, "trial_params": None}


def model_card(trainer_name: str, model_name: str, paper: str, citation: str, tags) -> str:
    """A model card with the fields of TRL's generate_model_card."""
    tag_lines = "\n".join(f"- {t}" for t in sorted(tags))
    return (f"---\nlibrary_name: transformers\nmodel_name: {model_name}\ntags:\n{tag_lines}\nlicence: license\n---\n\n"
            f"# Model Card for {model_name}\n\nThis model was trained with {trainer_name} ({paper}) on the "
            f"swh_trl_amd MI355X engine.\n\n## Citations\n\n```bibtex\n{citation}\n```\n")


GRPO_CITATION = ("@article{zhihong2024deepseekmath,\n    title        = {{DeepSeekMath: Pushing the Limits of "
                 "Mathematical Reasoning in Open Language Models}},\n    author       = {Zhihong Shao and Peiyi Wang "
                 "and Qihao Zhu and Runxin Xu and Junxiao Song and Mingchuan Zhang and Y. K. Li and Y. Wu and Daya "
                 "Guo},\n    year         = 2024,\n    eprint       = {arXiv:2402.03300},\n}")
PPO_CITATION = ("@article{mziegler2019fine-tuning,\n    title        = {{Fine-Tuning Language Models from Human "
                "Preferences}},\n    author       = {Daniel M. Ziegler and Nisan Stiennon and Jeffrey Wu and Tom B. "
                "Brown and Alec Radford and Dario Amodei and Paul F. Christiano and Geoffrey Irving},\n    year     "
                "    = 2019,\n    eprint       = {arXiv:1909.08593},\n}")


def scheduler_state_dict(global_step: int, lr: float, fn, n_groups: int = 2) -> dict:
    """torch LambdaLR.state_dict() of the Trainer's scheduler after `global_step`
    optimizer steps, `fn` the schedule's multiplier (schedule.py: the lambda of
    transformers get_scheduler for the configured lr_scheduler_type / warmup),
    over its `n_groups` param groups (decay / no decay).  Built from a real
    LambdaLR so the keys are the installed torch's own (lr_lambdas included:
    LambdaLR.load_state_dict pops it)."""
    p = [torch.nn.Parameter(torch.zeros(1)) for _ in range(n_groups)]
    opt = torch.optim.SGD([{"params": [q]} for q in p], lr=lr)
    sch = torch.optim.lr_scheduler.LambdaLR(opt, fn)
    sch.last_epoch = global_step
    sch._step_count = global_step + 1
    sch._last_lr = [lr * fn(global_step) for _ in range(n_groups)]
    return sch.state_dict()


LEGACY_TRAINER_STATE = "swh_trainer_state.pt"  # the single-file exact-resume state of earlier builds


def trainer_state_file(rank: int) -> str:
    return f"swh_trainer_state_{rank}.pt"


def save_master(opt, out_dir: str) -> None:
    from safetensors.torch import save_file
    save_file({"master": opt.master.detach().cpu().contiguous()}, os.path.join(out_dir, "swh_master.safetensors"))


def load_weights_into(model: CausalLM, ckpt_dir: str) -> None:
    """Weights of a save_pretrained / transformers directory into `model`."""
    from safetensors.torch import load_file
    sd = {}
    for fn in sorted(os.listdir(ckpt_dir)):
        if fn.endswith(".safetensors") and fn.startswith("model"):
            sd.update(load_file(os.path.join(ckpt_dir, fn), device=str(model.device)))
    if "lm_head.weight" not in sd and model.head == "lm" and not model.cfg.tie_word_embeddings:
        raise ValueError(f"{ckpt_dir}: lm_head.weight missing for an untied model")
    model.load_hf_state_dict(sd)


def latest_checkpoint(output_dir: str) -> Optional[str]:
    if not output_dir or not os.path.isdir(output_dir):
        return None
    cks = [(int(m.group(1)), d) for d in os.listdir(output_dir) if (m := re.fullmatch(r"checkpoint-(\d+)", d))]
    return os.path.join(output_dir, max(cks)[1]) if cks else None


def rotate_checkpoints(output_dir: str, limit: Optional[int]) -> None:
    """save_total_limit: keep the newest `limit` checkpoint-* directories."""
    import shutil
    if not limit or limit <= 0:
        return
    cks = sorted((int(m.group(1)), d) for d in os.listdir(output_dir) if (m := re.fullmatch(r"checkpoint-(\d+)", d)))
    for _, d in cks[:-limit]:
        shutil.rmtree(os.path.join(output_dir, d), ignore_errors=True)
