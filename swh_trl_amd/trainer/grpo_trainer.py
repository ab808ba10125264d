"""GRPOTrainer — drop-in for trl.GRPOTrainer's per-step loop on MI355X.

Constructor and config keep the reference's names (grpo_trainer.py:558-569,
grpo_config.py); the loop keeps its semantics (grpo_trainer.py:1411-1444
buffering, :1500-2003 rollout + scoring, :2058-2175 loss) while every
per-token stage runs on the HIP engine:

  rollout      DecodeEngine.generate        (graph-captured decode, device sampler)
  mask         ops.completion_mask          (:1812-1831)
  rewards      user callables on host       (:1446-1498, unchanged contract)
  advantages   ops.group_advantages         (:1914-1930)
  scoring      CausalLM forward -> lm head -> fused logp/entropy kernel
  loss         fused GRPO loss fwd+bwd kernel (all GA micro-batches in one pass)
  optimizer    flat-buffer AdamW + device grad-norm clip, RCCL all-reduce for DP

Fork-only additions of the reference (unsloth loading, CrossEncoder, private
validation JSON, OpenAI client) are not part of the drop-in.
"""
from __future__ import annotations

import math
import os
import time
from collections import defaultdict
from typing import Any, Callable, Optional, Union

import torch

from .. import dist as swh_dist
from .. import gemm_tuning
from .. import ops
from ..engine.config import DecoderConfig, PRESETS, from_hf_config
from ..engine import build_engine, build_model
from ..engine.gpt2 import warn_dropout
from ..engine.decode import DecodeEngine
from ..engine.model import CausalLM, dw_streams, dw_sync
from ..optim import FlatAdamW, sync_ref_model
from . import schedule
from .callbacks import CallbackHandler, new_state
from .grpo_config import GRPOConfig
from .utils import RepeatSampler, generation_batch_indices, left_pad, pad_left_cat, split_tensor_dict, \
    truncate_with_protected_tokens

RewardFunc = Union[str, Callable, torch.nn.Module]
from ..profiling import trace as _trace  # noqa: E402  (one clock for every phase line)


def model_dtype(model_init_kwargs: Optional[dict]) -> torch.dtype:
    """The model's parameter dtype from GRPOConfig/PPOConfig.model_init_kwargs
    (`torch_dtype` / `dtype`, as the reference passes them to from_pretrained,
    grpo_trainer.py:611-627): "float32" selects the fp32 reference-precision
    mode; anything else (default, "auto", "bfloat16") the bf16 engine."""
    kw = model_init_kwargs or {}
    d = kw.get("torch_dtype", kw.get("dtype"))
    if d in (torch.float32, "float32", "fp32"):
        return torch.float32
    if d in (None, "auto", torch.bfloat16, "bfloat16", "bf16"):
        return torch.bfloat16
    raise ValueError(f"model dtype {d!r}: the MI355X engine trains bfloat16 or float32 models")


def load_model(model, device, trainable=True, seed=0, head: str = "lm", dtype=None) -> CausalLM:
    """`model` may be a CausalLM, a preset name ("qwen2.5-0.5b", "llama-3-8b",
    "tiny"), a DecoderConfig (random init), a local directory holding a
    transformers config.json + safetensors, or a transformers PreTrainedModel.
    head="score": a sequence-classification model (value / reward model, one
    output), as transformers' *ForSequenceClassification.  `dtype`: parameter
    dtype of a model built from a name / config / directory (default bf16); a
    model object keeps its own precision (a CausalLM as is; a transformers
    module fp32 -> fp32, bf16 / fp16 -> bf16), as the reference trains the
    module it is given in its dtype."""
    if dtype is None:
        dtype = torch.bfloat16
        if hasattr(model, "parameters") and not isinstance(model, CausalLM):
            p0 = next(iter(model.parameters()), None)
            if p0 is not None and p0.dtype == torch.float32:
                dtype = torch.float32
    if isinstance(model, CausalLM):
        if model.head != head:
            raise ValueError(f"expected a model with a {head!r} head, got {model.head!r}")
        return model
    if isinstance(model, DecoderConfig):
        return build_model(model, device, head=head, seed=seed, trainable=trainable, dtype=dtype)
    if isinstance(model, str):
        if model in PRESETS:
            return build_model(PRESETS[model](), device, head=head, seed=seed, trainable=trainable, dtype=dtype)
        if os.path.isdir(model):
            import json

            from safetensors.torch import load_file
            with open(os.path.join(model, "config.json")) as f:
                cfg = from_hf_config(json.load(f))
            m = build_model(cfg, device, head=head, seed=None, trainable=trainable, dtype=dtype)
            sd = {}
            for fn in sorted(os.listdir(model)):
                if fn.endswith(".safetensors"):
                    sd.update(load_file(os.path.join(model, fn), device=str(device)))
            m.load_hf_state_dict(sd)
            return m
        raise ValueError(f"cannot load model {model!r}: no hub access; pass a preset, a local directory or a "
                         "model object")
    if hasattr(model, "config") and hasattr(model, "state_dict"):
        cfg = from_hf_config(model.config)
        if cfg.model_type == "gpt2":
            warn_dropout(model.config)
        m = build_model(cfg, device, head=head, seed=None, trainable=trainable, dtype=dtype)
        m.load_hf_state_dict({k: v.to(device) for k, v in model.state_dict().items()})
        return m
    raise TypeError(f"unsupported model type {type(model)}")


# GenerationConfig keys (transformers >= 4.53) -> how the engine treats them
_GEN_IMPLEMENTED = frozenset({"max_new_tokens", "min_new_tokens", "min_length", "do_sample", "pad_token_id",
                              "eos_token_id", "temperature", "top_p", "top_k", "min_p", "repetition_penalty"})
# cannot change the returned completion ids: cache / paged-attention / compile plumbing, the BOS id of a
# decoder-only prompt, beam-only knobs, extra outputs that generate() returns only with return_dict_in_generate,
# renormalisation after the processors (the sampled distribution is the same), max_length under max_new_tokens
_GEN_INERT = frozenset({"bos_token_id", "cache_implementation", "cache_config", "max_cache_len", "use_cache",
                        "max_batch_tokens", "num_blocks", "block_size", "compile_config", "disable_compile",
                        "prefill_chunk_size", "length_penalty", "early_stopping", "low_memory", "output_attentions",
                        "output_hidden_states", "output_scores", "output_logits", "renormalize_logits", "max_length",
                        "transformers_version", "_from_model_config", "_commit_hash", "decoder_start_token_id",
                        "is_assistant"})
# processors / search modes the engine does not implement: accepted only at their no-op value
_GEN_NOOP_VALUES = {"num_beams": (None, 1), "num_return_sequences": (None, 1), "num_beam_groups": (None, 1),
                    "typical_p": (None, 1.0), "epsilon_cutoff": (None, 0.0), "eta_cutoff": (None, 0.0),
                    "encoder_repetition_penalty": (None, 1.0), "guidance_scale": (None, 1.0),
                    "no_repeat_ngram_size": (None, 0), "encoder_no_repeat_ngram_size": (None, 0),
                    "diversity_penalty": (None, 0.0), "top_h": (None,), "penalty_alpha": (None,),
                    "bad_words_ids": (None,), "suppress_tokens": (None,), "begin_suppress_tokens": (None,),
                    "forced_bos_token_id": (None,), "forced_eos_token_id": (None,), "sequence_bias": (None,),
                    "exponential_decay_length_penalty": (None,), "watermarking_config": (None,),
                    "stop_strings": (None,), "max_time": (None,), "constraints": (None,), "force_words_ids": (None,),
                    "dola_layers": (None,), "prompt_lookup_num_tokens": (None,), "num_assistant_tokens": (None,),
                    "assistant_confidence_threshold": (None,), "assistant_early_exit": (None,),
                    "remove_invalid_values": (None, False), "return_dict_in_generate": (None, False),
                    "token_healing": (None, False), "use_mtp": (None, False)}


def generation_config(args: GRPOConfig, tokenizer=None) -> dict:
    """The sampling parameters of one rollout, built as grpo_trainer.py:995-1014
    builds its GenerationConfig: the config fields first (max_new_tokens =
    max_completion_length, do_sample, the tokenizer's pad / bos / eos, temperature,
    top_p, top_k, min_p, repetition_penalty, cache_implementation), then
    `args.generation_kwargs` on top.  Returns the resolved keys the engine
    implements (HF semantics: a key left None is off).  Keys that cannot change the
    completions are accepted and dropped; a processor or search mode the engine
    does not implement raises unless it is at its no-op value.  The scoring passes
    keep dividing by `args.temperature` (:1249), whatever the rollout sampled at."""
    g = {"max_new_tokens": args.max_completion_length, "do_sample": True,
         "pad_token_id": getattr(tokenizer, "pad_token_id", None), "bos_token_id": getattr(tokenizer, "bos_token_id", None),
         "eos_token_id": getattr(tokenizer, "eos_token_id", None), "temperature": args.temperature,
         "top_p": args.top_p, "top_k": args.top_k, "min_p": args.min_p,
         "repetition_penalty": args.repetition_penalty, "cache_implementation": args.cache_implementation}
    g.update(args.generation_kwargs or {})
    bad = []
    for k, v in g.items():
        if k in _GEN_IMPLEMENTED or k in _GEN_INERT:
            continue
        if k in _GEN_NOOP_VALUES:
            if v not in _GEN_NOOP_VALUES[k]:
                bad.append(f"{k}={v!r}")
            continue
        bad.append(f"{k}={v!r} (unknown generation key)")
    if bad:
        raise ValueError("generation_kwargs: the MI355X decode engine does not implement " + ", ".join(bad))
    if g["max_new_tokens"] is None or int(g["max_new_tokens"]) < 1:
        raise ValueError(f"max_new_tokens must be a positive integer, got {g['max_new_tokens']!r}")
    do_sample = bool(g["do_sample"])
    t = g["temperature"]
    if do_sample and t is not None and not (float(t) > 0.0):
        raise ValueError(f"`temperature` (={t}) has to be a strictly positive float, otherwise your next token "
                         "scores will be invalid. If you're looking for greedy decoding strategies, set "
                         "`do_sample=False`.")
    if do_sample and g["top_p"] is not None and not (0.0 <= float(g["top_p"]) <= 1.0):
        raise ValueError(f"`top_p` has to be a float > 0 and < 1, but is {g['top_p']}")
    if do_sample and g["min_p"] is not None and not (0.0 <= float(g["min_p"]) <= 1.0):
        raise ValueError(f"`min_p` has to be a float in the [0, 1] interval, but is {g['min_p']}")
    if g["top_k"] is not None and int(g["top_k"]) < 0:
        raise ValueError(f"`top_k` has to be a non-negative integer, but is {g['top_k']}")
    rp = g["repetition_penalty"]
    if rp is not None and not (float(rp) > 0.0):
        raise ValueError(f"`penalty` has to be a strictly positive float, but is {rp}")
    # _get_logits_processor: the warpers (temperature, top-k, top-p, min-p) only when sampling
    return {"max_new_tokens": int(g["max_new_tokens"]), "min_new_tokens": int(g.get("min_new_tokens") or 0),
            "min_length": int(g.get("min_length") or 0), "greedy": not do_sample,
            "temperature": float(t) if (do_sample and t is not None) else 1.0,
            "top_p": float(g["top_p"]) if (do_sample and g["top_p"] is not None) else 1.0,
            "top_k": int(g["top_k"]) if (do_sample and g["top_k"]) else None,
            "min_p": float(g["min_p"]) if (do_sample and g["min_p"] is not None) else None,
            "repetition_penalty": float(rp) if rp is not None else 1.0,
            "pad_token_id": g["pad_token_id"], "eos_token_id": g["eos_token_id"]}


def _is_pretrained_model(f) -> bool:
    """transformers PreTrainedModel (without importing transformers when absent)."""
    return any(c.__name__ == "PreTrainedModel" for c in type(f).__mro__)


class RewardModel:
    """A sequence-classification reward model (num_labels = 1) on the engine:
    the frozen CausalLM with its score head, called like the transformers
    module it replaces — `rm(input_ids=..., attention_mask=...).logits` is
    [B, 1], the score Linear at the rightmost token that is not
    `config.pad_token_id` (transformers GenericForSequenceClassification;
    batch size > 1 needs a pad id), positions 0.. as transformers assigns them
    without position_ids.  `config` is the transformers config object of a
    converted module (so the trainer's pad-id assignment reaches it, as the
    reference's does) or, for a directory, its config.json fields plus
    `_name_or_path`."""

    SUPPORTED = ("Qwen2ForSequenceClassification", "LlamaForSequenceClassification")

    def __init__(self, model: CausalLM, config):
        self.model, self.config = model, config
        self.device = model.device

    @classmethod
    def supports(cls, module) -> bool:
        score = getattr(module, "score", None)
        return (type(module).__name__ in cls.SUPPORTED and getattr(module.config, "num_labels", 1) == 1
                and getattr(score, "bias", None) is None)

    @classmethod
    def from_module(cls, module, device) -> "RewardModel":
        return cls(load_model(module, device, trainable=False, head="score"), module.config)

    @classmethod
    def from_pretrained(cls, path: str, device, dtype) -> "RewardModel":
        """AutoModelForSequenceClassification.from_pretrained(path, num_labels=1)
        from a local directory (no hub access here)."""
        import json
        import types
        if not os.path.isdir(path):
            raise ValueError(f"reward model {path!r}: not a local directory (no hub access); pass a directory holding "
                             "a transformers config.json + safetensors, or a model object")
        with open(os.path.join(path, "config.json")) as f:
            cj = json.load(f)
        if cj.get("num_labels", len(cj.get("id2label", {0: 0}))) != 1:
            raise ValueError(f"reward model {path!r}: num_labels must be 1")
        cfg = types.SimpleNamespace(**cj)
        cfg._name_or_path = path
        cfg.pad_token_id = cj.get("pad_token_id")
        return cls(load_model(path, device, trainable=False, head="score", dtype=dtype), cfg)

    def __call__(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None, **unused):
        import types
        ids = input_ids.to(self.device)
        B, L = ids.shape
        pad = self.config.pad_token_id
        if pad is None and B != 1:
            raise ValueError("Cannot handle batch sizes > 1 if no padding token is defined.")
        if pad is None:
            last = torch.full((B,), L - 1, device=self.device, dtype=torch.int64)
        else:
            last = (torch.arange(L, device=self.device) * (ids != pad)).argmax(-1)
        m = self.model
        with torch.no_grad():
            km = None if attention_mask is None else attention_mask.to(self.device)
            h = m.hidden_states(ids, key_mask=km)
            s = m.scores(h[torch.arange(B, device=self.device), last])
        return types.SimpleNamespace(logits=s.view(B, 1))


def _pad_completions(mb: dict, W: int, pad_token_id: int) -> dict:
    """A micro-batch's completion-side tensors right-padded to width W (pad ids,
    mask 0, log-probs 0): the extra columns are masked out of every sum."""
    out = dict(mb)
    w = mb["completion_ids"].shape[1]
    fill = {"completion_ids": pad_token_id, "completion_mask": 0, "old_per_token_logps": 0.0,
            "ref_per_token_logps": 0.0}
    for k, v in fill.items():
        if k in mb and mb[k] is not None:
            out[k] = torch.nn.functional.pad(mb[k], (0, W - w), value=v)
    return out


class GRPOTrainer:
    _tag_names = ["trl", "grpo"]

    def __init__(self, model, reward_funcs: Union[RewardFunc, list], args: Optional[GRPOConfig] = None,
                 train_dataset=None, eval_dataset=None, processing_class=None, reward_processing_classes=None,
                 callbacks=None, optimizers=(None, None), peft_config=None):
        if peft_config is not None:
            raise ValueError("peft_config: LoRA training is not part of the MI355X engine's scope")
        if optimizers is not None and any(o is not None for o in optimizers):
            raise ValueError("optimizers: the MI355X trainer updates its flat parameter buffer with the fused AdamW "
                             "kernel, configured by the GRPOConfig fields (learning_rate, adam_beta1/2, adam_epsilon, "
                             "weight_decay, max_grad_norm, lr_scheduler_type, lr_scheduler_kwargs, warmup_steps / "
                             "warmup_ratio); a torch optimizer or scheduler object cannot drive it")
        self.args = args if args is not None else GRPOConfig(output_dir="grpo-out")
        a = self.args
        self.rank, self.world, self.local_rank = swh_dist.init_from_env()
        if not torch.cuda.is_available():
            raise RuntimeError("GRPOTrainer runs the MI355X engine and needs a ROCm device (no CPU fallback)")
        self.device = torch.device("cuda", self.local_rank)
        torch.cuda.set_device(self.device)
        gemm_tuning.enable()
        torch.manual_seed(a.seed)
        self.model = load_model(model, self.device, trainable=True, seed=a.seed,
                                dtype=None if hasattr(model, "parameters") else model_dtype(a.model_init_kwargs))
        self.processing_class = processing_class
        if not isinstance(reward_funcs, list):
            reward_funcs = [reward_funcs]
        self._setup_reward_funcs(reward_funcs, reward_processing_classes)
        if a.reward_weights is not None:
            if len(a.reward_weights) != len(reward_funcs):
                raise ValueError(f"Number of reward weights ({len(a.reward_weights)}) must match number of reward "
                                 f"functions ({len(reward_funcs)})")
            self.reward_weights = torch.tensor(a.reward_weights, dtype=torch.float32, device=self.device)
        else:
            self.reward_weights = torch.ones(len(reward_funcs), dtype=torch.float32, device=self.device)
        self.train_dataset, self.eval_dataset = train_dataset, eval_dataset
        self.num_generations = a.num_generations
        self.temperature = a.temperature
        self.beta = a.beta
        self.epsilon_low = a.epsilon
        self.epsilon_high = a.epsilon_high if a.epsilon_high is not None else a.epsilon
        self.num_iterations = a.num_iterations
        self.loss_type = a.loss_type
        self.scale_rewards = a.scale_rewards
        self.importance_sampling_level = a.importance_sampling_level
        self.mask_truncated_completions = a.mask_truncated_completions
        self.top_entropy_quantile = a.top_entropy_quantile
        self.max_prompt_length = a.max_prompt_length
        self.max_completion_length = a.max_completion_length
        # the rollout's sampling parameters: config fields, then generation_kwargs on top (:995-1014)
        gen = generation_config(a, processing_class)
        # the trainer's own ids (prompt padding, completion mask :1812-1831) are the tokenizer's
        # (:720-721); without a tokenizer (token-id datasets) the generation config's stand in
        tok = processing_class
        self.pad_token_id = getattr(tok, "pad_token_id", None)
        self.eos_token_id = getattr(tok, "eos_token_id", None)
        if self.eos_token_id is None:
            self.eos_token_id = gen["eos_token_id"]
        if self.pad_token_id is None:
            self.pad_token_id = gen["pad_token_id"]
        if self.pad_token_id is None:
            self.pad_token_id = self.eos_token_id if isinstance(self.eos_token_id, int) else 0
        self.gen_max_new_tokens = gen.pop("max_new_tokens")
        self.gen_min_length = gen.pop("min_length")
        self.gen_eos_token_id = gen.pop("eos_token_id")
        self.gen_pad_token_id = gen.pop("pad_token_id")
        if self.gen_eos_token_id is None:
            self.gen_eos_token_id = self.eos_token_id
        if self.gen_pad_token_id is None:
            self.gen_pad_token_id = self.pad_token_id
        self.gen_kwargs = gen
        self.ref_model = None
        if self.beta != 0.0:
            self.ref_model = build_model(self.model.cfg, self.device, seed=None, trainable=False,
                                         dtype=self.model.dtype)
            self.ref_model.copy_from(self.model)
        self.optimizer = FlatAdamW(self.model.numel, self.device, lr=a.learning_rate,
                                   betas=(a.adam_beta1, a.adam_beta2), eps=a.adam_epsilon,
                                   weight_decay=a.weight_decay, max_grad_norm=a.max_grad_norm,
                                   no_decay_ranges=self.model.no_decay_ranges())
        self.optimizer.master.copy_(self.model.flat.float())
        self.state = new_state(self.rank, self.local_rank)
        self._step = 0
        self._buffered_inputs = None
        self._metrics = {"train": defaultdict(list), "eval": defaultdict(list)}
        self._engine: Optional[DecodeEngine] = None   # the engine of the latest generation
        self._engines: dict = {}
        self._gen_count = 0      # generation batches drawn so far (data-stream position, rollout RNG offset)
        self._shuffle_gen = torch.Generator().manual_seed(a.seed + 17 * self.rank)
        self._batches = None
        self._eval_count = 0     # eval generations so far (rollout RNG offset of the eval stream)
        self._ref_version = 0    # TR-DPO syncs of the reference so far
        self.callback_handler = CallbackHandler(callbacks, self)
        self.control = self.callback_handler.call("on_init_end")

    # ------------------------------------------------------------------ callbacks (transformers Trainer API)
    def add_callback(self, callback):
        self.callback_handler.add_callback(callback)

    def pop_callback(self, callback):
        return self.callback_handler.pop_callback(callback)

    def remove_callback(self, callback):
        self.callback_handler.remove_callback(callback)

    # ------------------------------------------------------------------ reward functions
    def _setup_reward_funcs(self, reward_funcs: list, reward_processing_classes):
        """grpo_trainer.py:727-772.  A string is a sequence-classification reward
        model (AutoModelForSequenceClassification, num_labels=1): here a local
        directory loaded onto the engine's score head.  A transformers Qwen2 /
        Llama sequence classifier is copied onto the engine too (reward models
        are frozen), so scoring runs the HIP forward; any other nn.Module is
        called as given.  Names: the model's `config._name_or_path` last path
        component, a callable's __name__.  A reward model without a processing
        class gets AutoTokenizer.from_pretrained(_name_or_path); a tokenizer
        without a pad token pads with EOS, and the model's config.pad_token_id
        is set to the tokenizer's (the score is read at the last non-pad token)."""
        dtype = model_dtype(self.args.model_init_kwargs)
        funcs, names = [], []
        for f in reward_funcs:
            if isinstance(f, str):
                f = RewardModel.from_pretrained(f, self.device, dtype)
            elif isinstance(f, torch.nn.Module) and RewardModel.supports(f):
                f = RewardModel.from_module(f, self.device)
            if isinstance(f, (RewardModel, torch.nn.Module)):
                names.append(f.config._name_or_path.split("/")[-1])
            else:
                names.append(getattr(f, "__name__", None) or type(f).__name__)
            funcs.append(f)
        if reward_processing_classes is None:
            rpcs = [None] * len(funcs)
        elif not isinstance(reward_processing_classes, list):
            rpcs = [reward_processing_classes]
        else:
            if len(reward_processing_classes) != len(funcs):
                raise ValueError("The number of reward processing classes must match the number of reward functions.")
            rpcs = list(reward_processing_classes)
        for i, (rtok, f) in enumerate(zip(rpcs, funcs)):
            if isinstance(f, RewardModel) or _is_pretrained_model(f):
                if rtok is None:
                    from transformers import AutoTokenizer
                    rtok = AutoTokenizer.from_pretrained(f.config._name_or_path)
                if rtok.pad_token_id is None:
                    rtok.pad_token = rtok.eos_token
                f.config.pad_token_id = rtok.pad_token_id
                rpcs[i] = rtok
        self.reward_funcs, self.reward_func_names, self.reward_processing_classes = funcs, names, rpcs

    # ------------------------------------------------------------------ data
    def _local_gen_batch_size(self) -> int:
        return self.args.per_device_train_batch_size * self.args.steps_per_generation

    def _generation_batches(self):
        """This rank's slice of every global generation batch (trainer/utils.py
        `generation_batch_indices`, the RepeatSampler + accelerate sharding)."""
        a = self.args
        for mine in generation_batch_indices(len(self.train_dataset), self.num_generations, a.generation_batch_size,
                                             self._local_gen_batch_size(), self.rank, a.seed,
                                             bool(a.shuffle_dataset)):
            yield [self.train_dataset[i] for i in mine]

    @staticmethod
    def _is_conversational(example: dict) -> bool:
        """trl/data_utils.py:31-69 (prompt-only datasets): the prompt is a list of
        {"role", "content"} messages."""
        p = example.get("prompt")
        return isinstance(p, list) and len(p) > 0 and isinstance(p[0], dict) and "role" in p[0] and "content" in p[0]

    def _tokenize_prompts(self, examples):
        if "prompt_ids" in examples[0]:
            ids, mask = left_pad([list(x["prompt_ids"]) for x in examples], self.pad_token_id, self.device)
            texts = [x.get("prompt") for x in examples]
        else:
            tok = self.processing_class
            if tok is None:
                raise ValueError("text prompts need a processing_class (tokenizer)")
            texts = []
            for x in examples:
                p = x["prompt"]
                if self._is_conversational(x):
                    # data_utils.py:100-116: a trailing assistant turn is continued,
                    # otherwise the generation prompt is added
                    last = p[-1]["role"]
                    if last not in ("user", "assistant"):
                        raise ValueError(f"Invalid role in the last message: {last}")
                    p = tok.apply_chat_template(p, continue_final_message=last == "assistant", tokenize=False,
                                                add_generation_prompt=last == "user")
                texts.append(p)
            enc = tok(text=texts, return_tensors="pt", padding=True, padding_side="left", add_special_tokens=False)
            ids, mask = enc["input_ids"].to(self.device), enc["attention_mask"].to(self.device).int()
        if self.max_prompt_length is not None and ids.shape[1] > self.max_prompt_length:
            ids, mask = truncate_with_protected_tokens(ids, mask, self.max_prompt_length, [])
        return ids, mask, texts

    def _engine_for(self, B: int, P: int) -> DecodeEngine:
        C = self.gen_max_new_tokens
        # the policy itself: bf16 on the DecodeEngine, an fp32 policy on the fp32
        # RefDecodeEngine (the reference generates in the model dtype, :1793-1810)
        # one engine per batch size (training and evaluation batches differ), built once
        gm = self.model
        e = self._engines.get(B)
        if e is None or e.Pmax < P or e.model is not gm:
            Pmax = max(P, self.max_prompt_length or P) if (self.max_prompt_length or 0) <= 4096 else P
            e = self._engines[B] = build_engine(gm, B, Pmax, C)
        self._engine = e
        return e

    # ------------------------------------------------------------------ rollout + scoring
    @torch.no_grad()
    def _generate_and_score_completions(self, examples: list[dict], mode: str = "train") -> dict:
        a = self.args
        prompt_ids, prompt_mask, prompts_text = self._tokenize_prompts(examples)
        B, P = prompt_ids.shape
        _trace(f"prompts tokenized {B}x{P}")
        eng = self._engine_for(B, P)
        # the sampler's Philox stream: training generations and evaluation generations
        # draw from separate keys, each advanced by its own generation count
        if mode == "train":
            seed, count = a.seed * 1_000_003 + self.rank, self._gen_count
            self._gen_count += 1
        else:
            seed, count = a.seed * 1_000_003 + 7919 * (self.world + self.rank + 1), self._eval_count
            self._eval_count += 1
        gk = dict(self.gen_kwargs)
        if self.gen_min_length:  # MinLengthLogitsProcessor counts the (padded) prompt: EOS off while P + t < min_length
            gk["min_new_tokens"] = max(gk["min_new_tokens"], self.gen_min_length - P)
        completion_ids, _ = eng.generate(prompt_ids, prompt_mask, self.gen_max_new_tokens,
                                         eos_token_id=self.gen_eos_token_id, pad_token_id=self.gen_pad_token_id,
                                         seed=seed, offset=count * (self.gen_max_new_tokens + 1),
                                         check_every=a.decode_check_every, group_size=self.num_generations,
                                         early_exit=a.decode_early_exit, **gk)
        _trace("generated")
        eos = [] if self.eos_token_id is None else self.eos_token_id
        completion_mask, lengths, has_eos = ops.completion_mask(completion_ids, eos,
                                                                self.mask_truncated_completions)
        # HF generate stops the batch once every row has emitted EOS: the reference's
        # completions are as wide as the longest row (:1793-1810); the columns past it
        # are pad with mask 0 in every row, so dropping them changes no value and
        # saves their scoring / training compute
        # rows of one prompt are consecutive here (RepeatSampler): a group id per row lets the
        # training forward share each prompt's tokens after the shuffle (_prompt_groups); the
        # group ids and per-row prompt padding travel to the host with the width (one sync),
        # so the scoring / training passes never read them back from the device
        same = (prompt_ids[1:] == prompt_ids[:-1]).all(1) & (prompt_mask[1:] == prompt_mask[:-1]).all(1)
        group = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.device), (~same).long().cumsum(0)])
        lh = torch.cat([torch.stack([lengths.max().to(torch.int64), has_eos.min().to(torch.int64)]), group,
                        (prompt_mask == 0).any(1).to(torch.int64)]).cpu()
        width = int(lh[0]) if int(lh[1]) else completion_ids.shape[1]
        group_h, padded_h = lh[2:2 + B], lh[2 + B:].bool()
        if width < completion_ids.shape[1]:
            completion_ids = completion_ids[:, :width].contiguous()
            completion_mask = completion_mask[:, :width].contiguous()
        # the reward functions see each completion up to its first EOS even when
        # mask_truncated_completions zeroes the row's training mask: the reference builds
        # completion_ids_list (:1821-1823) before the zeroing (:1829-1831)
        reward_mask = completion_mask
        if self.mask_truncated_completions:
            reward_mask = (torch.arange(completion_ids.shape[1], device=self.device)[None, :]
                           < lengths[:, None]).to(torch.int32)
        rewards_per_func = self._calculate_rewards(examples, prompts_text, prompt_ids, prompt_mask, completion_ids,
                                                   reward_mask)
        _trace("rewards")
        # grpo_trainer.py:1494-1497 / :1933-1938: the rewards of every rank are gathered
        # (a group of G completions may straddle ranks), the advantages are formed on
        # the global batch and this rank keeps its own rows
        rewards_per_func = swh_dist.all_gather_rows(rewards_per_func)
        adv, rewards, gmean, gstd, zstd = ops.group_advantages(rewards_per_func, self.reward_weights,
                                                               self.num_generations, self.scale_rewards)
        if self.world > 1:
            adv = adv[self.rank * B:(self.rank + 1) * B]
        # host tensors ("_" keys stay on the host through shuffle, split and checkpoints)
        out = {"prompt_ids": prompt_ids, "prompt_mask": prompt_mask, "completion_ids": completion_ids,
               "completion_mask": completion_mask, "advantages": adv, "_prompt_group": group_h + count * B,
               "_row_index": torch.arange(B) + count * B, "_prompt_padded": padded_h}
        # old-policy (:1854-1869) and frozen-reference (:1871-1899) log-probs: scored here only
        # for the micro-batches whose first use would see another policy / reference; the rest
        # are scored by the training pass itself, on its own batch layout (_loss_backward)
        eager_old, eager_ref = self._eager_scoring(mode)
        if eager_old:
            out["old_per_token_logps"] = self._score_logps(self.model, out)
        if eager_ref:
            out["ref_per_token_logps"] = self._score_logps(self.ref_model, out)
        m = self._metrics[mode]
        # per generation, resolved at the next log (no host sync here): this rank's
        # lengths / EOS flags (gathered across ranks at the log, :1945-1960), its
        # attention-mask token count (:1942), and the global reward statistics
        m["_lengths"].append(torch.stack([lengths.float(), has_eos.float()], 1))
        if mode == "train":  # :1941-1942: only training generations count toward num_input_tokens_seen
            m["_tokens"].append((prompt_mask.sum() + completion_mask.sum()).float().view(1, 1))
        m["_rewards"].append(gmean)
        m["_reward_std"].append(gstd)
        m["_zero_std"].append(zstd.float())
        m["_rpf"].append(rewards_per_func)
        return out

    def _needs_old_logps(self) -> bool:
        """:1854-1869: the old-policy log-probs are kept when the optimizer steps do
        not line up with the generations (GA not a multiple of spg x num_iterations)."""
        a = self.args
        return a.gradient_accumulation_steps % (a.steps_per_generation * self.num_iterations) != 0

    def _eager_scoring(self, mode: str) -> tuple[bool, bool]:
        """Whether the generation must be scored now for old-policy / reference
        log-probs.  The reference scores both at generation time, but a value is the
        same at the micro-batch's first use as long as the model that produced it has
        not changed: the policy until the next optimizer step, the frozen reference
        until the next TR-DPO sync.  Those micro-batches take the log-probs from the
        training pass's own batch (same rows, same positions: with ref == policy the
        k3 KL is exactly 0 and the first ratio exactly 1, as in the reference); the
        others need the generation-time pass.  Generation slot j (of
        steps_per_generation) is first used at micro-step k0 + j, in optimizer step
        _update_index(k0 + j) (GA micro-steps per update, the epoch's last one shorter)."""
        a = self.args
        if mode != "train":
            return False, False
        k0 = self._step
        s0 = self._update_index(k0)
        slot_steps = [self._update_index(k0 + j) for j in range(a.steps_per_generation)]
        eager_old = self._needs_old_logps() and any(st != s0 for st in slot_steps)
        eager_ref = False
        if self.beta != 0.0 and a.sync_ref_model:
            # a sync after optimizer step t (0-based) happens when (t + 1) % ref_model_sync_steps == 0
            eager_ref = any((t + 1) % a.ref_model_sync_steps == 0 for st in slot_steps for t in range(s0, st))
        return eager_old, eager_ref

    def _mark_fresh(self, mb: dict, mode: str) -> dict:
        """Tag a micro-batch with the optimizer step and reference version of its
        generation (tensors, so buffered micro-batches checkpoint with them)."""
        if self._needs_old_logps() or mode != "train":
            mb["_gen_step"] = torch.tensor(self.state.global_step)
        if self.beta != 0.0:
            mb["_ref_version"] = torch.tensor(self._ref_version)
        return mb

    def _completions_for_rewards(self, examples, ids_h, completion_ids_list):
        """grpo_trainer.py:1901-1908: decoded completions; for conversational
        prompts each becomes [{"role": "assistant", "content": bootstrap + text}]
        where bootstrap is the content of a trailing assistant prompt turn."""
        tok = self.processing_class
        if tok is None or not hasattr(tok, "batch_decode"):
            return completion_ids_list
        texts = tok.batch_decode(ids_h, skip_special_tokens=True)
        if not self._is_conversational(examples[0]):
            return texts
        out = []
        for x, t in zip(examples, texts):
            last = x["prompt"][-1]
            boot = last["content"] if last["role"] == "assistant" else ""
            out.append([{"role": "assistant", "content": boot + t}])
        return out

    def _calculate_rewards(self, examples, prompts_text, prompt_ids, prompt_mask, completion_ids, completion_mask):
        """grpo_trainer.py:1446-1498: reward callables on host (None -> NaN);
        reward models (nn.Module) score the prompt + completion text, chat-
        templated for conversational data (:1462-1473)."""
        import copy
        B = completion_ids.shape[0]
        F = len(self.reward_funcs)
        rpf = torch.zeros(B, F, dtype=torch.float32)
        ids_h = completion_ids.cpu()
        mask_h = completion_mask.cpu().bool()
        completion_ids_list = [row[m].tolist() for row, m in zip(ids_h, mask_h)]
        completions = self._completions_for_rewards(examples, ids_h, completion_ids_list)
        prompts = [copy.deepcopy(x.get("prompt")) for x in examples]  # original_prompts (:1508-1511)
        keys = [k for k in examples[0] if k not in ("prompt", "completion", "completion_ids")]
        kw = {k: [x[k] for x in examples] for k in keys}
        kw["trainer_state"] = self.state
        conversational = self._is_conversational(examples[0])
        for i, (fn, rtok) in enumerate(zip(self.reward_funcs, self.reward_processing_classes)):
            if isinstance(fn, (RewardModel, torch.nn.Module)):
                if rtok is None:
                    raise ValueError("a reward model needs its reward_processing_class (tokenizer)")
                if conversational:
                    texts = [rtok.apply_chat_template(p + c, tokenize=False) for p, c in zip(prompts, completions)]
                else:
                    texts = [p + c for p, c in zip(prompts, completions)]
                enc = rtok(text=texts, return_tensors="pt", padding=True, padding_side="right",
                           add_special_tokens=False)
                dev = fn.device if isinstance(fn, RewardModel) else next(fn.parameters()).device
                enc = {k: v.to(dev) for k, v in enc.items()}
                with torch.inference_mode():
                    rpf[:, i] = fn(**enc).logits[:, 0].float().cpu()
            else:
                vals = fn(prompts=prompts, completions=completions, completion_ids=completion_ids_list, **kw)
                rpf[:, i] = torch.tensor([float("nan") if v is None else float(v) for v in vals],
                                         dtype=torch.float32)
        self._last_reward_inputs = {"prompts": prompts, "completions": completions}
        return rpf.to(self.device)

    # ------------------------------------------------------------------ scoring forward
    def _completion_logps(self, model: CausalLM, batch: dict, compute_entropy: bool):
        """grpo_trainer.py:1205-1272: forward over prompt+completion with
        logits_to_keep=C+1, drop the last position, /T, selective_log_softmax
        and entropy_from_logits — lm head + log-prob + entropy fused and
        row-chunked (engine/model.py `_LMHeadLogp`)."""
        grp = (self._prompt_groups(batch) if getattr(model, "supports_shared_prefix", False)
               and model.options.shared_prefix else None)
        if grp is not None:
            # the G copies of each prompt share one prompt forward (CausalLM.hidden_states_grouped)
            perm, G = grp
            cid = batch["completion_ids"][perm]
            padded = batch.get("_prompt_padded")
            h_last, h_comp = model.hidden_states_grouped(batch["prompt_ids"][perm], batch["prompt_mask"][perm], cid, G,
                                                         padded=None if padded is None else bool(padded.any()))
            R, C = cid.shape
            U, H = h_last.shape
            first = h_last[:, None, None].expand(U, G, 1, H).reshape(R, 1, H)  # predicts completion token 0
            lp, ent = model.logp_entropy(torch.cat([first, h_comp[:, :C - 1]], 1), cid, self.temperature,
                                         compute_entropy)
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(R, device=perm.device)
            return lp[inv], (ent[inv] if ent is not None else None)
        ids = torch.cat([batch["prompt_ids"], batch["completion_ids"]], 1)
        P = batch["prompt_ids"].shape[1]
        C = batch["completion_ids"].shape[1]
        key_mask = torch.cat([batch["prompt_mask"], torch.ones_like(batch["completion_ids"], dtype=torch.int32)], 1)
        h = model.hidden_states(ids, key_mask=key_mask)
        return model.logp_entropy(h[:, P - 1:P + C - 1], batch["completion_ids"], self.temperature, compute_entropy)

    @staticmethod
    def _prompt_groups(batch: dict):
        """(row order putting each prompt's rows consecutively, G) when every
        prompt of the batch appears exactly G >= 2 times (GRPO's generations of
        one prompt, in any shuffled order); None otherwise.  The order is the
        generation's (`row_index`): a training pass over a whole shuffled
        generation then runs every row at the position the generation-time
        scoring pass gave it, so both see the same GEMM / attention layout and
        produce the same bits whatever the kernels' row-position dependence."""
        # the trainer's batches carry host copies ("_" keys: no device sync); device ids are
        # read back once (tools / tests that build batches by hand)
        gid = batch.get("_prompt_group", batch.get("prompt_group"))
        key = batch.get("_row_index", batch.get("row_index"))
        if gid is None:
            return None
        gid = gid.cpu()
        order = torch.argsort(key.cpu()) if key is not None else None
        rows: dict = {}
        for r, g in enumerate((gid[order] if order is not None else gid).tolist()):
            rows.setdefault(g, []).append(r)
        sizes = {len(v) for v in rows.values()}
        if len(sizes) != 1 or sizes.pop() < 2:
            return None
        pos = torch.tensor([r for v in rows.values() for r in v])  # positions in the (sorted) sequence
        perm = order[pos] if order is not None else pos
        return perm.to(batch["completion_ids"].device, non_blocking=True), len(pos) // len(rows)

    @torch.no_grad()
    def _score_logps(self, model: CausalLM, batch: dict) -> torch.Tensor:
        saved, model.grad = model.grad, None
        try:
            lp, _ = self._completion_logps(model, batch, False)
        finally:
            model.grad = saved
        return lp

    # ------------------------------------------------------------------ loss over fused micro-batches
    def _loss_backward(self, micro: list[dict], train: bool = True, accum: Optional[int] = None) -> dict:
        """One forward/backward over the given micro-batches.  Segment j keeps
        micro-batch j's own normaliser (bnpo tokens / grpo rows), every row is
        scaled by 1/GA as the Trainer's loss division — the gradient equals the
        reference's GA separate backward passes (`accum`: the micro-batches of this
        update, fewer than GA at a short epoch end).  train=False: the evaluation
        loss (prediction_step, grpo_trainer.py:2177-2183: compute_loss under
        no_grad, no GA division), forward only."""
        a = self.args
        GA = (accum or a.gradient_accumulation_steps) if train else 1
        orig = micro
        R_each = [m["completion_ids"].shape[0] for m in micro]
        W = max(m["completion_ids"].shape[1] for m in micro)
        if any(m["completion_ids"].shape[1] != W for m in micro):  # rollouts of different widths (early stop)
            micro = [_pad_completions(m, W, self.pad_token_id) for m in micro]
        batch = {
            "prompt_ids": pad_left_cat([m["prompt_ids"] for m in micro], self.pad_token_id),
            "prompt_mask": pad_left_cat([m["prompt_mask"] for m in micro], 0),
            "completion_ids": torch.cat([m["completion_ids"] for m in micro]),
            "completion_mask": torch.cat([m["completion_mask"] for m in micro]),
            "advantages": torch.cat([m["advantages"] for m in micro]),
        }
        for k in ("prompt_group", "row_index", "_prompt_group", "_row_index", "_prompt_padded"):
            if all(k in m for m in micro):
                batch[k] = torch.cat([m[k] for m in micro])
        for k in ("old_per_token_logps", "ref_per_token_logps"):
            if any(k in m for m in micro):
                batch[k] = torch.cat([m[k] if k in m else torch.zeros(m["completion_ids"].shape, device=self.device)
                                      for m in micro])
        # micro-batches at their first use whose generation-time model is unchanged take their
        # old-policy / reference log-probs from this pass's own layout (_eager_scoring)
        take_old = [self._needs_old_logps() and "_gen_step" in m and int(m["_gen_step"]) == self.state.global_step
                    for m in orig]
        take_ref = [self.beta != 0.0 and "_ref_version" in m and int(m["_ref_version"]) == self._ref_version
                    for m in orig]
        rows = torch.cat([torch.full((r,), j, dtype=torch.int64) for j, r in enumerate(R_each)]).to(self.device)
        seg = rows.to(torch.int32)
        R = seg.numel()
        row_scale = torch.full((R,), 1.0 / GA, device=self.device)
        if any(take_ref):
            ref_lp = self._score_logps(self.ref_model, batch)
            batch["ref_per_token_logps"] = self._merge_rows(batch.get("ref_per_token_logps"), ref_lp, take_ref, rows)
        _trace("loss inputs ready")
        with torch.set_grad_enabled(train):
            if train:
                logp, ent = self._completion_logps(self.model, batch, True)
            else:  # no weight-gradient accumulation into the flat buffer
                saved, self.model.grad = self.model.grad, None
                try:
                    logp, ent = self._completion_logps(self.model, batch, True)
                finally:
                    self.model.grad = saved
        _trace("policy forward + lm head + logp/entropy")
        if any(take_old):
            batch["old_per_token_logps"] = self._merge_rows(batch.get("old_per_token_logps"), logp.detach(), take_old,
                                                            rows)
        # the buffered micro-batches keep what this pass scored for their later uses (num_iterations > 1)
        r0 = 0
        for j, (m, r) in enumerate(zip(orig, R_each)):
            w = m["completion_ids"].shape[1]
            if take_old[j]:
                m["old_per_token_logps"] = batch["old_per_token_logps"][r0:r0 + r, :w].clone()
            if take_ref[j]:
                m["ref_per_token_logps"] = batch["ref_per_token_logps"][r0:r0 + r, :w].clone()
            m.pop("_gen_step", None)
            m.pop("_ref_version", None)
            r0 += r
        emask = None
        if self.top_entropy_quantile < 1.0:
            # :2079-2082, per micro-batch (segment).  The reference thresholds the entropies
            # entropy_from_logits returns in the logits' dtype (utils.py:1465-1490): for a bf16
            # model those are bf16 values, whose ties decide which tokens sit at the quantile,
            # so the fp32 entropies of the fused kernel are rounded to the model dtype first
            from . import utils as _u
            ent_q = ent.to(self.model.dtype) if self.model.dtype != torch.float32 else ent
            emask = torch.zeros_like(batch["completion_mask"], dtype=torch.bool)
            for j in range(len(micro)):
                sl = seg == j
                emask[sl] = _u.get_high_entropy_mask(ent_q[sl], batch["completion_mask"][sl],
                                                     1 - self.top_entropy_quantile)
        kw = dict(old_per_token_logps=batch.get("old_per_token_logps"),
                  ref_per_token_logps=batch.get("ref_per_token_logps"), entropy_mask=emask, entropies=ent,
                  row_scale=row_scale, segments=seg, num_segments=len(micro), beta=self.beta,
                  epsilon_low=self.epsilon_low, epsilon_high=self.epsilon_high, delta=a.delta,
                  loss_type=self.loss_type, importance_sampling_level=self.importance_sampling_level,
                  max_completion_length=self.max_completion_length, segment_metrics=True)
        if not train:
            loss, _, metrics = ops.grpo_loss_fwd_bwd(logp, batch["advantages"], batch["completion_mask"],
                                                     need_grad=False, **kw)
            return {"loss": loss[0], "metrics": metrics}
        loss, metrics = ops.grpo_loss(logp, batch["advantages"], batch["completion_mask"], **kw)
        _trace("loss")
        loss.backward()
        dw_sync(self.device)  # the weight-gradient side stream joins the compute stream
        _trace("backward")
        return {"loss": loss.detach(), "metrics": metrics}

    @staticmethod
    def _merge_rows(prev: Optional[torch.Tensor], new: torch.Tensor, take: list, rows: torch.Tensor) -> torch.Tensor:
        """Rows of micro-batch j from `new` where take[j], else from `prev`."""
        if all(take) or prev is None:
            return new.float()
        sel = torch.tensor(take, device=new.device)[rows]
        return torch.where(sel[:, None], new.float(), prev)

    # ------------------------------------------------------------------ the loop
    def _next_micro_batch(self) -> dict:
        """grpo_trainer.py:1411-1444 (_prepare_inputs, train mode)."""
        a = self.args
        generate_every = a.steps_per_generation * self.num_iterations
        if self._step % generate_every == 0 or self._buffered_inputs is None:
            if self._batches is None:
                self._batches = self._generation_batches()
                for _ in range(self._gen_count):  # resumed: skip the batches already trained on
                    next(self._batches)
            gen = self._generate_and_score_completions(next(self._batches))
            n = gen["completion_ids"].shape[0]
            perm_h = torch.randperm(n, generator=self._shuffle_gen)
            perm = perm_h.to(self.device)
            gen = {k: v[perm_h if v.device.type == "cpu" else perm] for k, v in gen.items()}
            self._buffered_inputs = [self._mark_fresh(mb, "train") for mb in split_tensor_dict(gen, a.steps_per_generation)]
        inputs = self._buffered_inputs[self._step % a.steps_per_generation]
        self._step += 1
        return inputs

    def _bucket_release(self, ar, bucket_bytes: int = 100 << 20):
        """Layer-completion callback for OverlappedAllReduce: layers finish in
        reverse order; a bucket of consecutive layers (>= bucket_bytes) is
        released when its lowest layer is done, the last at layer 0."""
        m = self.model
        state = {"hi": None}

        def cb(i: int):
            s, e = m.layer_range(i)
            if state["hi"] is None:
                state["hi"] = e
            if (state["hi"] - s) * m.flat.element_size() >= bucket_bytes or i == 0:
                ar.release(s, state["hi"])
                state["hi"] = None
        return cb

    def training_step_group(self) -> dict:
        """One optimizer step: GA micro-batches (fused), DP all-reduce, clip, AdamW.
        The last update of an epoch takes the remaining micro-batches when the epoch's
        count is not a multiple of GA, its loss divided by their number (transformers
        Trainer._run_epoch: `remainder`, current_gradient_accumulation_steps)."""
        a = self.args
        GA = self._update_size(self._step)
        self.model.zero_grad()
        micro = [self._next_micro_batch() for _ in range(GA)]
        outs = []
        tokens = sum(m["completion_ids"].shape[0] * (m["prompt_ids"].shape[1] + m["completion_ids"].shape[1])
                     for m in micro)
        # DP: each layer's gradient all-reduce starts as soon as the (last) backward
        # pass has finished that layer, overlapped with the rest of the backward
        ar = swh_dist.OverlappedAllReduce(self.model.grad, dw_streams(self.device)) if self.world > 1 else None
        groups = [micro] if (a.fuse_micro_batches and tokens <= a.fuse_token_budget) else [[m] for m in micro]
        for gi, grp in enumerate(groups):
            if ar is not None and gi == len(groups) - 1:
                self.model.on_layer_grads = self._bucket_release(ar)
            try:
                outs.append(self._loss_backward(grp, accum=GA))
            finally:
                self.model.on_layer_grads = None
        if ar is not None:
            ar.finish()
        lr = self._current_lr()
        self.control = self.callback_handler.call("on_pre_optimizer_step")
        norm = self.optimizer.step(self.model.grad, model_out=self.model.flat, lr=lr)
        self.control = self.callback_handler.call("on_optimizer_step")
        self.state.global_step += 1
        _trace(f"optimizer step {self.state.global_step}")
        if self.ref_model is not None and a.sync_ref_model and self.state.global_step % a.ref_model_sync_steps == 0:
            # TR-DPO mixup (callbacks.py:106-131): ref = alpha * policy + (1 - alpha) * ref
            sync_ref_model(self.ref_model.flat, self.model.flat, a.ref_model_mixup_alpha)
            self._ref_version += 1
        loss = sum(o["loss"] for o in outs) if len(outs) > 1 else outs[0]["loss"]
        if len(outs) > 1:
            loss = loss  # per-micro losses already carry the 1/GA row scale
        m = self._metrics["train"]
        m["_loss"].append(loss)
        # one row of metric sums per GA micro-batch (the loss kernel's segments)
        m["_met"].append(torch.cat([o["metrics"][1:] for o in outs]))
        m["_grad_norm"].append(norm.clone())
        return {"loss": loss, "grad_norm": norm}

    def _flush_logs(self) -> dict:
        """GRPOTrainer.log (grpo_trainer.py:2185-2196) of a training interval:
        every metric list averaged since the last log (`_metric_averages`),
        with the Trainer's loss, grad_norm and learning_rate (the scheduler's
        last lr, i.e. the rate of the next step, as transformers logs it)."""
        log = self._metric_averages("train")
        if not log:
            return {}
        log["step"] = self.state.global_step
        self.state.log_history.append(log)
        return log

    def _metric_averages(self, mode: str) -> dict:
        """The metrics of `mode` averaged since the last log.  The per-rank
        quantities are gathered across ranks as the reference gathers them —
        completion lengths and EOS flags (:1945-1960), token counts (:1942), the
        per-micro-batch masked means of KL / entropy / clip ratios (:2143-2174,
        nanmean / nanmin / nanmax over ranks) and the loss (transformers'
        Trainer gathers tr_loss) — in one host sync per log.  Eval keys carry
        the "eval_" prefix (:2191-2192)."""
        m = self._metrics[mode]
        if not m.get("_met"):
            return {}
        gather = swh_dist.all_gather_rows
        world = self.world
        n_gen = len(m["_lengths"])  # 0 when no rollout fell in this log interval (spg * mu > GA)
        seg = gather(torch.cat(m["_met"])).cpu()                # [world * n_micro, 8]
        lens = gather(torch.cat(m["_lengths"])).cpu() if n_gen else None  # [world * n_gen * B, 2]
        log = {}
        if mode == "train":
            losses = gather(torch.stack(m["_loss"]).view(-1, 1).float()).cpu()
            self._count_tokens()
            log = {"loss": float(losses.view(world, -1).mean(0).mean()),
                   "grad_norm": float(torch.stack(m["_grad_norm"]).mean()),
                   "learning_rate": self._lr_at(self.state.global_step)}
        log["num_tokens"] = self.state.num_input_tokens_seen
        n_micro = seg.shape[0] // world
        seg = seg.view(world, n_micro, 8)
        tok = seg[..., 0].clamp(min=1.0)  # completion_token_count = mask.sum().clamp(min=1.0) (:2142)
        rows = seg[..., 6]
        clip_den = rows if self.importance_sampling_level == "sequence" else tok

        def over_ranks(x):  # [world, n_micro]: nanmean over ranks per micro-batch, then the log's mean
            return float(torch.nanmean(x, 0).mean())

        def nanmin(x):
            return torch.stack([c[~c.isnan()].min() if (~c.isnan()).any() else torch.tensor(float("nan"))
                                for c in x.t()])

        def nanmax(x):
            return torch.stack([c[~c.isnan()].max() if (~c.isnan()).any() else torch.tensor(float("nan"))
                                for c in x.t()])

        # completions (:1945-1960), one entry per generation, averaged
        B = lens.shape[0] // (world * n_gen) if n_gen else 0
        per_gen = lens.view(world, n_gen, B, 2).transpose(0, 1).reshape(n_gen, world * B, 2) if n_gen else []
        agg = {k: [] for k in ("mean_length", "min_length", "max_length", "clipped_ratio", "mean_terminated_length",
                               "min_terminated_length", "max_terminated_length")}
        for g in per_gen:
            ln, eos = g[:, 0], g[:, 1].bool()
            term = ln[eos] if bool(eos.any()) else torch.zeros(1)
            agg["mean_length"].append(float(ln.mean()))
            agg["min_length"].append(float(ln.min()))
            agg["max_length"].append(float(ln.max()))
            agg["clipped_ratio"].append(1.0 - float(eos.sum()) / ln.numel())
            agg["mean_terminated_length"].append(float(term.mean()))
            agg["min_terminated_length"].append(float(term.min()))
            agg["max_terminated_length"].append(float(term.max()))
        for k, v in agg.items():
            if v:
                log[f"completions/{k}"] = sum(v) / len(v)
        # rewards (global after the gather at :1497), one entry per generation
        for i, name in enumerate(self.reward_func_names if n_gen else []):
            means = [float(torch.nanmean(r[:, i].cpu())) for r in m["_rpf"]]
            stds = []
            for r in m["_rpf"]:
                col = r[:, i].cpu()
                col = col[~col.isnan()]
                stds.append(float(col.std()) if col.numel() > 1 else float("nan"))
            log[f"rewards/{name}/mean"] = sum(means) / len(means)
            log[f"rewards/{name}/std"] = sum(stds) / len(stds)
        if n_gen:
            log["reward"] = sum(float(x.mean()) for x in m["_rewards"]) / n_gen
            log["reward_std"] = sum(float(x.mean()) for x in m["_reward_std"]) / n_gen
            log["frac_reward_zero_std"] = sum(float(x.mean()) for x in m["_zero_std"]) / n_gen
        # loss metrics (:2139-2174): per micro-batch masked means, gathered over ranks
        if self.beta != 0.0:
            log["kl"] = over_ranks(seg[..., 1] / tok)
        log["entropy"] = over_ranks(seg[..., 2] / tok)
        low, high, region = seg[..., 3] / clip_den, seg[..., 4] / clip_den, seg[..., 5] / clip_den
        log["clip_ratio/low_mean"] = over_ranks(low)
        log["clip_ratio/low_min"] = float(nanmin(low).mean())
        log["clip_ratio/high_mean"] = over_ranks(high)
        log["clip_ratio/high_max"] = float(nanmax(high).mean())
        log["clip_ratio/region_mean"] = over_ranks(region)
        m.clear()
        if mode == "eval":
            log = {f"eval_{k}": v for k, v in log.items()}
        return log

    def _count_tokens(self):
        """Fold the pending per-generation attention-mask token counts of every
        rank into state.num_input_tokens_seen (grpo_trainer.py:1942: the gathered
        sum of prompt + completion mask tokens); one gather."""
        m = self._metrics["train"]
        if m.get("_tokens"):
            self.state.num_input_tokens_seen += int(swh_dist.all_gather_rows(torch.cat(m["_tokens"])).sum())
            m["_tokens"] = []

    # ------------------------------------------------------------------ checkpoints
    def save_model(self, output_dir: Optional[str] = None, _internal_call: bool = False):
        """Trainer.save_model: the policy in transformers layout (config.json +
        safetensors) and the tokenizer, on the main process."""
        from . import checkpoint as ck
        out = output_dir or self.args.output_dir
        if out is None:
            raise ValueError("save_model needs an output_dir")
        if self.rank == 0:
            ck.save_pretrained(self.model, out, eos_token_id=self.eos_token_id, pad_token_id=self.pad_token_id)
            if self.processing_class is not None and hasattr(self.processing_class, "save_pretrained"):
                self.processing_class.save_pretrained(out)
        swh_dist.barrier()

    def create_model_card(self, model_name: Optional[str] = None, dataset_name: Optional[str] = None, tags=None):
        """grpo_trainer.py:2243-2306: README.md model card in output_dir."""
        from . import checkpoint as ck
        if self.rank != 0 or not self.args.output_dir:
            return
        tags = set([tags] if isinstance(tags, str) else (tags or []))
        tags.update(self._tag_names)
        os.makedirs(self.args.output_dir, exist_ok=True)
        with open(os.path.join(self.args.output_dir, "README.md"), "w") as f:
            f.write(ck.model_card("GRPO", model_name or os.path.basename(os.path.normpath(self.args.output_dir)),
                                  "DeepSeekMath, arXiv:2402.03300", ck.GRPO_CITATION, tags))

    def _save_checkpoint(self, model=None, trial=None):
        """grpo_trainer.py:2234-2241 + transformers Trainer._save_checkpoint:
        output_dir/checkpoint-<global_step>/ with model, optimizer, scheduler,
        trainer state and RNG/data-stream state (exact resume)."""
        import json

        from . import checkpoint as ck
        a = self.args
        name = a.hub_model_id.split("/")[-1] if a.hub_model_id else os.path.basename(os.path.normpath(a.output_dir))
        self.create_model_card(model_name=name)
        d = os.path.join(a.output_dir, f"checkpoint-{self.state.global_step}")
        self._count_tokens()  # every rank: a gather
        self.save_model(d)  # rank 0 creates d; ends in a barrier
        if not a.save_only_model:
            # every rank its own data-stream state: its shuffle generator and buffered
            # rollouts differ (transformers: rng_state_<process_index>.pth)
            torch.save(self._resume_state(), os.path.join(d, ck.trainer_state_file(self.rank)))
        if self.rank == 0:
            if not a.save_only_model:
                torch.save(ck.optimizer_state_dict(self.model, self.optimizer, a.weight_decay),
                           os.path.join(d, "optimizer.pt"))
                torch.save(ck.scheduler_state_dict(self.state.global_step, a.learning_rate, self._schedule()),
                           os.path.join(d, "scheduler.pt"))
                ck.save_master(self.optimizer, d)
                if self.ref_model is not None and a.sync_ref_model:  # the mixed reference is trainer state
                    from safetensors.torch import save_file
                    save_file({"ref": self.ref_model.flat.detach().cpu()}, os.path.join(d, "swh_ref.safetensors"))
            with open(os.path.join(d, "trainer_state.json"), "w") as f:
                json.dump(ck.trainer_state_json(self.state, a, a.per_device_train_batch_size), f, indent=2)
            ck.rotate_checkpoints(a.output_dir, a.save_total_limit)
        swh_dist.barrier()
        return d

    def _schedule(self):
        """The LambdaLR multiplier of transformers get_scheduler for the config's
        lr_scheduler_type / lr_scheduler_kwargs / warmup over max_steps (schedule.py)."""
        total = max(1, self.state.max_steps)
        key = (total, self.args.lr_scheduler_type)
        if getattr(self, "_sched_key", None) != key:
            self._sched_fn, self._sched_key = schedule.for_args(self.args, total), key
        return self._sched_fn

    def _lr_at(self, step: int) -> float:
        return self.args.learning_rate * self._schedule()(step)

    def _current_lr(self) -> float:
        """The rate of the next optimizer step: the Trainer steps the scheduler after
        the optimizer, so step k (0-based) uses lr * lambda(k)."""
        return self._lr_at(self.state.global_step)

    def _resume_state(self) -> dict:
        """Tensors only (loaded with weights_only=True): the data-stream position,
        the shuffle generator, the rollouts still buffered for the next steps."""
        st = {"gen_count": torch.tensor(self._gen_count), "micro_step": torch.tensor(self._step),
              "ref_version": torch.tensor(self._ref_version),
              "shuffle_gen": self._shuffle_gen.get_state(), "global_step": torch.tensor(self.state.global_step),
              "tokens_seen": torch.tensor(self.state.num_input_tokens_seen)}
        if self._buffered_inputs is not None:
            for i, mb in enumerate(self._buffered_inputs):
                for k, v in mb.items():
                    if v is not None:
                        st[f"buf.{i}.{k}"] = v.detach().cpu()
        return st

    def _load_checkpoint(self, d: str):
        import json

        from . import checkpoint as ck
        if os.path.exists(os.path.join(d, "swh_master.safetensors")):
            from safetensors.torch import load_file
            self.optimizer.master.copy_(load_file(os.path.join(d, "swh_master.safetensors"))["master"])
            self.model.flat.copy_(self.optimizer.master)
        else:  # a transformers checkpoint: the saved weights are the master
            ck.load_weights_into(self.model, d)
            self.optimizer.master.copy_(self.model.flat.float())
        ref_path = os.path.join(d, "swh_ref.safetensors")
        if self.ref_model is not None and self.args.sync_ref_model and os.path.exists(ref_path):
            from safetensors.torch import load_file
            self.ref_model.flat.copy_(load_file(ref_path)["ref"])
        opt_path = os.path.join(d, "optimizer.pt")
        if os.path.exists(opt_path):
            ck.load_optimizer_state_dict(self.model, self.optimizer, torch.load(opt_path, weights_only=True))
        with open(os.path.join(d, "trainer_state.json")) as f:
            js = json.load(f)
        self.state.global_step = int(js["global_step"])
        self.state.log_history = list(js.get("log_history", []))
        self.state.num_input_tokens_seen = int(js.get("num_input_tokens_seen", 0))
        sp = os.path.join(d, ck.trainer_state_file(self.rank))
        if not os.path.exists(sp) and any(f.startswith("swh_trainer_state_") for f in os.listdir(d)):
            raise ValueError(f"{d}: no {ck.trainer_state_file(self.rank)} (checkpoint saved by fewer ranks); the "
                             "exact-resume state is per rank")
        legacy = os.path.join(d, ck.LEGACY_TRAINER_STATE)
        if not os.path.exists(sp) and os.path.exists(legacy):
            # written by a single-rank run before the state became per rank
            if self.world != 1:
                raise ValueError(f"{d}: holds the single-rank exact-resume state {ck.LEGACY_TRAINER_STATE}; it "
                                 f"cannot resume a {self.world}-rank run")
            sp = legacy
        if os.path.exists(sp):
            st = torch.load(sp, weights_only=True)
            self._gen_count = int(st["gen_count"])
            self._step = int(st["micro_step"])
            self._ref_version = int(st.get("ref_version", 0))
            self._shuffle_gen.set_state(st["shuffle_gen"])
            bufs = {}
            for k, v in st.items():
                if k.startswith("buf."):
                    _, i, name = k.split(".", 2)
                    bufs.setdefault(int(i), {})[name] = v if name.startswith("_") else v.to(self.device)
            self._buffered_inputs = [bufs[i] for i in sorted(bufs)] if bufs else None
        else:  # transformers checkpoint: position from the step count
            self._gen_count = self.state.global_step * self.args.gradient_accumulation_steps // (
                self.args.steps_per_generation * self.num_iterations)
            self._step = self.state.global_step * self.args.gradient_accumulation_steps
        self._batches = None

    def _total_steps(self) -> int:
        """transformers Trainer.set_initial_training_values: max_steps, or
        ceil(num_train_epochs x optimizer steps per epoch)."""
        a = self.args
        if a.max_steps and a.max_steps > 0:
            return a.max_steps
        return max(1, int(math.ceil(self._steps_per_epoch() * a.num_train_epochs)))

    def _micro_steps_per_epoch(self) -> int:
        """len(train dataloader) per rank: the RepeatSampler's generation batches
        (grpo_trainer.py:1096-1130) times their repeat count spg x num_iterations, at
        batch size per_device x spg (:1075) — one training_step each."""
        a = self.args
        n_gen = len(self.train_dataset) // (a.generation_batch_size // self.num_generations)
        return n_gen * a.steps_per_generation * self.num_iterations

    def _steps_per_epoch(self) -> int:
        """Optimizer steps per epoch: ceil(micro-steps / GA) (the Trainer's last
        update of an epoch takes the remainder)."""
        GA = self.args.gradient_accumulation_steps
        return max(1, -(-self._micro_steps_per_epoch() // GA))

    def _epoch_micro_steps(self) -> Optional[int]:
        """Micro-steps per epoch, None without a training dataset (no epochs)."""
        return self._micro_steps_per_epoch() if self.train_dataset is not None else None

    def _update_size(self, k: int) -> int:
        """Micro-batches of the update that starts at micro-step k: GA, or the epoch's
        remainder for its last update (transformers Trainer._run_epoch)."""
        GA, mse = self.args.gradient_accumulation_steps, self._epoch_micro_steps()
        if not mse:
            return GA
        return min(GA, mse - k % mse)

    def _update_index(self, k: int) -> int:
        """The optimizer step (0-based, since training began) micro-step k belongs to."""
        GA, mse = self.args.gradient_accumulation_steps, self._epoch_micro_steps()
        if not mse:
            return k // GA
        return (k // mse) * (-(-mse // GA)) + (k % mse) // GA

    @staticmethod
    def _interval(x, total: int) -> int:
        """TrainingArguments logging/save/eval steps: an int, or a fraction of max_steps (rounded up)."""
        return int(x) if x >= 1 else max(1, math.ceil(total * x))

    def train(self, resume_from_checkpoint=None, trial=None, ignore_keys_for_eval=None, **kwargs):
        """transformers Trainer.train / _inner_training_loop around the GRPO step:
        callbacks (callbacks.py) with DefaultFlowCallback's log / evaluate / save
        decisions, evaluation on eval_dataset (eval_strategy "steps"), and the
        final train summary log.  Returns transformers' TrainOutput
        (global_step, training_loss, metrics)."""
        a = self.args
        if self.train_dataset is None:
            raise ValueError("train_dataset is required")
        if resume_from_checkpoint:
            from . import checkpoint as ck
            d = ck.latest_checkpoint(a.output_dir) if resume_from_checkpoint is True else resume_from_checkpoint
            if d is None:
                raise ValueError(f"No valid checkpoint found in output directory ({a.output_dir})")
            self._load_checkpoint(d)
        total = self._total_steps()
        st = self.state
        st.max_steps = total
        st.num_train_epochs = int(math.ceil(total / self._steps_per_epoch()))
        st.logging_steps = log_every = self._interval(a.logging_steps, total)
        st.save_steps = save_every = self._interval(a.save_steps, total)
        st.eval_steps = eval_every = self._interval(a.eval_steps if a.eval_steps is not None else a.logging_steps,
                                                    total)
        st.train_batch_size = a.per_device_train_batch_size
        if a.eval_strategy == "steps" and self.eval_dataset is None:
            raise ValueError("eval_strategy='steps' requires an eval_dataset")
        cb = self.callback_handler
        start_step, t0 = st.global_step, time.time()
        self.control = cb.call("on_train_begin")
        if a.eval_on_start and self.eval_dataset is not None:
            self.evaluate()
        self.control = cb.call("on_epoch_begin")
        loss_sum = torch.zeros((), device=self.device)
        while st.global_step < total and not self.control.should_training_stop:
            self.control = cb.call("on_step_begin")
            out = self.training_step_group()
            loss_sum += out["loss"].detach().float()
            st.epoch = self._step / self._micro_steps_per_epoch()  # Trainer: epoch + (step + 1) / steps_in_epoch
            # DefaultFlowCallback.on_step_end, then the user's callbacks may change the decisions
            c, gs = self.control, st.global_step
            if (gs == 1 and a.logging_first_step) or gs % log_every == 0:
                c.should_log = True
            if a.eval_strategy == "steps" and gs % eval_every == 0:
                c.should_evaluate = True
            if a.save_strategy == "steps" and gs % save_every == 0:
                c.should_save = True
            if gs >= total:
                c.should_training_stop = True
                if a.eval_strategy == "steps" and gs % eval_every != 0:
                    c.should_evaluate = True
                if a.save_strategy == "steps":
                    c.should_save = True
            self.control = cb.call("on_step_end")
            self._maybe_log_save_evaluate(t0)
        self.control = cb.call("on_epoch_end")
        self._maybe_log_save_evaluate(t0)
        runtime = time.time() - t0
        steps_done = st.global_step - start_step
        train_loss = float(loss_sum) / max(1, steps_done)
        n_samples = steps_done * a.generation_batch_size * self.num_iterations // max(1, a.steps_per_generation)
        metrics = {"train_runtime": round(runtime, 4), "train_samples_per_second": round(n_samples / runtime, 3),
                   "train_steps_per_second": round(steps_done / runtime, 3), "total_flos": 0.0,
                   "train_loss": train_loss}
        self._log(metrics)  # GRPOTrainer.log merges whatever metrics are still pending (:2185-2196)
        self.control = cb.call("on_train_end")
        try:
            from transformers.trainer_utils import TrainOutput
            return TrainOutput(st.global_step, train_loss, metrics)
        except ImportError:  # pragma: no cover
            return st.global_step, train_loss, metrics

    def _log(self, logs: dict) -> dict:
        """GRPOTrainer.log + Trainer.log: pending training metrics merged in, epoch and
        step added, appended to log_history, printed on the main process, on_log."""
        pending = self._metric_averages("train")
        logs = {**logs, **pending}
        if self.state.epoch is not None:
            logs["epoch"] = self.state.epoch
        logs["step"] = self.state.global_step
        self.state.log_history.append(logs)
        if self.rank == 0:
            print(logs, flush=True)
        self.control = self.callback_handler.call("on_log", logs=logs)
        return logs

    def _maybe_log_save_evaluate(self, t0: float):
        c = self.control
        if c.should_log:
            pending = self._metric_averages("train")
            if pending:
                pending["train_runtime"] = time.time() - t0
                self._log(pending)
            else:
                c.should_log = False
        if self.control.should_evaluate:
            self.evaluate()
        if self.control.should_save:
            if self.args.output_dir:
                self._save_checkpoint()
            self.control = self.callback_handler.call("on_save")

    # ------------------------------------------------------------------ evaluation (Trainer.evaluate)
    def _eval_batches(self, dataset):
        """Local evaluation batches: RepeatSampler(eval_dataset, mini_repeat_count=G,
        seed) (:1132-1138) in global batches of per_device_eval_batch_size x world,
        each rank its contiguous slice (accelerate sharding; a short last batch
        is completed from the start, as accelerate's even_batches does)."""
        a = self.args
        idx = list(RepeatSampler(range(len(dataset)), mini_repeat_count=self.num_generations, seed=a.seed))
        gb = a.per_device_eval_batch_size * self.world
        if gb % self.num_generations:
            raise ValueError(f"The global eval batch size ({self.world} x {a.per_device_eval_batch_size}) must be "
                             f"divisible by the number of generations per prompt ({self.num_generations}).")
        for s in range(0, len(idx), gb):
            chunk = idx[s:s + gb]
            if len(chunk) < gb:
                chunk = chunk + idx[:gb - len(chunk)]
            mine = chunk[self.rank * a.per_device_eval_batch_size:(self.rank + 1) * a.per_device_eval_batch_size]
            yield [dataset[i] for i in mine]

    @torch.no_grad()
    def evaluate(self, eval_dataset=None, ignore_keys=None, metric_key_prefix: str = "eval") -> dict:
        """Trainer.evaluate with GRPO's prediction_step (grpo_trainer.py:2177-2183):
        each local eval batch is generated and scored (no buffering, no
        iterations, :1440-1443), its loss computed under no_grad; eval_loss is
        the batch-size-weighted mean over every rank's batches, and the eval
        metrics of _generate_and_score_completions / _compute_loss are logged
        with the "eval_" prefix.  A dict of datasets is evaluated per entry
        with the prefix eval_<name>."""
        ds = eval_dataset if eval_dataset is not None else self.eval_dataset
        if ds is None:
            raise ValueError("Trainer: evaluation requires an eval_dataset.")
        if isinstance(ds, dict):
            out = {}
            for name, d in ds.items():
                out.update(self.evaluate(d, ignore_keys, f"{metric_key_prefix}_{name}"))
            return out
        t0 = time.time()
        losses, sizes = [], []
        n = 0
        for examples in self._eval_batches(ds):
            gen = self._mark_fresh(self._generate_and_score_completions(examples, mode="eval"), "eval")
            out = self._loss_backward([gen], train=False)
            m = self._metrics["eval"]
            m["_met"].append(out["metrics"][1:])
            losses.append(out["loss"].view(1).float())
            sizes.append(float(len(examples)))
            n += len(examples)
        loss_rows = torch.stack([torch.cat(losses), torch.tensor(sizes, device=self.device)], 1)
        allr = swh_dist.all_gather_rows(loss_rows).cpu()
        runtime = time.time() - t0
        steps = len(losses)
        metrics = {f"{metric_key_prefix}_loss": float((allr[:, 0] * allr[:, 1]).sum() / allr[:, 1].sum()),
                   f"{metric_key_prefix}_runtime": round(runtime, 4),
                   f"{metric_key_prefix}_samples_per_second": round(n * self.world / runtime, 3),
                   f"{metric_key_prefix}_steps_per_second": round(steps / runtime, 3)}
        avg = self._metric_averages("eval")
        metrics.update({metric_key_prefix + k[len("eval"):]: v for k, v in avg.items()})
        if self.state.epoch is not None:
            metrics["epoch"] = self.state.epoch
        log = dict(metrics, step=self.state.global_step)
        self.state.log_history.append(log)
        if self.rank == 0:
            print(log, flush=True)
        self.control = self.callback_handler.call("on_log", logs=log)
        self.control = self.callback_handler.call("on_evaluate", metrics=metrics)
        return metrics
