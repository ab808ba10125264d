"""GRPOConfig — field names and defaults of trl/trainer/grpo_config.py:227-616
(the subset that shapes the per-step hot path, plus the TrainingArguments
fields the loop reads).  Other TrainingArguments keywords are accepted only
where they cannot change the result (trainer/training_args.py: reporting,
hub, data-loader workers, ... kept in `extra`) and raise otherwise, e.g.
`optim="adafactor"`, `logging_strategy="epoch"`, `fp16=True`; vLLM / Liger
switches raise, as those paths are out of scope."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Optional

from ..dist import world_size_from_env as _world_size
from .training_args import split_known


@dataclass
class GRPOConfig:
    # TrainingArguments subset
    output_dir: Optional[str] = None
    per_device_train_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    num_train_epochs: float = 3.0
    max_steps: int = -1
    learning_rate: float = 1e-6            # grpo_config.py:227-230
    weight_decay: float = 0.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    max_grad_norm: float = 1.0
    lr_scheduler_type: str = "linear"
    lr_scheduler_kwargs: Optional[dict] = None
    warmup_steps: float = 0
    warmup_ratio: float = 0.0
    logging_steps: float = 10
    logging_first_step: bool = False
    per_device_eval_batch_size: int = 8
    eval_strategy: str = "no"              # "no" | "steps" (TrainingArguments)
    eval_steps: Optional[float] = None     # default: logging_steps
    eval_on_start: bool = False
    save_strategy: str = "steps"           # "steps" | "no" (TrainingArguments)
    save_steps: float = 500
    save_total_limit: Optional[int] = None
    save_only_model: bool = False
    hub_model_id: Optional[str] = None
    seed: int = 42
    bf16: Optional[bool] = None
    fp16: bool = False
    report_to: Any = None
    # model / data
    model_init_kwargs: Optional[dict] = None
    disable_dropout: bool = False
    remove_unused_columns: Optional[bool] = False
    max_prompt_length: Optional[int] = 512
    num_generations: Optional[int] = 8
    max_completion_length: Optional[int] = 256
    ds3_gather_for_generation: bool = True
    shuffle_dataset: Optional[bool] = True
    # generation
    generation_batch_size: Optional[int] = None
    steps_per_generation: Optional[int] = None
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: Optional[int] = None
    min_p: Optional[float] = None
    generation_kwargs: Optional[dict] = None
    repetition_penalty: float = 1.0
    use_transformers_paged: bool = False
    cache_implementation: Optional[str] = None
    use_vllm: bool = False
    vllm_mode: str = "server"
    # training
    beta: float = 0.0
    num_iterations: int = 1
    epsilon: float = 0.2
    delta: Optional[float] = None
    epsilon_high: Optional[float] = None
    importance_sampling_level: str = "token"
    reward_weights: Optional[list] = None
    scale_rewards: bool = True
    loss_type: str = "bnpo"
    mask_truncated_completions: bool = False
    sync_ref_model: bool = False
    ref_model_mixup_alpha: float = 0.6
    ref_model_sync_steps: int = 512
    top_entropy_quantile: float = 1.0
    use_liger_loss: bool = False
    # logging
    log_completions: bool = False
    num_completions_to_print: Optional[int] = None
    wandb_log_unique_prompts: Optional[bool] = False
    # MI355X engine knobs (no reference counterpart)
    fuse_micro_batches: bool = True        # run the GA micro-batches as one forward/backward
    fuse_token_budget: int = 1 << 17       # max rows*(P+C) tokens per fused pass
    decode_early_exit: bool = True         # stop decoding once every row has finished (HF _sample), no per-token sync
    decode_check_every: int = 0            # legacy synchronous all-finished poll every k steps (0 = off)
    extra: dict = field(default_factory=dict)

    def __init__(self, **kwargs):
        extra = split_known(type(self), kwargs, frozenset({"evaluation_strategy"}))
        for name, f in self.__dataclass_fields__.items():
            if name != "extra":
                setattr(self, name, kwargs.get(name, f.default))
        self.extra = extra
        self.__post_init__()

    def __post_init__(self):
        """grpo_config.py:574-616 batch bookkeeping and validation."""
        if self.fp16:
            raise ValueError("fp16=True: the MI355X engine trains bf16 (or fp32, model_init_kwargs torch_dtype) "
                             "models; fp16 mixed precision is not implemented")
        self.bf16 = (not self.fp16) if self.bf16 is None else self.bf16
        if self.use_vllm:
            raise ValueError("use_vllm=True: the vLLM generation path is out of scope; the device engine generates")
        if self.use_liger_loss:
            raise ValueError("use_liger_loss=True: the Liger (Triton) loss is out of scope; the fused HIP loss runs")
        if "evaluation_strategy" in self.extra:  # the older TrainingArguments name
            self.eval_strategy = self.extra.pop("evaluation_strategy")
        self.eval_strategy = getattr(self.eval_strategy, "value", self.eval_strategy)
        self.save_strategy = getattr(self.save_strategy, "value", self.save_strategy)
        if self.eval_strategy not in ("no", "steps"):
            raise ValueError(f"eval_strategy {self.eval_strategy!r}: the MI355X trainer evaluates on 'steps' (or 'no')")
        if self.save_strategy not in ("no", "steps"):
            raise ValueError(f"save_strategy {self.save_strategy!r}: the MI355X trainer saves on 'steps' (or 'no')")
        self.world_size = _world_size()
        n = self.world_size
        if self.generation_batch_size is None and self.steps_per_generation is None:
            self.steps_per_generation = self.gradient_accumulation_steps
            self.generation_batch_size = self.per_device_train_batch_size * n * self.steps_per_generation
        elif self.generation_batch_size is not None and self.steps_per_generation is None:
            if self.generation_batch_size % (self.per_device_train_batch_size * n) != 0:
                raise ValueError(f"generation_batch_size ({self.generation_batch_size}) must be divisible by the "
                                 f"global batch size ({self.per_device_train_batch_size * n}).")
            self.steps_per_generation = self.generation_batch_size // (self.per_device_train_batch_size * n)
        elif self.generation_batch_size is None and self.steps_per_generation is not None:
            self.generation_batch_size = self.per_device_train_batch_size * n * self.steps_per_generation
        else:
            raise ValueError("'generation_batch_size' and 'steps_per_generation' can not be both configured at the "
                             "same time")
        if self.generation_batch_size % self.num_generations != 0:
            raise ValueError(f"generation_batch_size ({self.generation_batch_size}) must be divisible by "
                             f"num_generations ({self.num_generations}).")
        if self.eval_strategy != "no":  # grpo_config.py: the eval batch must hold whole groups
            global_eval = self.per_device_eval_batch_size * n
            if global_eval % self.num_generations != 0:
                possible = [g for g in range(2, global_eval + 1) if global_eval % g == 0]
                raise ValueError(f"The global eval batch size ({n} x {self.per_device_eval_batch_size}) must be "
                                 f"divisible by the number of generations per prompt ({self.num_generations}). Given "
                                 f"the current eval batch size, the valid values for the number of generations are: "
                                 f"{possible}.")
        if self.num_generations < 2:
            raise ValueError("GRPO requires at least 2 generations per prompt to calculate the advantages. You "
                             f"provided {self.num_generations}, which is less than the minimum required.")
        if self.loss_type not in ("grpo", "bnpo", "dr_grpo"):
            raise ValueError(f"Unknown loss type: {self.loss_type}")
        if self.importance_sampling_level not in ("token", "sequence"):
            raise ValueError(f"Unknown importance sampling level: {self.importance_sampling_level}. Possible "
                             "values are 'token' and 'sequence'.")
