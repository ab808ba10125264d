"""PPOConfig — field names and defaults of trl/trainer/ppo_config.py:22-135 and
the OnPolicyConfig it extends (trl/trainer/utils.py:744-870), plus the
TrainingArguments fields the loop reads.  The derived batch sizes
(`local_batch_size`, `mini_batch_size`, ... ) are filled by PPOTrainer exactly
as ppo_trainer.py:228-250 does.  Other TrainingArguments keywords are accepted
only where they cannot change the result (trainer/training_args.py, kept in
`extra`) and raise otherwise."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Optional

from .training_args import split_known


@dataclass
class PPOConfig:
    # TrainingArguments subset
    output_dir: Optional[str] = None
    per_device_train_batch_size: int = 8
    per_device_eval_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    num_train_epochs: float = 3.0
    learning_rate: float = 5e-5
    weight_decay: float = 0.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    lr_scheduler_type: str = "linear"
    lr_scheduler_kwargs: Optional[dict] = None
    warmup_steps: float = 0
    warmup_ratio: float = 0.0
    logging_steps: float = 10              # OnPolicyConfig (utils.py:759)
    eval_steps: Optional[float] = None
    save_steps: float = 500
    save_strategy: str = "steps"           # "steps" | "no" (TrainingArguments)
    save_total_limit: Optional[int] = None
    seed: int = 42
    bf16: Optional[bool] = None            # OnPolicyConfig: not fp16 when unset (utils.py:870-873)
    fp16: bool = False
    report_to: Any = None
    # OnPolicyConfig (utils.py:744-870)
    run_name: Optional[str] = None
    dataset_num_proc: Optional[int] = None
    num_mini_batches: int = 1
    total_episodes: Optional[int] = None
    local_rollout_forward_batch_size: int = 64
    num_sample_generations: int = 10
    response_length: int = 53
    stop_token: Optional[str] = None
    stop_token_id: Optional[int] = None
    temperature: float = 0.7
    missing_eos_penalty: Optional[float] = None
    sft_model_path: str = "EleutherAI/pythia-160m"
    world_size: Optional[int] = None
    num_total_batches: Optional[int] = None
    micro_batch_size: Optional[int] = None
    local_batch_size: Optional[int] = None
    batch_size: Optional[int] = None
    local_mini_batch_size: Optional[int] = None
    mini_batch_size: Optional[int] = None
    push_to_hub: bool = False
    # PPOConfig (ppo_config.py:22-135)
    exp_name: str = "ppo_config"
    reward_model_path: str = "EleutherAI/pythia-160m"
    model_adapter_name: Optional[str] = None
    ref_adapter_name: Optional[str] = None
    num_ppo_epochs: int = 4
    whiten_rewards: bool = False
    kl_coef: float = 0.05
    kl_estimator: str = "k1"
    cliprange: float = 0.2
    vf_coef: float = 0.1
    cliprange_value: float = 0.2
    gamma: float = 1.0
    lam: float = 0.95
    ds3_gather_for_generation: bool = True
    # engine knobs (not in the reference)
    model_init_kwargs: Optional[dict] = None  # {"torch_dtype": "float32"}: reference precision for models built
    #                                           from names / configs (model objects keep their own dtype)
    decode_early_exit: bool = True         # stop decoding once every row has finished (HF _sample), no per-token sync
    decode_check_every: int = 0            # legacy synchronous all-finished poll every k steps (0 = off)
    fuse_micro_batches: bool = True        # a mini-batch's GA micro-batches as one forward/backward
    fuse_token_budget: int = 1 << 16       # max rows * (query + response) tokens per fused pass
    pad_token_id: Optional[int] = None     # token ids when no tokenizer object is given (processing_class None)
    eos_token_id: Optional[int] = None
    extra: dict = field(default_factory=dict)

    def __init__(self, **kwargs):
        # the PPO loop logs every update and never runs Trainer.evaluate (ppo_trainer.py:646-659)
        extra = split_known(type(self), kwargs, frozenset({"eval_strategy", "evaluation_strategy", "eval_on_start",
                                                           "logging_first_step", "max_steps"}))
        for name, f in self.__dataclass_fields__.items():
            if name != "extra":
                setattr(self, name, kwargs.get(name, f.default))
        self.extra = extra
        self.__post_init__()

    def __post_init__(self):
        if self.fp16:
            raise ValueError("fp16=True: the MI355X engine trains bf16 (or fp32) models; fp16 mixed precision is "
                             "not implemented")
        self.save_strategy = getattr(self.save_strategy, "value", self.save_strategy)
        if self.save_strategy not in ("no", "steps"):
            raise ValueError(f"save_strategy {self.save_strategy!r}: the MI355X trainer saves on 'steps' (or 'no')")
        if self.push_to_hub:
            raise ValueError("push_to_hub=True: no hub access from the MI355X trainer")
        self.bf16 = (not self.fp16) if self.bf16 is None else self.bf16
        if self.output_dir is None:
            self.output_dir = "trainer_output"

    def to_dict(self) -> dict:
        return {k: getattr(self, k) for k in self.__dataclass_fields__}
