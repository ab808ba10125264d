"""The transformers `TrainingArguments` fields a reference GRPOConfig / PPOConfig
may carry beyond the ones the MI355X trainers implement.

The reference configs ARE TrainingArguments (trl/trainer/grpo_config.py:23,
trl/trainer/utils.py:744 OnPolicyConfig) and are handed whole to the
transformers Trainer (grpo_trainer.py:837-846), which acts on every field.
A drop-in may therefore only accept a field it does not implement when that
field cannot change what is trained or saved: reporting, hub, data-loader
workers, DDP plumbing, evaluation-loop bookkeeping that GRPO/PPO override.
Such fields are kept in `config.extra`.  A field whose value would change the
result is accepted only at the value under which it is inert (`CONSTRAINED`);
any other value, and any field in neither table, raises ValueError instead
of being silently ignored.  Both tables cover transformers 4.53 (the
reference's floor, setup.cfg:44-47) and the installed 5.x names.
"""
from __future__ import annotations

from typing import Any, Callable

# cannot change the trained weights, the log values or the checkpoint contents
INERT = frozenset({
    # reporting / logging sinks
    "report_to", "run_name", "project", "logging_dir", "disable_tqdm", "log_level", "log_level_replica",
    "log_on_each_node", "logging_nan_inf_filter", "include_num_input_tokens_seen", "include_tokens_per_second",
    "skip_memory_metrics", "trackio_space_id", "trackio_bucket_id", "trackio_static_space_id", "ray_scope",
    # hub (the trainer never pushes; `push_to_hub=True` is refused below)
    "hub_token", "hub_private_repo", "hub_strategy", "hub_always_push", "hub_revision", "push_to_hub_model_id",
    "push_to_hub_organization", "push_to_hub_token",
    # data loading (the prompt stream is RepeatSampler's, grpo_trainer.py:1096-1130)
    "dataloader_num_workers", "dataloader_pin_memory", "dataloader_persistent_workers", "dataloader_prefetch_factor",
    "dataloader_multiprocessing_context", "dataloader_in_order", "data_seed", "train_sampling_strategy",
    "group_by_length", "length_column_name", "label_names",
    # process / DDP plumbing (the gradient mean is the same whatever the bucket layout)
    "ddp_find_unused_parameters", "ddp_bucket_cap_mb", "ddp_broadcast_buffers", "ddp_static_graph", "ddp_backend",
    "ddp_timeout", "local_rank", "do_train", "do_eval", "do_predict", "resume_from_checkpoint",
    "overwrite_output_dir", "save_on_each_node", "tpu_num_cores", "mp_parameters",
    # memory / speed switches with the same math
    "gradient_checkpointing", "gradient_checkpointing_kwargs", "use_cache", "torch_compile", "torch_compile_backend",
    "torch_compile_mode", "torch_empty_cache_steps", "full_determinism", "fp16_opt_level",
    # evaluation-loop details of Trainer.evaluate that GRPO's prediction_step / PPO's loop replace
    "prediction_loss_only", "eval_do_concat_batches", "eval_use_gather_object", "eval_accumulation_steps",
    "include_for_metrics", "include_inputs_for_metrics", "batch_eval_metrics", "past_index",
    "use_legacy_prediction_loop", "metric_for_best_model", "greater_is_better",
    # the loss is the trainer's own (compute_loss overridden, model_accepts_loss_kwargs False, :1016-1019)
    "label_smoothing_factor", "average_tokens_across_devices",
    # vLLM settings, inert while use_vllm is False (use_vllm=True raises)
    "vllm_server_base_url", "vllm_guided_decoding_regex", "vllm_server_host", "vllm_server_port",
    "vllm_server_timeout", "vllm_gpu_memory_utilization", "vllm_tensor_parallel_size",
})


def _falsy(v) -> bool:
    return v is None or v is False or v == "" or v == [] or v == {} or v == 0


def _one_of(*allowed) -> Callable[[Any], bool]:
    return lambda v: getattr(v, "value", v) in allowed


# field -> (predicate of the inert values, what the predicate admits)
CONSTRAINED: dict[str, tuple[Callable[[Any], bool], str]] = {
    "optim": (_one_of("adamw_torch", "adamw_torch_fused"), "'adamw_torch' / 'adamw_torch_fused' (the fused AdamW "
                                                           "kernel is torch AdamW)"),
    "optim_args": (_falsy, "None"),
    "optim_target_modules": (_falsy, "None"),
    "adafactor": (_falsy, "False"),
    "logging_strategy": (_one_of("steps"), "'steps'"),
    "tf32": (lambda v: v is None or v is False, "None / False (fp32 GEMMs stay fp32)"),
    "bf16_full_eval": (_falsy, "False"),
    "fp16_full_eval": (_falsy, "False"),
    "half_precision_backend": (_one_of("auto", None), "'auto'"),
    "fp16_backend": (_one_of("auto", None), "'auto'"),
    "use_cpu": (_falsy, "False (the engine runs on the ROCm device)"),
    "no_cuda": (_falsy, "False (the engine runs on the ROCm device)"),
    "use_mps_device": (_falsy, "False"),
    "use_ipex": (_falsy, "False"),
    "jit_mode_eval": (_falsy, "False"),
    "torchdynamo": (_falsy, "None"),
    "use_liger_kernel": (_falsy, "False"),
    "liger_kernel_config": (_falsy, "None"),
    "neftune_noise_alpha": (_falsy, "None"),
    "auto_find_batch_size": (_falsy, "False"),
    "dataloader_drop_last": (_falsy, "False"),
    "eval_delay": (_falsy, "0"),
    "load_best_model_at_end": (_falsy, "False"),
    "ignore_data_skip": (_falsy, "False"),
    "restore_callback_states_from_checkpoint": (_falsy, "False"),
    "enable_jit_checkpoint": (_falsy, "False"),
    "push_to_hub": (_falsy, "False (no hub access)"),
    "save_safetensors": (lambda v: v is None or v is True, "True (checkpoints are safetensors)"),
    "accelerator_config": (_falsy, "None"),
    "parallelism_config": (_falsy, "None"),
    "dispatch_batches": (_falsy, "None"),
    "split_batches": (_falsy, "None / False"),
    "fsdp": (_falsy, "'' / None (DDP replicas only)"),
    "fsdp_config": (_falsy, "None"),
    "fsdp_min_num_params": (_falsy, "0"),
    "fsdp_transformer_layer_cls_to_wrap": (_falsy, "None"),
    "deepspeed": (_falsy, "None"),
    "tp_size": (lambda v: v in (None, 0, 1), "0 / 1"),
    "debug": (_falsy, "''"),
}


def split_known(cls, kwargs: dict, extra_known: frozenset = frozenset()) -> dict:
    """Pop every keyword that is not a field of `cls` out of `kwargs` and
    return them after validating each one against INERT / CONSTRAINED."""
    known = {f for f in cls.__dataclass_fields__ if f != "extra"}
    extra = {k: kwargs.pop(k) for k in list(kwargs) if k not in known}
    bad = []
    for k, v in extra.items():
        if k in INERT or k in extra_known:
            continue
        if k in CONSTRAINED:
            ok, admitted = CONSTRAINED[k]
            if not ok(v):
                bad.append(f"{k}={v!r} (the MI355X trainer supports only {admitted})")
            continue
        bad.append(f"{k}={v!r} (not a field the MI355X trainer implements, and it could change the result)")
    if bad:
        raise ValueError(f"{cls.__name__}: unsupported TrainingArguments setting(s): " + "; ".join(bad))
    return extra
