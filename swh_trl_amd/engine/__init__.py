"""Decoder models + rollout engines."""
import torch

from .config import DecoderConfig, llama3_8b, qwen2_5_0_5b, tiny_llama, tiny_qwen2
from .decode import DecodeEngine
from .gpt2 import GPT2DecodeEngine, GPT2LM, gpt2_config
from .model import CausalLM
from .ref_decode import RefDecodeEngine


def build_model(cfg: DecoderConfig, device, **kw) -> CausalLM:
    """The model class of `cfg.model_type` (GPT-2, or the Qwen2 / Llama decoder)."""
    return (GPT2LM if cfg.model_type == "gpt2" else CausalLM)(cfg, device, **kw)


def build_engine(model: CausalLM, batch_size: int, max_prompt_len: int, max_new_tokens: int, **kw):
    """The rollout engine of `model`'s family and precision: GPT-2 (its own dtype), the
    bf16 Qwen2 / Llama DecodeEngine, or the fp32 reference-precision RefDecodeEngine."""
    if model.cfg.model_type == "gpt2":
        return GPT2DecodeEngine(model, batch_size, max_prompt_len, max_new_tokens, **kw)
    if model.dtype == torch.float32:
        return RefDecodeEngine(model, batch_size, max_prompt_len, max_new_tokens, **kw)
    return DecodeEngine(model, batch_size, max_prompt_len, max_new_tokens, **kw)


__all__ = ["DecoderConfig", "CausalLM", "DecodeEngine", "RefDecodeEngine", "GPT2LM", "GPT2DecodeEngine", "build_model",
           "build_engine",
           "gpt2_config", "qwen2_5_0_5b", "llama3_8b", "tiny_qwen2", "tiny_llama"]
