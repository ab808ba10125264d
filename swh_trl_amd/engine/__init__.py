"""Decoder model + rollout engine."""
from .config import DecoderConfig, llama3_8b, qwen2_5_0_5b, tiny_llama, tiny_qwen2
from .decode import DecodeEngine
from .model import CausalLM

__all__ = ["DecoderConfig", "CausalLM", "DecodeEngine", "qwen2_5_0_5b", "llama3_8b", "tiny_qwen2", "tiny_llama"]
