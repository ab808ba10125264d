"""Decoder configuration for the families the benchmarks name (Qwen2.5-0.5B:
BASELINE.json configs 2-4; Llama-3-8B: config 5; tiny GPT-2: config 1)."""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass


@dataclass
class DecoderConfig:
    vocab_size: int = 151936
    hidden_size: int = 896
    intermediate_size: int = 4864
    num_hidden_layers: int = 24
    num_attention_heads: int = 14
    num_key_value_heads: int = 2
    head_dim: int = 64
    rope_theta: float = 1_000_000.0
    rms_norm_eps: float = 1e-6
    tie_word_embeddings: bool = True
    attention_bias: bool = True          # q/k/v projections carry a bias (Qwen2)
    max_position_embeddings: int = 32768
    model_type: str = "qwen2"

    @property
    def q_dim(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def qkv_dim(self) -> int:
        return self.q_dim + 2 * self.kv_dim

    def num_params(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_hidden_layers
        per = H * self.qkv_dim + (self.qkv_dim if self.attention_bias else 0) + self.q_dim * H + 2 * I * H + I * H + 2 * H
        return V * H + L * per + H + (0 if self.tie_word_embeddings else V * H)

    def to_dict(self):
        return dataclasses.asdict(self)


def qwen2_5_0_5b() -> DecoderConfig:
    """Qwen2.5-0.5B architecture: 494.03M parameters."""
    return DecoderConfig()


def llama3_8b() -> DecoderConfig:
    """Meta-Llama-3-8B architecture (BASELINE.json config 5)."""
    return DecoderConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                         num_attention_heads=32, num_key_value_heads=8, head_dim=128, rope_theta=500000.0,
                         rms_norm_eps=1e-5, tie_word_embeddings=False, attention_bias=False,
                         max_position_embeddings=8192, model_type="llama")


def tiny_qwen2(vocab_size: int = 1024, layers: int = 2) -> DecoderConfig:
    """Small Qwen2-shaped model for parity tests (head_dim 64 as the kernels need)."""
    return DecoderConfig(vocab_size=vocab_size, hidden_size=256, intermediate_size=512, num_hidden_layers=layers,
                         num_attention_heads=4, num_key_value_heads=2, head_dim=64, rope_theta=10000.0,
                         max_position_embeddings=4096)


def tiny_llama(vocab_size: int = 2048, layers: int = 2) -> DecoderConfig:
    """Small Llama-3-shaped model for parity tests: head_dim 128, GQA 4:1,
    no attention bias, untied lm head (the config-5 code paths at test size)."""
    return DecoderConfig(vocab_size=vocab_size, hidden_size=1024, intermediate_size=2048, num_hidden_layers=layers,
                         num_attention_heads=8, num_key_value_heads=2, head_dim=128, rope_theta=500000.0,
                         rms_norm_eps=1e-5, tie_word_embeddings=False, attention_bias=False,
                         max_position_embeddings=4096, model_type="llama")


SUPPORTED_MODEL_TYPES = ("qwen2", "llama", "gpt2")


def from_hf_config(cfg) -> DecoderConfig:
    """Build from a transformers Qwen2Config / LlamaConfig (object or dict).

    Other architectures (GPT-2's learned positions / LayerNorm / GELU MLP, MoE,
    ...) have no kernels in this engine and are refused here with a clear error
    rather than failing later.  RoPE theta is read from `rope_parameters`
    (transformers >= 5) or the older top-level `rope_theta`; only the default
    (unscaled) RoPE is implemented."""
    g = (lambda k, d=None: cfg.get(k, d)) if isinstance(cfg, dict) else (lambda k, d=None: getattr(cfg, k, d))
    mt = g("model_type", "qwen2")
    if mt not in SUPPORTED_MODEL_TYPES:
        raise ValueError(f"model_type {mt!r} is not supported by the MI355X engine (supported: "
                         f"{', '.join(SUPPORTED_MODEL_TYPES)}: Llama-style decoders with RMSNorm, RoPE and a SiLU "
                         "gated MLP, and GPT-2)")
    if mt == "gpt2":  # transformers GPT2Config (BASELINE.json config 1)
        act = g("activation_function", "gelu_new")
        if act not in ("gelu_new", "gelu_pytorch_tanh"):
            raise ValueError(f"GPT-2 activation {act!r} is not supported (gelu_new only)")
        if g("scale_attn_by_inverse_layer_idx", False) or g("reorder_and_upcast_attn", False) or \
                not g("scale_attn_weights", True):
            raise ValueError("GPT-2 attention variants other than the default head_dim^-0.5 scaling are not supported")
        H, nh = g("n_embd"), g("n_head")
        return DecoderConfig(vocab_size=g("vocab_size"), hidden_size=H, intermediate_size=g("n_inner") or 4 * H,
                             num_hidden_layers=g("n_layer"), num_attention_heads=nh, num_key_value_heads=nh,
                             head_dim=H // nh, rope_theta=0.0, rms_norm_eps=float(g("layer_norm_epsilon", 1e-5)),
                             tie_word_embeddings=bool(g("tie_word_embeddings", True)), attention_bias=True,
                             max_position_embeddings=int(g("n_positions", 1024)), model_type="gpt2")
    rp = g("rope_parameters") or g("rope_scaling") or {}
    rtype = rp.get("rope_type", rp.get("type", "default")) if isinstance(rp, dict) else "default"
    if rtype not in ("default", None):
        raise ValueError(f"rope_type {rtype!r} is not supported (default RoPE only)")
    theta = (rp.get("rope_theta") if isinstance(rp, dict) else None) or g("rope_theta") or 10000.0
    heads = g("num_attention_heads")
    hd = g("head_dim") or g("hidden_size") // heads
    return DecoderConfig(vocab_size=g("vocab_size"), hidden_size=g("hidden_size"),
                         intermediate_size=g("intermediate_size"), num_hidden_layers=g("num_hidden_layers"),
                         num_attention_heads=heads, num_key_value_heads=g("num_key_value_heads", heads), head_dim=hd,
                         rope_theta=float(theta),
                         rms_norm_eps=float(g("rms_norm_eps", 1e-6)),
                         tie_word_embeddings=bool(g("tie_word_embeddings", False)),
                         attention_bias=bool(g("attention_bias", mt == "qwen2")),
                         max_position_embeddings=int(g("max_position_embeddings", 32768)), model_type=mt)


PRESETS = {"qwen2.5-0.5b": qwen2_5_0_5b, "llama-3-8b": llama3_8b, "tiny": tiny_qwen2, "tiny-llama": tiny_llama}
