"""Reference-precision rollout engine: KV-cache generation for an fp32 Qwen2 /
Llama policy.

The reference generates in the model's own dtype (grpo_trainer.py:1793-1810 ->
transformers `_sample`), so an fp32 policy rolls out in fp32.  This engine runs
the decode step in fp32 — library GEMMs, the HIP RMSNorm (+ residual) and SiLU
gate kernels in their fp32 instantiations, rotate-half RoPE with fp32 cos/sin,
SDPA over a static fp32 KV cache, the HIP sampler over fp32 logits — with the
DecodeEngine.generate contract (device-side step counter, finished flags and
RNG; the step captured once into a HIP graph and replayed; early exit by
`EarlyExitPoll`).  The prefill is the model's full forward over the prompt.

It exists for parity (greedy ids identical to transformers fp32 `generate` up
to fp32 ties), not speed: the bf16 DecodeEngine is the product's fast path.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import nn_ops, ops
from .._lib import load as _load_lib
from .decode import EarlyExitPoll, _capture
from .model import CausalLM


class RefDecodeEngine:
    def __init__(self, model: CausalLM, batch_size: int, max_prompt_len: int, max_new_tokens: int,
                 use_graph: bool = True):
        if model.dtype != torch.float32:
            raise ValueError("RefDecodeEngine serves fp32 models (the bf16 DecodeEngine serves bf16)")
        c = model.cfg
        self.model, self.cfg = model, c
        self.B, self.Pmax, self.Cmax = batch_size, max_prompt_len, max_new_tokens
        self.Tmax = max_prompt_len + max_new_tokens
        dev = model.device
        self.dev = dev
        B, L, Hkv, D = batch_size, c.num_hidden_layers, c.num_key_value_heads, c.head_dim
        f32 = dict(device=dev, dtype=torch.float32)
        self.kv = torch.zeros(L, 2, B, Hkv, self.Tmax, D, **f32)
        self.keyok = torch.zeros(B, self.Tmax, device=dev, dtype=torch.bool)  # valid cache slots
        self.logits_buf = torch.empty(B, c.vocab_size, **f32)
        self.state = torch.zeros(2, device=dev, dtype=torch.int32)   # {step, P}
        self.rng = torch.zeros(2, device=dev, dtype=torch.int64)
        self.finished = torch.zeros(B, device=dev, dtype=torch.int32)
        self.cur = torch.zeros(B, device=dev, dtype=torch.int64)
        self.out = torch.zeros(B, max_new_tokens, device=dev, dtype=torch.int64)
        self.out_logp = torch.zeros(B, max_new_tokens, **f32)
        self.plen = torch.zeros(B, device=dev, dtype=torch.int64)
        self.P = torch.zeros(1, device=dev, dtype=torch.int64)       # prompt width (cache slots [0, P))
        self.seen = torch.zeros(B, (c.vocab_size + 31) // 32, device=dev, dtype=torch.int32)
        self.ws = torch.empty(_load_lib().swh_sample_workspace_bytes(B, c.vocab_size), device=dev, dtype=torch.uint8)
        self.cos, self.sin = model.rope(self.Tmax + 1)   # fp32 [T, D/2] (exact fp32 values for an fp32 model)
        self.use_graph = use_graph and model.options.decode_graph
        self.graph = None
        self._graph_params = None
        self.params = ops.make_sample_params()
        self.want_logp = False
        self.fused = False
        self.steps_per_graph = 8
        self._exit_poll = EarlyExitPoll(self.finished)
        self.steps_run = 0

    def _sample(self):
        ops.sample_step(self.logits_buf, self.params, self.rng, self.state[0:1], self.finished, self.out, self.cur,
                        self.seen if self.params.repetition_penalty != 1.0 else None,
                        self.out_logp if self.want_logp else None, None, self.ws)

    def _rope(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        """x [B, H, 1, D]; cos/sin [B, 1, 1, D] (rotate-half, transformers apply_rotary_pos_emb)."""
        h = x.shape[-1] // 2
        rot = torch.cat((-x[..., h:], x[..., :h]), dim=-1)
        return x * cos + rot * sin

    def _step(self):
        """Token `cur` (drawn at step s - 1) at position plen + s - 1 into cache slot
        P + s - 1; one fp32 decoder pass; lm head; sample."""
        m, c = self.model, self.cfg
        p = m.p
        B = self.B
        Hq, Hkv, D = c.num_attention_heads, c.num_key_value_heads, c.head_dim
        q_dim, kv_dim = c.q_dim, c.kv_dim
        eps = c.rms_norm_eps
        t = self.state[0:1].to(torch.int64) - 1
        slot = self.P + t                                   # [1]
        pos = self.plen + t                                 # [B]
        self.keyok.index_fill_(1, slot, True)
        cos = self.cos.index_select(0, pos)
        sin = self.sin.index_select(0, pos)
        cos = torch.cat([cos, cos], -1).view(B, 1, 1, D)
        sin = torch.cat([sin, sin], -1).view(B, 1, 1, D)
        mask = self.keyok[:, None, None, :]
        x = F.embedding(self.cur, p["embed"])
        h, _ = nn_ops.rmsnorm_residual(x, None, p["l0.ln_in"], eps)
        for i in range(c.num_hidden_layers):
            b = p.get(f"l{i}.qkv_b")
            qkv = torch.addmm(b, h, p[f"l{i}.qkv_w"].t()) if b is not None else h @ p[f"l{i}.qkv_w"].t()
            q = qkv[:, :q_dim].view(B, Hq, 1, D)
            k = qkv[:, q_dim:q_dim + kv_dim].view(B, Hkv, 1, D)
            v = qkv[:, q_dim + kv_dim:].reshape(B, Hkv, 1, D)
            q, k = self._rope(q, cos, sin), self._rope(k, cos, sin)
            self.kv[i, 0].index_copy_(2, slot, k)
            self.kv[i, 1].index_copy_(2, slot, v)
            o = F.scaled_dot_product_attention(q, self.kv[i, 0], self.kv[i, 1], attn_mask=mask, scale=D ** -0.5,
                                               enable_gqa=Hq != Hkv)
            o = o.reshape(B, q_dim) @ p[f"l{i}.o_w"].t()
            h, x = nn_ops.rmsnorm_residual(o, x, p[f"l{i}.ln_post"], eps)
            gu = h @ p[f"l{i}.gu_w"].t()
            d = nn_ops.silu_mul(gu) @ p[f"l{i}.down_w"].t()
            nxt = p[f"l{i + 1}.ln_in"] if i + 1 < c.num_hidden_layers else p["norm"]
            h, x = nn_ops.rmsnorm_residual(d, x, nxt, eps)
        torch.mm(h, m.lm_weight().t(), out=self.logits_buf)
        self._sample()
        ops.step_advance(self.state[0:1])

    def _params_key(self):
        p = self.params
        return (p.temperature, p.top_p, p.min_p, p.repetition_penalty, p.top_k, p.greedy, p.min_new_tokens,
                p.pad_token_id, p.n_eos, tuple(p.eos_ids), self.want_logp)

    def _ensure_graph(self):
        key = self._params_key()
        if self.graph is not None and self._graph_params == key:
            return
        # the step state is restored after the warm-up; the K/V slot and key flag it appends are
        # not: generate() resets keyok and every slot a generation reads it writes first
        saved = [t.clone() for t in (self.state, self.finished, self.cur, self.out, self.out_logp, self.seen)]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up (library workspaces) outside capture, at an in-range step
            self.state[0] = 1
            self._step()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with _capture(self.graph):
            self._step()
        self._graph_params = key
        for t, v in zip((self.state, self.finished, self.cur, self.out, self.out_logp, self.seen), saved):
            t.copy_(v)

    @torch.no_grad()
    def generate(self, prompt_ids: torch.Tensor, prompt_mask: torch.Tensor, max_new_tokens: int, *,
                 temperature=1.0, top_p=1.0, top_k=None, min_p=None, repetition_penalty=1.0, greedy=False,
                 min_new_tokens=0, eos_token_id=None, pad_token_id=None, seed: int = 0, offset: int = 0,
                 return_logp: bool = False, check_every: int = 0, group_size: int = 0, early_exit: bool = True):
        """As DecodeEngine.generate, in fp32."""
        del group_size
        B, P = prompt_ids.shape
        if B != self.B or P > self.Pmax or max_new_tokens > self.Cmax:
            raise ValueError(f"engine sized for B={self.B}, P<={self.Pmax}, C<={self.Cmax}; got {B}x{P}, "
                             f"{max_new_tokens}")
        m = self.model
        eos = [] if eos_token_id is None else ([eos_token_id] if isinstance(eos_token_id, int) else list(eos_token_id))
        self.params = ops.make_sample_params(temperature, top_p, top_k, min_p, repetition_penalty, greedy,
                                             min_new_tokens, -1 if pad_token_id is None else pad_token_id, eos)
        self.want_logp = return_logp
        mask = prompt_mask.to(torch.int64)
        self.plen.copy_(mask.sum(-1))
        self.finished.zero_()
        self.out.fill_(pad_token_id if pad_token_id is not None else 0)
        if return_logp:  # columns an early exit never reaches read 0, not a previous generation's values
            self.out_logp.zero_()
        self.rng[0], self.rng[1] = int(seed) & ((1 << 63) - 1), int(offset)
        if repetition_penalty != 1.0:
            ops.seen_init(prompt_ids.to(torch.int64), None, self.cfg.vocab_size, self.seen)
        if self.use_graph:
            self._ensure_graph()
        # prefill: positions cumsum(mask) - 1 as generate(); post-RoPE K/V into slots [0, P)
        self.P.fill_(P)
        self.keyok.zero_()
        self.keyok[:, :P] = mask.bool()
        pos = (mask.cumsum(-1) - 1).clamp(min=0)
        saved = m.grad
        m.grad = None
        try:
            def kv_out(i, k, v):
                self.kv[i, 0, :, :, :P].copy_(k)
                self.kv[i, 1, :, :, :P].copy_(v)
            h = m.hidden_states(prompt_ids, positions=pos, key_mask=mask, kv_out=kv_out, max_pos=P - 1)
        finally:
            m.grad = saved
        torch.mm(h[:, -1], m.lm_weight().t(), out=self.logits_buf)
        self.state[0], self.state[1] = 0, P
        self._sample()
        ops.step_advance(self.state[0:1])
        poll = self._exit_poll if (early_exit and eos and not check_every) else None
        if poll is not None:
            poll.reset()
        self.steps_run = 0
        for s in range(1, max_new_tokens):
            if self.use_graph:
                self.graph.replay()
            else:
                self._step()
            self.steps_run = s
            if check_every and s % check_every == 0 and bool(self.finished.all()):
                break
            if poll is not None and s % self.steps_per_graph == 0 and poll.after_replay():
                break
        comp = self.out[:, :max_new_tokens]
        return comp.clone(), (self.out_logp[:, :max_new_tokens].clone() if return_logp else None)
