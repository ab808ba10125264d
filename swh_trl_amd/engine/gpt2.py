"""GPT-2 family (BASELINE.json config 1: the reference's tiny-random-GPT2
plumbing runs, tests/test_grpo_trainer.py) on the same flat-buffer engine.

Semantics follow transformers' GPT2LMHeadModel, the third-party modeling code
the reference scores and generates with (grpo_trainer.py:1249 forward, :1804
generate): learned position embeddings added to the token embeddings,
pre-LayerNorm blocks (LayerNorm with bias), fused c_attn (Conv1D: x W + b,
stored here transposed as a Linear [3H, H]), multi-head attention scaled by
head_dim^-0.5, c_proj, a gelu_new MLP (c_fc 4H, c_proj), final ln_f, lm head
tied to wte.  Dropout is not implemented (the reference's GRPOConfig has
`disable_dropout`; the trainers warn when a GPT-2 config carries dropout).

HIP kernels: LayerNorm (+ the residual add) and gelu_new forward / backward
(csrc/gpt2.hip), the embedding backward, the lm-head log-prob / loss /
sampler / AdamW kernels shared with the Qwen2 / Llama path.  Projections are
library GEMMs through the same weight-gradient-accumulating `_Linear`;
attention is torch SDPA (head_dim 16 at config 1 is below the MFMA
attention kernel's tile, as for the fp32 reference-precision mode).

Decode (`GPT2DecodeEngine`): prefill through the full forward, then one
graph-captured step per token over a static KV cache (positions and the
cache slot come from the device step counter, so the step replays with no
host sync) and the HIP sampler (`swh_sample_step`).
"""
from __future__ import annotations

import math
import warnings
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from .._lib import call, load as _load_lib
from ..ops import _dtype_code, _stream
from .config import DecoderConfig
from .model import CausalLM, _Embedding, _GradReady, _Linear, _OnStream, _dw_stream

_LN_RPB = 64  # rows per LayerNorm weight-gradient partial


def gpt2_config(vocab_size: int = 1024, n_positions: int = 64, n_embd: int = 32, n_layer: int = 2,
                n_head: int = 2, n_inner: Optional[int] = None, layer_norm_epsilon: float = 1e-5) -> DecoderConfig:
    """A GPT-2 architecture (default: SURVEY.md §8d cfg1's tiny random GPT-2)."""
    return DecoderConfig(vocab_size=vocab_size, hidden_size=n_embd, intermediate_size=n_inner or 4 * n_embd,
                         num_hidden_layers=n_layer, num_attention_heads=n_head, num_key_value_heads=n_head,
                         head_dim=n_embd // n_head, rope_theta=0.0, rms_norm_eps=layer_norm_epsilon,
                         tie_word_embeddings=True, attention_bias=True, max_position_embeddings=n_positions,
                         model_type="gpt2")


def layer_norm(x: torch.Tensor, residual: Optional[torch.Tensor], w: torch.Tensor, b: torch.Tensor, eps: float):
    """(y, s, mean, rstd): s = x + residual (or x), y = LayerNorm(s)."""
    xc = x.contiguous()
    H = xc.shape[-1]
    rows = xc.numel() // H
    y = torch.empty_like(xc)
    s = torch.empty_like(xc) if residual is not None else xc
    rc = residual.contiguous() if residual is not None else None
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    call("swh_layernorm_fwd", xc.data_ptr(), None if rc is None else rc.data_ptr(), w.data_ptr(), b.data_ptr(), rows,
         H, float(eps), y.data_ptr(), None if rc is None else s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
         _dtype_code(xc, "layer_norm"), _stream())
    return y, s, mean, rstd


class _AddLayerNorm(torch.autograd.Function):
    """s = x + r (r may be None), h = LayerNorm(s) with bias; returns (s, h).
    The backward forms ds + d(norm)/ds in one kernel pass and accumulates the
    weight / bias gradients into the flat-buffer views (fixed-order partials)."""

    @staticmethod
    def forward(ctx, x, r, w, b, gw, gb, eps):
        h, s, mean, rstd = layer_norm(x, r, w, b, eps)
        ctx.save_for_backward(s, w, mean, rstd)
        ctx.gw, ctx.gb, ctx.has_r = gw, gb, r is not None
        return s, h

    @staticmethod
    def backward(ctx, ds, dh):
        s, w, mean, rstd = ctx.saved_tensors
        H = s.shape[-1]
        rows = s.numel() // H
        if dh is None:
            g = ds
        else:
            dhc = dh.contiguous()
            dsc = ds.contiguous() if ds is not None else None
            g = torch.empty_like(s)
            nb = int(_load_lib().swh_layernorm_bwd_partial_rows(rows, _LN_RPB))
            pw = pb = None
            if ctx.gw is not None:
                pw = torch.empty(max(nb, 1), H, device=s.device, dtype=torch.float32)
                pb = torch.empty_like(pw)
            dt = _dtype_code(s, "layer_norm")
            call("swh_layernorm_bwd", s.data_ptr(), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dhc.data_ptr(),
                 None if dsc is None else dsc.data_ptr(), rows, H, _LN_RPB, g.data_ptr(),
                 None if pw is None else pw.data_ptr(), None if pb is None else pb.data_ptr(), dt, _stream())
            if pw is not None and nb > 0:
                with _OnStream(_dw_stream(s.device)) as side:
                    side.keep(pw, pb)
                    call("swh_rmsnorm_dw_accum", pw.data_ptr(), nb, H, ctx.gw.data_ptr(), dt, _stream())
                    call("swh_rmsnorm_dw_accum", pb.data_ptr(), nb, H, ctx.gb.data_ptr(), dt, _stream())
        return g, (g if ctx.has_r else None), None, None, None, None, None


class _LayerNorm(torch.autograd.Function):
    """h = LayerNorm(x) with bias (no residual add: the first block's ln_1)."""

    @staticmethod
    def forward(ctx, x, w, b, gw, gb, eps):
        s_out, h = _AddLayerNorm.forward(ctx, x, None, w, b, gw, gb, eps)
        return h

    @staticmethod
    def backward(ctx, dh):
        g = _AddLayerNorm.backward(ctx, None, dh)[0]
        return g, None, None, None, None, None


class GeluNewFn(torch.autograd.Function):
    """transformers NewGELUActivation (gelu_new) on HIP."""

    @staticmethod
    def forward(ctx, x):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        call("swh_gelu_tanh_fwd", xc.data_ptr(), xc.numel(), y.data_ptr(), _dtype_code(xc, "gelu"), _stream())
        ctx.save_for_backward(xc)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        d = dy.contiguous()
        dx = torch.empty_like(x)
        call("swh_gelu_tanh_bwd", x.data_ptr(), d.data_ptr(), x.numel(), dx.data_ptr(), _dtype_code(x, "gelu"),
             _stream())
        return dx


class GPT2LM(CausalLM):
    """GPT-2 causal LM in one flat buffer (the CausalLM interface: flat / grad,
    hidden_states, logp_entropy, hf_state_dict, ...)."""

    def _build_layout(self, add):
        c = self.cfg
        H, I, V = c.hidden_size, c.intermediate_size, c.vocab_size
        add("embed", V, H)
        add("wpe", c.max_position_embeddings, H)
        for i in range(c.num_hidden_layers):
            add(f"l{i}.ln_1_w", H)
            add(f"l{i}.ln_1_b", H)
            add(f"l{i}.attn_w", 3 * H, H)
            add(f"l{i}.attn_b", 3 * H)
            add(f"l{i}.proj_w", H, H)
            add(f"l{i}.proj_b", H)
            add(f"l{i}.ln_2_w", H)
            add(f"l{i}.ln_2_b", H)
            add(f"l{i}.fc_w", I, H)
            add(f"l{i}.fc_b", I)
            add(f"l{i}.mproj_w", H, I)
            add(f"l{i}.mproj_b", H)
        add("ln_f_w", H)
        add("ln_f_b", H)
        if self.head == "score":
            add("score", 1, H)

    supports_shared_prefix = False  # the grouped forward is the Qwen2 / Llama layer

    @property
    def _hip_attn(self) -> bool:
        return False  # SDPA: head_dim 16 (config 1) is below the MFMA attention tile

    def layer_range(self, i: int) -> tuple[int, int]:
        start = self.layout[f"l{i}.ln_1_w"][0]
        end = self.layout[f"l{i + 1}.ln_1_w"][0] if i + 1 < self.cfg.num_hidden_layers else self.layout["ln_f_w"][0]
        return start, end

    def init_weights(self, seed: int, std: float = 0.02):
        g = torch.Generator(device=self.device).manual_seed(seed)
        for k, t in self.p.items():
            if k.endswith(("ln_1_w", "ln_2_w")) or k == "ln_f_w":
                t.fill_(1.0)
            elif k.endswith("_b"):
                t.zero_()
            else:
                t.copy_(torch.randn(t.shape, generator=g, device=self.device, dtype=torch.float32).mul_(std))

    def no_decay_ranges(self) -> list[tuple[int, int]]:
        out = []
        for k, (o, s) in sorted(self.layout.items(), key=lambda kv: kv[1][0]):
            if k.endswith("_b") or "ln_" in k:
                out.append((o, o + math.prod(s)))
        return out

    def lm_weight(self) -> torch.Tensor:
        return self.p["embed"]

    def _lm_grad(self):
        return self.g["embed"] if self.grad is not None else None

    def rope(self, max_pos: int):
        return None

    # ------------------------------------------------------------------ HF interop (GPT2LMHeadModel names)
    _PAIRS = (("ln_1_w", "ln_1.weight"), ("ln_1_b", "ln_1.bias"), ("attn_b", "attn.c_attn.bias"),
              ("proj_b", "attn.c_proj.bias"), ("ln_2_w", "ln_2.weight"), ("ln_2_b", "ln_2.bias"),
              ("fc_b", "mlp.c_fc.bias"), ("mproj_b", "mlp.c_proj.bias"))
    _CONV = (("attn_w", "attn.c_attn.weight"), ("proj_w", "attn.c_proj.weight"), ("fc_w", "mlp.c_fc.weight"),
             ("mproj_w", "mlp.c_proj.weight"))

    def load_hf_state_dict(self, sd: dict):
        with torch.no_grad():
            self.p["embed"].copy_(sd["transformer.wte.weight"])
            self.p["wpe"].copy_(sd["transformer.wpe.weight"])
            for i in range(self.cfg.num_hidden_layers):
                pre = f"transformer.h.{i}."
                for mine, theirs in self._PAIRS:
                    self.p[f"l{i}.{mine}"].copy_(sd[pre + theirs])
                for mine, theirs in self._CONV:  # Conv1D weights are [in, out]
                    self.p[f"l{i}.{mine}"].copy_(sd[pre + theirs].t())
            self.p["ln_f_w"].copy_(sd["transformer.ln_f.weight"])
            self.p["ln_f_b"].copy_(sd["transformer.ln_f.bias"])
            if "score" in self.p and "score.weight" in sd:
                self.p["score"].copy_(sd["score.weight"])

    def hf_state_dict(self) -> dict:
        out = {"transformer.wte.weight": self.p["embed"], "transformer.wpe.weight": self.p["wpe"]}
        for i in range(self.cfg.num_hidden_layers):
            pre = f"transformer.h.{i}."
            for mine, theirs in self._PAIRS:
                out[pre + theirs] = self.p[f"l{i}.{mine}"]
            for mine, theirs in self._CONV:
                out[pre + theirs] = self.p[f"l{i}.{mine}"].t()
        out["transformer.ln_f.weight"] = self.p["ln_f_w"]
        out["transformer.ln_f.bias"] = self.p["ln_f_b"]
        if self.head == "lm":
            out["lm_head.weight"] = self.p["embed"]
        if "score" in self.p:
            out["score.weight"] = self.p["score"]
        return out

    # ------------------------------------------------------------------ full-sequence forward
    def _attention(self, i, h, mask, kv_out):
        c = self.cfg
        B, L, H = h.shape
        nh, hd = c.num_attention_heads, c.head_dim
        qkv = _Linear.apply(h, self.p[f"l{i}.attn_w"], self.p[f"l{i}.attn_b"], self._gv(f"l{i}.attn_w"),
                            self._gv(f"l{i}.attn_b"), self.options)
        q, k, v = qkv.view(B, L, 3, nh, hd).permute(2, 0, 3, 1, 4).unbind(0)  # [B, nh, L, hd] each
        if kv_out is not None:
            kv_out(i, k, v)
        if mask is None:
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=hd ** -0.5)
        else:
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=hd ** -0.5)
        o = o.transpose(1, 2).reshape(B, L, H)
        return _Linear.apply(o, self.p[f"l{i}.proj_w"], self.p[f"l{i}.proj_b"], self._gv(f"l{i}.proj_w"),
                             self._gv(f"l{i}.proj_b"), self.options)

    def _mlp(self, i, h):
        f = _Linear.apply(h, self.p[f"l{i}.fc_w"], self.p[f"l{i}.fc_b"], self._gv(f"l{i}.fc_w"),
                          self._gv(f"l{i}.fc_b"), self.options)
        a = GeluNewFn.apply(f)
        return _Linear.apply(a, self.p[f"l{i}.mproj_w"], self.p[f"l{i}.mproj_b"], self._gv(f"l{i}.mproj_w"),
                             self._gv(f"l{i}.mproj_b"), self.options)

    def hidden_states(self, ids: torch.Tensor, positions: Optional[torch.Tensor] = None,
                      key_mask: Optional[torch.Tensor] = None, kv_out=None, max_pos: Optional[int] = None,
                      padded: Optional[bool] = None) -> torch.Tensor:
        """ln_f(GPT2Model(ids)) [B, L, H].  positions default to arange (the
        reference's scoring forward passes none); key_mask: 0 = padding key."""
        c = self.cfg
        B, L = ids.shape
        if positions is None:
            positions = torch.arange(L, device=ids.device).expand(B, L)
        if max_pos is None:
            max_pos = int(positions.max().item()) if positions.numel() else 0
        if max_pos >= c.max_position_embeddings:
            raise ValueError(f"position {max_pos} >= n_positions {c.max_position_embeddings}")
        mask = None
        if padded is None:
            padded = key_mask is not None and not bool(key_mask.bool().all())
        if key_mask is not None and padded:
            km = key_mask.bool()
            causal = torch.ones(L, L, device=ids.device, dtype=torch.bool).tril()
            no_key = km.cumsum(-1) == 0
            eye = torch.eye(L, device=ids.device, dtype=torch.bool)
            mask = causal & (km[:, None, None, :] | (eye & no_key[:, None, :, None]))
        te = _Embedding.apply(ids, self.p["embed"], self._gv("embed"), self._anchor)
        pe = _Embedding.apply(positions.to(torch.int64), self.p["wpe"], self._gv("wpe"), self._anchor)
        x = te + pe
        d = None
        eps = c.rms_norm_eps
        for i in range(c.num_hidden_layers):
            if self.on_layer_grads is not None and torch.is_grad_enabled():
                x = _GradReady.apply(x, i, self.on_layer_grads)
            if d is None:
                h = _LayerNorm.apply(x, self.p[f"l{i}.ln_1_w"], self.p[f"l{i}.ln_1_b"], self._gv(f"l{i}.ln_1_w"),
                                     self._gv(f"l{i}.ln_1_b"), eps)
            else:  # the previous block's MLP residual add + this block's ln_1, one kernel
                x, h = _AddLayerNorm.apply(x, d, self.p[f"l{i}.ln_1_w"], self.p[f"l{i}.ln_1_b"],
                                           self._gv(f"l{i}.ln_1_w"), self._gv(f"l{i}.ln_1_b"), eps)
            a = self._attention(i, h, mask, kv_out)
            x, h = _AddLayerNorm.apply(x, a, self.p[f"l{i}.ln_2_w"], self.p[f"l{i}.ln_2_b"],
                                       self._gv(f"l{i}.ln_2_w"), self._gv(f"l{i}.ln_2_b"), eps)
            d = self._mlp(i, h)
        _, h = _AddLayerNorm.apply(x, d, self.p["ln_f_w"], self.p["ln_f_b"], self._gv("ln_f_w"), self._gv("ln_f_b"),
                                   eps)
        return h


class GPT2DecodeEngine:
    """KV-cache rollout for GPT2LM (the DecodeEngine.generate contract): prefill
    by the full forward, then one graph-captured step per token."""

    def __init__(self, model: GPT2LM, batch_size: int, max_prompt_len: int, max_new_tokens: int,
                 use_graph: bool = True):
        c = model.cfg
        self.model, self.cfg = model, c
        self.B, self.Pmax, self.Cmax = batch_size, max_prompt_len, max_new_tokens
        self.Tmax = max_prompt_len + max_new_tokens
        if self.Tmax > c.max_position_embeddings:
            raise ValueError(f"prompt + completion length {self.Tmax} > n_positions {c.max_position_embeddings}")
        dev, dt = model.device, model.dtype
        self.dev = dev
        L, nh, hd = c.num_hidden_layers, c.num_attention_heads, c.head_dim
        B = batch_size
        self.kv = torch.zeros(L, 2, B, nh, self.Tmax, hd, device=dev, dtype=dt)
        self.keyok = torch.zeros(B, self.Tmax, device=dev, dtype=torch.bool)  # valid cache slots
        self.logits_buf = torch.empty(B, c.vocab_size, device=dev, dtype=dt)
        self.state = torch.zeros(2, device=dev, dtype=torch.int32)   # {step, P}
        self.rng = torch.zeros(2, device=dev, dtype=torch.int64)
        self.finished = torch.zeros(B, device=dev, dtype=torch.int32)
        self.cur = torch.zeros(B, device=dev, dtype=torch.int64)
        self.out = torch.zeros(B, max_new_tokens, device=dev, dtype=torch.int64)
        self.out_logp = torch.zeros(B, max_new_tokens, device=dev, dtype=torch.float32)
        self.plen = torch.zeros(B, device=dev, dtype=torch.int64)
        self.P = torch.zeros(1, device=dev, dtype=torch.int64)       # prompt width (cache slots [0, P))
        self.seen = torch.zeros(B, (c.vocab_size + 31) // 32, device=dev, dtype=torch.int32)
        self.ws = torch.empty(_load_lib().swh_sample_workspace_bytes(B, c.vocab_size), device=dev, dtype=torch.uint8)
        self.use_graph = use_graph and model.options.decode_graph
        self.graph = None
        self._graph_params = None
        self.params = ops.make_sample_params()
        self.want_logp = False
        self.fused = False

    def _sample(self):
        ops.sample_step(self.logits_buf, self.params, self.rng, self.state[0:1], self.finished, self.out, self.cur,
                        self.seen if self.params.repetition_penalty != 1.0 else None,
                        self.out_logp if self.want_logp else None, None, self.ws)

    def _step(self):
        """Token `cur` (drawn at step s - 1) at position plen + s - 1 into cache
        slot P + s - 1; attention over the valid slots; lm head; sample."""
        m, c = self.model, self.cfg
        p = m.p
        B, H = self.B, c.hidden_size
        nh, hd = c.num_attention_heads, c.head_dim
        t = self.state[0:1].to(torch.int64) - 1
        slot = self.P + t                                   # [1]
        pos = self.plen + t                                 # [B]
        self.keyok.index_fill_(1, slot, True)
        x = F.embedding(self.cur, p["embed"]) + F.embedding(pos, p["wpe"])
        d = None
        eps = c.rms_norm_eps
        mask = self.keyok[:, None, None, :]
        for i in range(c.num_hidden_layers):
            x, h, _, _ = self._ln(x, d, f"l{i}.ln_1", eps)
            qkv = torch.addmm(p[f"l{i}.attn_b"], h, p[f"l{i}.attn_w"].t()).view(B, 3, nh, 1, hd)
            self.kv[i, 0].index_copy_(2, slot, qkv[:, 1])
            self.kv[i, 1].index_copy_(2, slot, qkv[:, 2])
            o = F.scaled_dot_product_attention(qkv[:, 0], self.kv[i, 0], self.kv[i, 1], attn_mask=mask,
                                               scale=hd ** -0.5)
            a = torch.addmm(p[f"l{i}.proj_b"], o.reshape(B, H), p[f"l{i}.proj_w"].t())
            x, h, _, _ = self._ln(x, a, f"l{i}.ln_2", eps)
            f = torch.addmm(p[f"l{i}.fc_b"], h, p[f"l{i}.fc_w"].t())
            g = torch.empty_like(f)
            call("swh_gelu_tanh_fwd", f.data_ptr(), f.numel(), g.data_ptr(), _dtype_code(f, "gelu"), _stream())
            d = torch.addmm(p[f"l{i}.mproj_b"], g, p[f"l{i}.mproj_w"].t())
        _, h, _, _ = self._ln(x, d, "ln_f", eps)
        torch.mm(h, p["embed"].t(), out=self.logits_buf)
        self._sample()
        ops.step_advance(self.state[0:1])

    def _ln(self, x, r, name, eps):
        p = self.model.p
        y, s, mean, rstd = layer_norm(x, r, p[name + "_w"], p[name + "_b"], eps)
        return s, y, mean, rstd

    def _params_key(self):
        p = self.params
        return (p.temperature, p.top_p, p.min_p, p.repetition_penalty, p.top_k, p.greedy, p.min_new_tokens,
                p.pad_token_id, p.n_eos, tuple(p.eos_ids), self.want_logp)

    def _ensure_graph(self):
        key = self._params_key()
        if self.graph is not None and self._graph_params == key:
            return
        saved = [t.clone() for t in (self.state, self.finished, self.cur, self.out, self.out_logp, self.seen,
                                     self.keyok, self.kv)]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up (library workspaces) outside capture
            self.state[0] = 1
            self._step()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._step()
        self._graph_params = key
        for t, v in zip((self.state, self.finished, self.cur, self.out, self.out_logp, self.seen, self.keyok, self.kv),
                        saved):
            t.copy_(v)

    @torch.no_grad()
    def generate(self, prompt_ids: torch.Tensor, prompt_mask: torch.Tensor, max_new_tokens: int, *,
                 temperature=1.0, top_p=1.0, top_k=None, min_p=None, repetition_penalty=1.0, greedy=False,
                 min_new_tokens=0, eos_token_id=None, pad_token_id=None, seed: int = 0, offset: int = 0,
                 return_logp: bool = False, check_every: int = 0, group_size: int = 0, early_exit: bool = True):
        """As DecodeEngine.generate: completion ids [B, max_new_tokens] (pad after
        EOS) and optional per-token log-probs under the processed distribution;
        early_exit: stop once every row has finished (polled every 8 steps,
        `EarlyExitPoll`)."""
        from .decode import EarlyExitPoll
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
        # prefill: positions cumsum(mask) - 1 as generate(); K/V into slots [0, P)
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
        poll = EarlyExitPoll(self.finished) if (early_exit and eos and not check_every) else None
        self.steps_run = 0
        for s in range(1, max_new_tokens):
            if self.use_graph:
                self.graph.replay()
            else:
                self._step()
            self.steps_run = s
            if check_every and s % check_every == 0 and bool(self.finished.all()):
                break
            if poll is not None and s % 8 == 0 and poll.after_replay():
                break
        comp = self.out[:, :max_new_tokens]
        return comp.clone(), (self.out_logp[:, :max_new_tokens].clone() if return_logp else None)


def warn_dropout(hf_cfg) -> None:
    """GPT-2 configs carry dropout (resid/embd/attn_pdrop 0.1 by default); this
    engine has none — as with the reference's `disable_dropout=True`."""
    g = (lambda k: hf_cfg.get(k, 0.0)) if isinstance(hf_cfg, dict) else (lambda k: getattr(hf_cfg, k, 0.0))
    if any((g(k) or 0.0) > 0 for k in ("resid_pdrop", "embd_pdrop", "attn_pdrop")):
        warnings.warn("GPT-2 dropout is not implemented by the MI355X engine: training runs as with "
                      "GRPOConfig(disable_dropout=True)", stacklevel=3)
