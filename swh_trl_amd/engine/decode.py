"""Rollout engine: batched KV-cache generation with a graph-captured decode step.

Replaces the HF `model.generate` loop the reference runs per rollout
(grpo_trainer.py:1793-1810 -> transformers `_sample`; PPO: utils.py:1059-1128).
Differences in mechanism, not in result:
  * static bf16 KV cache [L, 2, B, Hkv, Tmax, D] sized once (288 GB HBM);
  * the whole decode step — embedding gather, 24 x (RMSNorm, QKV GEMM,
    RoPE+append+attention kernel, O GEMM, fused residual+RMSNorm, gate/up GEMM,
    SiLU gate, down GEMM), final norm, lm-head GEMM, sampler, step advance —
    is captured ONCE into a HIP graph and replayed, with every step-dependent
    value (step index, prompt width, RNG counter, finished flags) in device
    memory: no host sync per token (the reference pays one per token in
    `unfinished_sequences.max()` and B*C more in `.item()` loops);
  * early exit once every row has finished (HF `_sample` stops the batch
    then): the host keeps at most two graph replays queued ahead of a pinned
    all-finished flag, so the check never drains the stream
    (`EarlyExitPoll`); `check_every` is the legacy synchronous poll.
Prefill runs the full-sequence forward once over the prompt and writes the
post-RoPE keys/values into the cache.
"""
from __future__ import annotations

import contextlib
import gc
from typing import Optional

import torch

from .. import _lib, nn_ops, ops
from ..profiling import trace as _trace
from .._lib import call
from .model import CausalLM
from .options import EngineOptions


class EarlyExitPoll:
    """Stop-when-all-finished without a host sync per token.  After each graph
    replay the device writes min(finished) into a slot of a pinned host ring and
    records an event; the host only waits for the event `depth` replays back,
    by which time the stream still holds `depth` replays of queued work, so the
    GPU never idles on the check.  Costs one tiny reduction + a 4-byte copy per
    replay; finds the batch finished at most `depth` replays late (the extra
    steps only write pad tokens)."""

    def __init__(self, finished: torch.Tensor, depth: int = 2):
        self.finished, self.depth = finished, depth
        self.host = torch.zeros(depth + 2, dtype=torch.int32, pin_memory=True)
        self.pending: list = []
        self.n = 0

    def reset(self):
        self.pending.clear()
        self.n = 0

    def after_replay(self) -> bool:
        """Queue the flag of the work issued so far; True once a flag shows every row finished."""
        j = self.n % self.host.numel()
        self.n += 1
        self.host[j:j + 1].copy_(self.finished.min().view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((ev, j))
        if len(self.pending) <= self.depth:
            return False
        ev0, j0 = self.pending.pop(0)
        ev0.synchronize()
        return bool(self.host[j0] != 0)


@contextlib.contextmanager
def _capture(graph: "torch.cuda.CUDAGraph"):
    """torch.cuda.graph with the Python GC held off for the capture: the graph
    context collects once on entry; a collection INSIDE the capture could destroy
    an unreachable engine's graphs or events mid-capture, which aborts."""
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph):
            yield
    finally:
        if was:
            gc.enable()


def _under_policy(fn):
    """Run an engine method's launches and graph captures under the launch policy
    the engine was built with (its routing and weight packing were decided by it;
    ADVICE r5): the library's policy is per host thread, set for the call and
    restored after it."""
    import functools

    @functools.wraps(fn)
    def wrapped(self, *a, **kw):
        with _lib.launch_policy(**self.policy):
            return fn(self, *a, **kw)
    return wrapped


class DecodeEngine:
    def __init__(self, model: CausalLM, batch_size: int, max_prompt_len: int, max_new_tokens: int,
                 use_graph: bool = True, fused: Optional[bool] = None, options: Optional[EngineOptions] = None):
        """`options`: the engine's mechanism choices (default: the model's,
        engine/options.py).  The engine snapshots the calling thread's launch policy
        (the library's kernel geometry, which also decides the weight copies packed
        below) and runs every launch and graph capture of its own under it."""
        c = model.cfg
        o = self.options = options if options is not None else model.options
        self.policy = _lib.get_launch_policy()
        if model.dtype != torch.bfloat16:
            raise ValueError("DecodeEngine: the decode kernels read bf16 weights (pass a bf16 copy of an fp32 model)")
        self.model, self.cfg = model, c
        self.B, self.Pmax, self.Cmax = batch_size, max_prompt_len, max_new_tokens
        self.Tmax = max_prompt_len + max_new_tokens
        dev = model.device
        self.dev = dev
        L, Hkv, D = c.num_hidden_layers, c.num_key_value_heads, c.head_dim
        self.kv = torch.zeros(L, 2, batch_size, Hkv, self.Tmax, D, device=dev, dtype=torch.bfloat16)
        B, H = batch_size, c.hidden_size
        bf = dict(device=dev, dtype=torch.bfloat16)
        self.x = torch.empty(B, H, **bf)          # embedding of the input token
        self.s = torch.empty(B, H, **bf)          # residual stream
        self.h = torch.empty(B, H, **bf)          # normed activations
        self.qkv = torch.empty(B, c.qkv_dim, **bf)
        self.att = torch.empty(B, c.q_dim, **bf)
        self.o = torch.empty(B, H, **bf)
        self.gu = torch.empty(B, 2 * c.intermediate_size, **bf)
        self.act = torch.empty(B, c.intermediate_size, **bf)
        self.d = torch.empty(B, H, **bf)
        self.logits_buf = torch.empty(B, c.vocab_size, **bf)
        self.ss = torch.empty(B, H // 16, device=dev, dtype=torch.float32)  # RMSNorm partial sums of s
        # zeroed once: the fused finalize keeps a self-resetting ticket at its end
        self.sample_ws = torch.zeros(ops._lib.load().swh_lm_head_sample_workspace_bytes(B, c.vocab_size, H),
                                     device=dev, dtype=torch.uint8)
        self.state = torch.zeros(2, device=dev, dtype=torch.int32)   # {step, P}
        self.rng = torch.zeros(2, device=dev, dtype=torch.int64)     # {seed, counter base}
        self.finished = torch.zeros(B, device=dev, dtype=torch.int32)
        self.cur = torch.zeros(B, device=dev, dtype=torch.int64)
        self.out = torch.zeros(B, max_new_tokens, device=dev, dtype=torch.int64)
        self.out_logp = torch.zeros(B, max_new_tokens, device=dev, dtype=torch.float32)
        self.plen = torch.zeros(B, device=dev, dtype=torch.int32)
        # GRPO's G copies of a prompt read one copy of its prompt K/V in the decode attention
        # (swh_attn_decode_shared; options.shared_kv False: every row its own copy)
        self.shared_kv = o.shared_kv
        self._own_rows = torch.arange(B, device=dev, dtype=torch.int32)
        self.prow = self._own_rows.clone()
        self.seen = torch.zeros(B, (c.vocab_size + 31) // 32, device=dev, dtype=torch.int32)
        self.ws = torch.empty(ops._lib.load().swh_sample_workspace_bytes(B, c.vocab_size), device=dev,
                              dtype=torch.uint8)
        self.cos, self.sin = model.rope(self.Tmax + 1)
        self.use_graph = use_graph and o.decode_graph
        ks = (c.hidden_size, c.intermediate_size, c.q_dim)
        self.fused = (fused if fused is not None else o.fused) and \
            all(k % 128 == 0 for k in ks) and c.hidden_size % 16 == 0 and c.qkv_dim % 16 == 0
        # Folded RMSNorm weights: W' = bf16(W * w_norm) for the normed projections,
        # so the decode GEMMs scale rows by rstd in the epilogue instead of
        # normalising X in every workgroup (rounding differs from transformers'
        # bf16(w * bf16(x * rstd)) at the last bf16 bit; options.fold_norm False keeps it)
        self.fold = self.fused and o.fold_norm
        self.fw = {}
        if self.fold:
            L = c.num_hidden_layers
            for i in range(L):
                self.fw[f"l{i}.qkv_w"] = torch.empty_like(model.p[f"l{i}.qkv_w"])
                self.fw[f"l{i}.gu_w"] = torch.empty_like(model.p[f"l{i}.gu_w"])
            self.fw["lm"] = torch.empty_like(model.lm_weight())
        # the launch policy's route to the bandwidth-regime GEMM (the library decides by it too)
        pol = self.policy
        wide_on, kmin = bool(pol["wide_gemm"]), int(pol["wide_kmin"])
        # Bandwidth-regime projections (Llama-3-8B widths: K >= the policy's wide_kmin, >= 1024 weight
        # rows) read a copy of their weight in wide_gemm's fragment order (contiguous 4 KB
        # runs per wave and round instead of 16 rows 64 B each, csrc/wide_gemm.hip), the
        # folded norm applied while packing; options.wide_pack False keeps the row-major weights
        self.packed = {}
        if self.fold and o.wide_pack and wide_on:
            for name, (N, K, silu, _norm) in self._projections().items():
                if K >= kmin and nn_ops.wide_gemm_eligible(B, N, K, silu):
                    self.packed[name] = torch.empty(N * K * (2 if silu else 1), **bf)
                    if name != "lm" or K > 1024:  # (the fused lm-head sampler, K <= 1024, reads fw["lm"])
                        self.fw.pop(name, None)  # served by the packed copy only
        # Fragment-order copies of the per-layer projections at the 0.5B widths (qkv and
        # gate/up folded with their RMSNorm weight, o, down): each weight load of a wave is
        # one contiguous 1 KB run instead of 16 rows x 64 B (swh_frag_pack /
        # swh_decode_gemm_fragw, bit-identical results); options.fragw False keeps the row-major
        # weights.  Not the shapes decode_gemm hands to the row-major wide GEMM (those keep
        # its result).  The lm head's copy serves the fused sampler and the logits path alike.
        self.fragw = {}
        if self.fused and o.fragw:
            for name, (N, K, silu, norm) in self._projections().items():
                if norm is not None and not self.fold:
                    continue
                wide = wide_on and K >= kmin and nn_ops.wide_gemm_eligible(B, N, K, silu)
                rows = 2 * N if silu else N
                if not wide and name not in self.packed and rows % 16 == 0 and K % 128 == 0:
                    self.fragw[name] = torch.empty(rows, K, **bf)
                    self.fw.pop(name, None)  # served by the fragment-order copy only
        # gate/up writes its SiLU output in the fragment order down_proj reads (register-
        # streamed, no LDS image; down 8.9 -> 6.9-7.6 us at 0.5B); options.act_frag False: row-major
        self.act_frag = (o.act_frag and B % 16 == 0 and
                         all(f"l{i}.gu_w" in self.fragw and f"l{i}.down_w" in self.fragw
                             for i in range(c.num_hidden_layers)) and c.intermediate_size % 32 == 0 and
                         c.hidden_size <= 1024 and c.intermediate_size <= 4864 and  # tile gate/up, <= 19 k-steps/wave
                         c.intermediate_size // 8 >= torch.cuda.get_device_properties(dev).multi_processor_count)
        # the attention writes its output in the fragment order o_proj reads (register-
        # streamed A operand as contiguous 1 KB runs); options.att_frag False keeps it row-major
        self.att_frag = (o.att_frag and B % 16 == 0 and c.q_dim % 32 == 0 and
                         all(f"l{i}.o_w" in self.fragw for i in range(c.num_hidden_layers)))
        self.graph = None
        self.graph_k = None
        self._prefill_graphs = {}
        self.steps_per_graph = o.graph_steps
        self._graph_params = None
        self.params = ops.make_sample_params()
        self.want_logp = False
        # Infinity Cache warm-up carried by the attention launch (swh_attn_decode_l3): its
        # B x Hkv workgroups leave CUs idle, extra workgroups on them read the weights of
        # the projections that follow (options.l3_attn = workgroups, 0: off, None: the
        # default; options.l3_set: comma list of o, down, gu, qkv (this layer), qkv1, o1,
        # gu1, down1 (next layer))
        self.l3_set = o.l3_set
        self.l3_attn = (self._l3_attn_default() if o.l3_attn is None else int(o.l3_attn)) if self.fused else 0
        self._l3a_jobs = None
        self._exit_poll = EarlyExitPoll(self.finished)
        self.steps_run = 0  # decode steps the last generate() ran (early exit: fewer than max_new_tokens - 1)

    # ------------------------------------------------------------------ one decode step (capturable)
    def _step(self):
        """One decode step: 5 fused kernels per layer when K % 128 == 0
        (norm+QKV+bias, RoPE+append+attention, O+residual, norm+gate/up+SiLU,
        down+residual), then norm+lm head, sampler, step advance.  With the
        fused sampler the step ends in the lm-head finalize, which also
        gathers the next input embedding and advances the step (the step
        then starts at layer 0: `_chained` steps)."""
        if self.fused:
            self._step_fused()
        else:
            self._step_unfused()
        if not self._fused_sample():
            self._sample()
            ops.step_advance(self.state[0:1])

    def _chained(self) -> bool:
        """Steps chained through the fused finalize: the step's input row
        (embedding + RMSNorm partials) was written by the previous step."""
        return self._fused_sample()

    def _fused_sample(self) -> bool:
        """lm head + sampler in one kernel (no logits): unfiltered sampling, with
        the per-token log-prob output too at K <= 1024 (swh_lm_head_sample_logp;
        PPO's rollout log-probs without the logits write and sample_step)."""
        # K > 1024: the wide-tile sampler (config 5's step 9.744 -> 9.682 s,
        # profiles/r5_wsamp_step_ab.log); options.fused_sample_wide False keeps logits + sample_step
        wide = "lm" in self.packed and self.options.fused_sample_wide
        return (self.fused and self.options.fused_sample and
                nn_ops.lm_head_sample_supported(self.params, self.cfg.vocab_size, self.cfg.hidden_size,
                                                wide_rows=self.B if wide else 0, logp=self.want_logp))

    def _projections(self) -> dict:
        """name -> (N, K, silu, RMSNorm weight name or None) of the decode GEMMs."""
        c = self.cfg
        out = {}
        for i in range(c.num_hidden_layers):
            out[f"l{i}.qkv_w"] = (c.qkv_dim, c.hidden_size, False, f"l{i}.ln_in")
            out[f"l{i}.o_w"] = (c.hidden_size, c.q_dim, False, None)
            out[f"l{i}.gu_w"] = (c.intermediate_size, c.hidden_size, True, f"l{i}.ln_post")
            out[f"l{i}.down_w"] = (c.hidden_size, c.intermediate_size, False, None)
        out["lm"] = (c.vocab_size, c.hidden_size, False, "norm")
        return out

    def _weight(self, name: str) -> torch.Tensor:
        return self.model.lm_weight() if name == "lm" else self.model.p[name]

    def _fold_jobs(self):
        """Device table of (W, w_norm, W') jobs for swh_fold_norm (built once)."""
        p = self.model.p
        projs = self._projections()
        rows, tab = 0, []
        for name, out in self.fw.items():
            w, nw = self._weight(name), p[projs[name][3]]
            tab += [w.data_ptr(), nw.data_ptr(), out.data_ptr(), w.shape[0], w.shape[1], rows]
            rows += w.shape[0]
        self._fold_tab = torch.tensor(tab, dtype=torch.int64).to(self.dev) if tab else None
        self._fold_rows = rows
        self._fold_n = len(self.fw)
        self._fold_built = True

    @torch.no_grad()
    def refresh_folded(self):
        """Re-derive the folded weights from the current parameters (once per
        generate(): the optimizer changes both W and the norm weights) — one
        launch for all row-major folded matrices (swh_fold_norm) and one
        swh_wide_pack per packed projection, swh_frag_pack per fragment-order copy."""
        projs = self._projections()
        for name, buf in self.fragw.items():
            N, K, silu, norm = projs[name]
            nn_ops.frag_pack(self._weight(name), self.model.p[norm] if norm else None, silu=silu, out=buf)
        if not self.fold:
            return
        if not getattr(self, "_fold_built", False):
            self._fold_jobs()
        if self._fold_n:
            call("swh_fold_norm", self._fold_tab.data_ptr(), self._fold_n, self._fold_rows, ops._stream())
        projs = self._projections()
        for name, buf in self.packed.items():
            N, K, silu, norm = projs[name]
            nn_ops.wide_pack(self._weight(name), self.model.p[norm] if norm else None, silu=silu, out=buf)

    def _normed(self, name: str, norm: str):
        """(weight, norm_w) of a normed projection: folded weight + row scale,
        or the raw weight + in-kernel RMSNorm."""
        if self.fold:
            return self.fw[name], None
        return self._weight(name), self.model.p[norm]

    def _lm_head_weight(self):
        """(weight, norm_w, fragment order?) the fused lm-head sampler reads
        (the wide_pack copy is in the same fragment order)."""
        if "lm" in self.fragw:
            return self.fragw["lm"], None, 1
        if "lm" in self.packed:
            return self.packed["lm"], None, 1
        return (*self._normed("lm", "norm"), False)

    def _proj(self, name: str, x: torch.Tensor, **kw):
        """One decode projection: the packed wide GEMM, or decode_gemm on the
        folded / raw weight (kw: bias, residual, silu, y, ss_in, ss_out)."""
        eps = self.cfg.rms_norm_eps
        if name in self.packed:
            return nn_ops.wide_gemm_packed(x, self.packed[name], self._projections()[name][0], eps=eps, **kw)
        if name in self.fragw:
            if self.act_frag and name.endswith(("gu_w", "down_w")):
                kw["act_frag"] = 1 if name.endswith("gu_w") else 2
            elif "act_frag" in kw and not name.endswith("o_w"):
                raise ValueError(f"{name}: act_frag serves gate/up, down and o only")
            return nn_ops.decode_gemm_fragw(x, self.fragw[name], eps=eps, **kw)
        norm = self._projections()[name][3]
        if norm is None:
            return nn_ops.decode_gemm(x, self._weight(name), eps=eps, **kw)
        w, nw = self._normed(name, norm)
        return nn_ops.decode_gemm(x, w, norm_w=nw, eps=eps, **kw)

    def _l3_attn_default(self) -> int:
        """Warm-up workgroups in the attention launch by default: 96 when the
        attention's B x Hkv workgroups leave that many CUs idle and one layer's
        o + down + next qkv weights are small beside the 256 MiB Infinity Cache
        (Qwen2.5-0.5B at 64 rows: 12.3 MB; decode step 972 -> 925 us, DESIGN.md
        §2e), else 0 (e.g. Llama-3-8B: 512 attention workgroups, 436 MB layers)."""
        c = self.cfg
        cus = torch.cuda.get_device_properties(self.dev).multi_processor_count
        per_layer = 2 * c.hidden_size * (c.q_dim + c.intermediate_size + c.qkv_dim)
        return 96 if self.B * c.num_key_value_heads + 96 <= cus and per_layer <= (64 << 20) else 0

    def _proj_weight(self, name: str) -> torch.Tensor:
        """The buffer _proj streams for a projection."""
        if name in self.packed:
            return self.packed[name]
        if name in self.fragw:
            return self.fragw[name]
        norm = self._projections()[name][3]
        return self._weight(name) if norm is None else self._normed(name, norm)[0]

    def _l3_job_tables(self, spec: str):
        """Per layer, a device table {ptr, bytes / 16, 0} of the weights `spec` names
        (comma list of o, down, gu, qkv: this layer; o1, down1, gu1, qkv1: the next)."""
        L = self.cfg.num_hidden_layers
        names = {"o": (0, "o_w"), "down": (0, "down_w"), "gu": (0, "gu_w"), "qkv": (0, "qkv_w"),
                 "qkv1": (1, "qkv_w"), "o1": (1, "o_w"), "gu1": (1, "gu_w"), "down1": (1, "down_w")}
        keys = [k.strip() for k in spec.split(",") if k.strip()]
        bad = [k for k in keys if k not in names]
        if bad:
            raise ValueError(f"warm-up set {spec!r}: unknown entries {bad} (expected {sorted(names)})")
        tabs = []
        for i in range(L):
            t = []
            for d, n in (names[k] for k in keys):
                if i + d < L:
                    w = self._proj_weight(f"l{i + d}.{n}")
                    t += [w.data_ptr(), w.numel() * w.element_size() // 16, 0]
            tabs.append(torch.tensor(t, dtype=torch.int64).to(self.dev) if t else None)
        return tabs

    def _qkv(self, i: int):
        p = self.model.p
        return self._proj(f"l{i}.qkv_w", self.s, bias=p.get(f"l{i}.qkv_b"), y=self.qkv, ss_in=self.ss)

    def _l3a_tables(self):
        """Per layer, the device job table of swh_attn_decode_l3 (SWH_DECODE_L3_SET)."""
        if self._l3a_jobs is None:
            self._l3a_jobs = self._l3_job_tables(self.l3_set)
            Hkv = self.cfg.num_key_value_heads
            self._l3a_sink = torch.zeros(-(-self.l3_attn // Hkv) * Hkv * 512, dtype=torch.int32, device=self.dev)
        return self._l3a_jobs

    def _attn(self, i: int):
        c = self.cfg
        jobs = self._l3a_tables()[i] if self.l3_attn > 0 else None
        if jobs is not None:
            return nn_ops.attn_decode_l3(self.qkv, self.kv[i, 0], self.kv[i, 1], self.cos, self.sin, self.plen,
                                         self.state, c.num_attention_heads, c.num_key_value_heads, c.head_dim,
                                         c.head_dim ** -0.5, self.att, self.prow, self.att_frag, jobs, self.l3_attn,
                                         self._l3a_sink)
        return nn_ops.attn_decode(self.qkv, self.kv[i, 0], self.kv[i, 1], self.cos, self.sin, self.plen, self.state,
                                  c.num_attention_heads, c.num_key_value_heads, c.head_dim, c.head_dim ** -0.5,
                                  out=self.att, prompt_row=self.prow, out_frag=self.att_frag)

    def _step_fused(self):
        c, m = self.cfg, self.model
        p = m.p
        eps = c.rms_norm_eps
        ss = self.ss  # every producer of s writes its RMSNorm partial sums, every normed GEMM reads them
        L = c.num_hidden_layers
        if not self._chained():
            nn_ops.embed_gather(p["embed"], self.cur, self.s, ss_out=ss)
        for i in range(L):
            self._qkv(i)
            self._attn(i)
            if self.att_frag:
                self._proj(f"l{i}.o_w", self.att, residual=self.s, ss_out=ss, act_frag=2)
            else:
                self._proj(f"l{i}.o_w", self.att, residual=self.s, ss_out=ss)
            self._proj(f"l{i}.gu_w", self.s, silu=True, y=self.act, ss_in=ss)
            self._proj(f"l{i}.down_w", self.act, residual=self.s, ss_out=ss)
        if self._fused_sample():
            w, nw, fr = self._lm_head_weight()
            nn_ops.lm_head_sample_step(self.s, w, self.params, self.rng, self.state[0:1], self.finished,
                                       self.out, self.cur, p["embed"], self.s, ss, norm_w=nw, eps=eps, ss_in=ss,
                                       workspace=self.sample_ws, fragw=fr,
                                       out_logp=self.out_logp if self.want_logp else None)
        else:
            self._proj("lm", self.s, y=self.logits_buf, ss_in=ss)

    def _step_unfused(self):
        c, m = self.cfg, self.model
        p = m.p
        nn_ops.embed_gather(p["embed"], self.cur, self.x)
        nn_ops.rmsnorm_residual(self.x, None, p["l0.ln_in"], c.rms_norm_eps, y=self.h)
        self.s.copy_(self.x)
        for i in range(c.num_hidden_layers):
            if c.attention_bias:
                torch.addmm(p[f"l{i}.qkv_b"], self.h, p[f"l{i}.qkv_w"].t(), out=self.qkv)
            else:
                torch.mm(self.h, p[f"l{i}.qkv_w"].t(), out=self.qkv)
            nn_ops.attn_decode(self.qkv, self.kv[i, 0], self.kv[i, 1], self.cos, self.sin, self.plen, self.state,
                               c.num_attention_heads, c.num_key_value_heads, c.head_dim, c.head_dim ** -0.5,
                               out=self.att, prompt_row=self.prow)
            torch.mm(self.att, p[f"l{i}.o_w"].t(), out=self.o)
            nn_ops.rmsnorm_residual(self.o, self.s, p[f"l{i}.ln_post"], c.rms_norm_eps, y=self.h, s_out=self.s)
            torch.mm(self.h, p[f"l{i}.gu_w"].t(), out=self.gu)
            nn_ops.silu_mul(self.gu, out=self.act)
            torch.mm(self.act, p[f"l{i}.down_w"].t(), out=self.d)
            nxt = p[f"l{i + 1}.ln_in"] if i + 1 < c.num_hidden_layers else p["norm"]
            nn_ops.rmsnorm_residual(self.d, self.s, nxt, c.rms_norm_eps, y=self.h, s_out=self.s)
        torch.mm(self.h, m.lm_weight().t(), out=self.logits_buf)

    def _sample(self):
        ops.sample_step(self.logits_buf, self.params, self.rng, self.state[0:1], self.finished, self.out, self.cur,
                        self.seen if self.params.repetition_penalty != 1.0 else None,
                        self.out_logp if self.want_logp else None, None, self.ws)

    def _params_key(self):
        p = self.params
        return (p.temperature, p.top_p, p.min_p, p.repetition_penalty, p.top_k, p.greedy, p.min_new_tokens,
                p.pad_token_id, p.n_eos, tuple(p.eos_ids), self.want_logp)

    def _ensure_graph(self):
        key = self._params_key()
        if self.graph is not None and self._graph_params == key:
            return
        # warm-up outside capture (hipBLASLt heuristics / workspaces), then capture.
        # The warm-up runs on a scratch copy of the step state, restored afterwards.
        # It also appends one K/V slot to the cache; that is not restored: every
        # cache slot a generation reads, the same generation writes first (the
        # prefill writes slots [0, P), decode step s appends slot P + s - 1 before
        # attending over it), so the slot's old content is never read.
        saved = [t.clone() for t in (self.state, self.finished, self.cur, self.out, self.out_logp, self.seen)]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            # a step index inside the buffers: after a finished generation the step
            # counter sits at max_new_tokens, one column past out / out_logp (whose
            # last row would then write past the allocation into its neighbour)
            self.state[0] = 1
            self._step()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with _capture(self.graph):
            self._step()
        # K steps per replay: one graph launch (~9 us of replay boundary) per K tokens
        self.graph_k = None
        if self.steps_per_graph > 1:
            self.graph_k = torch.cuda.CUDAGraph()
            with _capture(self.graph_k):
                for _ in range(self.steps_per_graph):
                    self._step()
        self._graph_params = key
        for t, v in zip((self.state, self.finished, self.cur, self.out, self.out_logp, self.seen), saved):
            t.copy_(v)

    # ------------------------------------------------------------------ live kernel timing
    @torch.no_grad()
    @_under_policy
    def kernel_timings(self, step_index: int, reps: int = 20, iters: int = 3) -> dict:
        """Device time of each kernel of one fused decode step at sampler index
        `step_index` (attention over P + step_index keys), plus the whole step.
        Each per-layer op is captured once per layer (layer i's weights and
        cache), the lm head `reps` times, into a HIP graph replayed `iters`
        times between HIP events on the capture stream, so a figure is the
        kernel plus its in-graph launch boundary (what the decode graph pays).
        Clobbers the decode scratch buffers and one cache slot: call between
        generations.  Returns {name: {avg_us, bytes_per_launch,
        launches_per_step}}; bytes are algorithmic."""
        if not self.fused:
            raise RuntimeError("kernel_timings needs the fused decode path")
        c, m = self.cfg, self.model
        p = m.p
        eps, B, H, I = c.rms_norm_eps, self.B, c.hidden_size, c.intermediate_size
        L = c.num_hidden_layers
        P = int(self.state[1])
        self.state[0] = step_index
        keys = P + step_index  # upper bound over rows (left padding shortens some)
        bf = 2
        # shared prompt K/V (self.prow): each distinct prompt row's keys are read once
        U = int(torch.unique(self.prow).numel())
        att_bytes = ((U * P + B * (keys - P)) * c.num_key_value_heads * c.head_dim * bf * 2 +
                     B * (c.qkv_dim + c.q_dim) * bf)

        def gemm_bytes(N, K, silu=False):
            wN = 2 * N if silu else N
            return wN * K * bf + B * K * bf + B * N * bf * (2 if not silu and N == H else 1)

        ss = self.ss
        # every per-layer op cycles through the L layers' weights / caches as the
        # decode step does: the figures carry the step's cache state (~1 GB of
        # weights per step streams from HBM; one layer's alone would sit in the
        # 256 MiB Infinity Cache and time optimistically)
        ops_ = {
            "decode_gemm.qkv": (lambda i: self._qkv(i),
                                gemm_bytes(c.qkv_dim, H), L),
            "attn_decode": (lambda i: self._attn(i), att_bytes, L),
            "decode_gemm.o": (lambda i: self._proj(f"l{i}.o_w", self.att, residual=self.s, ss_out=ss,
                                                   **({"act_frag": 2} if self.att_frag else {})),
                              gemm_bytes(H, c.q_dim), L),
            "decode_gemm.gate_up": (lambda i: self._proj(f"l{i}.gu_w", self.s, silu=True, y=self.act, ss_in=ss),
                                    gemm_bytes(I, H, silu=True), L),
            "decode_gemm.down": (lambda i: self._proj(f"l{i}.down_w", self.act, residual=self.s, ss_out=ss),
                                 gemm_bytes(H, I), L),
            "decode_gemm.lm_head": (lambda i: self._proj("lm", self.s, y=self.logits_buf, ss_in=ss),
                                    c.vocab_size * H * bf + B * c.vocab_size * bf, 1),
            "sample_step": (lambda i: self._sample(), B * c.vocab_size * bf, 1),
        }
        if self._fused_sample():  # what the decode graph runs instead of lm head + sample_step
            del ops_["decode_gemm.lm_head"], ops_["sample_step"]
            ops_["lm_head_sample"] = (
                lambda i: nn_ops.lm_head_sample(self.s, self._lm_head_weight()[0], self.params, self.rng,
                                                self.state[0:1], self.finished, self.out, self.cur,
                                                norm_w=self._lm_head_weight()[1], eps=eps, ss_in=ss,
                                                workspace=self.sample_ws, fragw=self._lm_head_weight()[2]),
                c.vocab_size * H * bf, 1)
        nn_ops.embed_gather(p["embed"], self.cur, self.s, ss_out=ss)
        out = {}
        stream = torch.cuda.current_stream()

        def timed(fn, n, cycle):
            fn(0)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                for r in range(n):
                    fn(r % cycle)
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                g.replay()
            e1.record(stream)
            e1.synchronize()
            return 1000.0 * e0.elapsed_time(e1) / (n * iters)

        for name, (fn, nbytes, per_step) in ops_.items():
            n = L if per_step == L else reps
            out[name] = {"avg_us": timed(fn, n, per_step), "bytes_per_launch": float(nbytes),
                         "launches_per_step": per_step}
        self.state[0] = step_index
        # the whole step the decode graph replays: with logits + sample_step that includes the
        # sampler and the step advance (the replays advance the step counter either way)
        out["decode_step"] = {"avg_us": timed(lambda i: self._step(), 2, 1), "bytes_per_launch": None,
                              "launches_per_step": 1}
        self.state[0] = step_index
        return out

    # ------------------------------------------------------------------ prefill
    @staticmethod
    def _unique_prompts(prompt_ids: torch.Tensor, prompt_mask: torch.Tensor, group_size: int = 0,
                        dedup: bool = True):
        """(representative row per distinct prompt, inverse map row -> distinct
        prompt), or None when every row differs.  GRPO rolls out G copies of
        each prompt (RepeatSampler, grpo_trainer.py:97-192): the prefill runs
        once per distinct prompt and its K/V and last-position logits are
        broadcast to the copies (row-independent arithmetic, same values)."""
        if not dedup:
            return None
        B = prompt_ids.shape[0]
        if group_size > 1 and B % group_size == 0:  # the caller's layout: G consecutive copies (checked)
            ids3 = prompt_ids.view(B // group_size, group_size, -1)
            m3 = prompt_mask.view(B // group_size, group_size, -1)
            if bool(((ids3 == ids3[:, :1]) & (m3 == m3[:, :1])).all()):
                rep = torch.arange(0, B, group_size, device=prompt_ids.device)
                inv = torch.arange(B, device=prompt_ids.device) // group_size
                return rep, inv
        key = torch.cat([prompt_ids.to(torch.int64), prompt_mask.to(torch.int64)], 1)
        uniq, inv = torch.unique(key, dim=0, return_inverse=True)
        U, B = uniq.shape[0], key.shape[0]
        if U == B:
            return None
        rep = torch.empty(U, dtype=torch.int64, device=key.device)
        rep.scatter_(0, inv, torch.arange(B, device=key.device))
        return rep, inv

    def _prefill_body(self, ids, mask, inv, rep, padded: bool):
        """The prefill forward on (distinct) prompt rows, K/V into the cache —
        into the representative rows `rep` only when the decode attention reads
        each group's prompt from there (`self.prow`), else broadcast through
        `inv` to every row — and last-position logits into logits_buf.  No host
        sync inside (graph-capturable)."""
        m = self.model
        P = ids.shape[1]
        pos = (mask.long().cumsum(-1) - 1).clamp(min=0)

        def kv_out(i, k, v):
            if inv is not None and self.shared_kv:
                self.kv[i, 0, :, :, :P].index_copy_(0, rep, k)
                self.kv[i, 1, :, :, :P].index_copy_(0, rep, v)
                return
            if inv is not None:
                k, v = k.index_select(0, inv), v.index_select(0, inv)
            self.kv[i, 0, :, :, :P].copy_(k)
            self.kv[i, 1, :, :, :P].copy_(v)

        h = m.hidden_states(ids, positions=pos, key_mask=mask, kv_out=kv_out, max_pos=P - 1, padded=padded)
        if inv is None:
            torch.mm(h[:, -1], m.lm_weight().t(), out=self.logits_buf)
        else:
            torch.index_select(h[:, -1] @ m.lm_weight().t(), 0, inv, out=self.logits_buf)

    def _prefill(self, prompt_ids: torch.Tensor, prompt_mask: torch.Tensor, group_size: int = 0):
        """Full forward over the prompt, K/V into cache slots [0, P), logits of the
        last position.  Positions follow generate(): cumsum(mask) - 1.  Copies
        of one prompt are prefilled once (`_unique_prompts`).  The forward is
        captured into a HIP graph per (rows, P, padded) and replayed from
        static input buffers (options.decode_graph False: eager)."""
        m = self.model
        dedup = self._unique_prompts(prompt_ids, prompt_mask, group_size, self.options.prefill_dedup)
        inv = rep = None
        if dedup is not None:
            rep, inv = dedup
            prompt_ids, prompt_mask = prompt_ids[rep], prompt_mask[rep]
            # row b's prompt keys / values live in row rep[inv[b]] (swh_attn_decode_shared)
            self.prow.copy_(rep[inv] if self.shared_kv else self._own_rows)
        else:
            self.prow.copy_(self._own_rows)
        padded = not bool(prompt_mask.bool().all())
        with torch.no_grad():
            saved = m.grad
            m.grad = None  # no grad accumulation in prefill
            try:
                if not self.use_graph:
                    self._prefill_body(prompt_ids, prompt_mask, inv, rep, padded)
                    return
                key = (tuple(prompt_ids.shape), inv is None, padded)
                gp = self._prefill_graphs.get(key)
                if gp is None:
                    st = {"ids": prompt_ids.clone(), "mask": prompt_mask.clone(),
                          "inv": None if inv is None else inv.clone(), "rep": None if rep is None else rep.clone()}
                    side = torch.cuda.Stream()
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):  # warm-up (library workspaces) outside capture
                        self._prefill_body(st["ids"], st["mask"], st["inv"], st["rep"], padded)
                    torch.cuda.current_stream().wait_stream(side)
                    g = torch.cuda.CUDAGraph()
                    with _capture(g):
                        self._prefill_body(st["ids"], st["mask"], st["inv"], st["rep"], padded)
                    gp = self._prefill_graphs[key] = (g, st)
                g, st = gp
                st["ids"].copy_(prompt_ids)
                st["mask"].copy_(prompt_mask)
                if inv is not None:
                    st["inv"].copy_(inv)
                    st["rep"].copy_(rep)
                g.replay()
            finally:
                m.grad = saved

    # ------------------------------------------------------------------ generate
    @torch.no_grad()
    @_under_policy
    def generate(self, prompt_ids: torch.Tensor, prompt_mask: torch.Tensor, max_new_tokens: int, *,
                 temperature=1.0, top_p=1.0, top_k=None, min_p=None, repetition_penalty=1.0, greedy=False,
                 min_new_tokens=0, eos_token_id=None, pad_token_id=None, seed: int = 0, offset: int = 0,
                 return_logp: bool = False, check_every: int = 0, group_size: int = 0, early_exit: bool = True):
        """prompt_ids [B, P] left-padded (B == engine batch).  Returns completion ids
        [B, max_new_tokens] (pad after EOS, like `_sample`) and optional per-token
        log-probs of the drawn tokens under the processed distribution.
        early_exit: stop replaying decode steps once every row has finished
        (`EarlyExitPoll`, no per-token sync); the remaining columns stay pad."""
        B, P = prompt_ids.shape
        if B != self.B or P > self.Pmax or max_new_tokens > self.Cmax:
            raise ValueError(f"engine sized for B={self.B}, P<={self.Pmax}, C<={self.Cmax}; got {B}x{P}, "
                             f"{max_new_tokens}")
        eos = [] if eos_token_id is None else ([eos_token_id] if isinstance(eos_token_id, int) else list(eos_token_id))
        self.params = ops.make_sample_params(temperature, top_p, top_k, min_p, repetition_penalty, greedy,
                                             min_new_tokens, -1 if pad_token_id is None else pad_token_id, eos)
        self.want_logp = return_logp
        prompt_mask = prompt_mask.to(torch.int32)
        self.plen.copy_(prompt_mask.sum(-1).to(torch.int32))
        self.finished.zero_()
        self.out.fill_(pad_token_id if pad_token_id is not None else 0)
        if return_logp:  # columns an early exit never reaches read 0, not a previous generation's values
            self.out_logp.zero_()
        self.rng[0], self.rng[1] = int(seed) & ((1 << 63) - 1), int(offset)
        if repetition_penalty != 1.0:
            # every prompt position, left pads included: transformers'
            # RepetitionPenaltyLogitsProcessor gathers over the whole input_ids
            ops.seen_init(prompt_ids.to(torch.int64), None, self.cfg.vocab_size, self.seen)
        _trace("generate: setup")
        self.refresh_folded()
        if self.use_graph:
            self._ensure_graph()
        _trace("generate: folded weights + graph")
        self.state[0], self.state[1] = 0, P
        self._prefill(prompt_ids, prompt_mask, group_size)
        _trace("generate: prefill")
        self._sample()                      # token 0 from the prefill logits
        ops.step_advance(self.state[0:1])
        if self.fused and self._chained():  # the first chained step's input row
            nn_ops.embed_gather(self.model.p["embed"], self.cur, self.s, ss_out=self.ss)
        s = 1
        K = self.steps_per_graph
        poll = self._exit_poll if (early_exit and eos and not check_every) else None
        if poll is not None:
            poll.reset()
        since = 0
        while s < max_new_tokens:
            if self.use_graph and self.graph_k is not None and not check_every and s + K <= max_new_tokens:
                self.graph_k.replay()
                s += K
                if poll is not None and poll.after_replay():
                    break
                continue
            if self.use_graph:
                self.graph.replay()
            else:
                self._step()
            s += 1
            since += 1
            if check_every and (s - 1) % check_every == 0 and bool(self.finished.all()):
                break
            if poll is not None and since >= K and poll.after_replay():
                break
            if since >= K:
                since = 0
        self.steps_run = s - 1
        comp = self.out[:, :max_new_tokens]
        return comp.clone(), (self.out_logp[:, :max_new_tokens].clone() if return_logp else None)
