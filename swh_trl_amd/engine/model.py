"""Llama-style causal decoder (Qwen2 / Llama-3 families) with flat buffers.

Every weight is a view into ONE bf16 buffer (`flat`), every weight gradient a
view into ONE bf16 buffer (`grad`): the optimizer is one streaming kernel and
the data-parallel all-reduce runs on a few large contiguous buckets.  The
training forward uses autograd, but weight gradients never go through
AccumulateGrad: the custom Functions below add them straight into the grad
views with GEMM epilogue accumulation (beta = 1), so there is no extra pass
and no per-parameter tensor churn.

Semantics follow the transformers modeling code the reference runs
(third-party; grpo_trainer.py:1249 scoring forward, :1804 generate):
RMSNorm casts before the weight multiply, residual adds in bf16, SiLU-gated
MLP, rotate-half RoPE with bf16 cos/sin, GQA attention scaled by D^-0.5.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from .. import nn_ops
from .._lib import call
from ..ops import _dtype_code, _stream
from .config import DecoderConfig
from .options import DEFAULT as DEFAULT_OPTIONS
from .options import EngineOptions

_ALIGN = 64  # elements; keeps every view 128-byte aligned


_DW_STREAMS: dict = {}


def _dw_stream(dev: torch.device):
    """Side stream for the weight-gradient launches (1.4 ms of the 0.5B half-step
    against inline).
    The backward's critical path is dX -> next layer; dW of a layer is a leaf, so
    it runs beside the chain (each launch waits for the compute stream's
    progress so far) and the compute stream joins it once, after backward
    (`dw_sync`).  Accumulation order into the gradient views is unchanged."""
    if dev.type != "cuda":
        return None
    st = _DW_STREAMS.get(dev.index)
    if st is None:
        st = _DW_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return st


def dw_streams(dev: torch.device) -> list:
    """The weight-gradient side streams in use on `dev` (for collectives that
    must wait for the final gradients)."""
    st = _DW_STREAMS.get(dev.index) if dev.type == "cuda" else None
    return [] if st is None else [st]


_DW_KEEP: list = []  # tensors the side stream reads, alive until the compute stream has joined it


def dw_sync(dev: torch.device):
    """The current stream waits for every weight-gradient launch issued so far
    (called at the end of every backward by the embedding node, which runs last)."""
    for st in dw_streams(dev):
        torch.cuda.current_stream(dev).wait_stream(st)
    _DW_KEEP.clear()
    _SIDE_GEMM.pop(dev.index, None)


_SIDE_GEMM: dict = {}  # device index -> event after the last library GEMM issued on the side stream


def _side_gemm_issued(st) -> None:
    """Mark that library GEMMs were just issued on side stream `st`."""
    if st is not None:
        ev = torch.cuda.Event()
        ev.record(st)
        _SIDE_GEMM[st.device.index] = ev


def _main_gemm_fence(dev: torch.device) -> None:
    """Before a library GEMM on the compute stream, wait for the side stream's
    GEMMs issued so far.  hipBLASLt may pick persistent (stream-K style)
    solutions whose workgroups wait on each other's partial tiles; two of them
    running at once on two streams each hold part of the CUs while waiting for
    workgroups that cannot be placed, and both spin forever (observed at the
    Llama-3-8B shapes with 10240-token passes, tools/phase_probe.py; no hang
    with the side stream off).  Each side GEMM already waits for the compute
    stream's work issued before it, so with this fence no two library GEMMs
    overlap; the side GEMMs still overlap the compute stream's HIP kernels
    (norm / SiLU / attention / log-prob backward)."""
    ev = _SIDE_GEMM.pop(dev.index, None) if dev.type == "cuda" else None
    if ev is not None:
        torch.cuda.current_stream(dev).wait_event(ev)


class _OnStream:
    """`with _OnStream(st):` — run on side stream `st` after the current stream's
    work so far (no-op for st None); `keep(t...)` marks tensors the side stream reads."""

    def __init__(self, st):
        self.st = st
        self.ctx = None

    def __enter__(self):
        if self.st is not None:
            self.st.wait_stream(torch.cuda.current_stream(self.st.device))
            self.ctx = torch.cuda.stream(self.st)
            self.ctx.__enter__()
        return self

    def keep(self, *ts):
        # references instead of record_stream: freeing a record_stream'd block
        # records an event on the side stream, which a later graph capture forbids
        if self.st is not None:
            _DW_KEEP.extend(t for t in ts if t is not None)

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


class _Linear(torch.autograd.Function):
    """y = x W^T (+ b); backward returns dx and ACCUMULATES dW (and db) into the
    flat-gradient views (hipBLASLt addmm with beta = 1), on the weight-gradient
    side stream."""

    @staticmethod
    def forward(ctx, x, w, b, gw, gb, opts):
        ctx.save_for_backward(x, w)
        ctx.gw, ctx.gb, ctx.opts = gw, gb, opts
        if _tgemm_serves(opts, w.shape[0], w.shape[1]) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
            x2 = x.reshape(-1, x.shape[-1])
            if nn_ops.gemm_nt_eligible(x2, w) and (b is None or b.dtype == torch.bfloat16):
                return nn_ops.gemm_nt(x2, w, b).view(*x.shape[:-1], w.shape[0])
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = None
        if ctx.needs_input_grad[0]:
            dy2 = dy.reshape(-1, dy.shape[-1])
            wt = None
            if _tgemm_serves(ctx.opts, w.shape[0], w.shape[1]) and w.shape[1] % 128 == 0 and w.shape[0] % 64 == 0 \
                    and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
                wt = w.t().contiguous()  # dy w = dy (w^T)^T: the transposed weight (N K elements) as B
            if wt is not None and nn_ops.gemm_nt_eligible(dy2, wt):
                dx = nn_ops.gemm_nt(dy2, wt).view(*dy.shape[:-1], w.shape[1])
            else:
                _main_gemm_fence(dy.device)
                dx = dy @ w
        if ctx.gw is not None:
            _accumulate_dw(ctx.gw, ctx.gb, dy, x, ctx.opts)
        return dx, None, None, None, None, None


# swh_gemm_nt / swh_gemm_tn (csrc/tgemm.hip) for the narrow projections (qkv, o:
# N, K <= 1536).  EngineOptions.tgemm = off | wgrad (the weight gradients only) | all
# (also the forward and input-gradient GEMMs).  A/B: tools/bench_tgemm.py, tools/train_kernels.py.
_TGEMM_MAX_N = 1536


def _tgemm_serves(opts: EngineOptions, n_out: int, k_in: int, wgrad: bool = False) -> bool:
    on = opts.tgemm == "all" or (wgrad and opts.tgemm == "wgrad")
    return on and n_out <= _TGEMM_MAX_N and k_in <= _TGEMM_MAX_N


def _accumulate_dw(gw, gb, dy, x, opts: EngineOptions = DEFAULT_OPTIONS):
    """gw += dy^T x (and gb += column sums of dy) on the weight-gradient stream."""
    with _OnStream(_dw_stream(dy.device)) as side:
        side.keep(dy, x)
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        S = _dw_split(dy2.shape[0], dy2.shape[1] * x2.shape[1])
        if _tgemm_serves(opts, dy2.shape[1], x2.shape[1], wgrad=True) and gw.is_contiguous() and \
                nn_ops.gemm_tn_eligible(dy2, x2):
            # fp32 partials over 8 token ranges (one per XCD), folded in order (no fence needed:
            # the kernel is not persistent).  The partials are allocated on this side stream,
            # so the caching allocator reuses their block only for later side-stream work:
            # released here, not kept to the end of the backward (~33 MB per layer at 0.5B)
            # (the bias gradient's token sums come out of the same kernel's staged dY)
            fused = gb is not None and gb.is_contiguous()
            nn_ops.gemm_tn_accumulate(gw.view(dy2.shape[1], x2.shape[1]), dy2, x2, opts.tgemm_splits,
                                      bias_grad=gb if fused else None)
            if gb is not None and not fused:
                bias_grad_accumulate(dy2, gb)
            return
        if S > 1:
            # few output tiles over a long token dimension: split the tokens into S
            # batched GEMMs (S x the workgroups), sum the partials into the gradient
            Kc = dy2.shape[0] // S
            parts = torch.bmm(dy2[:S * Kc].view(S, Kc, -1).transpose(1, 2), x2[:S * Kc].view(S, Kc, -1))
            # the S partials summed and folded into the gradient view in one pass
            call("swh_dw_reduce", parts.data_ptr(), S, gw.numel(), gw.data_ptr(), _dtype_code(gw, "dw_reduce"),
                 _stream())
            if S * Kc < dy2.shape[0]:
                gw.addmm_(dy2[S * Kc:].t(), x2[S * Kc:])
        else:
            gw.addmm_(dy2.t(), x2)
        _side_gemm_issued(side.st)
        if gb is not None:  # bias: token sums of dy, fixed order, folded into the view once
            bias_grad_accumulate(dy2, gb)


def bias_grad_accumulate(dy2: torch.Tensor, gb: torch.Tensor, rows_per_chunk: int = 256) -> None:
    """gb += column sums of dy2 [T, N] (swh_colsum_partials + swh_rmsnorm_dw_accum:
    chunk partials in fp32, folded in fixed order; torch's dim-0 reduce of a tall
    bf16 matrix ran ~140 us per call here)."""
    T, N = dy2.shape
    if not dy2.is_contiguous():
        dy2 = dy2.contiguous()
    nch = (T + rows_per_chunk - 1) // rows_per_chunk
    part = torch.empty(max(nch, 1), N, device=dy2.device, dtype=torch.float32)
    dt = _dtype_code(gb, "bias_grad")
    call("swh_colsum_partials", dy2.data_ptr(), T, N, rows_per_chunk, part.data_ptr(), dt, _stream())
    call("swh_rmsnorm_dw_accum", part.data_ptr(), nch, N, gb.data_ptr(), dt, _stream())


def _dw_split(tokens: int, outputs: int) -> int:
    """K split of a weight-gradient GEMM dW[N, M] = dY^T X over `tokens`: the
    small-output projections (o, qkv: <= 1.2M outputs = < 20 output tiles of
    256 x 256) leave most CUs idle at any token count (0.33-0.4 PFLOP/s at
    24576 tokens); splitting the tokens gives S x the tiles.  Measured at the
    bench step's 17408 tokens with the fold included (tools/gemm_eff.py): qkv
    (1.03M outputs) S 8 66 us against 147 at S 1; o (0.80M) S 2 75 us against
    134 at S 8, where the fold of eight partials dominates; down (4.4M) S 2-8
    200 us against 251."""
    if tokens < 8192:
        return 1
    if outputs <= 900_000:
        return 2
    if outputs <= 1_500_000:
        return 8
    if outputs <= 5_000_000:
        return 4
    return 1


class _Embedding(torch.autograd.Function):
    """Embedding lookup.  `anchor` is a 0-d tensor with requires_grad=True: the
    weights themselves are plain tensors (their gradients go to the flat
    buffer by side effect), so the anchor is what makes autograd record the
    graph at all."""

    @staticmethod
    def forward(ctx, ids, table, gtable, anchor):
        ctx.save_for_backward(ids)
        ctx.gtable = gtable
        return F.embedding(ids, table)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        # the first op of the forward: every weight gradient is issued by now.  Join
        # the side stream BEFORE the add: with tied embeddings the lm-head dW (side
        # stream) accumulates into this same view
        dw_sync(dy.device)
        if ctx.gtable is not None:
            embedding_backward(ids, dy, ctx.gtable)
        return None, None, None, None


def embedding_backward(ids: torch.Tensor, dy: torch.Tensor, gtable: torch.Tensor) -> None:
    """gtable[id] += sum of the dy rows of token id, deterministically: rows are
    visited in stable-sorted id order and each id's sum is folded in once
    (swh_embedding_bwd; torch's index_add_ accumulates with atomics, so its bf16
    result depends on the arrival order of duplicate ids)."""
    flat_ids = ids.reshape(-1)
    H = dy.shape[-1]
    d2 = dy.reshape(-1, H)
    if not d2.is_contiguous():
        d2 = d2.contiguous()
    sid, order = torch.sort(flat_ids, stable=True)
    N = flat_ids.numel()
    ws = torch.empty(max(1, N * H), device=dy.device, dtype=torch.float32)
    call("swh_embedding_bwd", sid.data_ptr(), order.data_ptr(), d2.data_ptr(), N, H, gtable.shape[0],
         gtable.data_ptr(), _dtype_code(gtable, "embedding_backward"), ws.data_ptr(), _stream())


class _RMSNorm(torch.autograd.Function):
    """Fused HIP RMSNorm forward/backward; dw accumulated into the grad view."""

    @staticmethod
    def forward(ctx, x, w, gw, eps):
        xc = x.contiguous()
        H = xc.shape[-1]
        rows = xc.numel() // H
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        y, _ = nn_ops.rmsnorm_residual(xc, None, w, eps, rstd=rstd)
        ctx.save_for_backward(xc, w, rstd)
        ctx.gw = gw
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        return _norm_backward(x, w, rstd, dy, None, ctx.gw), None, None, None


_NORM_RPB = 32  # rows per workgroup of the norm weight-gradient partials


def _norm_backward(x, w, rstd, dy, dres, gw):
    """dx of the RMSNorm (+ dres, the residual branch's gradient, in the same
    pass) and the weight gradient folded into its bf16 view in one launch."""
    H = x.shape[-1]
    rows = x.numel() // H
    rpb = _NORM_RPB  # rows per workgroup: 8 per wave, >= 3 workgroups per CU at 24576 rows
    nb = (rows + rpb - 1) // rpb
    part = torch.empty(nb, H, device=x.device, dtype=torch.float32)
    dx = torch.empty_like(x)
    dyc = dy.contiguous()
    dr = dres.contiguous() if dres is not None else None
    dt = _dtype_code(x, "rmsnorm")
    call("swh_rmsnorm_bwd", x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dyc.data_ptr(), rows, H, dx.data_ptr(),
         part.data_ptr(), rpb, None if dr is None else dr.data_ptr(), dt, _stream())
    if gw is not None:
        with _OnStream(_dw_stream(x.device)) as side:
            side.keep(part)
            call("swh_rmsnorm_dw_accum", part.data_ptr(), nb, H, gw.data_ptr(), dt, _stream())
    return dx


class _AddRMSNorm(torch.autograd.Function):
    """s = bf16(x + r) (the residual add), h = RMSNorm(s) in one kernel; the
    backward forms ds + d(norm)/ds in one pass and returns it for x and r."""

    @staticmethod
    def forward(ctx, x, r, w, gw, eps):
        xc, rc = x.contiguous(), r.contiguous()
        H = xc.shape[-1]
        rows = xc.numel() // H
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        h, s = nn_ops.rmsnorm_residual(xc, rc, w, eps, rstd=rstd)
        ctx.save_for_backward(s, w, rstd)
        ctx.gw = gw
        return s, h

    @staticmethod
    def backward(ctx, ds, dh):
        s, w, rstd = ctx.saved_tensors
        if dh is None:
            g = ds
        else:
            g = _norm_backward(s, w, rstd, dh, ds, ctx.gw)
        return g, g, None, None, None


class _LMHeadLogp(torch.autograd.Function):
    """lm head GEMM + fused log-prob/entropy, row-chunked.

    Each chunk's logits [rows, V] is a plain 2-D GEMM output kept below 2^30
    elements (a single [B, C, V] logits tensor passes 2^31 elements at the
    benchmark shape, beyond what the batched GEMM path indexes).  The chunks
    stay resident for the backward (HBM is plentiful; no recompute), and the
    backward overwrites each chunk in place with d logits before the two
    GEMMs (dh = dlogits W, dW += dlogits^T h)."""

    @staticmethod
    def forward(ctx, h, w, gw, ids, temperature, compute_entropy, chunk_rows):
        from .. import ops
        H = h.shape[-1]
        h2 = h.reshape(-1, H)
        if not h2.is_contiguous():
            h2 = h2.contiguous()
        idx = ids.reshape(-1)
        R = h2.shape[0]
        logp = torch.empty(R, device=h.device, dtype=torch.float32)
        ent = torch.empty(R, device=h.device, dtype=torch.float32) if compute_entropy else None
        lse = torch.empty(R, device=h.device, dtype=torch.float32)
        chunks = []
        # chunk k's (HBM-bound) log-prob pass runs on the side stream beside chunk
        # k+1's GEMM; the outputs are joined once after the loop
        side = _dw_stream(h.device) if R > chunk_rows else None
        for r0 in range(0, R, chunk_rows):
            r1 = min(R, r0 + chunk_rows)
            lg = h2[r0:r1] @ w.t()
            with _OnStream(side):
                lp_c, en_c, ls_c = ops.logp_entropy(lg, idx[r0:r1], temperature, compute_entropy)
                logp[r0:r1] = lp_c
                lse[r0:r1] = ls_c
                if compute_entropy:
                    ent[r0:r1] = en_c
            chunks.append(lg)
        if side is not None:
            torch.cuda.current_stream(h.device).wait_stream(side)
        ctx.chunks, ctx.gw, ctx.temperature, ctx.chunk_rows = chunks, gw, temperature, chunk_rows
        ctx.hshape = h.shape
        ctx.save_for_backward(h2, w, idx, lse)
        shp = ids.shape
        if ent is not None:
            ctx.mark_non_differentiable(ent)
            return logp.view(shp), ent.view(shp)
        return logp.view(shp), torch.zeros((), device=h.device)

    @staticmethod
    def backward(ctx, dlogp, dent):
        from .. import ops
        h2, w, idx, lse = ctx.saved_tensors
        g = dlogp.reshape(-1).contiguous()
        dh = torch.empty_like(h2) if ctx.needs_input_grad[0] else None
        for k, lg in enumerate(ctx.chunks):
            r0 = k * ctx.chunk_rows
            r1 = r0 + lg.shape[0]
            ops.logp_backward(lg, idx[r0:r1], lse[r0:r1], g[r0:r1], ctx.temperature, out=lg)  # in place
            if dh is not None:
                _main_gemm_fence(lg.device)
                torch.mm(lg, w, out=dh[r0:r1])
            if ctx.gw is not None:  # beside the next chunk's (HBM-bound) logp backward
                with _OnStream(_dw_stream(lg.device)) as side:
                    side.keep(lg, h2)
                    ctx.gw.addmm_(lg.t(), h2[r0:r1])
                    _side_gemm_issued(side.st)
        ctx.chunks = None
        return (dh.view(ctx.hshape) if dh is not None else None), None, None, None, None, None, None


class _GradReady(torch.autograd.Function):
    """Identity whose backward reports that the gradient has flowed past a
    layer input: every weight gradient of that layer is final by then (they
    are accumulated inside the layer's own backward nodes)."""

    @staticmethod
    def forward(ctx, x, layer, cb):
        ctx.layer, ctx.cb = layer, cb
        return x.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        ctx.cb(ctx.layer)
        return dy, None, None


def rope_tables(cfg: DecoderConfig, max_pos: int, device, dtype=torch.bfloat16) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 [max_pos, D/2] cos/sin holding values of the activation dtype
    (transformers computes them in fp32 and casts to the activation dtype
    before the multiply: bf16-rounded for a bf16 model, exact for fp32)."""
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, D, 2, dtype=torch.int64).float() / D))
    pos = torch.arange(max_pos, dtype=torch.float32)
    fr = torch.outer(pos, inv)
    return (fr.cos().to(dtype).float().to(device).contiguous(),
            fr.sin().to(dtype).float().to(device).contiguous())


def _apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, H, L, D] bf16; cos/sin [B, 1, L, D] bf16 (rotate-half convention)."""
    h = x.shape[-1] // 2
    rot = torch.cat((-x[..., h:], x[..., :h]), dim=-1)
    return x * cos + rot * sin


class CausalLM:
    """Weights + forward passes.  `head` is "lm" (vocabulary logits) or "score"
    (one scalar per position: the PPO value / reward model head)."""

    def __init__(self, cfg: DecoderConfig, device, head: str = "lm", dtype=torch.bfloat16, seed: Optional[int] = 0,
                 init_std: float = 0.02, trainable: bool = True, options: Optional[EngineOptions] = None):
        self.cfg, self.device, self.head, self.dtype = cfg, torch.device(device), head, dtype
        self.options = options if options is not None else DEFAULT_OPTIONS
        self.layout: dict[str, tuple[int, tuple]] = {}
        off = 0

        def add(name, *shape):
            nonlocal off
            n = 1
            for s in shape:
                n *= s
            self.layout[name] = (off, tuple(shape))
            off += (n + _ALIGN - 1) // _ALIGN * _ALIGN

        self._build_layout(add)
        self.numel = off
        self.flat = torch.zeros(off, device=self.device, dtype=dtype)
        self.p = {k: self.flat[o:o + math.prod(s)].view(s) for k, (o, s) in self.layout.items()}
        self.grad: Optional[torch.Tensor] = None
        self.g: dict[str, torch.Tensor] = {}
        if seed is not None:
            self.init_weights(seed, init_std)
        self._anchor = torch.zeros((), device=self.device, requires_grad=True)
        if trainable:
            self.enable_grad_buffer()
        self._rope = None
        # backward hook: called with layer index i once layer i's weight gradients are final
        self.on_layer_grads = None
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError(f"CausalLM dtype {dtype}: bf16 (the product path) or float32 (reference precision)")

    def _build_layout(self, add):
        """Weights in flat-buffer order: add(name, *shape) per tensor."""
        cfg = self.cfg
        H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
        add("embed", V, H)
        for i in range(cfg.num_hidden_layers):
            add(f"l{i}.ln_in", H)
            add(f"l{i}.qkv_w", cfg.qkv_dim, H)
            if cfg.attention_bias:
                add(f"l{i}.qkv_b", cfg.qkv_dim)
            add(f"l{i}.o_w", H, cfg.q_dim)
            add(f"l{i}.ln_post", H)
            add(f"l{i}.gu_w", 2 * I, H)
            add(f"l{i}.down_w", H, I)
        add("norm", H)
        if self.head == "score":
            add("score", 1, H)
        elif not cfg.tie_word_embeddings:
            add("lm_head", V, H)

    @property
    def _hip_attn(self) -> bool:
        """Full-sequence attention on csrc/attn.hip (fwd 95 + bwd 395 us per layer at the GRPO
        shape against aotriton's 150 + 430, rocprofv3 of tools/bench_attn.py);
        options.hip_attention False selects torch SDPA for A/B.  The MFMA kernel is bf16:
        an fp32 model (the reference-precision mode) runs SDPA."""
        return (nn_ops.attention_supported(self.cfg.head_dim) and self.dtype == torch.bfloat16
                and self.options.hip_attention)

    def layer_range(self, i: int) -> tuple[int, int]:
        """[start, end) of layer i's parameters (and gradients) in the flat buffers."""
        start = self.layout[f"l{i}.ln_in"][0]
        end = self.layout[f"l{i + 1}.ln_in"][0] if i + 1 < self.cfg.num_hidden_layers else self.layout["norm"][0]
        return start, end

    # ------------------------------------------------------------------ weights
    def init_weights(self, seed: int, std: float = 0.02):
        g = torch.Generator(device=self.device).manual_seed(seed)
        for k, t in self.p.items():
            if k.endswith(("ln_in", "ln_post")) or k == "norm":
                t.fill_(1.0)
            elif k.endswith("qkv_b"):
                t.zero_()
            else:
                t.copy_(torch.randn(t.shape, generator=g, device=self.device, dtype=torch.float32).mul_(std))

    def enable_grad_buffer(self):
        if self.grad is None:
            self.grad = torch.zeros(self.numel, device=self.device, dtype=self.dtype)
            self.g = {k: self.grad[o:o + math.prod(s)].view(s) for k, (o, s) in self.layout.items()}

    def zero_grad(self):
        if self.grad is not None:
            self.grad.zero_()

    def no_decay_ranges(self) -> list[tuple[int, int]]:
        """[start, end) ranges of the flat buffer excluded from weight decay, as
        transformers' Trainer.get_decay_parameter_names excludes biases and
        norm weights (ALL_LAYERNORM_LAYERS / names with "bias", "norm")."""
        out = []
        for k, (o, s) in sorted(self.layout.items(), key=lambda kv: kv[1][0]):
            if k.endswith(("ln_in", "ln_post", "qkv_b")) or k == "norm":
                out.append((o, o + math.prod(s)))
        return out

    def lm_weight(self) -> torch.Tensor:
        return self.p["embed"] if (self.cfg.tie_word_embeddings and self.head == "lm") else self.p.get("lm_head")

    def _lm_grad(self):
        if self.grad is None:
            return None
        return self.g["embed"] if (self.cfg.tie_word_embeddings and self.head == "lm") else self.g.get("lm_head")

    def rope(self, max_pos: int):
        if self._rope is None or self._rope[0].shape[0] < max_pos:
            n = max(max_pos, 4096)
            self._rope = rope_tables(self.cfg, n, self.device, self.dtype)
        return self._rope

    # ------------------------------------------------------------------ HF interop
    def load_hf_state_dict(self, sd: dict):
        """Load transformers Qwen2/Llama weights (q/k/v and gate/up are packed here)."""
        c = self.cfg
        with torch.no_grad():
            self.p["embed"].copy_(sd["model.embed_tokens.weight"])
            for i in range(c.num_hidden_layers):
                pre = f"model.layers.{i}."
                self.p[f"l{i}.ln_in"].copy_(sd[pre + "input_layernorm.weight"])
                self.p[f"l{i}.ln_post"].copy_(sd[pre + "post_attention_layernorm.weight"])
                self.p[f"l{i}.qkv_w"].copy_(torch.cat([sd[pre + f"self_attn.{n}_proj.weight"] for n in "qkv"], 0))
                if c.attention_bias:
                    self.p[f"l{i}.qkv_b"].copy_(torch.cat([sd[pre + f"self_attn.{n}_proj.bias"] for n in "qkv"], 0))
                self.p[f"l{i}.o_w"].copy_(sd[pre + "self_attn.o_proj.weight"])
                self.p[f"l{i}.gu_w"].copy_(torch.cat([sd[pre + "mlp.gate_proj.weight"], sd[pre + "mlp.up_proj.weight"]], 0))
                self.p[f"l{i}.down_w"].copy_(sd[pre + "mlp.down_proj.weight"])
            self.p["norm"].copy_(sd["model.norm.weight"])
            if "lm_head" in self.p:
                self.p["lm_head"].copy_(sd["lm_head.weight"])
            if "score" in self.p and "score.weight" in sd:
                self.p["score"].copy_(sd["score.weight"])

    def hf_state_dict(self) -> dict:
        c, out = self.cfg, {}
        q, kv = c.q_dim, c.kv_dim
        out["model.embed_tokens.weight"] = self.p["embed"]
        for i in range(c.num_hidden_layers):
            pre = f"model.layers.{i}."
            out[pre + "input_layernorm.weight"] = self.p[f"l{i}.ln_in"]
            out[pre + "post_attention_layernorm.weight"] = self.p[f"l{i}.ln_post"]
            w = self.p[f"l{i}.qkv_w"]
            out[pre + "self_attn.q_proj.weight"], out[pre + "self_attn.k_proj.weight"], \
                out[pre + "self_attn.v_proj.weight"] = w[:q], w[q:q + kv], w[q + kv:]
            if c.attention_bias:
                b = self.p[f"l{i}.qkv_b"]
                out[pre + "self_attn.q_proj.bias"], out[pre + "self_attn.k_proj.bias"], \
                    out[pre + "self_attn.v_proj.bias"] = b[:q], b[q:q + kv], b[q + kv:]
            out[pre + "self_attn.o_proj.weight"] = self.p[f"l{i}.o_w"]
            gu = self.p[f"l{i}.gu_w"]
            out[pre + "mlp.gate_proj.weight"], out[pre + "mlp.up_proj.weight"] = gu[:c.intermediate_size], \
                gu[c.intermediate_size:]
            out[pre + "mlp.down_proj.weight"] = self.p[f"l{i}.down_w"]
        out["model.norm.weight"] = self.p["norm"]
        if "lm_head" in self.p:
            out["lm_head.weight"] = self.p["lm_head"]
        elif self.head == "lm":
            out["lm_head.weight"] = self.p["embed"]
        if "score" in self.p:
            out["score.weight"] = self.p["score"]
        return out

    def copy_from(self, other: "CausalLM"):
        with torch.no_grad():
            self.flat.copy_(other.flat)

    # ------------------------------------------------------------------ full-sequence forward
    def _gv(self, name):
        return self.g.get(name) if self.grad is not None else None

    def _layer(self, i: int, x: torch.Tensor, h: torch.Tensor, positions, cos_t, sin_t, mask, kv_out=None):
        """Layer i on the residual stream x with h = RMSNorm_in(x) already formed;
        returns (x + attention, the MLP output d): the caller folds x + d into
        the next RMSNorm (`_AddRMSNorm`)."""
        c = self.cfg
        B, L, _ = x.shape
        Hq, Hkv, D = c.num_attention_heads, c.num_key_value_heads, c.head_dim
        qkv = _Linear.apply(h, self.p[f"l{i}.qkv_w"], self.p.get(f"l{i}.qkv_b"), self._gv(f"l{i}.qkv_w"),
                            self._gv(f"l{i}.qkv_b"), self.options)
        # split + rotate-half RoPE + [B, H, L, D] layout in one kernel each way
        q, k, v = nn_ops.QKVRopeFn.apply(qkv, positions, cos_t, sin_t, Hq, Hkv, D)
        if kv_out is not None:
            kv_out(i, k, v)
        o = self._attend(q, k, v, mask)
        return self._post_attention(i, x, o)

    def _attend(self, q, k, v, mask):
        """Causal GQA attention over [B, H, L, D] (padding mask as built by
        hidden_states) -> token-major [B, L, Hq D], the o_proj input."""
        c = self.cfg
        D = c.head_dim
        B, _, L, _ = q.shape
        if self._hip_attn:  # csrc/attn.hip: causal GQA flash attention, padding as transformers
            km, fv = (None, None) if mask is None else mask
            return nn_ops.AttentionTokFn.apply(q, k, v, D ** -0.5, km, fv)
        gqa = c.num_attention_heads != c.num_key_value_heads  # torch SDPA (aotriton), GQA inside the kernel
        if mask is None:
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=D ** -0.5, enable_gqa=gqa)
        else:
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=D ** -0.5, enable_gqa=gqa)
        return o.transpose(1, 2).reshape(B, L, c.q_dim)

    def _post_attention(self, i, x, o):
        """o-proj, residual + post-attention norm, the SiLU-gated MLP: (x + o, MLP output)."""
        c = self.cfg
        o = _Linear.apply(o, self.p[f"l{i}.o_w"], None, self._gv(f"l{i}.o_w"), None, self.options)
        x, h = _AddRMSNorm.apply(x, o, self.p[f"l{i}.ln_post"], self._gv(f"l{i}.ln_post"), c.rms_norm_eps)
        gu = _Linear.apply(h, self.p[f"l{i}.gu_w"], None, self._gv(f"l{i}.gu_w"), None, self.options)
        a = nn_ops.SiluMulFn.apply(gu)
        d = _Linear.apply(a, self.p[f"l{i}.down_w"], None, self._gv(f"l{i}.down_w"), None, self.options)
        return x, d

    def _mask(self, key_mask, L: int, padded: bool, device):
        """The attention mask of a key-padding mask [B, L] (None: causal only)."""
        if key_mask is None or not padded:
            return None
        if self._hip_attn:
            # (key_mask, index of the first valid key): the kernel's visibility rule
            km = key_mask.to(torch.int32).contiguous()
            return km, (km.cumsum(-1) == 0).sum(-1).to(torch.int32)
        km = key_mask.bool()
        causal = torch.ones(L, L, device=device, dtype=torch.bool).tril()
        # a query with no valid key at all (left padding) sees itself, so no
        # softmax row is empty; any other padded query (right padding after
        # a stop token) sees exactly the valid keys before it, as transformers
        no_key = km.cumsum(-1) == 0
        eye = torch.eye(L, device=device, dtype=torch.bool)
        return causal & (km[:, None, None, :] | (eye & no_key[:, None, :, None]))

    supports_shared_prefix = True

    def hidden_states_grouped(self, prompt_ids: torch.Tensor, prompt_mask: torch.Tensor,
                              completion_ids: torch.Tensor, G: int, padded: Optional[bool] = None):
        """The scoring / training forward of `hidden_states(cat(prompt, completion))`
        for rows in groups of G consecutive rows that share one prompt (GRPO's
        num_generations copies, grpo_trainer.py:97-192): every token-wise op
        (projections, norms, MLP) runs on the prompt tokens ONCE per group
        and on each row's completion tokens; attention sees, per row, the
        group's prompt keys followed by its own completion (positions and
        padding exactly as the per-row forward).  The prompt K/V/Q are
        broadcast to the group's rows by expand (their gradients are the
        fixed-order sums over the rows).  Returns (h_last [U, H]: the final
        hidden state of the last prompt position of each group, h_comp
        [R, C, H]: the completion positions).  `padded`: whether any prompt
        is left-padded, when the caller knows it on the host (None: read back)."""
        c = self.cfg
        R, C = completion_ids.shape
        if G < 1 or R % G:
            raise ValueError(f"{R} rows do not form groups of {G}")
        U = R // G
        dev = completion_ids.device
        pid = prompt_ids[::G].contiguous()
        pm = prompt_mask[::G]
        P = pid.shape[1]
        NP, H = U * P, c.hidden_size
        Hq, Hkv, D = c.num_attention_heads, c.num_key_value_heads, c.head_dim
        ids = torch.cat([pid.reshape(-1), completion_ids.reshape(-1)]).view(1, -1)
        pos_p = torch.arange(P, device=dev).expand(U, P)
        pos_c = torch.arange(P, P + C, device=dev).expand(R, C)
        cos_t, sin_t = self.rope(P + C)
        if padded is None:
            padded = not bool(pm.bool().all())
        km = torch.cat([pm.to(torch.int32).repeat_interleave(G, 0), torch.ones(R, C, dtype=torch.int32, device=dev)], 1)
        mask = self._mask(km, P + C, padded, dev)

        def bcast(t):  # [U, ...] -> [R, ...], the group's tensor for each of its rows
            return t[:, None].expand(U, G, *t.shape[1:]).reshape(R, *t.shape[1:])

        x = _Embedding.apply(ids, self.p["embed"], self._gv("embed"), self._anchor).view(-1, H)
        d = None
        eps = c.rms_norm_eps
        for i in range(c.num_hidden_layers):
            if self.on_layer_grads is not None and torch.is_grad_enabled():
                x = _GradReady.apply(x, i, self.on_layer_grads)
            if d is None:
                h = _RMSNorm.apply(x, self.p[f"l{i}.ln_in"], self._gv(f"l{i}.ln_in"), eps)
            else:
                x, h = _AddRMSNorm.apply(x, d, self.p[f"l{i}.ln_in"], self._gv(f"l{i}.ln_in"), eps)
            qkv = _Linear.apply(h, self.p[f"l{i}.qkv_w"], self.p.get(f"l{i}.qkv_b"), self._gv(f"l{i}.qkv_w"),
                                self._gv(f"l{i}.qkv_b"), self.options)
            if self._hip_attn:
                # one node for both segments' RoPE; the attention reads the group's prompt
                # Q/K/V in place and writes the token-major o_proj input (no cat / copies)
                q_p, k_p, v_p, q_c, k_c, v_c = nn_ops.QKVRopeSegFn.apply(qkv, pos_p, pos_c, cos_t, sin_t, U, P, R,
                                                                         C, Hq, Hkv, D)
                km, fv = (None, None) if mask is None else mask
                o = nn_ops.GroupedAttentionFn.apply(q_p, k_p, v_p, q_c, k_c, v_c, G, D ** -0.5, km, fv)
            else:
                q_p, k_p, v_p = nn_ops.QKVRopeFn.apply(qkv[:NP].view(U, P, -1), pos_p, cos_t, sin_t, Hq, Hkv, D)
                q_c, k_c, v_c = nn_ops.QKVRopeFn.apply(qkv[NP:].view(R, C, -1), pos_c, cos_t, sin_t, Hq, Hkv, D)
                q = torch.cat([bcast(q_p), q_c], 2)
                k = torch.cat([bcast(k_p), k_c], 2)
                v = torch.cat([bcast(v_p), v_c], 2)
                o = self._attend(q, k, v, mask).view(R, P + C, c.q_dim)
                o_p = o.view(U, G, P + C, c.q_dim)[:, 0, :P]  # the group's prompt rows, once
                o = torch.cat([o_p.reshape(NP, c.q_dim), o[:, P:].reshape(R * C, c.q_dim)])
            x, d = self._post_attention(i, x, o)
        _, h = _AddRMSNorm.apply(x, d, self.p["norm"], self._gv("norm"), eps)
        return h[:NP].view(U, P, H)[:, P - 1], h[NP:].view(R, C, H)

    def hidden_states(self, ids: torch.Tensor, positions: Optional[torch.Tensor] = None,
                      key_mask: Optional[torch.Tensor] = None, kv_out=None, max_pos: Optional[int] = None,
                      padded: Optional[bool] = None) -> torch.Tensor:
        """Final-normed hidden states [B, L, H].

        positions: [B, L] (default arange, the transformers training forward);
        key_mask: [B, L] bool/int, 0 = padding key (left-padded prompts).
        max_pos / padded: host-known bounds on positions and whether key_mask
        has zeros — given both, the forward makes no host sync (graph capture).
        """
        c = self.cfg
        B, L = ids.shape
        if positions is None:
            positions = torch.arange(L, device=ids.device).expand(B, L)
        if max_pos is None:
            max_pos = int(positions.max().item()) if positions.numel() else 0
        cos_t, sin_t = self.rope(max_pos + 1)
        positions = positions.to(torch.int64).contiguous()
        if padded is None:
            padded = key_mask is not None and not bool(key_mask.bool().all())
        mask = self._mask(key_mask, L, padded, ids.device)
        x = _Embedding.apply(ids, self.p["embed"], self._gv("embed"), self._anchor)
        d = None
        eps = c.rms_norm_eps
        for i in range(c.num_hidden_layers):
            # hook on the residual stream entering layer i's input norm: its gradient is
            # formed by that norm's backward, the last of layer i's backward nodes
            if self.on_layer_grads is not None and torch.is_grad_enabled():
                x = _GradReady.apply(x, i, self.on_layer_grads)
            if d is None:
                h = _RMSNorm.apply(x, self.p[f"l{i}.ln_in"], self._gv(f"l{i}.ln_in"), eps)
            else:  # previous layer's residual add + this layer's input norm, one kernel
                x, h = _AddRMSNorm.apply(x, d, self.p[f"l{i}.ln_in"], self._gv(f"l{i}.ln_in"), eps)
            x, d = self._layer(i, x, h, positions, cos_t, sin_t, mask, kv_out)
        _, h = _AddRMSNorm.apply(x, d, self.p["norm"], self._gv("norm"), eps)
        return h

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """lm head (bf16 logits) on selected hidden states [.., H]."""
        return _Linear.apply(hidden, self.lm_weight(), None, self._lm_grad(), None, self.options)

    def logp_entropy(self, hidden: torch.Tensor, ids: torch.Tensor, temperature: float = 1.0,
                     compute_entropy: bool = True, chunk_rows: Optional[int] = None):
        """Per-token log-probs (differentiable, fp32) and entropies (no grad) of
        `ids` under softmax(lm_head(hidden) / T), chunked over rows."""
        if chunk_rows is None:
            cap = self.options.logp_chunk  # A/B: tools/train_kernels.py
            chunk_rows = max(1, min(cap, (1 << 30) // self.cfg.vocab_size))
        lp, ent = _LMHeadLogp.apply(hidden, self.lm_weight(), self._lm_grad(), ids, float(temperature),
                                    bool(compute_entropy), int(chunk_rows))
        return lp, (ent if compute_entropy else None)

    def scores(self, hidden: torch.Tensor) -> torch.Tensor:
        """score head (value / reward), bf16 [..] as the transformers score Linear."""
        return _Linear.apply(hidden, self.p["score"], None, self._gv("score"), None, self.options).squeeze(-1)
