"""Decoder-layer ops on the HIP library (RMSNorm, SiLU gate, embedding gather,
decode attention), with autograd wrappers for the training forward.

Numerics follow the transformers Qwen2 / Llama bf16 modules the reference
runs (third-party code reached from grpo_trainer.py:1804 and :1249).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib
from ._lib import call
from .ops import _dev, _dtype_code, _p, _stream


def rmsnorm_residual(x: torch.Tensor, residual: Optional[torch.Tensor], weight: torch.Tensor, eps: float,
                     y: Optional[torch.Tensor] = None, s_out: Optional[torch.Tensor] = None,
                     rstd: Optional[torch.Tensor] = None):
    """s = x (+ residual, bf16 add); y = bf16(w * bf16(s * rsqrt(mean(s^2)+eps))).
    Returns (y, s)."""
    _dev(x, "rmsnorm")
    H = x.shape[-1]
    rows = x.numel() // H
    if y is None:
        y = torch.empty_like(x)
    if residual is not None and s_out is None:
        s_out = torch.empty_like(x)
    call("swh_rmsnorm_fwd", x.data_ptr(), _p(residual), _p(s_out), weight.data_ptr(), rows, H, float(eps),
         y.data_ptr(), _p(rstd), _dtype_code(x, "rmsnorm"), _stream())
    return y, (s_out if residual is not None else x)


class RMSNormFn(torch.autograd.Function):
    """y = RMSNorm(x) * w with the fused HIP forward and backward."""

    @staticmethod
    def forward(ctx, x, weight, eps):
        xc = x.contiguous()
        H = xc.shape[-1]
        rows = xc.numel() // H
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        y, _ = rmsnorm_residual(xc, None, weight, eps, rstd=rstd)
        ctx.save_for_backward(xc, weight, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        H = x.shape[-1]
        rows = x.numel() // H
        rpb = 64
        nb = (rows + rpb - 1) // rpb
        dx = torch.empty_like(x)
        part = torch.empty(nb, H, device=x.device, dtype=torch.float32)
        dyc = dy.contiguous()
        call("swh_rmsnorm_bwd", x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dyc.data_ptr(), rows, H, dx.data_ptr(),
             part.data_ptr(), rpb, None, _dtype_code(x, "rmsnorm"), _stream())
        return dx, part.sum(0).to(w.dtype), None


class SiluMulFn(torch.autograd.Function):
    """out = silu(gu[..., :I]) * gu[..., I:] (gate/up packed by the fused GEMM)."""

    @staticmethod
    def forward(ctx, gu):
        guc = gu.contiguous()
        I2 = guc.shape[-1]
        rows = guc.numel() // I2
        out = torch.empty(*guc.shape[:-1], I2 // 2, device=gu.device, dtype=gu.dtype)
        call("swh_silu_mul_fwd", guc.data_ptr(), rows, I2 // 2, out.data_ptr(), _dtype_code(guc, "silu_mul"),
             _stream())
        ctx.save_for_backward(guc)
        return out

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        I2 = gu.shape[-1]
        rows = gu.numel() // I2
        dgu = torch.empty_like(gu)
        d = dout.contiguous()
        call("swh_silu_mul_bwd", gu.data_ptr(), d.data_ptr(), rows, I2 // 2, dgu.data_ptr(),
             _dtype_code(gu, "silu_mul"), _stream())
        return dgu


def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    I2 = gu.shape[-1]
    rows = gu.numel() // I2
    if out is None:
        out = torch.empty(*gu.shape[:-1], I2 // 2, device=gu.device, dtype=gu.dtype)
    call("swh_silu_mul_fwd", gu.data_ptr(), rows, I2 // 2, out.data_ptr(), _dtype_code(gu, "silu_mul"), _stream())
    return out


def embed_gather(table: torch.Tensor, ids: torch.Tensor, out: torch.Tensor,
                 ss_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[b] = table[ids[b]]; ss_out f32 [B, H/16] (optional) gets the rows'
    per 16-column sums of squares for the next fused RMSNorm."""
    call("swh_embed_gather", table.data_ptr(), ids.data_ptr(), ids.numel(), table.shape[1], out.data_ptr(),
         _p(ss_out), _stream())
    return out


def attn_decode(qkv: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, rope_cos: torch.Tensor,
                rope_sin: torch.Tensor, prompt_len: torch.Tensor, state: torch.Tensor, Hq: int, Hkv: int, D: int,
                scale: float, out: Optional[torch.Tensor] = None,
                prompt_row: Optional[torch.Tensor] = None, out_frag: bool = False) -> torch.Tensor:
    """One decode step of GQA attention with in-kernel RoPE and KV append.
    k_cache / v_cache: [B, Hkv, Tmax, D] bf16 (one layer).
    prompt_row int32 [B] (optional): row b reads its prompt keys / values from
    row prompt_row[b]'s cache (swh_attn_decode_shared).  out_frag: `out` in the
    fragment order decode_gemm_fragw(act_frag=2) reads (swh_attn_decode_shared_frag)."""
    _dev(qkv, "attn_decode")
    B = qkv.shape[0]
    Tmax = k_cache.shape[2]
    if out is None:
        out = torch.empty(B, Hq * D, device=qkv.device, dtype=qkv.dtype)
    call("swh_attn_decode_shared_frag", qkv.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), rope_cos.data_ptr(),
         rope_sin.data_ptr(), prompt_len.data_ptr(), _p(prompt_row), state.data_ptr(), B, Hq, Hkv, D, Tmax,
         float(scale), out.data_ptr(), int(bool(out_frag)), _stream())
    return out


def attn_decode_l3(qkv: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, rope_cos: torch.Tensor,
                   rope_sin: torch.Tensor, prompt_len: torch.Tensor, state: torch.Tensor, Hq: int, Hkv: int, D: int,
                   scale: float, out: torch.Tensor, prompt_row: Optional[torch.Tensor], out_frag: bool,
                   l3_jobs: torch.Tensor, l3_wgs: int, l3_sink: torch.Tensor) -> torch.Tensor:
    """attn_decode whose launch also carries Infinity Cache warm-up workgroups
    over l3_jobs (int64 [n, 3] device table of {ptr, bytes / 16, 0})
    (swh_attn_decode_l3): identical results."""
    _dev(qkv, "attn_decode_l3")
    B = qkv.shape[0]
    wgs = -(-l3_wgs // Hkv) * Hkv
    if l3_sink.numel() * l3_sink.element_size() < wgs * 512 * 4:
        raise ValueError("attn_decode_l3: l3_sink smaller than the warm-up workgroups x 512 words")
    call("swh_attn_decode_l3", qkv.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), rope_cos.data_ptr(),
         rope_sin.data_ptr(), prompt_len.data_ptr(), _p(prompt_row), state.data_ptr(), B, Hq, Hkv, D,
         k_cache.shape[2], float(scale), out.data_ptr(), int(bool(out_frag)), l3_jobs.data_ptr(),
         l3_jobs.numel() // 3, int(l3_wgs), l3_sink.data_ptr(), _stream())
    return out


_GEMM_WS: dict = {}


def gemm_workspace(device, nbytes: int = 64 << 20) -> torch.Tensor:
    """Zero-initialised split-K workspace (counters reset themselves after use)."""
    key = (str(device), nbytes)
    if key not in _GEMM_WS:
        _GEMM_WS[key] = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    return _GEMM_WS[key]


def decode_gemm(x: torch.Tensor, w: torch.Tensor, *, norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6,
                bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None, silu: bool = False,
                y: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
                ss_in: Optional[torch.Tensor] = None, ss_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weight-streaming decode GEMM with fused RMSNorm prologue and bias /
    residual / SiLU-gate epilogues (include/swh_trl_amd.h swh_decode_gemm).
    x [M, K] bf16; w [N, K] (or [2N, K] with silu).  ss_in f32 [M, K/16]: the
    producer's chunk sums of squares of x (with norm_w); ss_out f32 [M, N/16]:
    written with residual."""
    _dev(x, "decode_gemm")
    M, K = x.shape
    N = w.shape[0] // 2 if silu else w.shape[0]
    if residual is None and y is None:
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
    ldy = residual.stride(0) if residual is not None else y.stride(0)
    ws = workspace if workspace is not None else gemm_workspace(x.device)
    call("swh_decode_gemm", x.data_ptr(), w.data_ptr(), M, N, K, _p(norm_w), float(eps), _p(bias), _p(residual),
         int(bool(silu)), _p(y), ldy, _p(ss_in), _p(ss_out), ws.data_ptr(), ws.numel(), _stream())
    return residual if residual is not None else y


def gemm_nt_eligible(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes swh_gemm_nt serves: bf16, N % 128 == 0, K % 64 == 0, unit inner strides."""
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2 and w.dim() == 2
            and x.shape[1] == w.shape[1] and w.shape[0] % 128 == 0 and w.shape[1] % 64 == 0
            and x.stride(1) == 1 and w.stride(1) == 1 and x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def gemm_nt(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x w^T (+ bias) on the training projection GEMM (include/swh_trl_amd.h
    swh_gemm_nt): x [M, K], w [N, K], bf16."""
    _dev(x, "gemm_nt")
    if not gemm_nt_eligible(x, w):
        raise ValueError(f"gemm_nt: unsupported operands {tuple(x.shape)} x {tuple(w.shape)}")
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    if bias is not None and (bias.dtype != torch.bfloat16 or not bias.is_contiguous() or bias.numel() != N):
        raise ValueError("gemm_nt: bias must be a contiguous bf16 vector of N elements")
    call("swh_gemm_nt", x.data_ptr(), w.data_ptr(), _p(bias), out.data_ptr(), M, N, K, x.stride(0), w.stride(0),
         out.stride(0), _stream())
    return out


def gemm_nt256_eligible(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> bool:
    """Shapes swh_gemm_nt256 serves: bf16, N % 8 == 0, K % 64 == 0, unit inner strides,
    32-bit staged offsets."""
    ok = (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2 and w.dim() == 2
          and x.shape[1] == w.shape[1] and w.shape[0] % 8 == 0 and w.shape[1] % 64 == 0 and w.shape[1] > 0
          and x.stride(1) == 1 and w.stride(1) == 1 and x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0
          and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
          and x.shape[0] * x.stride(0) < 2 ** 32 and w.shape[0] * w.stride(0) < 2 ** 32)
    if ok and out is not None:
        ok = (out.dtype == torch.bfloat16 and out.dim() == 2 and tuple(out.shape) == (x.shape[0], w.shape[0])
              and out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 8 == 0)
    return ok


def gemm_nt256(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x w^T (+ bias) on the wide training GEMM (include/swh_trl_amd.h
    swh_gemm_nt256): x [M, K], w [N, K], bf16."""
    _dev(x, "gemm_nt256")
    if not gemm_nt256_eligible(x, w, out):
        raise ValueError(f"gemm_nt256: unsupported operands {tuple(x.shape)} x {tuple(w.shape)}")
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    if bias is not None and (bias.dtype != torch.bfloat16 or not bias.is_contiguous() or bias.numel() != N
                             or bias.data_ptr() % 8):
        raise ValueError("gemm_nt256: bias must be a contiguous, 8-B aligned bf16 vector of N elements")
    call("swh_gemm_nt256", x.data_ptr(), w.data_ptr(), _p(bias), out.data_ptr(), M, N, K, x.stride(0), w.stride(0),
         out.stride(0), _stream())
    return out


def gemm_tn256_eligible(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """Shapes swh_gemm_tn256_partials serves: bf16 [M, N] / [M, K], M % 64, N and K % 16,
    31-bit byte offsets per operand."""
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.dim() == 2 and x.dim() == 2
            and dy.shape[0] == x.shape[0] and dy.shape[0] % 64 == 0 and dy.shape[1] % 16 == 0
            and x.shape[1] % 16 == 0 and dy.stride(1) == 1 and x.stride(1) == 1 and dy.stride(0) % 8 == 0
            and x.stride(0) % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0
            and dy.shape[0] * dy.stride(0) * 2 < 2 ** 31 and x.shape[0] * x.stride(0) * 2 < 2 ** 31)


def gemm_tn256_accumulate(grad: torch.Tensor, dy: torch.Tensor, x: torch.Tensor, splits: int) -> torch.Tensor:
    """grad [N, K] += dy^T x over the tokens on the 256 x 256 schedule
    (include/swh_trl_amd.h swh_gemm_tn256_partials + swh_gemm_tn_fold): `splits`
    token ranges in fp32 partials, folded in order and rounded once into grad.
    Returns the partials buffer (keep it alive until the stream has run the launches)."""
    _dev(dy, "gemm_tn256_accumulate")
    if not gemm_tn256_eligible(dy, x):
        raise ValueError(f"gemm_tn256_accumulate: unsupported operands {tuple(dy.shape)} / {tuple(x.shape)}")
    M, N = dy.shape
    K = x.shape[1]
    if grad.numel() != N * K or not grad.is_contiguous():
        raise ValueError("gemm_tn256_accumulate: grad must be a contiguous [N, K] view")
    part = torch.empty(splits * N * K, device=dy.device, dtype=torch.float32)
    call("swh_gemm_tn256_partials", dy.data_ptr(), x.data_ptr(), part.data_ptr(), M, N, K, dy.stride(0), x.stride(0),
         int(splits), _stream())
    call("swh_gemm_tn_fold", part.data_ptr(), int(splits), N * K, grad.data_ptr(),
         _dtype_code(grad, "gemm_tn256_accumulate"), _stream())
    return part


def gemm_tn_eligible(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """Shapes swh_gemm_tn_partials serves: bf16 [M, N] / [M, K], M % 64, N and K % 128."""
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.dim() == 2 and x.dim() == 2
            and dy.shape[0] == x.shape[0] and dy.shape[0] % 64 == 0 and dy.shape[1] % 128 == 0
            and x.shape[1] % 128 == 0 and dy.stride(1) == 1 and x.stride(1) == 1 and dy.stride(0) % 8 == 0
            and x.stride(0) % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def gemm_tn_accumulate(grad: torch.Tensor, dy: torch.Tensor, x: torch.Tensor, splits: int,
                       bias_grad: Optional[torch.Tensor] = None) -> torch.Tensor:
    """grad [N, K] += dy^T x over the tokens (include/swh_trl_amd.h
    swh_gemm_tn_partials + swh_gemm_tn_fold): `splits` token ranges in fp32
    partials, folded in order and rounded once into grad (bf16 / f32).  With
    bias_grad [N]: also bias_grad += the token sums of dy (the same kernel's
    per-split column sums, folded in split order by swh_rmsnorm_dw_accum).
    Returns the partials buffer (keep it alive until the stream has run the
    launches)."""
    _dev(dy, "gemm_tn_accumulate")
    if not gemm_tn_eligible(dy, x):
        raise ValueError(f"gemm_tn_accumulate: unsupported operands {tuple(dy.shape)} / {tuple(x.shape)}")
    M, N = dy.shape
    K = x.shape[1]
    if grad.numel() != N * K or not grad.is_contiguous():
        raise ValueError("gemm_tn_accumulate: grad must be a contiguous [N, K] view")
    if bias_grad is not None and (bias_grad.numel() != N or not bias_grad.is_contiguous()):
        raise ValueError("gemm_tn_accumulate: bias_grad must be a contiguous [N] view")
    part = torch.empty(splits * N * K + (splits * N if bias_grad is not None else 0), device=dy.device,
                       dtype=torch.float32)
    colsum = part[splits * N * K:] if bias_grad is not None else None
    call("swh_gemm_tn_partials", dy.data_ptr(), x.data_ptr(), part.data_ptr(), _p(colsum), M, N, K, dy.stride(0),
         x.stride(0), int(splits), _stream())
    call("swh_gemm_tn_fold", part.data_ptr(), int(splits), N * K, grad.data_ptr(),
         _dtype_code(grad, "gemm_tn_accumulate"), _stream())
    if bias_grad is not None:
        call("swh_rmsnorm_dw_accum", colsum.data_ptr(), int(splits), N, bias_grad.data_ptr(),
             _dtype_code(bias_grad, "gemm_tn_accumulate"), _stream())
    return part


def frag_pack(w: torch.Tensor, norm_w: Optional[torch.Tensor] = None, *, silu: bool = False,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """w [N, K] ([2N, K] gate|up with silu; K % 128 == 0), optionally folded
    with the RMSNorm weight, in the MFMA-fragment order decode_gemm_fragw reads
    (swh_frag_pack); same shape as w."""
    _dev(w, "frag_pack")
    rows, K = w.shape
    N = rows // 2 if silu else rows
    out = torch.empty_like(w) if out is None else out
    call("swh_frag_pack", w.data_ptr(), _p(norm_w), N, K, int(bool(silu)), out.data_ptr(), _stream())
    return out


def decode_gemm_fragw(x: torch.Tensor, w: torch.Tensor, *, eps: float = 1e-6, bias: Optional[torch.Tensor] = None,
                      residual: Optional[torch.Tensor] = None, silu: bool = False, y: Optional[torch.Tensor] = None,
                      workspace: Optional[torch.Tensor] = None, ss_in: Optional[torch.Tensor] = None,
                      ss_out: Optional[torch.Tensor] = None, act_frag: int = 0) -> torch.Tensor:
    """decode_gemm (no norm_w) over w packed by frag_pack ([N, K], [2N, K] with
    silu) (include/swh_trl_amd.h swh_decode_gemm_fragw): bit-identical results.
    act_frag bit 0: write the SiLU output in fragment order; bit 1: read x in it."""
    _dev(x, "decode_gemm_fragw")
    M, K = x.shape
    N = w.shape[0] // 2 if silu else w.shape[0]
    if residual is None and y is None:
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
    ldy = residual.stride(0) if residual is not None else y.stride(0)
    ws = workspace if workspace is not None else gemm_workspace(x.device)
    call("swh_decode_gemm_fragw", x.data_ptr(), w.data_ptr(), M, N, K, float(eps), _p(bias), _p(residual),
         int(bool(silu)), _p(y), ldy, _p(ss_in), _p(ss_out), int(act_frag), ws.data_ptr(), ws.numel(), _stream())
    return residual if residual is not None else y


def wide_gemm_eligible(M: int, N: int, K: int, silu: bool = False) -> bool:
    """Shapes swh_wide_gemm_packed serves (include/swh_trl_amd.h)."""
    return bool(_lib.load().swh_wide_gemm_eligible(M, N, K, int(bool(silu))))


def wide_pack(w: torch.Tensor, norm_w: Optional[torch.Tensor] = None, *, silu: bool = False,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """w [N, K] (or [2N, K] gate|up with silu) in swh_wide_gemm_packed's
    fragment order, optionally folded with the RMSNorm weight (swh_wide_pack).
    Returns a flat bf16 tensor of w.numel() elements."""
    _dev(w, "wide_pack")
    rows, K = w.shape
    N = rows // 2 if silu else rows
    if out is None:
        out = torch.empty(w.numel(), device=w.device, dtype=w.dtype)
    call("swh_wide_pack", w.data_ptr(), _p(norm_w), N, K, int(bool(silu)), out.data_ptr(), _stream())
    return out


def wide_gemm_packed(x: torch.Tensor, w_packed: torch.Tensor, N: int, *, eps: float = 1e-6,
                     bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None, silu: bool = False,
                     y: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
                     ss_in: Optional[torch.Tensor] = None, ss_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """decode_gemm over a wide_pack'ed weight (include/swh_trl_amd.h
    swh_wide_gemm_packed); N output columns."""
    _dev(x, "wide_gemm_packed")
    M, K = x.shape
    if w_packed.numel() != (2 if silu else 1) * N * K:
        raise ValueError("wide_gemm_packed: packed weight size does not match N, K")
    if residual is None and y is None:
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
    ldy = residual.stride(0) if residual is not None else y.stride(0)
    ws = workspace if workspace is not None else gemm_workspace(x.device)
    call("swh_wide_gemm_packed", x.data_ptr(), w_packed.data_ptr(), M, N, K, float(eps), _p(bias), _p(residual),
         int(bool(silu)), _p(y), ldy, _p(ss_in), _p(ss_out), ws.data_ptr(), ws.numel(), _stream())
    return residual if residual is not None else y


def lm_head_sample_supported(params, V: int, K: int, wide_rows: int = 0, logp: bool = False) -> bool:
    """The fused lm-head sampler covers unfiltered sampling (temperature,
    greedy, EOS suppression); the rest goes through logits + sample_step.
    K <= 1024: the tile kernel (any weight order), also with the drawn tokens'
    log-probs (logp); K > 1024: wide_gemm's 256-row tiles over a fragment-order
    (wide_pack) weight, for wide_rows (the batch, <= 64) rows and V % 256 == 0
    (wide_rows 0: not available), without log-probs."""
    filtered = not params.greedy and ((0 < params.top_k < V) or params.top_p < 1.0 or params.min_p > 0.0)
    if filtered or params.repetition_penalty != 1.0 or K % 64 or V % 16:
        return False
    if K <= 1024:
        return True
    if logp:
        return False
    return bool(wide_rows) and V % 256 == 0 and wide_gemm_eligible(wide_rows, V, K)


def _check_logp_out(out_logp: torch.Tensor, out_tokens: torch.Tensor) -> None:
    """The log-prob output shares out_tokens' row stride (out_ld) and shape."""
    if (out_logp.dtype != torch.float32 or out_logp.shape != out_tokens.shape
            or out_logp.stride() != out_tokens.stride() or out_logp.device != out_tokens.device):
        raise ValueError("lm_head_sample: out_logp must be fp32 with out_tokens' shape and strides")


def lm_head_sample(x: torch.Tensor, w: torch.Tensor, params, rng: torch.Tensor, step: torch.Tensor,
                   finished: torch.Tensor, out_tokens: torch.Tensor, cur_tokens: Optional[torch.Tensor] = None, *,
                   norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6, ss_in: Optional[torch.Tensor] = None,
                   workspace: Optional[torch.Tensor] = None, fragw: int = 0,
                   out_logp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """lm head + the unfiltered sampler in one pass, no logits tensor
    (include/swh_trl_amd.h swh_lm_head_sample; fragw 1: w packed by frag_pack,
    or the flat wide_pack copy at K > 1024, swh_lm_head_sample_fragw).  Writes out_tokens[:, *step], cur_tokens,
    finished; returns out_tokens.  out_logp (fp32, the layout of out_tokens): also the
    drawn tokens' log-probs under the processed distribution (swh_lm_head_sample_logp,
    K <= 1024)."""
    import ctypes
    _dev(x, "lm_head_sample")
    M, K = x.shape
    V = w.numel() // K  # [V, K], or the flat wide_pack copy
    need = _lib.load().swh_lm_head_sample_workspace_bytes(M, V, K)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    if fragw and norm_w is not None:
        raise ValueError("lm_head_sample: a fragment-order weight carries the folded norm (norm_w must be None)")
    if out_logp is not None:
        _check_logp_out(out_logp, out_tokens)
        call("swh_lm_head_sample_logp", x.data_ptr(), w.data_ptr(), M, V, K, _p(norm_w), float(eps), _p(ss_in),
             int(bool(fragw)), ctypes.byref(params), rng.data_ptr(), step.data_ptr(), finished.data_ptr(),
             out_tokens.data_ptr(), out_tokens.stride(0), _p(cur_tokens), out_logp.data_ptr(), None, None, None,
             workspace.data_ptr(), workspace.numel(), _stream())
        return out_tokens
    head = (x.data_ptr(), w.data_ptr(), M, V, K) + (() if fragw else (_p(norm_w),)) + (float(eps), _p(ss_in))
    call("swh_lm_head_sample_fragw" if fragw else "swh_lm_head_sample", *head,
         ctypes.byref(params), rng.data_ptr(), step.data_ptr(), finished.data_ptr(), out_tokens.data_ptr(),
         out_tokens.stride(0), _p(cur_tokens), workspace.data_ptr(), workspace.numel(), _stream())
    return out_tokens


def lm_head_sample_step(x: torch.Tensor, w: torch.Tensor, params, rng: torch.Tensor, step: torch.Tensor,
                        finished: torch.Tensor, out_tokens: torch.Tensor, cur_tokens: torch.Tensor,
                        embed: torch.Tensor, x_next: torch.Tensor, ss_next: Optional[torch.Tensor], *,
                        norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6, ss_in: Optional[torch.Tensor] = None,
                        workspace: torch.Tensor, fragw: int = 0,
                        out_logp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """lm_head_sample + the next step's input: x_next = embed[drawn token]
    (+ RMSNorm partials ss_next) and *step += 1 once every row has read it
    (include/swh_trl_amd.h swh_lm_head_sample_step).  `workspace` must have
    been zeroed once at allocation.  out_logp: the drawn tokens' log-probs too
    (swh_lm_head_sample_logp, K <= 1024)."""
    import ctypes
    _dev(x, "lm_head_sample_step")
    M, K = x.shape
    V = w.numel() // K  # [V, K], or the flat wide_pack copy
    if workspace.numel() < _lib.load().swh_lm_head_sample_workspace_bytes(M, V, K):
        raise ValueError("lm_head_sample_step: workspace too small")
    if fragw and norm_w is not None:
        raise ValueError("lm_head_sample_step: a fragment-order weight carries the folded norm (norm_w must be None)")
    if out_logp is not None:
        _check_logp_out(out_logp, out_tokens)
        call("swh_lm_head_sample_logp", x.data_ptr(), w.data_ptr(), M, V, K, _p(norm_w), float(eps), _p(ss_in),
             int(bool(fragw)), ctypes.byref(params), rng.data_ptr(), step.data_ptr(), finished.data_ptr(),
             out_tokens.data_ptr(), out_tokens.stride(0), cur_tokens.data_ptr(), out_logp.data_ptr(),
             embed.data_ptr(), x_next.data_ptr(), _p(ss_next), workspace.data_ptr(), workspace.numel(), _stream())
        return out_tokens
    head = (x.data_ptr(), w.data_ptr(), M, V, K) + (() if fragw else (_p(norm_w),)) + (float(eps), _p(ss_in))
    call("swh_lm_head_sample_step_fragw" if fragw else "swh_lm_head_sample_step", *head,
         ctypes.byref(params), rng.data_ptr(), step.data_ptr(), finished.data_ptr(), out_tokens.data_ptr(),
         out_tokens.stride(0), cur_tokens.data_ptr(), embed.data_ptr(), x_next.data_ptr(), _p(ss_next),
         workspace.data_ptr(), workspace.numel(), _stream())
    return out_tokens


class AttentionFn(torch.autograd.Function):
    """Causal GQA attention, q [B, Hq, L, D], k/v [B, Hkv, L, D] bf16 -> o
    [B, Hq, L, D] (include/swh_trl_amd.h swh_attn_fwd / swh_attn_bwd).
    key_mask int32 [B, L] (0 = padding) with first_valid int32 [B] (index of
    the first valid key), or both None: transformers' padded causal mask as
    engine/model.py builds it (a query with no valid key sees itself)."""

    @staticmethod
    def forward(ctx, q, k, v, scale: float, key_mask=None, first_valid=None):
        _dev(q, "attention")
        B, Hq, L, D = q.shape
        Hkv = k.shape[1]
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out = torch.empty_like(q)
        lse = torch.empty(B, Hq, L, device=q.device, dtype=torch.float32)
        call("swh_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), B, Hq, Hkv, L, D, float(scale),
             _p(key_mask), _p(first_valid), out.data_ptr(), lse.data_ptr(), _stream())
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.km, ctx.fv, ctx.scale = key_mask, first_valid, float(scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        B, Hq, L, D = q.shape
        Hkv = k.shape[1]
        dout = dout.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(B, Hq, L, device=q.device, dtype=torch.float32)
        args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), B, Hq,
                Hkv, L, D, ctx.scale, _p(ctx.km), _p(ctx.fv), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                dv.data_ptr())
        aux = _aux_stream(q.device)
        if aux is None:
            call("swh_attn_bwd_parts", *args, 7, _stream())
            return dq, dk, dv, None, None, None
        # dK/dV on the auxiliary stream beside dQ (both read delta only): the key
        # tiles' uneven causal work leaves CUs the dQ blocks fill
        main = torch.cuda.current_stream(q.device)
        call("swh_attn_bwd_parts", *args, 1, _stream())
        aux.wait_stream(main)
        with torch.cuda.stream(aux):
            call("swh_attn_bwd_parts", *args, 4, _stream())
        call("swh_attn_bwd_parts", *args, 2, _stream())
        main.wait_stream(aux)
        return dq, dk, dv, None, None, None


def attn_view(seg1, seg0=None):
    """swh_attn_view of an attention operand: seg = (tensor, stride per sequence,
    per head, per row, divisor) in elements; seg0 holds rows l < P (None: P = 0)."""
    v = _lib.AttnView()
    for i, seg in ((0, seg0), (1, seg1)):
        if seg is None:
            v.div[i] = 1
            continue
        t, sb, sh, sl, div = seg
        v.base[i] = t.data_ptr()
        v.sb[i], v.sh[i], v.sl[i], v.div[i] = int(sb), int(sh), int(sl), int(div)
    return v


def _bhld(t):
    """plain [B, H, L, D] tensor -> its view segment."""
    _, H, L, D = t.shape
    return (t, H * L * D, L * D, D, 1)


def _attn_bwd(views, lse, dims, scale, km, fv, delta, dviews, dev):
    """swh_attn_bwd_v_parts, dK/dV on the auxiliary stream beside dQ when one is on."""
    import ctypes as C
    B, Hq, Hkv, L, P, G, D = dims
    vq, vk, vv, vo, vd = (C.byref(x) for x in views)
    dq, dk, dv = (C.byref(x) for x in dviews)
    args = (vq, vk, vv, vo, vd, lse.data_ptr(), B, Hq, Hkv, L, P, G, D, float(scale), _p(km), _p(fv),
            delta.data_ptr(), dq, dk, dv)
    aux = _aux_stream(dev)
    if aux is None:
        call("swh_attn_bwd_v_parts", *args, 7, _stream())
        return
    main = torch.cuda.current_stream(dev)
    call("swh_attn_bwd_v_parts", *args, 1, _stream())
    aux.wait_stream(main)
    with torch.cuda.stream(aux):
        call("swh_attn_bwd_v_parts", *args, 4, _stream())
    call("swh_attn_bwd_v_parts", *args, 2, _stream())
    main.wait_stream(aux)


class AttentionTokFn(torch.autograd.Function):
    """AttentionFn with the output token-major, [B, L, Hq D] (the o_proj input
    as it stands: no transpose copy forward or backward)."""

    @staticmethod
    def forward(ctx, q, k, v, scale: float, key_mask=None, first_valid=None):
        _dev(q, "attention")
        B, Hq, L, D = q.shape
        Hkv = k.shape[1]
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out = torch.empty(B, L, Hq * D, device=q.device, dtype=q.dtype)
        lse = torch.empty(B, Hq, L, device=q.device, dtype=torch.float32)
        vo = attn_view((out, L * Hq * D, D, Hq * D, 1))
        import ctypes as C
        call("swh_attn_fwd_v", *(C.byref(x) for x in (attn_view(_bhld(q)), attn_view(_bhld(k)),
                                                    attn_view(_bhld(v)), vo)),
             B, Hq, Hkv, L, 0, 0, D, float(scale), _p(key_mask), _p(first_valid), lse.data_ptr(), _stream())
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.km, ctx.fv, ctx.scale = key_mask, first_valid, float(scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        B, Hq, L, D = q.shape
        Hkv = k.shape[1]
        dout = dout.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(B, Hq, L, device=q.device, dtype=torch.float32)
        tok = lambda t: attn_view((t, L * Hq * D, D, Hq * D, 1))  # noqa: E731
        views = (attn_view(_bhld(q)), attn_view(_bhld(k)), attn_view(_bhld(v)), tok(out), tok(dout))
        _attn_bwd(views, lse, (B, Hq, Hkv, L, 0, 0, D), ctx.scale, ctx.km, ctx.fv, delta,
                  (attn_view(_bhld(dq)), attn_view(_bhld(dk)), attn_view(_bhld(dv))), q.device)
        return dq, dk, dv, None, None, None


class GroupedAttentionFn(torch.autograd.Function):
    """Causal GQA attention of R = U G sequences whose first P positions are the
    prompt of their group (G consecutive sequences share it) — the GRPO
    shared-prompt forward (engine/model.py hidden_states_grouped).  The group's
    prompt q_p / k_p / v_p [U, H, P, D] are read by all G sequences in place,
    each sequence's completion q_c / k_c / v_c [R, H, C, D] are its own; the
    prompt queries are computed once per group (the group's first sequence).
    Output token-major [U P + R C, Hq D]: the groups' prompt tokens, then every
    sequence's completion tokens (the o_proj input).  Backward: d prompt Q from
    the first sequence, d prompt K / V summed over the group's sequences in
    fixed order; no concatenated copies either way (swh_attn_fwd_v / _bwd_v_parts)."""

    @staticmethod
    def forward(ctx, q_p, k_p, v_p, q_c, k_c, v_c, G: int, scale: float, key_mask=None, first_valid=None):
        _dev(q_c, "attention")
        import ctypes as C
        U, Hq, P, D = q_p.shape
        R, Hkv, Cn = k_c.shape[0], k_c.shape[1], k_c.shape[2]
        L = P + Cn
        q_p, k_p, v_p, q_c, k_c, v_c = (t.contiguous() for t in (q_p, k_p, v_p, q_c, k_c, v_c))
        NP = U * P
        out = torch.empty(NP + R * Cn, Hq * D, device=q_c.device, dtype=q_c.dtype)
        lse = torch.empty(R, Hq, L, device=q_c.device, dtype=torch.float32)
        ctx.views = GroupedAttentionFn._views(q_p, k_p, v_p, q_c, k_c, v_c, out, G)
        call("swh_attn_fwd_v", *(C.byref(x) for x in ctx.views), R, Hq, Hkv, L, P, G, D, float(scale),
             _p(key_mask), _p(first_valid), lse.data_ptr(), _stream())
        ctx.save_for_backward(q_p, k_p, v_p, q_c, k_c, v_c, out, lse)
        ctx.km, ctx.fv, ctx.scale, ctx.G = key_mask, first_valid, float(scale), G
        return out

    @staticmethod
    def _views(q_p, k_p, v_p, q_c, k_c, v_c, out, G):
        U, Hq, P, D = q_p.shape
        Cn = q_c.shape[2]

        def seg(tp, tc):
            return attn_view(_bhld(tc), (tp, tp.shape[1] * P * D, P * D, D, G))
        vo = attn_view((out[U * P:], Cn * Hq * D, D, Hq * D, 1), (out, P * Hq * D, D, Hq * D, G))
        return seg(q_p, q_c), seg(k_p, k_c), seg(v_p, v_c), vo

    @staticmethod
    def backward(ctx, dout):
        q_p, k_p, v_p, q_c, k_c, v_c, out, lse = ctx.saved_tensors
        U, Hq, P, D = q_p.shape
        R, Hkv, Cn = k_c.shape[0], k_c.shape[1], k_c.shape[2]
        G, L = ctx.G, P + Cn
        dout = dout.contiguous()
        vq, vk, vv, vo = GroupedAttentionFn._views(q_p, k_p, v_p, q_c, k_c, v_c, out, G)
        vd = attn_view((dout[U * P:], Cn * Hq * D, D, Hq * D, 1), (dout, P * Hq * D, D, Hq * D, G))
        dq_p, dq_c = torch.empty_like(q_p), torch.empty_like(q_c)
        dk_c, dv_c = torch.empty_like(k_c), torch.empty_like(v_c)
        dk_r = torch.empty(R, Hkv, P, D, device=q_c.device, dtype=q_c.dtype)  # per sequence: summed below
        dv_r = torch.empty_like(dk_r)
        vdq = attn_view(_bhld(dq_c), (dq_p, Hq * P * D, P * D, D, G))
        vdk = attn_view(_bhld(dk_c), _bhld(dk_r))
        vdv = attn_view(_bhld(dv_c), _bhld(dv_r))
        delta = torch.empty(R, Hq, L, device=q_c.device, dtype=torch.float32)
        _attn_bwd((vq, vk, vv, vo, vd), lse, (R, Hq, Hkv, L, P, G, D), ctx.scale, ctx.km, ctx.fv, delta,
                  (vdq, vdk, vdv), q_c.device)
        dk_p = dk_r.view(U, G, Hkv, P, D).sum(1)
        dv_p = dv_r.view(U, G, Hkv, P, D).sum(1)
        return dq_p, dk_p, dv_p, dq_c, dk_c, dv_c, None, None, None, None


_AUX_STREAMS: dict = {}


def _aux_stream(dev: torch.device):
    """Second stream for the dK/dV half of the attention backward.  Every tensor it
    touches was allocated on, and is joined back to, the calling stream before the
    backward returns."""
    if dev.type != "cuda":
        return None
    st = _AUX_STREAMS.get(dev.index)
    if st is None:
        st = _AUX_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return st


def attention_supported(D: int) -> bool:
    return D in (64, 128)


class QKVRopeSegFn(torch.autograd.Function):
    """QKVRopeFn over the two token segments of the shared-prompt forward in one
    node: qkv [U P + R C, (Hq+2Hkv) D] -> (q, k, v of the U prompts [U, H, P, D],
    of the R completions [R, H, C, D]); the backward writes both parts of
    d qkv into one buffer (no zero fill, copy and add of two slice gradients)."""

    @staticmethod
    def forward(ctx, qkv, pos_p, pos_c, cos, sin, U: int, P: int, R: int, C: int, Hq: int, Hkv: int, D: int):
        _dev(qkv, "qkv_rope")
        qkv_c = qkv.contiguous()
        NP = U * P
        outs = []
        pp = pos_p.reshape(-1).to(torch.int64).contiguous()
        pc = pos_c.reshape(-1).to(torch.int64).contiguous()
        for (B, L, pos, x) in ((U, P, pp, qkv_c[:NP]), (R, C, pc, qkv_c[NP:])):
            q = torch.empty(B, Hq, L, D, device=qkv.device, dtype=qkv.dtype)
            k = torch.empty(B, Hkv, L, D, device=qkv.device, dtype=qkv.dtype)
            v = torch.empty(B, Hkv, L, D, device=qkv.device, dtype=qkv.dtype)
            call("swh_qkv_rope", x.data_ptr(), pos.data_ptr(), cos.data_ptr(), sin.data_ptr(), B, L, Hq, Hkv, D,
                 q.data_ptr(), k.data_ptr(), v.data_ptr(), 0, _dtype_code(qkv_c, "qkv_rope"), _stream())
            outs += [q, k, v]
        ctx.save_for_backward(pp, pc, cos, sin)
        ctx.dims = (U, P, R, C, Hq, Hkv, D)
        ctx.dtype = qkv.dtype
        return tuple(outs)

    @staticmethod
    def backward(ctx, dq_p, dk_p, dv_p, dq_c, dk_c, dv_c):
        pp, pc, cos, sin = ctx.saved_tensors
        U, P, R, C, Hq, Hkv, D = ctx.dims
        dt = ctx.dtype
        NP = U * P
        dqkv = torch.empty(NP + R * C, (Hq + 2 * Hkv) * D, device=pp.device, dtype=dt)
        for (B, L, pos, x, grads) in ((U, P, pp, dqkv[:NP], (dq_p, dk_p, dv_p)),
                                      (R, C, pc, dqkv[NP:], (dq_c, dk_c, dv_c))):
            dq, dk, dv = (torch.zeros(B, H, L, D, device=pp.device, dtype=dt) if t is None else t.contiguous()
                          for t, H in zip(grads, (Hq, Hkv, Hkv)))
            call("swh_qkv_rope", x.data_ptr(), pos.data_ptr(), cos.data_ptr(), sin.data_ptr(), B, L, Hq, Hkv, D,
                 dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), 1, _dtype_code(dq, "qkv_rope"), _stream())
        return dqkv, None, None, None, None, None, None, None, None, None, None, None


class QKVRopeFn(torch.autograd.Function):
    """qkv [B, L, (Hq+2Hkv) D] -> q, k (rotated), v as contiguous [B, H, L, D]
    (include/swh_trl_amd.h swh_qkv_rope); backward writes d qkv in one pass."""

    @staticmethod
    def forward(ctx, qkv, positions, cos, sin, Hq: int, Hkv: int, D: int):
        _dev(qkv, "qkv_rope")
        B, L, _ = qkv.shape
        qkv_c = qkv.contiguous()
        pos = positions.reshape(-1).to(torch.int64).contiguous()
        q = torch.empty(B, Hq, L, D, device=qkv.device, dtype=qkv.dtype)
        k = torch.empty(B, Hkv, L, D, device=qkv.device, dtype=qkv.dtype)
        v = torch.empty(B, Hkv, L, D, device=qkv.device, dtype=qkv.dtype)
        call("swh_qkv_rope", qkv_c.data_ptr(), pos.data_ptr(), cos.data_ptr(), sin.data_ptr(), B, L, Hq, Hkv, D,
             q.data_ptr(), k.data_ptr(), v.data_ptr(), 0, _dtype_code(qkv_c, "qkv_rope"), _stream())
        ctx.save_for_backward(pos, cos, sin)
        ctx.dims = (B, L, Hq, Hkv, D)
        ctx.dtype = qkv.dtype
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        pos, cos, sin = ctx.saved_tensors
        B, L, Hq, Hkv, D = ctx.dims
        dt = ctx.dtype
        dq = torch.zeros(B, Hq, L, D, device=pos.device, dtype=dt) if dq is None else dq.contiguous()
        dk = torch.zeros(B, Hkv, L, D, device=pos.device, dtype=dt) if dk is None else dk.contiguous()
        dv = torch.zeros(B, Hkv, L, D, device=pos.device, dtype=dt) if dv is None else dv.contiguous()
        dqkv = torch.empty(B, L, (Hq + 2 * Hkv) * D, device=pos.device, dtype=dt)
        call("swh_qkv_rope", dqkv.data_ptr(), pos.data_ptr(), cos.data_ptr(), sin.data_ptr(), B, L, Hq, Hkv, D,
             dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), 1, _dtype_code(dq, "qkv_rope"), _stream())
        return dqkv, None, None, None, None, None, None
