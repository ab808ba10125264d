"""Timing of the training-step building blocks at the bench shape (Qwen2.5-0.5B,
64 sequences x 384 tokens): every GEMM of the forward/backward under each
BLAS backend torch offers on ROCm, SDPA with and without the GQA repeat, and
the fused RMSNorm backward.  Tuning aid, not part of the product.

    python tools/bench_train.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps  # ms


def gemms():
    T, H, I, Q, V, CH = 64 * 384, 896, 4864, 1152, 151936, 4096
    bf = dict(device="cuda", dtype=torch.bfloat16)
    shapes = {"qkv": (Q, H), "o": (H, H), "gate_up": (2 * I, H), "down": (H, I), "lm": (V, H)}
    backends = ["default"]
    for b in ("cublaslt", "cublas", "ck"):
        try:
            torch.backends.cuda.preferred_blas_library(b)
            backends.append(b)
        except Exception as e:  # not offered by this build
            print(f"[bench_train] backend {b}: {e!r}"[:200], flush=True)
    torch.backends.cuda.preferred_blas_library("cublaslt")
    print(f"{'gemm':10s} {'pass':6s} " + " ".join(f"{b:>18s}" for b in backends), flush=True)
    total = {b: 0.0 for b in backends}
    for name, (N, K) in shapes.items():
        rows = CH if name == "lm" else T
        mult = (T // CH) if name == "lm" else 24
        w = torch.randn(N, K, **bf) * 0.02
        x = torch.randn(rows, K, **bf)
        dy = torch.randn(rows, N, **bf)
        gw = torch.zeros(N, K, **bf)
        passes = {"fwd": lambda: x @ w.t(), "dgrad": lambda: dy @ w, "wgrad": lambda: gw.addmm_(dy.t(), x)}
        for pn, fn in passes.items():
            res = []
            for b in backends:
                if b != "default":
                    torch.backends.cuda.preferred_blas_library(b)
                try:
                    ms = _t(fn)
                    res.append(f"{ms * 1000:8.1f}us {2 * rows * N * K / ms / 1e9:5.0f}TF")
                    total[b] += ms * mult
                except Exception as e:
                    res.append(f"{'err':>18s}")
                torch.backends.cuda.preferred_blas_library("cublaslt")
            print(f"{name:10s} {pn:6s} " + " ".join(f"{r:>18s}" for r in res), flush=True)
    print("per-step GEMM ms: " + "  ".join(f"{b}={v:.1f}" for b, v in total.items()), flush=True)


def sdpa():
    B, Hq, Hkv, L, D = 64, 14, 2, 384, 64
    bf = dict(device="cuda", dtype=torch.bfloat16)
    q = torch.randn(B, Hq, L, D, **bf, requires_grad=True)
    k = torch.randn(B, Hkv, L, D, **bf, requires_grad=True)
    v = torch.randn(B, Hkv, L, D, **bf, requires_grad=True)
    go = torch.randn(B, Hq, L, D, **bf)
    F = torch.nn.functional

    def rep():
        kk, vv = k.repeat_interleave(7, 1), v.repeat_interleave(7, 1)
        o = F.scaled_dot_product_attention(q, kk, vv, is_causal=True, scale=D ** -0.5)
        o.backward(go)

    def gqa():
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=D ** -0.5, enable_gqa=True)
        o.backward(go)

    def rep_fwd():
        with torch.no_grad():
            kk, vv = k.repeat_interleave(7, 1), v.repeat_interleave(7, 1)
            F.scaled_dot_product_attention(q, kk, vv, is_causal=True, scale=D ** -0.5)

    def gqa_fwd():
        with torch.no_grad():
            F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=D ** -0.5, enable_gqa=True)

    flops = 4 * B * Hq * L * L * D / 2  # causal
    for name, fn, f in (("repeat fwd", rep_fwd, flops), ("gqa fwd", gqa_fwd, flops),
                        ("repeat fwd+bwd", rep, 3.5 * flops), ("gqa fwd+bwd", gqa, 3.5 * flops)):
        try:
            ms = _t(fn)
            print(f"sdpa {name:16s} {ms * 1000:8.1f} us  {f / ms / 1e9:6.0f} TF/s", flush=True)
        except Exception as e:
            print(f"sdpa {name:16s} error {e!r}"[:200], flush=True)


def norm_bwd():
    from swh_trl_amd.engine.model import _RMSNorm
    T, H = 64 * 384, 896
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(H, device="cuda", dtype=torch.bfloat16)
    gw = torch.zeros(H, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)

    def fb():
        y = _RMSNorm.apply(x, w, gw, 1e-6)
        y.backward(dy)

    ms = _t(fb)
    print(f"rmsnorm fwd+bwd (T={T}, H={H}) {ms * 1000:8.1f} us  ({5 * T * H * 2 / ms / 1e6:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    gemms()
    sdpa()
    norm_bwd()
