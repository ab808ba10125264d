"""Training-attention timing at the GRPO scoring shape (B=64, 14/2 heads,
L=384, D=64, causal, bf16): torch SDPA backends and GQA handling, forward
and forward+backward.  Tuning aid.   python tools/bench_attn.py
"""
import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    dev = torch.device("cuda:0")
    B, Hq, Hkv, L, D = 64, 14, 2, 384, 64
    q = torch.randn(B, Hq, L, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Hkv, L, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Hkv, L, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, Hq, L, D, device=dev, dtype=torch.bfloat16)
    mask = torch.ones(L, L, device=dev, dtype=torch.bool).tril()[None, None].expand(B, 1, L, L)

    def run(backend, gqa, use_mask, bwd):
        def f():
            kk, vv = (k, v) if gqa else (k.repeat_interleave(Hq // Hkv, 1), v.repeat_interleave(Hq // Hkv, 1))
            ctx = sdpa_kernel([backend]) if backend is not None else torch.enable_grad()
            with ctx:
                if use_mask:
                    o = F.scaled_dot_product_attention(q, kk, vv, attn_mask=mask, scale=D ** -0.5, enable_gqa=gqa)
                else:
                    o = F.scaled_dot_product_attention(q, kk, vv, is_causal=True, scale=D ** -0.5, enable_gqa=gqa)
            if bwd:
                o.backward(do)
        return f

    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from swh_trl_amd import nn_ops

    def hip(bwd):
        def f():
            o = nn_ops.AttentionFn.apply(q, k, v, D ** -0.5, None, None)
            if bwd:
                o.backward(do)
        return f
    print(f"hip (csrc/attn.hip)     fwd {timeit(hip(False)) * 1000:8.1f} us  fwd+bwd {timeit(hip(True)) * 1000:8.1f} us",
          flush=True)
    if os.environ.get("HIP_ONLY"):
        return
    for name, be in (("default", None), ("flash", SDPBackend.FLASH_ATTENTION),
                     ("efficient", SDPBackend.EFFICIENT_ATTENTION), ("math", SDPBackend.MATH)):
        for gqa in (True, False):
            for use_mask in (False, True):
                try:
                    tf = timeit(run(be, gqa, use_mask, False))
                    tb = timeit(run(be, gqa, use_mask, True))
                    print(f"{name:9s} gqa={int(gqa)} mask={int(use_mask)}  fwd {tf * 1000:8.1f} us  fwd+bwd {tb * 1000:8.1f} us",
                          flush=True)
                except Exception as e:  # backend refuses the combination
                    print(f"{name:9s} gqa={int(gqa)} mask={int(use_mask)}  n/a ({type(e).__name__})", flush=True)


if __name__ == "__main__":
    main()
