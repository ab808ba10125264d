"""Training attention at the bench shape (tuning aid, not part of the product):
the GRPO shared-prompt layout of config 2 — 8 groups x G 8, prompt 128 (left
padded) + completion 256, 14 / 2 heads x 64 — forward and backward through
nn_ops.GroupedAttentionFn, timed with events over graph-free repetitions.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python tools/bench_attn.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--P", type=int, default=128)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--hq", type=int, default=14)
    ap.add_argument("--hkv", type=int, default=2)
    a = ap.parse_args()
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    U, G, P, C, D = a.groups, a.G, a.P, a.C, a.D
    R, L = U * G, a.P + a.C

    def t(*shape):
        return (torch.randn(*shape, generator=g) * 0.5).to(dev, torch.bfloat16).requires_grad_(True)
    q_p, k_p, v_p = t(U, a.hq, P, D), t(U, a.hkv, P, D), t(U, a.hkv, P, D)
    q_c, k_c, v_c = t(R, a.hq, C, D), t(R, a.hkv, C, D), t(R, a.hkv, C, D)
    pad = torch.randint(0, P // 4, (U,), generator=g).repeat_interleave(G)  # left padding per group
    km = (torch.arange(L)[None] >= pad[:, None]).int()
    ends = torch.randint(C // 2, C + 1, (R,), generator=g)  # right padding after each row's end
    km[:, P:] &= (torch.arange(C)[None] < ends[:, None]).int()
    fv = pad.int()
    km, fv = km.to(dev), fv.to(dev)
    scale = D ** -0.5
    dout = torch.randn(U * P + R * C, a.hq * D, generator=g).to(dev, torch.bfloat16)
    fn = nn_ops.GroupedAttentionFn.apply

    def fwd():
        return fn(q_p, k_p, v_p, q_c, k_c, v_c, G, scale, km, fv)

    def step():
        out = fwd()
        torch.autograd.grad(out, (q_p, k_p, v_p, q_c, k_c, v_c), dout)

    for f in (fwd, step):
        f()
    torch.cuda.synchronize()
    res = {}
    for name, f in (("forward", fwd), ("forward+backward", step)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            f()
        e1.record()
        e1.synchronize()
        res[name] = 1000 * e0.elapsed_time(e1) / a.reps
    flops_fwd = 0
    for r in range(R):
        for qi in range(L):
            if r % G and qi < P:
                continue
            flops_fwd += 4 * D * (qi + 1)
    flops_fwd *= a.hq
    print(f"R {R} L {L} (P {P} + C {C}) heads {a.hq}/{a.hkv} D {D}: forward {res['forward']:.1f} us "
          f"({flops_fwd / res['forward'] / 1e6:.1f} TF/s causal), forward+backward {res['forward+backward']:.1f} us "
          f"(backward {res['forward+backward'] - res['forward']:.1f} us, "
          f"{2.5 * flops_fwd / (res['forward+backward'] - res['forward']) / 1e6:.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
