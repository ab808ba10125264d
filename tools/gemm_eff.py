"""Efficiency of every training GEMM at the bench step's shapes, through the
product's own path (TunableOp use-only table, swh_trl_amd/gemm_tuning.py):
the shared-prompt forward's 17408 tokens (8 x 128 prompt + 64 x 256 completion),
the 4096-row lm-head chunks, the token-split weight gradients of the small
projections.  Prints us per call, TFLOP/s and the per-step total.

    python tools/gemm_eff.py [--tokens 17408]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def _t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=17408)
    args = ap.parse_args()
    from swh_trl_amd import gemm_tuning
    from swh_trl_amd.engine.model import _dw_split
    gemm_tuning.enable()
    T, H, I, Q, V, CH, L = args.tokens, 896, 4864, 1152, 151936, 4096, 24
    bf = dict(device="cuda", dtype=torch.bfloat16)
    rows = []
    total = 0.0
    for name, (N, K) in {"qkv": (Q, H), "o": (H, H), "gate_up": (2 * I, H), "down": (H, I), "lm": (V, H)}.items():
        M = CH if name == "lm" else T
        per_step = (16384 // CH) if name == "lm" else L
        w = torch.randn(N, K, **bf) * 0.02
        x = torch.randn(M, K, **bf)
        dy = torch.randn(M, N, **bf)
        gw = torch.zeros(N, K, **bf)
        S = _dw_split(M, N * K)
        if S > 1:
            Kc = M // S

            def wgrad():
                torch.bmm(dy[:S * Kc].view(S, Kc, -1).transpose(1, 2), x[:S * Kc].view(S, Kc, -1))
        else:
            def wgrad():
                gw.addmm_(dy.t(), x)
        for pn, fn in (("fwd", lambda: x @ w.t()), ("dgrad", lambda: dy @ w), (f"wgrad/S{S}", wgrad)):
            ms = _t(fn)
            tf = 2 * M * N * K / ms / 1e9
            total += ms * per_step
            rows.append((name, pn, ms * 1000, tf, ms * per_step))
            print(f"{name:8s} {pn:9s} M={M:6d} N={N:6d} K={K:5d}  {ms * 1000:8.1f} us  {tf:6.0f} TF/s  "
                  f"x{per_step:2d} = {ms * per_step:6.2f} ms/step", flush=True)
    print(f"GEMM total {total:.1f} ms per training step", flush=True)
    # token-split sweep of the weight gradients (bmm of S partials + the fixed-order fold)
    from swh_trl_amd._lib import call
    from swh_trl_amd.ops import _dtype_code, _stream
    for name, (N, K) in {"qkv": (Q, H), "o": (H, H), "gate_up": (2 * I, H), "down": (H, I), "lm": (V, H)}.items():
        M = CH if name == "lm" else T
        x = torch.randn(M, K, **bf)
        dy = torch.randn(M, N, **bf)
        gw = torch.zeros(N, K, **bf)
        res = []
        for S in (1, 2, 4, 8):
            if M % S:
                continue
            Kc = M // S
            if S == 1:
                def fn():
                    gw.addmm_(dy.t(), x)
            else:
                def fn():
                    parts = torch.bmm(dy.view(S, Kc, -1).transpose(1, 2), x.view(S, Kc, -1))
                    call("swh_dw_reduce", parts.data_ptr(), S, gw.numel(), gw.data_ptr(), _dtype_code(gw, "dw"),
                         _stream())
            ms = _t(fn)
            res.append(f"S{S} {ms * 1000:7.1f}us {2 * M * N * K / ms / 1e9:5.0f}TF")
        print(f"wgrad split {name:8s} " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
