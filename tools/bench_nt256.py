"""swh_gemm_nt256 (256 x 256 tiles, eight-phase K loop) against hipBLASLt on the
TunableOp table and against swh_gemm_nt (128 x 128, two stages), at the wide
training shapes of the bench step and at square sizes (tuning aid, not part of
the product).  Random operands; max |diff| of nt256 against the fp32 product.

    python tools/bench_nt256.py [--reps 20] [--rounds 2] [--only names] [--wgrad-only]

Weight gradients: grad += dY^T X as the product's library path runs it (token-split
bmm + swh_dw_reduce, or addmm) against swh_gemm_tn256_partials + fold at several
token splits S (and swh_gemm_tn_partials at S 8 where it applies).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def _t(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return 1000 * e0.elapsed_time(e1) / reps


SHAPES = (("gate_up fwd", 17408, 9728, 896), ("lm fwd", 4096, 151936, 896), ("down dgrad", 17408, 4864, 896),
          ("down fwd", 17408, 896, 4864), ("gate_up dgrad", 17408, 896, 9728), ("sq 4096", 4096, 4096, 4096),
          ("sq 8192", 8192, 8192, 8192))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--only", default=None, help="comma-separated shape names")
    ap.add_argument("--wgrad-only", action="store_true")
    a = ap.parse_args()
    from swh_trl_amd import _lib, gemm_tuning, nn_ops
    _lib.load()
    gemm_tuning.enable()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    g = torch.Generator(device="cuda").manual_seed(0)
    only = set(a.only.split(",")) if a.only else None
    for name, M, N, K in () if a.wgrad_only else SHAPES:
        if only and name not in only:
            continue
        x = (torch.rand(M, K, generator=g, **bf) * 2 - 1)
        w = (torch.rand(N, K, generator=g, **bf) * 2 - 1) * 0.05
        y = nn_ops.gemm_nt256(x, w)
        torch.cuda.synchronize()
        ref = x.float() @ w.float().t()
        err = float((y.float() - ref).abs().max())
        del ref
        fl = 2 * M * N * K
        legs = [("hipBLASLt", lambda: torch.nn.functional.linear(x, w)), ("nt256", lambda: nn_ops.gemm_nt256(x, w, out=y))]
        if nn_ops.gemm_nt_eligible(x, w):
            legs.append(("gemm_nt", lambda: nn_ops.gemm_nt(x, w, out=y)))
        for r in range(a.rounds):
            res = [f"{name:14s} M {M} N {N} K {K} r{r}:"]
            for leg, fn in legs:
                us = _t(fn, a.reps)
                res.append(f"{leg} {us:8.1f} us ({fl / us / 1e6:5.0f} TF/s)")
            print("  ".join(res) + f"  max|d| {err:.2e}", flush=True)
        del x, w, y
        torch.cuda.empty_cache()
    from swh_trl_amd._lib import call
    from swh_trl_amd.engine.model import _dw_split
    from swh_trl_amd.ops import _dtype_code, _stream
    for name, M, N, K, splits in (("gate_up wgrad", 17408, 9728, 896, (1, 2, 3, 4, 5, 6)),
                                  ("down wgrad", 17408, 896, 4864, (2, 4, 6, 8, 10)),
                                  ("lm wgrad", 4096, 151936, 896, (1, 2)),
                                  ("qkv wgrad", 17408, 1152, 896, (4, 8, 16))):
        if only and name not in only:
            continue
        dy = (torch.rand(M, N, generator=g, **bf) * 2 - 1) * 0.05
        x = torch.rand(M, K, generator=g, **bf) * 2 - 1
        gw = torch.zeros(N, K, **bf)
        S = _dw_split(M, N * K)
        Kc = M // S

        def lib():
            if S > 1:
                parts = torch.bmm(dy[:S * Kc].view(S, Kc, -1).transpose(1, 2), x[:S * Kc].view(S, Kc, -1))
                call("swh_dw_reduce", parts.data_ptr(), S, gw.numel(), gw.data_ptr(), _dtype_code(gw, "dw"), _stream())
            else:
                gw.addmm_(dy.t(), x)
        fl = 2 * M * N * K
        g3 = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        nn_ops.gemm_tn256_accumulate(g3, dy, x, splits[-1])
        ref = dy.float().t() @ x.float()
        rel = float((g3 - ref).norm() / ref.norm())
        del g3, ref
        for r in range(a.rounds):
            res = [f"{name:14s} M {M} N {N} K {K} r{r}:"]
            us = _t(lib, a.reps)
            res.append(f"library S{S} {us:8.1f} us ({fl / us / 1e6:5.0f})")
            for S2 in splits:
                g2 = torch.zeros(N, K, **bf)
                us = _t(lambda: nn_ops.gemm_tn256_accumulate(g2, dy, x, S2), a.reps)
                res.append(f"tn256 S{S2} {us:8.1f} ({fl / us / 1e6:5.0f})")
            if nn_ops.gemm_tn_eligible(dy, x):
                g2 = torch.zeros(N, K, **bf)
                us = _t(lambda: nn_ops.gemm_tn_accumulate(g2, dy, x, 8), a.reps)
                res.append(f"tn S8 {us:8.1f} ({fl / us / 1e6:5.0f})")
            print("  ".join(res) + f"  rel {rel:.2e}", flush=True)
        del dy, x, gw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
