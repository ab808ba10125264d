"""swh_gemm_nt256 (256 x 256 tiles, eight-phase K loop) against hipBLASLt on the
TunableOp table and against swh_gemm_nt (128 x 128, two stages), at the wide
training shapes of the bench step and at square sizes (tuning aid, not part of
the product).  Random operands; max |diff| of nt256 against the fp32 product.

    python tools/bench_nt256.py [--reps 20] [--rounds 2]
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
    a = ap.parse_args()
    from swh_trl_amd import _lib, gemm_tuning, nn_ops
    _lib.load()
    gemm_tuning.enable()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    g = torch.Generator(device="cuda").manual_seed(0)
    only = set(a.only.split(",")) if a.only else None
    for name, M, N, K in SHAPES:
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


if __name__ == "__main__":
    main()
