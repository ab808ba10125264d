"""swh_gemm_nt against hipBLASLt (TunableOp table) at the training projection
shapes of the bench step (tuning aid, not part of the product): forward
x W^T (+ bias) and input gradient dy W (= dy (W^T)^T with W^T made contiguous),
random operands, max |diff| against the fp32 product, us per call and TFLOP/s.

    python tools/bench_tgemm.py [--tokens 17408] [--reps 20]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=17408)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--wgrad-only", action="store_true")
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--splits", type=int, nargs="*", default=None)
    a = ap.parse_args()
    from swh_trl_amd import _lib, gemm_tuning, nn_ops
    _lib.load()
    gemm_tuning.enable()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    g = torch.Generator(device="cpu").manual_seed(0)
    M = a.tokens
    for name, N, K, bias in () if a.wgrad_only else (("qkv fwd", 1152, 896, True), ("o fwd", 896, 896, False),
                             ("qkv dgrad", 896, 1152, False), ("o dgrad", 896, 896, False),
                             ("down-shaped", 896, 4864, False), ("gate_up-shaped", 9728, 896, False),
                             ("down dgrad", 4864, 896, False), ("gate_up dgrad", 896, 9728, False)):
        x = torch.randn(M, K, generator=g).to(**bf)
        w = (torch.randn(N, K, generator=g) * 0.03).to(**bf)
        b = (torch.randn(N, generator=g) * 0.1).to(**bf) if bias else None
        ref = x.float() @ w.float().t() + (b.float() if bias else 0)
        y = nn_ops.gemm_nt(x, w, b)
        torch.cuda.synchronize()
        err = float((y.float() - ref).abs().max())
        rel = float((y.float() - ref).norm() / ref.norm())
        tl = _t(lambda: torch.nn.functional.linear(x, w, b), a.reps)
        tm = _t(lambda: nn_ops.gemm_nt(x, w, b, out=y), a.reps)
        fl = 2 * M * N * K
        print(f"{name:15s} M {M} N {N} K {K}: hipBLASLt {tl:7.1f} us ({fl / tl / 1e6:5.0f} TF/s)  "
              f"gemm_nt {tm:7.1f} us ({fl / tm / 1e6:5.0f} TF/s)  max|d| {err:.3e} rel {rel:.2e}", flush=True)
    # weight gradients: the product's current path (token-split bmm + swh_dw_reduce) against gemm_tn
    from swh_trl_amd._lib import call
    from swh_trl_amd.engine.model import _dw_split
    from swh_trl_amd.ops import _dtype_code, _stream
    for name, N, K in () if a.fwd_only else (("qkv wgrad", 1152, 896), ("o wgrad", 896, 896), ("down wgrad", 896, 4864)):
        dy = (torch.randn(M, N, generator=g) * 0.01).to(**bf)
        x = torch.randn(M, K, generator=g).to(**bf)
        gw = torch.zeros(N, K, **bf)
        S = _dw_split(M, N * K)
        Kc = M // S

        def lib():
            if S > 1:
                parts = torch.bmm(dy[:S * Kc].view(S, Kc, -1).transpose(1, 2), x[:S * Kc].view(S, Kc, -1))
                call("swh_dw_reduce", parts.data_ptr(), S, gw.numel(), gw.data_ptr(), _dtype_code(gw, "dw"), _stream())
            else:
                gw.addmm_(dy.t(), x)
        tl = _t(lib, a.reps)
        fl = 2 * M * N * K
        res = [f"{name:15s} M {M} N {N} K {K}: library S{S} {tl:7.1f} us ({fl / tl / 1e6:5.0f} TF/s)"]
        for S2 in (a.splits or (4, 8, 16)):
            g2 = torch.zeros(N, K, device="cuda", dtype=torch.float32)
            tm = _t(lambda: nn_ops.gemm_tn_accumulate(g2, dy, x, S2), a.reps)
            res.append(f"tn S{S2} {tm:7.1f} us ({fl / tm / 1e6:5.0f})")
        g3 = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        nn_ops.gemm_tn_accumulate(g3, dy, x, 8)
        ref = dy.float().t() @ x.float()
        res.append(f"rel {float((g3 - ref).norm() / ref.norm()):.2e}")
        print("  ".join(res), flush=True)


if __name__ == "__main__":
    main()
