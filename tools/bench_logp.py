"""The lm-head log-prob backward at the bench's chunk shape (tuning aid, not part
of the product): d logits of a [4096, 151936] bf16 chunk written in place,
timed with events; prints us and the algorithmic HBM rate (read + write of the
chunk).  A/B builds with SWH_LIB_PATH.

    python tools/bench_logp.py [--rows 4096] [--reps 10]
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
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--V", type=int, default=151936)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from swh_trl_amd import _lib, ops
    _lib.load()
    dev = torch.device("cuda:0")
    R, V = a.rows, a.V
    logits = (torch.randn(R, V, device=dev) * 2).to(torch.bfloat16)
    ids = torch.randint(0, V, (R,), device=dev)
    logp, _, lse = ops.logp_entropy(logits, ids, 1.0, False)
    dlogp = torch.randn(R, device=dev)
    out = torch.empty_like(logits)
    ops.logp_backward(logits, ids, lse, dlogp, out=out)
    ref = out.clone()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        ops.logp_backward(logits, ids, lse, dlogp, out=out)
    e1.record()
    e1.synchronize()
    us = 1000 * e0.elapsed_time(e1) / a.reps
    assert torch.equal(out, ref)
    print(f"lib {os.environ.get('SWH_LIB_PATH', 'main')}: logp_bwd {R} x {V}: {us:.1f} us "
          f"({2 * R * V * 2 / us / 1e3:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
