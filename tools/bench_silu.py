"""Timing of the SiLU-gate kernels at the bench step's shape (17408 tokens x
I 4864, bf16): forward (read gate/up, write the activation) and backward (read
gate/up and d act, write d gate/up), with their HBM rates.  Tuning aid.

    python tools/bench_silu.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    from swh_trl_amd import nn_ops
    from swh_trl_amd._lib import call, dtype_code
    from swh_trl_amd.ops import _stream
    T, I = 17408, 4864
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
    d = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(T, I, device="cuda", dtype=torch.bfloat16)
    dgu = torch.empty_like(gu)

    def t(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1000

    fw = t(lambda: nn_ops.silu_mul(gu, out=out))
    bw = t(lambda: call("swh_silu_mul_bwd", gu.data_ptr(), d.data_ptr(), T, I, dgu.data_ptr(), dtype_code(gu, "silu_mul_bwd"), _stream()))
    print(f"silu_mul fwd {fw:7.1f} us {3 * T * I * 2 / fw / 1e3:6.0f} GB/s   bwd {bw:7.1f} us "
          f"{5 * T * I * 2 / bw / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
