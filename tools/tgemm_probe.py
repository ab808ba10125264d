"""A few launches of the training GEMM kernels at the bench shapes, for
rocprofv3 PMC passes (tuning aid, not part of the product): swh_gemm_nt at
the gate/up forward shape and swh_gemm_tn at the qkv weight gradient (S = 8).

    rocprofv3 --pmc <counters> -- python3 tools/tgemm_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    M = 17408
    x = torch.randn(M, 896, **bf)
    w = torch.randn(9728, 896, **bf) * 0.03
    dy = torch.randn(M, 1152, **bf) * 0.01
    gw = torch.zeros(1152, 896, device="cuda")
    for _ in range(3):
        nn_ops.gemm_nt(x, w)
        nn_ops.gemm_tn_accumulate(gw, dy, x, 8)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
