"""Time the register-streamed qkv / o projections (fragment-order weights) under
the cost model's geometry and forced ones (the launch policy's geometry override)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()

import torch

from swh_trl_amd import _lib, nn_ops


def main():
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    M, H = 64, 896
    bf = torch.bfloat16
    x = torch.randn(M, H, generator=g).to(bf).to(dev)
    ss = x.float().view(M, H // 16, 16).pow(2).sum(-1).contiguous()
    wq = nn_ops.frag_pack((torch.randn(1152, H, generator=g) * 0.03).to(bf).to(dev))
    bq = torch.zeros(1152, dtype=bf, device=dev)
    wo = nn_ops.frag_pack((torch.randn(H, H, generator=g) * 0.03).to(bf).to(dev))
    yq = torch.empty(M, 1152, dtype=bf, device=dev)
    res = torch.randn(M, H, generator=g).to(bf).to(dev)
    sso = torch.empty(M, H // 16, device=dev)
    shapes = {
        "qkv": lambda: nn_ops.decode_gemm_fragw(x, wq, bias=bq, y=yq, ss_in=ss),
        "o": lambda: nn_ops.decode_gemm_fragw(x, wo, residual=res, ss_out=sso),
    }
    for cfg in (None, "1,1,1", "2,1,1", "4,1,1", "1,2,1", "2,2,1"):
        _lib.set_launch_policy(gemm_cfg=cfg)
        row = []
        for name, fn in shapes.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(50):
                    fn()
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                graph.replay()
            e1.record()
            e1.synchronize()
            row.append(f"{name} {1000 * e0.elapsed_time(e1) / 500:6.2f} us")
        print(f"cfg {str(cfg):8s} " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
