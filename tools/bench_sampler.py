"""sample_step timing per processor configuration at the rollout shape
(64 rows x 151936 bf16 logits, scaled by LOGIT_SCALE).  Tuning aid.

    python tools/bench_sampler.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    from swh_trl_amd import ops
    dev = torch.device("cuda:0")
    B = 64
    V = int(os.environ.get("SAMPLER_V", "151936"))
    scale = float(os.environ.get("LOGIT_SCALE", "1.0"))
    g = torch.Generator(device=dev).manual_seed(0)
    logits = (torch.randn(B, V, device=dev, generator=g) * scale).to(torch.bfloat16)
    rng = torch.tensor([1234, 0], dtype=torch.int64, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    fin = torch.zeros(B, dtype=torch.int32, device=dev)
    out = torch.zeros(B, 8, dtype=torch.int64, device=dev)
    cur = torch.zeros(B, dtype=torch.int64, device=dev)
    ws = torch.empty(ops._lib.load().swh_sample_workspace_bytes(B, V), dtype=torch.uint8, device=dev)
    for name, kw in (("unfiltered", {}), ("T 0.7", dict(temperature=0.7)), ("greedy", dict(greedy=True)),
                     ("min_p 0.05", dict(min_p=0.05)), ("top_k 50", dict(top_k=50)),
                     ("top_p 0.9", dict(top_p=0.9)), ("top_p 0.5", dict(top_p=0.5))):
        p = ops.make_sample_params(**kw)

        def f():
            step.zero_()
            fin.zero_()
            ops.sample_step(logits, p, rng, step, fin, out, cur, None, None, None, ws)
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        e1.synchronize()
        print(f"{name:12s} {1000 * e0.elapsed_time(e1) / 20:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
