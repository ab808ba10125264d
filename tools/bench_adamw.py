"""FlatAdamW at the Qwen2.5-0.5B width (tuning aid, not part of the product):
one clipped update over a 494M-element flat buffer with bf16 gradients and the
bf16 model copy refreshed, timed with events; prints the grad-norm and update
times and the update's algorithmic HBM rate (28 B per element).

    SWH_LIB_PATH=tools/_build/x.so python tools/bench_adamw.py [--numel N] [--reps 20]
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
    ap.add_argument("--numel", type=int, default=494_032_768)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--weight-decay", type=float, default=0.01)
    ap.add_argument("--no-clip", action="store_true")
    ap.add_argument("--pairs", action="store_true", help="two optimizers alternating (PPO: policy + value)")
    a = ap.parse_args()
    from swh_trl_amd import _lib
    from swh_trl_amd.optim import FlatAdamW
    _lib.load()
    dev = torch.device("cuda:0")
    n = a.numel
    opt = FlatAdamW(n, dev, lr=1e-6, weight_decay=a.weight_decay, max_grad_norm=None if a.no_clip else 1.0,
                    no_decay_ranges=[(0, 4096)])
    grad = (torch.randn(n, device=dev) * 1e-3).to(torch.bfloat16)
    model = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        opt.step(grad, model)
    torch.cuda.synchronize()
    if a.pairs:  # PPO's two flat buffers stepped back to back, each timed on its own
        opt2 = FlatAdamW(n, dev, lr=1e-6, weight_decay=a.weight_decay, max_grad_norm=None if a.no_clip else 1.0,
                         no_decay_ranges=[(0, 4096)])
        grad2 = grad.clone()
        model2 = torch.empty_like(model)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t1 = t2 = 0.0
        for _ in range(a.reps):
            ev[0].record()
            opt.step(grad, model)
            ev[1].record()
            opt2.step(grad2, model2)
            ev[2].record()
            ev[2].synchronize()
            t1 += ev[0].elapsed_time(ev[1])
            t2 += ev[1].elapsed_time(ev[2])
        t1, t2 = 1000 * t1 / a.reps, 1000 * t2 / a.reps
        print(f"pairs: step incl. grad-norm: first {t1:.1f} us, second {t2:.1f} us "
              f"({28 * n / t1 / 1e3:.0f} / {28 * n / t2 / 1e3:.0f} GB/s incl. the norm pass)", flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tn = tu = 0.0
    for _ in range(a.reps):
        ev[0].record()
        opt.grad_norm(grad)
        ev[1].record()
        opt.step(grad, model)
        ev[2].record()
        ev[2].synchronize()
        tn += ev[0].elapsed_time(ev[1])
        tu += ev[1].elapsed_time(ev[2])
    tn, tu = 1000 * tn / a.reps, 1000 * tu / a.reps
    # step() runs its own grad-norm pass first: the update alone is tu - tn
    upd = tu - tn
    print(f"lib {os.environ.get('SWH_LIB_PATH', 'main')}: numel {n} wd {a.weight_decay} clip {not a.no_clip}: "
          f"grad-norm {tn:.1f} us "
          f"({2 * n / tn / 1e3:.0f} GB/s), update {upd:.1f} us ({28 * n / upd / 1e3:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
