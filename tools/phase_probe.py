"""Phase-by-phase timing of one training pass (forward, lm head + log-prob,
backward) at a given architecture and shape, with a device sync and a line of
output after each phase, and a Python stack dump every 30 s while a phase runs
(finds which launch a long or stuck phase sits in).

    python tools/phase_probe.py --preset llama-3-8b --layers 2 --B 8 --L 1280
"""
import argparse
import faulthandler
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama-3-8b")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--L", type=int, default=1280)
    ap.add_argument("--P", type=int, default=256)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--part", default="all", help="all | attn (attention fwd+bwd alone) | lmhead (lm head + logp alone)")
    args = ap.parse_args()
    faulthandler.dump_traceback_later(30, repeat=True)
    from swh_trl_amd.engine import CausalLM
    from swh_trl_amd.engine.config import PRESETS
    import dataclasses
    cfg = dataclasses.replace(PRESETS[args.preset](), num_hidden_layers=args.layers)
    dev = torch.device("cuda:0")
    m = CausalLM(cfg, dev, seed=0, options=_env.options())
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (args.B, args.L), generator=g).to(dev)
    P = args.P
    t0 = time.perf_counter()

    def mark(name):
        torch.cuda.synchronize()
        print(f"[probe] {name}: {time.perf_counter() - t0:.3f}s", flush=True)

    if args.part == "attn":
        from swh_trl_amd import nn_ops
        Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        q = torch.randn(args.B, Hq, args.L, D, generator=g).to(torch.bfloat16).to(dev).requires_grad_(True)
        k = torch.randn(args.B, Hkv, args.L, D, generator=g).to(torch.bfloat16).to(dev).requires_grad_(True)
        v = torch.randn(args.B, Hkv, args.L, D, generator=g).to(torch.bfloat16).to(dev).requires_grad_(True)
        o = nn_ops.AttentionFn.apply(q, k, v, D ** -0.5, None, None)
        mark("attention forward")
        o.float().sum().backward()
        mark("attention backward")
        return
    if args.part == "lmhead":
        h = torch.randn(args.B, args.L - P, cfg.hidden_size, generator=g).to(torch.bfloat16).to(dev)
        h.requires_grad_(True)
        lp, ent = m.logp_entropy(h, ids[:, P:], 1.0, True)
        mark("lm head + logp")
        lp.sum().backward()
        mark("lm head backward")
        return
    for r in range(args.reps):
        m.zero_grad()
        mark(f"rep {r} start")
        h = m.hidden_states(ids)
        mark("forward")
        lp, ent = m.logp_entropy(h[:, P - 1:-1], ids[:, P:], 1.0, True)
        mark("lm head + logp")
        lp.sum().backward()
        mark("backward")
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
