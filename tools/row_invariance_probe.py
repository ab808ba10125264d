"""Diagnostics: is the scoring / training forward independent of a row's
position in the batch?  (with ref == policy the reference's
step-1 KL is exactly 0; the product's frozen-reference pass and training pass
see the rows in other orders.)

Per model width it reports, bit for bit:
  * each library GEMM of the forward: F.linear(X[perm]) vs F.linear(X)[perm];
  * the lm-head log-prob chunk kernel with rows permuted;
  * the whole scoring forward (GRPOTrainer._completion_logps): natural order vs
    shuffled rows, no-grad vs grad + entropy (the training pass), trainable
    policy vs the frozen reference copy.

    python tools/row_invariance_probe.py [--width qwen|llama|both]
"""
import argparse
import dataclasses
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()
from swh_trl_amd import gemm_tuning, ops  # noqa: E402
from swh_trl_amd.engine import build_model  # noqa: E402
from swh_trl_amd.engine.config import llama3_8b, qwen2_5_0_5b  # noqa: E402
from swh_trl_amd.trainer.grpo_trainer import GRPOTrainer  # noqa: E402


class _Stub:
    temperature = 1.0
    _prompt_groups = staticmethod(GRPOTrainer._prompt_groups)


def score(model, batch, grad, entropy):
    with torch.set_grad_enabled(grad):
        lp, _ = GRPOTrainer._completion_logps(_Stub(), model, batch, entropy)
    return lp.detach()


def rows_differ(a, b):
    return int((a != b).reshape(a.shape[0], -1).any(1).sum())


def gemm_check(tag, M, N, K, dev, bias=False):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    x = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
    b = torch.randn(N, device=dev, generator=g).bfloat16() if bias else None
    perm = torch.randperm(M, device=dev, generator=g)
    y = F.linear(x, w, b)
    yp = F.linear(x[perm], w, b)
    print(f"  gemm {tag:10s} M {M:6d} N {N:6d} K {K:6d}: rows differing {rows_differ(yp, y[perm])} / {M}", flush=True)


def probe(name, cfg, U, G, P, C):
    dev = torch.device("cuda:0")
    print(f"== {name}: U {U} x G {G}, P {P}, C {C}", flush=True)
    R = U * G
    NP = U * P
    T = NP + R * C
    H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    gemm_check("qkv", T, cfg.qkv_dim, H, dev, bias=cfg.attention_bias)
    gemm_check("o", T, H, cfg.q_dim, dev)
    gemm_check("gate/up", T, 2 * I, H, dev)
    gemm_check("down", T, H, I, dev)
    chunk = max(1, min(4096, (1 << 30) // V))
    gemm_check("lm chunk", min(chunk, R * C), V, H, dev)
    # log-prob kernel on a permuted chunk
    g = torch.Generator(device=dev).manual_seed(7)
    lg = torch.randn(min(chunk, R * C), V, device=dev, generator=g).bfloat16()
    ids = torch.randint(0, V, (lg.shape[0],), device=dev, generator=g)
    perm = torch.randperm(lg.shape[0], device=dev, generator=g)
    lp, en, _ = ops.logp_entropy(lg, ids, 1.0, True)
    lp2, en2, _ = ops.logp_entropy(lg[perm], ids[perm], 1.0, True)
    lp3, _, _ = ops.logp_entropy(lg, ids, 1.0, False)
    print(f"  logp kernel: permuted rows differing {int((lp2 != lp[perm]).sum())}, entropy off vs on "
          f"{int((lp3 != lp).sum())}", flush=True)

    model = build_model(cfg, dev, seed=3, trainable=True, options=_env.options())
    ref = build_model(cfg, dev, seed=None, trainable=False, options=_env.options())
    ref.copy_from(model)
    gg = torch.Generator().manual_seed(5)
    pids = torch.randint(2, V, (U, P), generator=gg).repeat_interleave(G, 0).to(dev)
    cids = torch.randint(2, V, (R, C), generator=gg).to(dev)
    batch = {"prompt_ids": pids, "prompt_mask": torch.ones_like(pids, dtype=torch.int32),
             "completion_ids": cids, "prompt_group": torch.arange(U, device=dev).repeat_interleave(G)}
    rp = torch.randperm(R, generator=gg).to(dev)
    shuf = {k: v[rp] for k, v in batch.items()}
    base = score(model, batch, False, False)
    refl = score(ref, batch, False, False)
    print(f"  policy vs frozen ref (same order, no grad): rows differing {rows_differ(refl, base)} / {R}", flush=True)
    s = score(model, shuf, False, False)
    print(f"  policy shuffled vs natural (no grad): rows differing {rows_differ(s, base[rp])} / {R}", flush=True)
    t = score(model, shuf, True, True)
    print(f"  training pass (grad + entropy, shuffled) vs natural: rows differing {rows_differ(t, base[rp])} / {R}",
          flush=True)
    t2 = score(model, batch, True, True)
    print(f"  training pass natural vs scoring natural: rows differing {rows_differ(t2, base)} / {R}", flush=True)
    d = (t - base[rp]).abs()
    print(f"  max |training - scoring| {d.max().item():.3e}, mean {d.mean().item():.3e}", flush=True)
    model.grad = None
    del model, ref
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", choices=("qwen", "llama", "both"), default="both")
    a = ap.parse_args()
    print("gemm tuning:", gemm_tuning.enable(), flush=True)
    if a.width in ("qwen", "both"):
        probe("qwen2.5-0.5b width, 2 layers (test shape)", dataclasses.replace(qwen2_5_0_5b(), num_hidden_layers=2),
              4, 4, 12, 24)
        probe("qwen2.5-0.5b width, 2 layers (bench shape)", dataclasses.replace(qwen2_5_0_5b(), num_hidden_layers=2),
              8, 8, 128, 256)
    if a.width in ("llama", "both"):
        probe("llama-3-8b width, 2 layers (cfg5 test shape)", dataclasses.replace(llama3_8b(), num_hidden_layers=2),
              8, 8, 32, 128)


if __name__ == "__main__":
    main()
