"""Rollout log-probs at the PPO bench shape (tuning aid): Qwen2.5-0.5B width,
64 rows x (128 + 53), T = 0.7 + 1e-7, fused lm-head sampler with log-probs
against the logits -> sample_step path: NaN count, draws, max difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    from swh_trl_amd.engine import CausalLM, DecodeEngine, qwen2_5_0_5b
    from swh_trl_amd.engine.options import EngineOptions
    dev = torch.device("cuda:0")
    cfg = qwen2_5_0_5b()
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    cfg.num_hidden_layers = layers
    m = CausalLM(cfg, dev, seed=0, trainable=False)
    B, P, C = 64, 128, 53
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, cfg.vocab_size, (B, P), generator=g).to(dev)
    mask = torch.ones(B, P, dtype=torch.int32, device=dev)
    outs = {}
    for fused in (True, False):
        e = DecodeEngine(m, B, P, C, options=EngineOptions(fused_sample=fused))
        toks, lp = e.generate(ids, mask, C, temperature=0.7 + 1e-7, seed=3, eos_token_id=151645,
                              pad_token_id=151643, return_logp=True)
        torch.cuda.synchronize()
        outs[fused] = (toks, lp)
        print(f"fused={fused}: fused_sample={e._fused_sample()} nan={int(lp.isnan().sum())} "
              f"inf={int(lp.isinf().sum())} min={float(lp.nan_to_num().min()):.3f}", flush=True)
    (ta, la), (tb, lb) = outs[True], outs[False]
    same = ta == tb
    print(f"tokens equal {bool(same.all())} ({int(same.sum())}/{same.numel()}), max |dlogp| "
          f"{float((la - lb).abs().nan_to_num(1e9).max()):.3g}", flush=True)
    bad = la.isnan().nonzero()[:10].tolist()
    print("first NaN positions", bad, flush=True)


if __name__ == "__main__":
    main()
