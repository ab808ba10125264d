"""Diagnostic: NaN per-token log-probs in DecodeEngine.generate(return_logp=True)
after earlier generations on the same engine."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from swh_trl_amd.engine import CausalLM, DecodeEngine, tiny_llama  # noqa: E402

dev = torch.device("cuda:0")
m = CausalLM(tiny_llama(2048, 2), dev, seed=5, init_std=0.05)
g = torch.Generator().manual_seed(5)
B, P, C = 16, 12, 24
ids = torch.randint(0, m.cfg.vocab_size, (B, P), generator=g).to(dev)
mask = torch.ones(B, P, dtype=torch.int64, device=dev)
mask[3, :4] = 0
for seq in (("logp",), ("greedy", "logp"), ("sampled", "logp"), ("greedy", "sampled", "logp"), ("logp", "logp")):
    eng = DecodeEngine(m, B, P, C)
    for kind in seq:
        if kind == "greedy":
            eng.generate(ids, mask, C, greedy=True)
        elif kind == "sampled":
            eng.generate(ids, mask, C, temperature=0.9, seed=11)
        else:
            out, lp = eng.generate(ids, mask, C, temperature=0.9, seed=12, return_logp=True)
    bad = torch.isnan(lp).nonzero().tolist()
    print(seq, "nan at", bad[:4], "count", len(bad), "rows", sorted({r for r, _ in bad}), flush=True)
    if bad:
        eng.use_graph = False
        out2, lp2 = eng.generate(ids, mask, C, temperature=0.9, seed=12, return_logp=True)
        print("   no-graph rerun nan", int(torch.isnan(lp2).sum()), "same ids", bool(torch.equal(out, out2)), flush=True)
    del eng
