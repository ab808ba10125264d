"""Bit-identity check between two builds of the library (A/B of a kernel change):
generates with the bench-shaped decode engine (Qwen2.5-0.5B width, random init,
64 rows = 8 prompts x G 8, prompt 128) greedy and sampled, and prints one
sha256 over the completion ids and log-probs.  Run once per build:

    SWH_LIB_PATH=tools/_probe/libbase.so python tools/ab_generate.py
    python tools/ab_generate.py
"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    from swh_trl_amd.engine import CausalLM, DecodeEngine
    from swh_trl_amd.engine.config import DecoderConfig
    layers = int(os.environ.get("AB_LAYERS", "4"))
    dev = torch.device("cuda:0")
    m = CausalLM(DecoderConfig(num_hidden_layers=layers), dev, seed=7, init_std=0.02, options=_env.options())
    B, P, C, G = 64, 128, 96, 8
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, m.cfg.vocab_size, (B // G, P), generator=g).repeat_interleave(G, 0).to(dev)
    mask = torch.ones(B, P, dtype=torch.int32, device=dev)
    eng = DecodeEngine(m, B, P, C)
    h = hashlib.sha256()
    parts = []
    for kw in (dict(greedy=True), dict(seed=3), dict(seed=4, top_p=0.9, return_logp=True), dict(greedy=True)):
        out, lp = eng.generate(ids, mask, C, eos_token_id=2, pad_token_id=0, group_size=G, **kw)
        hp = hashlib.sha256(out.cpu().numpy().tobytes())
        if lp is not None:
            hp.update(lp.cpu().numpy().tobytes())
        parts.append(hp.hexdigest()[:12])
        h.update(hp.digest())
    print("ab_generate", os.environ.get("SWH_LIB_PATH", "default"), h.hexdigest(), "parts", parts)


if __name__ == "__main__":
    main()
