"""A/B of a per-call environment knob of the decode kernels in one process:
kernel_timings (each op cycling the 24 layers) and the whole decode step,
alternating the knob's values, then the generations under each value compared.
Tuning aid, not part of the product.

    python tools/env_ab.py SWH_ATTN_XCD_ROWS 1 0
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    knob, vals = sys.argv[1], sys.argv[2:]
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    from swh_trl_amd.engine.decode import DecodeEngine
    from swh_trl_amd.engine.model import CausalLM

    cfg = qwen2_5_0_5b()
    m = CausalLM(cfg, torch.device("cuda:0"), trainable=False, options=_env.options())
    B, P, C = 64, 128, 256
    eng = DecodeEngine(m, B, P, C)
    g = torch.Generator().manual_seed(0)
    # GRPO-shaped prompts: 8 distinct prompts x 8 rows (one prompt K/V copy per group)
    ids = torch.randint(0, cfg.vocab_size, (B // 8, P), generator=g).repeat_interleave(8, 0).cuda()
    mask = torch.ones(B, P, dtype=torch.int32, device="cuda")
    eng.generate(ids, mask, 8, seed=1, min_new_tokens=8, eos_token_id=151645, pad_token_id=151643, group_size=8)
    torch.cuda.synchronize()
    for rep in range(3):
        for v in vals:
            os.environ[knob] = v
            r = eng.kernel_timings(128)
            print(f"{knob}={v}: " + "  ".join(f"{k.replace('decode_gemm.', '')} {r[k]['avg_us']:.2f}"
                                               for k in r), flush=True)
    outs = []
    for v in vals:
        os.environ[knob] = v
        eng.graph = None
        outs.append(eng.generate(ids, mask, 32, seed=3, temperature=0.8, group_size=8))
    print("identical generations:", all(torch.equal(a, b) for o in outs[1:] for a, b in zip(outs[0], o)
                                        if isinstance(a, torch.Tensor)), flush=True)


if __name__ == "__main__":
    main()
