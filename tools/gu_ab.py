"""A/B of the decode gate/up kernels in one process (SWH_GU_ROWSPLIT read per
call): the gate/up launch alone (cycling the 24 layers' weights) and the whole
decode step, alternating.  Tuning aid, not part of the product.

    python tools/gu_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    from swh_trl_amd.engine.decode import DecodeEngine
    from swh_trl_amd.engine.model import CausalLM

    cfg = qwen2_5_0_5b()
    m = CausalLM(cfg, torch.device("cuda:0"), trainable=False)
    B, P, C = 64, 128, 256
    eng = DecodeEngine(m, B, P, C)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (B, P), generator=g).cuda()
    mask = torch.ones(B, P, dtype=torch.int32, device="cuda")
    eng.generate(ids, mask, 8, seed=1, min_new_tokens=8, eos_token_id=151645, pad_token_id=151643)
    torch.cuda.synchronize()
    for rep in range(3):
        for flag in ("1", "0"):
            os.environ["SWH_GU_ROWSPLIT"] = flag
            r = eng.kernel_timings(128)
            print(f"rowsplit {flag}: gate_up {r['decode_gemm.gate_up']['avg_us']:6.2f} us  "
                  f"down {r['decode_gemm.down']['avg_us']:6.2f}  decode_step {r['decode_step']['avg_us']:7.1f} us",
                  flush=True)
    # generations agree
    outs = []
    for flag in ("1", "0"):
        os.environ["SWH_GU_ROWSPLIT"] = flag
        eng.graph = None
        outs.append(eng.generate(ids, mask, 32, seed=3, temperature=0.8))
    print("identical generations:", all(torch.equal(a, b) for a, b in zip(outs[0], outs[1])
                                        if isinstance(a, torch.Tensor)), flush=True)


if __name__ == "__main__":
    main()
