"""A/B of the lm head's fragment-order layout (tile-major vs k-major,
SWH_LM_KMAJOR) in one process: the fused lm-head sampler alone and the whole
decode step, alternating, then the generations compared.  Tuning aid.

    python tools/lm_kmajor_ab.py
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
    ids = torch.randint(0, cfg.vocab_size, (B // 8, P), generator=g).repeat_interleave(8, 0).cuda()
    mask = torch.ones(B, P, dtype=torch.int32, device="cuda")
    eng.generate(ids, mask, 8, seed=1, min_new_tokens=8, eos_token_id=151645, pad_token_id=151643, group_size=8)
    torch.cuda.synchronize()
    for rep in range(3):
        for lm, gu in ((True, False), (False, False), (False, True), (True, True)):
            eng.lm_kmajor, eng.gu_kmajor = lm, gu
            eng.refresh_folded()
            eng.graph = None
            r = eng.kernel_timings(128)
            print(f"kmajor lm {int(lm)} gu {int(gu)}: lm_head_sample {r['lm_head_sample']['avg_us']:6.2f} us  "
                  f"gate_up {r['decode_gemm.gate_up']['avg_us']:6.2f}  decode_step {r['decode_step']['avg_us']:7.1f} us",
                  flush=True)
    outs = []
    for km in (True, False):
        eng.lm_kmajor = eng.gu_kmajor = km
        eng.refresh_folded()
        eng.graph = None
        outs.append(eng.generate(ids, mask, 32, seed=3, temperature=0.8, group_size=8))
    print("identical generations:", all(torch.equal(a, b) for a, b in zip(outs[0], outs[1])
                                        if isinstance(a, torch.Tensor)), flush=True)


if __name__ == "__main__":
    main()
