"""Llama-3-8B-architecture decode kernels on ONE MI355X at 64 rows (BASELINE.json
config 5's per-GPU generation batch: 8 prompts x G 8): random-init bf16
weights, one short generation to set up the folded / packed weights and the
decode graph, then DecodeEngine.kernel_timings at a mid-completion step.  One
JSON line; run it with SWH_WIDE_PACK=0 / 1 (or other knobs) for A/B.

    python tools/bench_llama8b_decode.py [--P 256] [--step 512]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=256)
    ap.add_argument("--step", type=int, default=512)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--distinct", action="store_true", help="64 distinct prompts instead of 8 x G 8")
    args = ap.parse_args()
    from swh_trl_amd.engine import CausalLM, DecodeEngine, llama3_8b
    t0 = time.perf_counter()
    cfg = llama3_8b()
    m = CausalLM(cfg, torch.device("cuda:0"), seed=0, init_std=0.02, options=_env.options())
    eng = DecodeEngine(m, args.B, args.P, args.step + 8)
    g = torch.Generator().manual_seed(0)
    G = 1 if args.distinct else 8  # config 5: 8 prompts x G 8 generations per GPU
    ids = torch.randint(0, cfg.vocab_size - 1000, (args.B // G, args.P), generator=g).repeat_interleave(G, 0).cuda()
    mask = torch.ones_like(ids)
    eng.generate(ids, mask, 4, temperature=1.0, seed=1, group_size=G)
    torch.cuda.synchronize()
    print(f"[l8dec] setup {time.perf_counter() - t0:.1f}s, packed {len(eng.packed)} matrices", file=sys.stderr,
          flush=True)
    dec = eng.kernel_timings(args.step)
    out = {"workload": "Llama-3-8B decode kernels, 1 GPU", "B": args.B, "P": args.P, "step": args.step,
           "wide_pack": os.environ.get("SWH_WIDE_PACK", "1"), "packed": len(eng.packed),
           "prompt_groups": int(torch.unique(eng.prow).numel())}
    for k, v in dec.items():
        e = {"avg_us": round(v["avg_us"], 2)}
        if v.get("bytes_per_launch"):
            e["TB_s"] = round(v["bytes_per_launch"] / (v["avg_us"] * 1e-6) / 1e12, 2)
        out[k] = e
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
