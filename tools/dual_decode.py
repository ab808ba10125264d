"""Decode as two concurrent half-batch chains (tuning aid, not
part of the product).

The cfg2 decode step at 64 rows is a chain of ~121 dependent launches per token,
each latency-bound.  This probe builds one 64-row DecodeEngine and
two 32-row engines over the same model (the 8 GRPO groups split 4 + 4), captures
their K-step decode graphs, and times at mid-generation:
  single   the 64-row graph replayed R times
  dual     the two 32-row graphs replayed alternately on two streams (no
           cross-stream edge: each branch forks once per replay pair)
  stagger  as dual, with the second stream's first replay behind a spin of
           ~half a layer (torch.cuda._sleep), so its weight reads trail the first
Per decode step = elapsed / (R * K).

    python tools/dual_decode.py [--reps 24] [--stagger-cycles 20000]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stagger-cycles", type=int, default=20000)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    from swh_trl_amd.engine import CausalLM, DecodeEngine, qwen2_5_0_5b
    dev = torch.device("cuda:0")
    cfg = qwen2_5_0_5b()
    m = CausalLM(cfg, dev, seed=0, trainable=False, options=_env.options())
    P, C, G = 128, 256, 8
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (8, P), generator=g).repeat_interleave(G, 0).to(dev)
    mask = torch.ones(64, P, dtype=torch.int32, device=dev)
    kw = dict(min_new_tokens=C, eos_token_id=151645, pad_token_id=151643, early_exit=False)
    e64 = DecodeEngine(m, 64, P, C)
    ea, eb = DecodeEngine(m, 32, P, C), DecodeEngine(m, 32, P, C)
    e64.generate(ids, mask, C, seed=1, group_size=G, **kw)
    ea.generate(ids[:32], mask[:32], C, seed=1, group_size=G, **kw)
    eb.generate(ids[32:], mask[32:], C, seed=2, group_size=G, **kw)
    torch.cuda.synchronize()
    K = e64.steps_per_graph
    R = min(a.reps, (C - 2) // K)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def reset(*engines):
        for e in engines:
            e.state[0] = 1
            e.finished.zero_()
        torch.cuda.synchronize()

    def time_single():
        reset(e64)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(R):
            e64.graph_k.replay()
        t1.record()
        t1.synchronize()
        return 1000.0 * t0.elapsed_time(t1) / (R * K)

    def time_dual(stagger: int):
        reset(ea, eb)
        cur = torch.cuda.current_stream()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            if stagger:
                torch.cuda._sleep(stagger)
        for _ in range(R):
            with torch.cuda.stream(s1):
                ea.graph_k.replay()
            with torch.cuda.stream(s2):
                eb.graph_k.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)
        t1.record()
        t1.synchronize()
        return 1000.0 * t0.elapsed_time(t1) / (R * K)

    with torch.no_grad():
        for it in range(a.iters):
            single = time_single()
            dual = time_dual(0)
            stag = time_dual(a.stagger_cycles)
            print(f"[dual_decode] iter {it}: per decode step single-64 {single:.1f} us, dual-32x2 {dual:.1f} us, "
                  f"dual staggered ({a.stagger_cycles} cycles) {stag:.1f} us", flush=True)


if __name__ == "__main__":
    main()
