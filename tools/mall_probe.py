"""How much would the decode projections gain if their weights were resident in
the 256 MiB Infinity Cache?  Times each projection captured n times in a HIP
graph while cycling over the weights of `c` layers: c = 24 (the decode step's
working set, ~1 GB per step, misses the Infinity Cache) against c = 2..6 (a
few layers' weights, resident in the Infinity Cache but larger than the
XCDs' L2 share).  Tuning aid, not part of the product.

    python tools/mall_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    from swh_trl_amd.engine.decode import DecodeEngine, _capture
    from swh_trl_amd.engine.model import CausalLM

    t0 = time.time()
    cfg = qwen2_5_0_5b()
    m = CausalLM(cfg, torch.device("cuda:0"), trainable=False, options=_env.options())
    B, P, C = 64, 128, 256
    eng = DecodeEngine(m, B, P, C)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (B, P), generator=g).cuda()
    mask = torch.ones(B, P, dtype=torch.int32, device="cuda")
    eng.generate(ids, mask, 8, seed=1, min_new_tokens=8, eos_token_id=151645, pad_token_id=151643)
    torch.cuda.synchronize()
    print(f"[mall_probe] setup {time.time() - t0:.1f}s", flush=True)
    p, ss = m.p, eng.ss
    eng.state[0] = 128
    L = cfg.num_hidden_layers
    from swh_trl_amd import nn_ops
    eps = cfg.rms_norm_eps

    def copies(name):
        # distinct copies of layer 0's fragment-order weight, > 400 MB in all: cycling
        # through all of them misses the Infinity Cache as the decode step does
        w = eng.fragw[f"l0.{name}"]
        n = max(24, (400 << 20) // (w.numel() * 2) + 1)
        return [w.clone() for _ in range(n)]

    W = {k: copies(k) for k in ("qkv_w", "o_w", "gu_w", "down_w")}
    af = lambda v: {"act_frag": v} if eng.act_frag else {}
    ops_ = {
        "qkv": lambda i: nn_ops.decode_gemm_fragw(eng.s, W["qkv_w"][i], eps=eps, bias=p.get("l0.qkv_b"), y=eng.qkv,
                                                  ss_in=ss),
        "o": lambda i: nn_ops.decode_gemm_fragw(eng.att, W["o_w"][i], eps=eps, residual=eng.s, ss_out=ss,
                                                **({"act_frag": 2} if eng.att_frag else {})),
        "gate_up": lambda i: nn_ops.decode_gemm_fragw(eng.s, W["gu_w"][i], eps=eps, silu=True, y=eng.act, ss_in=ss,
                                                      **af(1)),
        "down": lambda i: nn_ops.decode_gemm_fragw(eng.act, W["down_w"][i], eps=eps, residual=eng.s, ss_out=ss,
                                                   **af(2)),
    }
    print({k: len(v) for k, v in W.items()}, flush=True)
    steps_only = False
    stream = torch.cuda.current_stream()

    def timed(fn, n, cycle, iters=5):
        fn(0)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with _capture(gr):
            for r in range(n):
                fn(r % cycle)
        gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            gr.replay()
        e1.record(stream)
        e1.synchronize()
        return 1000.0 * e0.elapsed_time(e1) / (n * iters)

    # a 1 GB sweep between the graphs evicts the Infinity Cache
    flush = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    print(f"{'kernel':10s} " + " ".join(f"{'c=' + str(c):>8s}" for c in ("all", 12, 6, 4, 2, 1)), flush=True)
    for name, fn in ([] if steps_only else ops_.items()):
        row = []
        for c in (len(W[{"qkv": "qkv_w", "o": "o_w", "gate_up": "gu_w", "down": "down_w"}[name]]), 12, 6, 4, 2, 1):
            flush.add_(1)
            row.append(timed(fn, 240, c))
        print(f"{name:10s} " + " ".join(f"{v:8.2f}" for v in row), flush=True)

    # the layer chain (qkv, attention, o, gate/up, down) over all 24 layers vs cycling 4 layers
    def layer(i):
        ops_["qkv"](i)
        nn_ops.attn_decode(eng.qkv, eng.kv[i, 0], eng.kv[i, 1], eng.cos, eng.sin, eng.plen, eng.state,
                           cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim, cfg.head_dim ** -0.5,
                           out=eng.att, prompt_row=eng.prow, out_frag=eng.att_frag)
        ops_["o"](i)
        ops_["gate_up"](i)
        ops_["down"](i)

    for c in (() if steps_only else (24, 6, 4, 2)):
        flush.add_(1)
        print(f"layer chain cycling {c:2d} layers: {timed(layer, 48, c):8.2f} us per layer", flush=True)
    del W
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
