"""Per-kernel timing of one decode step at the bench configuration
(Qwen2.5-0.5B random init, B=64, P=128, C=256) — DecodeEngine.kernel_timings
at the middle of the completion.  Tuning aid, not part of the product.

    python tools/bench_decode.py [--step 128] [--gemm-cfg cb,nw,s]
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


def _time(fn, reps=20, iters=3):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    e1.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / (reps * iters)


def sweep(eng, m):
    from swh_trl_amd import _lib, nn_ops
    c, p = eng.cfg, m.p
    eps, ss = c.rms_norm_eps, eng.ss
    shapes = {
        "qkv": lambda: nn_ops.decode_gemm(eng.s, p["l0.qkv_w"], norm_w=p["l0.ln_in"], eps=eps, bias=p["l0.qkv_b"],
                                          y=eng.qkv, ss_in=ss),
        "o": lambda: nn_ops.decode_gemm(eng.att, p["l0.o_w"], residual=eng.s, ss_out=ss),
        "gate_up": lambda: nn_ops.decode_gemm(eng.s, p["l0.gu_w"], norm_w=p["l0.ln_post"], eps=eps, silu=True,
                                              y=eng.act, ss_in=ss),
        "gate_up_nonorm": lambda: nn_ops.decode_gemm(eng.s, p["l0.gu_w"], silu=True, y=eng.act),
        "gate_up_folded": lambda: nn_ops.decode_gemm(eng.s, eng._normed("l0.gu_w", "l0.ln_post")[0], silu=True,
                                                     y=eng.act, ss_in=ss),
        "down": lambda: nn_ops.decode_gemm(eng.act, p["l0.down_w"], residual=eng.s, ss_out=ss),
        "lm": lambda: nn_ops.decode_gemm(eng.s, m.lm_weight(), norm_w=p["norm"], eps=eps, y=eng.logits_buf,
                                         ss_in=ss),
        "lm_nonorm": lambda: nn_ops.decode_gemm(eng.s, m.lm_weight(), y=eng.logits_buf),
    }
    cfgs = [None, "1,1,1", "2,1,1", "4,1,1", "1,2,1", "2,2,1", "4,2,1", "4,4,1", "2,4,1", "1,1,2", "2,1,2",
            "4,1,4", "4,2,5", "1,1,4", "4,2,1,1", "4,4,1,1", "4,1,2", "2,1,4", "4,1,8", "4,2,4", "4,2,8", "2,2,2",
            "2,2,4", "1,2,2", "4,4,4"]
    print("cfg      " + " ".join(f"{k:>14s}" for k in shapes), flush=True)
    for cf in cfgs:
        _lib.set_launch_policy(gemm_cfg=cf)
        row = []
        for k, fn in shapes.items():
            if k.startswith("lm") and cf not in (None, "4,2,1,1", "4,4,1,1"):
                row.append(float("nan"))
                continue
            try:
                row.append(_time(fn, reps=10 if k.startswith("lm") else 20))
            except Exception as e:  # a geometry the shape does not divide into
                row.append(float("nan"))
        print(f"{str(cf):8s} " + " ".join(f"{v:14.2f}" for v in row), flush=True)
    _lib.set_launch_policy(gemm_cfg=None)


def ku_sweep(eng, m):
    """o / down / qkv under waves per workgroup (launch policy gemm_nw) x geometry."""
    from swh_trl_amd import _lib, nn_ops
    c, p = eng.cfg, m.p
    ss, L = eng.ss, c.num_hidden_layers
    shapes = {
        "o": lambda i: nn_ops.decode_gemm(eng.att, p[f"l{i}.o_w"], residual=eng.s, ss_out=ss),
        "down": lambda i: nn_ops.decode_gemm(eng.act, p[f"l{i}.down_w"], residual=eng.s, ss_out=ss),
        "qkv": lambda i: nn_ops.decode_gemm(eng.s, eng._normed(f"l{i}.qkv_w", f"l{i}.ln_in")[0],
                                            bias=p.get(f"l{i}.qkv_b"), y=eng.qkv, ss_in=ss),
        "gate_up": lambda i: nn_ops.decode_gemm(eng.s, eng._normed(f"l{i}.gu_w", f"l{i}.ln_post")[0], silu=True,
                                                y=eng.act, ss_in=ss),
    }

    def t(fn):
        fn(0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(L):
                fn(i)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        e1.synchronize()
        return 1000.0 * e0.elapsed_time(e1) / (3 * L)

    print("cfg          nw " + " ".join(f"{k:>9s}" for k in shapes), flush=True)
    cfgs = os.environ.get("SWH_SWEEP_CFGS")
    cfgs = [None if c == "None" else c for c in cfgs.split(";")] if cfgs else \
        (None, "1,1,1", "2,1,1", "2,1,2", "4,4,1,0,2", "4,4,1,0,4", "2,4,1,0,4", "2,2,1,0,2", "4,2,1,0,2",
         "1,2,1,0,2", "1,4,1,0,4", "2,2,2,0,2", "4,4,2,0,4", "4,2,1,1,2", "4,4,1,1,4")
    for cf in cfgs:
        for ku in ("",):
            for nw in ("8",):
                _lib.set_launch_policy(gemm_cfg=cf, gemm_nw=int(nw))
                row = []
                for name, fn in shapes.items():
                    try:
                        row.append(t(fn))
                    except Exception:
                        row.append(float("nan"))
                print(f"{str(cf):12s} {nw:>2s} " + " ".join(f"{v:9.2f}" for v in row), flush=True)
    _lib.set_launch_policy(gemm_cfg=None, gemm_nw=0)


def dual(eng, m):
    """Two half-batch chains on two streams of one graph vs one full-batch chain:
    does running independent decode kernels concurrently hide their latency?"""
    from swh_trl_amd import _lib, nn_ops
    c, p = eng.cfg, m.p
    eps, ss, B = c.rms_norm_eps, eng.ss, eng.B
    L, h = c.num_hidden_layers, eng.B // 2

    def gu(i, r0, r1):
        w = eng._normed(f"l{i}.gu_w", f"l{i}.ln_post")[0]
        nn_ops.decode_gemm(eng.s[r0:r1], w, silu=True, y=eng.act[r0:r1], ss_in=ss[r0:r1])

    def dn(i, r0, r1):
        nn_ops.decode_gemm(eng.act[r0:r1], p[f"l{i}.down_w"], residual=eng.s[r0:r1], ss_out=ss[r0:r1])

    def chain(r0, r1):
        for i in range(L):
            gu(i, r0, r1)
            dn(i, r0, r1)

    side = torch.cuda.Stream()

    def both():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        chain(0, h)
        with torch.cuda.stream(side):
            chain(h, B)
        main.wait_stream(side)

    for name, fn in (("full chain  (M=64)", lambda: chain(0, B)), ("half chain  (M=32)", lambda: chain(0, h)),
                     ("two halves (2 streams)", both)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        e1.synchronize()
        print(f"{name:24s} {1000 * e0.elapsed_time(e1) / 5 / L:8.2f} us per layer (gate_up + down)", flush=True)
    # two separately captured half-batch graphs replayed on two streams
    gs = []
    for r0, r1 in ((0, h), (h, B)):
        chain(r0, r1)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            chain(r0, r1)
        gs.append(g)
    s2 = [torch.cuda.Stream(), torch.cuda.Stream()]
    main = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        for g, st in zip(gs, s2):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                g.replay()
        for st in s2:
            main.wait_stream(st)
    e1.record()
    e1.synchronize()
    print(f"{'two graphs 2 streams':24s} {1000 * e0.elapsed_time(e1) / 5 / L:8.2f} us per layer (gate_up + down)",
          flush=True)


def lm_ab(eng, reps=20):
    """The fused lm-head sampler alone: sampling (Philox + Gumbel per element) against
    greedy (argmax only) on the same weights — what the per-element RNG costs."""
    from swh_trl_amd import nn_ops, ops
    c = eng.cfg
    w, nw, fw = eng._lm_head_weight()
    for name, params in (("sample T=0.7", ops.make_sample_params(temperature=0.7)),
                         ("sample T=1", ops.make_sample_params()),
                         ("greedy", ops.make_sample_params(greedy=True))):
        fn = lambda: nn_ops.lm_head_sample(eng.s, w, params, eng.rng, eng.state[0:1], eng.finished, eng.out,  # noqa
                                           eng.cur, norm_w=nw, eps=c.rms_norm_eps, ss_in=eng.ss,
                                           workspace=eng.sample_ws, fragw=fw)
        print(f"lm_head_sample {name:14s} {_time(fn, reps=reps):8.2f} us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--step", type=int, default=128)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--gemm-cfg", default=None)
    ap.add_argument("--sweep", action="store_true", help="time the GEMM shapes under several launch geometries")
    ap.add_argument("--dual", action="store_true", help="two half-batch chains on two streams vs one chain")
    ap.add_argument("--ku", action="store_true", help="weight-round depth x waves x geometry sweep (o, down, qkv)")
    ap.add_argument("--lm", action="store_true", help="lm-head sampler: sampling vs greedy")
    args = ap.parse_args()
    from swh_trl_amd import _lib
    if args.gemm_cfg:
        _lib.set_launch_policy(gemm_cfg=args.gemm_cfg)
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    from swh_trl_amd.engine.decode import DecodeEngine
    from swh_trl_amd.engine.model import CausalLM

    t0 = time.time()
    cfg = qwen2_5_0_5b()
    m = CausalLM(cfg, torch.device("cuda:0"), trainable=False, options=_env.options())
    B, P, C = args.batch, 128, 256
    eng = DecodeEngine(m, B, P, C)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (B, P), generator=g).cuda()
    mask = torch.ones(B, P, dtype=torch.int32, device="cuda")
    eng.generate(ids, mask, 8, seed=1, min_new_tokens=8, eos_token_id=151645, pad_token_id=151643)
    torch.cuda.synchronize()
    print(f"[bench_decode] setup {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    if args.sweep:
        sweep(eng, m)
        return
    if args.dual:
        dual(eng, m)
        return
    if args.ku:
        ku_sweep(eng, m)
        return
    if args.lm:
        lm_ab(eng)
        return
    res = eng.kernel_timings(args.step)
    tot = 0.0
    for k, v in res.items():
        gbs = v["bytes_per_launch"] / (v["avg_us"] * 1e-6) / 1e9 if v["bytes_per_launch"] else float("nan")
        per_step = v["avg_us"] * v["launches_per_step"]
        if k != "decode_step":
            tot += per_step
        print(f"{k:24s} {v['avg_us']:9.2f} us  x{v['launches_per_step']:3d} = {per_step:8.1f} us/step  "
              f"{gbs:8.1f} GB/s")
    print(f"{'sum of kernels':24s} {tot:9.1f} us/step (decode_step graph w/o sampler: "
          f"{res['decode_step']['avg_us']:.1f} us)")
    print(json.dumps({k: round(v["avg_us"], 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
