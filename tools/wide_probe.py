"""Phase timing of wide_gemm (csrc/wide_gemm.hip) from inside the kernel at the
Llama-3-8B decode shapes (64 rows): per workgroup, thread 0 stamps entry (0),
main loop done (1), slab stores drained (2), ticket taken (3), split-K sum done
(4, last arrivers only), exit (5).  Weights cycle over distinct copies larger
than the Infinity Cache, as in the decode step.  Needs the traced build:

    python tools/build_variant.py wtrace --only wide_gemm.hip -DSWH_WIDE_TRACE_ON
    SWH_LIB_PATH=tools/_build/wtrace.so python tools/wide_probe.py [--smax 8] [--cb 0]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()

SHAPES = {  # name: (N, K, silu, epilogue)
    "qkv": (6144, 4096, False, "norm"),
    "o": (4096, 4096, False, "residual"),
    "gate_up": (14336, 4096, True, "norm"),
    "down": (4096, 14336, False, "residual"),
}


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--smax", type=int, default=None)
    ap.add_argument("--cb", type=int, default=None)
    ap.add_argument("--reps", type=int, default=24)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    from swh_trl_amd import _lib, nn_ops
    lib = _lib.load()
    if not hasattr(lib, "swh_wide_probe_set_trace"):
        sys.exit("not a traced build (SWH_LIB_PATH -> tools/_build/wtrace.so)")
    pol = {}
    if args.smax is not None:
        pol["wide_smax"] = args.smax
    if args.cb is not None:
        pol["wide_cb"] = args.cb
    if pol:
        _lib.set_launch_policy(**pol)
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M = 64
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    trace = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
    lib.swh_wide_probe_set_trace.argtypes = [ctypes.c_void_p]
    for name in args.shapes.split(","):
        N, K, silu, epi = SHAPES[name]
        rows = 2 * N if silu else N
        copies = max(2, (600 << 20) // (rows * K * 2) + 1)  # > 256 MiB Infinity Cache
        ws_ = [nn_ops.wide_pack((torch.randn(rows, K, generator=g, device=dev) * 0.02).to(bf), silu=silu)
               for _ in range(copies)]
        x = torch.randn(M, K, generator=g, device=dev).to(bf)
        ss = x.float().view(M, K // 16, 16).pow(2).sum(-1).contiguous() if epi == "norm" else None
        res = torch.randn(M, N, generator=g, device=dev).to(bf) if epi == "residual" else None
        sso = torch.empty(M, N // 16, device=dev) if epi == "residual" else None
        y = None if epi == "residual" else torch.empty(M, N, dtype=bf, device=dev)

        def run(i):
            nn_ops.wide_gemm_packed(x, ws_[i % copies], N, bias=None, residual=res, silu=silu, y=y, workspace=ws,
                                    ss_in=ss, ss_out=sso)

        for i in range(4):
            run(i)
        torch.cuda.synchronize()
        spans, rows_out = [], []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for r in range(args.reps):
            trace.zero_()
            lib.swh_wide_probe_set_trace(ctypes.c_void_p(trace.data_ptr()))
            ev[0].record()
            run(r)
            ev[1].record()
            torch.cuda.synchronize()
            lib.swh_wide_probe_set_trace(ctypes.c_void_p(0))
            spans.append(ev[0].elapsed_time(ev[1]) * 1e3)
            t = trace.view(-1, 8).cpu()
            t = t[t[:, 0] > 0]
            t0 = t[:, 0].min().item()
            rel = lambda c: [(v - t0) * 0.01 for v in t[:, c].tolist() if v > 0]  # 100 MHz -> us
            rows_out.append([rel(c) for c in range(6)] + [t.shape[0]])
        # the last reps (weights cold as in the step) pooled
        pool = [sum((ro[c] for ro in rows_out[4:]), []) for c in range(6)]
        nwg = rows_out[-1][6]
        print(f"== {name} N {N} K {K} silu {int(silu)} {epi}: {nwg} workgroups, event span "
              f"p50 {pct(spans[4:], 0.5):.2f} us")
        labels = ["entry", "loop done", "slab drained", "ticket", "sum done", "exit"]
        for c in range(6):
            v = pool[c]
            if v:
                print(f"   {labels[c]:>13}: p10 {pct(v, 0.1):6.2f}  p50 {pct(v, 0.5):6.2f}  p90 {pct(v, 0.9):6.2f}"
                      f"  max {max(v):6.2f}  (n {len(v)})")
        if pool[1]:
            d = [b - a for a, b in zip(pool[0], pool[1])]
            print(f"   {'loop length':>13}: p10 {pct(d, 0.1):6.2f}  p50 {pct(d, 0.5):6.2f}  p90 {pct(d, 0.9):6.2f}")
        del ws_
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
