"""Phase timing of the decode attention (swh_attn_decode_shared) from inside the
kernel: per workgroup, wave 0 stamps entry, K/V loads issued, RoPE + LDS
barrier, main loop done (S = K Q^T, softmax, P V), wave merge barrier, exit
(wall clock, 10 ns).  Uses the instrumented build tools/_probe/libgemm_probe.so
(tools/gemm_probe.py builds it).  The bench shape: 64 rows in 8 GRPO groups
(shared prompt K/V), 2 KV heads x 7 query heads x 64, prompt 128, decode step
`--step`; each timed call follows a 1 GiB write so the caches hold what the
decode graph leaves them (the other 23 layers' weights have passed).

    python tools/attn_probe.py [--step 128] [--reps 5] [--llama]

--llama: the Llama-3-8B shape of config 5 (8 KV heads x 4 query heads x 128, prompt
256, 8 GRPO groups of 8 rows; two workgroups per CU in sequence).
"""
import argparse
import ctypes
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()
SO = os.environ.get("SWH_PROBE_SO", os.path.join(ROOT, "tools", "_probe", "libgemm_probe.so"))
PHASES = ["issued", "rope", "loop", "merge", "exit"]


def build():
    if os.path.exists(SO):
        return
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17",
                           "-munsafe-fp-atomics", os.path.join(ROOT, "tools", "gemm_probe.hip"),
                           os.path.join(ROOT, "swh_trl_amd", "csrc", "wide_gemm.hip"),
                           os.path.join(ROOT, "swh_trl_amd", "csrc", "lib.hip"), "-o", SO])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--step", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--llama", action="store_true")
    args = ap.parse_args()
    build()
    lib = ctypes.CDLL(SO)
    vp, i64, i32, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    lib.swh_attn_decode_shared.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32, f32, vp, vp,
                                           i64, i64, vp]
    lib.swh_attn_decode_shared.restype = i32
    lib.swh_probe_set_trace.argtypes = [vp]
    from swh_trl_amd.engine.config import DecoderConfig
    from swh_trl_amd.engine.model import rope_tables
    dev = torch.device("cuda:0")
    cfg = DecoderConfig()
    B, Hq, Hkv, D, P, C, G = 64, 14, 2, 64, 128, 256, 8
    if args.llama:
        from swh_trl_amd.engine import llama3_8b
        cfg = llama3_8b()
        Hq, Hkv, D, P, C = 32, 8, 128, 256, 1024
    T = P + C
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    kc = torch.randn(B, Hkv, T, D, generator=g, device=dev).to(bf)
    vc = torch.randn(B, Hkv, T, D, generator=g, device=dev).to(bf)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g, device=dev).to(bf)
    out = torch.empty(B, Hq * D, dtype=bf, device=dev)
    cos, sin = rope_tables(cfg, T + 1, dev)
    plen = torch.full((B,), P, dtype=torch.int32, device=dev)
    prow = (torch.arange(B, device=dev, dtype=torch.int32) // G) * G
    state = torch.tensor([args.step + 1, P], dtype=torch.int32, device=dev)
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    trace = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    P_ = lambda t: None if t is None else t.data_ptr()  # noqa: E731

    def call():
        rc = lib.swh_attn_decode_shared(P_(qkv), P_(kc), P_(vc), P_(cos), P_(sin), P_(plen), P_(prow), P_(state), B,
                                        Hq, Hkv, D, T, D ** -0.5, P_(out), None, 0, 0, st)
        assert rc == 0, rc

    lib.swh_probe_set_trace(None)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    for rep in range(args.reps):
        flush.fill_(rep)
        trace.zero_()
        lib.swh_probe_set_trace(ctypes.c_void_p(trace.data_ptr()))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call()
        e1.record()
        torch.cuda.synchronize()
        lib.swh_probe_set_trace(None)
        t = trace.view(-1, 8).cpu()
        t = t[t[:, 0] > 0]
        entry = t[:, 0]
        t0 = int(entry.min())
        span = (int(t[:, 1:6].max()) - t0) / 100.0
        print(f"rep {rep} keys={P + args.step + 1} WGs={t.shape[0]} event={1000 * e0.elapsed_time(e1):6.2f}us "
              f"span={span:6.2f}us entry p50={float((entry - t0).float().median()) / 100:5.2f} "
              f"max={float(entry.max() - t0) / 100:5.2f}")
        for i, ph in enumerate(PHASES, start=1):
            col = (t[:, i] - t0).float() / 100.0
            print(f"    at {ph:7s} p50 {float(col.median()):6.2f}  p90 {float(col.quantile(0.9)):6.2f}  "
                  f"max {float(col.max()):6.2f}")
        prev = entry
        for i, ph in enumerate(PHASES, start=1):
            col = t[:, i]
            d = (col - prev).float() / 100.0
            print(f"    {ph:7s} dt p50 {float(d.median()):6.2f}  p90 {float(d.quantile(0.9)):6.2f}  "
                  f"max {float(d.max()):6.2f}")
            prev = col
        sys.stdout.flush()


if __name__ == "__main__":
    main()
