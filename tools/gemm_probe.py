"""Phase timing of the decode GEMM from inside the kernel (wall clock, 10 ns):
per workgroup, wave 0 stamps entry, loads issued, statistic ready, MFMAs done,
merged, split-K reduced, exit.  Builds tools/_build/libgemm_probe.so if absent.

    python tools/gemm_probe.py [--cfg cb,nw,s]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.environ.get("SWH_PROBE_SO", os.path.join(ROOT, "tools", "_probe", "libgemm_probe.so"))
PHASES = ["p1", "p2", "p3", "p4", "p5", "exit"]


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
    ap.add_argument("--cfg", default=None)
    args = ap.parse_args()
    build()
    lib = ctypes.CDLL(SO)
    if args.cfg:  # the probe library's own launch policy (the library reads no environment)
        sys.path.insert(0, ROOT)
        from swh_trl_amd import _lib as L
        pol = L.LaunchPolicy()
        lib.swh_get_launch_policy(ctypes.byref(pol))
        for k, v in L._geometry_fields(args.cfg).items():
            setattr(pol, k, v)
        assert lib.swh_set_launch_policy(ctypes.byref(pol)) == 0, args.cfg
    vp, i64, i32, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    lib.swh_decode_gemm.argtypes = [vp, vp, i64, i64, i64, vp, f32, vp, vp, i32, vp, i64, vp, vp, vp, i64, vp]
    lib.swh_decode_gemm.restype = i32
    lib.swh_probe_set_trace.argtypes = [vp]
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    M, H, I, V = 64, 896, 4864, 151936
    bf = torch.bfloat16
    s = torch.randn(M, H, generator=g).to(bf).to(dev)
    att = torch.randn(M, H, generator=g).to(bf).to(dev)
    act = torch.randn(M, I, generator=g).to(bf).to(dev)
    ss = s.float().view(M, H // 16, 16).pow(2).sum(-1).contiguous()
    nw = torch.ones(H, dtype=bf, device=dev)
    wq = (torch.randn(1152, H, generator=g) * 0.02).to(bf).to(dev)
    bq = torch.zeros(1152, dtype=bf, device=dev)
    wo = (torch.randn(H, H, generator=g) * 0.02).to(bf).to(dev)
    wgu = (torch.randn(2 * I, H, generator=g) * 0.02).to(bf).to(dev)
    wd = (torch.randn(H, I, generator=g) * 0.02).to(bf).to(dev)
    wl = (torch.randn(V, H, generator=g) * 0.02).to(bf).to(dev)
    qkv = torch.empty(M, 1152, dtype=bf, device=dev)
    y_act = torch.empty(M, I, dtype=bf, device=dev)
    logits = torch.empty(M, V, dtype=bf, device=dev)
    ssout = torch.empty(M, H // 16, dtype=torch.float32, device=dev)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    trace = torch.zeros(1 << 22, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    shapes = {
        "qkv": (s, wq, 1152, H, None, bq, None, 0, qkv, 1152, ss, None),  # folded norm: rstd row scale
        "o": (att, wo, H, H, None, None, s, 0, None, H, None, ssout),
        "gate_up": (s, wgu, I, H, None, None, None, 1, y_act, I, ss, None),
        "down": (act, wd, H, I, None, None, s, 0, None, H, None, ssout),
        "lm": (s, wl, V, H, None, None, None, 0, logits, V, ss, None),
    }
    for name, (x, w, N, K, nrm, b, res, silu, y, ldy, ssin, sso) in shapes.items():
        def call():
            rc = lib.swh_decode_gemm(P(x), P(w), M, N, K, P(nrm), 1e-6, P(b), P(res), silu, P(y), ldy, P(ssin),
                                     P(sso), P(ws), ws.numel(), st)
            assert rc == 0, rc
        lib.swh_probe_set_trace(None)
        for _ in range(3):
            call()
        torch.cuda.synchronize()
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
        if t.shape[0] == 0:
            print(f"{name:8s} (no trace: a kernel without phase stamps)")
            continue
        entry = t[:, 0]
        t0 = int(entry.min())
        span = (int(t[:, 1:7].max()) - t0) / 100.0
        print(f"{name:8s} WGs={t.shape[0]:5d} event={1000 * e0.elapsed_time(e1):7.2f}us span={span:7.2f}us "
              f"entry spread p50={float((entry - t0).float().median()) / 100:6.2f} max={float(entry.max() - t0) / 100:6.2f}")
        prev = entry
        for i, ph in enumerate(PHASES, start=1):
            col = t[:, i]
            ok = col > 0
            if not bool(ok.any()):
                continue
            d = (col[ok] - prev[ok]).float() / 100.0
            print(f"    {ph:8s} dt p50 {float(d.median()):7.2f}  p90 {float(d.quantile(0.9)):7.2f}  max {float(d.max()):7.2f}"
                  f"   (n={int(ok.sum())})")
            prev = torch.where(ok, col, prev)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
