"""Fixed per-kernel costs (tuning aid): graph-replayed trivial kernels, the
latency of the first kernel-argument use and of one global load, and the
back-to-back launch period.  python tools/latency_probe.py"""
import ctypes
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "_build", "liblatency_probe.so")


def main():
    if not os.path.exists(SO):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared",
                               os.path.join(ROOT, "tools", "latency_probe.hip"), "-o", SO])
    lib = ctypes.CDLL(SO)
    lib.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    out = torch.zeros(256 * 4, dtype=torch.int64, device="cuda")
    src = torch.arange(1 << 20, dtype=torch.int32, device="cuda")
    for blocks in (1, 256):
        call = lambda: lib.probe_launch(out.data_ptr(), src.data_ptr(), src.numel(), blocks,  # noqa: E731
                                        torch.cuda.current_stream().cuda_stream)
        call()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(50):
                call()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        t = out.view(-1, 4)[:blocks].cpu().double()
        arg = (t[:, 1] - t[:, 0]).median().item() * 10
        ld = (t[:, 2] - t[:, 1]).median().item() * 10
        print(f"blocks={blocks:4d} graph period {1000 * e0.elapsed_time(e1) / 50:6.2f} us/kernel  "
              f"arg-use {arg:6.0f} ns  dependent load {ld:6.0f} ns  "
              f"HIP_FORCE_DEV_KERNARG={os.environ.get('HIP_FORCE_DEV_KERNARG', '(unset)')}", flush=True)


if __name__ == "__main__":
    main()
