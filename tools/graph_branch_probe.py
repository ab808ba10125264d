"""Do the branches of a captured HIP graph run concurrently on this ROCm?
A main chain of 24 short spin kernels, each forking a longer spin kernel onto
a side stream (the shape of the decode step's Infinity Cache warm-up branch),
against the main chain alone.  Run under different DEBUG_HIP_* settings.
Tuning aid, not part of the product.

    python tools/graph_branch_probe.py
"""
import os
import sys

import torch


def timed_graph(body, iters=10):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    e1.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / iters


def main():
    # calibrate the spin: cycles per microsecond
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(1_000_000)
    e1.record()
    e1.synchronize()
    cpu = 1_000_000 / (1000.0 * e0.elapsed_time(e1))
    short, long_ = int(5 * cpu), int(12 * cpu)
    side = torch.cuda.Stream()

    def chain():
        for _ in range(24):
            torch.cuda._sleep(short)

    def chain_branch():
        main = torch.cuda.current_stream()
        for i in range(24):
            if i + 1 < 24:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(long_)
            torch.cuda._sleep(short)
        main.wait_stream(side)

    def two():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        torch.cuda._sleep(long_ * 4)
        with torch.cuda.stream(side):
            torch.cuda._sleep(long_ * 4)
        main.wait_stream(side)

    env = {k: v for k, v in os.environ.items() if k.startswith("DEBUG_HIP") or k.startswith("DEBUG_CLR")}
    print(f"env {env}  cycles/us {cpu:.0f}", flush=True)
    print(f"  chain alone (24 x 5 us)              {timed_graph(chain):8.1f} us", flush=True)
    print(f"  chain + 23 forked 12 us branches      {timed_graph(chain_branch):8.1f} us", flush=True)
    print(f"  two 48 us kernels, two branches        {timed_graph(two):8.1f} us", flush=True)


if __name__ == "__main__":
    sys.exit(main())
