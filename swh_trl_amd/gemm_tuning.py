"""hipBLASLt solution table for the training-side library GEMMs.

The full-sequence forward/backward (policy scoring, loss backward, prefill)
runs its projections and lm head as plain hipBLASLt GEMMs through torch.  The
default heuristic picks a solution per shape without timing it; PyTorch's
TunableOp times every hipBLASLt / rocBLAS solution for a shape once and
records the winner.  This module ships the winners measured on MI355X for the
engine's shapes (`tuning/gemm_mi355x.csv`) and loads them, so a run never
tunes on the clock.  Same arithmetic, different kernel choice.

    enable(mode="use" (default) | "tune" | "off", path=the shipped table)

`tune` times every solution of every GEMM shape met in the process and writes
the table at exit (tools: `python bench.py` under SWH_GEMM_TUNING=tune, which
bench.py / the tools turn into the call's arguments).
"""
from __future__ import annotations

import os

HERE = os.path.dirname(os.path.abspath(__file__))
TABLE = os.path.join(HERE, "tuning", "gemm_mi355x.csv")
_done = False


def enable(mode: str | None = None, path: str | None = None) -> str:
    """Turn the table on for this process (idempotent).  Returns the mode used:
    'off' also when the table is missing or was written by another
    torch/ROCm/hipBLASLt build (its validators do not match)."""
    global _done
    import torch
    mode = mode or "use"
    path = path or TABLE
    if _done or mode == "off" or not torch.cuda.is_available():
        return "off"
    tun = torch.cuda.tunable
    if mode == "tune":
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(30)
        tun.set_filename(path, False)
        if os.path.exists(path):  # extend an existing table: only new shapes are tuned
            tun.read_file(path)
    elif mode == "use":
        if not os.path.exists(path):
            return "off"
        tun.enable(True)
        tun.tuning_enable(False)
        tun.set_filename(path, False)
        if not tun.read_file(path):
            tun.enable(False)
            return "off"
    else:
        raise ValueError(f"gemm tuning mode {mode!r}: expected use | tune | off")
    _done = True
    return mode
