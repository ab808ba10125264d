"""Data-parallel plumbing: one process per GPU, RCCL (torch "nccl") over xGMI.

The reference gets DDP from accelerate (trl/accelerate_configs/multi_gpu.yaml):
25 MB buckets all-reduced during backward.  Here every gradient is a view
into one flat bf16 buffer, so the exchange is a handful of large contiguous
all-reduces (bucket size chosen for per-link xGMI bandwidth, not NVSwitch):
fewer, larger collectives let RCCL spread each one over all 7 links.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def world_size_from_env() -> int:
    """WORLD_SIZE of the launcher (torchrun / bench.py), 1 without one: the
    process count the configs derive their global batch from, before (or
    without) a process group — accelerate's num_processes."""
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun).
    Returns (rank, world_size, device_index).  No-op for a single process.

    device_index is LOCAL_RANK (one process per GPU).  On gloo with more ranks
    than visible devices (tests rehearsing N ranks on one GPU) ranks share
    devices round-robin; RCCL refuses that, so the nccl backend raises."""
    world = world_size_from_env()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:  # SWH_DIST_BACKEND: tests run gloo ranks that share one GPU
        backend = os.environ.get("SWH_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:
        if backend == "nccl":
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} visible GPU(s): RCCL needs one GPU per rank")
        local = local % ndev
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(minutes=10))
    return rank, world, local


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def backend_name() -> str:
    """The collective backend in use ("nccl" is RCCL on ROCm), or "none"."""
    if dist.is_available() and dist.is_initialized():
        return str(dist.get_backend())
    return "none"


def allreduce_mean_(flat: torch.Tensor, bucket_elems: int = 1 << 27):
    """In-place mean over ranks of a flat buffer, in contiguous buckets
    (default 128M elements = 256 MB of bf16)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size()
    if world == 1:
        return
    backend = dist.get_backend()
    use_avg = backend == "nccl"
    works = []
    n = flat.numel()
    for s in range(0, n, bucket_elems):
        chunk = flat[s:min(n, s + bucket_elems)]
        works.append(dist.all_reduce(chunk, op=dist.ReduceOp.AVG if use_avg else dist.ReduceOp.SUM, async_op=True))
    for w in works:
        w.wait()
    if not use_avg:
        flat.div_(world)


class OverlappedAllReduce:
    """Gradient mean over ranks, launched DURING the backward pass: the caller
    releases contiguous ranges of the flat gradient buffer as they become
    final (the decoder layers in reverse order, from autograd hooks at each
    layer input, engine/model.py `CausalLM.on_layer_grads`), each range is
    all-reduced on a side stream behind an event of the compute stream, and
    `finish()` reduces what is left (embedding / final norm / heads) and makes
    the compute stream wait for every collective.  Replaces the reference's
    DDP bucket hooks (accelerate -> torch DDP, 25 MB buckets): ranges here
    are ~100 MB (a few whole layers), sized for per-link xGMI bandwidth.

    With one process this is a no-op; on gloo (CPU tests) it sums and divides."""

    def __init__(self, flat: torch.Tensor, wait_streams=(), force: bool = False):
        self.flat = flat
        self.wait_streams = list(wait_streams)  # producers of gradients beside the compute stream
        # force: run the collectives even in a one-rank group (tests exercising RCCL on one GPU)
        self.active = dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or force)
        self.world = dist.get_world_size() if self.active else 1
        self.nccl = self.active and dist.get_backend() == "nccl"
        self.stream = torch.cuda.Stream(device=flat.device) if (self.nccl and flat.is_cuda) else None
        self.works = []
        self.done = []  # released [start, end) ranges

    def release(self, start: int, end: int):
        if not self.active or end <= start:
            return
        chunk = self.flat[start:end]
        if self.stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.device))
            self.stream.wait_event(ev)
            for st in self.wait_streams:
                self.stream.wait_stream(st)
            with torch.cuda.stream(self.stream):
                w = dist.all_reduce(chunk, op=dist.ReduceOp.AVG, async_op=True)
        else:
            if chunk.is_cuda:  # gloo on device buffers orders after the current stream only
                for st in self.wait_streams:
                    torch.cuda.current_stream(chunk.device).wait_stream(st)
            w = dist.all_reduce(chunk, op=dist.ReduceOp.AVG if self.nccl else dist.ReduceOp.SUM, async_op=True)
        self.works.append((w, chunk))
        self.done.append((start, end))

    def finish(self):
        """Reduce every range not released yet, then wait for all of them."""
        if not self.active:
            return
        n = self.flat.numel()
        cur = 0
        for s, e in sorted(self.done):
            if s > cur:
                self.release(cur, s)
            cur = max(cur, e)
        if cur < n:
            self.release(cur, n)
        for w, chunk in self.works:
            w.wait()
            if not self.nccl:
                chunk.div_(self.world)
        self.works, self.done = [], []


def all_gather_rows(t: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's [n, ...] tensor along dim 0 in rank order (the
    reference's accelerate `gather(rewards_per_func)`, grpo_trainer.py:1497).
    Equal n on every rank; RCCL gathers in place on the device, gloo through
    host copies.  One process: returns t."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    world = dist.get_world_size()
    tc = t.contiguous()
    if dist.get_backend() == "nccl":
        out = torch.empty((world * tc.shape[0],) + tuple(tc.shape[1:]), dtype=tc.dtype, device=tc.device)
        dist.all_gather_into_tensor(out, tc)
        return out
    host = tc.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host)
    return torch.cat(parts).to(t.device)


def all_gather_objects(items: list) -> list:
    """accelerate gather_object: every rank's list concatenated in rank order."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(items)
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, list(items))
    return [x for part in out for x in part]


def barrier():
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_max(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
