"""GRPO step samples/sec (rollout + update), Qwen2.5-0.5B, 1..8 x MI355X.

Workload (BASELINE.json configs[1]): Qwen2.5-0.5B
architecture, random-init bf16 weights (no network for checkpoints), G = 8
generations x 8 prompts per GPU = 64 sequences, P = 128 synthetic prompt
tokens (uniform ids, seed 1234, no padding), C = 256 completion tokens
forced to full length (min_new_tokens = C), micro-batch 16 x GA 4, beta = 0,
T = 1, top_p = 1, deterministic dummy reward len(set(ids)) % 7.

A step = one full optimizer step of the GRPO loop: generation of 64 x 256
tokens, completion mask, rewards, group advantages, policy forward + fused
log-prob/entropy + fused loss + backward, (N>1: RCCL gradient all-reduce),
grad-norm clip and AdamW.  Weak scaling: per-GPU work is fixed as N grows.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` without torchrun's environment: this process never touches the
GPU; it starts `torch.distributed.run` with N ranks (one per GPU, RCCL) as a
child and exits with its status.  Under torchrun, N must equal WORLD_SIZE.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GRPO step samples/sec (rollout+update), Qwen2.5-0.5B at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
MFMA_BF16_PEAK_TF = 2500.0  # dense bf16

G, PROMPTS_PER_GPU, P, C, MB, GA = 8, 8, 128, 256, 16, 4
EOS, PAD = 151645, 151643


def dummy_reward(prompts=None, completions=None, completion_ids=None, **kw):
    return [float(len(set(ids)) % 7) for ids in completion_ids]


def make_dataset(n: int, V: int):
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, V, (n, P), generator=g)
    ids[ids == EOS] = 0
    return [{"prompt": None, "prompt_ids": ids[i].tolist()} for i in range(n)]


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def usable_cores() -> tuple:
    """the cores this process may run on — its affinity set —
    bounded by the cgroup CPU quota when one is set (threads beyond the quota
    only time-slice).  Returns (count, how it was determined)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    if quota is not None and quota < aff:
        return quota, f"cgroup cpu.max quota {quota} of {aff} CPUs in the affinity set"
    return aff, f"sched_getaffinity: {aff} CPUs"


def cpu_baseline(steps_note: str) -> dict:
    """The oracle's CPU restatement of the reference GRPO step (SURVEY.md §8d:
    reduced cfg2 = 1 prompt x G=8, P=128, C=256 at full length), timed on the
    host cores and reported per sample; nothing is extrapolated."""
    from oracle import grpo_step as og
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    threads, why = usable_cores()
    torch.set_num_threads(threads)
    cfg = qwen2_5_0_5b().to_dict()
    model = og.hf_qwen2_from_config(cfg, seed=0, dtype=torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-6)
    g = torch.Generator().manual_seed(1234)
    prompt = torch.randint(0, cfg["vocab_size"], (1, P), generator=g).repeat(G, 1)
    pm = torch.ones_like(prompt)

    def reward(cids, cmask):
        return [len(set(r[m.bool()].tolist())) % 7 for r, m in zip(cids, cmask)]

    kw = dict(num_generations=G, per_device_train_batch_size=G, gradient_accumulation_steps=1, eos_token_id=EOS,
              pad_token_id=PAD)
    og.grpo_step(model, opt, prompt[:, :16], pm[:, :16], reward, C=4, min_new_tokens=4, **kw)  # warm-up
    tm = {}
    t0 = time.perf_counter()
    og.grpo_step(model, opt, prompt, pm, reward, C=C, min_new_tokens=C, timings=tm, **kw)
    wall = time.perf_counter() - t0
    return {"value": G / wall, "unit": "samples/s", "cores": threads, "cores_source": why, "kind": "port",
            "cpu": _cpu_model(),
            "cfg1": cpu_cfg1(threads),
            "sample": (f"oracle/grpo_step.py (CPU restatement, transformers Qwen2 bf16, torch {torch.__version__}) on "
                       f"1 prompt x G={G}, P={P}, C={C} (full length): generate {tm['generate_s']:.2f}s + update "
                       f"{tm['update_s']:.2f}s = {wall:.2f}s wall for {G} samples, {threads} threads; {steps_note}")}


def cpu_cfg1(threads: int, steps: int = 2) -> dict:
    """BASELINE.json config 1 on the host (tiny random GPT-2, 4
    prompts x G=2 x 16 tokens, P=8, fp32, 2 optimizer steps) through the same
    oracle step; tools/bench_cfg1.py runs the product on the GPU beside it."""
    from oracle import grpo_step as og
    from swh_trl_amd.engine.gpt2 import gpt2_config
    torch.set_num_threads(threads)
    cfg = gpt2_config().to_dict()
    model = og.hf_gpt2_from_config(cfg, seed=0)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-6)
    g = torch.Generator().manual_seed(1234)
    prompt = torch.randint(2, cfg["vocab_size"], (4, 8), generator=g).repeat_interleave(2, 0)

    def reward(cids, cmask):
        return [len(set(r[m.bool()].tolist())) % 7 for r, m in zip(cids, cmask)]

    kw = dict(num_generations=2, per_device_train_batch_size=8, gradient_accumulation_steps=1, eos_token_id=EOS,
              pad_token_id=PAD, C=16, min_new_tokens=16)
    og.grpo_step(model, opt, prompt, torch.ones_like(prompt), reward, **kw)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        og.grpo_step(model, opt, prompt, torch.ones_like(prompt), reward, **kw)
    wall = time.perf_counter() - t0
    return {"value": 8 * steps / wall, "unit": "samples/s", "cores": threads,
            "sample": f"configs[0]: GPT-2 (vocab 1024, n_embd 32, 2 layers) 4 prompts x G=2 x 16 tok, P=8, fp32, "
                      f"{steps} steps in {wall:.3f}s"}


# PMC passes of the shipped build (tools/gpu_pmc.sh + tools/pmc_summary.py); SWH_PMC_FILE overrides
PMC_FILE = os.environ.get("SWH_PMC_FILE", os.path.join(ROOT, "profiles", "r6_final_pmc_decode.json"))


def pmc_traffic(kernel: str):
    """Per-launch memory-side traffic of `kernel` from the committed PMC passes
    (tools/pmc_summary.py: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE over
    tools/bench_decode.py, MI355X_MICROARCH.md §HBM corrections; each kernel its
    own instantiation, o and down included), or None."""
    try:
        with open(PMC_FILE) as f:
            k = json.load(f)["kernels"].get(kernel)
        return None if k is None else k["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def kernel_roofline(kern: dict, eng, steps: int, C: int) -> dict:
    """The `roofline` object of the bench line.  Eager kernels
    (log-prob, loss, AdamW ...) are timed by HIP events around each launch
    inside the timed region (`kern`, swh_trl_amd.profiling).  The decode
    kernels run inside the captured decode-step graph, where per-launch events
    do not exist, so each one is timed right after the timed region: the same
    kernel on the same buffers, replayed from a graph between HIP events on its
    stream (DecodeEngine.kernel_timings, mid-completion step C/2).  Dominant =
    the largest device time per step; achieved = algorithmic bytes per launch /
    its average duration; traffic = the committed PMC bytes per launch."""
    kinfo = {k: {"avg_us": v["avg_us"], "bytes_per_launch": v["bytes_per_launch"],
                 "per_step": v["launches"] / steps} for k, v in kern.items()}
    if eng is not None and getattr(eng, "fused", False):
        for k, v in eng.kernel_timings(C // 2).items():
            if k != "decode_step":
                kinfo[k] = {"avg_us": v["avg_us"], "bytes_per_launch": v["bytes_per_launch"],
                            "per_step": v["launches_per_step"] * C}
    dom_name, dom = max(kinfo.items(), key=lambda kv: kv[1]["avg_us"] * kv[1]["per_step"])
    achieved = dom["bytes_per_launch"] / (dom["avg_us"] * 1e-6) / 1e9
    return {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "avg_us": round(dom["avg_us"], 2), "bytes_per_launch": dom["bytes_per_launch"],
            "traffic": pmc_traffic(dom_name), "traffic_unit": "HBM bytes per launch (rocprofv3 PMC)",
            "traffic_source": os.path.relpath(PMC_FILE, ROOT),
            "all_kernels": {k: {"avg_us": round(v["avg_us"], 2), "launches_per_step": v["per_step"],
                                "ms_per_step": round(v["avg_us"] * v["per_step"] / 1000.0, 2),
                                "GB/s": round(v["bytes_per_launch"] / (v["avg_us"] * 1e-6) / 1e9, 1)}
                            for k, v in kinfo.items()}}


def _launch_ranks(n: int, argv: list) -> int:
    """Start N ranks under torch.distributed.run (127.0.0.1 rendezvous) as a
    child process; this parent has not initialised the GPU and never does."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--layers", type=int, default=None, help="debug only: shrink the model (invalid for reporting)")
    ap.add_argument("--variant", choices=("default", "top_p", "greedy"), default="default",
                    help="SURVEY.md §8d cfg2 sampling variants: top_p 0.9, or greedy decoding")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus, sys.argv[1:]))

    from swh_trl_amd import dist as sd
    from swh_trl_amd import profiling
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import _env  # A/B switches from the environment (SWH_TRACE, SWH_LIB_PATH, policy, EngineOptions fields)
    _env.apply()

    rank, world, local = sd.init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    ranks_seen = sd.world_info()[1]
    cfg = qwen2_5_0_5b()
    if args.layers:
        cfg.num_hidden_layers = args.layers
    steps, warm = args.steps, args.warmup
    n_prompts = PROMPTS_PER_GPU * world * (steps + warm + 1)
    ds = make_dataset(n_prompts, cfg.vocab_size)
    gen_kw = {"min_new_tokens": C, "eos_token_id": EOS, "pad_token_id": PAD}
    if args.variant == "greedy":
        gen_kw["do_sample"] = False
    gc = GRPOConfig(output_dir="/tmp/grpo-bench", per_device_train_batch_size=MB, gradient_accumulation_steps=GA,
                    num_generations=G, max_prompt_length=P, max_completion_length=C, learning_rate=1e-6,
                    beta=0.0, temperature=1.0, top_p=0.9 if args.variant == "top_p" else 1.0,
                    max_steps=steps + warm, logging_steps=10 ** 9, seed=0, shuffle_dataset=True,
                    generation_kwargs=gen_kw)
    tr = GRPOTrainer(model=cfg, reward_funcs=dummy_reward, args=gc, train_dataset=ds)
    tr.model.options = _env.options()  # the defaults unless an A/B switch is set
    tr.state.max_steps = steps + warm
    tb = time.perf_counter()
    for i in range(warm):
        tr.training_step_group()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup step {i + 1}/{warm} done at {time.perf_counter() - tb:.1f}s", file=sys.stderr,
                  flush=True)
    sd.barrier()
    torch.cuda.synchronize()
    profiling.reset()
    profiling.enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.training_step_group()
    torch.cuda.synchronize()
    sd.barrier()
    elapsed = time.perf_counter() - t0
    profiling.enable(False)
    elapsed = sd.all_max(elapsed)
    kern = profiling.summary()
    log = tr._flush_logs()
    samples = world * PROMPTS_PER_GPU * G * steps
    value = samples / elapsed
    ms = 1000.0 * elapsed / steps

    roof = kernel_roofline(kern, getattr(tr, "_engine", None), steps, C)
    # step-level roofline: t_roof = HBM bytes / 8 TB/s + FLOPs / 2.5 PF
    t_roof_ms = 70.5
    line = {"metric": METRIC, "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": steps,
            "warmup": warm, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
            "ranks_seen": ranks_seen, "backend": sd.backend_name(),
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (uniform prompt ids seed 1234, random-init weights, dummy reward)",
            "config": {"workload": "configs[1]: Qwen2.5-0.5B GRPO bf16, group_size=8, 256-tok completions" +
                       ("" if args.variant == "default" else f" ({args.variant} sampling variant)"),
                       "model": "Qwen2.5-0.5B (random init)", "global_batch": world * PROMPTS_PER_GPU * G,
                       "prompts_per_gpu": PROMPTS_PER_GPU, "num_generations": G, "prompt_len": P,
                       "completion_len": C, "seq_len": P + C, "micro_batch": MB, "grad_accum": GA, "beta": 0.0,
                       "parallelism": f"dp{world}", "layers": cfg.num_hidden_layers},
            "roofline": roof,
            "step_roofline": {"t_roof_ms_per_gpu": t_roof_ms, "frac": round(t_roof_ms / ms, 4)},
            "train_log": {k: log.get(k) for k in ("loss", "grad_norm", "reward", "entropy")}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.layers:
        try:
            line["cpu_baseline"] = cpu_baseline(f"GPU run: {steps} timed steps")
        except Exception as e:  # report, never hide
            line["cpu_baseline"] = {"value": None, "error": repr(e)[:300]}
    if rank == 0:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
