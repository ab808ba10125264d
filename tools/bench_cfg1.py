"""BASELINE.json config 1 (tiny random GPT-2 plumbing: 4 prompts x G=2 x 16
tokens, P=8, fp32, per_device_train_batch_size 8, GA 1) through GRPOTrainer on
the GPU, with the CPU restatement of the same steps beside it (bench.py
cpu_cfg1).  Prints one JSON line.

    python tools/bench_cfg1.py [--steps 10] [--warmup 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import bench
    from swh_trl_amd.engine import gpt2_config
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    n = 4 * (args.steps + args.warmup + 1)
    g = torch.Generator().manual_seed(1234)
    ds = [{"prompt": None, "prompt_ids": torch.randint(2, 1024, (8,), generator=g).tolist()} for _ in range(n)]

    def rew(prompts=None, completions=None, completion_ids=None, **kw):
        return [float(len(set(c)) % 7) for c in completion_ids]

    gc = GRPOConfig(output_dir="/tmp/grpo-cfg1", per_device_train_batch_size=8, gradient_accumulation_steps=1,
                    num_generations=2, max_prompt_length=8, max_completion_length=16, learning_rate=1e-6,
                    max_steps=args.steps + args.warmup, logging_steps=10 ** 9, save_strategy="no",
                    model_init_kwargs={"torch_dtype": "float32"},
                    generation_kwargs={"min_new_tokens": 16, "eos_token_id": 1, "pad_token_id": 0})
    tr = GRPOTrainer(model=gpt2_config(), reward_funcs=rew, args=gc, train_dataset=ds)
    tr.model.options = _env.options()
    tr.state.max_steps = args.steps + args.warmup
    for _ in range(args.warmup):
        tr.training_step_group()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.training_step_group()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    threads = min(16, len(os.sched_getaffinity(0)))
    cpu = bench.cpu_cfg1(threads)
    print(json.dumps({"workload": "configs[0]: tiny GPT-2 GRPO, 4 prompts x G=2 x 16 tok, fp32", "n_gpus": 1,
                      "samples_per_s": round(8 / dt, 2), "ms_per_step": round(1000 * dt, 2), "steps": args.steps,
                      "cpu_baseline": cpu, "cpu": bench._cpu_model()}), flush=True)


if __name__ == "__main__":
    main()
