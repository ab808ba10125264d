"""Llama-3-8B-architecture GRPO on ONE MI355X (BASELINE.json config 5 code paths
at full model size, reduced batch): random-init bf16 weights, frozen reference
copy (beta 0.04 -> ref log-probs + k3 KL), G = 8 generations of P synthetic
prompt tokens per GPU, C forced completion tokens.  Config 5 itself is 8 GPUs
x 8 prompts x C 1024 (the driver's scaling runs cover the 0.5B headline); this
measures the 8B shapes (head_dim 128, GQA 4, K 4096/14336, untied 128256-row
head) through the same engine.  Prints one JSON line.

    python tools/bench_llama8b.py [--prompts 1] [--P 256] [--C 256] [--steps 1] [--warmup 1]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompts", type=int, default=1)
    ap.add_argument("--P", type=int, default=256)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--fuse-budget", type=int, default=1 << 17,
                    help="GA micro-batches run as one pass up to this many tokens (activation memory)")
    args = ap.parse_args()
    from swh_trl_amd.engine import llama3_8b
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer

    G, P, C = 8, args.P, args.C
    cfg = llama3_8b()
    n = args.prompts * (args.steps + args.warmup + 1)
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, cfg.vocab_size - 1000, (n, P), generator=g)
    ds = [{"prompt": None, "prompt_ids": ids[i].tolist()} for i in range(n)]

    def rew(prompts=None, completions=None, completion_ids=None, **kw):
        return [float(len(set(c)) % 7) for c in completion_ids]

    B = args.prompts * G
    mb = min(B, 8)
    gc = GRPOConfig(output_dir="/tmp/grpo-llama", per_device_train_batch_size=mb, gradient_accumulation_steps=B // mb,
                    num_generations=G, max_prompt_length=P, max_completion_length=C, learning_rate=1e-6, beta=0.04,
                    max_steps=args.steps + args.warmup, logging_steps=10 ** 9, seed=0, save_strategy="no",
                    fuse_token_budget=args.fuse_budget,
                    generation_kwargs={"min_new_tokens": C, "eos_token_id": 128001, "pad_token_id": 128002})
    t0 = time.perf_counter()

    def heartbeat():  # long phases (backward of an 8B model) print nothing for minutes
        while True:
            time.sleep(20)
            print(f"[llama8b] alive {time.perf_counter() - t0:.0f}s, "
                  f"{torch.cuda.memory_allocated() / 2**30:.1f} GiB allocated", file=sys.stderr, flush=True)

    import threading
    threading.Thread(target=heartbeat, daemon=True).start()
    tr = GRPOTrainer(model=cfg, reward_funcs=rew, args=gc, train_dataset=ds)
    tr.model.options = _env.options()
    print(f"[llama8b] init {time.perf_counter() - t0:.1f}s, "
          f"{torch.cuda.memory_allocated() / 2**30:.1f} GiB allocated", file=sys.stderr, flush=True)
    tr.state.max_steps = args.steps + args.warmup
    for i in range(args.warmup):
        tr.training_step_group()
        torch.cuda.synchronize()
        print(f"[llama8b] warmup {i + 1} done", file=sys.stderr, flush=True)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        tr.training_step_group()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t1) / args.steps
    eng = tr._engine
    dec = eng.kernel_timings(C // 2) if eng is not None and eng.fused else {}
    log = tr._flush_logs()
    print(json.dumps({"workload": "Llama-3-8B architecture GRPO, 1 GPU", "prompts": args.prompts, "G": G, "P": P,
                      "C": C, "beta": 0.04, "samples_per_s": round(B / dt, 3), "s_per_step": round(dt, 3),
                      "decode_step_us": round(dec.get("decode_step", {}).get("avg_us", float("nan")), 1),
                      "decode_kernels_us": {k: round(v["avg_us"], 2) for k, v in dec.items()},
                      "peak_mem_GiB": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                      "fuse_token_budget": args.fuse_budget,
                      "loss": log.get("loss"), "kl": log.get("kl")}), flush=True)


if __name__ == "__main__":
    main()
