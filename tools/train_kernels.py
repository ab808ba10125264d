"""The training half of one GRPO step at the bench shape (Qwen2.5-0.5B, 64
sequences x (128 prompt + 256 completion) tokens, 4 GA micro-batches fused):
policy forward, fused lm-head log-prob/entropy, GRPO loss, backward and the
AdamW step, on synthetic completions (no rollout).  For rocprofv3 kernel
statistics and PMC passes over the training kernels (logp fwd/bwd, AdamW,
attention, norms, dW folds) without the ~30k decode launches of a full step.

    python tools/train_kernels.py [--reps 2]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--torch-prof", action="store_true",
                    help="torch.profiler over one step: aten ops by device time, grouped by input shape")
    args = ap.parse_args()
    from swh_trl_amd import profiling
    from swh_trl_amd.engine.config import qwen2_5_0_5b
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer

    cfg = qwen2_5_0_5b()
    if args.layers:
        cfg.num_hidden_layers = args.layers
    B, P, C, G, MB, GA = 64, 128, 256, 8, 16, 4
    g = torch.Generator().manual_seed(1234)
    ds = [{"prompt": None, "prompt_ids": torch.randint(0, cfg.vocab_size, (P,), generator=g).tolist()}
          for _ in range(8)]

    def rew(completion_ids=None, **kw):
        return [float(len(set(c)) % 7) for c in completion_ids]

    gc = GRPOConfig(per_device_train_batch_size=MB, gradient_accumulation_steps=GA, num_generations=G,
                    max_prompt_length=P, max_completion_length=C, learning_rate=1e-6, save_strategy="no",
                    max_steps=10, seed=0, generation_kwargs={"eos_token_id": 151645, "pad_token_id": 151643})
    tr = GRPOTrainer(model=cfg, reward_funcs=rew, args=gc, train_dataset=ds)
    tr.model.options = _env.options()
    dev = tr.device
    prompt = torch.randint(0, cfg.vocab_size, (B // G, P), generator=g).repeat_interleave(G, 0).to(dev)
    comp = torch.randint(0, cfg.vocab_size - 1000, (B, C), generator=g).to(dev)
    adv = torch.randn(B, generator=g).to(dev)
    micro = []
    for j in range(GA):
        sl = slice(j * MB, (j + 1) * MB)
        micro.append({"prompt_ids": prompt[sl], "prompt_mask": torch.ones(MB, P, dtype=torch.int32, device=dev),
                      "completion_ids": comp[sl], "completion_mask": torch.ones(MB, C, dtype=torch.int32, device=dev),
                      "advantages": adv[sl],
                      # generation-order group ids and prompt padding, host copies as the rollout records
                      # them: the shared-prompt forward without a device read-back
                      "_prompt_group": torch.arange(B)[sl] // G, "_prompt_padded": torch.zeros(MB, dtype=torch.bool)})

    def step():
        tr.model.zero_grad()
        tr._loss_backward(micro)
        tr.optimizer.step(tr.model.grad, model_out=tr.model.flat, lr=1e-6)

    step()
    torch.cuda.synchronize()
    if args.torch_prof:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            step()
            torch.cuda.synchronize()
        ka = prof.key_averages(group_by_input_shape=True)
        print(ka.table(sort_by="self_device_time_total", row_limit=70, max_name_column_width=40,
                       max_shapes_column_width=90), flush=True)
        return
    profiling.reset()
    profiling.enable(True)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    profiling.enable(False)
    print(f"[train_kernels] {dt * 1000:.1f} ms per training half-step (fwd + logp + loss + bwd + AdamW)", flush=True)
    for k, v in profiling.summary().items():
        print(f"  {k:22s} {v['avg_us']:10.1f} us  {v['bytes_per_launch'] / (v['avg_us'] * 1e-6) / 1e9:8.1f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
