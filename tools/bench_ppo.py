"""PPO update throughput at SURVEY.md §8d cfg3: Qwen2.5-0.5B policy (random
init), a same-size Qwen2ForSequenceClassification value model, a tiny reward
model (hidden 64, 2 layers); 64 queries x 128 tokens per GPU, response_length
53, num_ppo_epochs 4, micro-batch 16 x GA 4, one mini-batch.  Prints one JSON
line (samples/s = rollout rows per second of update).  Not the headline
bench (bench.py is); a measurement of the PPO row.

    python tools/bench_ppo.py [--steps 2] [--warmup 1]
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
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    from swh_trl_amd.engine import DecoderConfig, qwen2_5_0_5b
    from swh_trl_amd.trainer import PPOConfig, PPOTrainer

    cfg = qwen2_5_0_5b()
    rm_cfg = DecoderConfig(vocab_size=cfg.vocab_size, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                           num_attention_heads=1, num_key_value_heads=1, head_dim=64, rope_theta=cfg.rope_theta,
                           max_position_embeddings=cfg.max_position_embeddings)
    B, P = 64, 128
    # 16 batches per data epoch: the timed updates are ordinary ones.  At a data epoch's
    # last batch the reference's accelerate accumulation steps after every micro-batch
    # (PPOTrainer._accumulate_sync), a 4x costlier update at this configuration.
    n = B * max(16, args.steps + args.warmup + 1)
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(2, cfg.vocab_size - 1000, (n, P), generator=g)
    ds = [{"input_ids": ids[i].tolist()} for i in range(n)]
    pc = PPOConfig(per_device_train_batch_size=16, gradient_accumulation_steps=4, num_mini_batches=1,
                   num_ppo_epochs=4, response_length=53, local_rollout_forward_batch_size=64,
                   total_episodes=n, learning_rate=3e-6, stop_token_id=151645, pad_token_id=151643,
                   eos_token_id=151645, seed=0)
    tr = PPOTrainer(pc, None, cfg, None, rm_cfg, ds, cfg)
    tr.policy_model.options = _env.options()
    tr.state.global_step = 0
    from bench import kernel_roofline
    from swh_trl_amd import profiling
    for _ in range(args.warmup):
        tr.training_step()
    torch.cuda.synchronize()
    profiling.reset()
    profiling.enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.training_step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    profiling.enable(False)
    kern = profiling.summary()
    log = tr._flush_logs()
    # the rollout decodes with log-probs (logits + sampler path), the dominant kernel over the update
    roof = kernel_roofline(kern, tr._engine, args.steps, pc.response_length)
    print(json.dumps({"metric": "PPO update samples/sec (rollout + 4 PPO epochs), Qwen2.5-0.5B policy+value",
                      "value": round(B / dt, 3), "unit": "samples/s", "ms_per_step": round(1000 * dt, 1),
                      "dtype": "bf16", "data": "synthetic (uniform query ids seed 1234, random-init weights)",
                      "config": {"workload": "configs[2]: Qwen2.5-0.5B PPOTrainer + value head + tiny reward model",
                                 "queries": B, "query_len": P, "response_length": 53, "num_ppo_epochs": 4,
                                 "micro_batch": 16, "grad_accum": 4},
                      "roofline": roof,
                      "log": {k: log.get(k) for k in ("objective/kl", "loss/policy_avg", "loss/value_avg",
                                                      "val/ratio")}}), flush=True)


if __name__ == "__main__":
    main()
