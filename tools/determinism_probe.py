"""Diagnostics: is a GRPO step bit-reproducible?  Runs the same 3-step tiny
training twice (fresh trainers) and a resume from checkpoint-1, and reports
where the final fp32 master weights differ (per named parameter)."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()
from swh_trl_amd.engine import CausalLM, tiny_qwen2  # noqa: E402
from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer  # noqa: E402
from swh_trl_amd.trainer import checkpoint as ck  # noqa: E402

cfg = tiny_qwen2(512, 2)
dev = torch.device("cuda:0")
ds = [{"prompt": None, "prompt_ids": list(range(3 + i, 11 + i))} for i in range(16)]


def rew(completion_ids=None, **kw):
    return [float(len(set(c)) % 5) for c in completion_ids]


def run(out, steps, save, resume=None):
    args = GRPOConfig(output_dir=out, per_device_train_batch_size=8, gradient_accumulation_steps=2, num_generations=4,
                      max_prompt_length=8, max_completion_length=16, max_steps=steps, learning_rate=1e-3,
                      save_steps=1 if save else 10 ** 9, logging_steps=1, seed=3, weight_decay=0.01,
                      generation_kwargs={"eos_token_id": 1, "pad_token_id": 0})
    tr = GRPOTrainer(model=CausalLM(cfg, dev, seed=4, init_std=0.05, options=_env.options()), reward_funcs=rew, args=args, train_dataset=ds)
    tr.model.options = _env.options()
    caps = []
    gen = tr._generate_and_score_completions

    def cap(ex):
        o = gen(ex)
        caps.append(o["completion_ids"].clone())
        return o
    tr._generate_and_score_completions = cap
    tr.train(resume_from_checkpoint=resume)
    return tr, caps


def report(tag, a, b):
    if torch.equal(a.optimizer.master, b.optimizer.master):
        print(f"{tag}: master bit-identical")
        return
    va, vb = ck._flat_views(a.model, a.optimizer.master), ck._flat_views(b.model, b.optimizer.master)
    for k in va:
        d = (va[k] - vb[k]).abs()
        if d.max() > 0:
            print(f"{tag}: {k}: {(d > 0).sum().item()} / {d.numel()} differ, max {d.max().item():.3e}")


with tempfile.TemporaryDirectory() as t:
    a, ca = run(os.path.join(t, "a"), 3, True)
    b, cb = run(os.path.join(t, "b"), 3, False)
    print("rollouts equal:", [torch.equal(x, y) for x, y in zip(ca, cb)])
    report("rerun", a, b)
    c, cc = run(os.path.join(t, "c"), 3, False, resume=os.path.join(t, "a", "checkpoint-1"))
    print("resumed rollouts equal to steps 2-3:", [torch.equal(x, y) for x, y in zip(ca[1:], cc)])
    report("resume", a, c)
