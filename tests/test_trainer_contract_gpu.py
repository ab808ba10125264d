"""The transformers-Trainer half of the drop-in contract (-m gpu): what the
reference's GRPOTrainer inherits by passing `callbacks`, `optimizers`,
`eval_dataset` and the scheduler fields to `Trainer.__init__`
(grpo_trainer.py:837-846) and what PPOTrainer builds itself
(ppo_trainer.py:232-252, :404, :648-685).

* learning-rate schedules: every optimizer step runs at lr * lambda(step) of
  transformers `get_scheduler(lr_scheduler_type, warmup, max_steps)`, the log
  reports the scheduler's last lr, and scheduler.pt restores that scheduler;
* callbacks: transformers TrainerCallback objects (or classes) receive the
  Trainer's events in its order, and the control flags they set (stop, save)
  are obeyed;
* evaluation: `evaluate()` / eval_strategy="steps" generate and score each eval
  batch and report eval_loss = the reference's compute_loss on it (checked
  against the oracle in fp32) plus the eval_-prefixed metrics, without
  disturbing the training stream.
"""
import math
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu
EOS, PAD = 1, 0


def _ds(n=16, P=8, off=3):
    return [{"prompt": None, "prompt_ids": list(range(off + i, off + i + P))} for i in range(n)]


def rew(prompts=None, completions=None, completion_ids=None, **kw):
    return [float(sum(c) % 7) for c in completion_ids]


def _args(**kw):
    from swh_trl_amd.trainer import GRPOConfig
    base = dict(per_device_train_batch_size=8, gradient_accumulation_steps=1, num_generations=4, max_prompt_length=8,
                max_completion_length=12, learning_rate=1e-3, seed=3, save_strategy="no", logging_steps=1,
                generation_kwargs={"eos_token_id": EOS, "pad_token_id": PAD})
    base.update(kw)
    return GRPOConfig(**base)


def _trainer(args, dtype=torch.bfloat16, **kw):
    from swh_trl_amd.engine import CausalLM, tiny_qwen2
    from swh_trl_amd.trainer import GRPOTrainer
    model = CausalLM(tiny_qwen2(512, 2), torch.device("cuda:0"), seed=4, init_std=0.05, dtype=dtype)
    return GRPOTrainer(model=model, reward_funcs=rew, args=args, train_dataset=_ds(), **kw)


@pytest.mark.parametrize("kind,kw", [("cosine", None), ("constant_with_warmup", None),
                                     ("cosine_with_min_lr", {"min_lr_rate": 0.1}), ("linear", None)])
def test_lr_schedule_follows_transformers_get_scheduler(tmp_path, kind, kw):
    from transformers import get_scheduler
    steps, lr = 5, 1e-3
    args = _args(lr_scheduler_type=kind, lr_scheduler_kwargs=kw, warmup_ratio=0.4, max_steps=steps,
                 output_dir=str(tmp_path), save_strategy="steps", save_steps=steps)
    tr = _trainer(args)
    used = []
    step_fn = tr.optimizer.step

    def spy(grad, model_out=None, lr=None):
        used.append(lr)
        return step_fn(grad, model_out=model_out, lr=lr)

    tr.optimizer.step = spy
    tr.train()
    warm = math.ceil(steps * 0.4)
    opt = torch.optim.AdamW([{"params": [torch.nn.Parameter(torch.zeros(1))]} for _ in range(2)], lr=lr)
    ref = get_scheduler(kind, opt, num_warmup_steps=warm, num_training_steps=steps,
                        scheduler_specific_kwargs=dict(kw or {}))
    want = [lr * ref.lr_lambdas[0](s) for s in range(steps)]
    assert used == pytest.approx(want, rel=1e-12, abs=1e-15), (used, want)
    logged = [h["learning_rate"] for h in tr.state.log_history if "learning_rate" in h]
    assert logged == pytest.approx([lr * ref.lr_lambdas[0](s) for s in range(1, steps + 1)], rel=1e-12, abs=1e-15)
    ref.load_state_dict(torch.load(tmp_path / f"checkpoint-{steps}" / "scheduler.pt", weights_only=True))
    assert ref.last_epoch == steps
    assert ref.get_last_lr() == pytest.approx([lr * ref.lr_lambdas[0](steps)] * 2)


def test_callbacks_receive_trainer_events_and_control_the_loop(tmp_path):
    from transformers import TrainerCallback, TrainerControl, TrainerState

    events = []

    class Recorder(TrainerCallback):
        def __getattribute__(self, name):
            if name.startswith("on_"):
                def fn(args, state, control, **kw):
                    assert isinstance(state, TrainerState) and isinstance(control, TrainerControl)
                    events.append((name, state.global_step, dict(kw.get("logs") or {})))
                    return getattr(TrainerCallback, name)(self, args, state, control, **kw)
                return fn
            return object.__getattribute__(self, name)

    class StopAtTwo(TrainerCallback):
        def on_step_end(self, args, state, control, **kw):
            if state.global_step == 2:
                control.should_save = True          # save although save_strategy="no"
                control.should_training_stop = True  # stop before max_steps

    tr = _trainer(_args(max_steps=5, output_dir=str(tmp_path)), callbacks=[Recorder(), StopAtTwo])
    assert [e[0] for e in events] == ["on_init_end"]
    out = tr.train()
    assert out.global_step == 2 and tr.state.global_step == 2
    names = [e[0] for e in events]
    assert names[:4] == ["on_init_end", "on_train_begin", "on_epoch_begin", "on_step_begin"]
    assert names[4:7] == ["on_pre_optimizer_step", "on_optimizer_step", "on_step_end"]
    assert names[7] == "on_log" and "loss" in events[7][2] and events[7][1] == 1
    assert names.count("on_step_end") == 2 and names.count("on_save") == 1
    assert names[-1] == "on_train_end" and "train_runtime" in events[-2][2]
    assert (tmp_path / "checkpoint-2" / "trainer_state.json").exists()
    assert not (tmp_path / "checkpoint-1").exists()
    tr.pop_callback(StopAtTwo)
    assert not any(isinstance(c, StopAtTwo) for c in tr.callback_handler.callbacks)


def test_evaluate_loss_matches_oracle_fp32_and_leaves_training_unchanged():
    """evaluate(): RepeatSampler batches of the eval dataset, each generated and
    scored in eval mode (:1440-1443) and its loss the reference's compute_loss
    under no_grad (:2177-2183).  fp32 against the oracle (transformers Qwen2 fp32,
    trl_ref.grpo_loss) on the product's own eval rollouts: per batch loss within
    1e-4, eval_loss their batch-size-weighted mean, eval_entropy the mean of the
    per-batch masked entropies.  A training run with eval_strategy "steps" ends
    with the same weights, bit for bit, as the run without evaluation."""
    from oracle import grpo_step as og
    from oracle import trl_ref
    from swh_trl_amd.engine.config import tiny_qwen2

    args = _args(max_steps=2, per_device_eval_batch_size=8, model_init_kwargs={"torch_dtype": "float32"},
                 loss_type="grpo")
    tr = _trainer(args, dtype=torch.float32, eval_dataset=_ds(6, off=40))
    w0 = {k: v.detach().float().cpu().clone() for k, v in tr.model.hf_state_dict().items()}
    caps, losses = [], []
    gen_fn, loss_fn = tr._generate_and_score_completions, tr._loss_backward

    def gen_cap(examples, mode="train"):
        out = gen_fn(examples, mode=mode)
        if mode == "eval":
            caps.append({k: v.detach().cpu().clone() for k, v in out.items()})
        return out

    def loss_cap(micro, train=True):
        out = loss_fn(micro, train=train)
        if not train:
            losses.append(float(out["loss"]))
        return out

    tr._generate_and_score_completions, tr._loss_backward = gen_cap, loss_cap
    metrics = tr.evaluate()
    assert len(caps) == 3  # 6 prompts x G 4 = 24 samples in batches of 8
    for k in ("eval_loss", "eval_runtime", "eval_reward", "eval_reward_std", "eval_entropy",
              "eval_completions/mean_length", "eval_clip_ratio/region_mean", "eval_rewards/rew/mean"):
        assert k in metrics, k
    hf = og.hf_from_config(tiny_qwen2(512, 2).to_dict(), seed=0, dtype=torch.float32)
    hf.load_state_dict(w0, strict=False)
    ents = []
    for c, loss in zip(caps, losses):
        lp, ent = og.per_token_logps(hf, c["prompt_ids"], c["prompt_mask"].long(), c["completion_ids"],
                                     c["completion_mask"].long())
        sc = og.score_generation(hf, {"prompt_ids": c["prompt_ids"], "prompt_mask": c["prompt_mask"].long(),
                                      "completion_ids": c["completion_ids"]},
                                 lambda ids, m: [float(sum(r[mm.bool()].tolist()) % 7) for r, mm in zip(ids, m)],
                                 num_generations=4, eos_token_id=EOS)
        assert torch.equal(sc["cm"].int(), c["completion_mask"].int())
        torch.testing.assert_close(c["advantages"].float(), sc["a"].float(), rtol=0, atol=1e-6)
        ref_loss, met = trl_ref.grpo_loss(lp.detach(), sc["a"], sc["cm"].float(), entropies=ent, loss_type="grpo",
                                          max_completion_length=12)
        assert abs(loss - float(ref_loss)) <= 1e-4 * max(1.0, abs(float(ref_loss))), (loss, float(ref_loss))
        ents.append(met["entropy"])
    assert metrics["eval_loss"] == pytest.approx(sum(losses) / len(losses), rel=1e-6)
    assert metrics["eval_entropy"] == pytest.approx(sum(ents) / len(ents), rel=1e-4, abs=1e-5)
    # evaluation inside training: logged, and the training stream untouched
    a = _trainer(_args(max_steps=2, eval_strategy="steps", eval_steps=1, per_device_eval_batch_size=8),
                 eval_dataset=_ds(4, off=40))
    a.train()
    b = _trainer(_args(max_steps=2))
    b.train()
    assert len([h for h in a.state.log_history if "eval_loss" in h]) == 2
    assert torch.equal(a.model.flat, b.model.flat)


def _first_rollout(args, **kw):
    tr = _trainer(args, **kw)
    examples = [tr.train_dataset[i] for i in range(4) for _ in range(tr.num_generations)]
    out = tr._generate_and_score_completions(examples)
    return out["completion_ids"].cpu(), tr


def test_generation_kwargs_override_config_fields():
    """grpo_trainer.py:995-1014: generation_kwargs are applied on top of the config
    fields, so {"temperature": 0.7, "top_k": 50} there draws exactly what the
    config fields temperature 0.7 / top_k 50 draw (same Philox stream), and not what
    the config's T 1.0 draws; max_new_tokens / do_sample / min_new_tokens
    overrides shape the rollout the same way; the scoring temperature stays
    args.temperature (:1249)."""
    gk = {"eos_token_id": EOS, "pad_token_id": PAD}
    a, tra = _first_rollout(_args(temperature=0.7, top_k=50))
    b, trb = _first_rollout(_args(generation_kwargs={**gk, "temperature": 0.7, "top_k": 50}))
    c, _ = _first_rollout(_args())
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
    assert tra.temperature == 0.7 and trb.temperature == 1.0   # scoring divides by args.temperature
    short, trs = _first_rollout(_args(generation_kwargs={**gk, "max_new_tokens": 5, "min_new_tokens": 5}))
    assert short.shape[1] == 5 and trs._engine.Cmax == 5
    g1, _ = _first_rollout(_args(seed=3, generation_kwargs={**gk, "do_sample": False, "temperature": 0.3}))
    g2, _ = _first_rollout(_args(seed=9, generation_kwargs={**gk, "do_sample": False}))
    assert torch.equal(g1, g2)   # greedy: independent of the sampler seed and of the (dropped) warpers


@pytest.mark.parametrize("bad", [{"num_beams": 2}, {"no_repeat_ngram_size": 2}, {"typical_p": 0.9},
                                 {"bad_words_ids": [[5]]}, {"num_return_sequences": 2}, {"penalty_alpha": 0.6}])
def test_generation_kwargs_unimplemented_keys_raise(bad):
    """HF generation keys the engine does not implement raise at construction
    instead of being dropped."""
    with pytest.raises(ValueError, match=next(iter(bad))):
        _trainer(_args(generation_kwargs={"eos_token_id": EOS, "pad_token_id": PAD, **bad}))
