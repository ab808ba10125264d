"""Host-side logic of the product (no GPU): index streams, truncation, config
bookkeeping, and the data-parallel exchange over world-size-2 gloo."""
import json
import os

import pytest
import torch
import torch.multiprocessing as mp

from oracle import trl_ref
from swh_trl_amd.trainer import GRPOConfig
from swh_trl_amd.trainer import utils as U

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_repeat_sampler_matches_oracle():
    for (n, mini, bs, rep, seed) in [(7, 2, 1, 1, 0), (8, 1, 2, 2, 3), (7, 3, 2, 2, 42), (11, 8, 4, 1, 5)]:
        got = list(U.RepeatSampler(range(n), mini, bs, rep, shuffle=True, seed=seed))
        assert got == trl_ref.repeat_sampler_indices(n, mini, bs, rep, shuffle=True, seed=seed)
        assert len(got) == len(U.RepeatSampler(range(n), mini, bs, rep, shuffle=True, seed=seed))


def test_truncate_with_protected_tokens_kats():
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        cases = json.load(f)["truncate_with_protected_tokens"]["cases"]
    for c in cases:
        ids = torch.tensor(c["ids"])
        mask = torch.tensor(c["mask"]) if c["mask"] is not None else torch.ones_like(ids)
        if c.get("raises"):
            with pytest.raises(ValueError):
                U.truncate_with_protected_tokens(ids, mask, c["target"], c["protected"])
            continue
        ni, nm = U.truncate_with_protected_tokens(ids, mask, c["target"], c["protected"])
        assert ni.tolist() == c["expected_ids"]
        if c["expected_mask"] is not None:
            assert nm.tolist() == c["expected_mask"]


def test_high_entropy_mask_kats():
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        cases = json.load(f)["high_entropy_mask"]["cases"]
    for c in cases:
        got = U.get_high_entropy_mask(torch.tensor(c["entropies"]), torch.tensor(c["mask"]), c["threshold"])
        assert got.tolist() == [[bool(v) for v in r] for r in c["expected"]]


def test_grpo_config_bookkeeping():
    c = GRPOConfig(per_device_train_batch_size=16, gradient_accumulation_steps=4, num_generations=8)
    assert c.steps_per_generation == 4 and c.generation_batch_size == 64 and c.bf16
    with pytest.raises(ValueError):
        GRPOConfig(per_device_train_batch_size=3, num_generations=8)
    with pytest.raises(ValueError):
        GRPOConfig(num_generations=1, per_device_train_batch_size=8)
    with pytest.raises(ValueError):
        GRPOConfig(generation_batch_size=64, steps_per_generation=2)
    with pytest.raises(ValueError):
        GRPOConfig(use_vllm=True)
    with pytest.raises(ValueError, match="some_unknown_field"):
        GRPOConfig(some_unknown_field=1)


@pytest.mark.parametrize("bad", [{"optim": "adafactor"}, {"optim": "sgd"}, {"logging_strategy": "epoch"},
                                 {"fp16": True}, {"tf32": True}, {"neftune_noise_alpha": 5.0},
                                 {"load_best_model_at_end": True}, {"deepspeed": "ds.json"}, {"fsdp": "full_shard"},
                                 {"use_cpu": True}, {"push_to_hub": True}, {"auto_find_batch_size": True},
                                 {"dataloader_drop_last": True}, {"use_liger_kernel": True}, {"not_a_field": 0}])
def test_configs_raise_on_result_changing_training_args(bad):
    """The reference configs are TrainingArguments handed whole to the transformers
    Trainer (grpo_trainer.py:837-846): a field the drop-in does not implement is
    accepted only where it cannot change the result; these would, so they raise."""
    from swh_trl_amd.trainer import PPOConfig
    with pytest.raises(ValueError, match=next(iter(bad))):
        GRPOConfig(per_device_train_batch_size=8, num_generations=4, **bad)
    with pytest.raises(ValueError, match=next(iter(bad))):
        PPOConfig(**bad)


def test_configs_keep_inert_training_args():
    """Reporting / hub / data-loader / DDP plumbing fields and the inert values
    of the constrained ones construct unchanged and are kept in `extra`."""
    from swh_trl_amd.trainer import PPOConfig
    inert = dict(report_to=["wandb"], run_name="r", logging_dir="/tmp/x", dataloader_num_workers=4,
                 dataloader_pin_memory=False, ddp_timeout=60, gradient_checkpointing=True, optim="adamw_torch",
                 logging_strategy="steps", tf32=False, push_to_hub=False, hub_strategy="end",
                 vllm_server_port=8000, save_safetensors=True, data_seed=3, fsdp="", deepspeed=None)
    c = GRPOConfig(per_device_train_batch_size=8, num_generations=4, **inert)
    assert c.extra == {k: v for k, v in inert.items() if k not in c.__dataclass_fields__}
    assert c.report_to == ["wandb"] and c.extra["optim"] == "adamw_torch"
    p = PPOConfig(**inert, eval_strategy="no")
    assert p.extra["optim"] == "adamw_torch" and p.extra["eval_strategy"] == "no"


def test_generation_config_overrides_follow_reference():
    """grpo_trainer.py:995-1014: the GenerationConfig is the config fields with
    `generation_kwargs` applied on top; keys the engine does not implement raise
    unless at their no-op value; greedy decoding drops the warpers."""
    from types import SimpleNamespace

    from swh_trl_amd.trainer.grpo_trainer import generation_config
    tok = SimpleNamespace(pad_token_id=7, eos_token_id=9, bos_token_id=None)
    base = dict(per_device_train_batch_size=8, num_generations=4, max_completion_length=32, temperature=1.0,
                top_p=0.9, top_k=None, min_p=None, repetition_penalty=1.0)
    g = generation_config(GRPOConfig(**base), tok)
    assert g == {"max_new_tokens": 32, "min_new_tokens": 0, "min_length": 0, "greedy": False, "temperature": 1.0,
                 "top_p": 0.9, "top_k": None, "min_p": None, "repetition_penalty": 1.0, "pad_token_id": 7,
                 "eos_token_id": 9}
    over = dict(temperature=0.7, top_k=50, top_p=0.95, min_p=0.05, repetition_penalty=1.1, max_new_tokens=16,
                min_new_tokens=4, eos_token_id=[9, 11], pad_token_id=3, num_beams=1, use_cache=True,
                cache_implementation="static", output_scores=True)
    g = generation_config(GRPOConfig(**base, generation_kwargs=over), tok)
    assert (g["temperature"], g["top_k"], g["top_p"], g["min_p"], g["repetition_penalty"]) == (0.7, 50, 0.95, 0.05, 1.1)
    assert (g["max_new_tokens"], g["min_new_tokens"], g["eos_token_id"], g["pad_token_id"]) == (16, 4, [9, 11], 3)
    # the same values as config fields give the same parameters (the GPU test draws with both)
    same = generation_config(GRPOConfig(**{**base, "temperature": 0.7, "top_k": 50, "top_p": 0.95, "min_p": 0.05,
                                           "repetition_penalty": 1.1, "max_completion_length": 16},
                                        generation_kwargs={"min_new_tokens": 4, "eos_token_id": [9, 11],
                                                           "pad_token_id": 3}), tok)
    assert same == g
    greedy = generation_config(GRPOConfig(**base, generation_kwargs={"do_sample": False, "temperature": 0.5,
                                                                     "top_k": 3, "repetition_penalty": 1.3}), tok)
    assert greedy["greedy"] and greedy["temperature"] == 1.0 and greedy["top_k"] is None
    assert greedy["top_p"] == 1.0 and greedy["repetition_penalty"] == 1.3  # the penalty is a processor, not a warper
    for bad in ({"num_beams": 4}, {"no_repeat_ngram_size": 3}, {"typical_p": 0.5}, {"bad_words_ids": [[5]]},
                {"num_return_sequences": 2}, {"return_dict_in_generate": True}, {"stop_strings": ["x"]},
                {"not_a_generation_key": 1}, {"temperature": 0.0}, {"top_k": -1}, {"max_new_tokens": 0}):
        with pytest.raises(ValueError):
            generation_config(GRPOConfig(**base, generation_kwargs=bad), tok)


def test_grpo_config_eval_and_strategy_fields():
    """TrainingArguments fields the drop-in honours: eval_strategy "no"/"steps"
    (the older `evaluation_strategy` name too), eval batches of whole groups,
    save_strategy "no"/"steps"; other strategies raise instead of being ignored."""
    c = GRPOConfig(per_device_train_batch_size=8, num_generations=4, evaluation_strategy="steps",
                   per_device_eval_batch_size=8, eval_steps=2, lr_scheduler_type="cosine",
                   lr_scheduler_kwargs={"num_cycles": 1.0}, warmup_ratio=0.1)
    assert c.eval_strategy == "steps" and c.eval_steps == 2 and "evaluation_strategy" not in c.extra
    assert c.lr_scheduler_kwargs == {"num_cycles": 1.0} and c.warmup_ratio == 0.1
    with pytest.raises(ValueError, match="eval batch"):
        GRPOConfig(per_device_train_batch_size=8, num_generations=4, eval_strategy="steps",
                   per_device_eval_batch_size=6)
    for bad in ({"eval_strategy": "epoch"}, {"save_strategy": "epoch"}):
        with pytest.raises(ValueError):
            GRPOConfig(per_device_train_batch_size=8, num_generations=4, **bad)


def test_trainers_refuse_user_optimizers():
    """The reference hands `optimizers` to the transformers Trainer; the fused
    AdamW of the drop-in cannot be driven by a torch optimizer / scheduler, so a
    non-default `optimizers` raises (before anything touches a device)."""
    from swh_trl_amd.trainer import GRPOTrainer, PPOConfig, PPOTrainer
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p])
    with pytest.raises(ValueError, match="optimizers"):
        GRPOTrainer(model="tiny", reward_funcs=lambda **k: [0.0], args=GRPOConfig(per_device_train_batch_size=8,
                                                                                  num_generations=4),
                    optimizers=(opt, None))
    with pytest.raises(ValueError, match="optimizers"):
        PPOTrainer(args=PPOConfig(), processing_class=None, model="tiny", ref_model=None, reward_model="tiny",
                   train_dataset=[], value_model="tiny", optimizers=(None, torch.optim.lr_scheduler.LambdaLR(
                       opt, lambda s: 1.0)))


def test_ppo_config_bookkeeping():
    """ppo_trainer.py:224-250 derived batch sizes and their errors."""
    from swh_trl_amd.trainer import PPOConfig
    from swh_trl_amd.trainer.ppo_trainer import fill_batch_sizes
    c = fill_batch_sizes(PPOConfig(per_device_train_batch_size=4, gradient_accumulation_steps=2,
                                   num_mini_batches=2, num_train_epochs=2), dataset_len=50, world_size=4)
    assert (c.local_batch_size, c.micro_batch_size, c.batch_size) == (8, 16, 32)
    assert (c.mini_batch_size, c.local_mini_batch_size) == (16, 4)
    assert c.total_episodes == 100 and c.num_total_batches == 4  # ceil(100 / 32)
    assert c.kl_estimator == "k1" and c.response_length == 53 and c.temperature == 0.7 and c.bf16
    with pytest.raises(ValueError):
        fill_batch_sizes(PPOConfig(per_device_train_batch_size=3, num_mini_batches=2), 10, 1)
    with pytest.raises(ValueError):  # whitening needs >= 8 rows per rank mini-batch
        fill_batch_sizes(PPOConfig(per_device_train_batch_size=4, whiten_rewards=True), 10, 1)


def test_ppo_response_helpers_match_oracle():
    """first_true_indices / truncate_response (utils.py:877-897, :1036-1056)."""
    from swh_trl_amd.trainer.ppo_trainer import first_true_indices, truncate_response
    g = torch.Generator().manual_seed(0)
    r = torch.randint(0, 6, (9, 13), generator=g)
    r[0] = 5  # no stop token at all
    for stop in (0, 1, 3):
        assert torch.equal(first_true_indices(r == stop), trl_ref.first_true_indices(r == stop))
        assert torch.equal(truncate_response(stop, 4, r), trl_ref.truncate_response(stop, 4, r))
    assert first_true_indices(torch.zeros(2, 7, dtype=torch.bool)).tolist() == [7, 7]


def test_split_and_shuffle_dicts():
    d = {"x": torch.arange(12).reshape(6, 2), "y": torch.arange(6), "z": None}
    parts = U.split_tensor_dict(d, 3)
    assert [p["y"].tolist() for p in parts] == [[0, 1], [2, 3], [4, 5]] and parts[0]["z"] is None
    s = U.shuffle_sequence_dict({"x": torch.arange(6), "y": list("abcdef")}, torch.Generator().manual_seed(0))
    assert [("abcdef"[int(i)]) for i in s["x"]] == s["y"]


def test_generation_batches_reshuffle_every_epoch():
    """One RepeatSampler (one generator) across epochs, as the reference's
    dataloader re-iterates it: epoch 2 draws a fresh permutation, equal to the
    sampler's second pass."""
    two = list(U.generation_batch_indices(12, 2, 6, 6, 0, seed=4, shuffle=True, epochs=2))
    s = U.RepeatSampler(range(12), 2, 3, 1, shuffle=True, seed=4)
    ref = list(s) + list(s)
    assert [i for b in two for i in b] == ref
    assert two[:4] != two[4:]


def test_linear_lr():
    assert U.linear_lr(0, 10, 1.0) == 1.0 and U.linear_lr(5, 10, 1.0) == 0.5 and U.linear_lr(10, 10, 1.0) == 0.0
    assert U.linear_lr(1, 10, 1.0, warmup=2) == 0.5


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from swh_trl_amd import dist
    r, w, _ = dist.init_from_env(backend="gloo")
    buf = torch.full((1000,), float(r + 1), dtype=torch.bfloat16)
    dist.allreduce_mean_(buf, bucket_elems=300)
    gens = U.generation_batch_indices(40, 4, 16, 8, r, seed=7, shuffle=True, epochs=1)
    rows = dist.all_gather_rows(torch.full((3, 2), float(r)) + torch.arange(3.0).view(3, 1))
    q.put((r, buf.float().mean().item(), [list(b) for b in gens], dist.all_max(float(r)), rows.tolist()))
    torch.distributed.destroy_process_group()


def test_dp_exchange_and_sharding_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)])
    for p in ps:
        p.join(timeout=60)
    assert all(abs(m - 1.5) < 1e-6 for _, m, _, _, _ in res)
    assert all(mx == 1.0 for _, _, _, mx, _ in res)
    # the reward gather (grpo_trainer.py:1497): rank-ordered rows, identical on every rank
    exp = [[0.0, 0.0], [1.0, 1.0], [2.0, 2.0], [1.0, 1.0], [2.0, 2.0], [3.0, 3.0]]
    assert res[0][4] == exp and res[1][4] == exp
    b0, b1 = res[0][2], res[1][2]
    assert len(b0) == len(b1) == 10  # 40 prompts / 4 unique prompts per global generation batch
    glob = list(U.RepeatSampler(range(40), 4, 4, 1, shuffle=True, seed=7))
    for k in range(10):
        assert b0[k] + b1[k] == glob[k * 16:(k + 1) * 16]          # contiguous rank slices
        for lb in (b0[k], b1[k]):
            assert all(len(set(lb[i:i + 4])) == 1 for i in range(0, 8, 4))  # whole groups per rank


def _overlap_worker(rank, world, port, q):
    """A 4-'layer' chain whose weight gradients live in one flat buffer, with the
    layer-input hooks of engine/model.py releasing buckets during backward."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from swh_trl_amd import dist
    from swh_trl_amd.engine.model import _GradReady
    dist.init_from_env(backend="gloo")
    L, H = 4, 8
    flat_g = torch.zeros(3 + L * H * H + 5)        # [head | layers | tail], tail/head released by finish()
    g = torch.Generator().manual_seed(11)
    ws = [torch.randn(H, H, generator=g) for _ in range(L)]
    x = (torch.randn(6, H, generator=g) * (rank + 1)).requires_grad_(True)  # rank-dependent grads
    ar = dist.OverlappedAllReduce(flat_g)
    order = []

    def cb(i):
        order.append(i)
        s = 3 + i * H * H
        ar.release(s, s + H * H)

    h = x
    params = []
    for i in range(L):
        h = _GradReady.apply(h, i, cb)
        w = ws[i].clone().requires_grad_(True)
        params.append(w)
        h = torch.tanh(h @ w)
    h.sum().backward()
    ar.finish()  # drain pass 1 (its buffer held zeros)


    # the hook fired in reverse layer order; copy grads then (this test's stand-in for in-backward accumulation)
    local = torch.cat([torch.zeros(3)] + [w.grad.reshape(-1) for w in params] + [torch.full((5,), float(rank))])
    q.put((rank, order, local))
    # second pass: write grads first, then release in the hooks' order and finish
    flat_g.copy_(local)
    ar2 = dist.OverlappedAllReduce(flat_g)
    for i in reversed(range(L)):
        s = 3 + i * H * H
        ar2.release(s, s + H * H)
    ar2.finish()
    q.put((rank, "reduced", flat_g.clone()))
    torch.distributed.destroy_process_group()


def test_overlapped_allreduce_hooks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000)
    ps = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in range(4)]
    for p in ps:
        p.join(timeout=60)
    firsts = {r: (o, loc) for r, o, loc in got if not isinstance(o, str)}
    reduced = {r: t for r, o, t in got if isinstance(o, str)}
    assert firsts[0][0] == [3, 2, 1, 0] and firsts[1][0] == [3, 2, 1, 0]   # reverse layer order during backward
    mean = (firsts[0][1] + firsts[1][1]) / 2
    for r in (0, 1):
        torch.testing.assert_close(reduced[r], mean)                       # released ranges + finish() remainder


def test_ppo_accumulation_schedule_matches_accelerate():
    """The reference PPO loop steps its optimizer inside `accelerator.accumulate`
    (ppo_trainer.py:545-606): accelerate decides which micro-batches step.  The
    oracle's restatement (oracle/ppo_step.py accelerate_sync) and the product's
    counter (PPOTrainer._accumulate_sync) against the installed accelerate itself,
    driven like the reference: a prepared DataLoader repeated forever, one batch per
    update, every micro-batch of the PPO epochs inside `accumulate`; recorded: which
    micro-batches sync.  Includes data epochs whose last batch makes every
    micro-batch sync, and GA larger than the micro-batches of one mini-batch."""
    from types import SimpleNamespace

    from accelerate import Accelerator

    from oracle import ppo_step
    from swh_trl_amd.trainer.ppo_trainer import PPOTrainer

    for GA, micros_per_update, n_batches, updates in [(2, 4, 3, 7), (4, 4, 2, 5), (2, 2, 1, 3), (3, 6, 4, 9)]:
        acc = Accelerator(gradient_accumulation_steps=GA, cpu=True)
        loader = acc.prepare(torch.utils.data.DataLoader(list(range(n_batches)), batch_size=1))
        model = acc.prepare(torch.nn.Linear(1, 1))

        def repeat():
            while True:
                yield from loader

        it = iter(repeat())
        want = []
        for _ in range(updates):
            next(it)
            for _ in range(micros_per_update):
                with acc.accumulate(model):
                    want.append(acc.sync_gradients)
        # restatements: end_of_dataloader = the update's batch is the data epoch's last
        got_o, got_p, step = [], [], 0
        prod = SimpleNamespace(_accum_step=0, args=SimpleNamespace(gradient_accumulation_steps=GA))
        for u in range(updates):
            eod = u % n_batches == n_batches - 1
            for _ in range(micros_per_update):
                step, sync = ppo_step.accelerate_sync(step, GA, eod)
                got_o.append(sync)
                got_p.append(PPOTrainer._accumulate_sync(prod, eod))
        assert got_o == want, (GA, micros_per_update, n_batches, got_o, want)
        assert got_p == want
        acc.free_memory()


def test_grpo_epoch_accounting_follows_trainer():
    """transformers Trainer.set_initial_training_values over GRPO's dataloader
    (grpo_trainer.py:1063-1130: batches of per_device x spg, RepeatSampler repeating
    each generation batch spg x num_iterations times): optimizer steps per epoch =
    ceil(micro-steps / GA).  An epoch whose micro-batches are not a multiple of GA
    ends with a shorter update over the remainder (Trainer._run_epoch `remainder`);
    the next epoch's updates start at its first micro-batch."""
    import types

    from swh_trl_amd.trainer.grpo_trainer import GRPOTrainer

    def fake(n_prompts, **kw):
        a = GRPOConfig(**kw)
        ns = types.SimpleNamespace(args=a, num_generations=a.num_generations, num_iterations=a.num_iterations,
                                   train_dataset=list(range(n_prompts)))
        for name in ("_micro_steps_per_epoch", "_steps_per_epoch", "_total_steps", "_epoch_micro_steps",
                     "_update_size", "_update_index"):
            setattr(ns, name, types.MethodType(getattr(GRPOTrainer, name), ns))
        return ns

    def updates(t, n):  # (first micro-step, size) of the first n updates, as training_step_group takes them
        k, out = 0, []
        for u in range(n):
            size = t._update_size(k)
            assert all(t._update_index(k + j) == u for j in range(size))
            out.append((k, size))
            k += size
        return out

    # default: spg = GA, so every epoch is whole accumulations
    t = fake(20, per_device_train_batch_size=8, gradient_accumulation_steps=2, num_generations=4, num_train_epochs=2)
    assert t._micro_steps_per_epoch() == (20 // 4) * 2 and t._steps_per_epoch() == 5 and t._total_steps() == 10
    assert updates(t, 10) == [(2 * u, 2) for u in range(10)]
    # spg 2, GA 4, 3 generation batches per epoch: 6 micro-steps = 4 + a remainder of 2, per epoch
    t = fake(6, per_device_train_batch_size=4, gradient_accumulation_steps=4, steps_per_generation=2,
             num_generations=4, num_train_epochs=2)
    assert t._micro_steps_per_epoch() == 6 and t._steps_per_epoch() == 2 and t._total_steps() == 4
    assert updates(t, 4) == [(0, 4), (4, 2), (6, 4), (10, 2)]
    # GA larger than an epoch: one short update per epoch
    t = fake(4, per_device_train_batch_size=4, gradient_accumulation_steps=8, steps_per_generation=2,
             num_generations=4, num_train_epochs=3)
    assert t._micro_steps_per_epoch() == 4 and t._steps_per_epoch() == 1 and t._total_steps() == 3
    assert updates(t, 3) == [(0, 4), (4, 4), (8, 4)]
