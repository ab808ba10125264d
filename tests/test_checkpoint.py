"""Checkpoint format on the host: the saved directory is what
transformers' from_pretrained reads (config + safetensors, tied head dropped),
and optimizer.pt is a torch AdamW state_dict over the transformers parameters
in the Trainer's decay / no-decay grouping (transformers Trainer.create_optimizer,
get_decay_parameter_names), loadable by torch.optim.AdamW."""
import os

import pytest
import torch

from swh_trl_amd.engine import CausalLM
from swh_trl_amd.engine.config import tiny_llama, tiny_qwen2
from swh_trl_amd.trainer import checkpoint as ck


def _cpu_model(cfg, dtype=torch.bfloat16, head="lm"):
    return CausalLM(cfg, "cpu", seed=2, dtype=dtype, trainable=False, head=head)


@pytest.mark.parametrize("cfg_fn,dtype", [(tiny_qwen2, torch.bfloat16), (tiny_llama, torch.bfloat16),
                                          (tiny_qwen2, torch.float32)])
def test_save_pretrained_loads_in_transformers(tmp_path, cfg_fn, dtype):
    from transformers import AutoModelForCausalLM
    m = _cpu_model(cfg_fn(512, 2), dtype)
    ck.save_pretrained(m, str(tmp_path), eos_token_id=1, pad_token_id=0)
    assert os.path.exists(tmp_path / "config.json") and os.path.exists(tmp_path / "model.safetensors")
    hf = AutoModelForCausalLM.from_pretrained(str(tmp_path), dtype=dtype)
    assert hf.config.model_type == m.cfg.model_type
    ref = hf.state_dict()
    for k, v in m.hf_state_dict().items():
        assert torch.equal(ref[k], v), k
    # and back into the engine's layout
    from swh_trl_amd.trainer.grpo_trainer import load_model
    m2 = load_model(str(tmp_path), "cpu", trainable=False, dtype=dtype)
    assert m2.cfg == m.cfg and torch.equal(m2.flat, m.flat)


def test_score_head_saves_as_sequence_classifier(tmp_path):
    from transformers import AutoModelForSequenceClassification
    m = _cpu_model(tiny_qwen2(512, 2), head="score")
    ck.save_pretrained(m, str(tmp_path))
    hf = AutoModelForSequenceClassification.from_pretrained(str(tmp_path), dtype=torch.bfloat16)
    assert hf.config.num_labels == 1 and torch.equal(hf.score.weight, m.p["score"])


def test_sharded_save(tmp_path, monkeypatch):
    from transformers import AutoModelForCausalLM
    monkeypatch.setattr(ck, "SHARD_BYTES", 1 << 20)
    m = _cpu_model(tiny_qwen2(512, 2))
    ck.save_pretrained(m, str(tmp_path))
    assert os.path.exists(tmp_path / "model.safetensors.index.json")
    hf = AutoModelForCausalLM.from_pretrained(str(tmp_path), dtype=torch.bfloat16)
    assert torch.equal(hf.model.embed_tokens.weight, m.p["embed"])


def test_optimizer_state_is_a_torch_adamw_state_dict(tmp_path):
    from transformers import Qwen2Config, Qwen2ForCausalLM

    from swh_trl_amd.optim import FlatAdamW
    m = _cpu_model(tiny_qwen2(512, 2), torch.float32)
    opt = FlatAdamW(m.numel, "cpu", lr=3e-4, weight_decay=0.1, no_decay_ranges=m.no_decay_ranges())
    g = torch.Generator().manual_seed(0)
    opt.exp_avg.copy_(torch.randn(m.numel, generator=g))
    opt.exp_avg_sq.copy_(torch.rand(m.numel, generator=g))
    opt.step_count = 7
    sd = ck.optimizer_state_dict(m, opt, 0.1)
    torch.save(sd, tmp_path / "optimizer.pt")
    sd = torch.load(tmp_path / "optimizer.pt", weights_only=True)
    c = m.cfg
    hf = Qwen2ForCausalLM(Qwen2Config(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                      intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                      num_attention_heads=c.num_attention_heads,
                                      num_key_value_heads=c.num_key_value_heads, tie_word_embeddings=True))
    names = [n for n, _ in hf.named_parameters()]
    assert names == ck.hf_param_order(m)
    # the Trainer's grouping, built from transformers' own decay-name rule
    from transformers import Trainer
    decay = Trainer.get_decay_parameter_names(Trainer.__new__(Trainer), hf)
    params = dict(hf.named_parameters())
    groups = [{"params": [params[n] for n in names if n in decay], "weight_decay": 0.1},
              {"params": [params[n] for n in names if n not in decay], "weight_decay": 0.0}]
    topt = torch.optim.AdamW(groups, lr=3e-4)
    topt.load_state_dict(sd)
    exp_m, exp_v = ck._flat_views(m, opt.exp_avg), ck._flat_views(m, opt.exp_avg_sq)
    for n in names:
        st = topt.state[params[n]]
        assert int(st["step"]) == 7
        assert torch.equal(st["exp_avg"], exp_m[n]) and torch.equal(st["exp_avg_sq"], exp_v[n]), n
    # and back into a fresh flat optimizer
    opt2 = FlatAdamW(m.numel, "cpu", lr=1.0, weight_decay=0.1)
    ck.load_optimizer_state_dict(m, opt2, sd)
    assert opt2.step_count == 7 and opt2.lr == pytest.approx(3e-4)
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)


def test_checkpoint_rotation(tmp_path):
    for s in (1, 2, 3, 10):
        os.makedirs(tmp_path / f"checkpoint-{s}")
    assert ck.latest_checkpoint(str(tmp_path)).endswith("checkpoint-10")
    ck.rotate_checkpoints(str(tmp_path), 2)
    assert sorted(os.listdir(tmp_path)) == ["checkpoint-10", "checkpoint-3"]


def test_gpt2_checkpoint_round_trip_and_param_order(tmp_path):
    """BASELINE.json config 1 family: the GPT-2 layout saves as a transformers
    GPT2LMHeadModel (Conv1D weights transposed back), loads back bit-equal,
    its parameter order is GPT2LMHeadModel.named_parameters(), and the
    Trainer's no-decay set (biases + LayerNorms) matches."""
    from transformers import AutoModelForCausalLM, GPT2LMHeadModel
    from swh_trl_amd.engine import GPT2LM, gpt2_config
    from swh_trl_amd.engine.config import from_hf_config
    from swh_trl_amd.trainer.grpo_trainer import load_model
    m = GPT2LM(gpt2_config(), "cpu", seed=2, dtype=torch.float32, trainable=False)
    ck.save_pretrained(m, str(tmp_path), eos_token_id=1, pad_token_id=0)
    hf = AutoModelForCausalLM.from_pretrained(str(tmp_path), dtype=torch.float32)
    assert isinstance(hf, GPT2LMHeadModel) and from_hf_config(hf.config) == m.cfg
    ref = hf.state_dict()
    for k, v in m.hf_state_dict().items():
        assert torch.equal(ref[k], v), k
    assert ck.hf_param_order(m) == [n for n, _ in hf.named_parameters()]
    m2 = load_model(str(tmp_path), "cpu", trainable=False, dtype=torch.float32)
    assert isinstance(m2, GPT2LM) and torch.equal(m2.flat, m.flat)
    # no-decay ranges cover exactly the bias / LayerNorm parameters
    nd = set()
    for s, e in m.no_decay_ranges():
        nd.update(range(s, e))
    for name, (o, shape) in m.layout.items():
        want = name.endswith("_b") or "ln_" in name
        assert (o in nd) == want, name


SCHEDULES = [("linear", 0, None), ("linear", 3, None), ("constant", 0, None), ("constant_with_warmup", 3, None),
             ("cosine", 2, None), ("cosine", 0, {"num_cycles": 1.5}), ("cosine_with_restarts", 2, {"num_cycles": 3}),
             ("polynomial", 2, {"lr_end": 1e-5, "power": 2.0}), ("inverse_sqrt", 3, None),
             ("inverse_sqrt", 0, {"timescale": 4}), ("cosine_with_min_lr", 2, {"min_lr": 1e-4}),
             ("cosine_with_min_lr", 0, {"min_lr_rate": 0.2}),
             ("cosine_warmup_with_min_lr", 3, {"min_lr_rate": 0.1, "warmup_lr_rate": 0.05})]


@pytest.mark.parametrize("kind,warmup,kw", SCHEDULES)
def test_schedule_multiplier_matches_transformers(kind, warmup, kw):
    """schedule.multiplier == the LambdaLR lambda of transformers get_scheduler at
    every step of a 13-step run (and past its end), for each supported type."""
    from transformers import get_scheduler

    from swh_trl_amd.trainer import schedule
    total, lr = 13, 1e-3
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=lr)
    ref = get_scheduler(kind, opt, num_warmup_steps=warmup, num_training_steps=total,
                        scheduler_specific_kwargs=dict(kw or {}))
    fn = schedule.multiplier(kind, total, warmup, lr, kw)
    for s in range(total + 3):
        assert fn(s) == pytest.approx(ref.lr_lambdas[0](s), rel=1e-12, abs=1e-15), (kind, s)


def test_schedule_rejects_unsupported_and_warmup_ratio():
    from types import SimpleNamespace

    from swh_trl_amd.trainer import schedule
    with pytest.raises(ValueError, match="not supported"):
        schedule.multiplier("reduce_lr_on_plateau", 10, 0, 1e-3)
    with pytest.raises(ValueError, match="min_lr"):
        schedule.multiplier("cosine_with_min_lr", 10, 0, 1e-3)
    # TrainingArguments.get_warmup_steps: warmup_steps wins, else ceil(total * warmup_ratio)
    assert schedule.warmup_steps(SimpleNamespace(warmup_steps=0, warmup_ratio=0.25), 10) == 3
    assert schedule.warmup_steps(SimpleNamespace(warmup_steps=4, warmup_ratio=0.25), 10) == 4
    assert schedule.warmup_steps(SimpleNamespace(warmup_steps=0.5, warmup_ratio=0.0), 10) == 5


@pytest.mark.parametrize("kind,warmup,kw", SCHEDULES)
def test_scheduler_state_loads_into_transformers_lambdalr(kind, warmup, kw):
    """scheduler.pt is the LambdaLR state_dict transformers' Trainer saves: it
    loads into get_scheduler(...)'s LambdaLR (lr_lambdas key included) and
    equals the state of that scheduler stepped the same number of times."""
    import warnings

    from transformers import get_scheduler

    from swh_trl_amd.trainer import schedule
    total, steps, lr = 10, 4, 1e-3

    def fresh():
        opt = torch.optim.AdamW([{"params": [torch.nn.Parameter(torch.zeros(1))]} for _ in range(2)], lr=lr)
        return opt, get_scheduler(kind, opt, num_warmup_steps=warmup, num_training_steps=total,
                                  scheduler_specific_kwargs=dict(kw or {}))
    opt, stepped = fresh()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for _ in range(steps):
            opt.step()
            stepped.step()
    sd = ck.scheduler_state_dict(steps, lr, schedule.multiplier(kind, total, warmup, lr, kw))
    _, loaded = fresh()
    loaded.load_state_dict(sd)
    assert loaded.last_epoch == stepped.last_epoch == steps
    assert loaded.get_last_lr() == pytest.approx(stepped.get_last_lr())
    want = stepped.state_dict()
    assert set(sd) == set(want)
    for k in ("base_lrs", "last_epoch", "_step_count"):
        assert sd[k] == want[k], k
