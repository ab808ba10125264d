"""Reward paths and the TR-DPO reference sync of GRPOTrainer (-m gpu).

* conversational prompts (grpo_trainer.py:1534, :1901-1908; data_utils.py
  :100-116): the chat template continues a trailing assistant turn, and reward
  callables receive completions as [{"role": "assistant", "content":
  bootstrap + text}];
* a reward model given as an nn.Module (a transformers sequence classifier,
  :1462-1473): it scores the chat-templated prompt + completion messages
  (plain prompt + completion text otherwise), padded right, logits[:, 0];
* sync_ref_model (callbacks.py:106-131): every ref_model_sync_steps the
  reference becomes ref * (1 - alpha) + alpha * policy, rounded as torch's
  mul_ / add_ on the parameter dtype.
"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fake_tokenizer import make_byte_tokenizer, make_tokenizer  # noqa: E402

pytestmark = pytest.mark.gpu
V = 512


def _cfg():
    from swh_trl_amd.engine import tiny_qwen2
    return tiny_qwen2(V, 2)


def _classifier(dev):
    """A transformers reward model WITHOUT a pad id in its config: the trainer sets
    config.pad_token_id from the reward tokenizer (grpo_trainer.py:766-771)."""
    from transformers import Qwen2Config, Qwen2ForSequenceClassification
    torch.manual_seed(0)
    hc = Qwen2Config(vocab_size=V, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=2,
                     num_key_value_heads=1, num_labels=1)
    hc.pad_token_id = None
    return Qwen2ForSequenceClassification(hc).to(dev).eval()


RM_TOL = dict(rtol=1e-4, atol=1e-4)  # the fp32 engine copy of the reward model against transformers fp32


@pytest.mark.parametrize("bootstrap", [False, True])
def test_conversational_prompts_and_reward_model(bootstrap):
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    dev = torch.device("cuda:0")
    tok = make_tokenizer(V)
    g = torch.Generator().manual_seed(1)

    def conv(i):
        words = " ".join(f"w{int(x)}" for x in torch.randint(5, V, (4 + i % 3,), generator=g))
        p = [{"role": "system", "content": "w9 w10"}, {"role": "user", "content": words}]
        if bootstrap:
            p.append({"role": "assistant", "content": "w11 w12"})
        return {"prompt": p, "tag": i}

    ds = [conv(i) for i in range(8)]
    seen = {}

    def rew_fn(prompts=None, completions=None, completion_ids=None, tag=None, trainer_state=None, **kw):
        seen.setdefault("calls", []).append((prompts, completions, completion_ids, tag))
        return [float(len(c[0]["content"].split()) % 3) for c in completions]

    rm = _classifier(dev)
    args = GRPOConfig(per_device_train_batch_size=8, gradient_accumulation_steps=1, num_generations=4,
                      max_prompt_length=32, max_completion_length=12, learning_rate=1e-4, max_steps=1, seed=2,
                      shuffle_dataset=False, logging_steps=1, save_strategy="no")
    tr = GRPOTrainer(model=_cfg(), reward_funcs=[rew_fn, rm], args=args, train_dataset=ds, processing_class=tok,
                     reward_processing_classes=[None, tok])
    got = {}
    calc = tr._calculate_rewards

    def capture(examples, *a):
        out = calc(examples, *a)
        got["rpf"], got["examples"] = out.detach().cpu().clone(), examples
        got["ids"] = a[3].detach().cpu().clone()
        got["mask"] = a[4].detach().cpu().clone()
        return out

    tr._calculate_rewards = capture
    tr.train()
    prompts, completions, cids, tags = seen["calls"][0]
    examples = got["examples"]
    assert tags == [x["tag"] for x in examples]
    # the prompts the reward functions see are the originals, untouched
    assert prompts == [x["prompt"] for x in examples]
    texts = tok.batch_decode(got["ids"], skip_special_tokens=True)
    boot = "w11 w12" if bootstrap else ""
    assert completions == [[{"role": "assistant", "content": boot + t}] for t in texts]
    assert cids == [r[m.bool()].tolist() for r, m in zip(got["ids"], got["mask"])]
    # the prompt token ids: the chat template continues a trailing assistant turn
    p0 = tok.apply_chat_template(examples[0]["prompt"], tokenize=False, continue_final_message=bootstrap,
                                 add_generation_prompt=not bootstrap)
    assert p0.endswith("w11 w12") if bootstrap else p0.endswith("<assistant> ")
    # the reward model: logits[:, 0] on the chat-templated prompt + completion
    msgs = [tok.apply_chat_template(x["prompt"] + c, tokenize=False) for x, c in zip(examples, completions)]
    enc = tok(text=msgs, return_tensors="pt", padding=True, padding_side="right", add_special_tokens=False)
    with torch.inference_mode():
        exp = rm(**{k: v.to(dev) for k, v in enc.items()}).logits[:, 0].float().cpu()
    torch.testing.assert_close(got["rpf"][:, 1], exp, **RM_TOL)
    assert rm.config.pad_token_id == tok.pad_token_id  # set by the trainer (:770)
    torch.testing.assert_close(got["rpf"][:, 0], torch.tensor([float(len(c[0]["content"].split()) % 3)
                                                               for c in completions]))


def test_reward_model_plain_text_prompts():
    """Non-conversational text prompts: the reward model scores prompt + completion text."""
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    dev = torch.device("cuda:0")
    tok = make_tokenizer(V)
    ds = [{"prompt": " ".join(f"w{5 + (7 * i + j) % 400}" for j in range(6)) + " "} for i in range(4)]
    rm = _classifier(dev)
    args = GRPOConfig(per_device_train_batch_size=8, gradient_accumulation_steps=1, num_generations=4,
                      max_prompt_length=16, max_completion_length=8, max_steps=1, seed=3, shuffle_dataset=False,
                      save_strategy="no")
    tr = GRPOTrainer(model=_cfg(), reward_funcs=rm, args=args, train_dataset=ds, processing_class=tok,
                     reward_processing_classes=[tok])
    got = {}
    calc = tr._calculate_rewards

    def capture(examples, *a):
        out = calc(examples, *a)
        got["rpf"], got["examples"], got["ids"] = out.cpu().clone(), examples, a[3].cpu().clone()
        return out

    tr._calculate_rewards = capture
    tr.train()
    texts = [x["prompt"] + c for x, c in zip(got["examples"], tok.batch_decode(got["ids"], skip_special_tokens=True))]
    enc = tok(text=texts, return_tensors="pt", padding=True, padding_side="right", add_special_tokens=False)
    with torch.inference_mode():
        exp = rm(**{k: v.to(dev) for k, v in enc.items()}).logits[:, 0].float().cpu()
    torch.testing.assert_close(got["rpf"][:, 0], exp, **RM_TOL)


def _text_dataset(n=4):
    return [{"prompt": " ".join(f"w{5 + (7 * i + j) % 400}" for j in range(6)) + " "} for i in range(n)]


def _train_and_capture(tr):
    got = {}
    calc = tr._calculate_rewards

    def capture(examples, *a):
        out = calc(examples, *a)
        got["rpf"], got["examples"], got["ids"] = out.cpu().clone(), examples, a[3].cpu().clone()
        return out

    tr._calculate_rewards = capture
    tr.train()
    return got


def _expected_scores(rm, ptok, rtok, got, dev):
    """The reference's scores: completions decoded by the policy tokenizer, the
    texts encoded by the reward model's own."""
    texts = [x["prompt"] + c for x, c in zip(got["examples"], ptok.batch_decode(got["ids"], skip_special_tokens=True))]
    enc = rtok(text=texts, return_tensors="pt", padding=True, padding_side="right", add_special_tokens=False)
    with torch.inference_mode():
        return rm(**{k: v.to(dev) for k, v in enc.items()}).logits[:, 0].float().cpu()


@pytest.mark.parametrize("source", ["directory", "module"])
def test_reward_model_scores_match_transformers_at_ragged_lengths(tmp_path, source):
    """RewardModel (the engine's fp32 score-head copy, from a directory or from
    the module) against transformers at right-padded ragged lengths across the
    attention tile edges (1..130 tokens), with and without an attention mask."""
    from transformers import AutoModelForSequenceClassification

    from swh_trl_amd.trainer.grpo_trainer import RewardModel
    dev = torch.device("cuda:0")
    d = tmp_path / "rm"
    _classifier("cpu").save_pretrained(str(d))
    rm = AutoModelForSequenceClassification.from_pretrained(str(d), num_labels=1, dtype=torch.float32).to(dev).eval()
    rm.config.pad_token_id = 256
    mine = (RewardModel.from_pretrained(str(d), dev, torch.float32) if source == "directory"
            else RewardModel.from_module(rm, dev))
    mine.config.pad_token_id = 256
    g = torch.Generator().manual_seed(7)
    for L in (1, 17, 63, 64, 65, 100, 130):
        lens = torch.tensor([L] + [int(x) for x in torch.randint(1, L + 1, (5,), generator=g)])
        ids = torch.randint(0, 256, (6, L), generator=g)
        am = (torch.arange(L)[None] < lens[:, None]).long()
        ids = ids.masked_fill(am == 0, 256)
        with torch.inference_mode():
            exp = rm(input_ids=ids.to(dev), attention_mask=am.to(dev)).logits[:, 0].float().cpu()
            got = mine(input_ids=ids.to(dev), attention_mask=am.to(dev)).logits[:, 0].float().cpu()
            got_nomask = mine(input_ids=ids.to(dev)).logits[:, 0].float().cpu()
        torch.testing.assert_close(got, exp, **RM_TOL, msg=lambda m, L=L: f"L={L}: {m}")
        torch.testing.assert_close(got_nomask, exp, **RM_TOL, msg=lambda m, L=L: f"L={L} no mask: {m}")


def test_string_reward_model_loads_from_local_directory(tmp_path):
    """grpo_trainer.py:731-739, :754-771: a string reward function is loaded as
    AutoModelForSequenceClassification(num_labels=1) (here from a local directory,
    onto the engine's score head, in model_init_kwargs' dtype), named by the last
    component of its path, its tokenizer loaded from the same place when
    reward_processing_classes is None and its pad id written into the config."""
    from transformers import AutoModelForSequenceClassification, AutoTokenizer

    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    from swh_trl_amd.trainer.grpo_trainer import RewardModel
    dev = torch.device("cuda:0")
    tok = make_tokenizer(V)
    d = tmp_path / "my-reward-model"
    _classifier("cpu").save_pretrained(str(d))
    make_byte_tokenizer().save_pretrained(str(d))  # the reward model's own tokenizer, found through its path
    args = GRPOConfig(per_device_train_batch_size=8, gradient_accumulation_steps=1, num_generations=4,
                      max_prompt_length=16, max_completion_length=8, max_steps=1, seed=3, shuffle_dataset=False,
                      save_strategy="no", model_init_kwargs={"torch_dtype": "float32"})
    tr = GRPOTrainer(model=_cfg(), reward_funcs=str(d), args=args, train_dataset=_text_dataset(), processing_class=tok)
    assert tr.reward_func_names == ["my-reward-model"]
    assert isinstance(tr.reward_funcs[0], RewardModel) and tr.reward_funcs[0].model.dtype == torch.float32
    rtok = AutoTokenizer.from_pretrained(str(d))
    assert type(tr.reward_processing_classes[0]) is type(rtok) and rtok.pad_token_id == 256
    assert tr.reward_funcs[0].config.pad_token_id == 256
    got = _train_and_capture(tr)
    rm = AutoModelForSequenceClassification.from_pretrained(str(d), num_labels=1, dtype=torch.float32).to(dev).eval()
    rm.config.pad_token_id = rtok.pad_token_id
    torch.testing.assert_close(got["rpf"][:, 0], _expected_scores(rm, tok, rtok, got, dev), **RM_TOL)
    assert any("rewards/my-reward-model/mean" in h for h in tr.state.log_history)
    with pytest.raises(ValueError, match="not a local directory"):
        GRPOTrainer(model=_cfg(), reward_funcs="org/some-hub-model", args=args, train_dataset=_text_dataset(),
                    processing_class=tok)


def test_module_reward_model_pads_with_eos_and_is_named_by_path(tmp_path):
    """A reward tokenizer without a pad token pads with EOS (:766-767) and the
    model's config.pad_token_id follows (:770), so the score is read at the last
    non-EOS token, as transformers does.  A module's metric name is the last
    path component of its config._name_or_path (:737)."""
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast, Qwen2ForSequenceClassification

    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    dev = torch.device("cuda:0")
    vocab = {"[PAD]": 0, "[EOS]": 1, "<system>": 2, "<user>": 3, "<assistant>": 4}
    vocab.update({f"w{i}": i for i in range(5, V)})
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="[PAD]"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    nopad = PreTrainedTokenizerFast(tokenizer_object=tk, eos_token="[EOS]")
    assert nopad.pad_token_id is None
    d = tmp_path / "rm-nopad"
    _classifier("cpu").save_pretrained(str(d))
    rm = Qwen2ForSequenceClassification.from_pretrained(str(d), dtype=torch.float32).to(dev).eval()
    assert rm.config.pad_token_id is None
    tok = make_tokenizer(V)
    args = GRPOConfig(per_device_train_batch_size=8, gradient_accumulation_steps=1, num_generations=4,
                      max_prompt_length=16, max_completion_length=8, max_steps=1, seed=4, shuffle_dataset=False,
                      save_strategy="no")
    tr = GRPOTrainer(model=_cfg(), reward_funcs=[rm], args=args, train_dataset=_text_dataset(), processing_class=tok,
                     reward_processing_classes=nopad)
    rtok = tr.reward_processing_classes[0]
    assert rtok is nopad and rtok.pad_token == "[EOS]" and rtok.pad_token_id == 1
    assert rm.config.pad_token_id == 1 and tr.reward_func_names == ["rm-nopad"]
    got = _train_and_capture(tr)
    torch.testing.assert_close(got["rpf"][:, 0], _expected_scores(rm, tok, rtok, got, dev), **RM_TOL)
    with pytest.raises(ValueError, match="number of reward processing classes"):
        GRPOTrainer(model=_cfg(), reward_funcs=[rm], args=args, train_dataset=_text_dataset(),
                    processing_class=tok, reward_processing_classes=[tok, tok])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_sync_ref_model_kernel_matches_callback_formula(dtype):
    """swh_ema_mix == SyncRefModelCallback._sync_target_model on the same dtype:
    target.mul_(1 - alpha).add_(copy, alpha=alpha) (torch ops on the GPU)."""
    from swh_trl_amd.optim import sync_ref_model
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(4)
    ref = torch.randn(1_000_003, generator=g).to(dtype).to(dev)
    pol = torch.randn(1_000_003, generator=g).to(dtype).to(dev)
    for alpha in (0.6, 0.1, 0.9):
        exp = ref.clone().mul_(1.0 - alpha).add_(pol, alpha=alpha)
        got = ref.clone()
        sync_ref_model(got, pol, alpha)
        assert torch.equal(got, exp), (dtype, alpha, (got.float() - exp.float()).abs().max().item())


def test_trainer_syncs_reference_every_n_steps():
    from swh_trl_amd.engine import CausalLM
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
    dev = torch.device("cuda:0")
    ds = [{"prompt": None, "prompt_ids": list(range(5 + i, 13 + i))} for i in range(16)]

    def rew(completion_ids=None, **kw):
        return [float(len(set(c)) % 5) for c in completion_ids]

    args = GRPOConfig(per_device_train_batch_size=8, gradient_accumulation_steps=1, num_generations=4,
                      max_prompt_length=8, max_completion_length=8, learning_rate=1e-3, beta=0.04, max_steps=3,
                      sync_ref_model=True, ref_model_sync_steps=2, ref_model_mixup_alpha=0.6, seed=1,
                      save_strategy="no", generation_kwargs={"eos_token_id": 1, "pad_token_id": 0})
    tr = GRPOTrainer(model=CausalLM(_cfg(), dev, seed=5, init_std=0.05), reward_funcs=rew, args=args,
                     train_dataset=ds)
    ref0 = tr.ref_model.flat.clone()
    tr.training_step_group()
    assert torch.equal(tr.ref_model.flat, ref0)            # step 1: no sync
    tr.training_step_group()                               # step 2: sync
    exp = ref0.clone().mul_(1 - 0.6).add_(tr.model.flat, alpha=0.6)
    assert torch.equal(tr.ref_model.flat, exp)
