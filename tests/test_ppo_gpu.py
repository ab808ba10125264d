"""PPOTrainer parity on the GPU (-m gpu): the rollout scoring, the PPO
micro-batch loss/gradients and the update loop against the CPU restatement in
oracle/ppo_step.py (transformers Qwen2 models in fp32 on the host, loaded
with the engine's bf16 weights).  Parity for this path is unpinned by the
reference's own tests; tolerances below are the bf16
engine against an fp32 restatement."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

PAD, EOS = 0, 1


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _hf(m, seqcls: bool, sd: dict = None):
    from transformers import Qwen2Config, Qwen2ForCausalLM, Qwen2ForSequenceClassification
    c = m.cfg
    hc = Qwen2Config(vocab_size=c.vocab_size, hidden_size=c.hidden_size, intermediate_size=c.intermediate_size,
                     num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                     num_key_value_heads=c.num_key_value_heads, rope_theta=c.rope_theta, rms_norm_eps=c.rms_norm_eps,
                     tie_word_embeddings=c.tie_word_embeddings, max_position_embeddings=c.max_position_embeddings,
                     num_labels=1, pad_token_id=PAD)
    hc._attn_implementation = "eager"
    hf = (Qwen2ForSequenceClassification if seqcls else Qwen2ForCausalLM)(hc)
    sd = {k: v.detach().float().cpu() for k, v in (sd or m.hf_state_dict()).items()}
    missing, _ = hf.load_state_dict(sd, strict=False)
    assert not [k for k in missing if "rotary" not in k and k != "lm_head.weight"], missing
    return hf.float().eval()


def _trainer(dev, dtype=torch.bfloat16, width="tiny", **kw):
    import dataclasses

    from swh_trl_amd.engine import CausalLM, tiny_qwen2
    from swh_trl_amd.engine.config import DecoderConfig
    from swh_trl_amd.trainer import PPOConfig, PPOTrainer
    if width == "tiny":
        cfg, rcfg, std, mul = tiny_qwen2(512, 2), tiny_qwen2(512, 1), 0.05, 6.0
    else:  # the Qwen2.5-0.5B width (H 896, I 4864, V 151936, 14:2 heads), 2 layers; a 1-layer reward model
        cfg = DecoderConfig(num_hidden_layers=2)
        rcfg, std, mul = dataclasses.replace(cfg, num_hidden_layers=1), 0.02, 60.0
    policy = CausalLM(cfg, dev, seed=11, init_std=std, dtype=dtype)
    with torch.no_grad():  # make the stop token likely, so rows end at different lengths
        policy.p["embed"][EOS].mul_(mul)
    value = CausalLM(cfg, dev, head="score", seed=12, init_std=std, dtype=dtype)
    reward = CausalLM(rcfg, dev, head="score", seed=13, init_std=std, dtype=dtype)
    g = torch.Generator().manual_seed(3)
    ds = []
    for i in range(16):
        n = 6 + i % 5  # ragged prompts -> left padding
        ds.append({"input_ids": torch.randint(2, min(512, cfg.vocab_size), (n,), generator=g).tolist()})
    a = dict(per_device_train_batch_size=4, gradient_accumulation_steps=2, num_mini_batches=2, num_ppo_epochs=2,
             response_length=12, stop_token_id=EOS, temperature=0.7, learning_rate=1e-3, total_episodes=16,
             pad_token_id=PAD, eos_token_id=EOS, seed=5)
    a.update(kw)
    return PPOTrainer(PPOConfig(**a), None, policy, None, reward, ds, value), ds


def _cpu(d):
    return {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in d.items()}


@pytest.mark.parametrize("kw", [dict(), dict(kl_estimator="k3", whiten_rewards=True, missing_eos_penalty=1.0,
                                               gradient_accumulation_steps=4, num_mini_batches=1),
                                dict(stop_token_id=None)])
def test_ppo_rollout_matches_oracle(dev, kw):
    from oracle import ppo_step
    tr, ds = _trainer(dev, **kw)
    a = tr.args
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    assert responses.shape[1] <= a.response_length
    ro = tr.rollout_from(queries, responses, logprobs)
    pol, ref = _hf(tr.policy_model, False), _hf(tr.ref_model, False)
    val, rm = _hf(tr.value_model, True), _hf(tr.reward_model, True)
    q, r = queries.cpu(), responses.cpu()
    o = ppo_step.rollout_scores(pol, ref, val, rm, q, r, logprobs.cpu().float(), pad_token_id=PAD,
                                stop_token_id=tr.stop_token_id, eos_token_id=EOS, temperature=a.temperature,
                                kl_coef=a.kl_coef, kl_estimator=a.kl_estimator, whiten_rewards=a.whiten_rewards,
                                missing_eos_penalty=a.missing_eos_penalty, gamma=a.gamma, lam=a.lam)
    mine = _cpu(ro)
    if tr.stop_token_id is not None:  # ragged ends exercised: some rows stopped early
        assert (mine["sequence_lengths"] < responses.shape[1] - 1).any()
    for k in ("padding_mask", "padding_mask_p1", "sequence_lengths", "postprocessed_responses"):
        assert torch.equal(mine[k], o[k]), k
    keep = ~o["padding_mask"]
    # generation log-probs (decode kernels, bf16) vs the fp32 processed scores
    gl = ppo_step.generation_logprobs(pol, q, r, PAD, a.temperature)
    assert (logprobs.cpu()[keep] - gl[keep]).abs().max() < 6e-2
    # model forwards: bf16 engine vs fp32 transformers
    assert (mine["ref_logprobs"][keep] - o["ref_logprobs"][keep]).abs().max() < 6e-2
    keep1 = ~o["padding_mask_p1"]
    assert (mine["values"].float()[keep1] - o["values"][keep1]).abs().max() < 3e-2
    assert (mine["rm_scores"].float() - (o["scores"] + (0 if a.missing_eos_penalty is None else
            a.missing_eos_penalty * ~torch.any(o["postprocessed_responses"] == EOS, -1)))).abs().max() < 3e-2
    # the arithmetic after the forwards, on the engine's own forward outputs: fp32-tight
    oa = ppo_step.rollout_arith(logprobs.cpu().float(), mine["ref_logprobs"], mine["values"], mine["rm_scores"],
                                mine["postprocessed_responses"], pad_token_id=PAD, eos_token_id=EOS,
                                kl_coef=a.kl_coef, kl_estimator=a.kl_estimator, whiten_rewards=a.whiten_rewards,
                                missing_eos_penalty=a.missing_eos_penalty, gamma=a.gamma, lam=a.lam)
    for k in ("logprobs", "scores", "kl", "non_score_reward", "rewards", "returns", "advantages"):
        torch.testing.assert_close(mine[k].float(), oa[k].float(), rtol=1e-4, atol=1e-4, msg=k)


BF16_TOL = 2.0 ** -8  # one bf16 rounding, relative


def _hf_grads(hf) -> dict:
    return {k: p.grad.detach().float().clone() for k, p in hf.named_parameters() if p.grad is not None}


def _check_grads_bf16(tag, prod: dict, orc_bf: dict, orc_32: dict):
    """Every gradient tensor: the product's relative error against the fp32
    oracle within twice the reference's own bf16 error (oracle bf16 vs fp32)
    plus one bf16 rounding — the bound tests/test_step_parity_gpu.py applies
    to the GRPO step."""
    worst = []
    for k, g32 in orc_32.items():
        n32 = g32.norm().clamp_min(1e-20)
        rel_ref = float((orc_bf[k] - g32).norm() / n32)
        rel_p = float((prod[k] - g32).norm() / n32)
        worst.append((rel_p - 2 * rel_ref, k, rel_p, rel_ref))
        assert rel_p <= 2 * rel_ref + BF16_TOL, (tag, k, rel_p, rel_ref)
    return max(worst)


def _stat_band(k, sb: dict, sf: dict) -> float:
    """The band for a statistic (a mean over tokens): twice the reference's own
    bf16 error of it plus one bf16 rounding of the fp32 value.  That error is
    taken as the larger of its realised value |oracle_bf16 - oracle_fp32| and
    twice its expected size, the per-token error RMS over sqrt(n) (a single
    realisation of a mean can land near zero by chance)."""
    b, f = sb[k], sf[k]
    tb, tf = sb["tokens"][k].float(), sf["tokens"][k].float()
    se = float((tb - tf).pow(2).mean().sqrt()) / math.sqrt(max(tb.numel(), 1))
    return 2 * max(abs(b - f), 2 * se) + BF16_TOL * abs(f) + 1e-6


def _check_stat_bf16(tag, k, p, sb, sf):
    band = _stat_band(k, sb, sf)
    assert abs(p - sb[k]) <= band, (tag, k, p, sb[k], sf[k], band)


WIDTHS = ["tiny", "qwen2.5-0.5b-width"]


@pytest.mark.parametrize("width", WIDTHS)
def test_ppo_micro_batch_bf16_matches_oracle(dev, width):
    """One micro-batch of the bf16 path (ppo_trainer.py:557-605) against the
    reference's own bf16 computation (transformers bf16 policy and value models,
    bf16 logits / (T + 1e-7), the bf16 selective_log_softmax) and its fp32
    computation on the same weights: loss terms and every policy / value
    gradient within the bf16-rounding bounds (BASELINE config 3's width:
    Qwen2.5-0.5B, 2 layers)."""
    from oracle import ppo_step
    tr, ds = _trainer(dev, width=width, gradient_accumulation_steps=1, num_mini_batches=1,
                      per_device_train_batch_size=8)
    a = tr.args
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    ro = tr.rollout_from(queries, responses, logprobs)
    inds = torch.tensor([5, 0, 3, 6, 1, 2, 7, 4])
    tr.policy_model.zero_grad()
    tr.value_model.zero_grad()
    st = tr._micro_step(ro, inds.to(dev))[0].cpu()
    gp, gv = _grads(tr.policy_model), _grads(tr.value_model)
    oro = _cpu(ro)
    oro["values"] = oro["values"].float()
    res = {}
    for dt in (torch.bfloat16, torch.float32):
        pol, val = _hf(tr.policy_model, False).to(dt), _hf(tr.value_model, True).to(dt)
        loss, ost = ppo_step.micro_batch_loss(pol, val, oro, inds, context_length=queries.shape[1], pad_token_id=PAD,
                                              temperature=a.temperature, cliprange=a.cliprange,
                                              cliprange_value=a.cliprange_value, vf_coef=a.vf_coef,
                                              token_terms=True)
        loss.backward()
        res[dt] = (ost, _hf_grads(pol), _hf_grads(val))
    (sb, pb, vb), (sf, pf, vf) = res[torch.bfloat16], res[torch.float32]
    for i, k in ((0, "pg_loss"), (1, "vf_loss"), (4, "approxkl"), (5, "ratio"), (8, "entropy")):
        _check_stat_bf16(width, k, float(st[i]), sb, sf)
    print(width, "policy", _check_grads_bf16(width + "-policy", gp, pb, pf))
    print(width, "value", _check_grads_bf16(width + "-value", gv, vb, vf))


def _sync_groups(a, perms, end_of_dataloader: bool, step0: int = 0):
    """The micro-batches (row indices) between the reference's optimizer steps:
    accelerate's accumulation (oracle/ppo_step.py accelerate_sync) over the
    micro-batches of every epoch's permutation in order."""
    from oracle import ppo_step
    groups, cur, step = [], [], step0
    for p in perms:
        p = torch.as_tensor(p)
        for m0 in range(0, a.local_batch_size, a.local_mini_batch_size):
            mini = p[m0:m0 + a.local_mini_batch_size]
            for u0 in range(0, len(mini), a.per_device_train_batch_size):
                step, sync = ppo_step.accelerate_sync(step, a.gradient_accumulation_steps, end_of_dataloader)
                cur.append(mini[u0:u0 + a.per_device_train_batch_size])
                if sync:
                    groups.append(torch.cat(cur))
                    cur = []
    return groups


@pytest.mark.parametrize("width,eod", [("tiny", False), ("tiny", True), ("qwen2.5-0.5b-width", False)])
def test_ppo_update_schedule_bf16_matches_oracle(dev, width, eod):
    """A full PPO update (ppo_trainer.py:537-617: epochs x mini-batches x micro-
    batches, no clipping) on the bf16 path, with the optimizer steps where the
    reference's accelerate accumulation takes them: every GA-th micro-batch
    across mini-batches (per-device 4 x GA 2 with 2 mini-batches: one step per two
    mini-batches), or after every micro-batch at the data epoch's last batch
    (end_of_dataloader).  Before each optimizer step the accumulated policy and
    value gradients equal the reference's micro-batches since the previous step
    (loss / GA each) evaluated in bf16 and in fp32 at the product's weights of
    that step, within the bf16-rounding bounds.  Each step is checked from the product's own weights: after one
    AdamW step (whose first update is ~lr * sign(grad)) two bf16 trajectories
    part by the sign noise of near-zero gradient elements, which says nothing
    about the schedule; the update itself is the AdamW kernel's own test.  At
    the 0.5B width lr 1e-5: Adam's first steps move every weight by ~lr, and at
    1e-4 the random 896-wide policy leaves any sane regime within two steps
    (approx-KL ~1e4, ratios ~100, gradients ~1e-8), where the reference's own
    bf16 gradient is 30-80 % off its fp32 one."""
    from oracle import ppo_step
    tr, ds = _trainer(dev, width=width, learning_rate=1e-4 if width == "tiny" else 1e-5)
    a = tr.args
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    ro = tr.rollout_from(queries, responses, logprobs)
    perms = [torch.randperm(a.local_batch_size, generator=torch.Generator().manual_seed(e)).tolist()
             for e in range(a.num_ppo_epochs)]
    oro = _cpu(ro)
    oro["values"] = oro["values"].float()
    prod_steps = []
    step_fn = tr._optimizer_step

    def snap(m):
        return {k: v.detach().cpu().clone() for k, v in m.hf_state_dict().items()}

    def capture(lr):
        prod_steps.append((snap(tr.policy_model), snap(tr.value_model), _grads(tr.policy_model),
                           _grads(tr.value_model)))
        return step_fn(lr)

    tr._optimizer_step = capture
    tr.ppo_update(ro, a.learning_rate, permutations=perms, end_of_dataloader=eod)
    minis = _sync_groups(a, perms, eod)
    micros = a.num_ppo_epochs * a.local_batch_size // a.per_device_train_batch_size
    assert len(prod_steps) == len(minis) == (micros if eod else micros // a.gradient_accumulation_steps)
    models = {dt: (_hf(tr.policy_model, False).to(dt), _hf(tr.value_model, True).to(dt))
              for dt in (torch.bfloat16, torch.float32)}
    for s, ((wp, wv, gp, gv), mini) in enumerate(zip(prod_steps, minis)):
        grads = {}
        for dt, (pol, val) in models.items():
            pol.load_state_dict(wp, strict=False)
            val.load_state_dict(wv, strict=False)
            pol.zero_grad(set_to_none=True)
            val.zero_grad(set_to_none=True)
            ppo_step.mini_batch_backward(pol, val, oro, mini, per_device_train_batch_size=a.per_device_train_batch_size,
                                         gradient_accumulation_steps=a.gradient_accumulation_steps,
                                         context_length=queries.shape[1], pad_token_id=PAD,
                                         temperature=a.temperature, cliprange=a.cliprange,
                                         cliprange_value=a.cliprange_value, vf_coef=a.vf_coef)
            grads[dt] = (_hf_grads(pol), _hf_grads(val))
        ob, of = grads[torch.bfloat16], grads[torch.float32]
        _check_grads_bf16(f"{width}-step{s}-policy", gp, ob[0], of[0])
        _check_grads_bf16(f"{width}-step{s}-value", gv, ob[1], of[1])


@pytest.mark.parametrize("width", WIDTHS)
def test_ppo_two_update_bf16_trajectory_within_reference_bands(dev, width):
    """Two PPO optimizer updates on one rollout (2 epochs x 1 mini-batch of GA 2
    micro-batches, ppo_trainer.py:537-617) run as trajectories: the product's bf16 run, and the
    reference loop's own bf16 and fp32 runs (oracle ppo_update: the same micro-
    batches, loss / GA, torch AdamW over the policy + value parameters, no
    clipping) from the same initial weights.  For every micro-batch of both
    updates, the product's policy loss, value loss and approx-KL stay within
    twice the reference's own bf16-vs-fp32 trajectory gap (or twice that
    statistic's expected bf16 noise, whichever is larger) plus one bf16 rounding,
    against the reference's bf16 run and against its fp32 run.  The second
    update starts from weights one AdamW step apart on all three runs (the
    reference's bf16 run updates its bf16 parameters directly, the product keeps
    fp32 masters), so the band there is the reference's own trajectory spread."""
    from oracle import ppo_step
    lr = 1e-4 if width == "tiny" else 1e-5
    # local batch = per-device 4 x GA 2 = 8 rows, one mini-batch of 2 micro-batches per epoch
    tr, ds = _trainer(dev, width=width, learning_rate=lr, num_ppo_epochs=2, num_mini_batches=1)
    a = tr.args
    n_micro = a.local_mini_batch_size // a.per_device_train_batch_size
    assert n_micro == a.gradient_accumulation_steps == 2 and a.local_batch_size == 8
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    ro = tr.rollout_from(queries, responses, logprobs)
    perms = [torch.randperm(a.local_batch_size, generator=torch.Generator().manual_seed(7 + e)).tolist()
             for e in range(a.num_ppo_epochs)]
    pol0, val0 = _hf(tr.policy_model, False), _hf(tr.value_model, True)
    stats = tr.ppo_update(ro, lr, permutations=perms).cpu()[:, :, :n_micro].reshape(-1, 9)  # [updates x micro, 9]
    oro = _cpu(ro)
    oro["values"] = oro["values"].float()
    runs = {}
    for dt in (torch.bfloat16, torch.float32):
        pol, val = _hf(tr.policy_model, False, pol0.state_dict()).to(dt), _hf(tr.value_model, True,
                                                                             val0.state_dict()).to(dt)
        opt = torch.optim.AdamW(list(pol.parameters()) + list(val.parameters()), lr=lr,
                                betas=(a.adam_beta1, a.adam_beta2), eps=a.adam_epsilon, weight_decay=a.weight_decay,
                                foreach=False)
        runs[dt], _ = ppo_step.ppo_update(pol, val, opt, oro, perms, local_mini_batch_size=a.local_mini_batch_size,
                                       per_device_train_batch_size=a.per_device_train_batch_size,
                                       gradient_accumulation_steps=a.gradient_accumulation_steps,
                                       context_length=queries.shape[1], pad_token_id=PAD, temperature=a.temperature,
                                       cliprange=a.cliprange, cliprange_value=a.cliprange_value, vf_coef=a.vf_coef,
                                       token_terms=True)
        del pol, val, opt
    ob, of = runs[torch.bfloat16], runs[torch.float32]
    assert len(ob) == len(of) == stats.shape[0] == 4
    report = []
    for j in range(4):
        for i, k in ((0, "pg_loss"), (1, "vf_loss"), (4, "approxkl")):
            band = _stat_band(k, ob[j], of[j])
            p = float(stats[j, i])
            report.append((j // n_micro, k, p, ob[j][k], of[j][k], band))
            assert abs(p - ob[j][k]) <= band, (width, report[-1])
            assert abs(p - of[j][k]) <= band, (width, report[-1])
    print(width, "update, stat, product, oracle bf16, oracle fp32, band:", report)


def test_ppo_trainer_train_runs(dev):
    tr, _ = _trainer(dev)
    before = tr.policy_model.flat.clone()
    vbefore = tr.value_model.flat.clone()
    state = tr.train()
    assert state.global_step == tr.args.num_total_batches == 2
    assert not torch.equal(before, tr.policy_model.flat)
    assert not torch.equal(vbefore, tr.value_model.flat)
    log = state.log_history[-1]
    for k in ("objective/kl", "loss/policy_avg", "loss/value_avg", "policy/approxkl_avg", "val/ratio"):
        assert log[k] == log[k], k  # finite


def test_ppo_final_checkpoint_when_steps_not_multiple_of_save_steps(dev, tmp_path):
    """DefaultFlowCallback's end-of-training branch (the reference PPOTrainer's
    default callbacks): with save_strategy 'steps', the last update saves even
    when num_total_batches is not a multiple of save_steps."""
    import os
    tr, _ = _trainer(dev, total_episodes=24, save_steps=2, output_dir=str(tmp_path))
    state = tr.train()
    assert state.global_step == tr.args.num_total_batches == 3
    assert os.path.isdir(tmp_path / "checkpoint-2") and os.path.isdir(tmp_path / "checkpoint-3")


@pytest.mark.parametrize("width", WIDTHS)
def test_ppo_fused_micro_batches_equal_separate(dev, width):
    """A mini-batch's GA micro-batches in one fused pass give the gradient of GA
    separate passes (each micro keeps its own masked means), up to bf16
    accumulation order: both are bf16 evaluations of one function, so each sits
    within the reference's own bf16 error of it, and they differ by at most twice
    that (oracle bf16 vs fp32 over the same two micro-batches) plus one bf16
    rounding."""
    from oracle import ppo_step
    tr, ds = _trainer(dev, width=width, gradient_accumulation_steps=2, num_mini_batches=1)
    a = tr.args
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    ro = tr.rollout_from(queries, responses, logprobs)
    inds = torch.tensor([6, 2, 7, 1, 0, 4, 3, 5], device=dev)
    tr.policy_model.zero_grad()
    tr.value_model.zero_grad()
    st_f = tr._micro_step(ro, inds, 2)
    gp_f, gv_f = _grads(tr.policy_model), _grads(tr.value_model)
    tr.policy_model.zero_grad()
    tr.value_model.zero_grad()
    st_s = torch.cat([tr._micro_step(ro, inds[:4]), tr._micro_step(ro, inds[4:])])
    gp_s, gv_s = _grads(tr.policy_model), _grads(tr.value_model)
    oro = _cpu(ro)
    oro["values"] = oro["values"].float()
    res = {}
    for dt in (torch.bfloat16, torch.float32):
        pol, val = _hf(tr.policy_model, False).to(dt), _hf(tr.value_model, True).to(dt)
        stats = []
        for half in (inds[:4].cpu(), inds[4:].cpu()):
            loss, ost = ppo_step.micro_batch_loss(pol, val, oro, half, context_length=queries.shape[1],
                                                  pad_token_id=PAD, temperature=a.temperature,
                                                  cliprange=a.cliprange, cliprange_value=a.cliprange_value,
                                                  vf_coef=a.vf_coef, token_terms=True)
            (loss / a.gradient_accumulation_steps).backward()
            stats.append(ost)
        res[dt] = (stats, _hf_grads(pol), _hf_grads(val))
    (sb, pb, vb), (sf, pf, vf) = res[torch.bfloat16], res[torch.float32]
    for j in range(2):
        for i, k in ((0, "pg_loss"), (1, "vf_loss"), (4, "approxkl"), (5, "ratio"), (8, "entropy")):
            band = _stat_band(k, sb[j], sf[j])
            assert abs(float(st_f[j, i]) - float(st_s[j, i])) <= band, (width, j, k, band)
    for fused, sep, ob, of in ((gp_f, gp_s, pb, pf), (gv_f, gv_s, vb, vf)):
        for k, g32 in of.items():
            n32 = g32.norm().clamp_min(1e-20)
            rel_ref = float((ob[k] - g32).norm() / n32)
            assert float((fused[k] - sep[k]).norm() / n32) <= 2 * rel_ref + BF16_TOL, (width, k)


def _grads(m):
    saved = m.flat.clone()
    m.flat.copy_(m.grad)
    g = {k: v.float().cpu().clone() for k, v in m.hf_state_dict().items()}
    m.flat.copy_(saved)
    return g


@pytest.mark.parametrize("width", ["tiny", "qwen2.5-0.5b-width"])
def test_ppo_fp32_reference_precision_matches_oracle(dev, width):
    """PPO in the reference-precision mode (fp32 policy / value / reward models, the
    fp32 rollout engine): the whole rollout scoring (ppo_trainer.py:389-535) and a
    micro-batch's loss and gradients (:557-605) against oracle/ppo_step.py with
    transformers fp32 models — generation / ref log-probs, values, scores and the
    derived rewards / returns / advantages within 1e-4, the loss terms within 1e-4,
    every policy and value gradient within 1e-3 relative."""
    from oracle import ppo_step
    tr, ds = _trainer(dev, dtype=torch.float32, width=width, gradient_accumulation_steps=1, num_mini_batches=1,
                      per_device_train_batch_size=8)
    a = tr.args
    assert tr.policy_model.dtype == tr.value_model.dtype == tr.reward_model.dtype == torch.float32
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    ro = tr.rollout_from(queries, responses, logprobs)
    pol, ref = _hf(tr.policy_model, False), _hf(tr.ref_model, False)
    val, rm = _hf(tr.value_model, True), _hf(tr.reward_model, True)
    q, r = queries.cpu(), responses.cpu()
    o = ppo_step.rollout_scores(pol, ref, val, rm, q, r, logprobs.cpu().float(), pad_token_id=PAD,
                                stop_token_id=tr.stop_token_id, eos_token_id=EOS, temperature=a.temperature,
                                kl_coef=a.kl_coef, kl_estimator=a.kl_estimator, whiten_rewards=a.whiten_rewards,
                                missing_eos_penalty=a.missing_eos_penalty, gamma=a.gamma, lam=a.lam)
    mine = _cpu(ro)
    assert (mine["sequence_lengths"] < responses.shape[1] - 1).any()  # ragged ends
    for k in ("padding_mask", "padding_mask_p1", "sequence_lengths", "postprocessed_responses"):
        assert torch.equal(mine[k], o[k]), k
    keep = ~o["padding_mask"]
    gl = ppo_step.generation_logprobs(pol, q, r, PAD, a.temperature)
    assert (logprobs.cpu()[keep] - gl[keep]).abs().max() < 1e-4
    for k in ("ref_logprobs", "values", "scores", "kl", "non_score_reward", "rewards", "returns", "advantages"):
        torch.testing.assert_close(mine[k].float(), o[k].float(), rtol=1e-4, atol=1e-4, msg=k)
    # one micro-batch: loss terms and every gradient
    inds = torch.tensor([5, 0, 3, 6, 1, 2, 7, 4])
    tr.policy_model.zero_grad()
    tr.value_model.zero_grad()
    st = tr._micro_step(ro, inds.to(dev))[0].cpu()
    oro = _cpu(ro)
    loss, ost = ppo_step.micro_batch_loss(pol, val, oro, inds, context_length=queries.shape[1], pad_token_id=PAD,
                                          temperature=a.temperature, cliprange=a.cliprange,
                                          cliprange_value=a.cliprange_value, vf_coef=a.vf_coef)
    loss.backward()
    for i, k in ((0, "pg_loss"), (1, "vf_loss"), (4, "approxkl"), (5, "ratio"), (8, "entropy")):
        assert abs(float(st[i]) - ost[k]) <= 1e-4 * max(1.0, abs(ost[k])), (k, float(st[i]), ost[k])
    for m, hf in ((tr.policy_model, pol), (tr.value_model, val)):
        g = _grads(m)
        for name, p in hf.named_parameters():
            if p.grad is None:
                continue
            rel = ((g[name] - p.grad).norm() / p.grad.norm().clamp_min(1e-20)).item()
            assert rel <= 1e-3, (name, rel)
