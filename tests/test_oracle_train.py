"""The oracle's training loop (oracle/grpo_step.py `grpo_train`) on the host:
the reference's buffering semantics it restates (grpo_trainer.py:1411-1444
_prepare_inputs, :1854-1869 old log-probs) on a tiny transformers Qwen2 in
fp32.  These pin the loop the GPU step-parity tests compare the product with."""
import torch

from oracle import grpo_step as og
from swh_trl_amd.engine.config import tiny_qwen2

EOS = 1


def _reward(cids, cmask):
    return [float(len(set(r[m.bool()].tolist())) % 5) for r, m in zip(cids, cmask)]


def _gen(seed, rows, G, P, C, V):
    g = torch.Generator().manual_seed(seed)
    prompts = torch.randint(2, V, (rows // G, P), generator=g).repeat_interleave(G, 0)
    comp = torch.randint(2, V, (rows, C), generator=g)
    comp[0, 5] = EOS
    return {"prompt_ids": prompts, "prompt_mask": torch.ones(rows, P, dtype=torch.long), "completion_ids": comp,
            "perm": torch.randperm(rows, generator=g)}


def _model(cfg):
    m = og.hf_qwen2_from_config(cfg.to_dict(), seed=1, dtype=torch.float32)
    return m, torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=0.0, foreach=False)


def test_fork_config_scores_old_logps_and_reuses_the_rollout():
    """num_iterations 2 with steps_per_generation == GA: one rollout feeds two
    optimizer steps; old log-probs exist (GA % (spg * mu) != 0); the first step
    trains the policy that produced them (ratio 1), the second a changed one."""
    cfg = tiny_qwen2(128, 1)
    G, P, C, MB, GA = 4, 6, 10, 4, 2
    m, opt = _model(cfg)
    gens = [_gen(0, MB * GA, G, P, C, cfg.vocab_size)]
    recs = og.grpo_train(m, opt, gens, _reward, num_generations=G, C=C, per_device_train_batch_size=MB,
                         gradient_accumulation_steps=GA, n_steps=2, num_iterations=2,
                         importance_sampling_level="sequence", eos_token_id=EOS, capture=True)
    sc = recs[0]["gens"]
    assert len(sc) == 1 and sc[0]["old"] is not None
    perm = gens[0]["perm"]
    mask = sc[0]["cm"][perm].bool()
    old = sc[0]["old"][perm]
    torch.testing.assert_close(recs[0]["logps"][mask], old[mask], rtol=0, atol=1e-5)
    assert (recs[1]["logps"][mask] - old[mask]).abs().max() > 1e-4


def test_aligned_steps_have_no_old_logps():
    cfg = tiny_qwen2(128, 1)
    G, P, C, MB, GA = 4, 6, 10, 4, 2
    m, opt = _model(cfg)
    recs = og.grpo_train(m, opt, [_gen(0, MB * GA, G, P, C, cfg.vocab_size)], _reward, num_generations=G, C=C,
                         per_device_train_batch_size=MB, gradient_accumulation_steps=GA, n_steps=1,
                         eos_token_id=EOS, capture=True)
    assert recs[0]["gens"][0]["old"] is None


def test_steps_per_generation_below_ga_draws_two_rollouts_per_step():
    cfg = tiny_qwen2(128, 1)
    G, P, C, MB, GA, spg = 4, 6, 10, 4, 4, 2
    m, opt = _model(cfg)
    gens = [_gen(s, MB * spg, G, P, C, cfg.vocab_size) for s in (0, 1)]
    recs = og.grpo_train(m, opt, gens, _reward, num_generations=G, C=C, per_device_train_batch_size=MB,
                         gradient_accumulation_steps=GA, n_steps=1, steps_per_generation=spg, eos_token_id=EOS,
                         capture=True)
    assert len(recs[0]["gens"]) == 2 and recs[0]["gens"][0]["old"] is None
    assert recs[0]["logps"].shape == (MB * GA, C)


def test_grpo_step_is_one_step_of_the_loop():
    """grpo_step (one generation, spg = rows / micro-batch) equals grpo_train's first step."""
    cfg = tiny_qwen2(128, 1)
    G, P, C, MB, GA = 4, 6, 10, 4, 2
    g = _gen(3, MB * GA, G, P, C, cfg.vocab_size)
    m1, o1 = _model(cfg)
    loss1, out1 = og.grpo_step(m1, o1, g["prompt_ids"], g["prompt_mask"], _reward, num_generations=G, C=C,
                               per_device_train_batch_size=MB, gradient_accumulation_steps=GA, eos_token_id=EOS,
                               completion_ids=g["completion_ids"], perm=g["perm"], capture=True)
    m2, o2 = _model(cfg)
    rec = og.grpo_train(m2, o2, [g], _reward, num_generations=G, C=C, per_device_train_batch_size=MB,
                        gradient_accumulation_steps=GA, n_steps=1, eos_token_id=EOS, capture=True)[0]
    assert loss1 == rec["loss"] and torch.equal(out1["logps"], rec["logps"])
    for (k, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), k


def _reward_none(cids, cmask):
    return [None if i % 3 == 0 else float(m.sum()) for i, m in enumerate(cmask)]


def test_knobs_mask_truncated_rewards_and_weights():
    """mask_truncated_completions (grpo_trainer.py:1829-1831) zeroes the rows without
    EOS after the lengths and the reward functions' ids were taken (:1821-1826);
    several reward functions are weighted and nan-summed (:1918), None -> NaN."""
    cfg = tiny_qwen2(128, 1)
    G, P, C, MB, GA = 4, 6, 10, 4, 2
    m, opt = _model(cfg)
    g = _gen(0, MB * GA, G, P, C, cfg.vocab_size)
    recs = og.grpo_train(m, opt, [g], [_reward, _reward_none], num_generations=G, C=C,
                         per_device_train_batch_size=MB, gradient_accumulation_steps=GA, n_steps=1,
                         eos_token_id=EOS, mask_truncated_completions=True, reward_weights=[1.0, 0.25],
                         scale_rewards=False, capture=True)
    sc = recs[0]["gens"][0]
    has_eos = (g["completion_ids"] == EOS).any(1)
    assert torch.equal(sc["cm"].sum(1) > 0, has_eos) and int(has_eos.sum()) == 1
    assert int(sc["lengths"][0]) == 6 and bool((sc["lengths"][1:] == C).all())  # lengths before the zeroing
    rpf = sc["rewards_per_func"]
    assert bool(rpf[0::3, 1].isnan().all()) and torch.equal(rpf[1::3, 1], torch.full_like(rpf[1::3, 1], float(C)))
    r = torch.nansum(rpf * torch.tensor([1.0, 0.25]), 1)
    torch.testing.assert_close(sc["rewards"].view(-1), r)
    adv = r - r.view(-1, G).mean(1).repeat_interleave(G)  # scale_rewards=False (:1929-1930)
    torch.testing.assert_close(sc["a"], adv)


def test_knobs_entropy_mask_and_clipping_defaults():
    """top_entropy_quantile 1.0 / delta None / epsilon_high None are the default loop;
    top_entropy_quantile q keeps about (1 - q) of each micro-batch's valid tokens; a
    delta above every ratio changes nothing."""
    cfg = tiny_qwen2(128, 1)
    G, P, C, MB, GA = 4, 6, 10, 4, 2
    g = _gen(2, MB * GA, G, P, C, cfg.vocab_size)

    def run(**kw):
        m, opt = _model(cfg)
        return og.grpo_train(m, opt, [g], _reward, num_generations=G, C=C, per_device_train_batch_size=MB,
                             gradient_accumulation_steps=GA, n_steps=2, num_iterations=2, eos_token_id=EOS,
                             capture=True, **kw)
    base = run()
    same = run(top_entropy_quantile=1.0, delta=1e9, epsilon_high=0.2)
    for a, b in zip(base, same):
        assert a["loss"] == b["loss"] and "entropy_mask" not in a and "entropy_mask" not in b
    q = run(top_entropy_quantile=0.25)
    em = q[0]["entropy_mask"]
    frac = em.float().sum() / (MB * GA * C - 4)  # row 0 of the rollout stops at its EOS (token 5)
    assert 0.2 <= float(frac) <= 0.35, float(frac)
    assert q[0]["loss"] != base[0]["loss"]
    clipped = run(delta=1.0001, epsilon=0.01)
    assert clipped[1]["loss"] != base[1]["loss"]
