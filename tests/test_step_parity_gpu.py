"""Step-level GRPO parity (-m gpu): GRPOTrainer optimizer steps against the CPU
restatement of the reference loop (oracle/grpo_step.py `grpo_train`, which
follows grpo_trainer.py:1411-1444 buffering / shuffle / split, :1812-1938
scoring, :1854-1869 old log-probs, :1871-1899 frozen reference, :2058-2175 loss,
and the Trainer's loss / GA, clip_grad_norm_ + torch AdamW).

Both sides start from the same weights and see the same prompts, the same
completion ids (the engine's own rollouts are handed to the oracle) and the
same shuffle permutations.

fp32 (reference-precision mode, `model_init_kwargs={"torch_dtype": "float32"}`:
fp32 parameters through the same flat-buffer model, HIP norm / RoPE / SiLU /
log-prob / loss / AdamW kernels, SDPA attention) against transformers fp32:
  * completion mask and advantages equal (1e-6);
  * per-token log-probs of every micro-batch within 1e-4;
  * the loss (sum of the GA micro-batch losses / GA) within 1e-4;
  * the pre-clip gradient norm within 1e-4 relative, each weight gradient
    within 1e-3 relative;
  * the post-step weights: each weight moves by at most lr, and both sides'
    moves agree to 1e-3 lr on all but a 1e-3 fraction of weights (those with
    |g| near eps, where the first AdamW step is ill-conditioned).

bf16 (the benched path: bf16 weights, csrc/attn.hip training attention, the
shared-prompt forward, the chunked lm-head log-prob, fp32 master AdamW)
against the reference's own bf16 computation (SURVEY.md §7 "exact" mode:
transformers bf16, bf16 logits / T, the bf16 branch of selective_log_softmax,
bf16 AdamW on the parameters).  A 1e-4 bound is not meaningful against bf16
outputs (one bf16 ulp of a log-prob near -12 is 0.0625), so the bound is
derived from bf16 rounding itself: the oracle also runs in fp32 on the same
(bf16-valued) weights, and delta_ref = |oracle_bf16 - oracle_fp32| measures
how far the reference's bf16 arithmetic sits from exact.  Two bf16
implementations of one function can each sit that far from it, in opposite
directions, so the product must satisfy
  * mask and advantages exactly (integer / fp32 arithmetic on equal inputs);
  * log-probs: max |product - oracle_bf16| <= 2 max(delta_ref) + 1 ulp(bf16)
    of the largest |log-prob| (the reference rounds its output to bf16, the
    product keeps fp32), and the mean <= 2 mean(delta_ref) + ulp/2;
  * the product at least as close to oracle_fp32 as the reference is:
    mean |product - oracle_fp32| <= 1.5 mean(delta_ref) + ulp/4;
  * loss: |product - oracle_bf16| <= 2 |oracle_bf16 - oracle_fp32| + 1e-3 |loss|;
  * with beta > 0, the step-1 KL is exactly 0 in every micro-batch (ref == policy,
    scored on the training pass's own rows and positions, as the reference's is);
  * gradients: relative error against oracle_fp32 within 2x the reference's
    own (|g_bf16 - g_fp32| / |g_fp32|) + 2^-8, per weight tensor.
Run at the Qwen2.5-0.5B width (H 896, I 4864, V 151936, 14:2 heads) with 2
layers, and in the fork's own configuration (examples/scripts/grpo_train.py:
494-503: num_iterations 2, importance_sampling_level "sequence", beta 0.1),
whose second optimizer step reuses the buffered rollouts against their old
log-probs, in both precisions.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

EOS, PAD = 1, 0


def _reward_oracle(cids, cmask):
    return [float(sum(r[m.bool()].tolist()) % 7) for r, m in zip(cids, cmask)]


def _reward_product(prompts=None, completions=None, completion_ids=None, **kw):
    # varies within every group at any vocabulary size (a count of distinct ids is
    # constant once V >> C: all-zero advantages would leave nothing to compare)
    return [float(sum(c) % 7) for c in completion_ids]


def _grads_by_name(model):
    """The flat gradient buffer viewed through the transformers parameter names."""
    saved = model.flat.clone()
    model.flat.copy_(model.grad)
    out = {k: v.detach().float().cpu().clone() for k, v in model.hf_state_dict().items()}
    model.flat.copy_(saved)
    return out


def _weights(model):
    return {k: v.detach().float().cpu().clone() for k, v in model.hf_state_dict().items()}


def product_run(cfg, dtype, n_steps, *, std, lr, G=4, P=12, C=24, MB=8, GA=2, seed=11, n_prompts=None,
                min_new_tokens=4, gen_extra=None, reward_funcs=None, **grpo_kw):
    """n_steps GRPOTrainer optimizer steps; captures every generation (its
    output and the shuffle permutation drawn after it), every training pass's
    log-probs, and the loss / grad norm / gradients / weights of every step."""
    from swh_trl_amd.engine import CausalLM
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer

    dev = torch.device("cuda:0")
    spg = grpo_kw.get("steps_per_generation") or GA
    if n_prompts is None:  # whole updates per epoch: enough generation batches for n_steps x GA micro-steps
        mu = grpo_kw.get("num_iterations", 1)
        n_prompts = MB * spg // G * max(1, -(-max(1, n_steps) * GA // (spg * mu)))
    g = torch.Generator().manual_seed(seed)
    ds = [{"prompt": None, "prompt_ids": torch.randint(2, cfg.vocab_size, (P,), generator=g).tolist()}
          for _ in range(n_prompts)]
    args = GRPOConfig(per_device_train_batch_size=MB, gradient_accumulation_steps=GA, num_generations=G,
                      max_prompt_length=P, max_completion_length=C, learning_rate=lr, max_steps=n_steps,
                      lr_scheduler_type="constant", seed=5, shuffle_dataset=False,
                      model_init_kwargs={"torch_dtype": "float32" if dtype == torch.float32 else "bfloat16"},
                      generation_kwargs={"eos_token_id": EOS, "pad_token_id": PAD, "min_new_tokens": min_new_tokens,
                                         **(gen_extra or {})},
                      **grpo_kw)
    model = CausalLM(cfg, dev, seed=3, init_std=std, dtype=dtype)
    tr = GRPOTrainer(model=model, reward_funcs=reward_funcs or _reward_product, args=args, train_dataset=ds)
    assert tr.model.dtype == dtype
    w0 = _weights(tr.model)
    cap = {"gens": [], "logps": [], "masks": [], "emasks": []}
    gen_fn = tr._generate_and_score_completions

    def gen_capture(examples):
        out = gen_fn(examples)
        rec = {k: v.detach().cpu().clone() for k, v in out.items()}
        n = rec["completion_ids"].shape[0]
        rec["perm"] = torch.randperm(n, generator=torch.Generator().set_state(tr._shuffle_gen.get_state()))
        cap["gens"].append(rec)
        return out

    lp_fn = tr._completion_logps

    def lp_capture(model_, batch, compute_entropy):
        lp, ent = lp_fn(model_, batch, compute_entropy)
        if compute_entropy:  # the training pass (the scoring passes run without entropy)
            cap["logps"].append(lp.detach().float().cpu().clone())
            cap["masks"].append(batch["completion_mask"].detach().cpu().clone())
        return lp, ent

    from swh_trl_amd import ops as _ops
    loss_fn = _ops.grpo_loss

    def loss_capture(logp, adv, cmask, **kw):  # the entropy mask the trainer hands the loss kernel
        if kw.get("entropy_mask") is not None:
            cap["emasks"].append(kw["entropy_mask"].detach().cpu().clone())
        return loss_fn(logp, adv, cmask, **kw)

    tr._generate_and_score_completions = gen_capture
    tr._completion_logps = lp_capture
    _ops.grpo_loss = loss_capture
    steps = []
    try:
        for _ in range(n_steps):
            steps.append(_product_step(tr, cap, spg))
    finally:
        _ops.grpo_loss = loss_fn
    hip_attn = tr.model._hip_attn
    eng = tr._engine
    engine = {"B": eng.B, "fused_sample": bool(getattr(eng, "fused", False) and eng._fused_sample()),
              "gen_kwargs": dict(tr.gen_kwargs), "temperature": tr.temperature}
    del tr, eng
    torch.cuda.empty_cache()
    return {"w0": w0, "gens": cap["gens"], "steps": steps, "hip_attn": hip_attn, "engine": engine,
            "geometry": dict(G=G, C=C, MB=MB, GA=GA)}


def _product_step(tr, cap, spg):
    """One optimizer step of the trainer and what the checks compare."""
    out = tr.training_step_group()
    torch.cuda.synchronize()
    # old-policy log-probs scored by the training pass itself (the policy had not stepped
    # since the generation) live in the buffered micro-batches: back to generation order
    for mb in tr._buffered_inputs or []:
        if "old_per_token_logps" in mb and "_row_index" in mb:
            for ri, row in zip(mb["_row_index"].tolist(), mb["old_per_token_logps"].detach().cpu()):
                g = cap["gens"][ri // mb["completion_ids"].shape[0] // spg]
                if "old_per_token_logps" not in g:
                    g["old_per_token_logps"] = torch.zeros(g["completion_ids"].shape)
                g["old_per_token_logps"][ri % g["completion_ids"].shape[0]] = row
    return {"loss": float(out["loss"]), "grad_norm": float(out["grad_norm"]),
            "grads": _grads_by_name(tr.model), "w": _weights(tr.model),
            "logps": cap["logps"][-1], "mask": cap["masks"][-1],
            "emask": cap["emasks"][-1] if cap["emasks"] else None,
            "seg_metrics": tr._metrics["train"]["_met"][-1].detach().cpu().clone()}


def oracle_run(cfg, w0, dtype, prod, n_steps, *, lr, beta=0.0, loss_type="bnpo", device="cpu", reward_fn=None,
               **grpo_kw):
    """The reference loop (oracle/grpo_step.py grpo_train) in `dtype` — on the host, or
    for the 8B width with torch's own device kernels (the same restatement; the host
    would take minutes) — from the product's initial weights, over its rollouts."""
    from oracle import grpo_step as og
    geo = prod["geometry"]
    hf = og.hf_from_config(cfg.to_dict(), seed=0, dtype=dtype).to(device)
    missing, unexpected = hf.load_state_dict({k: v.to(dtype) for k, v in w0.items()}, strict=False)
    assert not unexpected and not [k for k in missing if "rotary" not in k], (missing, unexpected)
    ref = None
    if beta:
        ref = og.hf_from_config(cfg.to_dict(), seed=0, dtype=dtype).to(device)
        ref.load_state_dict({k: v.to(dtype) for k, v in w0.items()}, strict=False)
    opt = torch.optim.AdamW(hf.parameters(), lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, foreach=False)
    gens = [{"prompt_ids": g["prompt_ids"], "prompt_mask": g["prompt_mask"].long(),
             "completion_ids": g["completion_ids"], "perm": g["perm"]} for g in prod["gens"]]
    recs = og.grpo_train(hf, opt, gens, reward_fn or _reward_oracle, num_generations=geo["G"], C=geo["C"],
                         per_device_train_batch_size=geo["MB"], gradient_accumulation_steps=geo["GA"],
                         n_steps=n_steps, eos_token_id=EOS, beta=beta, loss_type=loss_type, ref_model=ref,
                         capture=True, **grpo_kw)
    for r in recs:
        r["grads"] = {k: v.float() for k, v in r["grads"].items()}
    recs[0]["w_after"] = {k: p.detach().float().cpu().clone() for k, p in hf.named_parameters()}
    del hf, ref, opt
    if device != "cpu":
        torch.cuda.empty_cache()
    return recs


def _check_rollout_bookkeeping(prod, orc):
    for g, sc in zip(prod["gens"], orc[0]["gens"]):
        assert torch.equal(sc["cm"].int(), g["completion_mask"].int())
        torch.testing.assert_close(g["advantages"].float(), sc["a"].float(), rtol=0, atol=1e-6)
    for st in prod["steps"]:
        assert st["mask"].shape == st["logps"].shape


def _check_fp32(name, prod, orc, lr):
    _check_rollout_bookkeeping(prod, orc)
    for s, (st, o) in enumerate(zip(prod["steps"], orc)):
        m = st["mask"].bool()
        d_lp = (st["logps"] - o["logps"].float()).abs()[m]
        assert d_lp.max().item() <= 1e-4, (name, s, d_lp.max().item())
        assert abs(st["loss"] - o["loss"]) <= 1e-4 * max(1.0, abs(o["loss"])), (name, s, st["loss"], o["loss"])
        assert abs(st["grad_norm"] - o["grad_norm"]) <= 1e-4 * o["grad_norm"], (name, s, st["grad_norm"],
                                                                                 o["grad_norm"])
        for k, gr in o["grads"].items():
            rel = ((st["grads"][k] - gr).norm() / gr.norm().clamp_min(1e-20)).item()
            assert rel <= 1e-3, (name, s, k, rel)
    if len(prod["steps"]) != 1:  # later steps' gradients already pin the weights the earlier steps left
        return
    w0, w1, params = prod["w0"], prod["steps"][0]["w"], orc[0]["w_after"]
    frac_bad, total = 0.0, 0
    for k, w_after in w1.items():
        if k not in params:
            continue
        mv_p = w_after - w0[k]
        mv_o = params[k] - w0[k]
        assert mv_p.abs().max().item() <= lr * 1.001 + 1e-7, k
        diff = (mv_p - mv_o).abs()
        frac_bad += (diff > 1e-3 * lr).sum().item()
        total += diff.numel()
    assert frac_bad / total <= 1e-3, (name, frac_bad / total)


def _ulp_bf16(x: float) -> float:
    import math
    return 2.0 ** (math.floor(math.log2(max(abs(x), 1e-30))) - 7)


def _check_bf16(name, prod, orc_bf, orc_32, beta=0.0):
    """The bf16-rounding bounds of the module docstring; returns the measured figures."""
    _check_rollout_bookkeeping(prod, orc_bf)
    stats = []
    for s, (st, ob, o32) in enumerate(zip(prod["steps"], orc_bf, orc_32)):
        m = st["mask"].bool()
        lp_p, lp_b, lp_32 = st["logps"][m], ob["logps"].float()[m], o32["logps"].float()[m]
        d_ref = (lp_b - lp_32).abs()
        d_pb = (lp_p - lp_b).abs()
        d_p32 = (lp_p - lp_32).abs()
        ulp = _ulp_bf16(lp_b.abs().max().item())
        rec = {"step": s, "lp_max_ref": d_ref.max().item(), "lp_mean_ref": d_ref.mean().item(),
               "lp_max_prod_vs_bf16": d_pb.max().item(), "lp_mean_prod_vs_bf16": d_pb.mean().item(),
               "lp_mean_prod_vs_fp32": d_p32.mean().item(), "ulp": ulp,
               "loss": (st["loss"], ob["loss"], o32["loss"])}
        assert d_pb.max().item() <= 2 * d_ref.max().item() + ulp, (name, rec)
        assert d_pb.mean().item() <= 2 * d_ref.mean().item() + ulp / 2, (name, rec)
        assert d_p32.mean().item() <= 1.5 * d_ref.mean().item() + ulp / 4, (name, rec)
        loss_band = 2 * abs(ob["loss"] - o32["loss"]) + 1e-3 * abs(o32["loss"]) + 1e-6
        assert abs(st["loss"] - ob["loss"]) <= loss_band, (name, rec)
        if beta and s == 0:
            # ref == policy at step 1: the frozen-reference log-probs are scored on the training
            # pass's own layout, so the k3 KL is exactly 0 as in the reference (:2085-2089)
            rec["kl_sums_step1"] = st["seg_metrics"][:, 1].tolist()
            assert torch.all(st["seg_metrics"][:, 1] == 0), (name, rec)
        worst = []
        for k, g32 in o32["grads"].items():
            n32 = g32.norm().clamp_min(1e-20)
            rel_ref = ((ob["grads"][k] - g32).norm() / n32).item()
            rel_p = ((st["grads"][k] - g32).norm() / n32).item()
            worst.append((rel_p - 2 * rel_ref, k, rel_p, rel_ref))
            assert rel_p <= 2 * rel_ref + 2.0 ** -8, (name, s, k, rel_p, rel_ref)
        rec["grad_worst"] = max(worst)
        stats.append(rec)
    print(name, stats)
    return stats


def _cases():
    from swh_trl_amd.engine.config import DecoderConfig, tiny_qwen2
    real = DecoderConfig(num_hidden_layers=2)  # Qwen2.5-0.5B width, 2 layers
    return [("tiny", tiny_qwen2(1024, 2), 0.05, "bnpo", 0.0),
            ("tiny-grpo-beta", tiny_qwen2(1024, 2), 0.05, "grpo", 0.04),
            ("qwen2.5-0.5b-width", real, 0.02, "dr_grpo", 0.0)]


@pytest.mark.parametrize("name,cfg,std,loss_type,beta", _cases(), ids=[c[0] for c in _cases()])
def test_grpo_step_matches_oracle_step_fp32(name, cfg, std, loss_type, beta):
    lr = 1e-3
    prod = product_run(cfg, torch.float32, 1, std=std, lr=lr, beta=beta, loss_type=loss_type)
    assert not prod["hip_attn"]
    orc = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr, beta=beta, loss_type=loss_type)
    _check_fp32(name, prod, orc, lr)


def test_grpo_step_bf16_benched_path_matches_oracle():
    """The benched configuration's numerics (bf16, HIP training attention,
    shared-prompt forward, chunked lm-head log-prob) against the reference's
    bf16 step, at the Qwen2.5-0.5B width with 2 layers."""
    from swh_trl_amd.engine.config import DecoderConfig
    cfg = DecoderConfig(num_hidden_layers=2)
    lr = 1e-3
    prod = product_run(cfg, torch.bfloat16, 1, std=0.02, lr=lr)
    assert prod["hip_attn"]
    orc_bf = oracle_run(cfg, prod["w0"], torch.bfloat16, prod, 1, lr=lr)
    orc_32 = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr)
    _check_bf16("bf16-0.5b-width", prod, orc_bf, orc_32)


FORK = dict(num_iterations=2, importance_sampling_level="sequence", beta=0.1)


def test_fork_config_fp32_matches_oracle():
    """examples/scripts/grpo_train.py:494-503 (num_iterations 2, GSPO sequence-level
    importance weights, beta 0.1): GA is not a multiple of steps_per_generation x
    num_iterations, so the rollout is scored once more for old_per_token_logps
    (grpo_trainer.py:1854-1869) and the second optimizer step revisits the buffered
    micro-batches (:1425-1438) with the updated policy; fp32, two steps."""
    from swh_trl_amd.engine.config import tiny_qwen2
    cfg = tiny_qwen2(1024, 2)
    lr = 1e-3
    prod = product_run(cfg, torch.float32, 2, std=0.05, lr=lr, **FORK)
    orc = oracle_run(cfg, prod["w0"], torch.float32, prod, 2, lr=lr, **FORK)
    assert len(prod["gens"]) == 1 and "old_per_token_logps" in prod["gens"][0]
    torch.testing.assert_close(prod["gens"][0]["old_per_token_logps"].float()[prod["gens"][0]["completion_mask"].bool()],
                               orc[0]["gens"][0]["old"].float()[orc[0]["gens"][0]["cm"].bool()], rtol=0, atol=1e-4)
    _check_fp32("fork-fp32", prod, orc, lr)


def test_fork_config_bf16_matches_oracle():
    """The fork's configuration on the benched bf16 path (0.5B width, 2 layers), two
    optimizer steps over one buffered rollout, against the reference's bf16 loop."""
    from swh_trl_amd.engine.config import DecoderConfig
    cfg = DecoderConfig(num_hidden_layers=2)
    lr = 1e-3  # moves of several bf16 ulps: the second step sees a changed policy on both sides
    prod = product_run(cfg, torch.bfloat16, 2, std=0.02, lr=lr, **FORK)
    orc_bf = oracle_run(cfg, prod["w0"], torch.bfloat16, prod, 2, lr=lr, **FORK)
    orc_32 = oracle_run(cfg, prod["w0"], torch.float32, prod, 2, lr=lr, **FORK)
    _check_bf16("fork-bf16-0.5b-width", prod, orc_bf, orc_32, beta=FORK["beta"])


def test_steps_per_generation_below_ga_fp32_matches_oracle():
    """steps_per_generation 2 < GA 4: one optimizer step draws two generation batches
    (_prepare_inputs regenerates every spg micro-steps, :1425-1433) and trains on the
    micro-batches of both, the second rollout coming from the same (not yet updated)
    policy; against the oracle's loop."""
    from swh_trl_amd.engine.config import tiny_qwen2
    cfg = tiny_qwen2(1024, 2)
    lr = 1e-3
    prod = product_run(cfg, torch.float32, 1, std=0.05, lr=lr, MB=4, GA=4, steps_per_generation=2, loss_type="grpo")
    assert len(prod["gens"]) == 2
    orc = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr, steps_per_generation=2, loss_type="grpo")
    _check_fp32("spg<GA", prod, orc, lr)


def test_cfg5_llama8b_width_step_matches_oracle():
    """BASELINE.json config 5's architecture at full width (Llama-3-8B: H 4096, I 14336,
    V 128256, 32:8 heads x 128, untied head) with 2 layers: one bf16 GRPO step with
    beta 0.04 against a frozen reference copy (grpo_trainer.py:1871-1899), 64 rows x
    (32 + 128) = 10240 tokens in the fused training pass — the shapes at which two
    hipBLASLt persistent solutions on the compute and weight-gradient streams once
    deadlocked (engine/model.py `_main_gemm_fence`).  The rollout runs on
    the bandwidth-regime decode GEMMs (csrc/wide_gemm.hip).  Checked against the
    reference loop with the bf16-rounding bounds of this module."""
    from swh_trl_amd.engine.config import llama3_8b
    import dataclasses
    cfg = dataclasses.replace(llama3_8b(), num_hidden_layers=2)
    lr = 1e-3
    kw = dict(G=8, P=32, C=128, MB=16, GA=4, beta=0.04)
    prod = product_run(cfg, torch.bfloat16, 1, std=0.02, lr=lr, **kw)
    assert prod["hip_attn"]
    rows = prod["steps"][0]["mask"].shape[0]
    assert rows * (32 + 128) >= 10240
    orc_bf = oracle_run(cfg, prod["w0"], torch.bfloat16, prod, 1, lr=lr, beta=0.04, device="cuda:0")
    orc_32 = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr, beta=0.04, device="cuda:0")
    _check_bf16("cfg5-llama8b-width", prod, orc_bf, orc_32, beta=0.04)


def test_cfg5_llama8b_width_full_length_step_matches_oracle():
    """BASELINE.json config 5 at its own workload length (grpo_trainer.py:1793-1810,
    :1871-1899): Llama-3-8B width with 2 layers, 8 prompts x G 8 of P 256, every row
    decoding all 1024 completion tokens (min_new_tokens), beta 0.04 against a frozen
    reference.  The rollout runs the D 128 shared-prompt decode attention out to 1,280
    keys and 1023 graph-replayed decode steps of the wide GEMMs; the fused training
    pass is 8 x 256 + 64 x 1024 = 67,584 tokens.  One bf16 step against the
    reference loop (oracle on the device) with this module's bf16 bounds, and the
    step-1 KL exactly 0."""
    from swh_trl_amd.engine.config import llama3_8b
    import dataclasses
    cfg = dataclasses.replace(llama3_8b(), num_hidden_layers=2)
    lr = 1e-3
    kw = dict(G=8, P=256, C=1024, MB=16, GA=4, beta=0.04)
    prod = product_run(cfg, torch.bfloat16, 1, std=0.02, lr=lr, min_new_tokens=1024, **kw)
    g = prod["gens"][0]
    assert g["completion_ids"].shape == (64, 1024) and bool(g["completion_mask"].all())
    orc_bf = oracle_run(cfg, prod["w0"], torch.bfloat16, prod, 1, lr=lr, beta=0.04, device="cuda:0")
    orc_32 = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr, beta=0.04, device="cuda:0")
    _check_bf16("cfg5-llama8b-width-C1024", prod, orc_bf, orc_32, beta=0.04)


def test_early_stopped_rollout_width_matches_oracle_fp32():
    """A rollout in which every row emits EOS (vocabulary 16, near-uniform logits,
    96-token budget): the trainer keeps the longest row's width, as transformers
    generate returns it (grpo_trainer.py:1793-1810), and trains on it; the step
    still equals the oracle's, dr_grpo's constant normaliser (max_completion_length,
    :2134-2135) included."""
    from swh_trl_amd.engine.config import tiny_qwen2
    cfg = tiny_qwen2(16, 2)
    lr = 1e-3
    prod = product_run(cfg, torch.float32, 1, std=0.02, lr=lr, C=96, loss_type="dr_grpo")
    w = prod["gens"][0]["completion_ids"].shape[1]
    assert w < 96 and bool(prod["gens"][0]["completion_mask"][:, -1].any()), w
    orc = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr, loss_type="dr_grpo")
    _check_fp32("early-stop-width", prod, orc, lr)


def test_generation_kwargs_temperature_step_matches_oracle_fp32():
    """generation_kwargs on top of the config fields (grpo_trainer.py:995-1014): the
    rollout samples at generation_kwargs' T 0.7 / top-k 50, while the scoring and
    training passes divide by the config's temperature 1.0 (:1249), as the
    reference's do; one fp32 step against the oracle loop scoring at T 1.0."""
    from swh_trl_amd.engine.config import tiny_qwen2
    cfg = tiny_qwen2(1024, 2)
    lr = 1e-3
    prod = product_run(cfg, torch.float32, 1, std=0.05, lr=lr, gen_extra={"temperature": 0.7, "top_k": 50})
    assert prod["engine"]["gen_kwargs"]["temperature"] == 0.7 and prod["engine"]["gen_kwargs"]["top_k"] == 50
    assert prod["engine"]["temperature"] == 1.0
    orc = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr)
    _check_fp32("gen-kwargs-T0.7", prod, orc, lr)


BENCH_LAYOUT = dict(G=8, P=128, C=256, MB=16, GA=4)


def test_bench_layout_bf16_step_matches_oracle():
    """One bf16 GRPO step in exactly the benched workload's layout (bench.py:
    8 prompts x G 8 = 64 rows, P 128, C 256 with min_new_tokens = C, micro-batch
    16 x GA 4 fused into one training pass, beta 0) at the Qwen2.5-0.5B width with
    2 layers: the rollout runs the M = 64 decode tiles (xstream / fragment-order
    projections) and the fused lm-head sampler, the training pass the shared-prompt
    HIP forward of 8 x 128 + 64 x 256 tokens.  Against the reference loop
    (grpo_trainer.py:1500-2003, :2058-2175) in bf16 and fp32 with this module's
    bf16-rounding bounds (oracle on the device: 16 x 384 x 151936 fp32 logits per
    micro-batch)."""
    from swh_trl_amd.engine.config import DecoderConfig
    cfg = DecoderConfig(num_hidden_layers=2)
    lr = 1e-3
    prod = product_run(cfg, torch.bfloat16, 1, std=0.02, lr=lr, min_new_tokens=BENCH_LAYOUT["C"], **BENCH_LAYOUT)
    assert prod["hip_attn"] and prod["engine"]["B"] == 64 and prod["engine"]["fused_sample"], prod["engine"]
    g = prod["gens"][0]
    assert g["completion_ids"].shape == (64, 256) and bool(g["completion_mask"].all())
    assert prod["steps"][0]["mask"].shape == (64, 256)  # the four micro-batches in one fused pass
    orc_bf = oracle_run(cfg, prod["w0"], torch.bfloat16, prod, 1, lr=lr, device="cuda:0")
    orc_32 = oracle_run(cfg, prod["w0"], torch.float32, prod, 1, lr=lr, device="cuda:0")
    _check_bf16("bench-layout-0.5b-width", prod, orc_bf, orc_32)


# ---------------------------------------------------------------------------------------------
# The GRPO knobs the default configuration leaves off, through the trainer's own wiring
# (grpo_trainer.py:1829-1831 mask_truncated_completions, :1485-1487 None -> NaN, :1918 reward
# weights, :1929-1930 scale_rewards, :2079-2082 top_entropy_quantile, :2110-2118 epsilon_high
# and delta), two optimizer steps over one buffered rollout (num_iterations 2), so the second
# step's ratios leave 1 and the clipping bites.
# ---------------------------------------------------------------------------------------------

def _reward_len_product(prompts=None, completions=None, completion_ids=None, **kw):
    # the completion's length up to its first EOS: a truncated row counts its full width in the
    # reference (completion_ids_list is built before mask_truncated_completions, :1821-1831);
    # None for some rows (nansum over the weighted functions, :1918)
    return [None if sum(c) % 4 == 0 else float(len(c) % 5) for c in completion_ids]


def _reward_len_oracle(cids, cmask):
    out = []
    for r, m in zip(cids, cmask):
        c = r[m.bool()].tolist()
        out.append(None if sum(c) % 4 == 0 else float(len(c) % 5))
    return out


KNOBS = dict(num_iterations=2, top_entropy_quantile=0.7, delta=1.015, epsilon=0.008, epsilon_high=0.012,
             mask_truncated_completions=True, reward_weights=[1.0, 0.5], scale_rewards=False)


def _knob_runs(cfg, dtype, *, std, lr, device="cpu", **kw):
    prod = product_run(cfg, dtype, 2, std=std, lr=lr, reward_funcs=[_reward_product, _reward_len_product],
                       **KNOBS, **kw)
    orcs = []
    for od in ([torch.float32] if dtype == torch.float32 else [torch.bfloat16, torch.float32]):
        orcs.append(oracle_run(cfg, prod["w0"], od, prod, 2, lr=lr, device=device,
                               reward_fn=[_reward_oracle, _reward_len_oracle], **KNOBS))
    g = prod["gens"][0]
    cm, has_eos = g["completion_mask"], (g["completion_ids"] == EOS).any(1)
    # the knobs are exercised: some rows truncated (all-zero mask), some not; some rewards None
    assert bool((cm.sum(1) == 0).any()) and bool((cm.sum(1) > 0).any()), cm.sum(1)
    assert torch.equal(cm.sum(1) > 0, has_eos)
    rpf = orcs[0][0]["gens"][0]["rewards_per_func"]
    assert bool(rpf[:, 1].isnan().any()) and bool((~rpf[:, 1].isnan()).any())
    # the entropy mask keeps roughly the top 30 % of each micro-batch's valid tokens
    for st in prod["steps"]:
        assert st["emask"] is not None and st["emask"].shape == st["mask"].shape
        assert not bool((st["emask"] & ~st["mask"].bool()).any())
    # clipping happened in the second step (ratios moved past 1 -/+ epsilon)
    clip = prod["steps"][1]["seg_metrics"][:, 3:6].sum().item()
    return prod, orcs, clip


def test_grpo_knobs_fp32_matches_oracle():
    """Every knob on, fp32 (vocabulary 16 so about a third of the rows stop at EOS): masks,
    advantages, the entropy masks, log-probs, losses, gradients and weights against the
    oracle loop within the fp32 bounds of _check_fp32."""
    from swh_trl_amd.engine.config import tiny_qwen2
    cfg = tiny_qwen2(16, 2)
    lr = 3e-3
    prod, (orc,), clip = _knob_runs(cfg, torch.float32, std=0.05, lr=lr)
    assert clip > 0, clip
    for s, (st, o) in enumerate(zip(prod["steps"], orc)):
        assert torch.equal(st["emask"], o["entropy_mask"].bool()), (s, (st["emask"] ^ o["entropy_mask"]).sum())
    _check_fp32("knobs-fp32", prod, orc, lr)


def test_grpo_knobs_bf16_benched_path_matches_oracle():
    """Every knob on the benched bf16 path (Qwen2.5-0.5B width, 2 layers, HIP training
    attention, shared-prompt forward, fused lm-head log-prob) with a 64-token vocabulary
    so that rows stop at EOS.  The entropy quantile runs on bf16 entropies as the
    reference's does; ties at the threshold can still differ from the reference's bf16
    arithmetic, so the entropy-masked set is bounded by the reference's own bf16-vs-fp32
    difference: |M_prod xor M_bf16| <= 2 |M_bf16 xor M_fp32| + 1 % of the valid tokens.
    Log-probs, losses and gradients within _check_bf16's bounds."""
    import dataclasses
    from swh_trl_amd.engine.config import DecoderConfig
    cfg = dataclasses.replace(DecoderConfig(num_hidden_layers=2), vocab_size=64)
    lr = 2e-3
    prod, (orc_bf, orc_32), clip = _knob_runs(cfg, torch.bfloat16, std=0.02, lr=lr, device="cuda:0")
    assert prod["hip_attn"]
    print("knobs-bf16 clip sums step 2:", clip)
    for s, (st, ob, o32) in enumerate(zip(prod["steps"], orc_bf, orc_32)):
        valid = int(st["mask"].sum())
        d_pb = int((st["emask"] ^ ob["entropy_mask"].bool()).sum())
        d_ref = int((ob["entropy_mask"].bool() ^ o32["entropy_mask"].bool()).sum())
        print(f"step {s}: entropy-mask differences product/bf16 {d_pb}, bf16/fp32 {d_ref}, valid {valid}")
        assert d_pb <= 2 * d_ref + 0.01 * valid, (s, d_pb, d_ref, valid)
    _check_bf16("knobs-bf16-0.5b-width", prod, orc_bf, orc_32)


def test_epoch_end_partial_accumulation_fp32_matches_oracle():
    """An epoch of 2 generation batches x steps_per_generation 2 = 4 micro-batches
    under GA 3: the Trainer's updates are 3, then the epoch's remainder 1 (its loss /
    1, transformers Trainer._run_epoch `remainder` and current_gradient_accumulation_
    steps), then the next epoch's 3.  Three fp32 optimizer steps against the oracle
    loop with micro_steps_per_epoch 4; GA 3 is not a multiple of spg, so rollouts are
    scored for old log-probs where an update boundary falls inside one (:1854-1869)."""
    from swh_trl_amd.engine.config import tiny_qwen2
    cfg = tiny_qwen2(1024, 2)
    lr = 1e-3
    kw = dict(MB=8, GA=3, steps_per_generation=2, n_prompts=8)
    prod = product_run(cfg, torch.float32, 3, std=0.05, lr=lr, **kw)
    assert len(prod["gens"]) == 4  # two epochs' worth of generation batches
    assert [st["logps"].shape[0] for st in prod["steps"]] == [24, 8, 24]
    orc = oracle_run(cfg, prod["w0"], torch.float32, prod, 3, lr=lr, steps_per_generation=2,
                     micro_steps_per_epoch=4)
    assert len(orc[0]["losses"]) == 3 and len(orc[1]["losses"]) == 1 and len(orc[2]["losses"]) == 3
    _check_fp32("epoch-remainder", prod, orc, lr)
