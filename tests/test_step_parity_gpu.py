"""Step-level GRPO parity (-m gpu): one GRPOTrainer optimizer step against the
CPU restatement of the reference step (oracle/grpo_step.py, which follows
grpo_trainer.py:1500-2003 rollout scoring, :1411-1444 shuffle/split,
:2058-2175 loss, and the Trainer's clip_grad_norm_ + torch AdamW).

Both sides start from the same weights and see the same prompts, the same
completion ids (the engine's own rollout is handed to the oracle) and the same
shuffle permutation.  The product runs in its fp32 reference-precision mode
(`model_init_kwargs={"torch_dtype": "float32"}`: fp32 parameters through the
same flat-buffer model, HIP norm / RoPE / SiLU / log-prob / loss / AdamW
kernels; the rollout reads a bf16 copy), the oracle is transformers Qwen2 in
fp32 on the host.  Checked:
  * completion mask and advantages equal (1e-6);
  * per-token log-probs of every micro-batch within 1e-4;
  * the loss (sum of the GA micro-batch losses / GA) within 1e-4;
  * the pre-clip gradient norm within 1e-4 relative, each weight gradient
    within 1e-3 relative;
  * the post-step weights: the AdamW step moves each weight by at most lr
    (first step: lr * g / (|g| + eps)), and both sides' moves agree to 1e-3 lr
    on all but a 1e-3 fraction of weights (those with |g| near eps, where the
    first AdamW step is ill-conditioned).
Run at the tiny Qwen2 preset and at the real Qwen2.5-0.5B width (H 896,
I 4864, V 151936, 14:2 heads) with 2 layers.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

EOS, PAD = 1, 0


def _reward_oracle(cids, cmask):
    return [float(len(set(r[m.bool()].tolist())) % 5) for r, m in zip(cids, cmask)]


def _reward_product(prompts=None, completions=None, completion_ids=None, **kw):
    return [float(len(set(c)) % 5) for c in completion_ids]


def _grads_by_name(model):
    """The flat gradient buffer viewed through the transformers parameter names."""
    saved = model.flat.clone()
    model.flat.copy_(model.grad)
    out = {k: v.detach().float().cpu().clone() for k, v in model.hf_state_dict().items()}
    model.flat.copy_(saved)
    return out


def _cases():
    from swh_trl_amd.engine.config import DecoderConfig, tiny_qwen2
    real = DecoderConfig(num_hidden_layers=2)  # Qwen2.5-0.5B width, 2 layers
    return [("tiny", tiny_qwen2(1024, 2), 0.05, "bnpo", 0.0),
            ("tiny-grpo-beta", tiny_qwen2(1024, 2), 0.05, "grpo", 0.04),
            ("qwen2.5-0.5b-width", real, 0.02, "dr_grpo", 0.0)]


@pytest.mark.parametrize("name,cfg,std,loss_type,beta", _cases(), ids=[c[0] for c in _cases()])
def test_grpo_step_matches_oracle_step_fp32(name, cfg, std, loss_type, beta):
    from oracle import grpo_step as og
    from swh_trl_amd.engine import CausalLM
    from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer

    dev = torch.device("cuda:0")
    G, P, C, MB, GA = 4, 12, 24, 8, 2
    n_prompts = MB * GA // G
    g = torch.Generator().manual_seed(11)
    ds = [{"prompt": None, "prompt_ids": torch.randint(2, cfg.vocab_size, (P,), generator=g).tolist()}
          for _ in range(n_prompts)]
    lr = 1e-3
    args = GRPOConfig(per_device_train_batch_size=MB, gradient_accumulation_steps=GA, num_generations=G,
                      max_prompt_length=P, max_completion_length=C, learning_rate=lr, beta=beta, loss_type=loss_type,
                      max_steps=1, lr_scheduler_type="constant", seed=5, shuffle_dataset=False,
                      model_init_kwargs={"torch_dtype": "float32"},
                      generation_kwargs={"eos_token_id": EOS, "pad_token_id": PAD, "min_new_tokens": 4})
    model = CausalLM(cfg, dev, seed=3, init_std=std, dtype=torch.float32)
    tr = GRPOTrainer(model=model, reward_funcs=_reward_product, args=args, train_dataset=ds)
    assert tr.model.dtype == torch.float32 and not tr.model._hip_attn
    w0 = {k: v.detach().float().cpu().clone() for k, v in tr.model.hf_state_dict().items()}

    captured = {}
    gen_fn = tr._generate_and_score_completions

    def gen_capture(examples):
        out = gen_fn(examples)
        captured["gen"] = {k: v.detach().clone() for k, v in out.items()}
        captured["shuffle_state"] = tr._shuffle_gen.get_state()
        return out

    lp_fn = tr._completion_logps

    def lp_capture(model_, batch, compute_entropy):
        lp, ent = lp_fn(model_, batch, compute_entropy)
        if compute_entropy:  # the training pass (the scoring passes run without entropy)
            captured["logps"] = lp.detach().float().cpu().clone()
            captured["mask"] = batch["completion_mask"].detach().cpu().clone()
        return lp, ent

    tr._generate_and_score_completions = gen_capture
    tr._completion_logps = lp_capture
    out = tr.training_step_group()
    torch.cuda.synchronize()
    loss = float(out["loss"])
    norm = float(out["grad_norm"])
    grads = _grads_by_name(tr.model)
    w1 = {k: v.detach().float().cpu().clone() for k, v in tr.model.hf_state_dict().items()}

    gen = {k: v.cpu() for k, v in captured["gen"].items()}
    n = gen["completion_ids"].shape[0]
    perm = torch.randperm(n, generator=torch.Generator().set_state(captured["shuffle_state"]))

    # the oracle: transformers Qwen2 fp32 on the host, same weights / completions / permutation
    hf = og.hf_qwen2_from_config(cfg.to_dict(), seed=0, dtype=torch.float32)
    missing, unexpected = hf.load_state_dict(w0, strict=False)
    assert not unexpected and not [k for k in missing if "rotary" not in k], (missing, unexpected)
    ref = None
    if beta:
        ref = og.hf_qwen2_from_config(cfg.to_dict(), seed=0, dtype=torch.float32)
        ref.load_state_dict(w0, strict=False)
    opt = torch.optim.AdamW(hf.parameters(), lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, foreach=False)
    oloss, inter = og.grpo_step(hf, opt, gen["prompt_ids"], gen["prompt_mask"].long(), _reward_oracle,
                                num_generations=G, C=C, per_device_train_batch_size=MB,
                                gradient_accumulation_steps=GA, eos_token_id=EOS, pad_token_id=PAD, beta=beta,
                                loss_type=loss_type, completion_ids=gen["completion_ids"], perm=perm,
                                ref_model=ref, capture=True)

    # rollout bookkeeping and advantages
    assert torch.equal(inter["completion_mask"].int(), gen["completion_mask"].int())
    torch.testing.assert_close(gen["advantages"].float(), inter["advantages"].float(), rtol=0, atol=1e-6)
    # per-token log-probs (the fused pass holds the GA micro-batches in permuted order)
    m = captured["mask"].bool()
    assert torch.equal(m, gen["completion_mask"][perm].bool())
    d_lp = (captured["logps"] - inter["logps"].float()).abs()[m]
    assert d_lp.max().item() <= 1e-4, (name, d_lp.max().item())
    # loss and gradient norm
    assert abs(loss - oloss) <= 1e-4 * max(1.0, abs(oloss)), (name, loss, oloss)
    assert abs(norm - inter["grad_norm"]) <= 1e-4 * inter["grad_norm"], (name, norm, inter["grad_norm"])
    # every weight gradient
    og_grads = inter["grads"]
    for k, gr in og_grads.items():
        gm = grads[k]
        rel = ((gm - gr).norm() / gr.norm().clamp_min(1e-20)).item()
        assert rel <= 1e-3, (name, k, rel)
    # post-step weights
    params = dict(hf.named_parameters())
    frac_bad, worst = 0.0, 0.0
    total = 0
    for k, w_after in w1.items():
        if k not in params:
            continue
        mv_p = w_after - w0[k]
        mv_o = params[k].detach().float() - w0[k]
        assert mv_p.abs().max().item() <= lr * 1.001 + 1e-7, k
        diff = (mv_p - mv_o).abs()
        frac_bad += (diff > 1e-3 * lr).sum().item()
        total += diff.numel()
        worst = max(worst, diff.max().item())
    assert frac_bad / total <= 1e-3, (name, frac_bad / total, worst)
