"""Parity of every HIP kernel with the CPU oracle (run on an MI355X: -m gpu).

Tolerances are written per test: bit-exact for integer/index work, the
reference's own tolerances (1e-5, tests/test_utils.py:540-640) for fp32, and
stated bounds for bf16 results.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from oracle import hf_sampling, trl_ref

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ops():
    from swh_trl_amd import ops as _ops
    from swh_trl_amd import _lib
    _lib.load()
    return _ops


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _gen(seed):
    return torch.Generator().manual_seed(seed)


# --------------------------------------------------------------------------- logp / entropy
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_logp_entropy_reference_shape(ops, dev, dtype):
    g = _gen(0)
    logits = torch.randn(4, 32, 1024, generator=g).to(dtype)
    ids = torch.randint(0, 1024, (4, 32), generator=g)
    logp, ent, lse = ops.logp_entropy(logits.to(dev), ids.to(dev))
    ref_lp = trl_ref.selective_log_softmax(logits.double(), ids)
    ref_ent = trl_ref.entropy_from_logits(logits.double())
    torch.testing.assert_close(logp.cpu().double(), ref_lp, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ent.cpu().double(), ref_ent, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(lse.cpu().double(), torch.logsumexp(logits.double(), -1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("V", [1024, 1000, 128, 100, 33, 7, 1])
def test_selective_log_softmax_lowp_bit_exact(ops, dev, dtype, V):
    """Reference test_utils.py:540-558: bf16/fp16 outputs equal
    gather(log_softmax) bit for bit (its shape is 4 x 32 x 1024; narrower rows
    exercise the sub-wave lane groups of torch's warp softmax)."""
    g = _gen(1)
    logits = (torch.randn(4, 32, V, generator=g) * 3).to(dtype).to(dev)
    ids = torch.randint(0, V, (4, 32), generator=g).to(dev)
    got = ops.selective_log_softmax(logits, ids)
    exp = torch.gather(logits.log_softmax(-1), -1, ids.unsqueeze(-1)).squeeze(-1)
    assert got.dtype == dtype
    assert torch.equal(got, exp), (got != exp).sum().item()
    # a strided [R, T, V] view (rows of a longer buffer) as the trainer slices logits
    wide = torch.randn(4, 33, V, generator=g).to(dtype).to(dev)[:, 1:]
    got = ops.selective_log_softmax(wide, ids)
    assert torch.equal(got, torch.gather(wide.log_softmax(-1), -1, ids.unsqueeze(-1)).squeeze(-1))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_selective_log_softmax_lowp_wide_rows(ops, dev, dtype):
    """Rows wider than 1024 (torch's block softmax, whose reduction order is not
    restated): the fused fp32 kernel rounded once; >= 99.9% bit-identical, the
    rest 1 ulp."""
    g = _gen(1)
    logits = torch.randn(4, 32, 4096, generator=g).to(dtype).to(dev)
    ids = torch.randint(0, 4096, (4, 32), generator=g).to(dev)
    got = ops.selective_log_softmax(logits, ids)
    exp = torch.gather(logits.log_softmax(-1), -1, ids.unsqueeze(-1)).squeeze(-1)
    assert got.dtype == dtype
    same = (got == exp).float().mean().item()
    assert same >= 0.999, same
    ulp = (got.float() - exp.float()).abs() / exp.float().abs().clamp_min(1e-3)
    assert (ulp <= 2 ** -7).all()


@pytest.mark.parametrize("chunk", [1, 16])
def test_entropy_reference_shape(ops, dev, chunk):
    g = _gen(2)
    logits = torch.randn(64, 384, 768, generator=g)
    got = ops.entropy_from_logits(logits.to(dev), chunk_size=chunk)
    p = logits.double().softmax(-1)
    exp = -(p * p.log()).sum(-1)
    torch.testing.assert_close(got.cpu().double(), exp, rtol=1e-5, atol=1e-5)


def test_logp_full_vocab_strided_temperature(ops, dev):
    """Qwen2.5 vocabulary, the [:, -C-1:-1] slice of a [B, L, V] bf16 tensor, T=0.7."""
    g = _gen(3)
    V, B, L, Cc = 151936, 2, 70, 64
    logits = (torch.randn(B, L, V, generator=g) * 3).to(torch.bfloat16)
    ids = torch.randint(0, V, (B, Cc), generator=g)
    sl = logits.to(dev)[:, -Cc - 1:-1]
    logp, ent, lse = ops.logp_entropy(sl, ids.to(dev), temperature=0.7)
    z = logits[:, -Cc - 1:-1].double() / 0.7
    torch.testing.assert_close(logp.cpu().double(), trl_ref.selective_log_softmax(z, ids), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ent.cpu().double(), trl_ref.entropy_from_logits(z), rtol=1e-5, atol=2e-5)


def test_logp_round_scaled_matches_bf16_division(ops, dev):
    g = _gen(4)
    logits = (torch.randn(3, 16, 4096, generator=g) * 2).to(torch.bfloat16)
    ids = torch.randint(0, 4096, (3, 16), generator=g)
    logp, _, _ = ops.logp_entropy(logits.to(dev), ids.to(dev), temperature=0.9, round_scaled=True)
    z = (logits / 0.9)  # bf16 division, as the reference's `logits / self.temperature`
    torch.testing.assert_close(logp.cpu().double(), trl_ref.selective_log_softmax(z.double(), ids),
                               rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_logp_backward_matches_autograd(ops, dev, dtype):
    g = _gen(5)
    logits = torch.randn(2, 24, 3000, generator=g).to(dtype)
    ids = torch.randint(0, 3000, (2, 24), generator=g)
    w = torch.randn(2, 24, generator=g)
    x = logits.double().requires_grad_(True)
    (trl_ref.selective_log_softmax(x / 0.8, ids) * w).sum().backward()
    xl = logits.to(dev).requires_grad_(True)
    lp, _ = ops.logp_entropy_autograd(xl, ids.to(dev), temperature=0.8)
    (lp * w.to(dev)).sum().backward()
    tol = 1e-6 if dtype == torch.float32 else 4e-3
    torch.testing.assert_close(xl.grad.cpu().double(), x.grad, rtol=tol, atol=tol)


def test_logp_edge_rows(ops, dev):
    """-inf entries (masked vocab), a one-hot row, V not a multiple of 8, unaligned base."""
    V = 1003
    logits = torch.randn(4, V + 1)
    logits[0, 5:] = float("-inf")
    logits[1, :] = -1e4
    logits[1, 7] = 10.0
    base = logits.to(dev)[:, 1:]  # 4-byte misaligned rows
    ids = torch.tensor([3, 7, 0, V - 1])
    logp, ent, _ = ops.logp_entropy(base, ids.to(dev))
    ref = trl_ref.selective_log_softmax(logits[:, 1:].double(), ids)
    torch.testing.assert_close(logp.cpu().double(), ref, rtol=1e-5, atol=1e-5)
    lp = torch.log_softmax(logits[:, 1:].double(), -1)
    ent_ref = -(lp.exp() * lp.nan_to_num(neginf=0.0)).sum(-1)
    torch.testing.assert_close(ent.cpu().double(), ent_ref, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------- completion mask / advantages
def test_completion_mask_mock_kat(ops, dev):
    import json
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        k = json.load(f)["mock_completion_masks"]
    ids = torch.tensor(k["completion_ids"], device=dev)
    m, lengths, has = ops.completion_mask(ids, k["eos"])
    assert m.cpu().tolist() == k["expected_mask"]
    assert lengths.cpu().tolist() == [8, 4, 8]
    assert has.cpu().tolist() == [0, 1, 1]
    mt, _, _ = ops.completion_mask(ids, k["eos"], mask_truncated=True)
    assert mt.cpu().tolist() == k["expected_mask_truncated"]


def test_completion_mask_random(ops, dev):
    g = _gen(6)
    ids = torch.randint(0, 20, (64, 256), generator=g)
    m, lengths, has = ops.completion_mask(ids.to(dev), [3, 17], mask_truncated=True)
    em, el, _ = trl_ref.completion_mask_from_eos(torch.where(ids == 17, 3, ids), 3, mask_truncated=True)
    assert torch.equal(m.cpu(), em)
    assert torch.equal(lengths.cpu().long(), el)


@pytest.mark.parametrize("scale", [True, False])
def test_group_advantage(ops, dev, scale):
    g = _gen(7)
    rpf = torch.rand(64, 3, generator=g)
    rpf[5, 1] = float("nan")
    rpf[8:16] = 0.25  # zero-std group
    w = torch.tensor([1.0, 0.5, 2.0])
    adv, rew, gm, gs, zs = ops.group_advantages(rpf.to(dev), w.to(dev), 8, scale)
    eadv, erew, egm, egs, ezs = trl_ref.group_advantages(rpf.double(), w.double(), 8, scale)
    torch.testing.assert_close(rew.cpu().double(), erew, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(gm.cpu().double(), egm, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(gs.cpu().double(), egs, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(adv.cpu().double(), eadv, rtol=1e-4, atol=1e-5)
    assert torch.equal(zs.cpu(), ezs)


# --------------------------------------------------------------------------- GRPO loss
CONFIGS = [
    dict(loss_type="bnpo", importance_sampling_level="token", beta=0.0, old=False),
    dict(loss_type="bnpo", importance_sampling_level="token", beta=0.04, old=True),
    dict(loss_type="grpo", importance_sampling_level="token", beta=0.1, old=True, delta=1.3),
    dict(loss_type="dr_grpo", importance_sampling_level="token", beta=0.0, old=True, eh=0.28),
    dict(loss_type="bnpo", importance_sampling_level="sequence", beta=0.1, old=True),
    dict(loss_type="grpo", importance_sampling_level="sequence", beta=0.0, old=False),
    dict(loss_type="bnpo", importance_sampling_level="token", beta=0.0, old=True, emask=True),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
def test_grpo_loss_and_grad(ops, dev, cfg):
    g = _gen(8)
    R, T = 16, 256
    lp = -torch.rand(R, T, generator=g, dtype=torch.float64) * 4
    old = (lp + 0.3 * torch.randn(R, T, generator=g, dtype=torch.float64)) if cfg["old"] else None
    ref = lp + 0.2 * torch.randn(R, T, generator=g, dtype=torch.float64)
    adv = torch.randn(R, generator=g, dtype=torch.float64)
    adv[3] = 0.0
    lens = torch.randint(1, T + 1, (R,), generator=g)
    lens[0] = 0
    mask = (torch.arange(T).view(1, -1) < lens.view(-1, 1)).int()
    ent = torch.rand(R, T, generator=g, dtype=torch.float64)
    em = (torch.rand(R, T, generator=g) > 0.5) if cfg.get("emask") else None
    kw = dict(beta=cfg["beta"], epsilon_low=0.2, epsilon_high=cfg.get("eh", 0.2), delta=cfg.get("delta"),
              loss_type=cfg["loss_type"], importance_sampling_level=cfg["importance_sampling_level"],
              max_completion_length=T)
    x = lp.clone().requires_grad_(True)
    eloss, emet = trl_ref.grpo_loss(x, adv, mask, old, ref, em, ent, **kw)
    eloss.backward()
    loss, dlogp, met = ops.grpo_loss_fwd_bwd(lp.to(dev), adv.to(dev), mask.to(dev), old_per_token_logps=
                                             None if old is None else old.to(dev), ref_per_token_logps=ref.to(dev),
                                             entropy_mask=None if em is None else em.to(dev), entropies=ent.to(dev),
                                             **kw)
    torch.testing.assert_close(loss.cpu().double()[0], eloss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dlogp.cpu().double(), x.grad, rtol=1e-5, atol=1e-7)
    met = met.cpu().double()
    tok = met[0].clamp(min=1.0)
    if cfg["importance_sampling_level"] == "token":
        assert met[3].item() / tok.item() == pytest.approx(emet["clip_ratio/low_mean"], abs=1e-6)
        assert met[5].item() / tok.item() == pytest.approx(emet["clip_ratio/region_mean"], abs=1e-6)
    else:
        assert met[3].item() / R == pytest.approx(emet["clip_ratio/low_mean"], abs=1e-6)
    if cfg["beta"]:
        assert met[1].item() / tok.item() == pytest.approx(emet["kl"], rel=1e-5)
    assert met[2].item() / tok.item() == pytest.approx(emet["entropy"], rel=1e-5)


def test_grpo_loss_segments_equal_separate_microbatches(ops, dev):
    """GA micro-batches fused into one kernel call == per-micro-batch losses / GA."""
    g = _gen(9)
    R, T, GA = 16, 64, 4
    lp = -torch.rand(R, T, generator=g) * 3
    adv = torch.randn(R, generator=g)
    mask = (torch.rand(R, T, generator=g) > 0.3).int()
    seg = torch.arange(R) // (R // GA)
    scale = torch.full((R,), 1.0 / GA)
    loss, dl, _ = ops.grpo_loss_fwd_bwd(lp.to(dev), adv.to(dev), mask.to(dev), row_scale=scale.to(dev),
                                        segments=seg.to(dev), num_segments=GA)
    tot, grads = 0.0, []
    for i in range(GA):
        sl = slice(i * R // GA, (i + 1) * R // GA)
        l_i, d_i, _ = ops.grpo_loss_fwd_bwd(lp[sl].to(dev), adv[sl].to(dev), mask[sl].to(dev))
        tot += l_i.item() / GA
        grads.append(d_i.cpu() / GA)
    assert loss.item() == pytest.approx(tot, rel=1e-5, abs=1e-7)
    torch.testing.assert_close(dl.cpu(), torch.cat(grads), rtol=1e-5, atol=1e-8)


# --------------------------------------------------------------------------- PPO pieces
def test_masked_whiten(ops, dev):
    g = _gen(10)
    v = torch.randn(8, 53, generator=g)
    m = torch.rand(8, 53, generator=g) > 0.3
    for shift in (True, False):
        out = ops.masked_whiten(v.to(dev), m.to(dev), shift_mean=shift)
        assert isinstance(out, torch.Tensor) and out.shape == v.shape
        exp = trl_ref.masked_whiten(v.double(), m.double(), shift_mean=shift)
        torch.testing.assert_close(out.cpu().double(), exp, rtol=1e-5, atol=1e-5)
    for unbiased in (True, False):
        torch.testing.assert_close(ops.masked_var(v.to(dev), m.to(dev), unbiased).cpu().double(),
                                   trl_ref.masked_var(v.double(), m.double(), unbiased), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ops.masked_mean(v.to(dev), m.to(dev)).cpu().double(),
                               trl_ref.masked_mean(v.double(), m.double()), rtol=1e-5, atol=1e-6)
    # core.py:57-62: an all-zero mask raises in masked_var(unbiased) and so in masked_whiten
    with pytest.raises(ValueError, match="sum of the mask is zero"):
        ops.masked_whiten(v.to(dev), torch.zeros_like(m).to(dev))
    with pytest.raises(ValueError, match="sum of the mask is zero"):
        ops.masked_var(v.to(dev), torch.zeros_like(m).to(dev))
    # core.py:51-56 without the correction: one unmasked element has variance 0, none is 0 / 0
    one = torch.zeros_like(m)
    one[3, 7] = True
    assert float(ops.masked_var(v.to(dev), one.to(dev), unbiased=False)) == 0.0
    assert float(trl_ref.masked_var(v.double(), one.double(), unbiased=False)) == 0.0
    assert torch.isnan(ops.masked_var(v.to(dev), torch.zeros_like(m).to(dev), unbiased=False))


@pytest.mark.parametrize("stop,est,pen", [(3, "k1", None), (3, "k3", 1.0), (None, "k1", 0.5)])
def test_ppo_rollout_postprocess_matches_oracle(ops, dev, stop, est, pen):
    """swh_ppo_truncate + swh_ppo_rewards against the oracle's restatement of
    ppo_trainer.py:478-516 (truncate_response, first_true_indices, masks,
    INVALID_LOGPROB, value masking, missing-EOS penalty, k1/k3 KL, the score
    scatter): stop at t = 0, no stop token, a row already full of pads."""
    g = _gen(40)
    B, T, PAD, EOS = 9, 23, 0, 3
    resp = torch.randint(4, 50, (B, T), generator=g)
    resp[0, 0] = 3
    resp[1, 7] = 3
    resp[2, 22] = 3
    resp[3, 5] = 3
    resp[3, 9] = 3
    resp[4, :] = PAD
    resp[5, 11] = PAD  # a pad token generated before any stop
    lp = -torch.rand(B, T, generator=g) * 3
    ref = lp + 0.1 * torch.randn(B, T, generator=g)
    vals = torch.randn(B, T, generator=g).to(torch.bfloat16)
    sc = torch.randn(B, generator=g).to(torch.bfloat16)
    post, seq = ops.ppo_truncate(resp.to(dev), stop, PAD)
    exp_post = trl_ref.truncate_response(stop, PAD, resp) if stop is not None else resp
    exp_seq = trl_ref.first_true_indices(exp_post == PAD) - 1
    assert torch.equal(post.cpu(), exp_post) and torch.equal(seq.cpu(), exp_seq)
    r = ops.ppo_rewards(post, seq, lp.to(dev), ref.to(dev), vals.to(dev), sc.to(dev), eos_token_id=EOS,
                        missing_eos_penalty=pen, kl_coef=0.05, kl_estimator=est)
    idx = torch.arange(T).repeat(B, 1)
    pm, pm1 = idx > exp_seq[:, None], idx > (exp_seq + 1)[:, None]
    assert torch.equal(r["padding_mask"].cpu(), pm) and torch.equal(r["padding_mask_p1"].cpu(), pm1)
    elp = lp.masked_fill(pm, trl_ref.INVALID_LOGPROB)
    eref = ref.masked_fill(pm, trl_ref.INVALID_LOGPROB)
    esc = sc.clone()
    if pen is not None:
        esc[~torch.any(exp_post == EOS, -1)] -= pen
    rew, kl, nsr = trl_ref.ppo_rewards(elp, eref, esc, exp_seq, 0.05, est)
    assert torch.equal(r["logprobs"].cpu(), elp) and torch.equal(r["ref_logprobs"].cpu(), eref)
    assert torch.equal(r["values"].cpu(), vals.masked_fill(pm1, 0)) and torch.equal(r["scores"].cpu(), esc)
    for k, e in (("kl", kl), ("non_score_reward", nsr), ("rewards", rew)):
        torch.testing.assert_close(r[k].cpu(), e, rtol=1e-6, atol=1e-6, msg=k)


def test_gae(ops, dev):
    g = _gen(11)
    r = torch.randn(64, 53, generator=g)
    v = torch.randn(64, 53, generator=g)
    adv, ret = ops.gae(r.to(dev), v.to(dev), 1.0, 0.95)
    eadv, eret = trl_ref.gae(r.double(), v.double(), 1.0, 0.95)
    torch.testing.assert_close(adv.cpu().double(), eadv, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ret.cpu().double(), eret, rtol=1e-5, atol=1e-5)


def test_ppo_loss(ops, dev):
    g = _gen(12)
    B, T = 16, 53
    new = -torch.rand(B, T, generator=g, dtype=torch.float64) * 3
    old = new + 0.3 * torch.randn(B, T, generator=g, dtype=torch.float64)
    adv = torch.randn(B, T, generator=g, dtype=torch.float64)
    vp = torch.randn(B, T, generator=g, dtype=torch.float64)
    ov = vp + 0.3 * torch.randn(B, T, generator=g, dtype=torch.float64)
    ret = torch.randn(B, T, generator=g, dtype=torch.float64)
    sl = torch.randint(0, T, (B,), generator=g)
    idx = torch.arange(T).view(1, -1)
    pm, pm1 = idx > sl.view(-1, 1), idx > (sl + 1).view(-1, 1)
    new = new.masked_fill(pm, trl_ref.INVALID_LOGPROB)
    vp = vp.masked_fill(pm1, 0.0)
    x, y = new.clone().requires_grad_(True), vp.clone().requires_grad_(True)
    eloss, _, _, est = trl_ref.ppo_losses(x, old, adv, y, ov, ret, pm, pm1, 0.2, 0.2, 0.1)
    eloss.backward()
    loss, dnl, dvp, st = ops.ppo_loss_fwd_bwd(new.to(dev), old.to(dev), adv.to(dev), vp.to(dev), ov.to(dev),
                                              ret.to(dev), pm.to(dev), pm1.to(dev), 0.2, 0.2, 0.1)
    torch.testing.assert_close(loss.cpu().double()[0], eloss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dnl.cpu().double(), x.grad.masked_fill(pm, 0), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(dvp.cpu().double(), y.grad.masked_fill(pm1, 0), rtol=1e-5, atol=1e-7)
    assert st[2].item() == pytest.approx(est["pg_clipfrac"], abs=1e-6)
    assert st[4].item() == pytest.approx(est["approxkl"], rel=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_value_head(ops, dev, dtype):
    g = _gen(13)
    h = torch.randn(4, 33, 896, generator=g).to(dtype)
    w = torch.randn(896, generator=g) * 0.02
    b = torch.randn(1, generator=g)
    got = ops.value_head(h.to(dev), w.to(dev), b.to(dev))
    exp = trl_ref.value_head(h.double(), w.double(), b.double())
    torch.testing.assert_close(got.cpu().double(), exp, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------- optimizer
def test_adamw_and_clip(dev):
    from swh_trl_amd import optim
    g = _gen(14)
    N = 1_000_003
    p0 = torch.randn(N, generator=g, dtype=torch.float64)
    st = optim.FlatAdamW(N, dev, lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    st.master.copy_(p0.float().to(dev))
    q, m, v = p0.float().double(), torch.zeros(N, dtype=torch.float64), torch.zeros(N, dtype=torch.float64)
    model = torch.empty(N, dtype=torch.bfloat16, device=dev)
    for step in range(1, 4):
        gr = (torch.randn(N, generator=g) * 0.01).to(torch.bfloat16)
        norm = st.step(gr.to(dev), model_out=model)
        total, coef = trl_ref.clip_coef([gr.double()], 1.0)
        assert norm.item() == pytest.approx(float(total), rel=1e-5)
        q, m, v = trl_ref.adamw_step(q, gr.double() * coef, m, v, step, 1e-3, weight_decay=0.01)
    torch.testing.assert_close(st.master.cpu().double(), q, rtol=1e-5, atol=1e-6)
    assert torch.equal(model.cpu(), st.master.cpu().to(torch.bfloat16))


def test_adamw_no_decay_ranges_and_fp32_model(dev):
    """weight_decay > 0 with the transformers Trainer grouping (no decay on
    biases / norm weights: CausalLM.no_decay_ranges) against torch AdamW with
    two param groups; the fp32 model copy is the master itself."""
    from swh_trl_amd import optim
    from swh_trl_amd.engine import CausalLM, tiny_qwen2
    m = CausalLM(tiny_qwen2(512, 2), "cpu", seed=1, dtype=torch.float32, trainable=False)
    N = m.numel
    nd = m.no_decay_ranges()
    assert len(nd) == 2 * 3 + 1  # per layer: ln_in, qkv_b, ln_post; the final norm
    decay = torch.ones(N, dtype=torch.bool)
    for s, e in nd:
        decay[s:e] = False
    g = _gen(15)
    p0 = torch.randn(N, generator=g)
    st = optim.FlatAdamW(N, dev, lr=1e-2, weight_decay=0.1, max_grad_norm=None, no_decay_ranges=nd)
    st.master.copy_(p0.to(dev))
    model = torch.empty(N, dtype=torch.float32, device=dev)
    pd = torch.nn.Parameter(p0[decay].double().clone())
    pn = torch.nn.Parameter(p0[~decay].double().clone())
    opt = torch.optim.AdamW([{"params": [pd], "weight_decay": 0.1}, {"params": [pn], "weight_decay": 0.0}],
                            lr=1e-2, foreach=False)
    for _ in range(3):
        gr = torch.randn(N, generator=g) * 0.1
        st.step(gr.to(dev), model_out=model)
        pd.grad, pn.grad = gr[decay].double(), gr[~decay].double()
        opt.step()
    out = st.master.cpu().double()
    torch.testing.assert_close(out[decay], pd.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out[~decay], pn.detach(), rtol=1e-5, atol=1e-6)
    assert torch.equal(model.cpu(), st.master.cpu())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_backward_deterministic(dev, dtype):
    """swh_embedding_bwd: the per-id sums of dy rows folded into the gradient
    table (fp64 reference: g + sum), with long runs of one id (pads) across
    many 32-row pieces, ids outside the table skipped, and bit-identical
    results on every call (no atomics)."""
    from swh_trl_amd.engine.model import embedding_backward
    g = _gen(16)
    V, H, N = 300, 896, 5000
    ids = torch.randint(0, V, (N,), generator=g)
    ids[1000:3000] = 7                      # a 2000-row run (pad tokens after EOS)
    ids[::97] = 5
    dy = (torch.randn(N, H, generator=g) * 0.1).to(dtype)
    g0 = (torch.randn(V, H, generator=g) * 0.01).to(dtype)
    exp = g0.double().index_add(0, ids, dy.double())
    outs = []
    for _ in range(3):
        gt = g0.to(dev)
        embedding_backward(ids.view(50, 100).to(dev), dy.view(50, 100, H).to(dev), gt)
        outs.append(gt.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(outs[0].double(), exp, rtol=tol, atol=tol * 0.1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_token_split_weight_gradient_fold(dev, dtype):
    """engine/model.py _accumulate_dw at a token count that takes the split
    path (S token ranges as one batched GEMM, swh_dw_reduce folding the S
    partials into the gradient view): gw + dy^T x against fp64, plus the bias
    column sums; the result is identical on every call."""
    from swh_trl_amd.engine.model import _accumulate_dw, _dw_split, dw_sync
    g = _gen(17)
    T, N, K = 16384 + 40, 896, 1152
    assert _dw_split(T, N * K) > 1
    dy = (torch.randn(T, N, generator=g) * 0.05).to(dtype)
    x = (torch.randn(T, K, generator=g) * 0.05).to(dtype)
    g0 = (torch.randn(N, K, generator=g) * 0.01).to(dtype)
    b0 = torch.zeros(N, dtype=dtype)
    exp = g0.double() + dy.double().t() @ x.double()
    outs = []
    for _ in range(2):
        gw, gb = g0.to(dev), b0.to(dev)
        _accumulate_dw(gw, gb, dy.to(dev), x.to(dev))
        dw_sync(dev)
        torch.cuda.synchronize()
        outs.append(gw.cpu())
    assert torch.equal(outs[0], outs[1])
    rel = ((outs[0].double() - exp).norm() / exp.norm()).item()
    assert rel < (3e-3 if dtype == torch.bfloat16 else 1e-5), rel
    torch.testing.assert_close(gb.cpu().double(), dy.double().sum(0), rtol=2e-2, atol=2e-2)
    gb2 = b0.to(dev)
    _accumulate_dw(g0.to(dev), gb2, dy.to(dev), x.to(dev))
    dw_sync(dev)
    assert torch.equal(gb2.cpu(), gb.cpu())  # the bias column sums are deterministic too


# --------------------------------------------------------------------------- sampler
def _oracle_lib():
    so = os.path.join(ROOT, "oracle", "_build", "libswh_oracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return ctypes.CDLL(so)


def _uniforms(lib, seed, offset, row, V):
    buf = (ctypes.c_float * V)()
    lib.swh_ref_row_uniforms(ctypes.c_uint64(seed), ctypes.c_uint64(offset), ctypes.c_int64(row),
                             ctypes.c_int64(V), buf)
    return torch.from_numpy(np.frombuffer(buf, dtype=np.float32).copy())


def _run_sampler(ops, dev, logits, params, seed=7, offset=11, step=0, seen=None, finished=None, C=4,
                 scores=False):
    B, V = logits.shape
    rng = torch.tensor([seed, offset], dtype=torch.int64, device=dev)
    stp = torch.tensor([step], dtype=torch.int32, device=dev)
    fin = finished.to(dev).int() if finished is not None else torch.zeros(B, dtype=torch.int32, device=dev)
    out = torch.full((B, C), -1, dtype=torch.int64, device=dev)
    cur = torch.empty(B, dtype=torch.int64, device=dev)
    olp = torch.zeros(B, C, dtype=torch.float32, device=dev)
    sc = torch.empty(B, V, dtype=torch.float32, device=dev) if scores else None
    ops.sample_step(logits.to(dev), params, rng, stp, fin, out, cur, seen, olp, sc)
    return out[:, step].cpu(), fin.cpu(), olp[:, step].cpu(), (sc.cpu() if scores else None), cur.cpu()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sampler_greedy_is_argmax(ops, dev, dtype):
    g = _gen(15)
    logits = torch.randn(64, 151936, generator=g).to(dtype)
    logits[0, 100] = logits[0, 200] = 50.0  # tie -> first index (torch.argmax)
    tok, _, _, _, cur = _run_sampler(ops, dev, logits, ops.make_sample_params(greedy=True))
    assert torch.equal(tok, logits.float().argmax(-1))
    assert torch.equal(cur, tok)


@pytest.mark.parametrize("case", ["plain", "temp", "topk", "topp", "minp", "all", "rep"])
def test_sampler_matches_oracle_draw(ops, dev, case):
    """Same logits, same Philox stream: the device pick equals the oracle's
    Gumbel-max pick on the oracle-processed scores (float64)."""
    g = _gen(16)
    B, V = 8, 32000
    logits = torch.randn(B, V, generator=g) * 2  # fp32: no ties at the thresholds
    kw = dict(plain={}, temp=dict(temperature=0.7), topk=dict(top_k=50), topp=dict(top_p=0.9),
              minp=dict(min_p=0.05), all=dict(temperature=0.8, top_k=200, top_p=0.8, min_p=0.02),
              rep=dict(repetition_penalty=1.3, top_p=0.95))[case]
    seen = None
    seen_mask = None
    if case == "rep":
        prev = torch.randint(0, V, (B, 40), generator=g)
        seen = torch.zeros(B, (V + 31) // 32, dtype=torch.int32, device=dev)
        ops.seen_init(prev.to(dev), None, V, seen)
        seen_mask = torch.zeros(B, V, dtype=torch.bool).scatter_(1, prev, True)
    params = ops.make_sample_params(**kw)
    tok, _, lp, sc, _ = _run_sampler(ops, dev, logits, params, seen=seen, scores=True)
    proc = hf_sampling.process_scores(logits, seen=seen_mask, rep_penalty=kw.get("repetition_penalty", 1.0),
                                      t=kw.get("temperature", 1.0), k=kw.get("top_k"), p=kw.get("top_p", 1.0),
                                      mp=kw.get("min_p"))
    kept_dev, kept_ref = torch.isfinite(sc), torch.isfinite(proc)
    assert torch.equal(kept_dev, kept_ref), (kept_dev ^ kept_ref).sum()
    torch.testing.assert_close(sc[kept_ref], proc[kept_ref], rtol=0, atol=0)
    lib = _oracle_lib()
    u = torch.stack([_uniforms(lib, 7, 11, b, V) for b in range(B)])
    exp = hf_sampling.gumbel_pick(proc, u)
    assert torch.equal(tok, exp)
    ref_lp = torch.log_softmax(proc.double(), -1).gather(1, exp.view(-1, 1)).squeeze(1)
    torch.testing.assert_close(lp.double(), ref_lp, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kw", [dict(top_p=0.9), dict(top_k=100), dict(top_p=0.8, min_p=0.05)])
def test_sampler_bf16_ties(ops, dev, kw):
    """bf16 logits have many equal values: at a threshold the device keeps the
    whole tie group while transformers' sort keeps an arbitrary part of it.
    Bound: device kept set == oracle kept set + (part of) the tie group at the
    oracle's smallest kept value."""
    g = _gen(21)
    logits = (torch.randn(8, 32000, generator=g) * 2).to(torch.bfloat16)
    _, _, _, sc, _ = _run_sampler(ops, dev, logits, ops.make_sample_params(**kw), scores=True)
    proc = hf_sampling.process_scores(logits, k=kw.get("top_k"), p=kw.get("top_p", 1.0), mp=kw.get("min_p"))
    kd, kr = torch.isfinite(sc), torch.isfinite(proc)
    assert not (kr & ~kd).any()
    for b in range(8):
        extra = kd[b] & ~kr[b]
        if extra.any():
            assert (logits[b][extra].float() == logits[b][kr[b]].float().min()).all()


@pytest.mark.parametrize("kw", [dict(top_p=0.9), dict(top_p=0.8, top_k=500, min_p=0.01), dict(top_k=100)])
def test_filtered_sampler_is_run_to_run_deterministic(ops, dev, kw):
    """The filtered path's radix-select histograms sum top-p weights in 2^-40
    fixed point (integer LDS atomics): the draw and its log-prob are the same
    bits in every run.  (Float LDS atomics summed the weights in arrival order:
    a top-p generation differed between runs of the same seed.)  bf16 logits
    with many ties at the threshold, 64 rows x 151936, 12 launches."""
    g = _gen(31)
    logits = (torch.randn(64, 151936, generator=g) * 3).to(torch.bfloat16).to(dev)
    params = ops.make_sample_params(**kw)
    ref = None
    for _ in range(12):
        tok, _, lp, _, _ = _run_sampler(ops, dev, logits, params, seed=5, offset=2)
        if ref is None:
            ref = (tok, lp)
        assert torch.equal(tok, ref[0]) and torch.equal(lp, ref[1])


@pytest.mark.parametrize("kw", [dict(top_p=0.9), dict(top_p=0.5, temperature=0.7), dict(top_k=50),
                                dict(top_k=1000, temperature=1.3), dict(top_p=0.8, min_p=0.05),
                                dict(top_p=0.95, min_new_tokens=3), dict(top_k=151936)])
@pytest.mark.parametrize("B,V,scale", [(64, 151936, 3.0), (8, 32000, 0.5), (5, 4096, 8.0)])
def test_filtered_bf16_path_equals_general_path(ops, dev, kw, B, V, scale):
    """bf16 logits with one top-k or top-p threshold take the 16-bit-key radix path
    (csrc/sampler.hip launch_filtered16: 2 digits over the bf16 bits, the per-row
    selects in the next pass's prologue); the same values as fp32 logits take the
    general 3-digit path over the fp32 scores.  Kept sets (ties at the threshold
    included), draws and processed scores are identical, the log-probs agree to
    fp32 summation order; EOS suppression (min_new_tokens) and a top-k that keeps
    everything included."""
    g = _gen(45)
    logits = (torch.randn(B, V, generator=g) * scale).to(torch.bfloat16)
    params = ops.make_sample_params(eos_token_ids=[3], **kw)
    t16, _, lp16, sc16, _ = _run_sampler(ops, dev, logits, params, scores=True)
    t32, _, lp32, sc32, _ = _run_sampler(ops, dev, logits.float(), params, scores=True)
    assert torch.equal(torch.isfinite(sc16), torch.isfinite(sc32))
    assert torch.equal(sc16, sc32)
    assert torch.equal(t16, t32)
    torch.testing.assert_close(lp16, lp32, rtol=1e-6, atol=1e-6)
    # the log-probs against float64 over the kept set (the device sums run in fp32)
    kept = torch.isfinite(sc32)
    z = torch.where(kept, sc32.double(), torch.tensor(float("-inf"), dtype=torch.float64))
    exact = z.gather(1, t32.view(-1, 1)).squeeze(1) - torch.logsumexp(z, 1)
    torch.testing.assert_close(lp16.double(), exact, rtol=2e-6, atol=2e-6)
    # without the scores output (the rollout's call) the draws and log-probs are the same
    t16n, _, lp16n, _, _ = _run_sampler(ops, dev, logits, params)
    assert torch.equal(t16n, t16) and torch.equal(lp16n, lp16)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kw", [dict(), dict(temperature=0.7), dict(top_p=0.99)])
def test_sampler_gumbel_near_one_uniform_does_not_win(ops, dev, dtype, kw):
    """A uniform within a few 2^-24 of 1 made -log(-log u) = +inf in fp32 (v_log_f32
    returns 0 there), so that element won whatever its logit — about 1 % of the rows of
    a 151936-wide step.  Rows whose stream holds such a uniform get a -30 logit at that
    column and +10 at another: the draw must take the +10 column (the float64 Gumbel-max
    of the oracle does), and its log-prob stays finite."""
    lib = _oracle_lib()
    V, seed, offset = 151936, 7, 11
    rows, cols = [], []
    for b in range(256):
        u = _uniforms(lib, seed, offset, b, V)
        j = int(u.argmax())
        if float(u[j]) >= 1.0 - 4.0 / 16777216.0:
            rows.append(b)
            cols.append(j)
    assert rows, "no near-one uniform in 256 rows (expected ~4)"
    B = max(rows) + 1
    logits = torch.zeros(B, V)
    win = torch.zeros(B, dtype=torch.int64)
    for b, j in zip(rows, cols):
        logits[b, j] = -30.0
        win[b] = (j + 1) % V
        logits[b, win[b]] = 40.0
    tok, _, lp, _, _ = _run_sampler(ops, dev, logits.to(dtype), ops.make_sample_params(**kw), seed=seed, offset=offset)
    for b, j in zip(rows, cols):
        assert int(tok[b]) != j, (b, j)
        assert int(tok[b]) == int(win[b]), (b, int(tok[b]))
    assert bool(torch.isfinite(lp[rows]).all())


def test_sampler_distribution_chi2(ops, dev):
    """Empirical frequencies over 4096 independent draws match softmax(z)."""
    V, N = 16, 4096
    z = torch.linspace(-2, 2, V)
    logits = z.repeat(N, 1)
    tok, _, _, _, _ = _run_sampler(ops, dev, logits, ops.make_sample_params(), seed=123, offset=0)
    counts = torch.bincount(tok, minlength=V).double()
    p = torch.softmax(z.double(), 0)
    chi2 = (((counts - N * p) ** 2) / (N * p)).sum().item()
    assert chi2 < 45.0  # df=15, p ~ 1e-4


def test_sampler_bookkeeping(ops, dev):
    """Finished rows emit pad; EOS finishes a row; min_new_tokens suppresses EOS."""
    V = 64
    logits = torch.full((3, V), -10.0)
    logits[:, 5] = 10.0  # EOS strongly preferred
    fin = torch.tensor([1, 0, 0])
    params = ops.make_sample_params(greedy=True, pad_token_id=9, eos_token_ids=[5])
    tok, f, _, _, _ = _run_sampler(ops, dev, logits, params, finished=fin)
    assert tok.tolist() == [9, 5, 5] and f.tolist() == [1, 1, 1]
    params = ops.make_sample_params(greedy=True, pad_token_id=9, eos_token_ids=[5], min_new_tokens=3)
    tok, f, _, _, _ = _run_sampler(ops, dev, logits, params, step=1)
    assert 5 not in tok.tolist() and f.tolist() == [0, 0, 0]


# --------------------------------------------------------------------------- decoder kernels
def test_rmsnorm_matches_hf_bf16(ops, dev):
    from swh_trl_amd import nn_ops
    g = _gen(17)
    x = torch.randn(37, 896, generator=g).to(torch.bfloat16).to(dev)
    r = torch.randn(37, 896, generator=g).to(torch.bfloat16).to(dev)
    w = (1 + 0.1 * torch.randn(896, generator=g)).to(torch.bfloat16).to(dev)
    y, s = nn_ops.rmsnorm_residual(x, r, w, 1e-6)
    s_ref = r + x
    hs = s_ref.float()
    hs = hs * torch.rsqrt(hs.pow(2).mean(-1, keepdim=True) + 1e-6)
    y_ref = w * hs.to(torch.bfloat16)
    assert torch.equal(s, s_ref)
    diff = (y.float() - y_ref.float()).abs()
    assert (diff <= y_ref.float().abs() * 2 ** -7 + 1e-6).all()
    assert (y == y_ref).float().mean() > 0.99


def test_rmsnorm_backward(ops, dev):
    from swh_trl_amd import nn_ops
    g = _gen(18)
    x = torch.randn(130, 896, generator=g).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(896, generator=g)).to(torch.bfloat16)
    dy = torch.randn(130, 896, generator=g).to(torch.bfloat16)
    xd, wd = x.to(dev).requires_grad_(True), w.to(dev).requires_grad_(True)
    y = nn_ops.RMSNormFn.apply(xd, wd, 1e-6)
    y.backward(dy.to(dev))
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    yr = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6))
    yr.backward(dy.double())
    torch.testing.assert_close(xd.grad.cpu().double(), xr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(wd.grad.cpu().double(), wr.grad, rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("rows", [6144, 77])
def test_rmsnorm_backward_dres_and_dw_accumulation(ops, dev, rows):
    """engine/model.py _norm_backward: dx + the residual branch's gradient in one
    pass, the weight gradient summed from the per-block partials (swh_rmsnorm_dw_accum)
    and added to an existing bf16 gradient; rows = one training micro-batch and a ragged count."""
    from swh_trl_amd.engine.model import _norm_backward, dw_sync
    g = _gen(21)
    H = 896
    x = torch.randn(rows, H, generator=g).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16)
    dy = torch.randn(rows, H, generator=g).to(torch.bfloat16)
    dres = torch.randn(rows, H, generator=g).to(torch.bfloat16)
    gw0 = torch.randn(H, generator=g).to(torch.bfloat16)
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1) + 1e-6)
    gw = gw0.to(dev)
    dx = _norm_backward(x.to(dev), w.to(dev), rstd.to(dev), dy.to(dev), dres.to(dev), gw)
    dw_sync(dev)  # the fold runs on the weight-gradient side stream
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    yr = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6))
    yr.backward(dy.double())
    torch.testing.assert_close(dx.cpu().double(), xr.grad + dres.double(), rtol=2e-2, atol=3e-2)
    # dW = sum over rows of dy * bf16(x * rstd) (Qwen2RMSNorm's rounding point, as the
    # forward computes it), then two bf16 roundings (the summed partial, the accumulated view)
    xhat = (xf * rstd[:, None]).to(torch.bfloat16).double()
    dw = (dy.double() * xhat).sum(0)
    ref_gw = gw0.double() + dw
    err = (gw.cpu().double() - ref_gw).abs()
    bound = 2.0 ** -7 * (dw.abs() + gw0.double().abs()) + 1e-2
    assert (err <= bound).all(), (err.max().item(), (err / bound).max().item())


def test_fold_norm_ragged_jobs(ops, dev):
    """swh_fold_norm over jobs whose row counts are not multiples of the kernel's
    8-row chunks (chunks straddle jobs) and of different widths: bit-identical to
    torch's bf16 W * w for every job."""
    from swh_trl_amd._lib import call
    g = _gen(31)
    shapes = [(5, 16), (13, 896), (3, 24), (1, 8), (40, 64)]
    ws = [torch.randn(r, c, generator=g).to(torch.bfloat16).to(dev) for r, c in shapes]
    nws = [(1 + 0.2 * torch.randn(c, generator=g)).to(torch.bfloat16).to(dev) for _, c in shapes]
    outs = [torch.zeros_like(w) for w in ws]
    tab, row0 = [], 0
    for w, nw, o in zip(ws, nws, outs):
        tab += [w.data_ptr(), nw.data_ptr(), o.data_ptr(), w.shape[0], w.shape[1], row0]
        row0 += w.shape[0]
    t = torch.tensor(tab, dtype=torch.int64).to(dev)
    call("swh_fold_norm", t.data_ptr(), len(shapes), row0, ops._stream())
    torch.cuda.synchronize()
    for w, nw, o in zip(ws, nws, outs):
        assert torch.equal(o, w * nw)


def test_degenerate_inputs(ops, dev):
    """Edge cases the reference defines: zero rows (empty batches from a
    completion-less rank), an all-zero mask (core.py:59 raises), groups with
    identical rewards (std 0: advantage 0 and is_std_zero, grpo_trainer.py:1921-1930),
    and an all-masked completion in the loss (bnpo clamps the token count at 1)."""
    V = 1000
    lg = torch.empty(0, 7, V, device=dev, dtype=torch.bfloat16)
    ix = torch.empty(0, 7, device=dev, dtype=torch.int64)
    assert ops.selective_log_softmax(lg, ix).shape == (0, 7)
    assert ops.entropy_from_logits(torch.empty(0, V, device=dev)).shape == (0,)
    with pytest.raises(ValueError):
        ops.masked_whiten(torch.randn(4, 3, device=dev), torch.zeros(4, 3, device=dev))
    # constant rewards within each group of 4: mean = the constant, std 0, advantage 0
    rpf = torch.tensor([[2.0], [2.0], [2.0], [2.0], [1.0], [3.0], [1.0], [3.0]], device=dev)
    adv, rew, gm, gs, zs = ops.group_advantages(rpf, torch.ones(1, device=dev), 4, True)
    assert zs.tolist() == [True, False]
    assert torch.equal(adv[:4].cpu(), torch.zeros(4))
    ref = (rpf[4:, 0] - rpf[4:, 0].mean()) / (rpf[4:, 0].std() + 1e-4)
    torch.testing.assert_close(adv[4:], ref, rtol=1e-6, atol=1e-6)
    # every completion token masked: bnpo loss = 0 / clamp(0, 1) = 0 and a zero gradient
    lp = torch.randn(2, 5, device=dev)
    loss, dlp, _ = ops.grpo_loss_fwd_bwd(lp, torch.tensor([1.0, -1.0], device=dev),
                                         torch.zeros(2, 5, device=dev, dtype=torch.int32), loss_type="bnpo",
                                         max_completion_length=5)
    assert float(loss.reshape(-1)[0]) == 0.0 and torch.count_nonzero(dlp) == 0


def test_silu_mul(ops, dev):
    from swh_trl_amd import nn_ops
    g = _gen(19)
    gu = torch.randn(33, 2 * 4864, generator=g).to(torch.bfloat16).to(dev).requires_grad_(True)
    out = nn_ops.SiluMulFn.apply(gu)
    gt, ut = gu.detach()[:, :4864], gu.detach()[:, 4864:]
    ref = torch.nn.functional.silu(gt) * ut
    assert torch.equal(out, ref)
    dout = torch.randn_like(out)
    out.backward(dout)
    gg = gu.detach().double().requires_grad_(True)
    rr = torch.nn.functional.silu(gg[:, :4864]) * gg[:, 4864:]
    rr.backward(dout.double())
    torch.testing.assert_close(gu.grad.double(), gg.grad, rtol=2e-2, atol=2e-2)


def _rope_tables(D, max_pos, theta, dev):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.int64).float() / D))
    pos = torch.arange(max_pos).float()
    fr = torch.outer(pos, inv)
    return fr.cos().to(torch.bfloat16).float().to(dev), fr.sin().to(torch.bfloat16).float().to(dev)


@pytest.mark.parametrize("B,L,Hq,Hkv,D,left_pad", [(3, 37, 14, 2, 64, False), (2, 50, 4, 4, 128, True),
                                                   (1, 1, 2, 1, 32, False)])
def test_qkv_rope_matches_torch_rotate_half(ops, dev, B, L, Hq, Hkv, D, left_pad):
    """Fused split + RoPE vs the torch bf16 ops it replaces (transformers'
    apply_rotary_pos_emb on q/k slices of the packed projection), forward and
    autograd backward: bit-exact."""
    from swh_trl_amd import nn_ops
    from swh_trl_amd.engine.model import _apply_rope
    g = _gen(23)
    W = (Hq + 2 * Hkv) * D
    qkv = torch.randn(B, L, W, generator=g).to(torch.bfloat16).to(dev)
    pos = torch.arange(L).expand(B, L).clone()
    if left_pad:  # left-padded prompts: positions = cumsum(mask) - 1, negative on pads
        pos = pos - torch.randint(0, L // 2, (B, 1), generator=g)
    pos = pos.to(dev)
    cos_t, sin_t = _rope_tables(D, L + 4, 1e6, dev)
    dq = torch.randn(B, Hq, L, D, generator=g).to(torch.bfloat16).to(dev)
    dk = torch.randn(B, Hkv, L, D, generator=g).to(torch.bfloat16).to(dev)
    dv = torch.randn(B, Hkv, L, D, generator=g).to(torch.bfloat16).to(dev)

    a = qkv.clone().requires_grad_(True)
    q, k, v = nn_ops.QKVRopeFn.apply(a, pos, cos_t, sin_t, Hq, Hkv, D)
    assert q.is_contiguous() and k.is_contiguous() and v.is_contiguous()
    torch.autograd.backward((q, k, v), (dq, dk, dv))

    b = qkv.clone().requires_grad_(True)
    pc = pos.clamp(min=0)
    cos = torch.cat([cos_t[pc], cos_t[pc]], -1).to(torch.bfloat16).unsqueeze(1)
    sin = torch.cat([sin_t[pc], sin_t[pc]], -1).to(torch.bfloat16).unsqueeze(1)
    qr = _apply_rope(b[..., :Hq * D].view(B, L, Hq, D).transpose(1, 2), cos, sin)
    kr = _apply_rope(b[..., Hq * D:(Hq + Hkv) * D].view(B, L, Hkv, D).transpose(1, 2), cos, sin)
    vr = b[..., (Hq + Hkv) * D:].view(B, L, Hkv, D).transpose(1, 2)
    torch.autograd.backward((qr, kr, vr), (dq, dk, dv))
    assert torch.equal(q, qr) and torch.equal(k, kr) and torch.equal(v, vr)
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("D,Hq,Hkv,Tmax,step", [(64, 14, 2, 320, 270), (128, 32, 8, 320, 270),
                                                (64, 14, 2, 1280, 1200), (128, 32, 8, 700, 600),
                                                (128, 32, 8, 1300, 1250)])  # config 5: 1,291 keys at D 128
def test_attn_decode(ops, dev, D, Hq, Hkv, Tmax, step):
    """One key round (<= 512 keys for D=64, 256 for D=128) and several."""
    from swh_trl_amd import nn_ops
    g = _gen(20)
    B, P = 5, 40
    plen = torch.tensor([40, 33, 1, 40, 17], dtype=torch.int32)
    kc = (torch.randn(B, Hkv, Tmax, D, generator=g)).to(torch.bfloat16)
    vc = (torch.randn(B, Hkv, Tmax, D, generator=g)).to(torch.bfloat16)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g).to(torch.bfloat16)
    cos, sin = _rope_tables(D, 2048, 1e6, dev)
    state = torch.tensor([step + 1, P], dtype=torch.int32, device=dev)  # sampler index = input + 1
    kcd, vcd = kc.to(dev), vc.to(dev)
    out = nn_ops.attn_decode(qkv.to(dev), kcd, vcd, cos, sin, plen.to(dev), state, Hq, Hkv, D, D ** -0.5)
    # reference: fp32 math on the same bf16 values
    slot = P + step
    q = qkv[:, :Hq * D].view(B, Hq, D).float()
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, Hkv, D).float()
    v = qkv[:, (Hq + Hkv) * D:].view(B, Hkv, D)
    c, s = cos.cpu(), sin.cpu()
    exp = torch.empty(B, Hq * D)
    for b in range(B):
        pos = int(plen[b]) + step
        cc, ss = torch.cat([c[pos], c[pos]]), torch.cat([s[pos], s[pos]])

        def rope(x):
            rot = torch.cat([-x[..., D // 2:], x[..., :D // 2]], -1)
            return ((x * cc).bfloat16().float() + (rot * ss).bfloat16().float()).bfloat16().float()

        qb, kb = rope(q[b]), rope(k[b])
        K = kc[b].float().clone()
        Vv = vc[b].float().clone()
        K[:, slot] = kb
        Vv[:, slot] = v[b].float()
        st = P - int(plen[b])
        for h in range(Hq):
            kvh = h // (Hq // Hkv)
            sc = (K[kvh, st:slot + 1] @ qb[h]) * D ** -0.5
            p = torch.softmax(sc, 0)
            exp[b, h * D:(h + 1) * D] = p @ Vv[kvh, st:slot + 1]
    torch.testing.assert_close(out.cpu().float(), exp, rtol=2e-2, atol=2e-2)
    # the new k/v were appended to the cache
    assert torch.equal(vcd[:, :, slot].cpu(), v)
    # a slot past the cache end writes NaN and leaves the cache alone
    bad = torch.tensor([Tmax - P + 1, P], dtype=torch.int32, device=dev)
    before = kcd.clone()
    out2 = nn_ops.attn_decode(qkv.to(dev), kcd, vcd, cos, sin, plen.to(dev), bad, Hq, Hkv, D, D ** -0.5)
    assert torch.isnan(out2.float()).all() and torch.equal(before, kcd)


@pytest.mark.parametrize("D,Hkv,G,P,step", [(64, 2, 8, 128, 100), (128, 8, 8, 256, 300), (64, 2, 4, 41, 5),
                                             (128, 8, 8, 256, 1023)])  # config 5's last decode step: 1,280 keys
def test_attn_decode_shared_prompt_rows(ops, dev, D, Hkv, G, P, step):
    """swh_attn_decode_shared: the rows of a group read their prompt keys /
    values from the group's first row (the other rows' prompt slots hold
    garbage here) and equal swh_attn_decode over a cache where every row holds
    its own copy — output and appended slot, bit for bit; left padding included."""
    from swh_trl_amd import nn_ops
    g = _gen(24)
    U, Hq, Tmax = 3, 4 * Hkv, P + step + 8
    B = U * G
    plen_u = torch.tensor([P, max(1, P - 7), 1], dtype=torch.int32)
    plen = plen_u.repeat_interleave(G).to(dev)
    kc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    vc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    rep = torch.arange(0, B, G, device=dev)
    full_k, full_v = kc.clone(), vc.clone()  # every row its group's prompt
    full_k[:, :, :P] = kc[rep].repeat_interleave(G, 0)[:, :, :P]
    full_v[:, :, :P] = vc[rep].repeat_interleave(G, 0)[:, :, :P]
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g).to(torch.bfloat16).to(dev)
    cos, sin = _rope_tables(D, 2048, 1e6, dev)
    state = torch.tensor([step + 1, P], dtype=torch.int32, device=dev)
    prow = rep.repeat_interleave(G).to(torch.int32)
    a = nn_ops.attn_decode(qkv, full_k, full_v, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5)
    k2, v2 = kc.clone(), vc.clone()
    b = nn_ops.attn_decode(qkv, k2, v2, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, prompt_row=prow)
    assert torch.equal(a, b)
    slot = P + step
    assert torch.equal(k2[:, :, slot], full_k[:, :, slot]) and torch.equal(v2[:, :, slot], full_v[:, :, slot])
    # own rows (prompt_row = arange) is swh_attn_decode
    k3, v3 = full_k.clone(), full_v.clone()
    own = torch.arange(B, device=dev, dtype=torch.int32)
    c = nn_ops.attn_decode(qkv, k3, v3, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, prompt_row=own)
    assert torch.equal(a, c)


@pytest.mark.parametrize("G,U,P,step,shared,zero", [(8, 8, 256, 300, True, False), (8, 3, 64, 5, True, False),
                                                     (3, 3, 33, 17, True, False), (8, 2, 40, 9, False, False),
                                                     (3, 3, 33, 17, True, True), (8, 2, 40, 9, False, True)])
def test_attn_decode_pair_matches_per_row(ops, dev, G, U, P, step, shared, zero, launch_policy):
    """D = 128 row-pair attention (attn_pair: two rows per workgroup, a shared
    prompt's keys read once for both) against one workgroup per row: the same
    appended K/V slots bit for bit, outputs (row-major and fragment order) within
    fp32 summation-order noise of each other and of the fp32 reference; odd row
    counts and pairs straddling two groups (G 3) included; without prompt rows too.
    zero: zero-length prompts (the first group's, or row 0 alone beside a row that
    has a prompt), whose first key segment is empty."""
    from swh_trl_amd import nn_ops
    g = _gen(26)
    D, Hkv, Hq = 128, 8, 32
    B, Tmax = U * G, P + step + 8
    plen = torch.tensor([max(1, P - (u * 7) % P) for u in range(U)], dtype=torch.int32).repeat_interleave(G).to(dev)
    if zero:
        if shared:
            plen[:G] = 0
        else:
            plen[0] = 0
    kc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    vc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g).to(torch.bfloat16).to(dev)
    cos, sin = _rope_tables(D, 4096, 5e5, dev)
    state = torch.tensor([step + 1, P], dtype=torch.int32, device=dev)
    prow = torch.arange(0, B, G, device=dev).repeat_interleave(G).to(torch.int32) if shared else None
    res = {}
    for pair in (1, 0):
        launch_policy(attn_pair=pair)
        k2, v2 = kc.clone(), vc.clone()
        o = nn_ops.attn_decode(qkv, k2, v2, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, prompt_row=prow)
        of = None
        if B % 16 == 0:
            k3, v3 = kc.clone(), vc.clone()
            of = nn_ops.attn_decode(qkv, k3, v3, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, prompt_row=prow,
                                    out_frag=True)
            assert torch.equal(k3, k2) and torch.equal(v3, v2)
        res[pair] = (o, of, k2, v2)
    (o1, f1, k1, v1), (o0, f0, k0, v0) = res[1], res[0]
    assert torch.equal(k1, k0) and torch.equal(v1, v0)
    assert not torch.isnan(o1.float()).any()
    # the keys meet the waves in another order: fp32 summation noise, then one bf16 rounding
    torch.testing.assert_close(o1.float(), o0.float(), rtol=2e-2, atol=2e-2)
    if f1 is not None:
        torch.testing.assert_close(f1.float(), f0.float(), rtol=2e-2, atol=2e-2)
    # fp32 reference of every row
    slot = P + step
    q = qkv[:, :Hq * D].view(B, Hq, D).float().cpu()
    kn = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, Hkv, D).float().cpu()
    c, s_ = cos.cpu(), sin.cpu()
    kfull, vfull = k1.float().cpu(), v1.float().cpu()
    ref = torch.empty(B, Hq, D)
    for b in range(B):
        pl = int(plen[b])
        pos = pl + step
        cc, ss = torch.cat([c[pos], c[pos]]), torch.cat([s_[pos], s_[pos]])
        rot = lambda x: torch.cat([-x[..., D // 2:], x[..., :D // 2]], -1)  # noqa: E731
        qb = ((q[b] * cc).bfloat16().float() + (rot(q[b]) * ss).bfloat16().float()).bfloat16().float()
        pr = int(prow[b]) if shared else b
        keys = torch.cat([kfull[pr, :, P - pl:P], kfull[b, :, P:slot + 1]], 1)  # [Hkv, n, D]
        vals = torch.cat([vfull[pr, :, P - pl:P], vfull[b, :, P:slot + 1]], 1)
        kq = keys.repeat_interleave(Hq // Hkv, 0)
        vq = vals.repeat_interleave(Hq // Hkv, 0)
        att = torch.softmax((qb[:, None, :] * kq).sum(-1) * D ** -0.5, -1)
        ref[b] = (att[..., None] * vq).sum(1)
    torch.testing.assert_close(o1.float().cpu().view(B, Hq, D), ref, rtol=3e-2, atol=3e-2)


def test_attn_decode_pair_bad_row_poisons_only_itself(ops, dev, launch_policy):
    """A row whose prompt length is out of range gets NaN and no KV append; its
    pair partner runs alone and equals the per-row kernel's result (rows 2 and 5
    bad: the first and the second row of a pair)."""
    from swh_trl_amd import nn_ops
    g = _gen(27)
    D, Hkv, Hq, B, P, step = 128, 8, 32, 8, 40, 9
    Tmax = P + step + 8
    plen = torch.tensor([40, 33, 41, 20, 7, -1, 40, 1], dtype=torch.int32, device=dev)
    kc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    vc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g).to(torch.bfloat16).to(dev)
    cos, sin = _rope_tables(D, 4096, 5e5, dev)
    state = torch.tensor([step + 1, P], dtype=torch.int32, device=dev)
    res = {}
    for pair in (1, 0):
        launch_policy(attn_pair=pair)
        k2, v2 = kc.clone(), vc.clone()
        o = nn_ops.attn_decode(qkv, k2, v2, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5)
        res[pair] = (o.float().cpu().view(B, Hq, D), k2.cpu(), v2.cpu())
    (o1, k1, v1), (o0, k0, v0) = res[1], res[0]
    bad = torch.tensor([False, False, True, False, False, True, False, False])
    assert bool(o1[bad].isnan().all()) and bool(o0[bad].isnan().all())
    assert not bool(o1[~bad].isnan().any())
    torch.testing.assert_close(o1[~bad], o0[~bad], rtol=2e-2, atol=2e-2)
    assert torch.equal(k1, k0) and torch.equal(v1, v0)
    slot = P + step
    assert torch.equal(k1[bad][:, :, slot], kc.cpu()[bad][:, :, slot])  # no append for the bad rows
    assert not torch.equal(k1[~bad][:, :, slot], kc.cpu()[~bad][:, :, slot])


@pytest.mark.parametrize("D,Hkv,Hq,B", [(64, 2, 14, 64), (128, 8, 32, 32)])
def test_attn_decode_frag_output_feeds_o_proj(ops, dev, D, Hkv, Hq, B):
    """swh_attn_decode_shared_frag with out_frag = 1 writes exactly the row-major
    output permuted into o_proj's fragment order (torch restatement of the
    layout), the same appended K/V slot, and o_proj reading it (act_frag bit 1)
    equals o_proj over the row-major output bit for bit, residual rows and
    chunk sums of squares."""
    from swh_trl_amd import nn_ops
    g = _gen(61)
    P, step = 40, 17
    Tmax = P + step + 8
    kc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    vc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g).to(torch.bfloat16).to(dev)
    cos, sin = _rope_tables(D, 2048, 1e6, dev)
    plen = torch.full((B,), P, dtype=torch.int32, device=dev)
    plen[3] = 9
    state = torch.tensor([step + 1, P], dtype=torch.int32, device=dev)
    k1, v1, k2, v2 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    a = nn_ops.attn_decode(qkv, k1, v1, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5)
    f = nn_ops.attn_decode(qkv, k2, v2, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, out_frag=True)
    Q = Hq * D
    assert torch.equal(f, a.view(B // 16, 16, Q // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(B, Q))
    assert torch.equal(k1, k2) and torch.equal(v1, v2)
    if Q != 896:  # o_proj on the fragment-order path: the 0.5B width (8B's o_proj is the packed wide GEMM)
        return
    H = 896
    wo = nn_ops.frag_pack((torch.randn(H, Q, generator=g) * Q ** -0.5).to(torch.bfloat16).to(dev))
    s0 = torch.randn(B, H, generator=g).to(torch.bfloat16).to(dev)
    outs = []
    for act, x in ((0, a), (2, f)):
        r, so = s0.clone(), torch.full((B, H // 16), float("nan"), device=dev)
        nn_ops.decode_gemm_fragw(x, wo, residual=r, ss_out=so, act_frag=act)
        outs.append((r, so))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


# --------------------------------------------------------------------------- fused decode GEMM
def _ref_norm(x, w, eps):
    xf = x.float()
    n = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(torch.bfloat16)
    return (w * n)  # bf16 * bf16 -> bf16 (transformers Qwen2RMSNorm)


@pytest.mark.parametrize("M,N,K", [(64, 1152, 896), (5, 896, 896), (130, 256, 4864), (64, 151936, 896),
                                   (100, 32768, 896), (100, 65536, 896)])
@pytest.mark.parametrize("norm", [False, True])
def test_decode_gemm_plain(ops, dev, M, N, K, norm):
    from swh_trl_amd import nn_ops
    g = _gen(30)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(torch.bfloat16).to(dev) if N == 1152 else None
    y = nn_ops.decode_gemm(x, w, norm_w=nw if norm else None, eps=1e-6, bias=b)
    xa = _ref_norm(x, nw, 1e-6) if norm else x
    ref = xa.float() @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("name,M,N,K", [("qkv", 64, 6144, 4096), ("o", 64, 4096, 4096), ("lm_head", 64, 128256, 4096),
                                        ("down", 64, 4096, 14336)])
def test_decode_gemm_llama3_8b_shapes(ops, dev, name, M, N, K):
    """BASELINE config 5 decode projections (Llama-3-8B: H 4096, I 14336, V
    128256, GQA 32:8 x 128, untied head) at 64 rows: plain / folded-norm /
    residual epilogues against an fp32 reference."""
    from swh_trl_amd import nn_ops
    g = _gen(33)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    if name == "down":
        s = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
        s0 = s.clone()
        nn_ops.decode_gemm(x, w, residual=s)
        ref = s0 + (x.float() @ w.float().t()).to(torch.bfloat16)
        torch.testing.assert_close(s.float(), ref.float(), rtol=1e-2, atol=2e-2)
        return
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16).to(dev)
    y = nn_ops.decode_gemm(x, w, norm_w=nw, eps=1e-5)
    ref = _ref_norm(x, nw, 1e-5).float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-2)


def test_decode_gemm_llama3_8b_gate_up(ops, dev):
    """Config 5 gate/up (2 x 14336 rows over K 4096) with the SiLU epilogue."""
    from swh_trl_amd import nn_ops
    g = _gen(34)
    M, H, I = 64, 4096, 14336
    s = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    wgu = (torch.randn(2 * I, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    act = nn_ops.decode_gemm(s, wgu, norm_w=nw, eps=1e-5, silu=True)
    gu = (_ref_norm(s, nw, 1e-5).float() @ wgu.float().t()).to(torch.bfloat16)
    ref = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    torch.testing.assert_close(act.float(), ref.float(), rtol=2e-2, atol=2e-2)


def test_decode_gemm_residual_and_silu(ops, dev):
    from swh_trl_amd import nn_ops
    g = _gen(31)
    M, H, I = 64, 896, 4864
    s = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    a = torch.randn(M, I, generator=g).to(torch.bfloat16).to(dev)
    wd = (torch.randn(H, I, generator=g) * I ** -0.5).to(torch.bfloat16).to(dev)
    s0 = s.clone()
    nn_ops.decode_gemm(a, wd, residual=s)
    ref = s0 + (a.float() @ wd.float().t()).to(torch.bfloat16)
    torch.testing.assert_close(s.float(), ref.float(), rtol=1e-2, atol=2e-2)
    wgu = (torch.randn(2 * I, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    act = nn_ops.decode_gemm(s, wgu, norm_w=nw, eps=1e-6, silu=True)
    gu = (_ref_norm(s, nw, 1e-6).float() @ wgu.float().t()).to(torch.bfloat16)
    ref = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    torch.testing.assert_close(act.float(), ref.float(), rtol=2e-2, atol=2e-2)


def test_decode_gemm_split_k_is_deterministic_across_launches(ops, dev):
    """The cross-workgroup split-K reduction sums slabs in a fixed order and
    resets its counters: repeated launches give bit-identical results."""
    from swh_trl_amd import nn_ops
    g = _gen(32)
    x = torch.randn(64, 4864, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(896, 4864, generator=g) * 0.02).to(torch.bfloat16).to(dev)
    outs = [nn_ops.decode_gemm(x, w).clone() for _ in range(4)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    torch.testing.assert_close(outs[0].float(), x.float() @ w.float().t(), rtol=1e-2, atol=1e-2)


def _chunk_ss(t):
    """Per 16-column chunk sums of squares (fp32) of a bf16 [M, H] tensor."""
    M, H = t.shape
    return t.float().view(M, H // 16, 16).pow(2).sum(-1)


def test_rmsnorm_statistic_handoff(ops, dev):
    """embed_gather / residual epilogues publish per-chunk sums of squares;
    the normed GEMM consuming them (ss_in) matches the in-kernel statistic."""
    from swh_trl_amd import nn_ops
    g = _gen(33)
    V, M, H, I = 1000, 64, 896, 4864
    table = torch.randn(V, H, generator=g).to(torch.bfloat16).to(dev)
    ids = torch.randint(0, V, (M,), generator=g).to(dev)
    s = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    ss = torch.empty(M, H // 16, dtype=torch.float32, device=dev)
    nn_ops.embed_gather(table, ids, s, ss_out=ss)
    assert torch.equal(s, table[ids])
    torch.testing.assert_close(ss, _chunk_ss(s), rtol=1e-5, atol=1e-5)
    a = torch.randn(M, I, generator=g).to(torch.bfloat16).to(dev)
    wd = (torch.randn(H, I, generator=g) * I ** -0.5).to(torch.bfloat16).to(dev)
    nn_ops.decode_gemm(a, wd, residual=s, ss_out=ss)
    torch.testing.assert_close(ss, _chunk_ss(s), rtol=1e-5, atol=1e-5)
    w = (torch.randn(1152, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    b = torch.randn(1152, generator=g).to(torch.bfloat16).to(dev)
    y1 = nn_ops.decode_gemm(s, w, norm_w=nw, eps=1e-6, bias=b, ss_in=ss)
    y0 = nn_ops.decode_gemm(s, w, norm_w=nw, eps=1e-6, bias=b)
    ref = _ref_norm(s, nw, 1e-6).float() @ w.float().t() + b.float()
    torch.testing.assert_close(y1.float(), ref, rtol=1e-2, atol=1e-2)
    # the two statistics differ only in fp32 summation order
    assert (y1 != y0).float().mean().item() < 0.01


@pytest.mark.parametrize("cfg,nw", [("1,1,1", None), ("2,1,1", None), ("4,1,1", None), ("1,2,2", None),
                                    ("2,4,1", None), ("4,4,3", None), ("1,1,3", None), ("2,2,2", None),
                                    ("4,2,1,1", None), ("4,4,1,1", None), ("1,1,1", "16"), ("2,1,2", "16"),
                                    ("1,1,1", "4"), ("2,2,1", "4"), ("4,1,3", "16"), ("4,4,1,0,4", None),
                                    ("4,4,1,0,2", None), ("2,2,2,0,2", None), ("4,2,1,1,2", None),
                                    ("4,4,1,0,4", "4"), ("1,4,3,0,4", None)])
def test_decode_gemm_launch_configs(ops, dev, cfg, nw, launch_policy):
    """Every (row blocks, column blocks, K split[, persistent]) geometry and
    wave count computes the same GEMM: normed + bias, residual + statistic,
    SiLU gate."""
    from swh_trl_amd import nn_ops
    launch_policy(gemm_cfg=cfg, gemm_nw=int(nw) if nw is not None else 0)
    g = _gen(34)
    M, H, I = 40, 896, 1024
    s = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    w = (torch.randn(1152, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    b = torch.randn(1152, generator=g).to(torch.bfloat16).to(dev)
    y = nn_ops.decode_gemm(s, w, norm_w=nw, eps=1e-6, bias=b)
    xn = _ref_norm(s, nw, 1e-6).float()
    torch.testing.assert_close(y.float(), xn @ w.float().t() + b.float(), rtol=1e-2, atol=1e-2)
    wgu = (torch.randn(2 * I, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    act = nn_ops.decode_gemm(s, wgu, norm_w=nw, eps=1e-6, silu=True)
    gu = (xn @ wgu.float().t()).to(torch.bfloat16)
    torch.testing.assert_close(act.float(), (torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]).float(),
                               rtol=2e-2, atol=2e-2)
    wd = (torch.randn(H, I, generator=g) * I ** -0.5).to(torch.bfloat16).to(dev)
    ss = torch.empty(M, H // 16, dtype=torch.float32, device=dev)
    s0 = s.clone()
    nn_ops.decode_gemm(act, wd, residual=s, ss_out=ss)
    ref = s0 + (act.float() @ wd.float().t()).to(torch.bfloat16)
    torch.testing.assert_close(s.float(), ref.float(), rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(ss, _chunk_ss(s), rtol=1e-5, atol=1e-5)


def test_decode_gemm_persistent_epilogues(ops, dev):
    """Workgroups looping over column blocks (more blocks than CUs) run every
    epilogue: bias, residual + statistic, SiLU gate; two M tiles."""
    from swh_trl_amd import nn_ops
    g = _gen(35)
    M, H, N = 70, 896, 8192
    s = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(torch.bfloat16).to(dev)
    xn = _ref_norm(s, nw, 1e-6).float()
    y = nn_ops.decode_gemm(s, w, norm_w=nw, eps=1e-6, bias=b)
    torch.testing.assert_close(y.float(), xn @ w.float().t() + b.float(), rtol=1e-2, atol=1e-2)
    wgu = (torch.randn(2 * N, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
    act = nn_ops.decode_gemm(s, wgu, norm_w=nw, eps=1e-6, silu=True)
    gu = (xn @ wgu.float().t()).to(torch.bfloat16)
    torch.testing.assert_close(act.float(), (torch.nn.functional.silu(gu[:, :N]) * gu[:, N:]).float(),
                               rtol=2e-2, atol=2e-2)
    a = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    r = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    ss = torch.empty(M, N // 16, dtype=torch.float32, device=dev)
    r0 = r.clone()
    nn_ops.decode_gemm(a, w, residual=r, ss_out=ss)
    ref = r0 + (a.float() @ w.float().t()).to(torch.bfloat16)
    torch.testing.assert_close(r.float(), ref.float(), rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(ss, _chunk_ss(r), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kw", [dict(), dict(temperature=0.7), dict(greedy=True), dict(min_new_tokens=5),
                                dict(temperature=1.3, min_new_tokens=1)])
@pytest.mark.parametrize("M,V,fold", [(64, 151936, False), (70, 32768, False), (64, 151936, True),
                                      (64, 151936, "fragw"), (70, 32768, "fragw")])
def test_lm_head_sample_equals_logits_then_sampler(ops, dev, kw, M, V, fold):
    """The fused lm head + sampler draws, bit for bit, the token swh_sample_step
    draws from the materialised bf16 logits (same rng, same step), including
    EOS suppression, pad-after-EOS and the finished flags."""
    from swh_trl_amd import nn_ops
    g = _gen(36)
    H = 896
    x = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(V, H, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, H // 16, 16).pow(2).sum(-1).contiguous()
    eos = [3, 77]
    w[3] += 0.2  # make EOS likely so suppression and bookkeeping matter
    params = ops.make_sample_params(eos_token_ids=eos, pad_token_id=5, **kw)
    step = 2
    rng = torch.tensor([123, 45], dtype=torch.int64, device=dev)
    stp = torch.tensor([step], dtype=torch.int32, device=dev)
    fin0 = (torch.arange(M) % 7 == 0).int().to(dev)
    if fold:  # folded norm weight, rstd row scale in the epilogue
        w = w * nw
        nw = None
    logits = nn_ops.decode_gemm(x, w, norm_w=nw, eps=1e-6, ss_in=ss)
    out_a = torch.full((M, 4), -1, dtype=torch.int64, device=dev)
    cur_a = torch.empty(M, dtype=torch.int64, device=dev)
    fin_a = fin0.clone()
    ops.sample_step(logits, params, rng, stp, fin_a, out_a, cur_a)
    out_b = torch.full((M, 4), -1, dtype=torch.int64, device=dev)
    cur_b = torch.empty(M, dtype=torch.int64, device=dev)
    fin_b = fin0.clone()
    if fold == "fragw":  # the folded weight in fragment order (swh_lm_head_sample_fragw)
        nn_ops.lm_head_sample(x, nn_ops.frag_pack(w), params, rng, stp, fin_b, out_b, cur_b, eps=1e-6, ss_in=ss,
                              fragw=True)
    else:
        nn_ops.lm_head_sample(x, w, params, rng, stp, fin_b, out_b, cur_b, norm_w=nw, eps=1e-6, ss_in=ss)
    assert torch.equal(out_b, out_a)
    assert torch.equal(cur_b, cur_a)
    assert torch.equal(fin_b, fin_a)
    if kw.get("min_new_tokens", 0) > step:
        assert not torch.isin(out_b[:, step], torch.tensor(eos, device=dev)).any()
    # the log-prob variant (swh_lm_head_sample_logp): the same draws, and the drawn tokens'
    # log-probs under the processed distribution as swh_sample_step computes them from
    # the materialised logits (fp32 summation order and the score recovered from its key)
    lp_a = torch.zeros(M, 4, dtype=torch.float32, device=dev)
    out_a2, fin_a2 = torch.full_like(out_a, -1), fin0.clone()
    ops.sample_step(logits, params, rng, stp, fin_a2, out_a2, torch.empty_like(cur_a), out_logp=lp_a)
    lp_c = torch.zeros(M, 4, dtype=torch.float32, device=dev)
    out_c, cur_c, fin_c = torch.full_like(out_a, -1), torch.empty_like(cur_a), fin0.clone()
    if fold == "fragw":
        nn_ops.lm_head_sample(x, nn_ops.frag_pack(w), params, rng, stp, fin_c, out_c, cur_c, eps=1e-6, ss_in=ss,
                              fragw=True, out_logp=lp_c)
    else:
        nn_ops.lm_head_sample(x, w, params, rng, stp, fin_c, out_c, cur_c, norm_w=nw, eps=1e-6, ss_in=ss,
                              out_logp=lp_c)
    assert torch.equal(out_c, out_a) and torch.equal(cur_c, cur_a) and torch.equal(fin_c, fin_a)
    assert bool((lp_a[:, step] <= 0).all())
    torch.testing.assert_close(lp_c[:, step], lp_a[:, step], rtol=1e-6, atol=1e-5)
    assert torch.equal(lp_c[:, :step], lp_a[:, :step]) and torch.equal(lp_c[:, step + 1:], lp_a[:, step + 1:])


@pytest.mark.parametrize("kw", [dict(), dict(temperature=0.7), dict(greedy=True), dict(min_new_tokens=5),
                                dict(temperature=1.3, min_new_tokens=1)])
@pytest.mark.parametrize("M,V", [(64, 4096), (37, 8192), (64, 128256)])
def test_lm_head_sample_wide_equals_logits_then_sampler(ops, dev, kw, M, V, launch_policy):
    """K > 1024 (Llama-3-8B, hidden 4096): the fused sampler over the wide_pack'ed
    folded lm-head weight (wide_gemm's 256-row tiles, sampler epilogue, one
    partial per row and tile) draws, bit for bit, the token swh_sample_step draws
    from the bf16 logits the same tiles write, with EOS suppression, pad-after-EOS
    and the finished flags."""
    from swh_trl_amd import nn_ops
    g = _gen(37)
    H = 4096
    x = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(H, generator=g)).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, H // 16, 16).pow(2).sum(-1).contiguous()
    eos = [3, 77]
    w[3] += 0.02  # make EOS likely so suppression and bookkeeping matter
    wp = nn_ops.wide_pack(w, nw)
    params = ops.make_sample_params(eos_token_ids=eos, pad_token_id=5, **kw)
    step = 2
    rng = torch.tensor([321, 54], dtype=torch.int64, device=dev)
    stp = torch.tensor([step], dtype=torch.int32, device=dev)
    fin0 = (torch.arange(M) % 7 == 0).int().to(dev)
    assert nn_ops.lm_head_sample_supported(params, V, H, wide_rows=M)
    launch_policy(wide_cb=2)  # the logits through the same 256-row tiles (no K split)
    logits = nn_ops.wide_gemm_packed(x, wp, V, eps=1e-6, ss_in=ss)
    out_a = torch.full((M, 4), -1, dtype=torch.int64, device=dev)
    cur_a = torch.empty(M, dtype=torch.int64, device=dev)
    fin_a = fin0.clone()
    ops.sample_step(logits, params, rng, stp, fin_a, out_a, cur_a)
    out_b = torch.full((M, 4), -1, dtype=torch.int64, device=dev)
    cur_b = torch.empty(M, dtype=torch.int64, device=dev)
    fin_b = fin0.clone()
    nn_ops.lm_head_sample(x, wp, params, rng, stp, fin_b, out_b, cur_b, eps=1e-6, ss_in=ss, fragw=True)
    assert torch.equal(out_b, out_a)
    assert torch.equal(cur_b, cur_a)
    assert torch.equal(fin_b, fin_a)
    if kw.get("min_new_tokens", 0) > step:
        assert not torch.isin(out_b[:, step], torch.tensor(eos, device=dev)).any()


def test_lm_head_sample_refuses_filtered(ops, dev):
    from swh_trl_amd import nn_ops
    x = torch.zeros(4, 896, dtype=torch.bfloat16, device=dev)
    w = torch.zeros(1024, 896, dtype=torch.bfloat16, device=dev)
    rng = torch.zeros(2, dtype=torch.int64, device=dev)
    stp = torch.zeros(1, dtype=torch.int32, device=dev)
    fin = torch.zeros(4, dtype=torch.int32, device=dev)
    out = torch.zeros(4, 2, dtype=torch.int64, device=dev)
    for kw in (dict(top_k=5), dict(top_p=0.9), dict(min_p=0.1), dict(repetition_penalty=1.2)):
        p = ops.make_sample_params(**kw)
        assert not nn_ops.lm_head_sample_supported(p, 1024, 896)
        with pytest.raises(ValueError):
            nn_ops.lm_head_sample(x, w, p, rng, stp, fin, out)


@pytest.mark.parametrize("M,N,K,silu", [(64, 1152, 896, False), (64, 4864, 896, True), (20, 151936, 896, False)])
def test_decode_gemm_folded_norm(ops, dev, M, N, K, silu):
    """ss_in without norm_w: y = rstd * (x W'^T), W' = bf16(W * w) — the decode
    engine's folded RMSNorm; equals the reference within bf16 rounding."""
    from swh_trl_amd import nn_ops
    g = _gen(37)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    wrows = 2 * N if silu else N
    w = (torch.randn(wrows, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16).to(dev)
    ss = _chunk_ss(x)
    y = nn_ops.decode_gemm(x, w * nw, ss_in=ss, eps=1e-6, silu=silu)
    ref = _ref_norm(x, nw, 1e-6).float() @ w.float().t()
    if silu:
        gu = ref.to(torch.bfloat16)
        ref = (torch.nn.functional.silu(gu[:, :N]) * gu[:, N:]).float()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)  # rounding of the fold, then SiLU's


@pytest.mark.parametrize("M,N,K", [(64, 896, 896), (64, 896, 4864), (37, 896, 4864), (5, 256, 512), (64, 896, 2048)])
def test_xstream_residual_equals_lds_image_kernel(ops, dev, M, N, K, launch_policy):
    """o_proj / down_proj with X fragments streamed into registers
    (xstream_gemm_kernel) vs decode_gemm_kernel's LDS image (launch policy xstream 0):
    the new residual rows and their chunk sums of squares are bit-identical
    (same k split, same wave merge tree), and equal the fp32 reference within
    bf16 rounding."""
    from swh_trl_amd import nn_ops
    g = _gen(43)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    s0 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    outs = {}
    for flag in ("1", "0"):
        launch_policy(xstream=int(flag))
        r = s0.clone()
        ss = torch.full((M, N // 16), float("nan"), device=dev)
        nn_ops.decode_gemm(x, w, residual=r, ss_out=ss)
        outs[flag] = (r, ss)
    torch.cuda.synchronize()
    assert torch.equal(outs["1"][0], outs["0"][0])
    assert torch.equal(outs["1"][1], outs["0"][1])
    ref = s0.float() + (x.float() @ w.float().t()).to(torch.bfloat16).float()
    torch.testing.assert_close(outs["1"][0].float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(outs["1"][1], outs["1"][0].float().view(M, N // 16, 16).pow(2).sum(-1),
                               rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,N,K,kind", [(64, 896, 896, "res"), (64, 896, 4864, "res"), (37, 896, 4864, "res"),
                                        (5, 256, 512, "res"), (64, 1152, 896, "qkv"), (37, 1152, 896, "qkv"),
                                        (64, 256, 1024, "plain"), (64, 4864, 896, "silu"), (37, 4864, 896, "silu"),
                                        (16, 512, 256, "silu")])
@pytest.mark.parametrize("cfg", [None, "1,1,2", "2,1,1", "4,2,1,1"])
def test_decode_gemm_fragw_equals_row_major(ops, dev, M, N, K, kind, cfg, launch_policy):
    """swh_frag_pack's layout element for element against a torch restatement,
    and swh_decode_gemm_fragw on it bit-identical to swh_decode_gemm on the
    row-major weight: residual + chunk sums of squares (o / down), folded norm
    + bias (qkv), plain — under the cost model's geometry and forced split-K /
    32-row / persistent ones (launch policy gemm_cfg)."""
    from swh_trl_amd import nn_ops
    g = _gen(53)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    wp = nn_ops.frag_pack(w)
    # restatement: element ((grp KS + ks) 64 + lane) 8 + e = W[16 grp + lane % 16, 32 ks + 8 (lane / 16) + e]
    ref = w.view(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N, K)
    assert torch.equal(wp, ref)
    if kind == "silu":  # 16-row groups of 8 gate + the 8 matching up rows, folded with the norm weight
        nw = (1 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16).to(dev)
        wu = torch.cat([w, w.flip(0)])
        wp = nn_ops.frag_pack(wu, nw, silu=True)
        inter = torch.stack([wu[:N].view(N // 8, 8, K), wu[N:].view(N // 8, 8, K)], 1).reshape(2 * N, K)
        ref = (inter.float() * nw.float()).to(torch.bfloat16)
        assert torch.equal(wp, ref.view(2 * N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(2 * N, K))
        w = (wu.float() * nw.float()).to(torch.bfloat16)
    if cfg:
        launch_policy(gemm_cfg=cfg)
    outs = []
    for fw in (True, False):
        kw = {}
        if kind == "res":
            kw = dict(residual=torch.randn(M, N, generator=_gen(5)).to(torch.bfloat16).to(dev),
                      ss_out=torch.full((M, N // 16), float("nan"), device=dev))
        elif kind == "qkv":
            kw = dict(bias=(0.1 * torch.randn(N, generator=_gen(6))).to(torch.bfloat16).to(dev), ss_in=_chunk_ss(x))
        elif kind == "silu":
            kw = dict(silu=True, ss_in=_chunk_ss(x))
        out = (nn_ops.decode_gemm_fragw(x, wp, eps=1e-6, **kw) if fw else nn_ops.decode_gemm(x, w, eps=1e-6, **kw))
        outs.append((out, kw.get("ss_out")))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    if kind == "res":
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("M", [64, 32])
def test_act_frag_gate_up_to_down_equals_row_major(ops, dev, M):
    """gate/up writing its SiLU output in fragment order (act_frag bit 0) is the
    row-major output permuted (torch restatement), and down_proj reading it
    (bit 1, register-streamed X at K 4864) equals down_proj over the row-major
    activation bit for bit, residual rows and chunk sums of squares."""
    from swh_trl_amd import nn_ops
    g = _gen(59)
    H, I = 896, 4864
    x = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    wgu = nn_ops.frag_pack((torch.randn(2 * I, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev), silu=True)
    wd = nn_ops.frag_pack((torch.randn(H, I, generator=g) * I ** -0.5).to(torch.bfloat16).to(dev))
    ss = _chunk_ss(x)
    y_rm = nn_ops.decode_gemm_fragw(x, wgu, silu=True, ss_in=ss)
    y_fr = nn_ops.decode_gemm_fragw(x, wgu, silu=True, ss_in=ss, act_frag=1)
    assert torch.equal(y_fr, y_rm.view(M // 16, 16, I // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(M, I))
    s0 = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
    outs = []
    for act, y in ((0, y_rm), (2, y_fr)):
        r, so = s0.clone(), torch.full((M, H // 16), float("nan"), device=dev)
        nn_ops.decode_gemm_fragw(y, wd, residual=r, ss_out=so, act_frag=act)
        outs.append((r, so))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("M,N,K", [(64, 1152, 896), (37, 1152, 896), (64, 384, 512), (20, 1152, 896)])
def test_xstream_qkv_equals_lds_image_kernel(ops, dev, M, N, K, launch_policy):
    """The qkv projection (folded RMSNorm row scale from the producer's chunk
    sums, bias) with X fragments streamed into registers equals
    decode_gemm_kernel's LDS-image form bit for bit (launch policy xstream 0), and the
    reference within the fold's rounding."""
    from swh_trl_amd import nn_ops
    g = _gen(47)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16).to(dev)
    b = (0.1 * torch.randn(N, generator=g)).to(torch.bfloat16).to(dev)
    ss = _chunk_ss(x)
    outs = {}
    for flag in ("1", "0"):
        launch_policy(xstream=int(flag))
        outs[flag] = nn_ops.decode_gemm(x, w * nw, ss_in=ss, eps=1e-6, bias=b)
    torch.cuda.synchronize()
    assert torch.equal(outs["1"], outs["0"])
    ref = _ref_norm(x, nw, 1e-6).float() @ w.float().t() + b.float()
    torch.testing.assert_close(outs["1"].float(), ref, rtol=2e-2, atol=3e-2)


# --------------------------------------------------------------------------- training attention (csrc/attn.hip)
def _ref_attention(q, k, v, scale, km=None):
    """fp32 reference: transformers' padded causal mask (a query with no valid
    key sees itself), GQA by head repetition."""
    B, Hq, L, D = q.shape
    G = Hq // k.shape[1]
    kf, vf = k.float().repeat_interleave(G, 1), v.float().repeat_interleave(G, 1)
    causal = torch.ones(L, L, dtype=torch.bool, device=q.device).tril()
    if km is None:
        mask = causal[None, None]
    else:
        kb = km.bool()
        no_key = kb.cumsum(-1) == 0
        eye = torch.eye(L, dtype=torch.bool, device=q.device)
        mask = causal & (kb[:, None, None, :] | (eye & no_key[:, None, :, None]))
    s = (q.float() @ kf.transpose(-1, -2)) * scale
    s = s.masked_fill(~mask, float("-inf"))
    return torch.softmax(s, -1) @ vf


@pytest.mark.parametrize("B,Hq,Hkv,L,D,pad", [(2, 14, 2, 384, 64, False), (3, 14, 2, 100, 64, True),
                                              (2, 4, 4, 77, 64, True), (1, 8, 2, 96, 128, False)])
def test_attention_fwd_bwd_matches_reference(ops, dev, B, Hq, Hkv, L, D, pad):
    """swh_attn_fwd/bwd vs an fp32 autograd reference of the same mask: output
    and dq/dk/dv within bf16 tolerance (bf16 P in the P V and dS products)."""
    from swh_trl_amd import nn_ops
    g = _gen(60 + L)
    q = torch.randn(B, Hq, L, D, generator=g).to(torch.bfloat16).to(dev)
    k = torch.randn(B, Hkv, L, D, generator=g).to(torch.bfloat16).to(dev)
    v = torch.randn(B, Hkv, L, D, generator=g).to(torch.bfloat16).to(dev)
    do = torch.randn(B, Hq, L, D, generator=g).to(torch.bfloat16).to(dev)
    km = fv = None
    if pad:
        km = torch.ones(B, L, dtype=torch.int32)
        for b in range(B):
            km[b, : (7 * b + 3) % (L // 2)] = 0  # left padding of different lengths
        km[0, L - 5:] = 0                       # and right padding on one row
        km = km.to(dev)
        fv = (km.cumsum(-1) == 0).sum(-1).to(torch.int32)
    scale = D ** -0.5
    qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = nn_ops.AttentionFn.apply(qa, ka, va, scale, km, fv)
    o.backward(do)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attention(qr, kr, vr, scale, km)
    ref.backward(do.float())
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    for mine, r in ((qa.grad, qr.grad), (ka.grad, kr.grad), (va.grad, vr.grad)):
        err = (mine.float() - r).abs().max().item()
        assert err <= 3e-2 * max(1.0, r.abs().max().item()), err


@pytest.mark.parametrize("pad", [False, True])
def test_attention_token_major_equals_plain(ops, dev, pad):
    """AttentionTokFn (swh_attn_fwd_v / _bwd_v_parts, output token-major) is
    AttentionFn's output transposed, and the same dq / dk / dv, bit for bit."""
    from swh_trl_amd import nn_ops
    g = _gen(71)
    B, Hq, Hkv, L, D = 3, 14, 2, 150, 64
    q = torch.randn(B, Hq, L, D, generator=g).to(torch.bfloat16).to(dev)
    k = torch.randn(B, Hkv, L, D, generator=g).to(torch.bfloat16).to(dev)
    v = torch.randn(B, Hkv, L, D, generator=g).to(torch.bfloat16).to(dev)
    do = torch.randn(B, Hq, L, D, generator=g).to(torch.bfloat16).to(dev)
    km = fv = None
    if pad:
        km = torch.ones(B, L, dtype=torch.int32)
        km[1, :17] = 0
        km = km.to(dev)
        fv = (km.cumsum(-1) == 0).sum(-1).to(torch.int32)
    res = []
    for fn in (nn_ops.AttentionFn, nn_ops.AttentionTokFn):
        qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
        o = fn.apply(qa, ka, va, D ** -0.5, km, fv)
        if fn is nn_ops.AttentionTokFn:
            o.backward(do.transpose(1, 2).reshape(B, L, Hq * D))
            o = o.view(B, L, Hq, D).transpose(1, 2)
        else:
            o.backward(do)
        res.append((o, qa.grad, ka.grad, va.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("P,C,G,pad", [(128, 256, 8, False), (128, 96, 4, True), (41, 30, 3, True)])
def test_grouped_attention_equals_concatenated(ops, dev, P, C, G, pad):
    """GroupedAttentionFn (each group's prompt Q/K/V read in place by its G
    sequences, prompt queries computed once, output token-major) against the
    concatenated form the shared-prompt forward used before: AttentionFn over
    cat(broadcast prompt, completion), the group's first prompt rows and every
    completion row taken from its output, gradients through the same cat /
    broadcast autograd.  Output, d prompt Q and completion gradients bit for
    bit; d prompt K / V (summed over the group) bit for bit when P is a
    multiple of 64 (the dK/dV query rounds align), else to fp32 rounding."""
    from swh_trl_amd import nn_ops
    g = _gen(72 + P)
    U, Hq, Hkv, D = 2, 14, 2, 64
    R, L = U * G, P + C
    bf = dict(dtype=torch.bfloat16)
    t = lambda *sh: torch.randn(*sh, generator=g).to(**bf).to(dev)  # noqa: E731
    q_p, k_p, v_p = t(U, Hq, P, D), t(U, Hkv, P, D), t(U, Hkv, P, D)
    q_c, k_c, v_c = t(R, Hq, C, D), t(R, Hkv, C, D), t(R, Hkv, C, D)
    do = t(U * P + R * C, Hq * D)
    km = fv = None
    if pad:
        kmu = torch.ones(U, P, dtype=torch.int32)
        kmu[1, :P // 3] = 0
        km = torch.cat([kmu.repeat_interleave(G, 0), torch.ones(R, C, dtype=torch.int32)], 1).to(dev)
        fv = (km.cumsum(-1) == 0).sum(-1).to(torch.int32)

    def bc(x):
        return x[:, None].expand(U, G, *x.shape[1:]).reshape(R, *x.shape[1:])

    ins1 = [x.clone().requires_grad_(True) for x in (q_p, k_p, v_p, q_c, k_c, v_c)]
    o1 = nn_ops.GroupedAttentionFn.apply(*ins1, G, D ** -0.5, km, fv)
    o1.backward(do)
    ins2 = [x.clone().requires_grad_(True) for x in (q_p, k_p, v_p, q_c, k_c, v_c)]
    q = torch.cat([bc(ins2[0]), ins2[3]], 2)
    k = torch.cat([bc(ins2[1]), ins2[4]], 2)
    v = torch.cat([bc(ins2[2]), ins2[5]], 2)
    o = nn_ops.AttentionFn.apply(q, k, v, D ** -0.5, km, fv).transpose(1, 2).reshape(R, L, Hq * D)
    o2 = torch.cat([o.view(U, G, L, -1)[:, 0, :P].reshape(U * P, -1), o[:, P:].reshape(R * C, -1)])
    o2.backward(do)
    assert torch.equal(o1, o2)
    for i in (0, 3, 4, 5):
        assert torch.equal(ins1[i].grad, ins2[i].grad), i
    for i in (1, 2):
        a, b = ins1[i].grad.float(), ins2[i].grad.float()
        if P % 64 == 0:
            assert torch.equal(a, b), i
        else:
            torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2 * b.abs().max().item())


@pytest.mark.parametrize("name,M,N,K", [("qkv_bias", 64, 6144, 4096), ("o_res", 8, 4096, 4096),
                                        ("gate_up", 33, 14336, 4096), ("down", 64, 4096, 14336),
                                        ("down_tiny_llama", 6, 1024, 2048), ("lm_head", 64, 128256, 4096),
                                        ("norm_long_k", 21, 4096, 14336)])
def test_wide_gemm_bandwidth_regime(ops, dev, name, M, N, K):
    """csrc/wide_gemm.hip (decode GEMMs with K >= 2048, the Llama-3-8B decode
    shapes of config 5) through swh_decode_gemm, in the forms the decode step
    uses: folded-RMSNorm row scale from the producer's partial sums (ss_in)
    with / without bias, SiLU gate, residual + the next norm's partial sums;
    64 rows and ragged row counts; split-K tiles bit-identical across launches."""
    from swh_trl_amd import nn_ops
    g = _gen(35)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, K // 16, 16).pow(2).sum(-1).contiguous()
    rstd = torch.rsqrt(ss.sum(-1, keepdim=True) / K + 1e-5)
    if name.startswith(("o_", "down")):
        w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
        s = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
        s0 = s.clone()
        sso = torch.empty(M, N // 16, device=dev)
        nn_ops.decode_gemm(x, w, residual=s, ss_out=sso)
        ref = (s0.float() + (x.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
        assert (s.float() - ref.float()).abs().max().item() <= 2e-2 * ref.float().abs().max().item() + 2e-2
        torch.testing.assert_close(sso, s.float().view(M, N // 16, 16).pow(2).sum(-1), rtol=1e-5, atol=1e-4)
        s2 = s0.clone()
        nn_ops.decode_gemm(x, w, residual=s2, ss_out=sso)
        assert torch.equal(s, s2)
        return
    if name == "gate_up":
        w = (torch.randn(2 * N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
        act = nn_ops.decode_gemm(x, w, silu=True, ss_in=ss, eps=1e-5)
        gu = ((x.float() @ w.float().t()) * rstd).to(torch.bfloat16)
        ref = (torch.nn.functional.silu(gu[:, :N].float()).to(torch.bfloat16).float() * gu[:, N:].float())
        torch.testing.assert_close(act.float(), ref, rtol=2e-2, atol=2e-2)
        assert torch.equal(act, nn_ops.decode_gemm(x, w, silu=True, ss_in=ss, eps=1e-5))
        return
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    b = (0.1 * torch.randn(N, generator=g)).to(torch.bfloat16).to(dev) if name == "qkv_bias" else None
    y = nn_ops.decode_gemm(x, w, ss_in=ss, eps=1e-5, bias=b)
    ref = (x.float() @ w.float().t()) * rstd + (b.float() if b is not None else 0.0)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-2)
    assert torch.equal(y, nn_ops.decode_gemm(x, w, ss_in=ss, eps=1e-5, bias=b))


def _wide_pack_ref(w, nw, silu):
    """Fragment order of swh_wide_pack restated in torch: tile row T -> weight
    row (SiLU: 8 gate rows then the 8 matching up rows per 16-row group), then
    [group, round, k-step, lane group, lane row, 8 elements]."""
    rows, K = w.shape
    wf = (w * nw) if nw is not None else w  # torch's bf16 mul: one rounding of the fp32 product
    if silu:
        N = rows // 2
        T = torch.arange(rows, device=w.device)
        base = (T >> 4) * 8 + (T & 7)
        wf = wf[torch.where((T & 15) < 8, base, N + base)]
    return wf.view(rows // 16, 16, K // 128, 4, 4, 8).permute(0, 2, 3, 4, 1, 5).reshape(-1)


@pytest.mark.parametrize("name,M,N,K", [("qkv_bias", 64, 6144, 4096), ("o_res", 64, 4096, 4096),
                                        ("gate_up", 64, 14336, 4096), ("down", 37, 4096, 14336),
                                        ("lm_head", 64, 128256, 4096), ("small", 5, 1024, 2048)])
def test_wide_gemm_packed_equals_row_major(ops, dev, name, M, N, K):
    """swh_wide_pack writes the fragment order (checked element for element
    against a torch restatement, with the folded norm), and
    swh_wide_gemm_packed over it equals the row-major wide GEMM on the folded
    weight bit for bit (same k order, same split-K reduction order)."""
    from swh_trl_amd import nn_ops
    g = _gen(36)
    silu = name == "gate_up"
    normed = name in ("qkv_bias", "gate_up", "lm_head", "small")
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, K // 16, 16).pow(2).sum(-1).contiguous()
    w = (torch.randn(2 * N if silu else N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    nw = (1.0 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16).to(dev) if normed else None
    assert nn_ops.wide_gemm_eligible(M, N, K, silu)
    wp = nn_ops.wide_pack(w, nw, silu=silu)
    assert torch.equal(wp, _wide_pack_ref(w, nw, silu))
    wf = w * nw if normed else w
    if name.startswith(("o_", "down")):
        s0 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
        s1, s2 = s0.clone(), s0.clone()
        so1, so2 = torch.empty(M, N // 16, device=dev), torch.empty(M, N // 16, device=dev)
        nn_ops.decode_gemm(x, wf, residual=s1, ss_out=so1)
        nn_ops.wide_gemm_packed(x, wp, N, residual=s2, ss_out=so2)
        assert torch.equal(s1, s2) and torch.equal(so1, so2)
        return
    b = (0.1 * torch.randn(N, generator=g)).to(torch.bfloat16).to(dev) if name == "qkv_bias" else None
    y1 = nn_ops.decode_gemm(x, wf, silu=silu, ss_in=ss, eps=1e-5, bias=b)
    y2 = nn_ops.wide_gemm_packed(x, wp, N, silu=silu, ss_in=ss, eps=1e-5, bias=b)
    assert torch.equal(y1, y2)


def test_wide_gemm_packed_rejects_ineligible(ops, dev):
    """No row-major fallback behind the packed entry: shapes wide_gemm does
    not serve are argument errors."""
    from swh_trl_amd import nn_ops
    assert not nn_ops.wide_gemm_eligible(64, 896, 4864)       # narrow output (0.5B down)
    assert not nn_ops.wide_gemm_eligible(65, 4096, 4096)      # more than 64 rows
    x = torch.zeros(65, 4096, dtype=torch.bfloat16, device=dev)
    wp = torch.zeros(4096 * 4096, dtype=torch.bfloat16, device=dev)
    with pytest.raises(ValueError):
        nn_ops.wide_gemm_packed(x, wp, 4096)


@pytest.mark.parametrize("name,N,K", [("gate_up", 14336, 4096), ("lm_head", 128256, 4096), ("plain", 16384, 2048)])
def test_wide_gemm_tilings_agree(ops, dev, name, N, K, launch_policy):
    """The two wide_gemm tilings (128 and 256 weight rows per workgroup,
    policy wide_cb 1/2) compute the same GEMM: they differ only in the K split,
    i.e. in fp32 summation order."""
    from swh_trl_amd import nn_ops
    g = _gen(37)
    silu = name == "gate_up"
    M = 64
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, K // 16, 16).pow(2).sum(-1).contiguous()
    w = (torch.randn(2 * N if silu else N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    wp = nn_ops.wide_pack(w, silu=silu)
    outs = []
    for cb in ("1", "2"):
        launch_policy(wide_cb=int(cb))
        outs.append(nn_ops.wide_gemm_packed(x, wp, N, silu=silu, ss_in=ss, eps=1e-5))
        assert torch.equal(outs[-1], nn_ops.wide_gemm_packed(x, wp, N, silu=silu, ss_in=ss, eps=1e-5))
    a, b = outs[0].float(), outs[1].float()
    torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2)
    assert (a != b).float().mean().item() < 0.02



@pytest.mark.parametrize("name,N,K,silu,waves", [("gate_up", 14336, 4096, True, (8, 7)),
                                                  ("qkv", 6144, 4096, False, (8, 6)),
                                                  ("wide_res", 5376, 4096, False, (8, 7, 6)),
                                                  ("long_k_res", 5376, 14336, False, (8, 7, 6))])
def test_wide_gemm_wave_counts_agree(ops, dev, name, N, K, silu, waves, launch_policy):
    """wide_gemm with 16 W weight rows per workgroup (W = 8, 7, 6 waves: the
    launch policy's wide_waves; the default picks the count whose grid fills the
    CUs) computes the same GEMM: within bf16 output rounding of the fp32 product
    for each W, deterministic for each, differing only in the K split (fp32
    summation order); folded norm, SiLU gate, residual + partial sums."""
    from swh_trl_amd import nn_ops
    g = _gen(39)
    M = 64
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, K // 16, 16).pow(2).sum(-1).contiguous()
    rstd = torch.rsqrt(ss.sum(-1, keepdim=True) / K + 1e-5)
    w = (torch.randn(2 * N if silu else N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    wp = nn_ops.wide_pack(w, silu=silu)
    residual = name.endswith("_res")
    s0 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    prod = x.float() @ w.float().t()

    def run():
        if residual:
            s, sso = s0.clone(), torch.empty(M, N // 16, device=dev)
            nn_ops.wide_gemm_packed(x, wp, N, residual=s, ss_out=sso)
            return s, sso
        return nn_ops.wide_gemm_packed(x, wp, N, silu=silu, ss_in=ss, eps=1e-5), None

    outs = {}
    for wv in waves:
        launch_policy(wide_waves=wv)
        y, sso = run()
        y2, sso2 = run()
        assert torch.equal(y, y2) and (sso is None or torch.equal(sso, sso2)), wv
        if residual:
            ref = (s0.float() + prod.to(torch.bfloat16).float()).to(torch.bfloat16).float()
            assert (y.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 2e-2, wv
            torch.testing.assert_close(sso, y.float().view(M, N // 16, 16).pow(2).sum(-1), rtol=1e-5, atol=1e-4)
        elif silu:
            gu = (prod * rstd).to(torch.bfloat16)
            ref = torch.nn.functional.silu(gu[:, :N].float()).to(torch.bfloat16).float() * gu[:, N:].float()
            torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        else:
            torch.testing.assert_close(y.float(), prod * rstd, rtol=1e-2, atol=2e-2)
        outs[wv] = y.float()
    for wv in waves[1:]:
        assert (outs[wv] != outs[waves[0]]).float().mean().item() < 0.05, wv


@pytest.mark.parametrize("B,Hkv,G", [(64, 2, 8), (24, 2, 8), (12, 1, 4)])
def test_attn_decode_l3_warmup_is_result_neutral(ops, dev, B, Hkv, G):
    """swh_attn_decode_l3 (warm-up workgroups reading {ptr, bytes/16, 0} ranges on
    the CUs the attention leaves idle) writes exactly what swh_attn_decode_shared
    writes — output and appended K/V slot — with shared prompt rows and left
    padding, and leaves the ranges it reads unchanged."""
    from swh_trl_amd import nn_ops
    g = _gen(77 + B)
    D, P, step = 64, 40, 9
    Hq, Tmax = 7 * Hkv, P + step + 8
    plen = torch.tensor([P - (i % 5) for i in range(B // G)], dtype=torch.int32).repeat_interleave(G).to(dev)
    kc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    vc = torch.randn(B, Hkv, Tmax, D, generator=g).to(torch.bfloat16).to(dev)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, generator=g).to(torch.bfloat16).to(dev)
    cos, sin = _rope_tables(D, 2048, 1e6, dev)
    state = torch.tensor([step + 1, P], dtype=torch.int32, device=dev)
    prow = torch.arange(0, B, G, device=dev).repeat_interleave(G).to(torch.int32)
    junk = [torch.randn(n, device=dev) for n in (4, 1 << 16, 4 * 7001)]
    before = [j.clone() for j in junk]
    jobs = torch.tensor(sum([[j.data_ptr(), j.numel() * 4 // 16, 0] for j in junk], []), dtype=torch.int64).to(dev)
    sink = torch.zeros(64 * 512, dtype=torch.int32, device=dev)
    k2, v2 = kc.clone(), vc.clone()
    a = nn_ops.attn_decode(qkv, k2, v2, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, prompt_row=prow)
    k3, v3 = kc.clone(), vc.clone()
    out = torch.empty_like(a)
    nn_ops.attn_decode_l3(qkv, k3, v3, cos, sin, plen, state, Hq, Hkv, D, D ** -0.5, out, prow, False, jobs, 32, sink)
    torch.cuda.synchronize()
    assert torch.equal(a, out) and torch.equal(k2, k3) and torch.equal(v2, v3)
    assert all(torch.equal(x, y) for x, y in zip(junk, before))


# --------------------------------------------------------------------------- training projection GEMM
@pytest.mark.parametrize("M,N,K,bias", [(17408, 1152, 896, True), (300, 128, 64, False), (1000, 896, 896, True),
                                        (2048, 896, 1152, False), (1, 256, 128, True), (2048, 9728, 896, False),
                                        (4096, 4864, 896, True), (300, 256, 64, False), (700, 512, 192, True)])
def test_gemm_nt_matches_fp32_product(dev, M, N, K, bias):
    """swh_gemm_nt (the qkv / o projections of the training pass) against the
    fp32 product of the same bf16 operands: the kernel accumulates in fp32 and
    rounds once, so each element is within one bf16 rounding of the fp32
    result (2^-8 relative) plus the fp32 summation-order difference."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(11)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
    b = (torch.randn(N, generator=g) * 0.1).to(torch.bfloat16) if bias else None
    ref = x.float() @ w.float().t() + (b.float() if bias else 0)
    y = nn_ops.gemm_nt(x.to(dev), w.to(dev), b.to(dev) if bias else None).cpu().float()
    bound = ref.abs() * 2.0 ** -8 + 1e-4 * float(ref.abs().max())
    assert bool(((y - ref).abs() <= bound).all()), float(((y - ref).abs() - bound).max())


def test_gemm_nt_row_invariant_and_strided(dev):
    """A row's result does not depend on its place in the batch (fixed K order),
    and strided views (a leading dimension larger than K) give the same bits."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(12)
    x = torch.randn(700, 1024, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(256, 896, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    xs = x[:, :896]  # lda 1024
    full = nn_ops.gemm_nt(xs, w)
    perm = torch.randperm(700, generator=g).to(dev)
    shuffled = nn_ops.gemm_nt(xs.contiguous()[perm], w)
    assert torch.equal(shuffled, full[perm])
    part = nn_ops.gemm_nt(xs[129:300].contiguous(), w)
    assert torch.equal(part, full[129:300])
    out = torch.empty(700, 384, device=dev, dtype=torch.bfloat16)
    nn_ops.gemm_nt(xs, w, out=out[:, 64:320])
    assert torch.equal(out[:, 64:320], full)


@pytest.mark.parametrize("M,N,K,bias", [(17408, 9728, 896, False), (4096, 151936, 896, False), (17408, 4864, 896, True),
                                        (300, 136, 64, False), (257, 264, 128, True), (1, 8, 192, False),
                                        (513, 1000, 960, True), (2048, 896, 4864, False)])
def test_gemm_nt256_matches_fp32_product(dev, M, N, K, bias):
    """swh_gemm_nt256 (the wide training projections: gate/up forward, the lm head,
    the down input gradient) against the fp32 product of the same bf16 operands,
    within one bf16 rounding plus the fp32 summation-order difference; ragged M and
    N tiles, one- and two-tile K loops."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(13)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    b = (torch.randn(N, generator=g) * 0.1).to(torch.bfloat16).to(dev) if bias else None
    y = nn_ops.gemm_nt256(x, w, b)
    ref = x.float() @ w.float().t() + (b.float() if bias else 0)
    bound = ref.abs() * 2.0 ** -8 + 1e-4 * float(ref.abs().max())
    excess = ((y.float() - ref).abs() - bound).max()
    assert float(excess) <= 0, float(excess)


def test_gemm_nt256_row_invariant_and_strided(dev):
    """A row's result does not depend on its place in the batch or on its tile
    (fixed K order), strided operands and output views give the same bits, and the
    columns of a ragged last tile equal those of a full one."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(14)
    x = torch.randn(700, 1024, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(520, 896, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    xs = x[:, :896]  # lda 1024
    full = nn_ops.gemm_nt256(xs, w)
    perm = torch.randperm(700, generator=g).to(dev)
    assert torch.equal(nn_ops.gemm_nt256(xs.contiguous()[perm], w), full[perm])
    assert torch.equal(nn_ops.gemm_nt256(xs[129:300].contiguous(), w), full[129:300])
    assert torch.equal(nn_ops.gemm_nt256(xs, w[264:].contiguous()), full[:, 264:])
    out = torch.empty(700, 640, device=dev, dtype=torch.bfloat16)
    nn_ops.gemm_nt256(xs, w, out=out[:, 64:584])
    assert torch.equal(out[:, 64:584], full)


@pytest.mark.parametrize("M,N,K,S,dtype", [(17408, 9728, 896, 5, torch.bfloat16), (17408, 896, 4864, 10, torch.float32),
                                           (4096, 2000, 896, 1, torch.float32), (640, 272, 144, 3, torch.bfloat16),
                                           (128, 16, 16, 5, torch.float32), (64, 512, 256, 1, torch.bfloat16)])
def test_gemm_tn256_weight_gradient_matches_fp64(dev, M, N, K, S, dtype):
    """swh_gemm_tn256_partials + swh_gemm_tn_fold (the wide weight gradients) against
    grad + dY^T X in fp64 from the same bf16 operands: fp32 partial sums over token
    ranges (S larger than the 64-token steps leaves empty splits), ragged N and K
    tiles, one rounding into the gradient dtype."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(15)
    dy = (torch.randn(M, N, generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    g0 = (torch.randn(N, K, generator=g) * 0.5).to(dtype)
    ref = g0.double() + dy.double().t() @ x.double()
    grad = g0.to(dev)
    nn_ops.gemm_tn256_accumulate(grad, dy.to(dev), x.to(dev), S)
    got = grad.cpu().double()
    ulp = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -22
    bound = ref.abs() * ulp + 1e-5 * float(ref.abs().max()) * (M / 4096) ** 0.5
    excess = ((got - ref).abs() - bound).max()
    assert float(excess) <= 0, float(excess)


def test_gemm_tn256_equals_split_sums(dev):
    """The split partials are plain token-range sums: S = 1 over a range equals the
    partial of that range inside an S = 4 launch (same tokens, same order), bit for bit;
    strided operands give the same bits."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(16)
    dy = (torch.randn(1024, 576, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    xw = torch.randn(1024, 640, generator=g).to(torch.bfloat16).to(dev)
    x = xw[:, :528]  # ldx 640
    p4 = nn_ops.gemm_tn256_accumulate(torch.zeros(576, 528, device=dev), dy, x, 4).view(4, 576, 528)
    p1 = nn_ops.gemm_tn256_accumulate(torch.zeros(576, 528, device=dev), dy[256:512].contiguous(),
                                      x[256:512].contiguous(), 1).view(576, 528)
    torch.cuda.synchronize()
    assert torch.equal(p4[1], p1)


@pytest.mark.parametrize("M,N,K,S,dtype", [(17408, 1152, 896, 8, torch.bfloat16), (17408, 896, 896, 4, torch.float32),
                                           (640, 128, 256, 3, torch.bfloat16), (128, 256, 128, 5, torch.float32)])
def test_gemm_tn_weight_gradient_matches_fp32(dev, M, N, K, S, dtype):
    """swh_gemm_tn_partials + swh_gemm_tn_fold (the qkv / o weight gradients)
    against grad + dY^T X in fp64 from the same bf16 operands: fp32 partial sums
    over token ranges (S larger than the number of 64-token steps leaves empty
    splits), one rounding into the gradient dtype."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(13)
    dy = (torch.randn(M, N, generator=g) * 0.01).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    g0 = (torch.randn(N, K, generator=g) * 0.1).to(dtype)
    ref = g0.double() + dy.double().t() @ x.double()
    gd = g0.to(dev)
    b0 = (torch.randn(N, generator=g) * 0.1).to(dtype)
    bd = b0.to(dev)
    part = nn_ops.gemm_tn_accumulate(gd, dy.to(dev), x.to(dev), S, bias_grad=bd)
    torch.cuda.synchronize()
    del part
    got = gd.cpu().double()
    ulp = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -23
    scale = (dy.double().abs().t() @ x.double().abs())  # bound of the fp32 summation error
    bound = ref.abs() * ulp + scale * 2.0 ** -22 * (M / S + S) + 1e-12
    assert bool(((got - ref).abs() <= bound).all()), float(((got - ref).abs() - bound).max())
    # the bias gradient from the same kernel (the split's token sums of dY, folded in split
    # order as swh_rmsnorm_dw_accum folds: bf16(grad + bf16(sum)) for bf16, grad + sum for f32)
    cs = dy.double().sum(0)
    bref = b0.double() + cs
    bgot = bd.cpu().double()
    bscale = dy.double().abs().sum(0)
    bbound = bref.abs() * 2 * ulp + (cs.abs() * ulp if dtype == torch.bfloat16 else 0) + bscale * 2.0 ** -22 * (M / S + S) + 1e-12
    assert bool(((bgot - bref).abs() <= bbound).all()), float(((bgot - bref).abs() - bbound).max())


def test_gemm_tn_partials_row_order_and_splits(dev):
    """Tokens enter in a fixed order: the same tokens give the same partial bits,
    and S = 1 equals the fp32 sum of an S = 2 split up to the fold's rounding."""
    from swh_trl_amd import _lib, nn_ops
    _lib.load()
    g = _gen(14)
    dy = (torch.randn(1024, 256, generator=g) * 0.01).to(torch.bfloat16).to(dev)
    x = torch.randn(1024, 384, generator=g).to(torch.bfloat16).to(dev)
    a = torch.zeros(256, 384, device=dev)
    b = torch.zeros(256, 384, device=dev)
    nn_ops.gemm_tn_accumulate(a, dy, x, 1)
    nn_ops.gemm_tn_accumulate(b, dy, x, 1)
    assert torch.equal(a, b)
    c = torch.zeros(256, 384, device=dev)
    nn_ops.gemm_tn_accumulate(c, dy, x, 2)
    torch.testing.assert_close(c, a, rtol=1e-5, atol=1e-6)


def test_two_threads_with_different_policies_keep_their_own_results(ops, dev):
    """The launch policy is per host thread: two threads launching the same
    wide_gemm concurrently on their own streams, one under wide_smax 1 (no K
    split) and one under wide_smax 8 (the qkv shape split over workgroups, so
    another fp32 summation order), each reproduce bit for bit the result their
    policy gives single-threaded, every repetition."""
    import threading

    from swh_trl_amd import _lib, nn_ops
    g = _gen(41)
    M, N, K = 64, 6144, 4096
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    ss = x.float().view(M, K // 16, 16).pow(2).sum(-1).contiguous()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    wp = nn_ops.wide_pack(w)
    want = {}
    for cb in (1, 8):
        with _lib.launch_policy(wide_smax=cb):
            want[cb] = nn_ops.wide_gemm_packed(x, wp, N, ss_in=ss, eps=1e-5)
    torch.cuda.synchronize()
    assert not torch.equal(want[1], want[8])  # the policies do change the bits
    errors, outs = [], {1: [], 8: []}
    barrier = threading.Barrier(2, timeout=60)

    def worker(cb):
        try:
            torch.cuda.set_device(dev)
            _lib.set_launch_policy(wide_smax=cb)
            st = torch.cuda.Stream(device=dev)
            barrier.wait()
            with torch.cuda.stream(st):
                for _ in range(20):
                    outs[cb].append(nn_ops.wide_gemm_packed(x, wp, N, ss_in=ss, eps=1e-5))
            st.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(cb,)) for cb in (1, 8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    for cb in (1, 8):
        assert len(outs[cb]) == 20 and all(torch.equal(o, want[cb]) for o in outs[cb]), cb
    assert _lib.get_launch_policy()["wide_smax"] == 8  # the main thread kept its own (default) policy
