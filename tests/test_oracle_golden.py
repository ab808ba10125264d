"""The CPU oracle checked against the reference's own known-answer tests (no GPU)."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest
import torch

from oracle import hf_sampling, trl_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def kats(golden_dir):
    with open(os.path.join(golden_dir, "reference_kats.json")) as f:
        return json.load(f)


def test_masked_stats(kats):
    k = kats["masked_stats"]
    x, m = torch.tensor(k["values"]), torch.tensor(k["mask"])
    assert trl_ref.masked_mean(x, m).item() == k["expected_mean"]
    assert trl_ref.masked_var(x, m).item() == pytest.approx(k["expected_var_unbiased"], abs=0)
    w = trl_ref.masked_whiten(x, m)[k["whiten_slice"][0]:k["whiten_slice"][1]]
    assert abs((w - torch.tensor(k["expected_whiten_slice"])).sum().item()) < k["whiten_tol"]


def test_masked_var_zero_mask_raises():
    with pytest.raises(ValueError):
        trl_ref.masked_var(torch.ones(3), torch.zeros(3))


def test_repeat_sampler_no_shuffle(kats):
    k = kats["repeat_sampler_no_shuffle"]
    got = trl_ref.repeat_sampler_indices(k["n"], k["mini_repeat_count"], k["batch_size"], k["repeat_count"],
                                         shuffle=False)
    assert got == k["expected"]


def test_repeat_sampler_props(kats):
    for c in kats["repeat_sampler_props"]["cases"]:
        got = trl_ref.repeat_sampler_indices(c["n"], c["mini"], c["bs"], c["rep"], shuffle=True, seed=42)
        assert len(got) == c["len"]
        assert set(got).issubset(range(c["n"]))
        per_chunk = c["bs"] * c["mini"]
        for s in range(0, len(got), per_chunk * c["rep"]):
            blk = got[s:s + per_chunk]
            for r in range(1, c["rep"]):
                assert got[s + r * per_chunk:s + (r + 1) * per_chunk] == blk
        for s in range(0, len(got), c["mini"]):
            assert len(set(got[s:s + c["mini"]])) == 1


def test_truncate_with_protected_tokens(kats):
    for c in kats["truncate_with_protected_tokens"]["cases"]:
        ids = torch.tensor(c["ids"])
        mask = torch.tensor(c["mask"]) if c["mask"] is not None else torch.ones_like(ids)
        if c.get("raises"):
            with pytest.raises(ValueError):
                trl_ref.truncate_with_protected_tokens(ids, mask, c["target"], c["protected"])
            continue
        ni, nm = trl_ref.truncate_with_protected_tokens(ids, mask, c["target"], c["protected"])
        assert torch.equal(ni, torch.tensor(c["expected_ids"]))
        if c["expected_mask"] is not None:
            assert torch.equal(nm, torch.tensor(c["expected_mask"]))


def test_high_entropy_mask(kats):
    for c in kats["high_entropy_mask"]["cases"]:
        got = trl_ref.get_high_entropy_mask(torch.tensor(c["entropies"]), torch.tensor(c["mask"]), c["threshold"])
        assert torch.equal(got, torch.tensor(c["expected"], dtype=torch.bool))


def test_mock_completion_masks(kats):
    k = kats["mock_completion_masks"]
    ids = torch.tensor(k["completion_ids"])
    m, lengths, _ = trl_ref.completion_mask_from_eos(ids, k["eos"])
    assert torch.equal(m, torch.tensor(k["expected_mask"], dtype=torch.int32))
    assert lengths.tolist() == [8, 4, 8]
    mt, _, _ = trl_ref.completion_mask_from_eos(ids, k["eos"], mask_truncated=True)
    assert torch.equal(mt, torch.tensor(k["expected_mask_truncated"], dtype=torch.int32))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16, torch.bfloat16])
def test_selective_log_softmax_spec(kats, dtype):
    spec = kats["selective_log_softmax_spec"]
    g = torch.Generator().manual_seed(0)
    b, t, v = spec["shape"]
    ids = torch.randint(0, v, (b, t), generator=g)
    logits = torch.randn(b, t, v, generator=g).to(dtype)
    exp = torch.gather(logits.log_softmax(-1), -1, ids.unsqueeze(-1)).squeeze(-1)
    got = trl_ref.selective_log_softmax(logits, ids)
    if dtype in (torch.float16, torch.bfloat16):
        assert torch.equal(got, exp)
    else:
        torch.testing.assert_close(got, exp, rtol=spec["fp32_rtol"], atol=spec["fp32_atol"])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.bfloat16])
def test_entropy_spec(kats, dtype):
    spec = kats["entropy_spec"]
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(8, 48, spec["shape"][2], generator=g).to(dtype)  # reduced rows, same V
    if dtype in (torch.float64, torch.float32):
        p = logits.softmax(-1)
        exp = -(p * p.log()).sum(-1)
    else:
        lp = logits.log_softmax(-1)
        exp = -(lp.exp() * lp).sum(-1)
    got = trl_ref.entropy_from_logits(logits, chunk_size=16)
    torch.testing.assert_close(got, exp, rtol=spec["rtol"], atol=spec["atol"])


def test_restatement_vectors_frozen(golden_dir):
    z = np.load(os.path.join(golden_dir, "restatement_vectors.npz"))
    logits, ids = torch.from_numpy(z["lse_logits"]), torch.from_numpy(z["lse_ids"])
    np.testing.assert_allclose(trl_ref.selective_log_softmax(logits, ids).numpy(), z["lse_logp"], rtol=1e-12)
    np.testing.assert_allclose(trl_ref.entropy_from_logits(logits).numpy(), z["lse_entropy"], rtol=1e-12)
    adv = trl_ref.group_advantages(torch.from_numpy(z["adv_rpf"]), torch.from_numpy(z["adv_w"]), 8, True)[0]
    np.testing.assert_allclose(adv.numpy(), z["adv_out"], rtol=1e-12)
    lp = torch.from_numpy(z["loss_lp"]).requires_grad_(True)
    loss, _ = trl_ref.grpo_loss(lp, torch.from_numpy(z["loss_adv"]), torch.from_numpy(z["loss_mask"]),
                                torch.from_numpy(z["loss_old"]), torch.from_numpy(z["loss_ref"]), beta=0.04)
    loss.backward()
    np.testing.assert_allclose(loss.item(), z["loss_value"], rtol=1e-12)
    np.testing.assert_allclose(lp.grad.numpy(), z["loss_grad"], rtol=1e-12)


def _oracle_lib():
    so = os.path.join(ROOT, "oracle", "_build", "libswh_oracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return ctypes.CDLL(so)


def test_philox_kat(golden_dir):
    lib = _oracle_lib()
    with open(os.path.join(golden_dir, "philox_kat.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        ctr = (ctypes.c_uint32 * 4)(*[int(x, 16) for x in c["ctr"]])
        key = (ctypes.c_uint32 * 2)(*[int(x, 16) for x in c["key"]])
        out = (ctypes.c_uint32 * 4)()
        lib.swh_ref_philox4x32_10(ctr, key, out)
        assert ["%08x" % x for x in out] == c["out"]


def test_hf_processors_semantics():
    s = torch.tensor([[1.0, 2.0, 3.0, 4.0, -1.0]])
    assert (~torch.isinf(hf_sampling.top_k(s, 2))).tolist() == [[False, False, True, True, False]]
    kept = ~torch.isinf(hf_sampling.top_p(s, 0.5))
    assert kept.tolist() == [[False, False, False, True, False]]
    seen = torch.tensor([[True, False, False, False, True]])
    rp = hf_sampling.repetition_penalty(s, seen, 2.0)
    assert rp.tolist() == [[0.5, 2.0, 3.0, 4.0, -2.0]]
    mp = hf_sampling.min_p(s, 0.3)
    assert (~torch.isinf(mp)).tolist() == [[False, False, True, True, False]]


def test_gae_matches_closed_form():
    g = torch.Generator().manual_seed(3)
    r = torch.randn(3, 7, generator=g, dtype=torch.float64)
    v = torch.randn(3, 7, generator=g, dtype=torch.float64)
    adv, ret = trl_ref.gae(r, v, 0.9, 0.8)
    # closed form: A_t = sum_l (gamma*lam)^l delta_{t+l}
    d = r + 0.9 * torch.cat([v[:, 1:], torch.zeros(3, 1, dtype=torch.float64)], 1) - v
    exp = torch.zeros_like(d)
    for t in range(7):
        for l in range(7 - t):
            exp[:, t] += (0.72 ** l) * d[:, t + l]
    torch.testing.assert_close(adv, exp)
    torch.testing.assert_close(ret, adv + v)


def test_adamw_oracle_matches_torch():
    g = torch.Generator().manual_seed(5)
    p0 = torch.randn(100, generator=g, dtype=torch.float64)
    grads = [torch.randn(100, generator=g, dtype=torch.float64) for _ in range(3)]
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([p], lr=1e-2, weight_decay=0.1, foreach=False)
    q, m, v = p0.clone(), torch.zeros(100, dtype=torch.float64), torch.zeros(100, dtype=torch.float64)
    for step, gr in enumerate(grads, 1):
        p.grad = gr.clone()
        opt.step()
        q, m, v = trl_ref.adamw_step(q, gr, m, v, step, 1e-2, weight_decay=0.1)
    torch.testing.assert_close(p.detach(), q, rtol=1e-12, atol=1e-12)


def test_pad_kats(kats):
    """TestPad (test_utils.py:51-133): the oracle's pad() and the product's."""
    from swh_trl_amd.trainer.utils import pad
    for c in kats["pad"]["cases"]:
        xs = [torch.tensor(x) for x in c["inputs"]]
        kw = dict(padding_value=c["padding_value"], padding_side=c["padding_side"],
                  pad_to_multiple_of=c["pad_to_multiple_of"])
        assert trl_ref.pad(xs, **kw).tolist() == c["expected"]
        assert pad(xs, **kw).tolist() == c["expected"]


def _hf_chain(ids, scores, *, rep, eos, min_new, cur_new, t, k, p, mp):
    """The installed transformers processors in `_get_logits_processor` order
    (repetition penalty, min-new-tokens, temperature, top-k, top-p, min-p),
    each added under the same condition generation/utils.py uses."""
    from transformers.generation import logits_process as lp
    procs = []
    if rep is not None and rep != 1.0:
        procs.append(lp.RepetitionPenaltyLogitsProcessor(penalty=rep))
    if min_new:
        procs.append(lp.MinNewTokensLengthLogitsProcessor(prompt_length_to_skip=ids.shape[1] - cur_new,
                                                          min_new_tokens=min_new, eos_token_id=eos))
    if t is not None and t != 1.0:
        procs.append(lp.TemperatureLogitsWarper(t))
    if k:
        procs.append(lp.TopKLogitsWarper(top_k=k))
    if p is not None and p < 1.0:
        procs.append(lp.TopPLogitsWarper(top_p=p))
    if mp is not None:
        procs.append(lp.MinPLogitsWarper(min_p=mp))
    s = scores.clone()
    for pr in procs:
        s = pr(ids, s)
    return s


@pytest.mark.parametrize("rep,min_new,t,k,p,mp", [
    (1.0, 0, 1.0, None, 1.0, None), (1.3, 0, 1.0, None, 1.0, None), (1.0, 5, 1.0, None, 1.0, None),
    (1.0, 0, 0.7, None, 1.0, None), (1.0, 0, 1.0, 50, 1.0, None), (1.0, 0, 1.0, None, 0.9, None),
    (1.0, 0, 1.0, None, 1.0, 0.05), (1.2, 5, 0.8, 40, 0.9, None), (0.8, 5, 1.3, 100, 0.95, 0.02),
    (1.1, 0, 0.6, 7, 0.5, 0.1)])
def test_hf_sampling_matches_transformers_processors(rep, min_new, t, k, p, mp):
    """Pins oracle/hf_sampling.process_scores to the installed transformers
    logits processors (third-party arithmetic) on random fp32
    logits, for each flag and their combination; input_ids hold left pads, which
    the repetition penalty counts like any other id."""
    g = torch.Generator().manual_seed(int(rep * 100 + min_new + t * 10 + (k or 0) + p * 7 + (mp or 0) * 1000))
    B, V, L = 6, 997, 24
    scores = torch.randn(B, V, generator=g) * 3
    ids = torch.randint(0, V, (B, L), generator=g)
    ids[:2, :5] = 0  # left pads (pad id 0)
    eos = [3, 11]
    cur_new = 2
    exp = _hf_chain(ids, scores, rep=rep, eos=eos, min_new=min_new, cur_new=cur_new, t=t, k=k, p=p, mp=mp)
    seen = torch.zeros(B, V, dtype=torch.bool).scatter_(1, ids, True)
    got = hf_sampling.process_scores(scores, seen=seen, rep_penalty=rep, eos_ids=eos,
                                     suppress_eos_now=bool(min_new) and cur_new < min_new, t=t, k=k, p=p, mp=mp)
    assert torch.equal(torch.isinf(got), torch.isinf(exp))
    fin = ~torch.isinf(exp)
    torch.testing.assert_close(got[fin], exp[fin], rtol=1e-6, atol=1e-6)
