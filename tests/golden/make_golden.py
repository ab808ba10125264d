"""Writes the golden fixtures under tests/golden/ (run: python tests/golden/make_golden.py).

reference_kats.json — known-answer tests held by the reference's OWN test-suite,
transcribed as data (inputs + expected outputs), each with its source file:line.
No reference code is imported or executed.

philox_kat.json — the published Philox4x32-10 known-answer vectors
(Salmon et al. SC'11, Random123 distribution) that pin the sampler RNG oracle.

restatement_vectors.npz — small seeded vectors produced by the CPU restatement
(`oracle/`) itself.  LABEL: restatement-derived, parity unpinned by reference
tests; they freeze the oracle's behaviour so later edits cannot drift silently.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import trl_ref  # noqa: E402


def reference_kats():
    k = {}
    # tests/test_core.py:22-46
    k["masked_stats"] = {
        "source": "tests/test_core.py:22-46",
        "values": [1.0, 2.0, 3.0, 4.0], "mask": [0.0, 1.0, 1.0, 0.0],
        "expected_mean": 2.5, "expected_var_unbiased": 0.5,
        "whiten_slice": [1, 3], "whiten_tol": 1e-5,
        "expected_whiten_slice": [-0.7071067690849304, 0.7071067690849304],
    }
    # tests/test_grpo_trainer.py:153-160
    k["repeat_sampler_no_shuffle"] = {
        "source": "tests/test_grpo_trainer.py:153-160",
        "n": 7, "mini_repeat_count": 2, "batch_size": 1, "repeat_count": 1,
        "expected": [0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6],
    }
    # tests/test_grpo_trainer.py:142-251 — structural properties (random order)
    k["repeat_sampler_props"] = {
        "source": "tests/test_grpo_trainer.py:142-251",
        "cases": [
            {"n": 7, "mini": 2, "bs": 1, "rep": 1, "len": 14},
            {"n": 7, "mini": 1, "bs": 1, "rep": 1, "len": 7},
            {"n": 8, "mini": 1, "bs": 2, "rep": 2, "len": 16},
            {"n": 7, "mini": 1, "bs": 2, "rep": 2, "len": 12},
            {"n": 7, "mini": 2, "bs": 3, "rep": 2, "len": 24},
            {"n": 7, "mini": 3, "bs": 2, "rep": 2, "len": 36},
            {"n": 7, "mini": 2, "bs": 2, "rep": 3, "len": 36},
        ],
    }
    # tests/test_grpo_trainer.py:254-386
    k["truncate_with_protected_tokens"] = {
        "source": "tests/test_grpo_trainer.py:254-386",
        "cases": [
            {"ids": [[1, 2, 3, 4, 5], [6, 7, 8, 9, 10]], "mask": None, "protected": [2, 3, 6], "target": 3,
             "expected_ids": [[2, 3, 5], [6, 9, 10]], "expected_mask": [[1, 1, 1], [1, 1, 1]]},
            {"ids": [[1, 2, 3]], "mask": None, "protected": [2], "target": 3,
             "expected_ids": [[1, 2, 3]], "expected_mask": [[1, 1, 1]]},
            {"ids": [[1, 2, 3, 4, 5]], "mask": None, "protected": [], "target": 3,
             "expected_ids": [[3, 4, 5]], "expected_mask": None},
            {"ids": [[1, 2, 3, 4, 5]], "mask": None, "protected": [3, 4, 5], "target": 3,
             "expected_ids": [[3, 4, 5]], "expected_mask": None},
            {"ids": [[1, 2, 3, 4, 5]], "mask": None, "protected": [1, 2, 3, 4], "target": 3,
             "raises": "ValueError"},
            {"ids": [[5]], "mask": None, "protected": [5], "target": 1,
             "expected_ids": [[5]], "expected_mask": None},
            {"ids": [[1, 2, 3, 4, 5]], "mask": [[1, 0, 1, 0, 1]], "protected": [2, 4], "target": 3,
             "expected_ids": [[2, 4, 5]], "expected_mask": [[0, 0, 1]]},
            {"ids": [[1, 2, 3, 4, 5], [2, 6, 7, 8, 9], [10, 11, 12, 2, 13]], "mask": None, "protected": [2],
             "target": 3, "expected_ids": [[2, 4, 5], [2, 8, 9], [12, 2, 13]], "expected_mask": None},
            {"ids": [[10, 2, 20, 3, 30, 40]], "mask": None, "protected": [2, 3], "target": 4,
             "expected_ids": [[2, 3, 30, 40]], "expected_mask": None},
            {"ids": [[1, 2, 3, 4, 5]], "mask": None, "protected": [], "target": 2,
             "expected_ids": [[4, 5]], "expected_mask": None},
        ],
    }
    # tests/test_grpo_trainer.py:389-440
    e1 = [[0.1, 0.2, 0.3, 0.4, 0.5, 0.6], [0.7, 0.8, 0.9, 1.0, 1.1, 1.2]]
    m1 = [[1, 1, 1, 1, 1, 1], [1, 1, 1, 1, 0, 0]]
    k["high_entropy_mask"] = {
        "source": "tests/test_grpo_trainer.py:389-440",
        "cases": [
            {"entropies": e1, "mask": m1, "threshold": 0.8,
             "expected": [[0, 0, 0, 0, 0, 0], [0, 0, 1, 1, 0, 0]]},
            {"entropies": [[0.1, 0.2, 0.3, 1.4, 0.5, 0.14], [0.5, 0.6, 0.7, 0.8, 0.9, 1.0]],
             "mask": [[1, 1, 1, 1, 0, 0], [1, 1, 1, 1, 0, 0]], "threshold": 0.8,
             "expected": [[0, 0, 0, 1, 0, 0], [0, 0, 0, 1, 0, 0]]},
            {"entropies": e1, "mask": m1, "threshold": 0.5,
             "expected": [[0, 0, 0, 0, 0, 1], [1, 1, 1, 1, 0, 0]]},
            {"entropies": e1, "mask": m1, "threshold": 0.0, "expected": m1},
            {"entropies": e1, "mask": m1, "threshold": 1.0,
             "expected": [[0, 0, 0, 0, 0, 0], [0, 0, 0, 1, 0, 0]]},
            {"entropies": e1, "mask": [[0] * 6, [0] * 6], "threshold": 0.5, "expected": [[0] * 6, [0] * 6]},
        ],
    }
    # tests/test_grpo_trainer.py:1308-1327 (mocked generate output) + SURVEY.md §8c derived masks
    k["mock_completion_masks"] = {
        "source": "tests/test_grpo_trainer.py:1315-1325",
        "pad": 151643, "eos": 151645,
        "completion_ids": [[1, 2, 3, 4, 5, 6, 7, 8],
                           [9, 10, 11, 151645, 151643, 151643, 151643, 151643],
                           [12, 13, 14, 15, 16, 17, 18, 151645]],
        "expected_mask": [[1] * 8, [1, 1, 1, 1, 0, 0, 0, 0], [1] * 8],
        "expected_mask_truncated": [[0] * 8, [1, 1, 1, 1, 0, 0, 0, 0], [1] * 8],
    }
    # tests/test_utils.py:540-558 and :622-640 — shapes and tolerances of the op tests
    k["selective_log_softmax_spec"] = {
        "source": "tests/test_utils.py:540-558", "shape": [4, 32, 1024],
        "lowp_bit_exact": True, "fp32_rtol": 1e-5, "fp32_atol": 1e-5,
    }
    k["entropy_spec"] = {
        "source": "tests/test_utils.py:622-640", "shape": [64, 384, 768], "rtol": 1e-5, "atol": 1e-5,
        "chunk_sizes": [1, 16],
    }
    return k


def philox_kats():
    return {
        "source": "Philox4x32-10 known-answer vectors, Random123 kat_vectors (Salmon et al. SC'11)",
        "cases": [
            {"ctr": ["00000000"] * 4, "key": ["00000000"] * 2,
             "out": ["6627e8d5", "e169c58d", "bc57ac4c", "9b00dbd8"]},
            {"ctr": ["ffffffff"] * 4, "key": ["ffffffff"] * 2,
             "out": ["408f276d", "41c83b0e", "a20bc7c6", "6d5451fd"]},
            {"ctr": ["243f6a88", "85a308d3", "13198a2e", "03707344"], "key": ["a4093822", "299f31d0"],
             "out": ["d16cfe09", "94fdcceb", "5001e420", "24126ea1"]},
        ],
    }


def restatement_vectors():
    g = torch.Generator().manual_seed(1234)
    out = {}
    logits = torch.randn(2, 16, 512, generator=g, dtype=torch.float64)
    ids = torch.randint(0, 512, (2, 16), generator=g)
    out["lse_logits"] = logits.numpy()
    out["lse_ids"] = ids.numpy()
    out["lse_logp"] = trl_ref.selective_log_softmax(logits, ids).numpy()
    out["lse_entropy"] = trl_ref.entropy_from_logits(logits).numpy()
    rpf = torch.rand(32, 2, generator=g, dtype=torch.float64)
    rpf[3, 1] = float("nan")
    w = torch.tensor([1.0, 0.5], dtype=torch.float64)
    adv, r, mean, std, zero = trl_ref.group_advantages(rpf, w, 8, True)
    out["adv_rpf"], out["adv_w"], out["adv_out"] = rpf.numpy(), w.numpy(), adv.numpy()
    lp = (torch.rand(8, 16, generator=g, dtype=torch.float64) * -3).requires_grad_(True)
    old = lp.detach() + 0.3 * torch.randn(8, 16, generator=g, dtype=torch.float64)
    ref = lp.detach() + 0.2 * torch.randn(8, 16, generator=g, dtype=torch.float64)
    a = torch.randn(8, generator=g, dtype=torch.float64)
    m = (torch.rand(8, 16, generator=g) > 0.2).int()
    loss, _ = trl_ref.grpo_loss(lp, a, m, old, ref, beta=0.04, loss_type="bnpo")
    loss.backward()
    out["loss_lp"], out["loss_old"], out["loss_ref"] = lp.detach().numpy(), old.numpy(), ref.numpy()
    out["loss_adv"], out["loss_mask"] = a.numpy(), m.numpy()
    out["loss_value"], out["loss_grad"] = np.array(loss.item()), lp.grad.numpy()
    return out


def main():
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(reference_kats(), f, indent=1)
    with open(os.path.join(HERE, "philox_kat.json"), "w") as f:
        json.dump(philox_kats(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "restatement_vectors.npz"), **restatement_vectors())
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
