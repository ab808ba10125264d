"""Diagnose the PPO update schedule at the Qwen2.5-0.5B width (tuning aid, not
part of the product): per optimizer step, every gradient tensor's relative
error against the oracle at the product's own weights (bf16 and fp32 oracle),
and the product's forward log-probs at the final weights against the fp32
oracle's.

    python tools/ppo_step_probe.py [tiny|qwen2.5-0.5b-width] [lr]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _env  # noqa: E402  (tools only: A/B switches from the environment)
_env.apply()

import test_ppo_gpu as T  # noqa: E402
from oracle import ppo_step, trl_ref  # noqa: E402


def main(width, lr):
    dev = torch.device("cuda:0")
    tr, ds = T._trainer(dev, width=width, learning_rate=lr)
    a = tr.args
    queries = tr._queries(ds[:a.local_batch_size])
    responses, logprobs = tr.generate(queries)
    ro = tr.rollout_from(queries, responses, logprobs)
    perms = [torch.randperm(a.local_batch_size, generator=torch.Generator().manual_seed(e)).tolist()
             for e in range(a.num_ppo_epochs)]
    oro = T._cpu(ro)
    oro["values"] = oro["values"].float()
    steps = []
    step_fn = tr._optimizer_step

    def snap(m):
        return {k: v.detach().cpu().clone() for k, v in m.hf_state_dict().items()}

    def capture(lr):
        steps.append((snap(tr.policy_model), snap(tr.value_model), T._grads(tr.policy_model),
                      T._grads(tr.value_model)))
        return step_fn(lr)

    tr._optimizer_step = capture
    tr.ppo_update(ro, a.learning_rate, permutations=perms)
    minis = T._sync_groups(a, perms, False)  # the micro-batches between the reference's optimizer steps
    models = {dt: (T._hf(tr.policy_model, False).to(dt), T._hf(tr.value_model, True).to(dt))
              for dt in (torch.bfloat16, torch.float32)}
    kw = dict(context_length=queries.shape[1], pad_token_id=T.PAD, temperature=a.temperature,
              cliprange=a.cliprange, cliprange_value=a.cliprange_value, vf_coef=a.vf_coef)
    for s, ((wp, wv, gp, gv), mini) in enumerate(zip(steps, minis)):
        grads, stats = {}, {}
        for dt, (pol, val) in models.items():
            pol.load_state_dict(wp, strict=False)
            val.load_state_dict(wv, strict=False)
            pol.zero_grad(set_to_none=True)
            val.zero_grad(set_to_none=True)
            stats[dt] = ppo_step.mini_batch_backward(pol, val, oro, mini,
                                                     per_device_train_batch_size=a.per_device_train_batch_size,
                                                     gradient_accumulation_steps=a.gradient_accumulation_steps, **kw)
            grads[dt] = (T._hf_grads(pol), T._hf_grads(val))
        print(f"step {s}: oracle fp32 stats", [{k: round(v, 5) for k, v in st.items() if k != "tokens"}
                                               for st in stats[torch.float32]])
        for side, (prod, ob, of) in (("policy", (gp, grads[torch.bfloat16][0], grads[torch.float32][0])),
                                     ("value", (gv, grads[torch.bfloat16][1], grads[torch.float32][1]))):
            for k, g32 in of.items():
                n32 = g32.norm().clamp_min(1e-20)
                rel_ref = float((ob[k] - g32).norm() / n32)
                rel_p = float((prod[k] - g32).norm() / n32)
                flag = "  <-- over" if rel_p > 2 * rel_ref + T.BF16_TOL else ""
                if flag or "layers.0.self_attn.q_proj.weight" in k or "embed" in k or "score" in k:
                    print(f"  {side:6s} {k:48s} |g| {float(g32.norm()):.3e} prod {rel_p:.4f} ref {rel_ref:.4f}{flag}")
    # forward at the final weights: product vs fp32 oracle
    pol32 = T._hf(tr.policy_model, False)
    qr = ro["query_responses"]
    ids, mask, pos = __import__("swh_trl_amd.trainer.ppo_trainer", fromlist=["_forward_inputs"])._forward_inputs(
        qr, tr.pad_token_id)
    P, Tn = queries.shape[1], ro["responses"].shape[1]
    with torch.no_grad():
        hp = tr.policy_model.hidden_states(ids, positions=pos, key_mask=mask)
        lp, _ = tr.policy_model.logp_entropy(hp[:, P - 1:P + Tn - 1], ro["responses"], a.temperature + 1e-7, True)
        out = ppo_step.forward(pol32, qr.cpu(), T.PAD)
        lg = out.logits[:, P - 1:-1] / (a.temperature + 1e-7)
        lp32 = trl_ref.selective_log_softmax(lg, ro["responses"].cpu())
    keep = ~ro["padding_mask"].cpu()
    d = (lp.float().cpu() - lp32)[keep].abs()
    print(f"final-weights forward: |product - fp32| max {float(d.max()):.4f} mean {float(d.mean()):.5f}")
    d0 = (ro["logprobs"].float().cpu() - lp32)[keep].abs()
    print(f"final vs rollout logprobs (how far the policy moved): max {float(d0.max()):.4f} mean {float(d0.mean()):.4f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "qwen2.5-0.5b-width", float(sys.argv[2]) if len(sys.argv) > 2 else 1e-5)
