"""PPOTrainer — drop-in for trl.PPOTrainer's training loop on MI355X.

Constructor and config keep the reference's names (ppo_trainer.py:102-119,
ppo_config.py); `train()` keeps the semantics of ppo_trainer.py:347-646 while
every per-token stage runs on the HIP engine:

  rollout       DecodeEngine.generate, log-probs of the drawn tokens from the
                sampler's processed fp32 scores (utils.py:1094, :1119 — the
                reference's `selective_log_softmax(logitss, response)`)
  ref log-prob  no-grad full forward -> fused lm head + log-prob kernel
  value / score score-head forwards (get_reward, utils.py:900-947)
  rewards       KL-shaped token rewards + score at the sequence end (:496-516)
  whiten / GAE  ops.masked_whiten, ops.gae (reverse scan kernel) (:518-535)
  update        num_ppo_epochs x mini-batches x GA micro-batches: policy and
                value forwards, fused clipped PG + value loss fwd/bwd kernel,
                flat-buffer AdamW per mini-batch (:537-617), RCCL all-reduce
                of both models' gradients for DP

Out of scope: PEFT adapters, DeepSpeed, sample-generation
tables, hub pushes, checkpoints.
"""
from __future__ import annotations

import math
import os
import time
from collections import defaultdict
from typing import Optional

import numpy as np
import torch

from .. import dist as swh_dist
from .. import gemm_tuning
from .. import ops
from ..engine import build_engine, build_model
from ..engine.decode import DecodeEngine
from ..engine.model import CausalLM, dw_sync
from ..optim import FlatAdamW
from . import schedule
from .callbacks import CallbackHandler, new_state
from .grpo_trainer import _trace, load_model, model_dtype
from .ppo_config import PPOConfig
from .utils import left_pad

INVALID_LOGPROB = 1.0  # ppo_trainer.py:81


def exact_div(a: int, b: int, msg: str) -> int:
    """trl/trainer/utils.py exact_div."""
    q = a // b
    if a != q * b:
        raise ValueError(f"{msg}, {a} / {b} = {a / b}")
    return q


def fill_batch_sizes(args: PPOConfig, dataset_len: int, world_size: int) -> PPOConfig:
    """ppo_trainer.py:224-250: the derived batch sizes, in place."""
    if args.total_episodes is None:
        args.total_episodes = int(args.num_train_epochs * dataset_len)
    args.world_size = world_size
    args.local_batch_size = args.per_device_train_batch_size * args.gradient_accumulation_steps
    args.micro_batch_size = int(args.per_device_train_batch_size * args.world_size)
    args.batch_size = int(args.local_batch_size * args.world_size)
    args.mini_batch_size = exact_div(args.batch_size, args.num_mini_batches,
                                     "`batch_size` must be a multiple of `num_mini_batches`")
    args.local_mini_batch_size = exact_div(args.local_batch_size, args.num_mini_batches,
                                           "`local_batch_size` must be a multiple of `num_mini_batches`")
    if args.whiten_rewards and args.local_mini_batch_size < 8:
        raise ValueError(f"Per-rank minibatch size {args.local_mini_batch_size} is insufficient for whitening")
    args.num_total_batches = math.ceil(args.total_episodes / args.batch_size)
    return args


def first_true_indices(bools: torch.Tensor, dtype=torch.long) -> torch.Tensor:
    """utils.py:877-897: per row, the index of the first True, or the row
    length when there is none (argmax returns the first maximum)."""
    first = bools.to(torch.uint8).argmax(-1)
    return torch.where(bools.any(-1), first, bools.size(-1)).to(dtype)


def truncate_response(stop_token_id: int, pad_token_id: int, responses: torch.Tensor) -> torch.Tensor:
    """utils.py:1036-1056: every token after the first stop token becomes pad.
    Device tensors: one kernel (ops.ppo_truncate); host tensors (tests, data
    prep): the same rule in torch."""
    if responses.is_cuda:
        return ops.ppo_truncate(responses, stop_token_id, pad_token_id)[0]
    cut = first_true_indices(responses == stop_token_id)
    after = torch.arange(responses.shape[1], device=responses.device) > cut.unsqueeze(1)
    return torch.where(after, torch.full_like(responses, pad_token_id), responses)


def _forward_inputs(query_responses: torch.Tensor, pad_token_id: int):
    """utils.py:900-979 `forward` / `get_reward` inputs: mask = ids != pad,
    exclusive-cumsum positions, pad ids replaced by 0."""
    attention_mask = query_responses != pad_token_id
    position_ids = attention_mask.cumsum(1) - attention_mask.long()
    input_ids = torch.masked_fill(query_responses, ~attention_mask, 0)
    return input_ids, attention_mask, position_ids


class PPOTrainer:
    _tag_names = ["trl", "ppo"]

    def __init__(self, args: PPOConfig, processing_class, model, ref_model, reward_model, train_dataset,
                 value_model, data_collator=None, eval_dataset=None, optimizers=(None, None), callbacks=None,
                 peft_config=None):
        if ref_model is model and model is not None:
            raise ValueError("`model` and `ref_model` cannot be the same object. If you want `ref_model` to be the "
                             "same as `model`, you must make a copy of it, or `None` if you use peft.")
        if peft_config is not None:
            raise ValueError("peft_config: LoRA training is not part of the MI355X engine's scope")
        if optimizers is not None and any(o is not None for o in optimizers):
            raise ValueError("optimizers: the MI355X trainer updates policy and value with the fused AdamW kernel, "
                             "configured by the PPOConfig fields (learning_rate, adam_beta1/2, adam_epsilon, "
                             "weight_decay, lr_scheduler_type, lr_scheduler_kwargs, warmup_steps / warmup_ratio); a "
                             "torch optimizer or scheduler object cannot drive it")
        self.args = args
        self.processing_class = processing_class
        tok = processing_class
        self.pad_token_id = getattr(tok, "pad_token_id", None)
        self.eos_token_id = getattr(tok, "eos_token_id", None)
        if args.pad_token_id is not None:  # token ids without a tokenizer object
            self.pad_token_id = args.pad_token_id
        if args.eos_token_id is not None:
            self.eos_token_id = args.eos_token_id
        if self.pad_token_id is None:
            raise ValueError("PPOTrainer needs a pad token id (processing_class.pad_token_id)")
        # stop token (ppo_trainer.py:134-145)
        if args.stop_token and args.stop_token_id:
            raise ValueError("You cannot set both `stop_token` and `stop_token_id`.")
        elif args.stop_token:
            if args.stop_token == "eos":
                self.stop_token_id = self.eos_token_id
            else:
                raise ValueError(f"Unknown `stop_token` {args.stop_token}. Allowed values are: `'eos'` and `None` "
                                 "(no stop token).")
        else:
            self.stop_token_id = args.stop_token_id
        if args.kl_estimator not in {"k1", "k3"}:
            raise ValueError("kl_estimator must be either 'k1' (straightforward, unbiased) or 'k3' (lower variance, "
                             "unbiased, appears to be a strictly better estimator). See [Approximating KL "
                             "Divergence](http://joschu.net/blog/kl-approx.html) for details.")
        self.rank, self.world, self.local_rank = swh_dist.init_from_env()
        if not torch.cuda.is_available():
            raise RuntimeError("PPOTrainer runs the MI355X engine and needs a ROCm device (no CPU fallback)")
        self.device = torch.device("cuda", self.local_rank)
        torch.cuda.set_device(self.device)
        gemm_tuning.enable()
        # models: policy (lm head), frozen ref copy, value model + reward model (score heads).
        # Model objects keep their precision (the reference trains the modules it is given,
        # ppo_trainer.py:144-152); names / configs take model_init_kwargs' dtype (bf16
        # default; "float32" = the reference-precision mode, fp32 rollout included)
        dt = None if hasattr(model, "parameters") else model_dtype(args.model_init_kwargs)
        self.policy_model = load_model(model, self.device, trainable=True, seed=args.seed, dtype=dt)
        pdt = self.policy_model.dtype
        side = lambda m: None if hasattr(m, "parameters") else pdt  # noqa: E731
        if ref_model is not None:
            self.ref_model = load_model(ref_model, self.device, trainable=False, seed=args.seed, dtype=side(ref_model))
        else:  # create_reference_model (modeling_base.py:592-664): a frozen deep copy
            self.ref_model = build_model(self.policy_model.cfg, self.device, seed=None, trainable=False,
                                         dtype=self.policy_model.dtype)
            self.ref_model.copy_from(self.policy_model)
        self.value_model = load_model(value_model, self.device, trainable=True, seed=args.seed + 1, head="score",
                                      dtype=side(value_model))
        self.reward_model = load_model(reward_model, self.device, trainable=False, seed=args.seed + 2, head="score",
                                       dtype=side(reward_model))
        self.train_dataset, self.eval_dataset = train_dataset, eval_dataset
        self.train_dataset_len = len(train_dataset)
        fill_batch_sizes(args, self.train_dataset_len, self.world)
        self.local_seed = args.seed + self.rank * 100003  # ppo_trainer.py:251
        # one AdamW over policy + value parameters (PolicyAndValueWrapper), no
        # gradient clipping in the reference loop: two flat buffers, same update
        mk = lambda m: FlatAdamW(m.numel, self.device, lr=args.learning_rate,  # noqa: E731
                                 betas=(args.adam_beta1, args.adam_beta2), eps=args.adam_epsilon,
                                 weight_decay=args.weight_decay, max_grad_norm=None,
                                 no_decay_ranges=m.no_decay_ranges())
        self.opt_policy, self.opt_value = mk(self.policy_model), mk(self.value_model)
        self.opt_policy.master.copy_(self.policy_model.flat.float())
        self.opt_value.master.copy_(self.value_model.flat.float())
        self.state = new_state(self.rank, self.local_rank)
        self.state.episode = 0
        self.model, self.optimizer = self.policy_model, self.opt_policy   # what callbacks receive
        self.callback_handler = CallbackHandler(callbacks, self)
        self.control = self.callback_handler.control
        self._engine: Optional[DecodeEngine] = None
        self._engines: dict = {}
        self._accum_step = 0     # accelerate's Accelerator.step (gradient-accumulation counter)
        self._gen_count = 0
        self._np_rng = np.random.default_rng(self.local_seed)
        self._data_gen = torch.Generator().manual_seed(args.seed)
        self._metrics = defaultdict(list)

    # ------------------------------------------------------------------ data
    def _batches(self):
        """DataLoader(shuffle=True, drop_last=True, batch_size=local_batch_size)
        sharded over ranks, repeated forever (ppo_trainer.py:311-318, :358-362).
        Yields (examples, last): `last` is accelerate's end_of_dataloader for the
        batch (DataLoaderShard looks one batch ahead and flags the epoch's last)."""
        a = self.args
        n, per = self.train_dataset_len, a.local_batch_size
        glob = per * self.world
        while True:
            perm = torch.randperm(n, generator=self._data_gen).tolist()
            starts = list(range(0, n - glob + 1, glob))
            for k, s in enumerate(starts):
                mine = perm[s + self.rank * per: s + (self.rank + 1) * per]
                yield [self.train_dataset[i] for i in mine], k == len(starts) - 1

    def _queries(self, examples) -> torch.Tensor:
        if "input_ids" not in examples[0]:
            raise ValueError("PPO datasets carry tokenized `input_ids` (ppo_trainer.py:364)")
        ids, _ = left_pad([list(x["input_ids"]) for x in examples], self.pad_token_id, self.device)
        return ids

    def _engine_for(self, B: int, P: int) -> DecodeEngine:
        """One engine per batch size (rollout and sample-generation batches may
        differ), kept for the run: a rebuild repacks the weights and recaptures
        the decode graph."""
        C = self.args.response_length
        e = self._engines.get(B)
        if e is None or e.Pmax < P:
            e = self._engines[B] = build_engine(self.policy_model, B, P, C)
        self._engine = e
        return e

    # ------------------------------------------------------------------ rollout (ppo_trainer.py:362-535)
    @torch.no_grad()
    def _no_grad_hidden(self, model: CausalLM, query_responses: torch.Tensor) -> torch.Tensor:
        saved, model.grad = model.grad, None
        try:
            ids, mask, pos = _forward_inputs(query_responses, self.pad_token_id)
            return model.hidden_states(ids, positions=pos, key_mask=mask)
        finally:
            model.grad = saved

    @torch.no_grad()
    def generate(self, queries: torch.Tensor):
        """batch_generation (utils.py:1059-1128): sampled responses and the
        log-probs of the drawn tokens under the processed (T + 1e-7) scores.
        Generation ends when every row has stopped (transformers stops the
        batch there), so the response width is the longest row."""
        a = self.args
        B, P = queries.shape
        eng = self._engine_for(B, P)
        attention_mask = (queries != self.pad_token_id).to(torch.int32)
        input_ids = torch.masked_fill(queries, attention_mask == 0, 0)
        seed = a.seed * 1_000_003 + self.rank
        resp, logp = eng.generate(input_ids, attention_mask, a.response_length, temperature=a.temperature + 1e-7,
                                  top_p=1.0, top_k=None, eos_token_id=self.stop_token_id,
                                  pad_token_id=self.pad_token_id, seed=seed,
                                  offset=self._gen_count * (a.response_length + 1), return_logp=True,
                                  check_every=a.decode_check_every, early_exit=a.decode_early_exit)
        self._gen_count += 1
        T = resp.shape[1]
        if self.stop_token_id is not None:
            stopped = first_true_indices(resp == self.stop_token_id)  # T where none
            T = int(torch.clamp(stopped + 1, max=resp.shape[1]).max())
        return resp[:, :T].contiguous(), logp[:, :T].contiguous()

    @torch.no_grad()
    def rollout_from(self, queries: torch.Tensor, responses: torch.Tensor, logprobs: torch.Tensor) -> dict:
        """Everything after generation (ppo_trainer.py:389-535) for given
        queries [B, P], responses [B, T] and their generation log-probs."""
        a = self.args
        pad = self.pad_token_id
        P = queries.shape[1]
        T = responses.shape[1]
        temp = a.temperature + 1e-7
        query_responses = torch.cat([queries, responses], 1)
        # ref log-probs: forward, logits[:, P-1:-1] / (T + 1e-7), selective_log_softmax
        h = self._no_grad_hidden(self.ref_model, query_responses)
        ref_logprobs, _ = self.ref_model.logp_entropy(h[:, P - 1:P + T - 1], responses, temp, False)
        # response processing 1: truncate after the first stop token, sequence lengths (one launch)
        post, sequence_lengths = ops.ppo_truncate(responses, self.stop_token_id, pad)
        # values: value model over the raw query_responses, positions P-1 .. P+T-2 (bf16 like the score Linear)
        hv = self._no_grad_hidden(self.value_model, query_responses)
        values = self.value_model.scores(hv[:, P - 1:P + T - 1])
        # response processing 2: reward model score at the last non-pad token of query + truncated response
        pqr = torch.cat([queries, post], 1)
        hr = self._no_grad_hidden(self.reward_model, pqr)
        scores = self.reward_model.scores(hr[torch.arange(hr.shape[0], device=hr.device), sequence_lengths + P])
        rm_scores = scores.clone()
        # 3.-4. missing-stop penalty, masks, INVALID_LOGPROB, KL and KL-shaped rewards (one launch)
        r = ops.ppo_rewards(post, sequence_lengths, logprobs, ref_logprobs, values, scores,
                            eos_token_id=self.eos_token_id, missing_eos_penalty=a.missing_eos_penalty,
                            kl_coef=a.kl_coef, kl_estimator=a.kl_estimator)
        logprobs, ref_logprobs, values, scores = r["logprobs"], r["ref_logprobs"], r["values"], r["scores"]
        padding_mask, padding_mask_p1, rewards = r["padding_mask"], r["padding_mask_p1"], r["rewards"]
        kl, non_score_reward = r["kl"], r["non_score_reward"]
        # 5. whiten rewards
        if a.whiten_rewards:
            rewards = ops.masked_whiten(rewards, ~padding_mask_p1, shift_mean=False)
            rewards = torch.masked_fill(rewards, padding_mask_p1, 0)
        # 6. advantages and returns (reverse GAE scan), whitened advantages
        advantages, returns = ops.gae(rewards, values.float(), a.gamma, a.lam)
        advantages = ops.masked_whiten(advantages, ~padding_mask)
        advantages = torch.masked_fill(advantages, padding_mask, 0)
        return {"queries": queries, "responses": responses, "query_responses": query_responses,
                "logprobs": logprobs, "ref_logprobs": ref_logprobs, "values": values, "scores": scores, "rm_scores": rm_scores,
                "rewards": rewards, "advantages": advantages, "returns": returns, "kl": kl,
                "non_score_reward": non_score_reward, "padding_mask": padding_mask,
                "padding_mask_p1": padding_mask_p1, "sequence_lengths": sequence_lengths,
                "postprocessed_responses": post}

    # ------------------------------------------------------------------ PPO update (ppo_trainer.py:537-617)
    def _micro_step(self, ro: dict, inds: torch.Tensor, n_micro: int = 1) -> torch.Tensor:
        """`n_micro` micro-batches of equal size (rows `inds`, micro j = the j-th
        slice) in ONE policy + value forward/backward: the fused loss kernel runs
        per micro-batch slice (each keeps its own masked means, as the
        reference's separate passes), every micro's gradient is scaled by 1/GA
        (accelerate's accumulate) — the summed gradient equals GA separate
        backward passes.  Returns stats [n_micro, 9] = kernel stats f32[8] +
        mean entropy."""
        a = self.args
        P = ro["queries"].shape[1]
        T = ro["responses"].shape[1]
        temp = a.temperature + 1e-7
        mb_qr = ro["query_responses"][inds]
        mb_resp = ro["responses"][inds]
        pm, pm1 = ro["padding_mask"][inds], ro["padding_mask_p1"][inds]
        ids, mask, pos = _forward_inputs(mb_qr, self.pad_token_id)
        hp = self.policy_model.hidden_states(ids, positions=pos, key_mask=mask)
        new_logprobs, entropy = self.policy_model.logp_entropy(hp[:, P - 1:P + T - 1], mb_resp, temp, True)
        hv = self.value_model.hidden_states(ids, positions=pos, key_mask=mask)
        vpred = self.value_model.scores(hv[:, P - 1:P + T - 1])
        nl = torch.masked_fill(new_logprobs.detach(), pm, INVALID_LOGPROB)
        vp = torch.masked_fill(vpred.detach().float(), pm1, 0)
        old_lp, adv = ro["logprobs"][inds], ro["advantages"][inds]
        old_v, ret = ro["values"][inds].float(), ro["returns"][inds]
        ga = a.gradient_accumulation_steps
        R = inds.numel() // n_micro
        dnl, dvp = torch.empty_like(nl), torch.empty_like(vp)
        out = torch.empty(n_micro, 9, device=self.device, dtype=torch.float32)
        for j in range(n_micro):
            sl = slice(j * R, (j + 1) * R)
            _, d1, d2, stats = ops.ppo_loss_fwd_bwd(nl[sl], old_lp[sl], adv[sl], vp[sl], old_v[sl], ret[sl], pm[sl],
                                                    pm1[sl], a.cliprange, a.cliprange_value, a.vf_coef)
            dnl[sl], dvp[sl] = d1, d2
            out[j, :8] = stats
            out[j, 8] = entropy[sl].detach().float().mean()
        # masked_fill blocks the gradient at padded positions (the kernel's d is 0 there too)
        dnl = torch.masked_fill(dnl, pm, 0.0) / ga
        dvp = torch.masked_fill(dvp, pm1, 0.0) / ga
        torch.autograd.backward([new_logprobs, vpred], [dnl.to(new_logprobs.dtype), dvp.to(vpred.dtype)])
        dw_sync(self.device)
        return out

    def _optimizer_step(self, lr: float):
        if self.world > 1:
            swh_dist.allreduce_mean_(self.policy_model.grad)
            swh_dist.allreduce_mean_(self.value_model.grad)
        self.opt_policy.step(self.policy_model.grad, model_out=self.policy_model.flat, lr=lr)
        self.opt_value.step(self.value_model.grad, model_out=self.value_model.flat, lr=lr)
        self.policy_model.zero_grad()
        self.value_model.zero_grad()

    def _accumulate_sync(self, end_of_dataloader: bool) -> bool:
        """accelerate's `Accelerator.accumulate` sync decision for one micro-batch
        (accelerate/accelerator.py `_do_sync`, gradient_accumulation_steps = GA,
        sync_with_dataloader on): at the data epoch's last batch every micro-batch
        syncs (and the counter resets); otherwise the counter, which runs across
        mini-batches, epochs and updates, syncs every GA-th.  The reference calls
        optimizer.step() / zero_grad() after every micro-batch (ppo_trainer.py:
        604-606); the AcceleratedOptimizer acts only on a sync."""
        if end_of_dataloader:
            self._accum_step = 0
            return True
        self._accum_step += 1
        return self._accum_step % self.args.gradient_accumulation_steps == 0

    def ppo_update(self, ro: dict, lr: float, permutations=None, end_of_dataloader: bool = False) -> torch.Tensor:
        """num_ppo_epochs x mini-batches x micro-batches (ppo_trainer.py:537-617), with
        the optimizer steps where the reference's accelerate accumulation takes them
        (_accumulate_sync; loss / GA every micro-batch).  The micro-batches between
        two steps see the same weights, so they run as ONE fused forward/backward
        (each micro keeps its own masked means in the loss kernel; the gradient is
        their sum) when the token budget allows.  Gradients of micro-batches after
        the last sync stay accumulated for the next update, as the reference's do.
        `permutations` (tests): one index array per epoch instead of the RNG."""
        a = self.args
        stats = torch.zeros(a.num_ppo_epochs, a.num_mini_batches, a.gradient_accumulation_steps, 9,
                            device=self.device)
        mbs = a.per_device_train_batch_size
        n_micro = a.local_mini_batch_size // mbs
        width = ro["query_responses"].shape[1]
        pending = []  # (epoch, mini, micro, row indices) since the last optimizer step

        def run_pending():
            if not pending:
                return
            if a.fuse_micro_batches and len(pending) * mbs * width <= a.fuse_token_budget:
                out = self._micro_step(ro, torch.cat([p[3] for p in pending]), len(pending))
                for (ep, mi, gi, _), row in zip(pending, out):
                    stats[ep, mi, gi] = row
            else:  # the reference schedule, one pass per micro-batch
                for ep, mi, gi, inds in pending:
                    stats[ep, mi, gi] = self._micro_step(ro, inds)[0]
            pending.clear()

        for ep in range(a.num_ppo_epochs):
            b_inds = permutations[ep] if permutations is not None else self._np_rng.permutation(a.local_batch_size)
            b_inds = torch.as_tensor(np.asarray(b_inds), device=self.device, dtype=torch.long)
            for mi, mb0 in enumerate(range(0, a.local_batch_size, a.local_mini_batch_size)):
                mini = b_inds[mb0:mb0 + a.local_mini_batch_size]
                for gi in range(n_micro):
                    pending.append((ep, mi, gi, mini[gi * mbs:(gi + 1) * mbs]))
                    if self._accumulate_sync(end_of_dataloader):
                        run_pending()
                        self._optimizer_step(lr)
        run_pending()
        return stats

    # ------------------------------------------------------------------ the loop
    def training_step(self, examples=None, end_of_dataloader: bool = False) -> dict:
        """One PPO update: rollout of local_batch_size queries, rewards, GAE,
        then the PPO epochs (ppo_trainer.py:356-617).  Given `examples`, the batch
        counts as a non-final batch of its data epoch unless `end_of_dataloader`."""
        a = self.args
        if examples is None:
            if getattr(self, "_iter", None) is None:
                self._iter = self._batches()
            examples, end_of_dataloader = next(self._iter)
        self.state.episode += a.batch_size
        queries = self._queries(examples)
        _trace(f"queries {tuple(queries.shape)}")
        responses, logprobs = self.generate(queries)
        _trace("generated")
        ro = self.rollout_from(queries, responses, logprobs)
        _trace("rollout scored")
        # create_optimizer_and_scheduler(num_training_steps=num_total_batches), stepped once per update (:232-234, :648)
        lr = a.learning_rate * schedule.for_args(a, max(1, a.num_total_batches))(self.state.global_step)
        stats = self.ppo_update(ro, lr, end_of_dataloader=end_of_dataloader)
        _trace("ppo epochs")
        self.state.global_step += 1
        m = self._metrics
        m["kl"].append(ro["kl"].sum(1).mean())
        m["entropy"].append((-ro["logprobs"]).sum(1).mean())
        m["non_score_reward"].append(ro["non_score_reward"].sum(1).mean())
        m["scores"].append(ro["scores"].mean())
        m["stats"].append(stats)
        m["num_eos"].append((ro["responses"] == self.eos_token_id).sum() if self.eos_token_id is not None
                            else torch.zeros((), device=self.device))
        m["lr"].append(lr)
        return ro

    def _flush_logs(self) -> dict:
        """ppo_trainer.py:619-646 metric names (one host sync per log)."""
        m = self._metrics
        if not m.get("stats"):
            return {}
        st = torch.stack(m["stats"]).float()  # [n, epochs, mini, ga, 9]
        flat = st.reshape(-1, 9)
        kl = float(torch.stack(m["kl"]).mean())
        nsr = float(torch.stack(m["non_score_reward"]).mean())
        sc = float(torch.stack(m["scores"]).mean())
        log = {
            "objective/kl": kl,
            "objective/entropy": float(torch.stack(m["entropy"]).mean()),
            "objective/non_score_reward": nsr,
            "objective/rlhf_reward": nsr + sc,
            "objective/scores": sc,
            "policy/approxkl_avg": float(flat[:, 4].mean()),
            "policy/clipfrac_avg": float(flat[:, 2].mean()),
            "loss/policy_avg": float(flat[:, 0].mean()),
            "loss/value_avg": float(flat[:, 1].mean()),
            "val/clipfrac_avg": float(flat[:, 3].mean()),
            "policy/entropy_avg": float(flat[:, 8].mean()),
            "val/ratio": float(flat[:, 5].mean()),
            "val/ratio_var": float(flat[:, 5].var()) if flat.shape[0] > 1 else 0.0,
            "val/num_eos_tokens": float(torch.stack(m["num_eos"]).float().mean()),
            "lr": m["lr"][-1],
            "episode": self.state.episode,
            "step": self.state.global_step,
        }
        m.clear()
        self.state.log_history.append(log)
        return log

    # ------------------------------------------------------------------ checkpoints
    def save_model(self, output_dir: Optional[str] = None, _internal_call: bool = False):
        """ppo_trainer.py:332-346: only the policy is saved (transformers layout)."""
        from . import checkpoint as ck
        out = output_dir or self.args.output_dir
        if self.rank == 0:
            ck.save_pretrained(self.policy_model, out, eos_token_id=self.eos_token_id, pad_token_id=self.pad_token_id)
            if self.processing_class is not None and hasattr(self.processing_class, "save_pretrained"):
                self.processing_class.save_pretrained(out)
        swh_dist.barrier()

    def create_model_card(self, model_name: Optional[str] = None, dataset_name: Optional[str] = None, tags=None):
        """ppo_trainer.py:760-: README.md model card in output_dir."""
        from . import checkpoint as ck
        if self.rank != 0 or not self.args.output_dir:
            return
        tags = set([tags] if isinstance(tags, str) else (tags or []))
        tags.update(self._tag_names)
        os.makedirs(self.args.output_dir, exist_ok=True)
        with open(os.path.join(self.args.output_dir, "README.md"), "w") as f:
            f.write(ck.model_card("PPO", model_name or os.path.basename(os.path.normpath(self.args.output_dir)),
                                  "Fine-Tuning Language Models from Human Preferences, arXiv:1909.08593",
                                  ck.PPO_CITATION, tags))

    def _save_checkpoint(self, model=None, trial=None):
        """ppo_trainer.py:752-758 + transformers Trainer._save_checkpoint: the
        policy weights, the AdamW state of the policy + value wrapper
        (PolicyAndValueWrapper parameter names), trainer state, model card."""
        import json

        from . import checkpoint as ck
        a = self.args
        self.create_model_card(model_name=os.path.basename(os.path.normpath(a.output_dir)))
        d = os.path.join(a.output_dir, f"checkpoint-{self.state.global_step}")
        self.save_model(d)
        if self.rank == 0:
            parts = [("policy.", self.policy_model, self.opt_policy), ("value_model.", self.value_model, self.opt_value)]
            torch.save(ck.optimizer_state_dict(self.policy_model, self.opt_policy, a.weight_decay, parts=parts),
                       os.path.join(d, "optimizer.pt"))
            with open(os.path.join(d, "trainer_state.json"), "w") as f:
                js = ck.trainer_state_json(self.state, a, a.per_device_train_batch_size)
                js["episode"] = self.state.episode
                json.dump(js, f, indent=2)
            ck.rotate_checkpoints(a.output_dir, a.save_total_limit)
        swh_dist.barrier()
        return d

    def add_callback(self, callback):
        self.callback_handler.add_callback(callback)

    def pop_callback(self, callback):
        return self.callback_handler.pop_callback(callback)

    def remove_callback(self, callback):
        self.callback_handler.remove_callback(callback)

    @torch.no_grad()
    def generate_completions(self, sampling: bool = False) -> dict:
        """ppo_trainer.py:687-749: the policy's completions of the eval dataset
        (per_device_eval_batch_size batches, drop_last, no shuffle) sampled at
        temperature 0.01 + 1e-7, truncated after the stop token and scored by
        the reward model; `sampling` stops after the first batch.  Returns the
        table {"query", "model response", "score"} (rank 0 prints its first 5
        rows); queries / responses are decoded when the processing class can."""
        a = self.args
        table = {"query": [], "model response": [], "score": []}
        if self.eval_dataset is None:
            return table
        tok = self.processing_class
        # the eval DataLoader through accelerator.prepare (ppo_trainer.py:290): every
        # global batch of bs x world rows is split into contiguous per-rank slices
        n, bs = len(self.eval_dataset), a.per_device_eval_batch_size
        glob = bs * self.world
        for s0 in range(0, n - glob + 1, glob):
            s = s0 + self.rank * bs
            query = self._queries([self.eval_dataset[i] for i in range(s, s + bs)])
            B, P = query.shape
            eng = self._engine_for(B, P)
            attention_mask = (query != self.pad_token_id).to(torch.int32)
            input_ids = torch.masked_fill(query, attention_mask == 0, 0)
            resp, _ = eng.generate(input_ids, attention_mask, a.response_length, temperature=0.01 + 1e-7, top_p=1.0,
                                   top_k=None, eos_token_id=self.stop_token_id, pad_token_id=self.pad_token_id,
                                   seed=a.seed * 1_000_003 + 7919 * (self.rank + 1), offset=s * (a.response_length + 1),
                                   early_exit=a.decode_early_exit)
            post = resp
            if self.stop_token_id is not None:
                post, _ = ops.ppo_truncate(resp, self.stop_token_id, self.pad_token_id)
            pqr = torch.cat([query, post], 1)
            hr = self._no_grad_hidden(self.reward_model, pqr)
            # get_reward: the score at the last non-pad token after the context
            seq = first_true_indices(pqr[:, P:] == self.pad_token_id) - 1 + P
            score = self.reward_model.scores(hr[torch.arange(B, device=hr.device), seq.clamp(min=0)])
            dec = (lambda t, **k: tok.batch_decode(t, **k)) if hasattr(tok, "batch_decode") else \
                (lambda t, **k: t.tolist())
            table["query"].extend(swh_dist.all_gather_objects(dec(query.cpu(), skip_special_tokens=True)))
            table["model response"].extend(swh_dist.all_gather_objects(dec(post.cpu())))
            table["score"].extend(swh_dist.all_gather_rows(score.float().view(-1, 1)).view(-1).cpu().tolist())
            if sampling:
                break
        if self.rank == 0:
            for i in range(min(5, len(table["query"]))):
                print({k: v[i] for k, v in table.items()}, flush=True)
        return table

    def train(self):
        """ppo_trainer.py:347-685: per update a rollout, the PPO epochs, a log of
        the metrics (self.log every update, :646), on_step_end with
        DefaultFlowCallback's save decision (save_steps), sample generations on
        the eval dataset every num_total_batches // num_sample_generations
        updates (:657-659), on_train_end."""
        a = self.args
        st = self.state
        st.global_step = 0
        st.episode = 0
        st.max_steps = a.num_total_batches
        st.num_train_epochs = a.total_episodes / self.train_dataset_len
        st.logging_steps = int(a.logging_steps) if a.logging_steps >= 1 else math.ceil(st.max_steps * a.logging_steps)
        st.save_steps = int(a.save_steps) if a.save_steps >= 1 else max(1, math.ceil(st.max_steps * a.save_steps))
        if a.eval_steps is not None:
            st.eval_steps = int(a.eval_steps) if a.eval_steps >= 1 else math.ceil(st.max_steps * a.eval_steps)
        sample_freq = max(1, a.num_total_batches // a.num_sample_generations) if a.num_sample_generations > 0 else 0
        cb = self.callback_handler
        self.control = cb.call("on_train_begin")
        t0 = time.time()
        for update in range(1, a.num_total_batches + 1):
            self.training_step()
            log = self._flush_logs()
            log["eps"] = int(st.episode / max(time.time() - t0, 1e-9))
            st.epoch = st.episode / self.train_dataset_len
            log["epoch"] = st.epoch
            if self.rank == 0:
                print(log, flush=True)
            self.control = cb.call("on_log", logs=log)
            # DefaultFlowCallback.on_step_end: save every save_steps, and stop (saving
            # under the "steps" strategy) once max_steps is reached
            if a.save_strategy == "steps" and st.global_step % st.save_steps == 0:
                self.control.should_save = True
            if st.global_step >= st.max_steps:
                self.control.should_training_stop = True
                if a.save_strategy == "steps":
                    self.control.should_save = True
            self.control = cb.call("on_step_end")
            if self.control.should_save:
                if a.output_dir:
                    self._save_checkpoint()
                self.control = cb.call("on_save")
            if sample_freq and (update - 1) % sample_freq == 0:
                self.generate_completions(sampling=True)
            if self.control.should_training_stop:
                break
        self.control = cb.call("on_train_end")
        if self.control.should_save:
            if a.output_dir:
                self._save_checkpoint()
            self.control = cb.call("on_save")
        return st
