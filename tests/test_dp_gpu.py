"""Data-parallel GRPO step on the GPU with two ranks (-m gpu).

Both ranks share cuda:0 and talk over gloo (SWH_DIST_BACKEND=gloo): the
collective differs from the RCCL runs of bench.py, but the trainer's DP data
path is the one under test — per-layer gradient ranges released from the
backward hooks (OverlappedAllReduce) while the weight-gradient side stream is
still producing, the remainder in finish(), then AdamW on each replica.  The
replicas must stay bit-identical, and differ from a single-rank run on the
same rank-0 prompts (the other rank's gradients were averaged in).
"""
import hashlib
import json
import multiprocessing as mp
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q, steps, pdb=8, ga=2):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SWH_DIST_BACKEND="gloo")
    try:
        from swh_trl_amd.engine import tiny_qwen2
        from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
        cfg = tiny_qwen2(512, 4)
        ds = [{"prompt": None, "prompt_ids": list(range(3 + i, 11 + i))} for i in range(32)]

        def rew(prompts=None, completions=None, completion_ids=None, **kw):
            return [float(len(set(c)) % 5) for c in completion_ids]

        args = GRPOConfig(per_device_train_batch_size=pdb, gradient_accumulation_steps=ga, num_generations=4,
                          max_prompt_length=8, max_completion_length=16, max_steps=steps, learning_rate=1e-3,
                          generation_kwargs={"eos_token_id": 1, "pad_token_id": 0, "min_new_tokens": 16},
                          logging_steps=1, seed=7)
        tr = GRPOTrainer(model=cfg, reward_funcs=rew, args=args, train_dataset=ds)
        tr.train()
        torch.cuda.synchronize()
        flat = tr.model.flat.float().cpu().numpy()
        log = [h for h in tr.state.log_history if "loss" in h][-1]
        q.put((rank, (hashlib.sha256(flat.tobytes()).hexdigest(), float(flat.astype("float64").sum()),
                      log["reward"], log["loss"])))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e)))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(world, steps, pdb=8, ga=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 1000) + world + 7 * pdb
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, steps, pdb, ga)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r, v in got.items():
        assert isinstance(v, tuple), (r, v)
    return got


def test_dp_two_ranks_keep_replicas_identical():
    got = _run(2, 2)  # (sha256 of the fp32 weights, their sum) per rank
    assert got[0][0] == got[1][0]
    single = _run(1, 2)
    assert single[0][0] != got[0][0]


def test_dp_groups_straddling_ranks():
    """per_device_train_batch_size 2 with G = 4 on two ranks: every group of 4
    completions is split over both ranks.  The reference gathers the rewards
    (grpo_trainer.py:1497), forms advantages on the global batch and keeps each
    rank's slice (:1933-1938); the replicas stay identical and both ranks log
    the same (global) mean reward."""
    got = _run(2, 2, pdb=2, ga=1)
    assert got[0][0] == got[1][0]
    assert got[0][2] == got[1][2]


def _oracle_worker(rank, world, port, q, out_dir, pdb, ga, loss_type, G=4):
    """One fp32 GRPO step on this rank; saves its rollout, shuffle permutation, the
    all-reduced gradient and its log line for the parent's oracle check."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SWH_DIST_BACKEND="gloo")
    try:
        from swh_trl_amd.engine import CausalLM, tiny_qwen2
        from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
        cfg = tiny_qwen2(512, 2)
        ds = [{"prompt": None, "prompt_ids": list(range(3 + 5 * i, 11 + 5 * i))} for i in range(32)]

        def rew(prompts=None, completions=None, completion_ids=None, **kw):
            return [float(len(set(c)) % 5) for c in completion_ids]

        args = GRPOConfig(per_device_train_batch_size=pdb, gradient_accumulation_steps=ga, num_generations=G,
                          max_prompt_length=8, max_completion_length=16, max_steps=1, learning_rate=1e-3,
                          lr_scheduler_type="constant", loss_type=loss_type, shuffle_dataset=False,
                          generation_kwargs={"eos_token_id": 1, "pad_token_id": 0, "min_new_tokens": 4},
                          model_init_kwargs={"torch_dtype": "float32"}, logging_steps=1, seed=7)
        tr = GRPOTrainer(model=CausalLM(cfg, torch.device("cuda:0"), seed=3, init_std=0.05, dtype=torch.float32),
                         reward_funcs=rew, args=args, train_dataset=ds)
        w0 = {k: v.detach().cpu().clone() for k, v in tr.model.hf_state_dict().items()}
        cap = {}
        gen_fn = tr._generate_and_score_completions

        def gen_capture(examples):
            out = gen_fn(examples)
            cap["gen"] = {k: v.detach().cpu().clone() for k, v in out.items()}
            n = out["completion_ids"].shape[0]
            cap["perm"] = torch.randperm(n, generator=torch.Generator().set_state(tr._shuffle_gen.get_state()))
            return out

        tr._generate_and_score_completions = gen_capture
        tr.training_step_group()
        torch.cuda.synchronize()
        saved = tr.model.flat.clone()
        tr.model.flat.copy_(tr.model.grad)  # the averaged gradient, through the transformers names
        grads = {k: v.detach().cpu().clone() for k, v in tr.model.hf_state_dict().items()}
        tr.model.flat.copy_(saved)
        log = tr._flush_logs()
        torch.save({"w0": w0, "gen": cap["gen"], "perm": cap["perm"], "grads": grads,
                    "log": {k: float(v) for k, v in log.items()}}, os.path.join(out_dir, f"rank{rank}.pt"))
        q.put((rank, "ok"))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,pdb,ga,G,loss_type", [(2, 8, 2, 4, "bnpo"), (2, 2, 1, 4, "bnpo"), (2, 4, 2, 4, "grpo"),
                                                      (4, 16, 4, 8, "bnpo")],
                         ids=["whole-groups-bnpo", "straddling-bnpo", "whole-groups-grpo", "bench-split-4-ranks"])
def test_dp_averaged_gradient_equals_mean_of_oracle_rank_gradients(tmp_path, world, pdb, ga, G, loss_type):
    """fp32 ranks, one step.  The gradient each rank holds after the
    overlapped all-reduce equals the mean over ranks of the oracle's gradient on that
    rank's own split (oracle/grpo_step.py grpo_train): rewards gathered across ranks,
    advantages on the global batch sliced per rank (grpo_trainer.py:1497, :1933-1938;
    pdb 2 with G 4 puts every group across both ranks) and the loss normalised by the
    rank-local token count under bnpo (grpo_config.py:500-503).  The loss metrics of
    the log are the reference's cross-rank gathers: every rank logs the same values.
    bench-split-4-ranks: four ranks at the bench's per-rank split (8 prompts x G 8 = 64
    rows per rank, micro-batch 16 x GA 4), the 4-rank case of cfg4's data path."""
    from oracle import grpo_step as og
    from swh_trl_amd.engine import tiny_qwen2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() % 1000) + 13 * pdb + ga + 101 * world
    ps = [ctx.Process(target=_oracle_worker, args=(r, world, port, q, str(tmp_path), pdb, ga, loss_type, G))
          for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in got.values()), got
    runs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for r in range(1, world):
        assert runs[0]["log"] == runs[r]["log"]
        for k in runs[0]["grads"]:
            assert torch.equal(runs[0]["grads"][k], runs[r]["grads"][k]), k  # one averaged gradient
    all_ids = torch.cat([r["gen"]["completion_ids"] for r in runs])

    def rew(cids, cmask):
        return [float(len(set(row[m.bool()].tolist())) % 5) for row, m in zip(cids, cmask)]

    cfg = tiny_qwen2(512, 2)
    per_rank = []
    for r, run in enumerate(runs):
        hf = og.hf_qwen2_from_config(cfg.to_dict(), dtype=torch.float32)
        hf.load_state_dict(run["w0"], strict=False)
        opt = torch.optim.SGD(hf.parameters(), lr=0.0)
        g = {"prompt_ids": run["gen"]["prompt_ids"], "prompt_mask": run["gen"]["prompt_mask"].long(),
             "completion_ids": run["gen"]["completion_ids"], "perm": run["perm"], "world_completion_ids": all_ids,
             "rank": r}
        rec = og.grpo_train(hf, opt, [g], rew, num_generations=G, C=16, per_device_train_batch_size=pdb,
                            gradient_accumulation_steps=ga, n_steps=1, eos_token_id=1, loss_type=loss_type,
                            capture=True)[0]
        torch.testing.assert_close(run["gen"]["advantages"], rec["gens"][0]["a"], rtol=0, atol=1e-6)
        per_rank.append(rec["grads"])
    for k, mine in runs[0]["grads"].items():
        if k not in per_rank[0]:
            continue
        want = sum(p[k] for p in per_rank) / world
        rel = ((mine.float() - want).norm() / want.norm().clamp_min(1e-20)).item()
        assert rel <= 1e-3, (k, rel)


def _resume_worker(rank, world, port, q, out_dir, resume_from):
    """GRPO on two gloo ranks with steps_per_generation 4 > GA 2 (a rollout feeds two
    optimizer steps): 3 steps saving every step, or resumed from `resume_from`."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SWH_DIST_BACKEND="gloo")
    try:
        from swh_trl_amd.engine import CausalLM, tiny_qwen2
        from swh_trl_amd.trainer import GRPOConfig, GRPOTrainer
        ds = [{"prompt": None, "prompt_ids": list(range(3 + 5 * i, 11 + 5 * i))} for i in range(32)]

        def rew(prompts=None, completions=None, completion_ids=None, **kw):
            return [float(len(set(c)) % 5) for c in completion_ids]

        args = GRPOConfig(output_dir=out_dir, per_device_train_batch_size=4, gradient_accumulation_steps=2,
                          steps_per_generation=4, num_generations=4, max_prompt_length=8, max_completion_length=16,
                          max_steps=3, learning_rate=1e-3, save_steps=1 if resume_from is None else 10 ** 9,
                          logging_steps=1, seed=7, generation_kwargs={"eos_token_id": 1, "pad_token_id": 0})
        tr = GRPOTrainer(model=CausalLM(tiny_qwen2(512, 2), torch.device("cuda:0"), seed=3, init_std=0.05),
                         reward_funcs=rew, args=args, train_dataset=ds)
        tr.train(resume_from_checkpoint=resume_from)
        torch.cuda.synchronize()
        flat = tr.model.flat.float().cpu().numpy()
        q.put((rank, hashlib.sha256(flat.tobytes()).hexdigest()))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, "ERR " + traceback.format_exc() + repr(e)))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(target, world, extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34500 + (os.getpid() % 500) + abs(hash(str(extra))) % 400
    ps = [ctx.Process(target=target, args=(r, world, port, q, *extra)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert not any(str(v).startswith("ERR") for v in got.values()), got
    return got


def test_dp_resume_restores_each_rank_state(tmp_path):
    """Exact resume on two ranks: each rank saves its own data-stream state
    (swh_trainer_state_<rank>.pt: its buffered rollouts and shuffle generator, which
    differ per rank) and reloads its own.  Checkpoint-1 falls mid-generation
    (steps_per_generation 4, GA 2): the resumed run must train step 2 on each rank's
    buffered rollouts and end bit-identical to the uninterrupted run on both ranks."""
    full = _spawn(_resume_worker, 2, (str(tmp_path / "a"), None))
    assert full[0] == full[1]
    for r in range(2):
        assert (tmp_path / "a" / "checkpoint-1" / f"swh_trainer_state_{r}.pt").exists()
    res = _spawn(_resume_worker, 2, (str(tmp_path / "b"), str(tmp_path / "a" / "checkpoint-1")))
    assert res[0] == res[1] == full[0]


@pytest.mark.parametrize("n", [2, 4])
def test_bench_launches_n_ranks_itself(n):
    """`python bench.py --gpus N` (no torchrun environment) starts N ranks itself;
    rank 0 prints one line with n_gpus N and the world size the process group
    reports.  gloo here, every rank on the one GPU of this box: RCCL needs one GPU
    per rank.  Weak scaling: the global batch is N x 64 rows."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SWH_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--layers", "2", "--steps", "1", "--warmup",
                        "1", "--no-cpu-baseline"], cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["ranks_seen"] == n and line["backend"] == "gloo"
    assert line["config"]["global_batch"] == 64 * n and line["value"] > 0


def _rccl_worker(port, q):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch.distributed as dist
        from swh_trl_amd import dist as swh_dist
        rank, world, local = swh_dist.init_from_env("nccl")
        if not dist.is_initialized():  # init_from_env leaves a one-process run alone
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", rank=0, world_size=1)
        dev = torch.device("cuda", local)
        g = torch.Generator(device=dev).manual_seed(0)
        flat = torch.randn(3 << 20, generator=g, device=dev).to(torch.bfloat16)
        ref = flat.clone()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # a producer beside the compute stream, as the dW stream
            flat[1 << 20:2 << 20].mul_(2)
            ref[1 << 20:2 << 20].mul_(2)
        ar = swh_dist.OverlappedAllReduce(flat, [side], force=True)
        assert ar.nccl and ar.stream is not None
        ar.release(2 << 20, 3 << 20)
        ar.release(1 << 20, 2 << 20)
        ar.finish()  # the remainder [0, 1M), then every collective joins the compute stream
        torch.cuda.synchronize()
        ok = bool(torch.equal(flat, ref))
        rows = torch.arange(12, device=dev, dtype=torch.float32).view(4, 3)
        out = torch.empty_like(rows)
        dist.all_gather_into_tensor(out, rows)
        swh_dist.barrier()
        q.put(("ok", ok and bool(torch.equal(out, rows)), dist.get_backend()))
    except Exception as e:
        q.put(("err", repr(e), None))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rccl_one_rank_overlapped_allreduce():
    """The RCCL branch of OverlappedAllReduce on real hardware: a one-rank
    "nccl" (RCCL) group, ranges released out of order behind a producer side
    stream, the remainder in finish(), AVG over one rank = identity; plus
    all_gather_into_tensor and the device barrier the launcher uses."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(32700 + os.getpid() % 500, q))
    p.start()
    status, ok, backend = q.get(timeout=240)
    p.join(timeout=60)
    assert status == "ok", ok
    assert ok and backend == "nccl"
