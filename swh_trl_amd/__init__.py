"""swh_trl_amd — MI355X-native GRPO/PPO rollout-and-update engine.

A drop-in for the `trl.GRPOTrainer` / `trl.PPOTrainer` hot path of
shiwanghua/swh-trl (TRL 0.21.0.dev0 fork): the per-step loop runs on
hand-written HIP kernels for gfx950 behind the C-ABI in
include/swh_trl_amd.h; transformer GEMMs run on hipBLASLt (MFMA); data
parallelism is one process per GPU over RCCL.
"""
__version__ = "0.1.0"
