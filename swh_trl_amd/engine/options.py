"""EngineOptions — the engine's explicit configuration surface.

Every mechanism choice of the rollout engine and the training passes that is not
a TRL / transformers config field lives here, with its default in code.  The
product reads no environment variable: a caller that wants another choice (an
A/B tool, a test pinning that two mechanisms give identical results) builds an
EngineOptions and hands it to the model (`CausalLM(..., options=...)`,
`model.options = ...`) or to the engine (`DecodeEngine(..., options=...)`;
default: the model's).  None of these fields changes what is computed except
where noted: `fold_norm` rounds the folded decode RMSNorm once (last-bit
differences), `fused_sample` / `fused_sample_wide` draw the same
ids through another kernel, and `hip_attention` / `shared_prefix` reorder fp32
sums of the training forward.

The kernels' own launch geometry is the C-ABI launch policy
(`swh_trl_amd._lib.launch_policy`), held per host thread by the library; a
DecodeEngine snapshots the policy it was built under and runs its launches and
graph captures under that snapshot.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Optional

TGEMM_MODES = ("off", "wgrad", "all")


@dataclass(frozen=True)
class EngineOptions:
    # ---- rollout (engine/decode.py, ref_decode.py, gpt2.py) --------------------------------------
    decode_graph: bool = True        # decode steps and the prefill forward captured into HIP graphs
    graph_steps: int = 8             # decode steps per graph replay (the ~9 us replay boundary per K)
    fused: bool = True               # the fused decode kernels (5 launches per layer + lm-head sampler)
    fold_norm: bool = True           # RMSNorm weight folded into the decode weights (one rounding, §8)
    wide_pack: bool = True           # wide_gemm's fragment-order weight copies (Llama-3-8B widths)
    fragw: bool = True               # fragment-order weight copies at the 0.5B widths
    act_frag: bool = True            # gate/up writes its activation in down_proj's fragment order
    att_frag: bool = True            # the attention writes its output in o_proj's fragment order
    shared_kv: bool = True           # one copy of a GRPO group's prompt K/V in the decode attention
    prefill_dedup: bool = True       # prefill once per distinct prompt
    fused_sample: bool = True        # lm head + unfiltered sampler in one kernel (no logits tensor)
    fused_sample_wide: bool = True   # ... also at K > 1024 on the wide tiles (config 5)
    l3_set: str = "o,down,qkv1"      # weights the attention launch's spare workgroups warm (§2e)
    l3_attn: Optional[int] = None    # warm-up workgroups (None: the engine's default, 0: off)
    # ---- training / scoring passes (engine/model.py) ---------------------------------------------
    hip_attention: bool = True       # csrc/attn.hip for the bf16 training attention (else torch SDPA)
    shared_prefix: bool = True       # a GRPO group's prompt tokens through the layers once (§12b)
    tgemm: str = "wgrad"             # csrc/tgemm.hip for narrow projections: off | wgrad | all (§14c)
    tgemm_splits: int = 8            # token splits of the gemm_tn weight gradient
    logp_chunk: int = 4096           # rows per fused lm-head log-prob chunk

    def __post_init__(self):
        if self.tgemm not in TGEMM_MODES:
            raise ValueError(f"EngineOptions.tgemm={self.tgemm!r}: expected one of {TGEMM_MODES}")
        if self.graph_steps < 1 or self.tgemm_splits < 1 or self.logp_chunk < 1:
            raise ValueError("EngineOptions: graph_steps, tgemm_splits and logp_chunk must be >= 1")

    def replace(self, **kw) -> "EngineOptions":
        return dataclasses.replace(self, **kw)


DEFAULT = EngineOptions()
