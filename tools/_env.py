"""Tools-only: the A/B environment switches of the measurement scripts, turned
into the product's explicit configuration (the product reads no environment).

    SWH_LIB_PATH=<.so>            another build of the library (_lib.set_library_path)
    SWH_TRACE=1                   phase timings on stderr (profiling.set_trace)
    SWH_GEMM_TUNING=use|tune|off  with SWH_GEMM_TABLE=<csv> (gemm_tuning.enable)
    SWH_WIDE_KMIN, SWH_WIDE_GEMM, SWH_WIDE_SMAX, SWH_WIDE_CB, SWH_GEMM_NW, SWH_XSTREAM,
    SWH_LM_RING14, SWH_FILT_WGS, SWH_WIDE_WAVES, SWH_ATTN_PAIR, SWH_GEMM_CFG
                                  the launch policy of the calling thread
    SWH_DECODE_GRAPH, SWH_DECODE_GRAPH_STEPS, SWH_DECODE_FUSED, SWH_DECODE_FOLD, SWH_WIDE_PACK,
    SWH_FRAGW, SWH_ACT_FRAG, SWH_ATT_FRAG, SWH_DECODE_SHARED_KV, SWH_PREFILL_DEDUP,
    SWH_FUSED_SAMPLE, SWH_FUSED_SAMPLE_WIDE, SWH_DECODE_L3_SET, SWH_DECODE_L3_ATTN, SWH_ATTN,
    SWH_SHARED_PREFIX, SWH_TGEMM, SWH_TGEMM_SPLITS, SWH_LOGP_CHUNK
                                  fields of engine.options.EngineOptions (`options()`)

`apply()` is called by every tool before it touches the library; a tool hands
`options()` to the models / engines it builds (`model.options = options()`).
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_POLICY = {"SWH_WIDE_KMIN": "wide_kmin", "SWH_WIDE_GEMM": "wide_gemm", "SWH_WIDE_SMAX": "wide_smax",
           "SWH_WIDE_CB": "wide_cb", "SWH_GEMM_NW": "gemm_nw", "SWH_XSTREAM": "xstream",
           "SWH_LM_RING14": "lm_ring14", "SWH_FILT_WGS": "filt_wgs", "SWH_WIDE_WAVES": "wide_waves",
           "SWH_ATTN_PAIR": "attn_pair"}

_BOOL = {"SWH_DECODE_GRAPH": "decode_graph", "SWH_DECODE_FUSED": "fused", "SWH_DECODE_FOLD": "fold_norm",
         "SWH_WIDE_PACK": "wide_pack", "SWH_FRAGW": "fragw", "SWH_ACT_FRAG": "act_frag", "SWH_ATT_FRAG": "att_frag",
         "SWH_DECODE_SHARED_KV": "shared_kv", "SWH_PREFILL_DEDUP": "prefill_dedup",
         "SWH_FUSED_SAMPLE": "fused_sample", "SWH_FUSED_SAMPLE_WIDE": "fused_sample_wide",
         "SWH_SHARED_PREFIX": "shared_prefix"}
_INT = {"SWH_DECODE_GRAPH_STEPS": "graph_steps", "SWH_DECODE_L3_ATTN": "l3_attn", "SWH_TGEMM_SPLITS": "tgemm_splits",
        "SWH_LOGP_CHUNK": "logp_chunk"}
_STR = {"SWH_DECODE_L3_SET": "l3_set", "SWH_TGEMM": "tgemm"}


def options(**overrides):
    """EngineOptions from the environment's switches (defaults for the rest)."""
    from swh_trl_amd.engine.options import EngineOptions
    kw = {}
    for e, f in _BOOL.items():
        if os.environ.get(e):
            kw[f] = os.environ[e] != "0"
    for e, f in _INT.items():
        if os.environ.get(e):
            kw[f] = int(os.environ[e])
    for e, f in _STR.items():
        if os.environ.get(e):
            kw[f] = os.environ[e]
    if os.environ.get("SWH_ATTN"):
        kw["hip_attention"] = os.environ["SWH_ATTN"] != "torch"
    kw.update(overrides)
    return EngineOptions(**kw)


def apply() -> None:
    """Library path, launch policy, tracing and GEMM tuning from the environment."""
    from swh_trl_amd import _lib, gemm_tuning, profiling
    if os.environ.get("SWH_LIB_PATH"):
        _lib.set_library_path(os.environ["SWH_LIB_PATH"])
    kw = {f: int(os.environ[e]) for e, f in _POLICY.items() if os.environ.get(e)}
    if os.environ.get("SWH_GEMM_CFG"):
        kw["gemm_cfg"] = os.environ["SWH_GEMM_CFG"]
    if kw:
        _lib.set_launch_policy(**kw)
    if os.environ.get("SWH_TRACE") == "1":
        profiling.set_trace(True)
    if os.environ.get("SWH_GEMM_TUNING") or os.environ.get("SWH_GEMM_TABLE"):
        gemm_tuning.enable(os.environ.get("SWH_GEMM_TUNING"), os.environ.get("SWH_GEMM_TABLE"))
