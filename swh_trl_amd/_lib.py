"""ctypes binding of the C-ABI in include/swh_trl_amd.h.

The shared library is the ONLY compute path of this package: there is no CPU
fallback.  If `libswh_trl_amd.so` is missing the import of any op raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libswh_trl_amd.so")

c_i32, c_i64, c_f32, c_vp, c_u64 = C.c_int32, C.c_int64, C.c_float, C.c_void_p, C.c_uint64

SWH_F32, SWH_BF16, SWH_F16 = 0, 1, 2
SWH_LOGP_ROUND_SCALED = 1
LOSS_TYPES = {"grpo": 0, "bnpo": 1, "dr_grpo": 2}
IS_LEVELS = {"token": 0, "sequence": 1}


class AttnView(C.Structure):
    """swh_attn_view (include/swh_trl_amd.h)."""
    _fields_ = [("base", C.c_void_p * 2), ("sb", c_i64 * 2), ("sh", c_i64 * 2), ("sl", c_i64 * 2),
                ("div", c_i32 * 2)]


class SampleParams(C.Structure):
    """swh_sample_params (include/swh_trl_amd.h)."""
    _fields_ = [("temperature", c_f32), ("top_p", c_f32), ("min_p", c_f32), ("repetition_penalty", c_f32),
                ("top_k", c_i32), ("greedy", c_i32), ("min_new_tokens", c_i32), ("pad_token_id", c_i32),
                ("n_eos", c_i32), ("eos_ids", c_i32 * 4)]


class GRPOLossParams(C.Structure):
    """swh_grpo_loss_params (include/swh_trl_amd.h)."""
    _fields_ = [("beta", c_f32), ("epsilon_low", c_f32), ("epsilon_high", c_f32), ("delta", c_f32),
                ("loss_type", c_i32), ("is_level", c_i32), ("max_completion_length", c_i32),
                ("num_segments", c_i32)]


class LaunchPolicy(C.Structure):
    """swh_launch_policy (include/swh_trl_amd.h): geometry choices of the decode
    GEMMs, attention and samplers, set explicitly and held per host thread.  Every
    alternative is bit-identical except wide_smax, wide_cb, wide_waves and
    attn_pair, which change the fp32 summation order (each deterministic)."""
    _fields_ = [("wide_kmin", c_i64), ("wide_gemm", c_i32), ("wide_smax", c_i32), ("wide_cb", c_i32),
                ("gemm_ms", c_i32), ("gemm_cb", c_i32), ("gemm_s", c_i32), ("gemm_persist", c_i32),
                ("gemm_wn", c_i32), ("gemm_tile", c_i32), ("gemm_nw", c_i32), ("xstream", c_i32),
                ("lm_ring14", c_i32), ("filt_wgs", c_i32), ("wide_waves", c_i32), ("attn_pair", c_i32)]


# name -> (restype, argtypes)
SIGNATURES = {
    "swh_version": (C.c_char_p, []),
    "swh_status_string": (C.c_char_p, [c_i32]),
    "swh_launch_policy_default": (c_i32, [C.POINTER(LaunchPolicy)]),
    "swh_get_launch_policy": (c_i32, [C.POINTER(LaunchPolicy)]),
    "swh_set_launch_policy": (c_i32, [C.POINTER(LaunchPolicy)]),
    "swh_logp_entropy_fwd": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_f32, c_i32,
                                     c_vp, c_vp, c_vp, c_vp]),
    "swh_log_softmax_gather_exact": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "swh_logp_bwd": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_f32, c_i32, c_vp, c_vp,
                             c_vp, c_i64, c_i64, c_vp]),
    "swh_sample_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "swh_sample_step": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, C.POINTER(SampleParams), c_vp, c_vp, c_vp,
                                c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "swh_seen_init": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "swh_step_advance": (c_i32, [c_vp, c_vp]),
    "swh_completion_mask": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "swh_group_advantage": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_vp]),
    "swh_grpo_loss_workspace_bytes": (c_i64, [c_i64]),
    "swh_grpo_loss_fwd_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                      C.POINTER(GRPOLossParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "swh_masked_whiten_workspace_bytes": (c_i64, [c_i64]),
    "swh_masked_whiten": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "swh_gae_scan": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_vp, c_vp, c_vp]),
    "swh_ppo_loss_workspace_bytes": (c_i64, [c_i64]),
    "swh_ppo_loss_fwd_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32,
                                     c_f32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "swh_ppo_truncate": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "swh_ppo_rewards": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_i32, c_f32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "swh_value_head_fwd": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "swh_sqnorm_partials": (c_i64, [c_i64]),
    "swh_grad_sqnorm": (c_i32, [c_vp, c_i32, c_i64, c_vp, c_vp]),
    "swh_finalize_clip": (c_i32, [c_vp, c_i64, c_f32, c_vp, c_vp]),
    "swh_adamw": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32,
                          c_i64, c_vp, c_vp, c_i32, c_vp]),
    "swh_accumulate": (c_i32, [c_vp, c_vp, c_i32, c_i64, c_f32, c_vp]),
    "swh_dw_reduce": (c_i32, [c_vp, c_i32, c_i64, c_vp, c_i32, c_vp]),
    "swh_gemm_nt": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "swh_gemm_nt256": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "swh_gemm_tn_partials": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp]),
    "swh_gemm_tn256_partials": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp]),
    "swh_gemm_tn_fold": (c_i32, [c_vp, c_i32, c_i64, c_vp, c_i32, c_vp]),
    "swh_ema_mix": (c_i32, [c_vp, c_vp, c_i32, c_i64, c_f32, c_f32, c_vp]),
    "swh_rmsnorm_fwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_vp, c_vp, c_i32, c_vp]),
    "swh_rmsnorm_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "swh_rmsnorm_dw_accum": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_vp]),
    "swh_colsum_partials": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp]),
    "swh_layernorm_fwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "swh_layernorm_bwd_partial_rows": (c_i64, [c_i64, c_i64]),
    "swh_layernorm_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i32,
                                  c_vp]),
    "swh_gelu_tanh_fwd": (c_i32, [c_vp, c_i64, c_vp, c_i32, c_vp]),
    "swh_gelu_tanh_bwd": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "swh_silu_mul_fwd": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_vp]),
    "swh_silu_mul_bwd": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i32, c_vp]),
    "swh_attn_fwd": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "swh_attn_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp,
                             c_vp, c_vp, c_vp, c_vp, c_vp]),
    "swh_attn_bwd_parts": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i64, c_i32, c_f32, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "swh_attn_fwd_v": (c_i32, [C.POINTER(AttnView)] * 4 + [c_i64, c_i32, c_i32, c_i64, c_i64, c_i32, c_i32, c_f32,
                                                            c_vp, c_vp, c_vp, c_vp]),
    "swh_attn_bwd_v_parts": (c_i32, [C.POINTER(AttnView)] * 5 + [c_vp, c_i64, c_i32, c_i32, c_i64, c_i64, c_i32,
                                                                  c_i32, c_f32, c_vp, c_vp, c_vp] +
                             [C.POINTER(AttnView)] * 3 + [c_i32, c_vp]),
    "swh_fold_norm": (c_i32, [c_vp, c_i32, c_i64, c_vp]),
    "swh_embedding_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "swh_embedding_bwd": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "swh_embed_gather": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "swh_qkv_rope": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32,
                             c_i32, c_vp]),
    "swh_attn_decode": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32,
                                c_f32, c_vp, c_vp]),
    "swh_attn_decode_shared": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32,
                                       c_i32, c_f32, c_vp, c_vp]),
    "swh_attn_decode_shared_frag": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32,
                                            c_i32, c_i32, c_f32, c_vp, c_i32, c_vp]),
    "swh_decode_gemm_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "swh_lm_head_sample_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "swh_lm_head_sample": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, C.POINTER(SampleParams),
                                   c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "swh_lm_head_sample_step": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, C.POINTER(SampleParams),
                                        c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "swh_lm_head_sample_fragw": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_vp, C.POINTER(SampleParams),
                                         c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "swh_lm_head_sample_step_fragw": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_vp, C.POINTER(SampleParams),
                                              c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                              c_vp]),
    "swh_lm_head_sample_logp": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, c_i32,
                                        C.POINTER(SampleParams), c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                        c_vp, c_vp, c_vp, c_i64, c_vp]),
    "swh_decode_gemm": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, c_vp, c_i32, c_vp, c_i64,
                                c_vp, c_vp, c_vp, c_i64, c_vp]),
    "swh_wide_gemm_eligible": (c_i32, [c_i64, c_i64, c_i64, c_i32]),
    "swh_wide_pack": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp]),
    "swh_frag_pack": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp]),
    "swh_decode_gemm_fragw": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp,
                                      c_vp, c_i32, c_vp, c_i64, c_vp]),
    "swh_wide_gemm_packed": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp,
                                     c_vp, c_vp, c_i64, c_vp]),
    "swh_attn_decode_l3": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32,
                                   c_f32, c_vp, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp]),
}

_lib = None
_lock = threading.Lock()
_path = [LIB_PATH]


def set_library_path(path: str) -> None:
    """Load another build of the library (A/B timing of two builds, tools only);
    must precede the first load()."""
    if _lib is not None and os.path.abspath(path) != os.path.abspath(_path[0]):
        raise RuntimeError("swh_trl_amd library already loaded from " + _path[0])
    _path[0] = path


def load() -> C.CDLL:
    """Load the HIP library (once).  Raises if it is not built: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = _path[0]
            if not os.path.exists(path):
                raise RuntimeError(f"{path} is missing: build it with `python swh_trl_amd/build.py` "
                                   "(the swh_trl_amd ops have no CPU fallback)")
            lib = C.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def _geometry_fields(cfg: str) -> dict:
    """"ms,cb,s[,p[,wn]]" or "t" (the tile kernel) -> policy fields."""
    if cfg == "t":
        return {"gemm_tile": 1}
    v = [int(x) for x in cfg.split(",")]
    if len(v) < 3:
        raise ValueError(f"decode_gemm geometry {cfg!r}: expected 'ms,cb,s[,persist[,wn]]'")
    v = v + [0, 1][len(v) - 3:]  # persist 0, wn 1 unless given
    return dict(zip(("gemm_ms", "gemm_cb", "gemm_s", "gemm_persist", "gemm_wn"), v))


def get_launch_policy() -> dict:
    """The calling thread's launch policy (the library holds one per host thread)."""
    p = LaunchPolicy()
    check(load().swh_get_launch_policy(C.byref(p)), "swh_get_launch_policy")
    return {f: getattr(p, f) for f, _ in LaunchPolicy._fields_}


def set_launch_policy(**fields) -> dict:
    """Set policy fields (the others keep their value); `gemm_cfg="ms,cb,s[,p[,wn]]"`
    / "t" / None sets or clears the decode_gemm geometry override.  Returns the
    previous policy."""
    lib = load()
    old = get_launch_policy()
    new = dict(old)
    if "gemm_cfg" in fields:
        cfg = fields.pop("gemm_cfg")
        new.update(gemm_ms=0, gemm_cb=0, gemm_s=0, gemm_persist=0, gemm_wn=0, gemm_tile=0)
        if cfg:
            new.update(_geometry_fields(cfg))
    unknown = set(fields) - set(new)
    if unknown:
        raise ValueError(f"unknown launch policy fields {sorted(unknown)}")
    new.update(fields)
    check(lib.swh_set_launch_policy(C.byref(LaunchPolicy(**new))), "swh_set_launch_policy")
    return old


class launch_policy:
    """Context manager: `with launch_policy(xstream=0): ...` runs the block's
    launches (and graph captures) on this thread under the given policy, then
    restores the thread's previous one.  Other threads keep their own."""

    def __init__(self, **fields):
        self.fields = fields

    def __enter__(self):
        self.old = set_launch_policy(**self.fields)
        return self

    def __exit__(self, *exc):
        lib = load()
        check(lib.swh_set_launch_policy(C.byref(LaunchPolicy(**self.old))), "swh_set_launch_policy")
        return False


def check(status: int, name: str) -> None:
    if status == 0:
        return
    msg = load().swh_status_string(status).decode()
    if status in (-1, -3):
        raise ValueError(f"{name}: {msg} (status {status})")
    raise RuntimeError(f"{name}: {msg} (status {status})")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def dtype_code(t, name: str) -> int:
    """The `int dtype` argument of an entry point, taken from the tensor it
    describes.  The C-ABI cannot see buffer sizes, so a code that does not match
    the buffer makes the kernel read / write the wrong element width (round 4:
    a literal SWH_F32 passed for bf16 buffers wrote past both allocations);
    every call site derives its code here (tests/test_abi.py checks that no
    call passes a literal)."""
    import torch
    codes = {torch.float32: SWH_F32, torch.bfloat16: SWH_BF16, torch.float16: SWH_F16}
    if t.dtype not in codes:
        raise ValueError(f"swh_trl_amd.{name}: unsupported dtype {t.dtype}")
    return codes[t.dtype]
