"""The C-ABI library loads and exports every symbol include/swh_trl_amd.h declares
(no GPU needed: nothing is launched)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "swh_trl_amd.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char \*)\s*(swh_\w+)\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    from swh_trl_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from swh_trl_amd import build
        build.build()
    return _lib.load()


def test_header_declares_entry_points():
    names = _declared()
    assert len(names) >= 25
    for must in ("swh_logp_entropy_fwd", "swh_sample_step", "swh_grpo_loss_fwd_bwd", "swh_adamw",
                 "swh_attn_decode", "swh_gae_scan", "swh_ppo_loss_fwd_bwd"):
        assert must in names


def test_every_declared_symbol_exported_and_bound(lib):
    from swh_trl_amd import _lib
    for name in _declared():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} missing from the ctypes signature table"
    assert set(_lib.SIGNATURES) <= set(_declared())


def test_host_only_calls(lib):
    assert lib.swh_version().decode().startswith("swh_trl_amd")
    assert lib.swh_status_string(-1) == b"invalid argument"
    assert lib.swh_sqnorm_partials(10) == 1
    assert lib.swh_sqnorm_partials(10 ** 9) == 1024
    assert lib.swh_sample_workspace_bytes(64, 151936) > 0
    # argument errors are detected on the host, before any launch
    from swh_trl_amd import _lib
    with pytest.raises(ValueError):
        _lib.call("swh_logp_entropy_fwd", None, 1, 1, 1, 0, 0, 10, None, 1.0, 0, None, None, None, None)
    with pytest.raises(ValueError):
        _lib.call("swh_adamw", None, None, None, None, 1, None, 1, 10, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, None, None,
                  0, None)
    with pytest.raises(ValueError):  # dtype code outside {f32, bf16} for an fp32-model op
        _lib.call("swh_silu_mul_fwd", 8, 1, 8, 8, 7, None)


def test_struct_layouts_match_c(tmp_path):
    """ctypes mirrors of the parameter structs have the C sizes/offsets."""
    from swh_trl_amd._lib import GRPOLossParams, SampleParams
    c = tmp_path / "sz.c"
    c.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "swh_trl_amd.h"\n'
                 'int main(){printf("%zu %zu %zu %zu\\n", sizeof(swh_sample_params), '
                 'offsetof(swh_sample_params, eos_ids), sizeof(swh_grpo_loss_params), '
                 'offsetof(swh_grpo_loss_params, num_segments));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(SampleParams)
    assert int(out[1]) == SampleParams.eos_ids.offset
    assert int(out[2]) == ctypes.sizeof(GRPOLossParams)
    assert int(out[3]) == GRPOLossParams.num_segments.offset


def test_ops_refuse_cpu_tensors(lib):
    import torch
    from swh_trl_amd import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.logp_entropy(torch.randn(2, 8), torch.zeros(2, dtype=torch.long))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.group_advantages(torch.randn(8, 1), torch.ones(1), 4)
