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


def _dtype_positions():
    """{entry point: [argument positions whose C parameter is a dtype code]} from
    the header's prototypes (parameters named `dtype`, `grad_dtype`, ...)."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for name, params in re.findall(r"(?:int|int64_t)\s+(swh_\w+)\(([^;{]*)\)\s*;", src):
        names = [p.strip().split()[-1].lstrip("*") for p in params.split(",") if p.strip() and p.strip() != "void"]
        pos = [i for i, n in enumerate(names) if n == "dtype" or n.endswith("_dtype")]
        if pos:
            out[name] = pos
    return out


def _python_sources():
    skip = {os.path.join(ROOT, "tests", "test_abi.py")}  # the argument-error probes above pass bad codes on purpose
    for top in ("swh_trl_amd", "tools", "tests"):
        for d, _, files in os.walk(os.path.join(ROOT, top)):
            for f in files:
                if f.endswith(".py") and os.path.join(d, f) not in skip:
                    yield os.path.join(d, f)
    yield os.path.join(ROOT, "bench.py")
    yield os.path.join(ROOT, "__graft_entry__.py")


def test_no_call_site_passes_a_literal_dtype_code():
    """Every dtype code handed to the C-ABI comes from the tensor it describes
    (`_lib.dtype_code`).  Round 4's hipErrorIllegalAddress came from a literal 0
    (SWH_F32) passed for bf16 buffers in a tool: the library cannot see buffer
    sizes, so the kernel read and wrote 4-byte elements over 2-byte allocations.
    Checked statically over every `call("swh_...", ...)` / `lib.swh_...(...)`."""
    import ast
    pos = _dtype_positions()
    assert {"swh_dw_reduce", "swh_adamw", "swh_logp_entropy_fwd", "swh_rmsnorm_fwd"} <= set(pos)
    assert pos["swh_adamw"] == [4, 6]
    bad, seen = [], 0
    for path in _python_sources():
        tree = ast.parse(open(path).read(), path)
        for node in ast.walk(tree):
            if not isinstance(node, ast.Call):
                continue
            f, args = node.func, node.args
            if isinstance(f, ast.Name) and f.id == "call" or isinstance(f, ast.Attribute) and f.attr == "call":
                if not args or not isinstance(args[0], ast.Constant) or not isinstance(args[0].value, str):
                    continue
                name, args = args[0].value, args[1:]
            elif isinstance(f, ast.Attribute) and f.attr.startswith("swh_"):
                name = f.attr
            else:
                continue
            for i in pos.get(name, []):
                if i >= len(args):
                    continue
                seen += 1
                a = args[i]
                literal = isinstance(a, ast.Constant) or (isinstance(a, (ast.Name, ast.Attribute)) and
                                                          (getattr(a, "id", None) or a.attr).startswith("SWH_"))
                if literal:
                    bad.append(f"{os.path.relpath(path, ROOT)}:{node.lineno} {name} arg {i}")
    assert seen >= 30, seen
    assert not bad, bad
