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


def test_launch_policy_roundtrip_and_validation(lib):
    """The launch policy is the library's only settable state: defaults, a
    round trip, range checks on the host, and restore."""
    from swh_trl_amd import _lib
    d = _lib.LaunchPolicy()
    assert lib.swh_launch_policy_default(ctypes.byref(d)) == 0
    assert (d.wide_kmin, d.wide_gemm, d.wide_smax, d.xstream, d.lm_ring14, d.filt_wgs, d.wide_waves,
            d.attn_pair) == (2048, 1, 8, 1, 1, 1024, 0, 1)
    before = _lib.get_launch_policy()
    try:
        with _lib.launch_policy(gemm_cfg="4,2,1,1", xstream=0, wide_cb=2, wide_waves=7):
            p = _lib.get_launch_policy()
            assert (p["gemm_ms"], p["gemm_cb"], p["gemm_s"], p["gemm_persist"], p["gemm_wn"]) == (4, 2, 1, 1, 1)
            assert p["xstream"] == 0 and p["wide_cb"] == 2 and p["wide_waves"] == 7
        assert _lib.get_launch_policy() == before
        for bad in ({"wide_smax": 9}, {"wide_cb": 3}, {"gemm_cfg": "3,1,1"}, {"gemm_nw": 5}, {"filt_wgs": 1}, {"wide_waves": 5}, {"attn_pair": 2},
                    {"gemm_cb": 2}):  # a geometry field without gemm_ms
            with pytest.raises(ValueError):
                _lib.set_launch_policy(**bad)
            assert _lib.get_launch_policy() == before
        with pytest.raises(ValueError, match="unknown"):
            _lib.set_launch_policy(not_a_field=1)
    finally:
        _lib.set_launch_policy(**before)


def test_host_entry_points_are_thread_safe(lib):
    """Host-side entry points (eligibility, workspace sizing over the cost model
    and the per-device CU table, the policy) called from 8 host threads at once,
    while another thread flips its own launch policy, agree with single-threaded
    answers: the per-device tables are initialised under std::call_once and each
    thread holds its own policy."""
    import threading

    from swh_trl_amd import _lib
    shapes = [(64, 896, 896, 0), (64, 1152, 896, 0), (64, 4864, 896, 1), (64, 896, 4864, 0), (64, 4096, 4096, 0),
              (64, 14336, 4096, 1), (64, 4096, 14336, 0), (64, 128256, 4096, 0), (5, 256, 512, 0)]

    def answers():
        out = []
        for M, N, K, silu in shapes:
            out.append((lib.swh_wide_gemm_eligible(M, N, K, silu), lib.swh_decode_gemm_workspace_bytes(M, N, K),
                        lib.swh_lm_head_sample_workspace_bytes(M, N, K), lib.swh_sample_workspace_bytes(M, N)))
        return out

    want = answers()
    before = _lib.get_launch_policy()
    errors, stop = [], threading.Event()

    def worker():
        try:
            for _ in range(200):
                assert answers() == want
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def flipper():  # policy changes that leave every answer above unchanged
        while not stop.is_set():
            for v in (0, 1):
                _lib.set_launch_policy(xstream=v, lm_ring14=v)

    ts = [threading.Thread(target=worker) for _ in range(8)]
    f = threading.Thread(target=flipper)
    f.start()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    stop.set()
    f.join()
    _lib.set_launch_policy(**before)
    assert not errors, errors


def test_library_holds_no_hidden_state():
    """csrc/ reads no environment variable and declares no mutable static
    outside the call_once-guarded per-device tables (csrc/lib.hip, the LDS
    opt-in of common.hpp); the launch policy is thread_local (one per host
    thread), nothing process-wide."""
    csrc = os.path.join(ROOT, "swh_trl_amd", "csrc")
    allowed = {("lib.hip", "static std::once_flag once[kMaxDevices];"), ("lib.hip", "static int cus[kMaxDevices];"),
               ("common.hpp", "static std::once_flag once[kMaxDevices];"),
               ("common.hpp", "static bool ok[kMaxDevices];")}
    found = set()
    for f in sorted(os.listdir(csrc)):
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(csrc, f)).read(), flags=re.S)
        for line in src.split("\n"):
            code = line.split("//")[0].strip()
            assert "getenv" not in code, (f, line)
            m = re.match(r"static\s+(?!constexpr|inline|__|void\b)([\w:<>, ]+?)\s+(\w+)\s*(\[[^\]]*\])?\s*(=|;|\{)", code)
            if m and "(" not in code.split("=")[0]:
                found.add((f, code))
    assert found == allowed, found ^ allowed
    lib_src = open(os.path.join(csrc, "lib.hip")).read()
    assert "thread_local swh_launch_policy" in lib_src and "std::call_once" in lib_src
    assert "g_policy" not in lib_src and "std::mutex" not in lib_src


def test_launch_policy_is_per_thread(lib):
    """Two host threads hold their own launch policies: a thread's set does not
    reach another thread, a new thread starts at the defaults, and each thread
    reads back exactly what it set (include/swh_trl_amd.h: no process-wide
    mutable state)."""
    import threading

    from swh_trl_amd import _lib
    d = _lib.LaunchPolicy()
    lib.swh_launch_policy_default(ctypes.byref(d))
    default = {f: getattr(d, f) for f, _ in _lib.LaunchPolicy._fields_}
    before = _lib.get_launch_policy()
    barrier = threading.Barrier(2, timeout=30)
    seen, errors = {}, []

    def worker(name, fields):
        try:
            seen[name + ".start"] = _lib.get_launch_policy()
            _lib.set_launch_policy(**fields)
            barrier.wait()  # both threads have set theirs
            for _ in range(100):
                p = _lib.get_launch_policy()
                assert all(p[k] == v for k, v in fields.items()), (name, p)
            barrier.wait()
            seen[name + ".end"] = _lib.get_launch_policy()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ta = threading.Thread(target=worker, args=("a", {"xstream": 0, "wide_cb": 1, "attn_pair": 0}))
    tb = threading.Thread(target=worker, args=("b", {"xstream": 1, "wide_cb": 2, "filt_wgs": 512}))
    ta.start()
    tb.start()
    ta.join()
    tb.join()
    assert not errors, errors
    assert seen["a.start"] == default and seen["b.start"] == default
    assert seen["a.end"]["wide_cb"] == 1 and seen["b.end"]["wide_cb"] == 2 and seen["b.end"]["attn_pair"] == 1
    assert _lib.get_launch_policy() == before  # this thread untouched


def test_product_reads_no_environment():
    """The product's configuration is explicit (engine/options.py EngineOptions,
    the per-thread launch policy, call arguments): no module under swh_trl_amd/
    reads os.environ / os.getenv, except dist.py's launcher contract
    (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*, torchrun's)."""
    import ast
    pkg = os.path.join(ROOT, "swh_trl_amd")
    bad = []
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if not fn.endswith(".py"):
                continue
            path = os.path.join(dirpath, fn)
            rel = os.path.relpath(path, ROOT)
            if rel == os.path.join("swh_trl_amd", "dist.py"):
                continue
            for node in ast.walk(ast.parse(open(path).read())):
                if isinstance(node, ast.Attribute) and node.attr in ("environ", "getenv", "putenv") and \
                        isinstance(node.value, ast.Name) and node.value.id == "os":
                    bad.append(f"{rel}:{node.lineno}")
    assert not bad, bad
