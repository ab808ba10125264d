"""Build an A/B variant of libswh_trl_amd.so with extra hipcc defines into
tools/_build/<name>.so (load it with SWH_LIB_PATH=...).  Tuning aid only.

    python tools/build_variant.py NAME [--only attn.hip,...] -DSWH_KU=16 [...]

--only: recompile just those sources with the defines; the others are linked
from the main build's objects (swh_trl_amd/_build, current after build()).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from swh_trl_amd import build as b  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    only = None
    if defs and defs[0] == "--only":
        only, defs = set(defs[1].split(",")), defs[2:]
        b.build()
    out_dir = os.path.join(ROOT, "tools", "_build", name)
    os.makedirs(out_dir, exist_ok=True)
    objs = []
    for src in b._sources():
        base = os.path.basename(src)
        if only is not None and base not in only:
            objs.append(os.path.join(b.OBJ, base.replace(".hip", ".o")))
            continue
        obj = os.path.join(out_dir, base.replace(".hip", ".o"))
        subprocess.run([b.HIPCC, *b.FLAGS, *defs, "-c", src, "-o", obj], check=True)
        objs.append(obj)
    lib = os.path.join(ROOT, "tools", "_build", name + ".so")
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
