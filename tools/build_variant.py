"""Build an A/B variant of libswh_trl_amd.so with extra hipcc defines into
tools/_build/<name>.so (load it with SWH_LIB_PATH=...).  Tuning aid only.

    python tools/build_variant.py NAME -DSWH_KU=16 [...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from swh_trl_amd import build as b  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(ROOT, "tools", "_build", name)
    os.makedirs(out_dir, exist_ok=True)
    objs = []
    for src in b._sources():
        obj = os.path.join(out_dir, os.path.basename(src).replace(".hip", ".o"))
        subprocess.run([b.HIPCC, *b.FLAGS, *defs, "-c", src, "-o", obj], check=True)
        objs.append(obj)
    lib = os.path.join(ROOT, "tools", "_build", name + ".so")
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
