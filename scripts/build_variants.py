"""Build diagnostic / A-B variants of the library into build/variants/<name>.so (CPU, here; the
.so files travel to the GPU box with the tree).  usage:
    python scripts/build_variants.py NAME=-DFLAG=1,-DOTHER=2 NAME2= ...
An empty flag list builds the default library under that name."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def one(spec):
    name, _, flags = spec.partition("=")
    out = os.path.join(ROOT, "build", "variants", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    fl = [f for f in flags.split(",") if f] or ["-DHG_VARIANT_DEFAULT=1"]   # non-empty: force a rebuild
    ge.build_lib(fl, out)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)
