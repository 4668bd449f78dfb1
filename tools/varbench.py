#!/usr/bin/env python3
"""A/B microbenchmark of libmte.so variants (tools/variants.sh): one process per
variant (ctypes cannot unload a library).  Usage: varbench.py [variant ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys
sys.path.insert(0, ROOT)
from fluidframework_amd import _native
orig = _native.lib_path
_native.lib_path = lambda name: LIB if name == "libmte.so" else orig(name)
sys.argv = ["microbench"] + EXPS
__file__ = os.path.join(ROOT, "tools", "microbench.py")
exec(open(__file__).read().replace('if __name__ == "__main__":', "if True:"))
'''


def main():
    names = sys.argv[1:] or sorted(os.listdir(os.path.join(ROOT, "build_var")))
    exps = os.environ.get("EXPS", "scale types").split()
    for name in names:
        lib = os.path.join(ROOT, "build_var", name, "libmte.so")
        print(f"=== {name}", flush=True)
        code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(lib)).replace("EXPS", repr(exps))
        r = subprocess.run([sys.executable, "-c", code], timeout=600)
        if r.returncode != 0:
            print(f"variant {name} failed rc={r.returncode}", flush=True)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
