#!/usr/bin/env python3
"""bench.py on an A/B variant of libmte.so (tools/variants.sh):
  python3 tools/bench_var.py build_var/<name>/libmte.so [bench.py args]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fluidframework_amd import _native  # noqa: E402

LIB = os.path.abspath(sys.argv[1])
_orig = _native.lib_path
_native.lib_path = lambda name: LIB if name == "libmte.so" else _orig(name)
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
