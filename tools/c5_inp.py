"""bench.py with the hybrid's Mamba in_proj split-K forced (A/B of MAMBA_INP_SPLIT at c5). Developer tool.
    python tools/c5_inp.py NSPLIT [bench.py args ...]"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import zonos_amd.hybrid as Hy  # noqa: E402

Hy.MAMBA_INP_SPLIT = int(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
               run_name="__main__")
