"""bench.py with the decode attention's key-split count forced (A/B of attn_splits_for at c3). Developer tool.
    python tools/c3_splits.py NSPLIT [bench.py args ...]"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import zonos_amd.engine as E  # noqa: E402

n = int(sys.argv[1])
E.attn_splits_for = lambda R, Hkv, smax, target_blocks=512: max(1, min(n, smax // 128))
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
               run_name="__main__")
