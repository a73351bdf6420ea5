"""BERT bench with the attention block shape forced: python tools/r2/bench_attn_waves.py <2|4> [bench args]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mipipe.ops._native import native  # noqa: E402
import bench  # noqa: E402

native().set_attn_waves(int(sys.argv[1]))
sys.argv = ["bench.py"] + sys.argv[2:]
sys.exit(bench.main())
