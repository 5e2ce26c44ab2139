#!/usr/bin/env python3
"""The per-rank legs of bench.py (c3_rank_slab, c4_rank_slab) alone, one JSON
line: experiment tool (GDM_HIP_LIB selects a variant library)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
print(json.dumps({"c3": bench.c3_rank_slab(steps), "c4": bench.c4_rank_slab(steps)}))
