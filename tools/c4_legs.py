#!/usr/bin/env python3
"""bench.py's C4 legs alone (c4_wave_stage: full 256^3 p = 7 wave stencil, mass
inverse, RK stage, and the rank-3-of-8 slab), one JSON line: experiment tool
(GDM_HIP_LIB selects a variant library)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

import bench  # noqa: E402

print(json.dumps(bench.c4_wave_stage(int(sys.argv[1]) if len(sys.argv) > 1 else 20)))
