"""Exactly one HIP runtime per process ("What's weak" 2).

libgdm_hip.so NEEDs libamdhip64.so.7 with RUNPATH /opt/rocm; torch ships its
own copy with the same soname.  gdm_amd.load() preloads torch's copy so both
the engine and torch bind to ONE runtime (and one libhsa-runtime64) whichever
is imported first.  Checked from /proc/self/maps of a fresh interpreter.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dealii-galerkin-difference-methods_amd")

_MAPS = """
libs = set()
for line in open("/proc/self/maps"):
    f = line.split()[-1]
    if "libamdhip64" in f or "libhsa-runtime64" in f:
        libs.add(os.path.realpath(f))
print(repr(sorted(libs)))
"""

ORDERS = {
    "engine_first": "import gdm_amd\ngdm_amd.load()\nimport torch\n",
    "engine_count_first": "import gdm_amd\nfrom gdm_amd import _capi\n_capi.device_count()\nimport torch\n",
    "torch_first": "import torch\nimport gdm_amd\ngdm_amd.load()\n",
}


def _run(body):
    code = "import os, sys\nsys.path.insert(0, %r)\n" % PKG + body
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip().splitlines()


@pytest.mark.parametrize("order", sorted(ORDERS))
def test_one_hip_runtime_mapped(order):
    libs = eval(_run(ORDERS[order] + _MAPS)[-1])
    hip = [f for f in libs if "libamdhip64" in f]
    hsa = [f for f in libs if "libhsa-runtime64" in f]
    assert len(hip) == 1 and len(hsa) == 1, libs


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["engine_first", "engine_count_first"])
def test_torch_sees_gpu_after_engine_loads(order):
    """The failure mode of gpurun_out/cutapp/pt.log:58 ("No HIP GPUs are
    available" after the engine initialised its own runtime)."""
    out = _run(ORDERS[order] + "x = torch.ones(4, device='cuda')\nprint(float(x.sum()))\n")
    assert out[-1] == "4.0"
