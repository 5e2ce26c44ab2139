"""gdm_amd -- MI355X-native operator engine for the Galerkin-difference-method
hot path of peterrum/dealii-galerkin-difference-methods.

Product path: HIP kernels in ../csrc behind the C ABI ../../include/gdm_hip.h
(libgdm_hip.so), driven from these host-side mirrors of the reference's
operator classes.  No CPU fallback exists.
"""
from ._capi import GdmError, load, declared_symbols, device_count  # noqa: F401
from .operator import GdmOperator  # noqa: F401
from .sparse import CutPoisson, SparseMatrix, solve_cg  # noqa: F401
from .problem import Advection01, AdvectionProblem, DiscreteTime, WaveProblem  # noqa: F401
from .cut_advection import CutAdvection, CutAdvectionCompositeProblem, CutAdvectionProblem  # noqa: F401
from .cut_wave import CutWave, CutWaveCompositeProblem, CutWaveProblem  # noqa: F401

__all__ = ["GdmError", "GdmOperator", "SparseMatrix", "CutPoisson", "solve_cg", "load", "declared_symbols", "device_count",
           "Advection01", "AdvectionProblem", "WaveProblem", "DiscreteTime", "CutAdvection", "CutAdvectionProblem", "CutAdvectionCompositeProblem",
           "CutWave", "CutWaveProblem", "CutWaveCompositeProblem"]
