"""pint_amd — MI355X-native implementation of PINT's fit-and-residual hot path.

Reference API kept (Jackson-D-Taylor/PINT): get_model / get_model_and_toas
(model_builder.py:777/:859), Residuals (residuals.py:40), WLSFitter / GLSFitter /
DownhillWLSFitter / DownhillGLSFitter / Fitter.auto (fitter.py), grid_chisq
(gridutils.py:166).  Compute runs in libpint_hip.so (hand-written HIP for gfx950) via a
ctypes C-ABI (include/pint_amd.h); there is no CPU fallback.
"""
from .timing_model import TimingModel, get_model  # noqa: F401
from .toa import TOAs, get_TOAs, get_model_and_toas  # noqa: F401
from .residuals import Residuals, WidebandDMResiduals, WidebandTOAResiduals  # noqa: F401
from .fitter import (Fitter, WLSFitter, GLSFitter, DownhillWLSFitter, DownhillGLSFitter, WidebandTOAFitter,  # noqa: F401
                     WidebandDownhillFitter,  # noqa: F401
                     MaxiterReached, StepProblem, InvalidModelParameters, CorrelatedErrors)
from .gridutils import grid_chisq, grid_chisq_derived, tuple_chisq, tuple_chisq_derived  # noqa: F401

__version__ = "0.1.0"
