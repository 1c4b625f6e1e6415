"""MI355X-native GP blur/denoise hot path (RBF + Cholesky + MLL/ELBO) for
SepKfr/Fine_grained_Gaussian_Process_Forcasting, behind the reference's own
class surface."""
from . import _native, ops, library  # noqa: F401  (library registers the gpk:: ops)
from . import gp, mlls, likelihoods  # noqa: F401
from .gp import settings  # noqa: F401
from .errors import GPInputWarning, GpkInternalError, NanError, NotPSDError, NumericalWarning  # noqa: F401

__version__ = "0.1.0"
