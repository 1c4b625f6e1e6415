"""gpytorch.mlls equivalents used at forecast_denoising.py:86-89 (and GPModel's partner)."""
from .gp import DeepApproximateMLL, ExactMarginalLogLikelihood, VariationalELBO  # noqa: F401
