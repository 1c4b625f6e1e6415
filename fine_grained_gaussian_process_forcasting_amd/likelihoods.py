"""gpytorch.likelihoods equivalents used on the path (train.py:57, DeepGP.py:88)."""
from .gp import GaussianLikelihood  # noqa: F401
