"""Error / warning types mirroring linear_operator.utils.errors and gpytorch.utils.warnings."""


class NotPSDError(RuntimeError):
    pass


class NanError(RuntimeError):
    pass


class NumericalWarning(RuntimeWarning):
    """Mirror of gpytorch.utils.warnings.NumericalWarning."""
    pass
