"""Error / warning types mirroring linear_operator.utils.errors and gpytorch.utils.warnings."""


class NotPSDError(RuntimeError):
    pass


class NanError(RuntimeError):
    pass


class GpkInternalError(RuntimeError):
    """A kernel reported an internal failure (e.g. a bounded LDS spin-wait timed out,
    info = 1 << 20): a bug or a hardware fault, never a property of the inputs."""
    pass


class NumericalWarning(RuntimeWarning):
    """Mirror of gpytorch.utils.warnings.NumericalWarning."""
    pass


class GPInputWarning(UserWarning):
    """Mirror of gpytorch.utils.warnings.GPInputWarning."""
    pass
