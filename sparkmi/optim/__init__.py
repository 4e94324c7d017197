"""Fused optimizers.  On GPU with a FlatParams model, one HIP launch updates every parameter
(fp32 master + moments), refreshes the bf16 shadow and optionally zeroes the gradient
(csrc/kernels/optim.hip).  On CPU the identical formulas run in torch."""
from .adam import Adam, AdamW  # noqa: F401
from .sgd import SGD  # noqa: F401
from .lbfgs import LBFGS  # noqa: F401
