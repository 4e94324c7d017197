"""sparkmi fused ops: autograd Functions whose GPU path is a hand-written HIP/CDNA4 kernel
(sparkmi._C) and whose CPU path is the same math in fp32 torch (the numerics reference)."""
from .attention import attention_reference, cross_attention, self_attention  # noqa: F401
from .embedding import embedding, sinusoid_table  # noqa: F401
from .layernorm import add_dropout_layernorm  # noqa: F401
from .linear import linear  # noqa: F401
from .loss import cross_entropy  # noqa: F401
from .rng import DropoutRNG  # noqa: F401
