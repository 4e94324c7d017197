"""Model families of the reference: MLP (R03), CNN (R10), LSTM (R18), Transformer (R24-R38)."""
from .cnn import CNN, FashionMNISTModel  # noqa: F401
from .lstm import LSTM  # noqa: F401
from .mlp import Multilayer_perceptor, MultilayerPerceptron  # noqa: F401
from .transformer import Transformer  # noqa: F401
