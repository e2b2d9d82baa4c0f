"""hipps — MI355X-native parameter-server training (capabilities of stsievert/pytorch-ps-mpi).

Public API (reference __init__.py:1 exports MPI_PS, Adam, SGD):

    from hipps import MPI_PS, SGD, Adam, PSConfig, get_codec
"""
from .config import PSConfig
from .codecs import Codec, Identity, Int8, TopK, TopKInt8, get_codec
from .optim import MPI_PS, SGD, Adam
from .ops.nn import set_deterministic

__version__ = "0.1.0"
__all__ = ["MPI_PS", "SGD", "Adam", "PSConfig", "Codec", "Identity", "Int8", "TopK", "TopKInt8", "get_codec",
           "set_deterministic"]
