"""asrx — MI355X-native (gfx950) Speech-Transformer attention path.

Drop-in modules for shockless/asr-transformer's modules/Transformer/{layers,model}.py backed by the C-ABI
library libasrx.so (hand-written HIP/CDNA4 kernels).  There is no CPU fallback: the modules require the
native library and a GPU.
"""
from .layers import MHA, FeedForward, LayerNorm, TrainablePositionalEncoding  # noqa: F401
from .model import Decoder, DecoderLayer, Encoder, EncoderLayer, FrontEnd, Transformer, subsampled  # noqa: F401

__version__ = "0.1.0"


def native():
    """The loaded ctypes library (raises if libasrx.so is missing)."""
    from ._lib import lib
    return lib()
