"""asrx.new — the reference's second model family (modules/Transformer/new/: post-LN layers, full-width heads,
length masks) as drop-in modules on libasrx.so.  See asrx/new/model.py."""
from .layers import MHA, FeedForward, TrainablePositionalEncoding  # noqa: F401
from .model import Decoder, DecoderLayer, Encoder, EncoderLayer, Transformer  # noqa: F401
from .train import clip_grad_norm_, eval_epoch, remove_after_eos, train_epoch, word_error_rate  # noqa: F401
