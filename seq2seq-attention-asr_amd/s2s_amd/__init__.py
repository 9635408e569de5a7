"""MI355X-native host layer for the seq2seq-attention-asr training step.

Mirrors the reference's Torch7 nn.Module surface for the hot path -- GRU / LSTM cells
driven by RNN, the Attention decoder (with its RNNAttention unroll), Maxout, the loss seed
and the whole Chorowski autoencoder step -- over the C ABI of libs2s_hip.so
(include/s2s_hip.h).  torch is used only for device memory and streams.
"""
from ._lib import S2SError, lib  # noqa: F401  (fails loudly when the HIP library is missing)
from .nn import (GRU, LSTM, RNN, BiRNN, Attention, MaxoutMLP, nll_seed, Context, get_context, precision,
                 overlap_param_grads)  # noqa: F401
from .model import ModelConfig, ChorowskiBaseline, param_shapes  # noqa: F401
from . import optim  # noqa: F401
from . import frontend, data, checkpoint, train_utils  # noqa: F401
from .frontend import ConvBiLSTMEncoder, VGGEncoder, VGGAttentionModel, ConvBiLSTMAttentionModel  # noqa: F401
