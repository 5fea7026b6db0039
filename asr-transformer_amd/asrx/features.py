"""GPU featuriser: the power spectrogram of the reference's data pipeline (modules/dataset.py:34-55).

`Spectrogram` mirrors torchaudio.transforms.Spectrogram for the configuration the reference builds
(dataset.py:34-35: n_fft=1024, center=False; torchaudio's defaults win_length=n_fft, hop_length=win_length//2,
periodic Hann window, power=2.0, normalized=False, onesided) and its forward contract: (..., time) fp32 waveform
-> (..., n_fft//2 + 1, frames), frequency-major with time innermost — the layout the model's front-end reads
(dataset.py:51-55 -> model.py:168).  It runs in libasrx.so (asrx_spectrogram: one fp32 MFMA GEMM of the framed
waveform against the windowed DFT basis, then a square/transpose pass); `pad_spectrum` is the dataset's padding and
frame mask (dataset.py:42-55).

Not covered: center=True (reflect padding), complex output (power=None), window functions other than Hann.
"""
import math

import torch
from torch import nn

from . import kernels as K
from ._lib import call


def _hann_periodic(n):
    k = torch.arange(n, dtype=torch.float64)
    return 0.5 - 0.5 * torch.cos(2.0 * math.pi * k / n)


def dft_basis(n_fft, win_length, device):
    """[2 * (n_fft//2 + 1), n_fft] fp32: rows 2n, 2n+1 = w[k] cos(2 pi n k / n_fft), -w[k] sin(...), with the
    periodic Hann window of win_length zero-padded to n_fft centred (torch.stft's window placement)."""
    nb = n_fft // 2 + 1
    w = torch.zeros(n_fft, dtype=torch.float64)
    left = (n_fft - win_length) // 2
    w[left:left + win_length] = _hann_periodic(win_length)
    k = torch.arange(n_fft, dtype=torch.float64)
    n = torch.arange(nb, dtype=torch.float64)
    ang = 2.0 * math.pi * torch.outer(n, k).remainder(n_fft) / n_fft   # exact phase: (n k) mod n_fft first
    basis = torch.empty(2 * nb, n_fft, dtype=torch.float64)
    basis[0::2] = torch.cos(ang) * w
    basis[1::2] = -torch.sin(ang) * w
    return basis.to(device=device, dtype=torch.float32).contiguous()


class Spectrogram(nn.Module):
    """torchaudio.transforms.Spectrogram(n_fft=400, win_length=None, hop_length=None, pad=0, power=2.0,
    normalized=False, center=True, onesided=True) restricted to center=False (the reference's setting), Hann
    window, power 1 or 2."""

    def __init__(self, n_fft=400, win_length=None, hop_length=None, pad=0, power=2.0, normalized=False,
                 center=True, onesided=True):
        super().__init__()
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        if center:
            raise NotImplementedError("asrx.features.Spectrogram: center=True (reflect padding) is not built; "
                                      "the reference uses center=False (dataset.py:34-35)")
        if power not in (1, 1.0, 2, 2.0):
            raise NotImplementedError("asrx.features.Spectrogram: power must be 1 or 2")
        if not onesided:
            raise NotImplementedError("asrx.features.Spectrogram: onesided=False is not built")
        if self.win_length > n_fft:
            raise ValueError("win_length must be <= n_fft")
        self.pad, self.power, self.normalized, self.center = pad, int(power), normalized, center
        self._basis = {}

    def basis(self, device):
        key = str(device)
        if key not in self._basis:
            self._basis[key] = dft_basis(self.n_fft, self.win_length, device)
        return self._basis[key]

    def forward(self, waveform):
        if not waveform.is_cuda:
            raise RuntimeError("asrx.features.Spectrogram computes on the GPU (libasrx.so); move the waveform "
                               "with .cuda()")
        shape = waveform.shape
        x = waveform.reshape(-1, shape[-1]).float()
        if self.pad > 0:
            x = torch.nn.functional.pad(x, (self.pad, self.pad))
        x = x.contiguous()
        B, T = x.shape
        nb = self.n_fft // 2 + 1
        if T < self.n_fft:
            raise ValueError(f"waveform of {T} samples is shorter than n_fft={self.n_fft}")
        frames = (T - self.n_fft) // self.hop_length + 1
        out = torch.empty(B, nb, frames, device=x.device, dtype=torch.float32)
        ws = torch.empty(B * frames * 2 * nb, device=x.device, dtype=torch.float32)
        # normalized=True (torchaudio "window"): divide the STFT by the window's L2 norm (power applies after)
        scale = 1.0
        if self.normalized:
            wn = float(_hann_periodic(self.win_length).pow(2).sum().sqrt())
            scale = 1.0 / wn ** self.power
        call("asrx_spectrogram", x.data_ptr(), B, T, x.stride(0), self.basis(x.device).data_ptr(), self.n_fft,
             self.hop_length, nb, self.power, scale, ws.data_ptr(), ws.numel(), out.data_ptr(), K.stream())
        return out.reshape(shape[:-1] + (nb, frames))


def spectrum_len(n_samples, win_length=1024, hop_length=512):
    """dataset.py:40-41 (_calculate_spectrum_len)."""
    return math.floor((n_samples - win_length) / hop_length) + 1


def pad_spectrum(spectrogram, max_frames_len, win_length=1024, hop_length=512):
    """dataset.py:47-55: pad (channels, freq, frames) with zero frames to spectrum_len(max_frames_len) and return
    (spectrogram, spectrum_mask) — ones for the real frames, zeros for the padding."""
    channels, freq, frames = spectrogram.shape
    padding_length = spectrum_len(max_frames_len, win_length, hop_length) - frames
    if padding_length < 0:
        raise ValueError(f"{frames} frames exceed the padded length {frames + padding_length} "
                         f"(dataset.py:50 would fail the same way)")
    dev = spectrogram.device
    mask = torch.cat([torch.ones(frames, device=dev), torch.zeros(padding_length, device=dev)])
    out = torch.cat([spectrogram, torch.zeros(channels, freq, padding_length, device=dev, dtype=spectrogram.dtype)],
                    dim=-1)
    return out, mask
