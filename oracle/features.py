"""Test oracle (never imported by the product): numpy restatement of the reference featuriser,
modules/dataset.py:34-55 — torchaudio.transforms.Spectrogram(n_fft=1024, center=False).

torchaudio is not installed here, so this follows torchaudio's published algorithm
(torchaudio.functional.spectrogram, torchaudio 2.x): torch.stft(waveform, n_fft, hop_length, win_length,
window=hann_window(win_length) [periodic], center=False, normalized=False, onesided=True, return_complex=True),
then .abs().pow(power).  The restatement is pinned against torch.stft itself — the function torchaudio calls —
in tests/test_features.py (the reference's own call chain below torchaudio), not against torchaudio's output.
"""
import math

import numpy as np


def hann_periodic(n):
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)


def spectrogram(audio, n_fft=1024, win_length=None, hop_length=None, power=2.0, normalized=False):
    """audio (..., T) float -> (..., n_fft//2 + 1, frames) float64; center=False framing (dataset.py:34-35)."""
    win_length = win_length or n_fft
    hop_length = hop_length or win_length // 2
    a = np.asarray(audio, dtype=np.float64)
    lead, T = a.shape[:-1], a.shape[-1]
    a = a.reshape(-1, T)
    frames = (T - n_fft) // hop_length + 1
    w = np.zeros(n_fft)
    left = (n_fft - win_length) // 2
    w[left:left + win_length] = hann_periodic(win_length)
    idx = np.arange(frames)[:, None] * hop_length + np.arange(n_fft)[None, :]
    fr = a[:, idx] * w                                   # (B, frames, n_fft)
    spec = np.abs(np.fft.rfft(fr, axis=-1))              # (B, frames, nbins)
    if normalized:
        spec = spec / math.sqrt((hann_periodic(win_length) ** 2).sum())
    spec = spec ** power
    return spec.transpose(0, 2, 1).reshape(lead + (n_fft // 2 + 1, frames))
