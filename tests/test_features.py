"""The GPU featuriser (asrx.features; reference modules/dataset.py:34-55) against the numpy oracle, and the oracle
against torch.stft — the function torchaudio.transforms.Spectrogram calls (torchaudio itself is not installed)."""
import numpy as np
import pytest
import torch

from oracle import features as F


@pytest.mark.parametrize("T,n_fft,hop,win", [(16000, 1024, 512, 1024), (5000, 400, 200, 400), (3000, 512, 128, 400)])
def test_oracle_matches_torch_stft(T, n_fft, hop, win):
    g = torch.Generator().manual_seed(T)
    x = torch.randn(2, T, generator=g, dtype=torch.float64)
    ref = torch.stft(x, n_fft, hop_length=hop, win_length=win, window=torch.hann_window(win, dtype=torch.float64),
                     center=False, normalized=False, onesided=True, return_complex=True).abs().pow(2.0)
    got = F.spectrogram(x.numpy(), n_fft=n_fft, win_length=win, hop_length=hop)
    assert got.shape == tuple(ref.shape)
    np.testing.assert_allclose(got, ref.numpy(), rtol=1e-9, atol=1e-9 * float(ref.abs().max()))


def test_pad_spectrum_and_len():
    from asrx.features import pad_spectrum, spectrum_len
    assert spectrum_len(2048) == 3 and spectrum_len(16000) == 30
    s = torch.ones(1, 5, 2)
    out, mask = pad_spectrum(s, 2048)
    assert out.shape == (1, 5, 3) and mask.tolist() == [1.0, 1.0, 0.0] and float(out[..., 2].abs().sum()) == 0.0
    with pytest.raises(ValueError):
        pad_spectrum(torch.ones(1, 5, 4), 2048)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,n_fft,hop,win,power,normalized", [
    ((4, 16000), 1024, 512, 1024, 2, False),      # the reference's setting (dataset.py:34-35), 1 s at 16 kHz
    ((2, 1, 12345), 1024, 512, 1024, 2, False),   # (batch, channel, time) as torchaudio.load returns
    ((3, 7001), 400, 160, 400, 1, True),
    ((1, 4096), 512, 128, 300, 2, False),         # win_length < n_fft: window zero-padded, centred
    ((2, 1024), 1024, 512, 1024, 2, False),       # exactly one frame
])
def test_spectrogram_gpu_vs_oracle(shape, n_fft, hop, win, power, normalized):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from asrx.features import Spectrogram
    g = torch.Generator().manual_seed(sum(shape) + n_fft)
    x = torch.randn(*shape, generator=g) * 0.3
    spec = Spectrogram(n_fft=n_fft, win_length=win, hop_length=hop, power=power, normalized=normalized,
                       center=False)
    out = spec(x.cuda())
    ref = F.spectrogram(x.numpy(), n_fft=n_fft, win_length=win, hop_length=hop, power=power, normalized=normalized)
    assert tuple(out.shape) == ref.shape
    err = np.abs(out.cpu().double().numpy() - ref).max() / np.abs(ref).max()
    assert err < 2e-5, err


@pytest.mark.gpu
def test_spectrogram_feeds_the_model_frontend():
    """waveform -> GPU spectrogram -> model.input_layer: the (B, 1, F, T) layout of dataset.py:52 / model.py:168."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import asrx
    from asrx.features import Spectrogram
    spec = Spectrogram(n_fft=1024, center=False)
    wav = torch.randn(2, 1, 16000).cuda() * 0.1          # 1 s at 16 kHz: (16000 - 1024) // 512 + 1 = 30 frames
    s = spec(wav)
    assert s.shape == (2, 1, 513, 30)
    m = asrx.Transformer(250, 513, 128, 16, 30, 1, 1, 4, 512, dropout=0.0, precision="bf16").cuda().eval()
    text = torch.ones(2, 4, dtype=torch.int64).cuda()
    with torch.no_grad():
        out = m(torch.log1p(s), text, torch.ones(2, 4).cuda())
    assert out.shape == (2, 4, 250) and bool(torch.isfinite(out).all())
