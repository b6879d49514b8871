"""Pin the log-mel oracle (oracle/logmel.py) on the CPU.

librosa (the reference's dependency, speechcommands.py:113) is not installed, so the oracle's restatement
of librosa's defaults is held to transformers.audio_utils -- an independent implementation documented to
reproduce librosa's Slaney filter bank and power spectrogram -- and the product's host tables
(melspec.py: filter bank, filter runs, window) are held to the oracle.  No GPU needed."""
import numpy as np
import pytest

from oracle import logmel as olm

ta = pytest.importorskip("transformers.audio_utils")

CASES = [(16000, 2048, 40), (16000, 512, 80), (22050, 2048, 128), (8000, 256, 20)]


@pytest.mark.parametrize("sr,n_fft,n_mels", CASES)
def test_mel_bank_matches_transformers(sr, n_fft, n_mels):
    ref = ta.mel_filter_bank(num_frequency_bins=1 + n_fft // 2, num_mel_filters=n_mels, min_frequency=0.0,
                             max_frequency=sr / 2.0, sampling_rate=sr, norm="slaney", mel_scale="slaney")
    ours = olm.mel_bank(sr, n_fft, n_mels)
    assert ours.dtype == np.float32 and ours.shape == (n_mels, 1 + n_fft // 2)
    np.testing.assert_allclose(ours, ref.T, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("sr,n_fft,hop,n_mels,L", [(16000, 2048, 512, 40, 16000), (16000, 512, 160, 80, 7001),
                                                   (8000, 256, 100, 20, 999)])
def test_power_and_mel_match_transformers(sr, n_fft, hop, n_mels, L):
    rng = np.random.default_rng(L)
    y = (0.1 * rng.standard_normal(L) + 0.3 * np.sin(2 * np.pi * 440 * np.arange(L) / sr)).astype(np.float32)
    win = ta.window_function(n_fft, "hann", periodic=True)
    ref_pow = ta.spectrogram(y, win, frame_length=n_fft, hop_length=hop, power=2.0, center=True,
                             pad_mode="constant", dtype=np.float64)
    ours = olm.power_spectrogram(y, n_fft, hop)
    assert ours.shape == ref_pow.shape == (1 + n_fft // 2, 1 + L // hop)
    scale = ref_pow.max()
    np.testing.assert_allclose(ours, ref_pow, rtol=1e-4, atol=1e-6 * scale)
    bank = ta.mel_filter_bank(1 + n_fft // 2, n_mels, 0.0, sr / 2.0, sr, norm="slaney", mel_scale="slaney")
    ref_mel = ta.spectrogram(y, win, frame_length=n_fft, hop_length=hop, power=2.0, center=True,
                             pad_mode="constant", mel_filters=bank, mel_floor=0.0, dtype=np.float64)
    mel = olm.mel_bank(sr, n_fft, n_mels) @ ours
    np.testing.assert_allclose(mel, ref_mel, rtol=1e-4, atol=1e-6 * ref_mel.max())


def test_log_floor_and_minmax_semantics():
    """np.where(mel < 1e-10, 0, log(mel)) then per-clip min-max (speechcommands.py:114-119): a silent
    stretch yields log-power 0 (not -inf), and the output spans exactly [0, 1]."""
    sr = 16000
    y = np.zeros(8000, np.float32)
    y[4000:] = 0.2 * np.random.default_rng(0).standard_normal(4000).astype(np.float32)
    m = olm.log_mel(y, sr, 40)
    raw = olm.log_mel(y, sr, 40, normalize=False)
    assert np.isfinite(raw).all()
    assert (raw[:, 0] == 0).all()             # all-zero first frame: floored to 0, not log(0)
    assert m.min() == 0.0 and m.max() == 1.0


def test_product_host_tables_match_oracle():
    """melspec.py's host-side constant tables (built once per configuration) against the oracle."""
    from nn_conformer_for_speech_recognition_amd import melspec
    for sr, n_fft, n_mels in CASES:
        w = melspec.mel_filter_bank(sr, n_fft, n_mels)
        np.testing.assert_array_equal(w, olm.mel_bank(sr, n_fft, n_mels))
        lo, cnt, off, packed = melspec.filter_runs(w)
        dense = np.zeros_like(w)
        for m in range(n_mels):
            dense[m, lo[m]:lo[m] + cnt[m]] = packed[off[m]:off[m] + cnt[m]]
        np.testing.assert_array_equal(dense, w)
        np.testing.assert_allclose(melspec.hann_periodic(n_fft), 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft))


def test_logmel_rejects_bad_config():
    from nn_conformer_for_speech_recognition_amd import melspec
    with pytest.raises(ValueError):
        melspec.LogMel(16000, 40, n_fft=400)
    with pytest.raises(ValueError):
        melspec.LogMel(16000, 40, hop_length=0)
