"""Oracle: log-mel front-end (TEST INFRASTRUCTURE ONLY), numpy on the CPU.

Restates /root/reference/lib/standard/speechcommands.py:113-119 for one clip:
    mel = librosa.feature.melspectrogram(y=y, sr=sr, n_mels=n_mels)
    mel = np.where(mel < 1e-10, 0, np.log(mel))
    mel -= np.min(mel); mel /= np.max(mel)
librosa is a third-party dependency (requirements.txt:4, unpinned) and is not installed here; its
published 0.10 defaults are restated: periodic Hann window (scipy get_window 'hann', fftbins=True),
center=True with pad_mode='constant' (n_fft // 2 zeros each side), frames = 1 + len // hop, rfft of
the float64 windowed frame stored complex64, |.|**2 in float32, Slaney mel bank
(librosa.filters.mel: htk=False, norm='slaney', float32) @ power in float32.
Pinned against transformers.audio_utils (mel_filter_bank(norm='slaney', mel_scale='slaney') and
spectrogram(..., pad_mode='constant', power=2.0)), an independent implementation documented to match
librosa (tests/test_logmel_oracle.py); librosa itself is "parity unpinned" here.
"""
from __future__ import annotations

import numpy as np


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    out = np.array(mels, dtype=np.float64)
    sel = f >= min_log_hz
    out[sel] = min_log_mel + np.log(f[sel] / min_log_hz) / logstep
    return out


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    sel = m >= min_log_mel
    freqs[sel] = min_log_hz * np.exp(logstep * (m[sel] - min_log_mel))
    return freqs


def mel_bank(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr=sr, n_fft=n_fft, n_mels=n_mels) -> (n_mels, 1 + n_fft // 2) float32."""
    fmax = sr / 2.0 if fmax is None else fmax
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(np.array([fmin]))[0], _hz_to_mel(np.array([fmax]))[0], n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def power_spectrogram(y, n_fft=2048, hop=512):
    """|stft(y)|**2 with librosa's defaults -> (1 + n_fft // 2, 1 + len(y) // hop) float32."""
    y = np.asarray(y, dtype=np.float32)
    n = np.arange(n_fft)
    window = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / n_fft)             # float64, periodic
    yp = np.pad(y, (n_fft // 2, n_fft // 2), mode="constant")
    n_frames = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = yp[idx] * window[None, :]                               # float32 x float64 -> float64
    spec = np.fft.rfft(frames, axis=-1).astype(np.complex64).T       # stored complex64
    return (np.abs(spec) ** 2).astype(np.float32)


def log_mel(y, sr, n_mels, n_fft=2048, hop=512, normalize=True):
    """speechcommands.py:113-119 for one clip -> (n_mels, 1 + len(y) // hop) float32."""
    mel = mel_bank(sr, n_fft, n_mels) @ power_spectrogram(y, n_fft, hop)
    mel = np.where(mel < 1e-10, 0, np.log(mel)).astype(np.float32)
    if normalize:
        mel = np.array(mel)
        mel -= np.min(mel)
        mel /= np.max(mel)
    return mel


def log_mel_batch(waves, lengths, sr, n_mels, n_fft=2048, hop=512, normalize=True):
    """Per-clip log_mel of waves[b, :lengths[b]], zero-padded to 1 + max_len // hop frames
    (the collate's padding, speechcommands.py:188,198-210)."""
    Lm = waves.shape[1]
    nT = 1 + Lm // hop
    out = np.zeros((waves.shape[0], n_mels, nT), dtype=np.float32)
    for b in range(waves.shape[0]):
        m = log_mel(waves[b, :int(lengths[b])], sr, n_mels, n_fft, hop, normalize)
        out[b, :, :m.shape[1]] = m
    return out
