"""On-device log-mel front-end: the data step before SpecAugment.

Reference: lib/standard/speechcommands.py:113-119 computes, per clip on the CPU,
    mel = librosa.feature.melspectrogram(y=wave, sr=sr, n_mels=hp.n_mels)
    mel = np.where(mel < 1e-10, 0, np.log(mel))
    mel -= np.min(mel); mel /= np.max(mel)
and the collate zero-pads shorter clips (speechcommands.py:188,198-210).  librosa's defaults:
n_fft 2048, hop 512, periodic Hann window, center=True with zero padding, power 2, Slaney mel
scale and Slaney area normalisation, fmin 0, fmax sr/2.

Here the whole batch is one `cfm_logmel_fwd` call (logmel.hip): per (frame, utterance) workgroup
an LDS radix-2 FFT, |X|^2, the sparse Slaney filters, log; then a per-utterance min-max pass.
The host only builds the constant tables (window, twiddles, filter runs) once per configuration,
the way librosa builds its filter bank (librosa.filters.mel).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib as L

_F_SP = 200.0 / 3.0
_MIN_LOG_HZ = 1000.0
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = math.log(6.4) / 27.0


def hz_to_mel(f):
    """Slaney mel scale (librosa.hz_to_mel, htk=False): linear below 1 kHz, logarithmic above."""
    f = np.asarray(f, dtype=np.float64)
    lin = f / _F_SP
    with np.errstate(divide="ignore"):
        log = _MIN_LOG_MEL + np.log(np.maximum(f, 1e-300) / _MIN_LOG_HZ) / _LOGSTEP
    return np.where(f >= _MIN_LOG_HZ, log, lin)


def mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    return np.where(m >= _MIN_LOG_MEL, _MIN_LOG_HZ * np.exp(_LOGSTEP * (m - _MIN_LOG_MEL)), _F_SP * m)


def mel_filter_bank(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """(n_mels, 1 + n_fft // 2) float32 Slaney-normalised triangular filters (librosa.filters.mel
    defaults): triangles between n_mels + 2 points equally spaced on the Slaney mel scale, each
    scaled by 2 / (its Hz width).  Triangles are evaluated in float64 and stored float32 before the
    (float64) normalisation factor is applied, as librosa does."""
    if fmax is None:
        fmax = sr / 2.0
    fftfreqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, len(fftfreqs)), dtype=np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return w


def filter_runs(w):
    """Compress each filter to its contiguous run of non-zero bins: (lo, cnt, off, packed weights)."""
    lo, cnt, off, packed = [], [], [], []
    pos = 0
    for row in w:
        nz = np.nonzero(row)[0]
        if len(nz) == 0:
            lo.append(0)
            cnt.append(0)
        else:
            a, b = int(nz[0]), int(nz[-1]) + 1
            lo.append(a)
            cnt.append(b - a)
            packed.append(row[a:b])
        off.append(pos)
        pos += cnt[-1]
    packed = np.concatenate(packed).astype(np.float32) if packed else np.zeros(1, np.float32)
    return (np.asarray(lo, np.int32), np.asarray(cnt, np.int32), np.asarray(off, np.int32), packed)


def hann_periodic(n):
    """scipy.signal.get_window('hann', n, fftbins=True)."""
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / n)


class LogMel:
    """Batch log-mel front-end on the GPU with librosa.feature.melspectrogram semantics.

    LogMel(sr, n_mels, n_fft=2048, hop_length=512)(wave (B, L) fp32 cuda, lengths (B,) samples)
      -> (mels (B, n_mels, 1 + L // hop) fp32, frames (B,) int32 = 1 + lengths // hop)
    normalize=True applies the reference's log floor + per-utterance min-max (speechcommands.py:114-119);
    normalize=False returns the floored log-mels.  Padded frames are 0 either way."""

    def __init__(self, sr=22050, n_mels=128, n_fft=2048, hop_length=512, fmin=0.0, fmax=None):
        if n_fft < 16 or n_fft > 4096 or n_fft & (n_fft - 1):
            raise ValueError("n_fft must be a power of two in [16, 4096] on the MI355X path")
        if hop_length <= 0:
            raise ValueError("hop_length must be positive")
        self.sr, self.n_mels, self.n_fft, self.hop = sr, n_mels, n_fft, hop_length
        self.weights = mel_filter_bank(sr, n_fft, n_mels, fmin, fmax)
        k = np.arange(n_fft // 2)
        tw = np.exp(-2j * np.pi * k / n_fft)
        self._host = {
            "window": hann_periodic(n_fft).astype(np.float32),
            "twiddle": np.stack([tw.real, tw.imag], 1).astype(np.float32).reshape(-1),
        }
        self._host["lo"], self._host["cnt"], self._host["off"], self._host["w"] = filter_runs(self.weights)
        self._dev = {}

    def _tables(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = {n: torch.from_numpy(a.copy()).to(device) for n, a in self._host.items()}
        return self._dev[key]

    def frames(self, lengths):
        return 1 + lengths // self.hop

    def __call__(self, wave, lengths=None, normalize=True):
        if wave.dim() != 2:
            raise ValueError(f"expected wave (B, L), got {tuple(wave.shape)}")
        if not wave.is_cuda:
            raise L.CfmError("LogMel runs on libcfm HIP kernels: move the waveforms to the GPU")
        wave = wave.float().contiguous()
        B, Lm = wave.shape
        if lengths is None:
            lengths = torch.full((B,), Lm, dtype=torch.int32, device=wave.device)
        lens = lengths.to(device=wave.device, dtype=torch.int32).contiguous()
        nT = 1 + Lm // self.hop
        tb = self._tables(wave.device)
        out = torch.empty(B, self.n_mels, nT, device=wave.device, dtype=torch.float32)
        ws = torch.empty(max(1, L.size_call("cfm_logmel_ws_bytes", B, nT) // 4), device=wave.device,
                         dtype=torch.float32)
        L.call("cfm_logmel_fwd", L.ptr(wave), Lm, L.ptr(lens), B, self.n_fft, self.hop, L.ptr(tb["window"]),
               L.ptr(tb["twiddle"]), L.ptr(tb["lo"]), L.ptr(tb["cnt"]), L.ptr(tb["off"]), L.ptr(tb["w"]),
               self.n_mels, nT, int(bool(normalize)), L.ptr(out), L.ptr(ws), L.stream())
        return out, self.frames(lens)


def melspectrogram_log_norm(wave, sr, n_mels, lengths=None, **kw):
    """speechcommands.py:113-119 for a batch: LogMel(sr, n_mels, **kw)(wave, lengths)."""
    return LogMel(sr=sr, n_mels=n_mels, **kw)(wave, lengths)
