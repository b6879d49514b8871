"""Statistical check of the attention-dropout element hash (cfm_common.h attn_mix: two 24-bit multiplies) over
the index pattern the attention kernels use, ((b H + h) T + i) T2 + j/2 (+ the key) with 16 bits per element: keep rate,
and the correlation of keep decisions at key lags 1..8, query lags 1..8 and both diagonals, next to lowbias32
(cfm_mix32, the hash of every other dropout) as the reference quality.  numpy only (CPU)."""
import numpy as np
import pytest

M = 0xFFFFFFFF


def _lowbias32(x):
    x = x & M
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= x >> 15
    x = (x * 0x846CA68B) & M
    x ^= x >> 16
    return x


def _attn_mix(x):
    x = x & M
    x ^= x >> 16
    x = ((x & 0xFFFFFF) * 0x9E3779) & M
    x ^= x >> 15
    x = ((x & 0xFFFFFF) * 0x85EBCA) & M
    x ^= x >> 16
    return x


def _keep(f, nbh, T, key, p=0.1):
    T2 = (T + 1) // 2
    thr = int(p * 65536 + 0.5)
    bh = np.arange(nbh, dtype=np.uint64)[:, None, None]
    i = np.arange(T, dtype=np.uint64)[None, :, None]
    jp = np.arange(T2, dtype=np.uint64)[None, None, :]
    h = f(((bh * T + i) * T2 + jp + np.uint64(key)) & M) if f is _attn_mix else f(((bh * T + i) * T2 + jp) ^ np.uint64(key))
    k = np.stack([(h & 0xFFFF) >= thr, (h >> 16) >= thr], -1).reshape(nbh, T, 2 * T2)[:, :, :T]
    return k.astype(np.float64)


def _corr(a, b):
    a = a - a.mean()
    b = b - b.mean()
    return float((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean()))


def _worst_corr(k):
    w = 0.0
    for lag in range(1, 9):
        w = max(w, abs(_corr(k[:, :, :-lag], k[:, :, lag:])), abs(_corr(k[:, :-lag, :], k[:, lag:, :])))
    w = max(w, abs(_corr(k[:, :-1, :-1], k[:, 1:, 1:])), abs(_corr(k[:, :-1, 1:], k[:, 1:, :-1])))
    return w


@pytest.mark.parametrize("T,nbh", [(373, 16), (1498, 4)])
def test_attn_mix_keep_statistics(T, nbh):
    rng = np.random.default_rng(T)
    for key in rng.integers(0, 2 ** 32, 2, dtype=np.uint64):
        k = _keep(_attn_mix, nbh, T, int(key))
        ref = _keep(_lowbias32, nbh, T, int(key))
        n = k.size
        assert abs(k.mean() - 0.9) < 4 * np.sqrt(0.09 / n)           # keep rate 1 - p within 4 sigma
        noise = 5.0 / np.sqrt(n)
        assert _worst_corr(k) < max(noise, 1.5 * _worst_corr(ref))  # no structure beyond lowbias32's / noise
        rows = k.mean(axis=2)                                         # per-query keep rates ~ binomial
        assert rows.std() < 1.25 * np.sqrt(0.09 / T)
