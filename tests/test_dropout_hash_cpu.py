"""Checks of the dropout element hash (cfm_common.h attn_mix: two 24-bit multiply-adds), which every dropout of the
library uses (attention probabilities, GEMM epilogues, scale_dropout, the LayerNorm backward's g2; lowbias32 =
cfm_mix32 only derives the per-call key):
* it is one-to-one on 32 bits (2^25 consecutive pair indices under a random key all hash apart; x and
  x ^ (d * 0x01000100), the collision class of round 4's form, never collide);
* keep rate and keep-decision correlations at lags 1..8 along both axes and both diagonals, next to lowbias32 as
  the reference quality, over the attention index pattern ((b H + h) T + i) T2 + j/2 (+ key) and over the GEMM
  epilogue layout doff + (z M + m) N + n at the L15 FFN-up size (M 11,936, N 2048).  numpy only (CPU)."""
import numpy as np
import pytest

from tests.dropout_hash import M, attn_mix, mix32


def _lowbias32_keyed(x, key):
    return mix32((x ^ np.uint64(key)) & M)


def _attn_keyed(x, key):
    return attn_mix((x + np.uint64(key)) & M)


def _halves(h, thr):
    return np.stack([(h & 0xFFFF) >= thr, (h >> 16) >= thr], -1)


def _keep_attn(f, nbh, T, key, p=0.1):
    T2 = (T + 1) // 2
    thr = int(p * 65536 + 0.5)
    bh = np.arange(nbh, dtype=np.uint64)[:, None, None]
    i = np.arange(T, dtype=np.uint64)[None, :, None]
    jp = np.arange(T2, dtype=np.uint64)[None, None, :]
    h = f((bh * T + i) * T2 + jp, key)
    return _halves(h, thr).reshape(nbh, T, 2 * T2)[:, :, :T].astype(np.float32)


def _keep_gemm(f, Mrows, N, doff, key, p=0.1):
    """the GEMM epilogue's keep mask of an (Mrows, N) output: element e = doff + m N + n, pair e / 2 (N even, doff
    even, so each pair is two neighbouring columns of one row)."""
    thr = int(p * 65536 + 0.5)
    m = np.arange(Mrows, dtype=np.uint64)[:, None]
    jp = np.arange(N // 2, dtype=np.uint64)[None, :]
    h = f((doff // 2 + m * (N // 2) + jp) & M, key)
    return _halves(h, thr).reshape(1, Mrows, N).astype(np.float32)


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


def _check(k, ref, row_len):
    n = k.size
    assert abs(k.mean() - 0.9) < 4 * np.sqrt(0.09 / n)           # keep rate 1 - p within 4 sigma
    noise = 5.0 / np.sqrt(n)
    assert _worst_corr(k) < max(noise, 1.5 * _worst_corr(ref))  # no structure beyond lowbias32's / noise
    rows = k.mean(axis=2)                                         # per-row keep rates ~ binomial
    assert rows.std() < 1.25 * np.sqrt(0.09 / row_len)


@pytest.mark.parametrize("T,nbh", [(373, 16), (1498, 4)])
def test_attn_mix_keep_statistics(T, nbh):
    rng = np.random.default_rng(T)
    for key in rng.integers(0, 2 ** 32, 2, dtype=np.uint64):
        _check(_keep_attn(_attn_keyed, nbh, T, key), _keep_attn(_lowbias32_keyed, nbh, T, key), T)


def test_gemm_epilogue_keep_statistics():
    """the FFN-up epilogue's dropout at L15 (M 11,936 rows, N 2048): 24.4 M elements, 12.2 M pairs."""
    rng = np.random.default_rng(2048)
    key = rng.integers(0, 2 ** 32, dtype=np.uint64)
    doff = 2 * int(rng.integers(0, 2 ** 20))
    _check(_keep_gemm(_attn_keyed, 11936, 2048, doff, key), _keep_gemm(_lowbias32_keyed, 11936, 2048, doff, key), 2048)


def test_attn_mix_is_one_to_one():
    rng = np.random.default_rng(5)
    key = np.uint64(rng.integers(0, 2 ** 32, dtype=np.uint64))
    h = attn_mix((np.arange(1 << 25, dtype=np.uint64) + key) & M).astype(np.uint32)
    assert np.unique(h).size == h.size                           # 2^25 pair indices, all distinct
    x = rng.integers(0, 2 ** 32, 1 << 16, dtype=np.uint64)
    hx = attn_mix(x)
    for d in range(1, 256):                                      # round 4's collision class
        assert not np.any(attn_mix(x ^ np.uint64(d * 0x01000100)) == hx)
    # each round x + lo24(x) * C is a bijection: 2^16 random lo24 values under all 256 high bytes stay distinct
    lo = rng.integers(0, 1 << 24, 1 << 16, dtype=np.uint64)
    lo = np.unique(lo)[:, None]
    w = lo + (np.arange(256, dtype=np.uint64)[None, :] << np.uint64(24))
    for C in (0x9E3778, 0x85EBCA):
        r = (w + (w & 0xFFFFFF) * C) & M
        assert np.unique(r.astype(np.uint32)).size == r.size
