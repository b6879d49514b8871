"""numpy restatement of the device dropout hash (test infrastructure; cfm_common.h cfm_mix32 / attn_mix / drop_key /
drop_bits).  Element idx of a call keyed by `seed` keeps iff the 16-bit half (idx & 1) of attn_mix(idx/2 + key) is
>= round(p * 65536)."""
import numpy as np

M = 0xFFFFFFFF


def mix32(x):
    """lowbias32 (cfm_mix32): derives the per-call key."""
    x = np.asarray(x).astype(np.uint64) & M
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= x >> 15
    x = (x * 0x846CA68B) & M
    x ^= x >> 16
    return x


def attn_mix(x):
    """the element hash: two rounds x += lo24(x) * C (C even) -- a bijection of the 32-bit word."""
    x = np.asarray(x).astype(np.uint64) & M
    x ^= x >> 16
    x = (x + (x & 0xFFFFFF) * 0x9E3778) & M
    x ^= x >> 15
    x = (x + (x & 0xFFFFFF) * 0x85EBCA) & M
    x ^= x >> 16
    return x


def drop_key(seed, jhi=0):
    inner = int(mix32(np.array([((seed >> 32) + 0x9E3779B9) & M]))[0])
    return int(mix32(np.array([(jhi ^ (seed & M) ^ inner) & M]))[0])


def drop_thr(p):
    return int(np.float32(p) * np.float32(65536.0) + np.float32(0.5))


def keep_bits(idx, key):
    """16 uniform bits of element idx (idx < 2^33, where drop_key's high word is 0)."""
    idx = np.asarray(idx).astype(np.uint64)
    h = attn_mix(((idx >> 1) + np.uint64(key)) & M)
    return np.where(idx & 1, h >> 16, h & 0xFFFF)
