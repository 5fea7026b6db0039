"""numpy restatement of the dropout RNG in asr-transformer_amd/csrc/common.h (test oracle only): one keyed
32-bit mix per pair of elements, 16-bit halves compared against round(p * 65536)."""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def threshold(p):
    if p <= 0:
        return 0
    if p >= 1:
        return 65536
    return int(p * 65536.0 + 0.5)


def rng_hash(seed, pidx):
    seed = int(seed) & ((1 << 64) - 1)
    x = (np.asarray(pidx, dtype=np.uint64) & M32) ^ np.uint64(seed & 0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B) + np.uint64(seed >> 32)) & M32
    x ^= x >> np.uint64(16)
    return x


def _half(h, which):
    return np.where(which, h >> np.uint64(16), h & np.uint64(0xFFFF))


def elem_keep(seed, n, p):
    """keep mask of the element streams (GEMM epilogue, LayerNorm backward, embedding, asrx_dropout_mask)"""
    idx = np.arange(n, dtype=np.uint64)
    return _half(rng_hash(seed, idx >> np.uint64(1)), (idx & np.uint64(1)).astype(bool)) >= threshold(p)


def attn_keep(seed, bh, lq, lk, p):
    """keep mask [bh, lq, lk] of the attention probabilities (pairs run along queries)"""
    b = np.arange(bh, dtype=np.uint64)[:, None, None]
    q = np.arange(lq, dtype=np.uint64)[None, :, None]
    k = np.arange(lk, dtype=np.uint64)[None, None, :]
    pidx = ((b * np.uint64((lq + 1) // 2) + (q >> np.uint64(1))) * np.uint64(lk) + k) & M32
    return _half(rng_hash(seed, pidx), np.broadcast_to((q & np.uint64(1)).astype(bool), pidx.shape)) >= threshold(p)
