"""Philox4x32-10 streams of the engine (include/mz_detmath.h), pure Python: the
host mirrors (replay_buffer.py, selfplay.py) draw from the same streams as the
kernels, keyed (seed, purpose, id, step, index) — Julia's global RNG (quirk Q6)
made reproducible."""
_M = 0xFFFFFFFF


def _philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (include/mz_detmath.h mz_philox), pure Python."""
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        hi0, lo0 = (p0 >> 32) & _M, p0 & _M
        hi1, lo1 = (p1 >> 32) & _M, p1 & _M
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + 0x9E3779B9) & _M
        k1 = (k1 + 0xBB67AE85) & _M
    return c0, c1, c2, c3


def rng_u32(seed, purpose, ident, step, idx):
    return _philox(idx & _M, ident & _M, step & _M, purpose, seed & _M, (seed >> 32) & _M)[0]


def rng_below(r, n):
    return (r * n) >> 32


def philox_np(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 over numpy arrays (broadcast), the same rounds as _philox;
    returns four uint32 arrays."""
    import numpy as np
    m = np.uint64(_M)
    c0, c1, c2, c3 = (np.asarray(c, np.uint64) & m for c in (c0, c1, c2, c3))
    k0, k1 = np.asarray(k0, np.uint64) & m, np.asarray(k1, np.uint64) & m
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & m, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & m
        k0 = (k0 + np.uint64(0x9E3779B9)) & m
        k1 = (k1 + np.uint64(0xBB67AE85)) & m
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))
