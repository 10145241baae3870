"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Counter-based Philox4x32-10 in numpy, bit-identical to the device version in
`muzero-breakout_amd/csrc/rng.h`. The reference draws every random number from the
single global torch CPU generator (parallel_breakout.py:116,126,127,136,
mcts.py:114,297, train_torch.py:196-198); a GPU cannot replay that serial stream, so
parity is defined on injected randomness: both the oracle and the HIP kernels draw
from this keyed stream, and the golden fixtures are produced by running the
reference with its torch RNG calls replaced by draws from the same stream
(tests/golden/make_golden.py).

Counter layout (c0, c1, c2, c3) = (global env id, stream, step, call):
  stream 0 RESET   : step = reset/episode index, call = kind (0 paddle off, 1 ball col,
                     2 ball row, 3 dx)
  stream 1 TIE     : step = search index, call = per-env ucb_action call counter
  stream 2 NOISE   : step = search index, call = gamma-sampler draw counter
  stream 3 SAMPLE  : step = acting-step index, call = 0
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_RESET = 0
STREAM_TIE = 1
STREAM_NOISE = 2
STREAM_SAMPLE = 3


def philox4x32(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10. Inputs broadcast; returns 4 uint32 arrays."""
    c0, c1, c2, c3 = np.broadcast_arrays(*(np.asarray(x, dtype=np.uint64) & MASK32 for x in (c0, c1, c2, c3)))
    c0 = c0.copy(); c1 = c1.copy(); c2 = c2.copy(); c3 = c3.copy()
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64(seed >> 32)
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(W0)) & MASK32
            k1 = (k1 + np.uint64(W1)) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32), c3.astype(np.uint32))


def u32(env, stream, step, call, seed):
    return philox4x32(env, stream, step, call, seed)[0]


def uniform(env, stream, step, call, seed):
    """f32 uniform in [0,1): (x >> 8) * 2^-24 (exact in f32)."""
    x = u32(env, stream, step, call, seed)
    return ((x >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)


def randbelow(env, stream, step, call, seed, n):
    """Integer in [0, n): ((x >> 8) * n) >> 24, exact integer arithmetic (n < 2^32)."""
    x = u32(env, stream, step, call, seed).astype(np.uint64)
    n = np.asarray(n, dtype=np.uint64)
    return (((x >> np.uint64(8)) * n) >> np.uint64(24)).astype(np.int64)
