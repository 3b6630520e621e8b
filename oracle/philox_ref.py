"""Oracle: numpy restatement of the counter-based epsilon generator (TEST INFRASTRUCTURE ONLY).

The reference draws epsilons with torch's global generator (``eps.normal_()`` inside
bayesian-torch's forward), which cannot be reproduced on the GPU; the
product instead uses Philox4x32-10 (Salmon et al., SC'11) + Box-Muller keyed by
(seed, MC sample, layer, element quad) so the backward pass can regenerate them.  This
module restates that generator so the GPU integer stream is checked bit-exactly and the
normal transform to fp32 rounding.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(q, sample, layer, seed):
    """q: uint64 array of quad indices -> uint32 array [len(q), 4]."""
    q = np.asarray(q, dtype=np.uint64)
    c0 = q & MASK
    c1 = np.full_like(q, np.uint64(sample) & MASK)
    c2 = np.full_like(q, np.uint64(layer) & MASK)
    c3 = np.full_like(q, (np.uint64(sample) >> np.uint64(32)) & MASK)
    k0 = np.uint64(seed) & MASK
    k1 = (np.uint64(seed) >> np.uint64(32)) & MASK
    for _ in range(10):
        p0 = c0 * M0
        p1 = c2 * M1
        lo0, hi0 = p0 & MASK, p0 >> np.uint64(32)
        lo1, hi1 = p1 & MASK, p1 >> np.uint64(32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return np.stack([c0, c1, c2, c3], axis=1).astype(np.uint32)


def normal4(raw):
    """Box-Muller on Philox words exactly as mauv_common.h::normal4 (in float64)."""
    u = (raw.astype(np.float64) + 0.5) * 2.0 ** -32
    m0 = np.sqrt(-2.0 * np.log(u[:, 0]))
    m1 = np.sqrt(-2.0 * np.log(u[:, 2]))
    return np.stack([m0 * np.cos(2 * np.pi * u[:, 1]), m0 * np.sin(2 * np.pi * u[:, 1]),
                     m1 * np.cos(2 * np.pi * u[:, 3]), m1 * np.sin(2 * np.pi * u[:, 3])], axis=1)


def eps_for_layer(numel, seed, sample, layer):
    """The epsilon tensor (parameter order) the GPU draws for one layer / MC sample."""
    nq = (numel + 3) // 4
    return normal4(philox4x32_10(np.arange(nq, dtype=np.uint64), sample, layer, seed)).reshape(-1)[:numel]
