"""ORACLE (test infrastructure only) — counter-based normal noise stream.

The reference draws its sampler noise with ``torch.randn_like`` / ``torch.randn``
(model/diffusion.py:172,187,207,220,285,306; model/model.py:68,216).  Torch's
generator cannot be reproduced on the GPU nor sharded across ranks, so the
build defines the stream:

    z(seed, draw, e)  for global element index e = row * N + n

* Philox4x32-10 (Salmon et al., SC'11) with counter
  (lo32(e >> 2), hi32(e >> 2), draw, 0x5DD3) and key (lo32(seed), hi32(seed));
* the 4 output words give two Box–Muller pairs: lane e & 3 uses words
  (0,1) for lanes 0/1 and (2,3) for lanes 2/3;
* u = ((w >> 8) | 1) * 2**-24 (exact 24-bit odd fractions in (0,1)),
  r = sqrt(-2 ln u_a), z = r * cos(2 pi u_b) for even lanes, r * sin(2 pi u_b)
  for odd lanes.

Draw ids: 0 = x_T (get_x_T / randn_like at the start of infer), t = the noise
of ``p_transition*`` at step t (t > 1).  The HIP kernels compute exactly the
same Philox words (bit-exact integers) and the Box–Muller in fp32; the oracle
computes Box–Muller in float64 rounded to fp32 (differences are ~1 ulp).
"""
import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint64(0x9E3779B9)
_W1 = np.uint64(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)
TAG = 0x5DD3


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32 with 10 rounds. Inputs: uint64 arrays holding 32-bit values."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _MASK for c in (c0, c1, c2, c3))
    k0 = np.uint64(int(k0) & 0xFFFFFFFF)
    k1 = np.uint64(int(k1) & 0xFFFFFFFF)
    s32 = np.uint64(32)
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> s32, p0 & _MASK
        hi1, lo1 = p1 >> s32, p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK, lo1, (hi0 ^ c3 ^ k1) & _MASK, lo0
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return c0, c1, c2, c3


def _unit(w):
    return (((w >> np.uint64(8)) | np.uint64(1)).astype(np.float64)) * (2.0 ** -24)


def normal_from_index(seed, draw, e):
    """Standard normals (float32) for global element indices ``e`` (int array)."""
    e = np.asarray(e, dtype=np.uint64)
    q = e >> np.uint64(2)
    lane = (e & np.uint64(3)).astype(np.int64)
    w0, w1, w2, w3 = philox4x32_10(q & _MASK, q >> np.uint64(32),
                                   np.full_like(q, np.uint64(int(draw) & 0xFFFFFFFF)),
                                   np.full_like(q, np.uint64(TAG)),
                                   int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)
    ua = np.where(lane < 2, _unit(w0), _unit(w2))
    ub = np.where(lane < 2, _unit(w1), _unit(w3))
    r = np.sqrt(-2.0 * np.log(ua))
    ang = 2.0 * np.pi * ub
    z = np.where((lane & 1) == 0, r * np.cos(ang), r * np.sin(ang))
    return z.astype(np.float32)


def normal(seed, draw, shape, row_offset=0):
    """Noise tensor of ``shape`` = (B, ..., N): element (b, ..., n) has global index
    (row_offset + b) * prod(shape[1:]) + flat_rest."""
    shape = tuple(int(s) for s in shape)
    per_row = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    e = np.arange(shape[0] * per_row, dtype=np.uint64) + np.uint64(row_offset * per_row)
    return normal_from_index(seed, draw, e).reshape(shape)


def uniform_from_index(seed, stream, e):
    """Uniform [0,1) floats (float64, 24-bit) from Philox word 0 — used by the
    deterministic test-weight generator (tests/_weights.py)."""
    e = np.asarray(e, dtype=np.uint64)
    w0, w1, w2, w3 = philox4x32_10(e & _MASK, e >> np.uint64(32),
                                   np.full_like(e, np.uint64(int(stream) & 0xFFFFFFFF)),
                                   np.full_like(e, np.uint64(0x7E57)),
                                   int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)
    return (w0 >> np.uint64(8)).astype(np.float64) * (2.0 ** -24)
