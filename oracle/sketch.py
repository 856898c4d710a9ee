"""numpy restatement of the count-min / HyperLogLog sketch updates (TEST INFRASTRUCTURE ONLY).

The sketches are new (no reference code); this restates DESIGN.md
section 6 independently of the product so the device state can be checked bit for bit.
"""

from __future__ import annotations

import numpy as np

U64 = np.uint64
M1, M2 = U64(0xff51afd7ed558ccd), U64(0xc4ceb9fe1a85ec53)
CMS_SEED, HLL_SEED = U64(0x5EED5EED5EED5EED), U64(0xA5A5A5A5DEADBEEF)


def fmix64(k: np.ndarray) -> np.ndarray:
    k = k.astype(U64, copy=True)
    with np.errstate(over="ignore"):
        k ^= k >> U64(33)
        k *= M1
        k ^= k >> U64(33)
        k *= M2
        k ^= k >> U64(33)
    return k


def cms_cols(base: np.ndarray, r: int, width: int) -> np.ndarray:
    """Row r's column: h1 + r*h2 (double hashing of the 64-bit base; h2 odd)."""
    h1 = base & U64(0xFFFFFFFF)
    h2 = (base >> U64(32)) | U64(1)
    with np.errstate(over="ignore"):
        return ((h1 + U64(r) * h2) & U64(width - 1)).astype(np.int64)


def cms_update(cms: np.ndarray, src, dst, ports, proto) -> None:
    """cms: uint32 [depth, width]; one +1 per record per row."""
    depth, width = cms.shape
    lo = src.astype(U64) | (dst.astype(U64) << U64(32))
    hi = ports.astype(U64) | (proto.astype(U64) << U64(32))
    base = fmix64(lo ^ fmix64(hi ^ CMS_SEED))
    for r in range(depth):
        cms[r] += np.bincount(cms_cols(base, r, width), minlength=width).astype(np.uint32)


def _bitlen64(w: np.ndarray) -> np.ndarray:
    hi = (w >> U64(32)).astype(np.float64)
    lo = (w & U64(0xFFFFFFFF)).astype(np.float64)
    bl_hi = np.frexp(hi)[1]
    bl_lo = np.frexp(lo)[1]
    return np.where(hi > 0, 32 + bl_hi, bl_lo)


def hll_update(regs: np.ndarray, slot: np.ndarray, dst: np.ndarray, p: int) -> None:
    """regs: uint8 [slots, 2^p]; rows with slot < 0 are skipped."""
    keep = slot >= 0
    slot, dst = slot[keep], dst[keep]
    h = fmix64(dst.astype(U64) ^ HLL_SEED)
    idx = (h >> U64(64 - p)).astype(np.int64)
    w = (h << U64(p)) | U64(1 << (p - 1))
    rho = (64 - _bitlen64(w) + 1).astype(np.uint8)
    np.maximum.at(regs, (slot.astype(np.int64), idx), rho)


def hll_estimate(reg: np.ndarray) -> float:
    m = reg.size
    alpha = 0.7213 / (1.0 + 1.079 / m)
    e = alpha * m * m / np.sum(np.ldexp(1.0, -reg.astype(np.int64)))
    zeros = int(np.sum(reg == 0))
    if e <= 2.5 * m and zeros:
        e = m * np.log(m / zeros)
    return float(e)


def cms_estimate(cms: np.ndarray, src, dst, ports, proto) -> np.ndarray:
    """Count-min point queries (min over rows) for arrays of 5-tuples."""
    depth, width = cms.shape
    lo = np.asarray(src).astype(U64) | (np.asarray(dst).astype(U64) << U64(32))
    hi = np.asarray(ports).astype(U64) | (np.asarray(proto).astype(U64) << U64(32))
    base = fmix64(lo ^ fmix64(hi ^ CMS_SEED))
    est = None
    for r in range(depth):
        v = cms[r, cms_cols(base, r, width)].astype(np.int64)
        est = v if est is None else np.minimum(est, v)
    return est
