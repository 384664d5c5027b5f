"""Row-slab decomposition helpers.

Image domains split into contiguous slabs of rows, one per rank — the reference's
CPU-MT outer-dimension split (API/src/backend_cpu_mt.t:716-737) applied across GPUs:
rank r owns rows [r*H/n, (r+1)*H/n) (last rank takes the remainder) and holds `halo`
extra rows of each neighbour.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict


@dataclass(frozen=True)
class Slab:
    rank: int
    world: int
    y_lo: int      # first owned row (global)
    y_hi: int      # one past the last owned row
    mem_lo: int    # first row held in memory (owned rows plus halo)
    mem_hi: int

    @property
    def rows(self) -> int:
        return self.y_hi - self.y_lo

    @property
    def mem_rows(self) -> int:
        return self.mem_hi - self.mem_lo


def slab(H: int, rank: int, world: int, halo: int) -> Slab:
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base = H // world
    y_lo = rank * base
    y_hi = H if rank == world - 1 else (rank + 1) * base
    if y_hi - y_lo < max(1, halo):
        raise ValueError(f"slab of {y_hi - y_lo} rows is thinner than the halo ({halo})")
    return Slab(rank, world, y_lo, y_hi, max(0, y_lo - halo), min(H, y_hi + halo))


def slice_rows(arr, W: int, channels: int, s: Slab):
    """Rows [s.mem_lo, s.mem_hi) of a flat row-major image with `channels` per pixel."""
    return arr[s.mem_lo * W * channels: s.mem_hi * W * channels]


IW_CHANNELS = (("Offset", 2), ("Angle", 1), ("UrShape", 2), ("Constraints", 2), ("Mask", 1))
SFS_CHANNELS = (("X", 1), ("D_i", 1), ("Im", 1), ("edgeMaskR", 1), ("edgeMaskC", 1))


def local_image(w: Dict, s: Slab, arrays) -> Dict:
    """The per-pixel arrays (name, channels) of one slab (memory rows incl. halo)."""
    W = w["W"]
    out = dict(w)
    for name, ch in arrays:
        out[name] = slice_rows(w[name], W, ch, s).copy()
    out["H"] = s.mem_rows
    return out


def local_image_warping(w: Dict, s: Slab) -> Dict:
    """The image_warping problem arrays of one slab (memory rows incl. halo)."""
    return local_image(w, s, IW_CHANNELS)


def owned(arr, W: int, channels: int, s: Slab):
    """The owned rows of a slab-local flat image array."""
    a = (s.y_lo - s.mem_lo) * W * channels
    return arr[a: a + s.rows * W * channels]


def owned_vec(vec, W: int, s: Slab):
    """Owned part of a slab-local unknown vector [Offset.xy | Angle] as two arrays."""
    N = W * s.mem_rows
    return owned(vec[: 2 * N], W, 2, s), owned(vec[2 * N:], W, 1, s)
