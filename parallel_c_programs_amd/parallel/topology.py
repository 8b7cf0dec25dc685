"""Cartesian process topology for 2-D domain decomposition.

Reference: MPI_Dims_create / MPI_Cart_create(periods={0,0}, reorder=0) / MPI_Cart_coords / MPI_Cart_shift /
MPI_Cart_rank in 2-mpi-region-growing/region.c:537-548 (+ :113, :413, :470). Pure functions here, so every
rank derives the same layout without communication.

Deviation (B8): the reference mixes local_image_size[0]/[1] with x/y, so only square process grids
(1, 4, 16, ...) decompose correctly; here rows split over dims[0] and columns over dims[1] with the
remainder spread over the first blocks, so any world size (1/2/4/8 on one MI355X node) tiles any image.
"""
from __future__ import annotations

from dataclasses import dataclass


def prime_factors(n: int) -> list[int]:
    f, p = [], 2
    while p * p <= n:
        while n % p == 0:
            f.append(p)
            n //= p
        p += 1
    if n > 1:
        f.append(n)
    return f


def dims_create(nnodes: int, ndims: int = 2) -> list[int]:
    """Balanced factorisation in non-increasing order (MPI_Dims_create semantics): 1->[1,1], 2->[2,1],
    4->[2,2], 8->[4,2], 12->[4,3]."""
    if nnodes < 1:
        raise ValueError("nnodes must be >= 1")
    dims = [1] * ndims
    for p in sorted(prime_factors(nnodes), reverse=True):
        i = dims.index(min(dims))
        dims[i] *= p
    return sorted(dims, reverse=True)


def split(n: int, parts: int, i: int) -> tuple[int, int]:
    """[start, stop) of block i when n items are split into `parts` near-equal blocks."""
    q, r = divmod(n, parts)
    start = i * q + min(i, r)
    return start, start + q + (1 if i < r else 0)


@dataclass(frozen=True)
class CartTopology:
    size: int
    dims: tuple[int, int]

    @staticmethod
    def create(size: int, dims: tuple[int, int] | None = None) -> "CartTopology":
        d = tuple(dims) if dims is not None else tuple(dims_create(size, 2))
        if d[0] * d[1] != size:
            raise ValueError(f"dims {d} do not multiply to {size}")
        return CartTopology(size, d)

    def coords(self, rank: int) -> tuple[int, int]:
        """Row-major rank -> (row, col) like MPI_Cart_coords with reorder=0."""
        return divmod(rank, self.dims[1])

    def rank_of(self, row: int, col: int) -> int:
        """MPI_Cart_rank for a non-periodic grid; -1 outside."""
        if 0 <= row < self.dims[0] and 0 <= col < self.dims[1]:
            return row * self.dims[1] + col
        return -1

    def shift(self, rank: int, dim: int, disp: int = 1) -> tuple[int, int]:
        """MPI_Cart_shift: (source, dest) neighbours along dim (-1 = MPI_PROC_NULL)."""
        r, c = self.coords(rank)
        if dim == 0:
            return self.rank_of(r - disp, c), self.rank_of(r + disp, c)
        return self.rank_of(r, c - disp), self.rank_of(r, c + disp)

    def neighbours(self, rank: int) -> dict[str, int]:
        north, south = self.shift(rank, 0)
        west, east = self.shift(rank, 1)
        return {"north": north, "south": south, "west": west, "east": east}

    def tile(self, rank: int, height: int, width: int) -> tuple[int, int, int, int]:
        """(row0, row1, col0, col1) of this rank's block of a height x width image."""
        r, c = self.coords(rank)
        r0, r1 = split(height, self.dims[0], r)
        c0, c1 = split(width, self.dims[1], c)
        return r0, r1, c0, c1

    def owner(self, y: int, x: int, height: int, width: int) -> int:
        """Rank owning global pixel (y, x)."""
        for rank in range(self.size):
            r0, r1, c0, c1 = self.tile(rank, height, width)
            if r0 <= y < r1 and c0 <= x < c1:
                return rank
        return -1
