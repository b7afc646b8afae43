"""Box decomposition of a level over ranks (one box per GPU).

The reference splits the domain into boxes of at most max_grid_size in
multiples of block_factor and load-balances them over MPI ranks
(Source/SetGrids.cpp:54-58).  On MI355X a rank owns one large box (288 GB
of HBM per GPU): N ranks get a near-cubic process grid with the split in z
first, so 2 ranks exchange contiguous xy faces (512x512x256 slabs), 4 ranks
get 1x2x2 and 8 ranks 2x2x2 boxes of 256^3 at 512^3.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

Box6 = Tuple[int, int, int, int, int, int]


def process_grid(nranks: int) -> Tuple[int, int, int]:
    """(px, py, pz) with px*py*pz == nranks, split z first, then y, then x."""
    p = [1, 1, 1]
    n = nranks
    d = 2
    while n > 1:
        f = 2 if n % 2 == 0 else next(k for k in range(3, n + 1) if n % k == 0)
        p[d] *= f
        n //= f
        d = (d - 1) % 3
    return p[0], p[1], p[2]


def split_domain(domain: Box6, parts: Sequence[int]) -> List[Box6]:
    """Split `domain` into parts[0] x parts[1] x parts[2] boxes; box b has
    index (bx + px*(by + py*bz)) and lies in that order (x fastest)."""
    lo, hi = domain[:3], domain[3:]
    cuts = []
    for d in range(3):
        n = hi[d] - lo[d] + 1
        if n % parts[d]:
            raise ValueError(f"extent {n} not divisible by {parts[d]} in dir {d}")
        s = n // parts[d]
        cuts.append([(lo[d] + i * s, lo[d] + (i + 1) * s - 1) for i in range(parts[d])])
    boxes = []
    for bz in range(parts[2]):
        for by in range(parts[1]):
            for bx in range(parts[0]):
                boxes.append((cuts[0][bx][0], cuts[1][by][0], cuts[2][bz][0],
                              cuts[0][bx][1], cuts[1][by][1], cuts[2][bz][1]))
    return boxes


def decompose(n: Sequence[int], nranks: int, boxes_per_rank: Sequence[int] = (1, 1, 1)
              ) -> Tuple[Box6, List[Box6], List[int]]:
    """Domain [0, n) split over `nranks` ranks, each rank's share optionally
    split further into boxes_per_rank boxes (multi-box per GPU).  Returns
    (domain, boxes, owners)."""
    domain = (0, 0, 0, n[0] - 1, n[1] - 1, n[2] - 1)
    pg = process_grid(nranks)
    parts = [pg[d] * boxes_per_rank[d] for d in range(3)]
    boxes = split_domain(domain, parts)
    owners = []
    for b in boxes:
        idx = []
        for d in range(3):
            ext = (n[d]) // pg[d]
            idx.append(b[d] // ext)
        owners.append(idx[0] + pg[0] * (idx[1] + pg[1] * idx[2]))
    return domain, boxes, owners


def chombo_domain_split(domain: Box6, max_grid_size: int, block_factor: int) -> List[Box6]:
    """domainSplit (Chombo) as used by set_grids: boxes of at most
    max_grid_size cells per side (multiples of block_factor)."""
    parts = []
    for d in range(3):
        n = domain[3 + d] - domain[d] + 1
        if n % block_factor:
            raise ValueError("domain not a multiple of block_factor")
        nb = -(-n // max_grid_size)
        while n % nb or (n // nb) % block_factor:
            nb += 1
        parts.append(nb)
    return split_domain(domain, parts)
