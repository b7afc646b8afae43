"""A short correctness check of a job's halo transport on the devices it runs
on, before a run trusts it (bench.py's transport choice).

Every rank takes part.  A periodic n^3 field, split over the ranks as the
bench splits its domain (z first), is filled with a function of the global
cell index and its ghost layer poisoned; one exchange must then deliver
that function on every face ghost cell (the other ranks' cells arrive
through the transport, periodic images included), and a max-norm reduction
of a rank-dependent field must give the same value on every rank.  The
peer-mapped transport's polls are bounded in time, so a transport that
cannot deliver raises instead of hanging.
"""
from __future__ import annotations

import numpy as np

from .core import Comm, Grid, LevelData, OperatorParams, defineOperatorFactory
from .decomposition import decompose


def _value(k, j, i, n):
    return ((np.mod(k, n) * n + np.mod(j, n)) * n + np.mod(i, n)) + 1.0


def check_transport(comm: Comm, world: int, n: int = 32, rounds: int = 4) -> bool:
    """True when `rounds` exchanges (each of a different field, so a value
    left over from an earlier round is caught) and one reduction over `comm`
    give exactly the expected values on this rank (the caller combines the
    ranks' answers)."""
    dom, boxes, owners = decompose((n, n, n), world)
    grid = Grid(comm, dom, boxes, 1.0, periodic=(1, 1, 1), owners=owners)
    f = LevelData(grid)
    ok = True
    for r in range(rounds):
        expect = []
        for li in range(grid.num_local):
            b = grid.local_box(li)
            k, j, i = np.meshgrid(np.arange(b[2] - 1, b[5] + 2), np.arange(b[1] - 1, b[4] + 2),
                                  np.arange(b[0] - 1, b[3] + 2), indexing="ij")
            want = _value(k, j, i, n) + r * float(n) ** 3
            full = np.full(want.shape, -1.0)
            full[1:-1, 1:-1, 1:-1] = want[1:-1, 1:-1, 1:-1]
            f.upload(li, full, with_ghosts=True)
            expect.append(want)
        f.exchange()
        comm.synchronize()
        for li, want in enumerate(expect):
            g = f.download(li, with_ghosts=True)
            for ax in range(3):  # the six face ghost layers (edges / corners are not exchanged)
                for side in (0, -1):
                    sl = [slice(1, -1)] * 3
                    sl[ax] = side
                    ok &= bool(np.array_equal(g[tuple(sl)], want[tuple(sl)]))
    # a reduction across the ranks: every rank's cells hold rank + 1
    fr = LevelData(grid)
    fr.set_val(float(comm.rank + 1))
    b1 = LevelData(grid)
    b1.set_val(1.0)
    op = defineOperatorFactory(grid, b1, b1, OperatorParams(alpha=1.0, beta=-1.0)).AMRnewOp()
    ranks_with_boxes = sorted(set(owners))
    ok &= op.norm(fr, 0) == float(max(ranks_with_boxes) + 1)
    return ok
