"""world_size = 2, 4 and 8 tests of the multi-rank path on CPU (gloo).

The GPU path moves halos with RCCL over xGMI, and the data it moves is
fixed by the per-rank CopyPlan. These tests take that exact plan from
libmgic (`mgic_plan_*`, no GPU needed). They run it across two processes
with gloo standing in for RCCL, and check:
  * the face ghost exchange with interleaved box ownership and periodic
    images delivers exactly the neighbour values (edges/corners and
    non-periodic domain faces untouched), i.e. pack order on the sender
    == unpack order on the receiver for every peer pair;
  * a distributed GSRB sweep (exchange -> homogeneous Dirichlet BC ->
    GSRBHELMHOLTZVC3D per local box, per colour) equals the single-box
    oracle bit for bit (levelGSRB, VariableCoeffPoissonOperator.cpp:290-331);
  * the coarse-level gather to rank 0 and the scatter back (valid + face
    ghosts) used for agglomeration.
"""
import numpy as np
import pytest

from mg_ic_code_amd.decomposition import split_domain
from mg_ic_code_amd.plan import HostPlan
from tests import dist_emul as de


def _global(shape):
    nz, ny, nx = shape
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return (x + 100.0 * y + 10000.0 * z).astype(np.float64)


def _exchange_worker(rank, world, dom, parts, owners, periodic):
    boxes = split_domain(dom, parts)
    plan = HostPlan(rank, world, dom, boxes, owners, periodic=periodic)
    n = [dom[3 + d] - dom[d] + 1 for d in range(3)]
    G = _global(n[::-1])
    flats = [de.alloc(plan, 0, i) for i in range(len(plan.src_local))]
    for i, b in enumerate(plan.src_local):
        bx = boxes[b]
        de.box_view(flats[i], plan.geom(0, i), bx)[...] = G[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1,
                                                          bx[0]:bx[3] + 1]
    de.execute(plan, flats, flats)
    bad = 0
    for i, b in enumerate(plan.src_local):
        bx = boxes[b]
        full = de.box_view(flats[i], plan.geom(0, i), bx, ghost=1)
        nz, ny, nx = full.shape
        for z in range(nz):
            for y in range(ny):
                for x in range(nx):
                    g = (bx[0] - 1 + x, bx[1] - 1 + y, bx[2] - 1 + z)
                    outside = [d for d in range(3) if g[d] < bx[d] or g[d] > bx[3 + d]]
                    if not outside:
                        continue
                    v = full[z, y, x]
                    if len(outside) > 1:  # edge / corner: trimmed
                        bad += not np.isnan(v)
                        continue
                    d = outside[0]
                    gg = list(g)
                    if gg[d] < 0 or gg[d] >= n[d]:
                        if not periodic[d]:
                            bad += not np.isnan(v)
                            continue
                        gg[d] %= n[d]
                    bad += v != G[gg[2], gg[1], gg[0]]
    return bad, len(plan.local), len(plan.pack), len(plan.unpack)


@pytest.mark.parametrize("periodic", [(0, 0, 0), (1, 0, 1)])
def test_two_rank_exchange_plan_delivers_face_ghosts(periodic):
    dom = (0, 0, 0, 11, 9, 7)
    parts = (2, 2, 1)
    owners = [0, 1, 1, 0]  # interleaved: same-rank and cross-rank faces
    res = de.run_world(_exchange_worker, 2, (dom, parts, owners, periodic))
    for bad, nl, npk, nun in res:
        assert bad == 0
        assert npk > 0 and nun > 0  # the cross-rank path is exercised
    # what rank 0 sends is what rank 1 receives
    assert res[0][2] == res[1][3] and res[1][2] == res[0][3]


def _gsrb_worker(rank, world, n, parts, owners, seed):
    import oracle
    from oracle import Fab
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    boxes = split_domain(dom, parts)
    rng = np.random.default_rng(seed)
    u0 = rng.uniform(-1, 1, (n, n, n))
    rhs = rng.uniform(-1, 1, (n, n, n))
    a = rng.uniform(-2.0, -0.5, (n, n, n))
    b = rng.uniform(0.5, 2.0, (n, n, n))
    dx, alpha, beta = 0.1, 1.0, -1.0
    plan = HostPlan(rank, world, dom, boxes, owners)
    flats = [de.alloc(plan, 0, i, 0.0) for i in range(len(plan.src_local))]

    def sl(bx):
        return np.s_[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1, bx[0]:bx[3] + 1]

    for i, bi in enumerate(plan.src_local):
        de.box_view(flats[i], plan.geom(0, i), boxes[bi])[...] = u0[sl(boxes[bi])]
    for colour in (0, 1):
        de.execute(plan, flats, flats)  # .cpp:301
        for i, bi in enumerate(plan.src_local):
            bx = boxes[bi]
            full = de.box_view(flats[i], plan.geom(0, i), bx, ghost=1)
            # homogeneous DiriBC order 1 on domain faces: ghost = -near (.cpp:307-310)
            if bx[0] == 0:
                full[1:-1, 1:-1, 0] = -full[1:-1, 1:-1, 1]
            if bx[3] == n - 1:
                full[1:-1, 1:-1, -1] = -full[1:-1, 1:-1, -2]
            if bx[1] == 0:
                full[1:-1, 0, 1:-1] = -full[1:-1, 1, 1:-1]
            if bx[4] == n - 1:
                full[1:-1, -1, 1:-1] = -full[1:-1, -2, 1:-1]
            if bx[2] == 0:
                full[0, 1:-1, 1:-1] = -full[1, 1:-1, 1:-1]
            if bx[5] == n - 1:
                full[-1, 1:-1, 1:-1] = -full[-2, 1:-1, 1:-1]
            uf = np.ascontiguousarray(full)
            lo = tuple(bx[:3])
            glo = tuple(v - 1 for v in lo)
            hi = tuple(bx[3:])
            ab, bb, rb = (np.ascontiguousarray(x[sl(bx)]) for x in (a, b, rhs))
            lam = np.zeros_like(ab)
            oracle.lam(Fab(lam, lo), Fab(ab, lo), lo, hi, alpha, beta, dx)
            oracle.gsrb(Fab(uf, glo), Fab(rb, lo), lo, hi, dx, alpha, Fab(ab, lo), beta, Fab(bb, lo),
                        Fab(lam, lo), colour)
            full[...] = uf
    out = {}
    for i, bi in enumerate(plan.src_local):
        out[bi] = np.array(de.box_view(flats[i], plan.geom(0, i), boxes[bi]))
    return out


def test_two_rank_gsrb_sweep_matches_single_box_oracle():
    import oracle
    n, parts, owners, seed = 16, (2, 1, 2), [0, 1, 1, 0], 3
    res = de.run_world(_gsrb_worker, 2, (n, parts, owners, seed))
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    boxes = split_domain(dom, parts)
    got = np.zeros((n, n, n))
    for r in res:
        for bi, arr in r.items():
            bx = boxes[bi]
            got[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1, bx[0]:bx[3] + 1] = arr
    rng = np.random.default_rng(seed)
    u0 = rng.uniform(-1, 1, (n, n, n))
    rhs = rng.uniform(-1, 1, (n, n, n))
    a = rng.uniform(-2.0, -0.5, (n, n, n))
    b = rng.uniform(0.5, 2.0, (n, n, n))
    o = oracle.OracleMG([dom], dom, 0.1, alpha=1.0, beta=-1.0, nlevels=1)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs), (oracle.PHI, u0)):
        o.set(0, f, 0, arr)
    o.setup()
    o.level_gsrb(0, oracle.PHI, oracle.RHS)
    assert np.array_equal(got, o.get(0, oracle.PHI, 0))


def _gather_worker(rank, world, dom, parts, owners):
    boxes = split_domain(dom, parts)
    n = [dom[3 + d] - dom[d] + 1 for d in range(3)]
    G = _global(n[::-1])
    # gather: 4 boxes on 2 ranks -> one box on rank 0 (valid cells)
    g = HostPlan(rank, world, dom, boxes, owners, [dom], [0], with_valid=True, with_faces=False)
    src = [de.alloc(g, 0, i) for i in range(len(g.src_local))]
    for i, b in enumerate(g.src_local):
        bx = boxes[b]
        de.box_view(src[i], g.geom(0, i), bx)[...] = G[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1,
                                                       bx[0]:bx[3] + 1]
    dst = [de.alloc(g, 1, i) for i in range(len(g.dst_local))]
    de.execute(g, src, dst)
    gathered_ok = True
    if rank == 0:
        gathered_ok = bool(np.array_equal(de.box_view(dst[0], g.geom(1, 0), dom), G))
    else:
        gathered_ok = len(dst) == 0
    # scatter back: valid + face ghosts from the single box
    s = HostPlan(rank, world, dom, [dom], [0], boxes, owners, with_valid=True, with_faces=True)
    back = [de.alloc(s, 1, i) for i in range(len(s.dst_local))]
    de.execute(s, dst, back)
    bad = 0
    for i, b in enumerate(s.dst_local):
        bx = boxes[b]
        full = de.box_view(back[i], s.geom(1, i), bx, ghost=1)
        assert np.array_equal(full[1:-1, 1:-1, 1:-1], G[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1,
                                                         bx[0]:bx[3] + 1])
        if bx[0] > 0:
            bad += not np.array_equal(full[1:-1, 1:-1, 0], G[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1,
                                                            bx[0] - 1])
        if bx[0] == 0:
            bad += not np.all(np.isnan(full[1:-1, 1:-1, 0]))
    return gathered_ok, bad


def test_two_rank_gather_to_rank0_and_scatter_back():
    dom = (0, 0, 0, 15, 7, 7)
    res = de.run_world(_gather_worker, 2, (dom, (2, 1, 2), [0, 1, 1, 0]))
    for ok, bad in res:
        assert ok and bad == 0


def _deep_worker(rank, world, n, parts, owners, periodic, seed):
    """Deep-halo schedule across ranks: one 4-deep ghost-shell exchange, then
    sweep 1 on the box grown by 2 across exchanged faces and sweep 2 on the
    box (each as the fused sweep's passes: RED on the region grown by one
    more, then BLACK), with no exchange in between."""
    import oracle
    from oracle import Fab
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    boxes = list(parts) if isinstance(parts, list) else split_domain(dom, parts)
    rng = np.random.default_rng(seed)
    u0, rhs = rng.uniform(-1, 1, (n, n, n)), rng.uniform(-1, 1, (n, n, n))
    a, b = rng.uniform(-2.0, -0.5, (n, n, n)), rng.uniform(0.5, 2.0, (n, n, n))
    dx, alpha, beta, G = 0.1, 1.0, -1.0, 4
    plan = HostPlan(rank, world, dom, boxes, owners, periodic=periodic, shell=G)
    flats = [de.alloc(plan, 0, i) for i in range(len(plan.src_local))]
    for i, bi in enumerate(plan.src_local):
        bx = boxes[bi]
        de.box_view(flats[i], plan.geom(0, i), bx)[...] = u0[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1,
                                                              bx[0]:bx[3] + 1]
    de.execute(plan, flats, flats)
    for grow in (2, 0):
        for i, bi in enumerate(plan.src_local):
            bx = boxes[bi]
            full = de.box_view(flats[i], plan.geom(0, i), bx, ghost=G)
            glo = tuple(v - G for v in bx[:3])
            # coefficient fabs over the box grown by G (periodic images)
            idx = [np.arange(bx[d] - G, bx[3 + d] + G + 1) for d in range(3)]
            idx = [np.mod(ix, n) if periodic[d] else np.clip(ix, 0, n - 1) for d, ix in enumerate(idx)]
            ax = np.ix_(idx[2], idx[1], idx[0])
            ag, bg, rg = (np.ascontiguousarray(x[ax]) for x in (a, b, rhs))
            lam = np.zeros_like(ag)
            exch = [[periodic[d] or bx[d] > 0, periodic[d] or bx[3 + d] < n - 1] for d in range(3)]
            hi_g = tuple(v + G for v in bx[3:])
            oracle.lam(Fab(lam, glo), Fab(ag, glo), glo, hi_g, alpha, beta, dx)
            for colour, g in ((0, grow + 1), (1, grow)):
                lo = tuple(bx[d] - (g if exch[d][0] else 0) for d in range(3))
                hi = tuple(bx[3 + d] + (g if exch[d][1] else 0) for d in range(3))
                # homogeneous DiriBC order 1 on domain faces: ghost = -near
                if not exch[0][0]:
                    full[:, :, G - 1] = -full[:, :, G]
                if not exch[0][1]:
                    full[:, :, -G] = -full[:, :, -G - 1]
                if not exch[1][0]:
                    full[:, G - 1, :] = -full[:, G, :]
                if not exch[1][1]:
                    full[:, -G, :] = -full[:, -G - 1, :]
                if not exch[2][0]:
                    full[G - 1] = -full[G]
                if not exch[2][1]:
                    full[-G] = -full[-G - 1]
                uf = np.ascontiguousarray(full)
                oracle.gsrb(Fab(uf, glo), Fab(rg, glo), lo, hi, dx, alpha, Fab(ag, glo), beta,
                            Fab(bg, glo), Fab(lam, glo), colour)
                full[...] = uf
    return {bi: np.array(de.box_view(flats[i], plan.geom(0, i), boxes[bi]))
            for i, bi in enumerate(plan.src_local)}


@pytest.mark.parametrize("periodic", [(0, 0, 0), (1, 1, 0)])
def test_two_rank_deep_halo_two_sweeps_match_single_box_oracle(periodic):
    # the 4-deep shell plan across ranks carries everything two sweeps need
    import oracle
    n, parts, owners, seed = 16, (2, 2, 2), [0, 1, 1, 0, 1, 0, 0, 1], 5
    res = de.run_world(_deep_worker, 2, (n, parts, owners, periodic, seed))
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    boxes = split_domain(dom, parts)
    got = np.full((n, n, n), np.nan)
    for r in res:
        for bi, arr in r.items():
            bx = boxes[bi]
            got[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1, bx[0]:bx[3] + 1] = arr
    rng = np.random.default_rng(seed)
    u0, rhs = rng.uniform(-1, 1, (n, n, n)), rng.uniform(-1, 1, (n, n, n))
    a, b = rng.uniform(-2.0, -0.5, (n, n, n)), rng.uniform(0.5, 2.0, (n, n, n))
    o = oracle.OracleMG([dom], dom, 0.1, alpha=1.0, beta=-1.0, nlevels=1, periodic=periodic)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs), (oracle.PHI, u0)):
        o.set(0, f, 0, arr)
    o.setup()
    o.level_gsrb(0, oracle.PHI, oracle.RHS)
    o.level_gsrb(0, oracle.PHI, oracle.RHS)
    assert np.array_equal(got, o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("world", [4, 8])
def test_bench_split_deep_halo_two_sweeps_match_single_box_oracle(world):
    # the exact splits bench.py --gpus 4 / 8 run (decompose: 1x2x2 slabs /
    # 2x2x2 boxes, one box per rank), rehearsed with `world` gloo ranks on the
    # CPU: one 4-deep shell exchange carries two sweeps, bit-identical to the
    # single-box oracle
    import oracle
    from mg_ic_code_amd.decomposition import decompose
    n, seed = 16, 7
    dom, boxes, owners = decompose((n, n, n), world)
    assert len(boxes) == world and sorted(owners) == list(range(world))
    res = de.run_world(_deep_worker, world, (n, list(boxes), list(owners), (0, 0, 0), seed))
    got = np.full((n, n, n), np.nan)
    for r in res:
        for bi, arr in r.items():
            bx = boxes[bi]
            got[bx[2]:bx[5] + 1, bx[1]:bx[4] + 1, bx[0]:bx[3] + 1] = arr
    rng = np.random.default_rng(seed)
    u0, rhs = rng.uniform(-1, 1, (n, n, n)), rng.uniform(-1, 1, (n, n, n))
    a, b = rng.uniform(-2.0, -0.5, (n, n, n)), rng.uniform(0.5, 2.0, (n, n, n))
    o = oracle.OracleMG([dom], dom, 0.1, alpha=1.0, beta=-1.0, nlevels=1)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs), (oracle.PHI, u0)):
        o.set(0, f, 0, arr)
    o.setup()
    o.level_gsrb(0, oracle.PHI, oracle.RHS)
    o.level_gsrb(0, oracle.PHI, oracle.RHS)
    assert np.array_equal(got, o.get(0, oracle.PHI, 0))


def test_gather_plan_with_many_peers_is_rccl_executable():
    # the coarse-level gather of a 40-rank job onto rank 0 receives from 39
    # peers: RCCL executes such a plan (its tables are built whatever the
    # peer count); the peer-mapped transport, whose launch tables hold at most
    # 32 peers, refuses it -- and only a plan that transport executes builds
    # its tables (an RCCL job must not trip the IPC peer limit)
    from mg_ic_code_amd._lib import MgicError
    world = 40
    dom = (0, 0, 0, 79, 31, 15)
    boxes = split_domain(dom, (10, 2, 2))
    owners = list(range(world))
    plan = HostPlan(0, world, dom, boxes, owners, dst_boxes=[dom], dst_owners=[0],
                    with_valid=True, with_faces=False)
    assert len(plan.peers) == world - 1
    plan.check_transport("rccl")
    with pytest.raises(MgicError, match="too many peers"):
        plan.check_transport("ipc")
    # a rank's own face-exchange plan (at most 26 neighbours) suits both
    ex = HostPlan(5, world, dom, boxes, owners)
    ex.check_transport("rccl")
    ex.check_transport("ipc")


def _message_rows(plans, world, block_elems=2048):
    """{(sender, receiver): (put rows, get rows)} of every message, each as
    sorted (flag, first element, count) tuples."""
    msgs = {}
    for r, plan in enumerate(plans):
        for side, peer, flag, first, cnt in plan.ipc_blocks(block_elems).tolist():
            assert 0 < cnt <= block_elems  # blocks of at most the configured size
            key = (r, peer) if side == 0 else (peer, r)
            msgs.setdefault(key, ([], []))[side].append((flag, first, cnt))
    return {k: (sorted(p), sorted(g)) for k, (p, g) in msgs.items()}


@pytest.mark.parametrize("world,shell,periodic", [(2, 4, (0, 0, 0)), (4, 4, (0, 0, 0)),
                                                  (8, 4, (0, 0, 0)), (8, 0, (0, 0, 0)),
                                                  (8, 4, (1, 1, 1)), (3, 1, (1, 0, 1))])
@pytest.mark.parametrize("block_elems", [512, 1024, 1536, 2048, 4096])
def test_ipc_message_blocks_agree_on_both_sides(world, shell, periodic, block_elems):
    # the peer-mapped transport's hand-off: get block f of a message waits for
    # the flag of put block f, so both sides must split every message into the
    # same blocks, numbered by message offset 0, 1, ... (bench.py's splits,
    # shells and faces, periodic images as self messages, small edge items;
    # world 3: six boxes, two per rank)
    from mg_ic_code_amd.decomposition import decompose
    n = 40
    if world == 3:
        dom = (0, 0, 0, 47, n - 1, n - 1)
        boxes, owners = split_domain(dom, (3, 2, 1)), [0, 1, 2, 2, 1, 0]
    else:
        dom, boxes, owners = decompose((n, n, n), world)
    plans = [HostPlan(r, world, dom, list(boxes), list(owners), periodic=periodic, shell=shell)
             for r in range(world)]
    msgs = _message_rows(plans, world, block_elems)
    assert msgs
    for (s, r), (put, get) in msgs.items():
        assert put == get, (s, r)
        flags = [f for f, _, _ in put]
        assert flags == list(range(len(put)))
        firsts = [a for _, a, _ in put]
        assert firsts == sorted(firsts) and firsts[0] == 0
        # the blocks tile the message: contiguous, no gaps
        assert all(a + c == b for (_, a, c), (_, b, _) in zip(put, put[1:]))
        send = next(p for p in plans[s].peers if p["peer"] == r)
        assert firsts[-1] + put[-1][2] == send["send_cnt"]


def test_ipc_message_blocks_agree_for_the_gather_to_rank0():
    # agglomeration: the coarse level's boxes gathered onto rank 0 and
    # scattered back, the plans bench.py's N > 1 runs build
    world = 8
    dom = (0, 0, 0, 31, 31, 31)
    boxes = split_domain(dom, (2, 2, 2))
    owners = list(range(world))
    gather = [HostPlan(r, world, dom, boxes, owners, dst_boxes=[dom], dst_owners=[0],
                       with_valid=True, with_faces=False) for r in range(world)]
    scatter = [HostPlan(r, world, dom, [dom], [0], boxes, owners, with_valid=True,
                        with_faces=True) for r in range(world)]
    for plans in (gather, scatter):
        msgs = _message_rows(plans, world)
        assert len(msgs) == world - 1
        for (s, r), (put, get) in msgs.items():
            assert put == get and [f for f, _, _ in put] == list(range(len(put)))
