"""CPU emulation of the multi-rank path for world_size > 1 tests (gloo).

`run_world` starts one process per rank with a gloo process group on
127.0.0.1. `execute` runs a `HostPlan` the way `CopyPlan::execute` does on
the GPU, with numpy fabs in the device layout (FabGeom: padded rows, valid-lo
at `origin`):
  1. copy the same-rank items,
  2. pack the sends in plan order into one buffer (one slice per peer),
  3. exchange one message per peer (gloo isend/irecv here, ncclSend/ncclRecv
     over xGMI on the GPU),
  4. unpack in plan order.
Test infrastructure only.
"""
from __future__ import annotations

import os
import socket
import traceback

import numpy as np


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, args, q):
    import torch.distributed as dist
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        out = fn(rank, world, *args)
        q.put((rank, "ok", out))
    except Exception:  # report to the parent, which fails the test
        q.put((rank, "error", traceback.format_exc()))
    finally:
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def run_world(fn, world=2, args=(), timeout=240):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{out}")
            results[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]


# ------------------------------------------------------------------ fabs
def alloc(plan, layout, n, fill=np.nan):
    sy, sz, origin, total = plan.geom(layout, n)
    return np.full(total, fill)


def region(flat, off, sy, sz, nx, ny, nz):
    base = flat[off:]
    return np.lib.stride_tricks.as_strided(base, shape=(nz, ny, nx), strides=(sz * 8, sy * 8, 8))


def box_view(flat, geom, box, ghost=0):
    """(nz, ny, nx) view of a local box (valid region grown by `ghost`)."""
    sy, sz, origin, _ = geom
    nx, ny, nz = (box[3 + d] - box[d] + 1 + 2 * ghost for d in range(3))
    return region(flat, origin - ghost * (1 + sy + sz), sy, sz, nx, ny, nz)


def _copy(it, src_flats, src_geoms, dst_flats, dst_geoms, sbuf=None, rbuf=None):
    src, dst, soff, doff, ssy, ssz, dsy, dsz, nx, ny, nz, _ = (int(v) for v in it)
    if src >= 0:
        s = region(src_flats[src], src_geoms[src][2] + soff, ssy, ssz, nx, ny, nz)
    else:
        s = region(rbuf, soff, ssy, ssz, nx, ny, nz)
    if dst >= 0:
        d = region(dst_flats[dst], dst_geoms[dst][2] + doff, dsy, dsz, nx, ny, nz)
    else:
        d = region(sbuf, doff, dsy, dsz, nx, ny, nz)
    d[...] = s


def execute(plan, src_flats, dst_flats):
    import torch
    import torch.distributed as dist
    sg = [plan.geom(0, n) for n in range(len(plan.src_local))]
    dg = [plan.geom(1, n) for n in range(len(plan.dst_local))]
    for it in plan.local:
        _copy(it, src_flats, sg, dst_flats, dg)
    sbuf = np.zeros(max(plan.send_total, 1))
    rbuf = np.zeros(max(plan.recv_total, 1))
    for it in plan.pack:
        _copy(it, src_flats, sg, None, None, sbuf=sbuf)
    reqs, recvs = [], []
    for p in plan.peers:
        if p["send_cnt"]:
            t = torch.from_numpy(sbuf[p["send_off"]:p["send_off"] + p["send_cnt"]].copy())
            reqs.append(dist.isend(t, p["peer"]))
        if p["recv_cnt"]:
            t = torch.empty(p["recv_cnt"], dtype=torch.float64)
            reqs.append(dist.irecv(t, p["peer"]))
            recvs.append((p, t))
    for r in reqs:
        r.wait()
    for p, t in recvs:
        rbuf[p["recv_off"]:p["recv_off"] + p["recv_cnt"]] = t.numpy()
    for it in plan.unpack:
        _copy(it, None, None, dst_flats, dg, rbuf=rbuf)
