"""Host-side view of the ghost-exchange / gather plans (no GPU needed).

``HostPlan`` returns the plan that rank ``rank`` of ``size`` executes for a
pair of layouts (``mgic_plan_*`` in include/mgic.h). The on-device
``CopyPlan`` is built by the same code. The plan mirrors Chombo's Copier built by
``exchangeDefine(grids, IntVect::Unit)`` + ``trimEdges``
(Source/VariableCoeffPoissonOperatorFactory.cpp:82-99,179-185): face ghosts
only, periodic images included. With ``with_valid`` it is a
``LevelData::copyTo`` between layouts, e.g. the gather of a coarse level to
rank 0 and the scatter back.

Each item is one rectangular copy:
``{src, dst, soff, doff, ssy, ssz, dsy, dsz, nx, ny, nz, peer}``. ``src``
and ``dst`` are local box indices, or -1 for the per-peer message buffer.
Offsets count doubles from the box's valid-lo cell (or from the start of
the buffer); strides are in doubles. Local copies run first. Then each
rank packs its sends in plan order, exchanges one message per peer (RCCL on
the GPU), and unpacks.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

FIELDS = ("src", "dst", "soff", "doff", "ssy", "ssz", "dsy", "dsz", "nx", "ny", "nz", "peer")


def _ints(v):
    v = [int(x) for x in v]
    return (ctypes.c_int * len(v))(*v)


class HostPlan:
    def __init__(self, rank, size, domain, src_boxes, src_owners, dst_boxes=None,
                 dst_owners=None, periodic=(0, 0, 0), with_valid=False, with_faces=True,
                 shell=0):
        """shell > 0: the `shell`-deep ghost-shell exchange of the src layout
        (faces, edges, corners; mgic_plan_create_shell) instead."""
        if dst_boxes is None:
            dst_boxes, dst_owners = src_boxes, src_owners
        h = ctypes.c_void_p()
        if shell > 0:
            _lib.call("mgic_plan_create_shell", int(rank), int(size), _ints(domain),
                      _ints(periodic), len(src_boxes), _ints([v for b in src_boxes for v in b]),
                      _ints(src_owners), int(shell), ctypes.byref(h))
        else:
            _lib.call("mgic_plan_create", int(rank), int(size), _ints(domain), _ints(periodic),
                      len(src_boxes), _ints([v for b in src_boxes for v in b]), _ints(src_owners),
                      len(dst_boxes), _ints([v for b in dst_boxes for v in b]),
                      _ints(dst_owners), int(bool(with_valid)), int(bool(with_faces)),
                      ctypes.byref(h))
        self._h = h
        self.rank, self.size = int(rank), int(size)
        self.src_local = [i for i, o in enumerate(src_owners) if o == rank]
        self.dst_local = [i for i, o in enumerate(dst_owners) if o == rank]
        n = [ctypes.c_int() for _ in range(4)]
        _lib.call("mgic_plan_sizes", h, *[ctypes.byref(x) for x in n])
        self.local, self.pack, self.unpack = (self._items(w, n[w].value) for w in range(3))
        npeer = n[3].value
        peers = (ctypes.c_int * max(npeer, 1))()
        arrs = [(ctypes.c_longlong * max(npeer, 1))() for _ in range(4)]
        _lib.call("mgic_plan_peers", h, peers, *arrs)
        self.peers = [dict(peer=peers[i], send_cnt=arrs[0][i], send_off=arrs[1][i],
                           recv_cnt=arrs[2][i], recv_off=arrs[3][i]) for i in range(npeer)]
        self.send_total = sum(p["send_cnt"] for p in self.peers)
        self.recv_total = sum(p["recv_cnt"] for p in self.peers)

    def _items(self, which, n):
        out = np.zeros((n, 12), dtype=np.int64)
        if n:
            _lib.call("mgic_plan_items", self._h, which,
                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)))
        return out

    def check_transport(self, transport: str) -> None:
        """Build the host tables `transport` ("rccl" / "ipc") executes this
        plan with; raises when it cannot (the peer-mapped transport takes at
        most 32 peers per plan)."""
        _lib.call("mgic_plan_check_transport", self._h, {"rccl": 1, "ipc": 2}[transport])

    def ipc_blocks(self, block_elems: int = 2048) -> np.ndarray:
        """The peer-mapped transport's put / get blocks: rows (side 0 put /
        1 get, peer rank, flag, first message element, element count), for
        blocks of at most block_elems elements (MGIC_IPC_BLOCK_ELEMS; one
        size per plan)."""
        n = ctypes.c_int()
        _lib.call("mgic_plan_ipc_blocks_per", self._h, int(block_elems), ctypes.byref(n), None)
        out = np.zeros((n.value, 5), dtype=np.int64)
        if n.value:
            _lib.call("mgic_plan_ipc_blocks_per", self._h, int(block_elems), ctypes.byref(n),
                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)))
        return out

    def geom(self, layout, n):
        """(sy, sz, origin, total) of local box n; layout 0 = src, 1 = dst."""
        g = (ctypes.c_longlong * 4)()
        _lib.call("mgic_plan_geom", self._h, int(layout), int(n), g)
        return tuple(int(x) for x in g)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib.mgic_plan_destroy(h)
            self._h = None
