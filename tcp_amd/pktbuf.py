"""ctypes mirror of the reference's packet buffer, for driving the drop-in ABI.

Layouts follow include/tcsum_legacy.h, which restates net/net/list.h:9-34,
net/net/pktbuf.h:15-41 and net/net/ipaddr.h:12-22 (LP64).  A PktBuf built
here is byte-for-byte what the stack hands to checksum_peso /
pktbuf_checksum16: a list of blocks, each exposing `size` bytes at `data`,
plus a cursor (pos, curr_blk, blk_offset).
"""
from __future__ import annotations

import ctypes

PKTBUF_BLK_SIZE = 127  # net/net/net_cfg.h:31


class Node(ctypes.Structure):
    pass


Node._fields_ = [("pre", ctypes.POINTER(Node)), ("next", ctypes.POINTER(Node))]


class List(ctypes.Structure):
    _fields_ = [("first", ctypes.POINTER(Node)), ("last", ctypes.POINTER(Node)), ("count", ctypes.c_int)]


class PktBlk(ctypes.Structure):
    _fields_ = [("node", Node), ("size", ctypes.c_int), ("data", ctypes.c_void_p),
                ("payload", ctypes.c_uint8 * PKTBUF_BLK_SIZE)]


class PktBufStruct(ctypes.Structure):
    _fields_ = [("total_size", ctypes.c_int), ("blk_list", List), ("ref", ctypes.c_int), ("node", Node),
                ("pos", ctypes.c_int), ("curr_blk", ctypes.POINTER(PktBlk)), ("blk_offset", ctypes.c_void_p)]


class IpAddr(ctypes.Structure):
    class _U(ctypes.Union):
        _fields_ = [("q_addr", ctypes.c_uint32), ("addr", ctypes.c_uint8 * 4)]

    _anonymous_ = ("u",)
    _fields_ = [("type", ctypes.c_int), ("u", _U)]

    @classmethod
    def v4(cls, a) -> "IpAddr":
        ip = cls()
        ip.type = 0  # IPADDR_V4
        for i, b in enumerate(bytes(a)[:4]):
            ip.addr[i] = b
        return ip


assert ctypes.sizeof(PktBlk) == 160 and ctypes.sizeof(PktBufStruct) == 80 and ctypes.sizeof(IpAddr) == 8


class PktBuf:
    """A chained packet buffer whose blocks hold the given pieces.

    Each piece is copied into its block's inline payload (right-aligned, as
    pktbuf_alloc's head insertion does, pktbuf.c:73-79) when it fits, or
    into a side buffer otherwise; `data` points at it.
    """

    def __init__(self, pieces):
        pieces = [bytes(p) for p in pieces]
        self.blocks = (PktBlk * max(1, len(pieces)))()
        self._side = []
        self.s = PktBufStruct()
        self.s.ref = 1
        total = 0
        prev = None
        for i, p in enumerate(pieces):
            b = self.blocks[i]
            b.size = len(p)
            if len(p) <= PKTBUF_BLK_SIZE:
                at = PKTBUF_BLK_SIZE - len(p)
                ctypes.memmove(ctypes.addressof(b.payload) + at, p, len(p))
                b.data = ctypes.addressof(b.payload) + at
            else:
                side = ctypes.create_string_buffer(p, len(p))
                self._side.append(side)
                b.data = ctypes.addressof(side)
            node = ctypes.pointer(b.node)
            if prev is None:
                self.s.blk_list.first = node
            else:
                prev.contents.next = node
                node.contents.pre = prev
            prev = node
            total += len(p)
        if pieces:
            self.s.blk_list.last = prev
        self.s.blk_list.count = len(pieces)
        self.s.total_size = total
        self.npieces = len(pieces)
        self.reset_access()

    @property
    def ptr(self) -> int:
        return ctypes.addressof(self.s)

    def _blk_addr(self, i: int) -> int:
        return ctypes.addressof(self.blocks[i])

    def reset_access(self) -> None:  # pktbuf.c:446-458
        self.s.pos = 0
        if self.npieces:
            self.s.curr_blk = ctypes.pointer(self.blocks[0])
            self.s.blk_offset = self.blocks[0].data
        else:
            self.s.curr_blk = ctypes.POINTER(PktBlk)()
            self.s.blk_offset = None

    def _index_of(self, blk) -> int | None:
        if not blk:
            return None
        addr = ctypes.addressof(blk.contents)
        for i in range(self.npieces):
            if self._blk_addr(i) == addr:
                return i
        raise AssertionError("cursor outside the chain")

    def _move_forward(self, size: int) -> None:  # pktbuf.c:463-483
        self.s.pos += size
        self.s.blk_offset = (self.s.blk_offset or 0) + size
        i = self._index_of(self.s.curr_blk)
        b = self.blocks[i]
        if self.s.blk_offset >= b.data + b.size:
            if i + 1 < self.npieces:
                self.s.curr_blk = ctypes.pointer(self.blocks[i + 1])
                self.s.blk_offset = self.blocks[i + 1].data
            else:
                self.s.curr_blk = ctypes.POINTER(PktBlk)()
                self.s.blk_offset = None

    def seek(self, offset: int) -> None:
        """pktbuf_seek (pktbuf.c:545-580): walk the cursor block by block."""
        if offset == self.s.pos:
            return
        if offset < 0 or offset >= self.s.total_size:
            raise ValueError("seek outside the buffer")
        if offset < self.s.pos:
            self.reset_access()
            move = offset
        else:
            move = offset - self.s.pos
        while move:
            i = self._index_of(self.s.curr_blk)
            b = self.blocks[i]
            remain = b.data + b.size - (self.s.blk_offset or 0)
            step = min(move, remain)
            self._move_forward(step)
            move -= step

    def cursor(self):
        """(pos, block index or None, offset inside the block)."""
        i = self._index_of(self.s.curr_blk)
        if i is None:
            return self.s.pos, None, 0
        return self.s.pos, i, (self.s.blk_offset or 0) - self.blocks[i].data
