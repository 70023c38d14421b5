"""Reader of the agent's raw slot stream in shared memory.

Rank 0's agent started with ``slot_ring="name"`` republishes every 256-byte
counter slot it receives (all ranks) into a lock-free SPSC ring
(src/ring/RingBuffer.h ShmRing: ``/dev/shm/<name>.hdr`` + ``<name>.data``).
This reader is the single consumer: it copies whole slots out and advances
the tail, so another process (a dashboard, the daemon, a notebook) sees the
full 1 kHz stream, not just the per-interval aggregates.

    r = SlotRingReader("dynolog_gpu_slots")
    slots = r.read()          # numpy structured array, dynolog_amd.utils.slots.SLOT_DTYPE
"""
from __future__ import annotations

import mmap
import os
import struct

import numpy as np

from dynolog_amd.utils.slots import SLOT_BYTES, SLOT_DTYPE

# RingHeader<NoExtra> layout (64-B aligned fields): head @0, inWriteTx @8,
# tail @64, inReadTx @72, size @128, mask @136, magic @144.
_HEAD, _TAIL, _SIZE, _MAGIC = 0, 64, 128, 144
_RING_MAGIC = 0x52494E4748445231


class SlotRingReader:
    def __init__(self, name: str):
        self._hdr = self._map("/dev/shm/" + name + ".hdr", writable=True)
        if struct.unpack_from("=Q", self._hdr, _MAGIC)[0] != _RING_MAGIC:
            raise ValueError(f"{name}: not a dynolog shm ring")
        self.size = struct.unpack_from("=Q", self._hdr, _SIZE)[0]
        self._data = self._map("/dev/shm/" + name + ".data", writable=False)

    @staticmethod
    def _map(path: str, writable: bool) -> mmap.mmap:
        fd = os.open(path, os.O_RDWR if writable else os.O_RDONLY)
        try:
            return mmap.mmap(fd, 0, prot=mmap.PROT_READ | (mmap.PROT_WRITE if writable else 0))
        finally:
            os.close(fd)

    def pending(self) -> int:
        head, tail = self._cursors()
        return (head - tail) // SLOT_BYTES

    def _cursors(self):
        return (struct.unpack_from("=Q", self._hdr, _HEAD)[0], struct.unpack_from("=Q", self._hdr, _TAIL)[0])

    def read(self, max_slots: int = 1 << 20) -> np.ndarray:
        """Consume up to max_slots whole slots (oldest first)."""
        head, tail = self._cursors()
        n = min((head - tail) // SLOT_BYTES, max_slots)
        if n <= 0:
            return np.zeros(0, dtype=SLOT_DTYPE)
        nbytes = n * SLOT_BYTES
        off = tail & (self.size - 1)
        first = min(nbytes, self.size - off)
        buf = bytes(self._data[off:off + first]) + bytes(self._data[0:nbytes - first])
        # release the space (aligned 8-byte store: atomic on x86-64)
        struct.pack_into("=Q", self._hdr, _TAIL, tail + nbytes)
        return np.frombuffer(buf, dtype=SLOT_DTYPE).copy()

    def close(self) -> None:
        self._hdr.close()
        self._data.close()
