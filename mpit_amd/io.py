"""MPI-IO on a node-local (or shared) POSIX file system (SURVEY Appendix A "I/O", 52
wrappers; Tier 3 in the build plan).

Every rank opens the same file; data moves with ``os.pread`` / ``os.pwrite`` on the bytes
of a tensor (HBM tensors are staged through host memory). File views (displacement,
etype, filetype) are honoured: the filetype's typemap, tiled by its extent, maps etype
offsets to byte offsets. Individual file pointers live in the File object; the shared
file pointer lives in a small sidecar file updated under ``fcntl`` locks, so
``*_shared`` / ``*_ordered`` operations are consistent across processes.
"""
from __future__ import annotations

import fcntl
import os
import struct
from typing import Optional

import torch

from .comm import COMM_WORLD, MAX, SUM, Comm, Request, Status
from .datatypes import BYTE, Datatype
from .misc import Info

MODE_RDONLY, MODE_RDWR, MODE_WRONLY, MODE_CREATE = 2, 8, 4, 1
MODE_EXCL, MODE_DELETE_ON_CLOSE, MODE_UNIQUE_OPEN, MODE_SEQUENTIAL, MODE_APPEND = 64, 16, 32, 256, 128
SEEK_SET, SEEK_CUR, SEEK_END = 600, 602, 604
DISPLACEMENT_CURRENT = -54278278


def _bytes_of(buf: torch.Tensor) -> bytes:
    return buf.detach().contiguous().cpu().reshape(-1).view(torch.uint8).numpy().tobytes()


def _fill(buf: torch.Tensor, data: bytes):
    n = len(data)
    if n == 0:
        return
    src = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    dst = buf.reshape(-1).view(torch.uint8)
    dst[:n].copy_(src.to(dst.device))


class File:
    def __init__(self, comm: Comm, path: str, amode: int, info: Optional[Info]):
        self.comm, self.path, self.amode, self.info = comm, path, amode, info or Info()
        flags = 0
        if amode & MODE_RDWR:
            flags |= os.O_RDWR
        elif amode & MODE_WRONLY:
            flags |= os.O_WRONLY
        else:
            flags |= os.O_RDONLY
        if amode & MODE_CREATE:
            flags |= os.O_CREAT
        if amode & MODE_APPEND:
            flags |= os.O_APPEND
        if (amode & MODE_EXCL) and comm.Get_rank() == 0:
            flags |= os.O_EXCL
        if comm.Get_rank() == 0:
            self.fd = os.open(path, flags, 0o644)
            comm.Barrier()
        else:
            comm.Barrier()
            self.fd = os.open(path, flags & ~(os.O_CREAT | os.O_EXCL), 0o644)
        self._sfp_path = path + ".mpit_sfp"
        if comm.Get_rank() == 0:
            with open(self._sfp_path, "wb") as f:
                f.write(struct.pack("<q", 0))
        comm.Barrier()
        self.disp, self.etype, self.filetype, self.datarep = 0, BYTE, BYTE, "native"
        self.pos = 0  # individual pointer, in etypes
        self.atomic = False
        self._errhandler = None
        if amode & MODE_APPEND:
            self.pos = os.fstat(self.fd).st_size // self.etype.Get_size()

    # ------------------------------------------------------------ views / offsets
    def Set_view(self, disp: int = 0, etype: Datatype = BYTE, filetype: Optional[Datatype] = None,
                 datarep: str = "native", info=None):
        self.disp = disp if disp != DISPLACEMENT_CURRENT else self.Get_byte_offset(self.pos)
        self.etype, self.filetype = etype, filetype or etype
        self.datarep = datarep
        self.pos = 0
        self.comm.Barrier()

    def Get_view(self):
        return self.disp, self.etype, self.filetype, self.datarep

    def Get_byte_offset(self, offset: int) -> int:
        """Absolute byte position of etype offset `offset` within the view."""
        if self._contiguous():
            return self.disp + offset * self.etype.Get_size()
        pieces = self._pieces()
        tile, k = divmod(offset, len(pieces))
        return self.disp + tile * self.filetype.extent + pieces[k]

    def _contiguous(self) -> bool:
        return self.filetype.is_contiguous_basic() and self.filetype.Get_size() == self.etype.Get_size()

    def _pieces(self):
        """Byte offsets (within one filetype tile) of its etype-sized pieces; the etype is
        a basic type, as in every MPI-IO use of the reference's era."""
        return sorted({d for d, _ in self.filetype.typemap})

    def _ranges(self, offset: int, nbytes: int):
        """Split [offset(etypes), +nbytes) of the view into contiguous file byte ranges."""
        if self._contiguous():
            yield self.disp + offset * self.etype.Get_size(), nbytes
            return
        es = self.etype.Get_size()
        pieces = self._pieces()
        i, left = offset, nbytes
        while left > 0:
            tile, k = divmod(i, len(pieces))
            n = min(es, left)
            yield self.disp + tile * self.filetype.extent + pieces[k], n
            left -= n
            i += 1

    def _pread(self, offset: int, nbytes: int) -> bytes:
        out = bytearray()
        for start, n in self._ranges(offset, nbytes):
            out += os.pread(self.fd, n, start)
        return bytes(out)

    def _pwrite(self, offset: int, data: bytes):
        o = 0
        for start, n in self._ranges(offset, len(data)):
            os.pwrite(self.fd, data[o: o + n], start)
            o += n

    def _count_etypes(self, nbytes: int) -> int:
        return nbytes // max(1, self.etype.Get_size())

    # ------------------------------------------------------------ explicit offsets
    def Read_at(self, offset: int, buf: torch.Tensor, status: Optional[Status] = None) -> Status:
        data = self._pread(offset, buf.numel() * buf.element_size())
        _fill(buf, data)
        st = Status(self.comm.Get_rank(), 0, 0, len(data), itemsize=buf.element_size())
        if status is not None:
            status._fill(st)
        return st

    def Write_at(self, offset: int, buf: torch.Tensor, status: Optional[Status] = None) -> Status:
        data = _bytes_of(buf)
        self._pwrite(offset, data)
        st = Status(self.comm.Get_rank(), 0, 0, len(data), itemsize=buf.element_size())
        if status is not None:
            status._fill(st)
        return st

    def Read_at_all(self, offset, buf, status=None):
        st = self.Read_at(offset, buf, status)
        self.comm.Barrier()
        return st

    def Write_at_all(self, offset, buf, status=None):
        st = self.Write_at(offset, buf, status)
        self.comm.Barrier()
        return st

    def Iread_at(self, offset, buf) -> Request:
        r = Request(self.comm)
        r._complete(self.Read_at(offset, buf))
        return r

    def Iwrite_at(self, offset, buf) -> Request:
        r = Request(self.comm)
        r._complete(self.Write_at(offset, buf))
        return r

    # ------------------------------------------------------------ individual pointer
    def Read(self, buf, status=None):
        st = self.Read_at(self.pos, buf, status)
        self.pos += self._count_etypes(st.count)
        return st

    def Write(self, buf, status=None):
        st = self.Write_at(self.pos, buf, status)
        self.pos += self._count_etypes(st.count)
        return st

    def Read_all(self, buf, status=None):
        st = self.Read(buf, status)
        self.comm.Barrier()
        return st

    def Write_all(self, buf, status=None):
        st = self.Write(buf, status)
        self.comm.Barrier()
        return st

    def Iread(self, buf) -> Request:
        r = Request(self.comm)
        r._complete(self.Read(buf))
        return r

    def Iwrite(self, buf) -> Request:
        r = Request(self.comm)
        r._complete(self.Write(buf))
        return r

    # split collectives
    def Read_all_begin(self, buf):
        self._split = self.Read_all(buf)

    def Read_all_end(self, buf=None):
        return self._split

    def Write_all_begin(self, buf):
        self._split = self.Write_all(buf)

    def Write_all_end(self, buf=None):
        return self._split

    def Read_at_all_begin(self, offset, buf):
        self._split = self.Read_at_all(offset, buf)

    def Read_at_all_end(self, buf=None):
        return self._split

    def Write_at_all_begin(self, offset, buf):
        self._split = self.Write_at_all(offset, buf)

    def Write_at_all_end(self, buf=None):
        return self._split

    def Seek(self, offset: int, whence: int = SEEK_SET):
        if whence == SEEK_SET:
            self.pos = offset
        elif whence == SEEK_CUR:
            self.pos += offset
        else:
            self.pos = self._count_etypes(max(0, self.Get_size() - self.disp)) + offset

    def Get_position(self) -> int:
        return self.pos

    # ------------------------------------------------------------ shared pointer
    def _sfp_update(self, delta: int) -> int:
        with open(self._sfp_path, "r+b") as f:
            fcntl.lockf(f, fcntl.LOCK_EX)
            try:
                cur = struct.unpack("<q", f.read(8))[0]
                f.seek(0)
                f.write(struct.pack("<q", cur + delta))
                f.flush()
            finally:
                fcntl.lockf(f, fcntl.LOCK_UN)
        return cur

    def Read_shared(self, buf, status=None):
        n = self._count_etypes(buf.numel() * buf.element_size())
        return self.Read_at(self._sfp_update(n), buf, status)

    def Write_shared(self, buf, status=None):
        n = self._count_etypes(buf.numel() * buf.element_size())
        return self.Write_at(self._sfp_update(n), buf, status)

    def Iread_shared(self, buf) -> Request:
        r = Request(self.comm)
        r._complete(self.Read_shared(buf))
        return r

    def Iwrite_shared(self, buf) -> Request:
        r = Request(self.comm)
        r._complete(self.Write_shared(buf))
        return r

    def _ordered(self, buf):
        n = torch.tensor([self._count_etypes(buf.numel() * buf.element_size())], dtype=torch.int64)
        before = torch.zeros(1, dtype=torch.int64)
        self.comm.Exscan(n, before, SUM)
        total = torch.zeros(1, dtype=torch.int64)
        self.comm.Allreduce(n, total, SUM)
        if self.comm.Get_rank() == 0:
            base = self._sfp_update(int(total.item()))
        else:
            base = 0
        b = torch.tensor([base], dtype=torch.int64)
        self.comm.Bcast(b, 0)
        return int(b.item()) + (int(before.item()) if self.comm.Get_rank() > 0 else 0)

    def Read_ordered(self, buf, status=None):
        return self.Read_at(self._ordered(buf), buf, status)

    def Write_ordered(self, buf, status=None):
        return self.Write_at(self._ordered(buf), buf, status)

    def Read_ordered_begin(self, buf):
        self._split = self.Read_ordered(buf)

    def Read_ordered_end(self, buf=None):
        return self._split

    def Write_ordered_begin(self, buf):
        self._split = self.Write_ordered(buf)

    def Write_ordered_end(self, buf=None):
        return self._split

    def Seek_shared(self, offset: int, whence: int = SEEK_SET):
        self.comm.Barrier()
        if self.comm.Get_rank() == 0:
            cur = self._sfp_update(0)
            if whence == SEEK_SET:
                new = offset
            elif whence == SEEK_CUR:
                new = cur + offset
            else:
                new = self._count_etypes(max(0, self.Get_size() - self.disp)) + offset
            self._sfp_update(new - cur)
        self.comm.Barrier()

    def Get_position_shared(self) -> int:
        return self._sfp_update(0)

    # ------------------------------------------------------------ file properties
    def Get_size(self) -> int:
        return os.fstat(self.fd).st_size

    def Set_size(self, size: int):
        if self.comm.Get_rank() == 0:
            os.ftruncate(self.fd, size)
        self.comm.Barrier()

    def Preallocate(self, size: int):
        if self.comm.Get_rank() == 0 and self.Get_size() < size:
            os.posix_fallocate(self.fd, 0, size)
        self.comm.Barrier()

    def Sync(self):
        os.fsync(self.fd)
        self.comm.Barrier()

    def Get_amode(self) -> int:
        return self.amode

    def Get_group(self):
        return self.comm.Get_group()

    def Get_info(self) -> Info:
        return self.info

    def Set_info(self, info: Info):
        self.info = info

    def Get_atomicity(self) -> bool:
        return self.atomic

    def Set_atomicity(self, flag: bool):
        self.atomic = bool(flag)

    def Get_type_extent(self, datatype: Datatype) -> int:
        return datatype.extent

    def Set_errhandler(self, eh):
        self._errhandler = eh

    def Get_errhandler(self):
        return self._errhandler

    def Call_errhandler(self, code):
        if self._errhandler:
            self._errhandler(self, code)

    def Close(self):
        if self.fd is None:
            return
        os.close(self.fd)
        self.fd = None
        self.comm.Barrier()
        if self.comm.Get_rank() == 0:
            try:
                os.unlink(self._sfp_path)
            except FileNotFoundError:
                pass
            if self.amode & MODE_DELETE_ON_CLOSE:
                os.unlink(self.path)
        self.comm.Barrier()

    @classmethod
    def Open(cls, comm: Optional[Comm], path: str, amode: int = MODE_RDONLY, info: Optional[Info] = None) -> "File":
        return cls(comm or COMM_WORLD(), path, amode, info)

    @staticmethod
    def Delete(path: str, info=None):
        os.unlink(path)


def File_open(comm, path, amode=MODE_RDONLY, info=None) -> File:
    return File.Open(comm, path, amode, info)


def File_delete(path, info=None):
    File.Delete(path, info)
