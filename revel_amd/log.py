"""``log::Writer`` / ``log::Reader`` (src/log_writer.rs, src/log_reader.rs) via the C-ABI.

Mirrors the reference names and semantics:

* ``Writer(dest)`` / ``Writer.new_with_block_offset(dest, off)``;
  ``add_record(data)`` raises :class:`RevelError` where the reference returns
  ``Err``.
* ``Reader(file, checksum, initial_offset, gpu=...)``; ``read_record()``
  returns the logical record's bytes, ``None`` at EOF (the reference returns an
  empty Slice, log_reader.rs:140), and raises ``RevelError(IOError)`` on a
  checksum mismatch (log_reader.rs:142-152).  With ``checksum=True`` the CRCs
  are verified on the GPU: ``gpu``'s, or without one the calling thread's
  default context on its current device (the reference's 3-argument
  ``Reader::new(file, checksum, initial_offset)``, log_reader.rs:62).
"""
from __future__ import annotations

import ctypes
from ctypes import c_size_t, c_void_p
from typing import Optional

from ._lib import INVALID_ARGUMENT, check, lib
from .env import SequentialFile, WritableFile


class Writer:
    def __init__(self, dest: WritableFile, block_offset: int = 0):
        self._dest = dest  # keep the file alive (the reference shares it via Rc)
        self._h = lib().revel_log_writer_new(dest.handle, block_offset)
        if not self._h:
            raise ValueError("null destination file")

    @classmethod
    def new_with_block_offset(cls, dest: WritableFile, block_offset: int) -> "Writer":
        return cls(dest, block_offset)

    def add_record(self, data: bytes) -> None:
        check(lib().revel_log_writer_add_record(self._h, data, len(data)))

    @property
    def block_offset(self) -> int:
        return lib().revel_log_writer_block_offset(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().revel_log_writer_free(self._h)
            self._h = None


class Reader:
    def __init__(self, file: SequentialFile, checksum: bool = True, initial_offset: int = 0,
                 gpu=None, window_bytes: int = 0):
        self._gpu = gpu  # keep the context alive
        h = c_void_p()
        fh = file.take()
        # the reader owns the file from here on, also when construction fails
        check(lib().revel_log_reader_new(fh, 1 if checksum else 0, initial_offset,
                                         gpu.handle if gpu is not None else None, window_bytes, ctypes.byref(h)))
        self._h = h.value

    def read_record(self) -> Optional[bytes]:
        p, n = c_void_p(), c_size_t()
        check(lib().revel_log_reader_read_record(self._h, ctypes.byref(p), ctypes.byref(n)))
        if not p.value:
            return None
        return ctypes.string_at(p.value, n.value) if n.value else b""

    def read_record_into(self, scratch: bytearray) -> Optional[int]:
        """``read_record(&mut scratch)`` with the reference's ownership
        (log_reader.rs:76): the record is written into ``scratch``, grown
        when the library reports the bytes it needs; returns the record's
        length ``n`` (the record is ``scratch[:n]``, valid until the next
        call, as the reference's ``Slice<'b>`` borrows the scratch), ``None``
        at EOF.  No view of ``scratch`` is held between calls, so the scratch
        may grow on any call."""
        n, eof = c_size_t(), ctypes.c_int()
        while True:
            buf = (ctypes.c_char * len(scratch)).from_buffer(scratch) if len(scratch) else None
            rc = lib().revel_log_reader_read_record_into(self._h, buf, len(scratch), ctypes.byref(n),
                                                         ctypes.byref(eof))
            del buf
            if rc == INVALID_ARGUMENT and n.value > len(scratch):
                scratch.extend(bytes(n.value - len(scratch)))  # scratch.reserve(n), then call again
                continue
            check(rc)
            if eof.value:
                return None
            return n.value

    def last_record_offset(self) -> int:
        return lib().revel_log_reader_last_record_offset(self._h)

    def __iter__(self):
        while True:
            r = self.read_record()
            if r is None:
                return
            yield r

    def __del__(self):
        if getattr(self, "_h", None):
            lib().revel_log_reader_free(self._h)
            self._h = None
