"""File abstractions of src/env.rs:25-266, via the C-ABI."""
from __future__ import annotations

import ctypes
from ctypes import c_size_t, c_void_p

from ._lib import check, lib


class WritableFile:
    """``trait WritableFile`` (env.rs:40-50)."""

    def __init__(self, handle: int, memory: bool):
        self._h = handle
        self.memory = memory

    @property
    def handle(self) -> int:
        if not self._h:
            raise ValueError("file already freed")
        return self._h

    def append(self, data: bytes) -> None:
        check(lib().revel_writable_file_append(self.handle, data, len(data)))

    def flush(self) -> None:
        check(lib().revel_writable_file_flush(self.handle))

    def close(self) -> None:
        check(lib().revel_writable_file_close(self.handle))

    def sync(self) -> None:
        check(lib().revel_writable_file_sync(self.handle))

    def contents(self) -> bytes:
        """Bytes of a memory file (accessor the reference lacks)."""
        p, n = c_void_p(), c_size_t()
        check(lib().revel_memory_writable_file_contents(self.handle, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p.value, n.value) if n.value else b""

    def free(self) -> None:
        if self._h:
            lib().revel_writable_file_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class MemoryWritableFile(WritableFile):
    """env.rs:201-230."""

    def __init__(self):
        super().__init__(lib().revel_memory_writable_file_new(), True)


class PosixWritableFile(WritableFile):
    """env.rs:25-38 ``new_writable_file(filename)``."""

    def __init__(self, path: str):
        h = c_void_p()
        check(lib().revel_posix_writable_file_new(path.encode(), ctypes.byref(h)))
        super().__init__(h.value, False)


class SequentialFile:
    """``trait SequentialFile`` (env.rs:52-57).  Ownership moves to a Reader."""

    def __init__(self, handle: int):
        self._h = handle

    def read(self, n: int) -> bytes:
        buf = ctypes.create_string_buffer(n)
        got = c_size_t()
        check(lib().revel_sequential_file_read(self._h, buf, n, ctypes.byref(got)))
        return buf.raw[:got.value]

    def skip(self, n: int) -> None:
        check(lib().revel_sequential_file_skip(self._h, n))

    def take(self) -> int:
        h, self._h = self._h, None
        if not h:
            raise ValueError("sequential file already consumed")
        return h

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().revel_sequential_file_free(self._h)
            except Exception:
                pass
            self._h = None


class MemorySequentialFile(SequentialFile):
    """env.rs:232-266 (copies ``data``)."""

    def __init__(self, data: bytes):
        super().__init__(lib().revel_memory_sequential_file_new(data, len(data)))


class PosixSequentialFile(SequentialFile):
    """Posix sequential file (the reference has no constructor, env.rs:153-158)."""

    def __init__(self, path: str):
        h = c_void_p()
        check(lib().revel_posix_sequential_file_new(path.encode(), ctypes.byref(h)))
        super().__init__(h.value)
