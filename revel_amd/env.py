"""File abstractions of src/env.rs:25-266, via the C-ABI."""
from __future__ import annotations

import ctypes
from ctypes import c_size_t, c_void_p

from ._lib import (APPEND_FN, FILE_OP_FN, INVALID_ARGUMENT, IO_ERROR, READ_FN, RELEASE_FN, SKIP_FN, OK, RevelError,
                   check, lib)

# Objects handed to the library as a callback file's `user`, keyed by the
# integer passed as user: the library's release callback drops the entry,
# as dropping the Box / Rc clone does in the Rust binding.
_owned: dict = {}
_next_key = [1]


def _own(obj) -> int:
    k = _next_key[0]
    _next_key[0] += 1
    _owned[k] = obj
    return k


def _status(fn, *args) -> int:
    """Run a Python file method for the library: Ok -> 0, RevelError -> its
    code, any other exception -> IOError (error.rs:25-29 maps io::Error)."""
    try:
        fn(*args)
        return OK
    except RevelError as e:
        return e.code
    except Exception:
        return IO_ERROR


@RELEASE_FN
def _release(user):
    _owned.pop(user, None)


@APPEND_FN
def _cb_append(user, data, n):
    obj = _owned[user]
    return _status(obj.append, ctypes.string_at(data, n) if n else b"")


@FILE_OP_FN
def _cb_flush(user):
    return _status(_owned[user].flush)


@FILE_OP_FN
def _cb_close(user):
    return _status(_owned[user].close)


@FILE_OP_FN
def _cb_sync(user):
    return _status(_owned[user].sync)


@READ_FN
def _cb_read(user, scratch, n, got):
    try:
        data = _owned[user].read(n)
        if len(data) > n:
            return INVALID_ARGUMENT
        ctypes.memmove(scratch, data, len(data))
        got[0] = len(data)
        return OK
    except RevelError as e:
        return e.code
    except Exception:
        return IO_ERROR


@SKIP_FN
def _cb_skip(user, n):
    return _status(_owned[user].skip, n)


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


class CallbackWritableFile(WritableFile):
    """A caller-implemented ``dyn WritableFile`` (env.rs:40-50) behind the
    C-ABI: ``obj`` provides ``append(bytes)``, ``flush()``, ``close()`` and
    ``sync()``; raising :class:`RevelError` returns its code to the writer,
    any other exception IOError."""

    def __init__(self, obj):
        h = c_void_p()
        key = _own(obj)
        rc = lib().revel_writable_file_from_callbacks(key, _cb_append, _cb_flush, _cb_close, _cb_sync, _release,
                                                      ctypes.byref(h))
        if rc != OK:
            _owned.pop(key, None)
            check(rc)
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


class CallbackSequentialFile(SequentialFile):
    """A caller-implemented ``Box<dyn SequentialFile>`` (env.rs:52-57):
    ``obj.read(n) -> bytes`` (up to n bytes, b"" at end of file) and
    ``obj.skip(n)`` (relative).  Ownership moves to the Reader it is given to."""

    def __init__(self, obj, skip: bool = True):
        h = c_void_p()
        key = _own(obj)
        rc = lib().revel_sequential_file_from_callbacks(key, _cb_read, _cb_skip if skip else SKIP_FN(),
                                                        _release, ctypes.byref(h))
        if rc != OK:
            _owned.pop(key, None)
            check(rc)
        super().__init__(h.value)
