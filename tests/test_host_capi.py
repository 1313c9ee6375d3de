"""The C-ABI library on the CPU: symbol surface, host CRC, writer, files and
the checksum=False reader, all against the oracle and the golden fixtures.
No compute is sent to a GPU here."""
import hashlib
import os
import re

import numpy as np
import pytest

import revel_amd
from revel_amd import _lib, crc, env, gpu, log
from revel_amd._lib import RevelError
from conftest import ROOT, golden_image
from oracle import crc32c_oracle as po
from oracle import oracle_c as oc


def header_symbols():
    with open(os.path.join(ROOT, "include", "revel_wal.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(revel_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = revel_amd.lib()
    syms = header_symbols()
    assert len(syms) >= 45
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_integration_rust_binding_matches_header():
    """INTEGRATION.md's Rust extern blocks (section 2 + 2b) declare every
    function of include/revel_wal.h exactly once, with the header's argument
    count (the binding a Revel maintainer would compile)."""
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    rust = dict(re.findall(r"pub fn (revel_\w+)\s*\(([^)]*)\)", doc))
    names = re.findall(r"pub fn (revel_\w+)\s*\(", doc)
    assert len(names) == len(set(names)), "a function is bound twice"
    with open(os.path.join(ROOT, "include", "revel_wal.h")) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    protos = dict(re.findall(r"\b(revel_[a-z0-9_]+)\s*\(([^;{)]*(?:\([^)]*\)[^;{)]*)*)\)\s*;", text))
    assert set(rust) == set(protos), set(rust) ^ set(protos)
    for name, cargs in protos.items():
        n_c = 0 if cargs.strip() in ("", "void") else cargs.count(",") + 1
        n_r = 0 if not rust[name].strip() else rust[name].count(",") + 1
        assert n_c == n_r, (name, cargs, rust[name])


def test_gpu_entry_points_fail_loudly_without_device():
    if gpu.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RevelError) as e:
        gpu.GpuContext(0)
    assert e.value.code == _lib.NOT_SUPPORT
    # checksum verification needs the GPU: no silent CPU fallback
    f = env.MemorySequentialFile(b"")
    with pytest.raises(RevelError) as e:
        log.Reader(f, checksum=True)
    assert e.value.code == _lib.NOT_SUPPORT


def test_host_crc_matches_oracle_and_kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        kat = json.load(f)
    for v in kat["value"]:
        assert crc.value(bytes.fromhex(v["data_hex"])) == v["crc"]
    assert crc.value(b"hello world") == crc.extend(ord("h"), b"ello world")
    rng = np.random.default_rng(3)
    for n in [0, 1, 5, 8, 9, 63, 64, 65, 777, 32761, 100000]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert crc.value(d) == oc.value(d)
        assert crc.extend(n & 0xFF, d) == oc.extend(n & 0xFF, d)
        c = crc.value(d)
        assert crc.mask(c) == po.mask(c) and crc.unmask(crc.mask(c)) == c


def write_mem(records, block_offset=0):
    f = env.MemoryWritableFile()
    w = log.Writer(f, block_offset)
    for r in records:
        w.add_record(r)
    return f.contents()


def test_writer_hello_world_golden():
    assert write_mem([b"hello world"]) == golden_image("hello_world")


def test_writer_matches_every_golden_edge(golden_index):
    from tests_gen import edge_records
    for name, ent in golden_index.items():
        recs = edge_records(name)
        img = write_mem(recs, ent["block_offset"])
        if ent["post"] is None:
            assert hashlib.sha256(img).hexdigest() == ent["sha256"], name
        else:
            assert img == po.write_image(recs, ent["block_offset"]), name


def test_writer_random_vs_oracle():
    rng = np.random.default_rng(4)
    for trial in range(5):
        sizes = rng.integers(0, 80000, 30)
        recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
        boff = int(rng.integers(0, 32768))
        assert write_mem(recs, boff) == oc.write_image(recs, boff)


def test_writer_c1_golden_digest():
    z = np.load(os.path.join(ROOT, "tests", "golden", "c1_records.npz"))
    words = po.splitmix64_np(np.uint64(0x5EED0001) ^ np.arange(10000, dtype=np.uint64), 512)
    img = write_mem([words[i].tobytes() for i in range(10000)])
    assert len(img) == 41038750
    assert hashlib.sha256(img).digest() == z["sha256"].tobytes()


def test_posix_files_roundtrip(tmp_path):
    path = str(tmp_path / "000001.log")
    f = env.PosixWritableFile(path)
    w = log.Writer(f)
    recs = [b"a" * 10, b"b" * 70000, b"", b"c" * 200000]
    for r in recs:
        w.add_record(r)
    f.sync()
    f.close()
    with open(path, "rb") as fh:
        data = fh.read()
    assert data == oc.write_image(recs)  # (the reference's Posix file writes zeros: App. A #4)
    s = env.PosixSequentialFile(path)
    assert s.read(7) == data[:7]
    s.skip(10)
    assert s.read(5) == data[17:22]
    rd = log.Reader(env.PosixSequentialFile(path), checksum=False)
    assert list(rd) == recs


def test_posix_missing_file_is_not_found(tmp_path):
    with pytest.raises(RevelError) as e:
        env.PosixSequentialFile(str(tmp_path / "nope.log"))
    assert e.value.code == _lib.NOT_FOUND


def test_memory_sequential_file_semantics():
    s = env.MemorySequentialFile(b"0123456789")
    assert s.read(3) == b"012"
    s.skip(2)  # relative
    assert s.read(100) == b"56789"
    assert s.read(4) == b""


def test_reader_nochecksum_all_golden(golden_index):
    for name, ent in golden_index.items():
        img = golden_image(name)
        rd = log.Reader(env.MemorySequentialFile(img), checksum=False, window_bytes=65536)
        try:
            got = list(rd)
        except RevelError:
            got = "error"
        try:
            want = po.read_all(img, checksum=False)
        except po.CorruptionError:
            want = "error"
        if want == "error":
            assert got == "error", name
        else:
            assert got == want, name


def reader_events(rd, into=None, limit=100000):
    """Every event a Reader yields until EOF, continuing after errors (the
    reader resumes after a bad record): record bytes, or ("error", code).
    into = a bytearray: read through read_record_into with that scratch."""
    out = []
    for _ in range(limit):
        try:
            r = rd.read_record() if into is None else rd.read_record_into(into)
        except RevelError as e:
            out.append(("error", e.code))
            continue
        if r is None:
            return out
        out.append(bytes(r) if into is None else bytes(into[:r]))
    raise AssertionError("reader did not reach EOF")


@pytest.mark.parametrize("start", [0, 1, 100, 1 << 20])
def test_read_record_into_caller_scratch_every_golden(golden_index, start):
    """read_record_into (log_reader.rs:76's `&mut Vec<u8>` scratch): the same
    events as read_record on every golden image, whatever the scratch's size
    to begin with (it grows by the bytes the library says it needs)."""
    for name in sorted(golden_index):
        img = golden_image(name)
        for chunk in (1 << 30, 4096):
            a = log.Reader(env.CallbackSequentialFile(PySequential(img, chunk)), checksum=False, window_bytes=65536)
            b = log.Reader(env.CallbackSequentialFile(PySequential(img, chunk)), checksum=False, window_bytes=65536)
            scratch = bytearray(start)
            assert reader_events(a, into=scratch) == reader_events(b), (name, chunk, start)


def test_read_record_into_natural_loop_grows_scratch():
    """The loop a caller writes (`while (n := rd.read_record_into(buf)) is not
    None`) with records that grow past the scratch mid-loop: the call returns
    a length, holds no view of the scratch, so growing it never fails."""
    recs = [b"a" * 3, b"b" * 50000, b"", b"c" * 70000, b"d" * 9]
    rd = log.Reader(env.MemorySequentialFile(oc.write_image(recs)), checksum=False, window_bytes=65536)
    buf = bytearray(4)
    got = []
    while (n := rd.read_record_into(buf)) is not None:
        got.append(bytes(buf[:n]))
    assert got == recs and len(buf) >= 70000


def test_read_record_into_short_buffer_keeps_the_record():
    """A short scratch returns InvalidArgument with the bytes needed and
    keeps the record for the next call (either read entry point)."""
    import ctypes
    recs = [b"x" * 10, b"y" * 70000, b"", b"z" * 5]
    img = oc.write_image(recs)
    rd = log.Reader(env.MemorySequentialFile(img), checksum=False, window_bytes=65536)
    L = revel_amd.lib()
    n, eof = ctypes.c_size_t(), ctypes.c_int()
    buf = ctypes.create_string_buffer(16)
    assert L.revel_log_reader_read_record_into(rd._h, buf, 16, ctypes.byref(n), ctypes.byref(eof)) == _lib.OK
    assert (n.value, eof.value, buf.raw[:10]) == (10, 0, recs[0])
    # the 70 000-byte record spans three blocks: too long for 16 bytes, twice
    for _ in range(2):
        assert L.revel_log_reader_read_record_into(rd._h, buf, 16, ctypes.byref(n), ctypes.byref(eof)) == \
            _lib.INVALID_ARGUMENT
        assert n.value == 70000
    assert rd.read_record() == recs[1]  # the kept record, through the other entry point
    assert L.revel_log_reader_read_record_into(rd._h, buf, 16, ctypes.byref(n), ctypes.byref(eof)) == _lib.OK
    assert (n.value, eof.value) == (0, 0)  # the empty record: not EOF
    assert L.revel_log_reader_read_record_into(rd._h, buf, 0, ctypes.byref(n), None) == _lib.INVALID_ARGUMENT
    assert n.value == 5
    assert L.revel_log_reader_read_record_into(rd._h, buf, 16, ctypes.byref(n), ctypes.byref(eof)) == _lib.OK
    assert buf.raw[:5] == recs[3]
    assert L.revel_log_reader_read_record_into(rd._h, buf, 16, ctypes.byref(n), ctypes.byref(eof)) == _lib.OK
    assert (n.value, eof.value) == (0, 1)


@pytest.mark.parametrize("window", [32768, 65536, 1 << 20])
def test_reader_windows_and_fragments(window):
    rng = np.random.default_rng(5)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 150000, 40)]
    img = oc.write_image(recs)
    rd = log.Reader(env.MemorySequentialFile(img), checksum=False, window_bytes=window)
    assert list(rd) == recs


def test_reader_initial_offset():
    recs = [bytes([i]) * 20000 for i in range(10)]
    img = oc.write_image(recs)
    for off in [0, 1, 20007, 32768, 40000, 100000, len(img)]:
        rd = log.Reader(env.MemorySequentialFile(img), checksum=False, initial_offset=off)
        got = list(rd)
        want = po.read_all(img, checksum=False, initial_offset=off)
        assert got == want, off


def test_framed_size_matches_writer():
    import ctypes
    rng = np.random.default_rng(9)
    for boff in [0, 1, 7, 32760, 32762, 32768]:
        recs = [b"x" * int(s) for s in rng.integers(0, 70000, 30)] + [b""] * 5
        lens = np.array([len(r) for r in recs], dtype=np.uint64)
        n = revel_amd.lib().revel_log_framed_size(lens.ctypes.data, len(lens), boff)
        assert n == len(po.write_image(recs, boff))


def test_property_writer_and_host_reader_vs_oracle():
    """Hypothesis (CPU): product writer at random block offsets == C oracle
    writer; host-walk reader (checksum off) == oracle LogReader under bit
    flips, truncation and initial offsets."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as hs
    edge = hs.sampled_from([0, 1, 6, 7, 8, 32754, 32755, 32760, 32761, 32762, 65522])
    size = hs.one_of(edge, hs.integers(0, 70000))

    def drain(read_record):
        out = []
        for _ in range(100000):
            try:
                r = read_record()
            except (RevelError, po.CorruptionError):
                out.append("E")
                continue
            if r is None:
                return out
            out.append(r)
        raise AssertionError("no EOF")

    @settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
    @given(sizes=hs.lists(size, max_size=20), seed=hs.integers(0, 2**32 - 1), boff=hs.integers(0, 32768),
           flip=hs.booleans(), cut=hs.integers(0, 40), off=hs.integers(0, 150000),
           window=hs.sampled_from([32768, 65536, 1 << 20]))
    def prop(sizes, seed, boff, flip, cut, off, window):
        rng = np.random.default_rng(seed)
        recs = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
        assert write_mem(recs, boff) == oc.write_image(recs, boff)
        img = bytearray(oc.write_image(recs))
        if flip and img:
            img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
        if cut and len(img) > cut:
            img = img[:len(img) - cut]
        img = bytes(img)
        off = min(off, len(img))
        rd = log.Reader(env.MemorySequentialFile(img), checksum=False, initial_offset=off, window_bytes=window)
        assert drain(rd.read_record) == drain(po.LogReader(img, False, off).read_record)

    prop()


# ---- caller-implemented files (the drop-in for dyn WritableFile / SequentialFile) ----

class PyWritable:
    """A caller's `dyn WritableFile` (env.rs:40-50), kept by the caller (the
    Rc<RefCell<..>> clone db.rs:56-63 holds to sync the log)."""

    def __init__(self, fail_after=None):
        self.data = bytearray()
        self.calls = []
        self.fail_after = fail_after

    def append(self, d):
        if self.fail_after is not None and len(self.data) + len(d) > self.fail_after:
            raise OSError("disk full")
        self.data += d
        self.calls.append("append")

    def flush(self):
        self.calls.append("flush")

    def close(self):
        self.calls.append("close")

    def sync(self):
        self.calls.append("sync")


class PySequential:
    """A caller's `Box<dyn SequentialFile>` (env.rs:52-57) returning short
    reads of at most `chunk` bytes."""

    def __init__(self, data, chunk=1 << 30):
        self.data, self.pos, self.chunk = data, 0, chunk

    def read(self, n):
        d = self.data[self.pos:self.pos + min(n, self.chunk)]
        self.pos += len(d)
        return d

    def skip(self, n):
        self.pos += n


def test_callback_writer_reproduces_every_golden_image(golden_index):
    from tests_gen import edge_records
    for name, ent in golden_index.items():
        recs = edge_records(name)
        f = PyWritable()
        w = log.Writer(env.CallbackWritableFile(f), ent["block_offset"])
        for r in recs:
            w.add_record(r)
        if ent["post"] is None:
            assert hashlib.sha256(bytes(f.data)).hexdigest() == ent["sha256"], name
        else:
            assert bytes(f.data) == po.write_image(recs, ent["block_offset"]), name
    # hello world (log_reader.rs:231): header, payload, flush per record (log_writer.rs:114-119)
    f = PyWritable()
    w = log.Writer(env.CallbackWritableFile(f))
    w.add_record(b"hello world")
    assert bytes(f.data) == golden_image("hello_world")
    assert f.calls == ["append", "append", "flush"]


def test_callback_writer_shared_file_sync_and_errors():
    f = PyWritable(fail_after=100)
    wf = env.CallbackWritableFile(f)
    w = log.Writer(wf)
    w.add_record(b"x" * 50)
    wf.sync()  # the DB's own clone syncs the shared file (db.rs:109-111)
    assert f.calls[-1] == "sync"
    with pytest.raises(RevelError) as e:
        w.add_record(b"y" * 100)  # append raises OSError -> io::Error -> IOError (error.rs:25-29)
    assert e.value.code == _lib.IO_ERROR
    wf.close()
    assert f.calls[-1] == "close"


class ScriptedFailFile:
    """A `dyn WritableFile` whose n-th call of one kind fails once: kind
    "append" counts every append (trailers, headers and payloads alike),
    "flush" every flush.  Used identically by the library's writer (through
    callbacks) and by the oracle writer, which restates the reference's `?`
    early returns (log_writer.rs:70, :114-121)."""

    def __init__(self, kind, n):
        self.kind, self.n = kind, n
        self.counts = {"append": 0, "flush": 0}
        self.data = bytearray()

    def _tick(self, kind):
        self.counts[kind] += 1
        if kind == self.kind and self.counts[kind] == self.n:
            raise OSError(f"{kind} #{self.n} fails")

    def append(self, d):
        self._tick("append")
        self.data += d

    def flush(self):
        self._tick("flush")

    def sync(self):
        pass

    def close(self):
        pass


@pytest.mark.parametrize("start", [0, 32761, 32766, 100])
@pytest.mark.parametrize("kind,n", [("append", k) for k in range(1, 12)] + [("flush", k) for k in range(1, 6)])
def test_writer_error_path_state_matches_reference(kind, n, start):
    """A failed add_record leaves the bytes written before the failing call and
    the block_offset of that point (log_writer.rs:114-121 advance it only after
    header append, payload append and flush all succeed; a failed trailer append
    keeps it too, :66-71); a retry then frames from there.  The failure hits
    the trailer (start 32766: a 2-byte trailer), a header, a payload or a flush
    of a FIRST/MIDDLE/LAST split or of FULL records."""
    recs = [b"a" * 40000, b"b" * 10, b"", b"c" * 70000, b"d" * 5]
    mine_f, ref_f = ScriptedFailFile(kind, n), ScriptedFailFile(kind, n)
    w = log.Writer(env.CallbackWritableFile(mine_f), start)
    ow = po.LogWriter(block_offset=start, file=ref_f)
    for r in recs:
        for attempt in range(2):  # the record that fails is retried once
            try:
                ow.add_record(r)
                ref_err = None
            except OSError as e:
                ref_err = e
            try:
                w.add_record(r)
                my_err = None
            except RevelError as e:
                my_err = e
            assert (ref_err is None) == (my_err is None), (kind, n, start, r[:1], attempt)
            if my_err is not None:
                assert my_err.code == _lib.IO_ERROR  # io::Error -> IOError (error.rs:25-29)
            assert w.block_offset == ow.block_offset, (kind, n, start, r[:1], attempt)
            assert bytes(mine_f.data) == bytes(ref_f.data), (kind, n, start, r[:1], attempt)
            if ref_err is None:
                break
    assert mine_f.counts == ref_f.counts


def test_callback_writer_release_and_required_append():
    import ctypes
    L = revel_amd.lib()
    h = ctypes.c_void_p()
    rc = L.revel_writable_file_from_callbacks(None, _lib.APPEND_FN(), _lib.FILE_OP_FN(), _lib.FILE_OP_FN(),
                                              _lib.FILE_OP_FN(), _lib.RELEASE_FN(), ctypes.byref(h))
    assert rc == _lib.INVALID_ARGUMENT and not h.value
    before = len(env._owned)
    f = env.CallbackWritableFile(PyWritable())
    assert len(env._owned) == before + 1
    f.free()  # release drops the caller's object (the Rc clone)
    assert len(env._owned) == before


@pytest.mark.parametrize("chunk", [1, 7, 4096, 1 << 30])
def test_callback_reader_nochecksum_short_reads(chunk):
    rng = np.random.default_rng(11)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 90000, 12)]
    img = oc.write_image(recs)
    before = len(env._owned)
    rd = log.Reader(env.CallbackSequentialFile(PySequential(img, chunk)), checksum=False, window_bytes=65536)
    assert list(rd) == recs
    del rd  # the reader owns the file: releasing it drops the caller's object
    assert len(env._owned) == before


def test_callback_reader_initial_offset_with_and_without_skip():
    recs = [bytes([i]) * 20000 for i in range(10)]
    img = oc.write_image(recs)
    for off in [0, 20007, 40000, len(img)]:
        want = po.read_all(img, checksum=False, initial_offset=off)
        for skip in (True, False):
            rd = log.Reader(env.CallbackSequentialFile(PySequential(img, 5000), skip=skip), checksum=False,
                            initial_offset=off)
            assert list(rd) == want, (off, skip)


def test_callback_reader_read_error_is_ioerror():
    class Broken(PySequential):
        def read(self, n):
            raise OSError("EIO")
    rd = log.Reader(env.CallbackSequentialFile(Broken(b"")), checksum=False)
    with pytest.raises(RevelError) as e:
        rd.read_record()
    assert e.value.code == _lib.IO_ERROR


def test_three_arg_reader_fails_loudly_without_gpu():
    """Reader::new(file, checksum=true, 0) with no context: the thread's
    default context needs a gfx950 device -- NOT_SUPPORT, no CPU fallback."""
    if gpu.device_count() > 0:
        pytest.skip("a GPU is visible")
    before = len(env._owned)
    with pytest.raises(RevelError) as e:
        log.Reader(env.CallbackSequentialFile(PySequential(golden_image("hello_world"))), True, 0)
    assert e.value.code == _lib.NOT_SUPPORT
    assert len(env._owned) == before  # the file was consumed and released
