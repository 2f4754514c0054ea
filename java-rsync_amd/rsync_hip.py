"""rsync_hip.py -- Python host binding of librsynchip.so (the C-ABI in include/rsync_hip.h).

Mirrors the reference's hot-path surface (paths relative to core/src/main/java/com/github/java/rsync/internal/):

  Generator.getBlockLengthFor / getDigestLength   session/Generator.java:198-212  -> block_length_for, digest_length_for
  Checksum.Header(3-arg) / (4-arg)                session/Checksum.java:75-113    -> Header.make, Header.validate
  Generator.sendItemizeAndChecksums (hot loop)    session/Generator.java:866-909  -> Context.block_sums
  Sender.sendMatchesAndData / skipMatchSendData   session/Sender.java:1235-1399   -> Context.match_scan
  Sender channel bytes (sendDataFrom / putInt)    session/Sender.java:794-809     -> tokens
  a file larger than one JVM buffer (FileView)    io/FileView.java:235-278        -> Context.*_pieces

Errors raise the Python analogue of the reference's exception (ValueError ~ IllegalArgumentException,
ProtocolError ~ RsyncProtocolException, OverflowError ~ Checksum.ChunkOverflow).  There is no CPU
fallback: without a gfx950 device Context() raises DeviceError.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RSH_LIB") or os.path.join(HERE, "lib", "librsynchip.so")  # RSH_LIB: A/B builds

RSH_OK, RSH_E_INVAL, RSH_E_PROTOCOL, RSH_E_OVERFLOW, RSH_E_NOSPACE, RSH_E_DEVICE, RSH_E_NOMEM, RSH_E_BUSY = \
    0, -1, -2, -3, -4, -5, -6, -7
RSH_E_NOTFOUND, RSH_E_OPEN = -8, -9
EV_LITERAL, EV_MATCH = 1, 2


class ProtocolError(Exception):
    """RsyncProtocolException (Connection.receiveChecksumHeader, Connection.java:28-38)."""


class FileViewNotFound(FileNotFoundError):
    """RSH_E_NOTFOUND (io/FileViewNotFound: new FileView on a missing file, FileView.java:74-75)."""


class FileViewOpenFailed(OSError):
    """RSH_E_OPEN (io/FileViewOpenFailed, FileView.java:76-78)."""


class ContextBusyError(RuntimeError):
    """RSH_E_BUSY: a Context was called from two threads at once (use one Context per thread)."""


class DeviceError(RuntimeError):
    """HIP failure or no gfx950 device."""


class Header(ctypes.Structure):
    _fields_ = [("chunk_count", ctypes.c_int32), ("block_length", ctypes.c_int32),
                ("digest_length", ctypes.c_int32), ("remainder", ctypes.c_int32)]

    def as_dict(self):
        return dict(chunk_count=self.chunk_count, block_length=self.block_length,
                    digest_length=self.digest_length, remainder=self.remainder)

    def smallest_chunk_size(self):  # Checksum.java:131-137
        return self.remainder if self.remainder > 0 else self.block_length


class Event(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("length", ctypes.c_int64), ("kind", ctypes.c_int32),
                ("index", ctypes.c_int32), ("count", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class ScanStats(ctypes.Structure):
    _fields_ = [("chain_matches", ctypes.c_int64), ("events", ctypes.c_int64), ("probe_launches", ctypes.c_int64),
                ("host_md5_windows", ctypes.c_int64), ("flushes", ctypes.c_int64),
                ("device_ms", ctypes.c_double), ("resolver_ms", ctypes.c_double), ("table_ms", ctypes.c_double),
                ("head_steps", ctypes.c_int64), ("speculation_aborted", ctypes.c_int64),
                ("device_bytes", ctypes.c_int64), ("phase_launches", ctypes.c_int64),
                ("phase_matches", ctypes.c_int64), ("spec_kernel_ms", ctypes.c_double),
                ("phase_kernel_ms", ctypes.c_double), ("phase_guesses", ctypes.c_int64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class BlockJob(ctypes.Structure):
    """rsh_block_job: one basis file of a batched Generator pass (device pointers)."""
    _fields_ = [("d_data", ctypes.c_void_p), ("n", ctypes.c_int64), ("h", Header), ("d_weak", ctypes.c_void_p),
                ("d_strong", ctypes.c_void_p)]


class ScanJob(ctypes.Structure):
    """rsh_scan_job: one source file of a batched Sender scan (device pointers; ev is host memory)."""
    _fields_ = [("d_src", ctypes.c_void_p), ("n", ctypes.c_int64), ("h", Header), ("d_weak", ctypes.c_void_p),
                ("d_strong", ctypes.c_void_p), ("ev", ctypes.c_void_p), ("ev_cap", ctypes.c_int64),
                ("n_ev", ctypes.c_int64), ("literal", ctypes.c_int64), ("matched", ctypes.c_int64),
                ("status", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class CombineResult(ctypes.Structure):
    """rsh_combine_result (Receiver.combineDataToFile outcome)."""
    _fields_ = [("tokens_used", ctypes.c_int64), ("target_len", ctypes.c_int64), ("literal", ctypes.c_int64),
                ("matched", ctypes.c_int64), ("intact", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("md5", ctypes.c_uint8 * 16)]


class Piece(ctypes.Structure):
    """rsh_piece: one host buffer of a file handed over in pieces (rsh_*_pieces)."""
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_int64)]


class CombineJob(ctypes.Structure):
    """rsh_combine_job: one file of a segment's Receiver pass (rsh_receiver_combine_batch)."""
    _fields_ = [("tokens", ctypes.c_void_p), ("tokens_len", ctypes.c_int64), ("h", Header),
                ("replica", ctypes.POINTER(Piece)), ("nreplica", ctypes.c_int32), ("defer_write", ctypes.c_int32),
                ("target", ctypes.c_void_p), ("target_cap", ctypes.c_int64), ("status", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("res", CombineResult)]


class BlockBatchJob(ctypes.Structure):
    """rsh_block_batch_job: one basis file of a segment's Generator pass from host memory (rsh_block_sums_batch)."""
    _fields_ = [("pieces", ctypes.POINTER(Piece)), ("npieces", ctypes.c_int32), ("status", ctypes.c_int32),
                ("h", Header), ("weak_out", ctypes.c_void_p), ("strong_out", ctypes.c_void_p)]


class ScanBatchJob(ctypes.Structure):
    """rsh_scan_batch_job: one source file of a segment's Sender pass from host memory (rsh_match_scan_batch)."""
    _fields_ = [("pieces", ctypes.POINTER(Piece)), ("npieces", ctypes.c_int32), ("status", ctypes.c_int32),
                ("h", Header), ("weak", ctypes.c_void_p), ("strong", ctypes.c_void_p), ("ev", ctypes.c_void_p),
                ("ev_cap", ctypes.c_int64), ("n_ev", ctypes.c_int64), ("literal", ctypes.c_int64),
                ("matched", ctypes.c_int64), ("file_md5", ctypes.c_uint8 * 16)]


class Md5Job(ctypes.Structure):
    """rsh_md5_job: one file of rsh_file_md5_batch."""
    _fields_ = [("pieces", ctypes.POINTER(Piece)), ("npieces", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("md5", ctypes.c_uint8 * 16)]


EVENT_DTYPE = np.dtype([("offset", "<i8"), ("length", "<i8"), ("kind", "<i4"), ("index", "<i4"),
                        ("count", "<i4"), ("reserved", "<i4")])

# every symbol include/rsync_hip.h declares
EXPORTS = ["rsh_abi_version", "rsh_strerror", "rsh_last_error", "rsh_device_count", "rsh_ctx_create", "rsh_ctx_destroy",
           "rsh_ctx_stream", "rsh_block_length_for", "rsh_digest_length_for", "rsh_header_make",
           "rsh_header_validate", "rsh_block_sums", "rsh_block_sums_device", "rsh_ctx_sync", "rsh_ctx_trim", "rsh_match_scan",
           "rsh_match_scan_device", "rsh_match_scan_tiled", "rsh_fetch_events", "rsh_file_md5", "rsh_tokens_size", "rsh_tokens_write", "rsh_generator_bytes",
           "rsh_block_sums_batch_device", "rsh_match_scan_batch_device", "rsh_receiver_combine",
           "rsh_receiver_combine_device", "rsh_receiver_combine_batch", "rsh_block_sums_file", "rsh_match_scan_file", "rsh_block_sums_pieces", "rsh_match_scan_pieces", "rsh_block_sums_batch", "rsh_match_scan_batch", "rsh_block_sums_batch_multi", "rsh_match_scan_batch_multi", "rsh_receiver_combine_batch_multi", "rsh_shard_files", "rsh_file_md5_batch", "rsh_dev_alloc", "rsh_dev_free", "rsh_memcpy_h2d", "rsh_memcpy_d2h", "rsh_fill_splitmix_device"]
# include/rsync_hip_debug.h (testing / diagnostics ABI)
DEBUG_EXPORTS = ["rsh_debug_set_option", "rsh_debug_get_option", "rsh_debug_reset_options", "rsh_debug_k1_clock",
                 "rsh_debug_streams_busy", "rsh_debug_kernel_ms", "rsh_debug_multi_selftest", "rsh_debug_generation"]

_LIB = None


def build(force=False):
    """Compile librsynchip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-s", "-C", HERE] + (["-B"] if force else [])
    subprocess.run(cmd, check=True)


def stale_sources():
    """Sources that changed since the loaded library was built (the build's sha256 stamp next to it,
    lib/librsynchip.srchash or lib/diag/librsynchip.srchash): a stale library must never be the one a test or the
    bench measures.  [] when the stamp or the sources are absent (a binary-only install)."""
    import hashlib
    stamp = os.path.splitext(LIB_PATH)[0] + ".srchash"
    if not os.path.exists(stamp):
        return []
    out = []
    for line in open(stamp):
        digest, _, rel = line.strip().partition("  ")
        path = os.path.join(HERE, rel)
        if os.path.exists(path) and hashlib.sha256(open(path, "rb").read()).hexdigest() != digest:
            out.append(rel)
    return out


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise DeviceError(f"{LIB_PATH} missing: run rsync_hip.build() (or __graft_entry__.build())")
    stale = stale_sources()
    if stale:
        raise DeviceError(f"{LIB_PATH} was built from other sources than {', '.join(stale)}: rebuild it")
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    HP = ctypes.POINTER(Header)
    sig = {
        "rsh_abi_version": ([], ctypes.c_int),
        "rsh_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "rsh_last_error": ([], ctypes.c_char_p),
        "rsh_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "rsh_ctx_create": ([ctypes.c_int, ctypes.POINTER(P)], ctypes.c_int),
        "rsh_ctx_destroy": ([P], None),
        "rsh_ctx_stream": ([P], P),
        "rsh_block_length_for": ([I64], I32),
        "rsh_digest_length_for": ([I64, I32, I32], I32),
        "rsh_header_make": ([I32, I32, I64, HP], ctypes.c_int),
        "rsh_header_validate": ([HP], ctypes.c_int),
        "rsh_block_sums": ([P, P, I64, HP, P, P, P], ctypes.c_int),
        "rsh_block_sums_device": ([P, P, I64, HP, P, P, P], ctypes.c_int),
        "rsh_ctx_sync": ([P], ctypes.c_int),
        "rsh_ctx_trim": ([P], ctypes.c_int),
        "rsh_match_scan": ([P, P, I64, HP, P, P, P, P, I64, ctypes.POINTER(I64), P, ctypes.POINTER(I64),
                            ctypes.POINTER(I64), ctypes.POINTER(ScanStats)], ctypes.c_int),
        "rsh_match_scan_device": ([P, P, I64, HP, P, P, P, P, I64, ctypes.POINTER(I64), ctypes.POINTER(I64),
                                   ctypes.POINTER(I64), ctypes.POINTER(ScanStats)], ctypes.c_int),
        "rsh_match_scan_tiled": ([P, P, I64, HP, P, P, P, I64, P, I64, ctypes.POINTER(I64), P, ctypes.POINTER(I64),
                                  ctypes.POINTER(I64), ctypes.POINTER(ScanStats)], ctypes.c_int),
        "rsh_fetch_events": ([P, P, I64, ctypes.POINTER(I64)], ctypes.c_int),
        "rsh_file_md5": ([P, I64, P], ctypes.c_int),
        "rsh_tokens_size": ([P, I64], I64),
        "rsh_tokens_write": ([P, P, I64, P, P, I64], ctypes.c_int),
        "rsh_generator_bytes": ([HP, P, P, P, I64], I64),
        "rsh_block_sums_batch_device": ([P, ctypes.POINTER(BlockJob), I32, P], ctypes.c_int),
        "rsh_match_scan_batch_device": ([P, ctypes.POINTER(ScanJob), I32, P, ctypes.POINTER(ScanStats)],
                                        ctypes.c_int),
        "rsh_receiver_combine": ([P, P, I64, HP, P, I64, I32, P, I64, ctypes.POINTER(CombineResult)], ctypes.c_int),
        "rsh_receiver_combine_batch": ([P, ctypes.POINTER(CombineJob), I32], ctypes.c_int),
        "rsh_receiver_combine_device": ([P, P, I64, HP, P, I64, I32, P, I64, ctypes.POINTER(CombineResult)],
                                        ctypes.c_int),
        "rsh_block_sums_file": ([P, ctypes.c_char_p, I64, HP, P, P, P, ctypes.POINTER(I32)], ctypes.c_int),
        "rsh_match_scan_file": ([P, ctypes.c_char_p, I64, HP, P, P, P, P, I64, ctypes.POINTER(I64), P,
                                 ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(ScanStats),
                                 ctypes.POINTER(I32)], ctypes.c_int),
        "rsh_block_sums_pieces": ([P, ctypes.POINTER(Piece), I32, HP, P, P, P], ctypes.c_int),
        "rsh_match_scan_pieces": ([P, ctypes.POINTER(Piece), I32, HP, P, P, P, P, I64, ctypes.POINTER(I64), P,
                                   ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(ScanStats)], ctypes.c_int),
        "rsh_block_sums_batch": ([P, ctypes.POINTER(BlockBatchJob), I32, P], ctypes.c_int),
        "rsh_match_scan_batch": ([P, ctypes.POINTER(ScanBatchJob), I32, P, ctypes.POINTER(ScanStats)], ctypes.c_int),
        "rsh_block_sums_batch_multi": ([ctypes.POINTER(P), I32, ctypes.POINTER(BlockBatchJob), I32, P], ctypes.c_int),
        "rsh_match_scan_batch_multi": ([ctypes.POINTER(P), I32, ctypes.POINTER(ScanBatchJob), I32, P,
                                        ctypes.POINTER(ScanStats)], ctypes.c_int),
        "rsh_receiver_combine_batch_multi": ([ctypes.POINTER(P), I32, ctypes.POINTER(CombineJob), I32], ctypes.c_int),
        "rsh_shard_files": ([P, I32, I32, P], ctypes.c_int),
        "rsh_file_md5_batch": ([ctypes.POINTER(Md5Job), I32, I32], ctypes.c_int),
        "rsh_dev_alloc": ([P, I64, ctypes.POINTER(P)], ctypes.c_int),
        "rsh_dev_free": ([P, P], ctypes.c_int),
        "rsh_memcpy_h2d": ([P, P, P, I64], ctypes.c_int),
        "rsh_memcpy_d2h": ([P, P, P, I64], ctypes.c_int),
        "rsh_fill_splitmix_device": ([P, P, I64, ctypes.c_uint64, I64], ctypes.c_int),
        "rsh_debug_set_option": ([ctypes.c_char_p, I64], ctypes.c_int),
        "rsh_debug_get_option": ([ctypes.c_char_p, ctypes.POINTER(I64)], ctypes.c_int),
        "rsh_debug_reset_options": ([], None),
        "rsh_debug_k1_clock": ([P, P, I64, I32, I32, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "rsh_debug_streams_busy": ([P, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
        "rsh_debug_generation": ([P, I32, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
        "rsh_debug_kernel_ms": ([P, I32, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "rsh_debug_multi_selftest": ([P, I32, I32, I32, P, P, P], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _LIB = L
    return L


def _check(rc):
    if rc == RSH_OK:
        return
    msg = lib().rsh_strerror(rc).decode()
    if rc == RSH_E_INVAL:
        raise ValueError(msg)
    if rc == RSH_E_PROTOCOL:
        raise ProtocolError(msg)
    if rc == RSH_E_OVERFLOW:
        raise OverflowError(msg)
    if rc == RSH_E_NOMEM:
        raise MemoryError(msg)
    if rc == RSH_E_BUSY:
        raise ContextBusyError(msg)
    if rc == RSH_E_NOTFOUND:
        raise FileViewNotFound(msg)
    if rc == RSH_E_OPEN:
        raise FileViewOpenFailed(msg)
    detail = lib().rsh_last_error().decode()
    raise DeviceError(f"{msg}: {detail}" if detail else msg)


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _u8(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.view(np.uint8).reshape(-1))
    return np.frombuffer(bytes(data), dtype=np.uint8)


def block_length_for(n):
    return lib().rsh_block_length_for(n)


def digest_length_for(n, blen, min_digest=2):
    return lib().rsh_digest_length_for(n, blen, min_digest)


def header_make(blen, dlen, n):
    h = Header()
    _check(lib().rsh_header_make(blen, dlen, n, ctypes.byref(h)))
    return h


def header_validate(h):
    _check(lib().rsh_header_validate(ctypes.byref(h)))


def file_md5(data):
    a = _u8(data)
    out = np.zeros(16, np.uint8)
    _check(lib().rsh_file_md5(_ptr(a), a.size, _ptr(out)))
    return out.tobytes()


def _piece_list(pieces):
    arrs = [_u8(p) for p in pieces]
    pl = (Piece * max(len(arrs), 1))()
    for i, a in enumerate(arrs):
        pl[i].data, pl[i].len = (a.ctypes.data if a.size else None), a.size
    return arrs, pl, sum(a.size for a in arrs)


def file_md5_batch(files, threads=0):
    """Whole-file MD5 of each file (a list of pieces each; rsh_file_md5_batch): several files per core."""
    keep, jobs = [], (Md5Job * max(len(files), 1))()
    for i, pieces in enumerate(files):
        arrs, pl, _ = _piece_list(pieces)
        keep.append((arrs, pl))
        jobs[i].pieces, jobs[i].npieces = ctypes.cast(pl, ctypes.POINTER(Piece)), len(arrs)
    _check(lib().rsh_file_md5_batch(jobs, len(files), threads))
    return [bytes(jobs[i].md5) for i in range(len(files))]


def scan_event_cap(n, h):
    """An event buffer no scan of n source bytes can overflow: every MATCH consumes a window of B bytes but
    possibly the last, every LITERAL but the last precedes a MATCH or ends a 10*B flush interval."""
    if h.block_length <= 0:
        return n // 8192 + 2
    return 2 * (n // h.block_length + 1) + n // (10 * h.block_length) + 4


def events_as_tuples(ev, block_length):
    """Expand MATCH runs into one (MATCH, offset, length, index) per chunk, the oracle's granularity.
    Every window of a run is a full block except possibly the file's last one."""
    out = []
    for e in ev:
        if e["kind"] == EV_LITERAL:
            out.append((EV_LITERAL, int(e["offset"]), int(e["length"]), 0))
        else:
            off, left, cnt = int(e["offset"]), int(e["length"]), int(e["count"])
            for j in range(cnt):
                w = left if j == cnt - 1 else block_length
                out.append((EV_MATCH, off, w, int(e["index"]) + j))
                off += w
                left -= w
    return out


def tokens(src, ev, file_md5_bytes):
    a = _u8(src)
    ev = np.ascontiguousarray(ev, dtype=EVENT_DTYPE)
    n = ev.size
    size = lib().rsh_tokens_size(_ptr(ev) if n else None, n)
    out = np.zeros(size, np.uint8)
    fm = np.frombuffer(file_md5_bytes, np.uint8).copy()
    _check(lib().rsh_tokens_write(_ptr(a), _ptr(ev) if n else None, n, _ptr(fm), _ptr(out), size))
    return out.tobytes()


def set_option(name, value):
    """A library tunable or diagnostic switch (include/rsync_hip_debug.h; tests and A/B runs only)."""
    _check(lib().rsh_debug_set_option(name.encode(), int(value)))


def get_option(name):
    v = ctypes.c_int64()
    _check(lib().rsh_debug_get_option(name.encode(), ctypes.byref(v)))
    return v.value


def reset_options():
    lib().rsh_debug_reset_options()


class option:
    """Context manager: `with option("k1_gather", 0): ...` sets a switch and restores its previous value."""

    def __init__(self, name, value):
        self.name, self.value = name, value

    def __enter__(self):
        self.old = get_option(self.name)
        set_option(self.name, self.value)
        return self

    def __exit__(self, *a):
        set_option(self.name, self.old)


def device_count():
    c = ctypes.c_int(0)
    rc = lib().rsh_device_count(ctypes.byref(c))
    return c.value if rc == RSH_OK else 0


class Context:
    """One per calling thread (the reference's Generator and Sender threads each get their own)."""

    def __init__(self, device=0):
        self._p = ctypes.c_void_p()
        _check(lib().rsh_ctx_create(device, ctypes.byref(self._p)))

    def close(self):
        if self._p:
            lib().rsh_ctx_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._p

    def kernel_ms(self, which):
        """The last Generator (0) or speculation (1) K1's duration from its own dispatch events (-1: not timed)."""
        ms = ctypes.c_double(-1.0)
        _check(lib().rsh_debug_kernel_ms(self._p, which, ctypes.byref(ms)))
        return ms.value

    def generation(self, set_to=-1):
        """The context's launch generation, after setting it to set_to when >= 0 (rsh_debug_generation)."""
        g = ctypes.c_int32(0)
        _check(lib().rsh_debug_generation(self._p, set_to, ctypes.byref(g)))
        return g.value

    def streams_busy(self):
        """Bit mask of the context's streams with work still queued (rsh_debug_streams_busy)."""
        m = ctypes.c_int32(-1)
        _check(lib().rsh_debug_streams_busy(self._p, ctypes.byref(m)))
        return m.value

    def sync(self):
        _check(lib().rsh_ctx_sync(self._p))

    # the segment calls' entry points (DeviceSet: the multi-context forms)
    def _block_batch(self, jobs, n, seed):
        return lib().rsh_block_sums_batch(self._p, jobs, n, seed)

    def _scan_batch(self, jobs, n, seed, stats):
        return lib().rsh_match_scan_batch(self._p, jobs, n, seed, stats)

    def _combine_batch(self, jobs, n):
        return lib().rsh_receiver_combine_batch(self._p, jobs, n)

    def trim(self):
        """Release the pass-sized buffers (rsh_ctx_trim); the next call allocates what it needs again."""
        _check(lib().rsh_ctx_trim(self._p))

    def alloc(self, nbytes):
        """Device buffer (DeviceBuffer) owned by this context's device."""
        return DeviceBuffer(self, nbytes)

    def block_sums(self, data, h, seed):
        """Generator.sendItemizeAndChecksums hot loop: (weak int32[C], strong uint8[C*dl])."""
        a = _u8(data)
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        weak = np.zeros(max(h.chunk_count, 1), np.int32)
        strong = np.zeros(max(h.chunk_count * h.digest_length, 1), np.uint8)
        _check(lib().rsh_block_sums(self._p, _ptr(a), a.size, ctypes.byref(h), _ptr(s), _ptr(weak), _ptr(strong)))
        return weak[:h.chunk_count], strong[:h.chunk_count * h.digest_length]

    def match_scan(self, src, h, weak, strong, seed, ev_cap=None):
        """Sender.sendMatchesAndData: (events ndarray[EVENT_DTYPE], file_md5, literal, matched, stats)."""
        a = _u8(src)
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        w = np.ascontiguousarray(weak, dtype=np.int32)
        st = np.ascontiguousarray(strong, dtype=np.uint8)
        # upper estimate: one literal per flush interval plus a literal and a match run per chunk
        cap = ev_cap if ev_cap is not None else int(a.size // max(10 * h.block_length, 1) + 2 * h.chunk_count + 64)
        ev = np.zeros(max(cap, 1), EVENT_DTYPE)
        n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        fm = np.zeros(16, np.uint8)
        stats = ScanStats()
        rc = lib().rsh_match_scan(self._p, _ptr(a), a.size, ctypes.byref(h), _ptr(w) if w.size else None,
                                  _ptr(st) if st.size else None, _ptr(s), _ptr(ev), cap, ctypes.byref(n_ev),
                                  _ptr(fm), ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(stats))
        if rc == RSH_E_NOSPACE and ev_cap is None:  # the context kept them: fetch, no rescan
            ev = np.zeros(n_ev.value, EVENT_DTYPE)
            rc = lib().rsh_fetch_events(self._p, _ptr(ev), n_ev.value, ctypes.byref(n_ev))
        _check(rc)
        return ev[:n_ev.value], fm.tobytes(), lit.value, mat.value, stats.as_dict()

    def match_scan_tiled(self, src, h, weak, strong, seed, tile_bytes=0, digest=True, ev_cap=None):
        """The scan with HBM holding one tile of the source at a time (rsh_match_scan_tiled): as match_scan;
        file_md5 is None when digest is False."""
        a = _u8(src)
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        w = np.ascontiguousarray(weak, dtype=np.int32)
        st = np.ascontiguousarray(strong, dtype=np.uint8)
        cap = ev_cap if ev_cap is not None else int(a.size // max(10 * h.block_length, 1) + 2 * h.chunk_count + 64)
        ev = np.zeros(max(cap, 1), EVENT_DTYPE)
        n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        fm = np.zeros(16, np.uint8)
        stats = ScanStats()
        rc = lib().rsh_match_scan_tiled(self._p, _ptr(a), a.size, ctypes.byref(h), _ptr(w) if w.size else None,
                                        _ptr(st) if st.size else None, _ptr(s), tile_bytes, _ptr(ev), cap,
                                        ctypes.byref(n_ev), _ptr(fm) if digest else None, ctypes.byref(lit),
                                        ctypes.byref(mat), ctypes.byref(stats))
        if rc == RSH_E_NOSPACE and ev_cap is None:
            ev = np.zeros(n_ev.value, EVENT_DTYPE)
            rc = lib().rsh_fetch_events(self._p, _ptr(ev), n_ev.value, ctypes.byref(n_ev))
        _check(rc)
        return ev[:n_ev.value], (fm.tobytes() if digest else None), lit.value, mat.value, stats.as_dict()

    @staticmethod
    def _pieces(pieces):
        return _piece_list(pieces)

    def block_sums_batch(self, files, seed, statuses=None):
        """A segment's Generator pass from host memory (rsh_block_sums_batch; Generator.itemizeSegment):
        files = [(pieces, Header)] -> [(weak, strong)] per file.  statuses (a list): receives the call's code and
        every file's status instead of raising (tests of the failure paths)."""
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        jobs = (BlockBatchJob * max(len(files), 1))()
        keep, outs = [], []
        for i, (pieces, h) in enumerate(files):
            arrs, pl, _ = _piece_list(pieces)
            w = np.zeros(max(h.chunk_count, 1), np.int32)
            st = np.zeros(max(h.chunk_count * h.digest_length, 1), np.uint8)
            keep.append((arrs, pl))
            outs.append((w, st, h))
            jobs[i].pieces, jobs[i].npieces, jobs[i].h = ctypes.cast(pl, ctypes.POINTER(Piece)), len(arrs), h
            jobs[i].weak_out, jobs[i].strong_out = w.ctypes.data, st.ctypes.data
        rc = self._block_batch(jobs, len(files), _ptr(s))
        if statuses is not None:
            statuses[:] = [rc] + [jobs[i].status for i in range(len(files))]
        else:
            _check(rc)
        return [(w[:h.chunk_count], st[:h.chunk_count * h.digest_length]) for w, st, h in outs]

    def match_scan_batch(self, files, seed, ev_caps=None, statuses=None):
        """A segment's Sender pass from host memory (rsh_match_scan_batch; Sender.sendFiles):
        files = [(pieces, Header, weak, strong)] -> ([(events, file_md5, literal, matched, status)], stats).
        A file's status is RSH_E_NOSPACE when its ev_caps entry was short (its events are then not kept).
        statuses (a list): receives the call's code instead of raising."""
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        jobs = (ScanBatchJob * max(len(files), 1))()
        keep, evs = [], []
        for i, (pieces, h, weak, strong) in enumerate(files):
            arrs, pl, n = _piece_list(pieces)
            w = np.ascontiguousarray(weak, dtype=np.int32)
            st = np.ascontiguousarray(strong, dtype=np.uint8)
            cap = ev_caps[i] if ev_caps is not None else scan_event_cap(n, h)
            ev = np.zeros(max(cap, 1), EVENT_DTYPE)
            keep.append((arrs, pl, w, st))
            evs.append(ev)
            j = jobs[i]
            j.pieces, j.npieces, j.h = ctypes.cast(pl, ctypes.POINTER(Piece)), len(arrs), h
            j.weak, j.strong = (w.ctypes.data if w.size else None), (st.ctypes.data if st.size else None)
            j.ev, j.ev_cap = ev.ctypes.data, cap
        stats = ScanStats()
        rc = self._scan_batch(jobs, len(files), _ptr(s), ctypes.byref(stats))
        if statuses is not None:
            statuses[:] = [rc]
        elif rc != RSH_E_NOSPACE:
            _check(rc)
        out = []
        for i in range(len(files)):
            j = jobs[i]
            ev = evs[i][:j.n_ev] if j.status == RSH_OK else evs[i][:0]
            out.append((ev, bytes(j.file_md5), j.literal, j.matched, j.status))
        return out, stats.as_dict()

    def block_sums_pieces(self, pieces, h, seed):
        """As block_sums over the concatenation of `pieces` (host buffers; rsh_block_sums_pieces)."""
        arrs, pl, _ = self._pieces(pieces)
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        weak = np.zeros(max(h.chunk_count, 1), np.int32)
        strong = np.zeros(max(h.chunk_count * h.digest_length, 1), np.uint8)
        _check(lib().rsh_block_sums_pieces(self._p, pl, len(arrs), ctypes.byref(h), _ptr(s), _ptr(weak), _ptr(strong)))
        return weak[:h.chunk_count], strong[:h.chunk_count * h.digest_length]

    def match_scan_pieces(self, pieces, h, weak, strong, seed):
        """As match_scan over the concatenation of `pieces` (rsh_match_scan_pieces)."""
        arrs, pl, n = self._pieces(pieces)
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        w = np.ascontiguousarray(weak, dtype=np.int32)
        st = np.ascontiguousarray(strong, dtype=np.uint8)
        cap = int(n // max(10 * h.block_length, 1) + 2 * h.chunk_count + 64) if h.block_length else n // 8192 + 2
        ev = np.zeros(max(cap, 1), EVENT_DTYPE)
        n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        fm = np.zeros(16, np.uint8)
        stats = ScanStats()
        rc = lib().rsh_match_scan_pieces(self._p, pl, len(arrs), ctypes.byref(h), _ptr(w) if w.size else None,
                                         _ptr(st) if st.size else None, _ptr(s), _ptr(ev), cap, ctypes.byref(n_ev),
                                         _ptr(fm), ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(stats))
        if rc == RSH_E_NOSPACE:
            ev = np.zeros(n_ev.value, EVENT_DTYPE)
            rc = lib().rsh_fetch_events(self._p, _ptr(ev), n_ev.value, ctypes.byref(n_ev))
        _check(rc)
        return ev[:n_ev.value], fm.tobytes(), lit.value, mat.value, stats.as_dict()

    def block_sums_file(self, path, size, h, seed):
        """Generator pass over a file (FileView reads of `size` bytes): (weak, strong, read_error)."""
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        weak = np.zeros(max(h.chunk_count, 1), np.int32)
        strong = np.zeros(max(h.chunk_count * h.digest_length, 1), np.uint8)
        err = ctypes.c_int32()
        _check(lib().rsh_block_sums_file(self._p, os.fsencode(path), size, ctypes.byref(h), _ptr(s), _ptr(weak),
                                         _ptr(strong), ctypes.byref(err)))
        return weak[:h.chunk_count], strong[:h.chunk_count * h.digest_length], bool(err.value)

    def match_scan_file(self, path, size, h, weak, strong, seed):
        """Sender pass over a file: (events, file_md5, literal, matched, stats, read_error)."""
        s = np.frombuffer(bytes(seed), np.uint8).copy()
        w = np.ascontiguousarray(weak, dtype=np.int32)
        st = np.ascontiguousarray(strong, dtype=np.uint8)
        cap = int(size // max(10 * h.block_length, 1) + 2 * h.chunk_count + 64) if h.block_length else size // 8192 + 2
        ev = np.zeros(max(cap, 1), EVENT_DTYPE)
        n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        fm = np.zeros(16, np.uint8)
        stats = ScanStats()
        err = ctypes.c_int32()
        rc = lib().rsh_match_scan_file(self._p, os.fsencode(path), size, ctypes.byref(h), _ptr(w) if w.size else None,
                                       _ptr(st) if st.size else None, _ptr(s), _ptr(ev), cap, ctypes.byref(n_ev),
                                       _ptr(fm), ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(stats),
                                       ctypes.byref(err))
        if rc == RSH_E_NOSPACE:
            ev = np.zeros(n_ev.value, EVENT_DTYPE)
            rc = lib().rsh_fetch_events(self._p, _ptr(ev), n_ev.value, ctypes.byref(n_ev))
        _check(rc)
        return ev[:n_ev.value], fm.tobytes(), lit.value, mat.value, stats.as_dict(), bool(err.value)

    def receiver_combine_batch(self, files, statuses=None):
        """A segment's Receiver from host memory (rsh_receiver_combine_batch; Receiver.receiveFiles):
        files = [(tokens, Header, replica pieces or None, defer_write, target_cap or None)] ->
        [(status, target bytes, CombineResult)].  statuses (a list): receives the call's code instead of raising."""
        jobs = (CombineJob * max(len(files), 1))()
        keep, tgts = [], []
        for i, (tokens, h, replica, defer, cap) in enumerate(files):
            t = _u8(tokens)
            arrs, pl, rn = _piece_list(replica) if replica is not None else ([], None, 0)
            if cap is None:
                cap = t.size + (t.size // 4) * max(h.block_length, 1) + 16
            tgt = np.zeros(max(cap, 1), np.uint8)
            keep.append((t, arrs, pl))
            tgts.append(tgt)
            j = jobs[i]
            j.tokens, j.tokens_len, j.h = (t.ctypes.data if t.size else None), t.size, h
            if replica is not None:
                j.replica, j.nreplica = ctypes.cast(pl, ctypes.POINTER(Piece)), len(arrs)
            j.defer_write, j.target, j.target_cap = int(bool(defer)), tgt.ctypes.data, cap
        rc = self._combine_batch(jobs, len(files))
        if statuses is not None:
            statuses[:] = [rc]
        elif rc not in (RSH_OK, RSH_E_NOSPACE, RSH_E_PROTOCOL, RSH_E_INVAL):
            _check(rc)
        out = []
        for i in range(len(files)):
            j = jobs[i]
            r = CombineResult.from_buffer_copy(j.res)
            n = r.target_len if j.status == RSH_OK else 0
            out.append((j.status, tgts[i][:n].tobytes(), r))
        return out

    def receiver_combine(self, tokens, h, replica, defer_write=False, target_cap=None):
        """Receiver.combineDataToFile (Receiver.java:459-555): (target bytes, CombineResult).  The target is
        empty when the deferred write left the file intact (result.intact)."""
        t = _u8(tokens)
        rep = None if replica is None else _u8(replica)
        cap = target_cap if target_cap is not None else t.size + (t.size // 4) * max(h.block_length, 1) + 16
        tgt = np.zeros(max(cap, 1), np.uint8)
        r = CombineResult()
        _check(lib().rsh_receiver_combine(self._p, _ptr(t), t.size, ctypes.byref(h), _ptr(rep),
                                          0 if rep is None else rep.size, int(bool(defer_write)), _ptr(tgt), cap,
                                          ctypes.byref(r)))
        return tgt[:r.target_len].tobytes(), r


class DeviceSet(Context):
    """The calling thread's contexts over several GPUs (rsh_*_batch_multi): the segment calls block_sums_batch,
    match_scan_batch and receiver_combine_batch split their files over the contexts (rsh_shard_files) and run each
    context's share beside the others.  devices: one context per entry (a device may repeat).  The single-context
    methods run on the first context."""

    def __init__(self, devices):
        self.members = [Context(d) for d in devices]
        self._p = self.members[0].handle
        self._arr = (ctypes.c_void_p * len(self.members))(*[c.handle.value for c in self.members])

    def close(self):
        for c in getattr(self, "members", []):
            c.close()
        self.members, self._p = [], ctypes.c_void_p()

    def trim(self):
        for c in self.members:
            c.trim()

    def _block_batch(self, jobs, n, seed):
        return lib().rsh_block_sums_batch_multi(self._arr, len(self.members), jobs, n, seed)

    def _scan_batch(self, jobs, n, seed, stats):
        return lib().rsh_match_scan_batch_multi(self._arr, len(self.members), jobs, n, seed, stats)

    def _combine_batch(self, jobs, n):
        return lib().rsh_receiver_combine_batch_multi(self._arr, len(self.members), jobs, n)


def shard_files(sizes, parts):
    """rsh_shard_files: the part (context) each file goes to."""
    b = np.ascontiguousarray(sizes, dtype=np.int64)
    out = np.zeros(max(b.size, 1), np.int32)
    _check(lib().rsh_shard_files(_ptr(b), b.size, parts, _ptr(out)))
    return out[:b.size]


class DeviceBuffer:
    """A hipMalloc'd buffer for the *_device entry points (no torch needed)."""

    def __init__(self, ctx, nbytes):
        self.ctx, self.nbytes = ctx, int(nbytes)
        self.ptr = ctypes.c_void_p()
        _check(lib().rsh_dev_alloc(ctx.handle, self.nbytes, ctypes.byref(self.ptr)))

    def upload(self, arr, offset=0):
        a = np.ascontiguousarray(arr)
        _check(lib().rsh_memcpy_h2d(self.ctx.handle, ctypes.c_void_p(self.ptr.value + offset),
                                    ctypes.c_void_p(a.ctypes.data), a.nbytes))

    def download(self, nbytes=None, dtype=np.uint8, offset=0):
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype)
        _check(lib().rsh_memcpy_d2h(self.ctx.handle, ctypes.c_void_p(out.ctypes.data),
                                    ctypes.c_void_p(self.ptr.value + offset), out.nbytes))
        return out

    def free(self):
        if self.ptr:
            lib().rsh_dev_free(self.ctx.handle, self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
