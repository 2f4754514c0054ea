"""oracle_ctypes.py -- TEST INFRASTRUCTURE ONLY: ctypes access to oracle/lib/liboracle.so.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg to check (never to produce)
the HIP path's results.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Header(ctypes.Structure):
    _fields_ = [("chunk_count", ctypes.c_int32), ("block_length", ctypes.c_int32),
                ("digest_length", ctypes.c_int32), ("remainder", ctypes.c_int32)]

    def as_dict(self):
        return dict(chunk_count=self.chunk_count, block_length=self.block_length,
                    digest_length=self.digest_length, remainder=self.remainder)


class Event(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("length", ctypes.c_int64),
                ("kind", ctypes.c_int32), ("index", ctypes.c_int32)]


class ScanResult(ctypes.Structure):
    _fields_ = [("ev", ctypes.POINTER(Event)), ("n_ev", ctypes.c_int64), ("cap", ctypes.c_int64),
                ("file_md5", ctypes.c_uint8 * 16), ("literal", ctypes.c_int64),
                ("matched", ctypes.c_int64), ("md5_windows", ctypes.c_int64)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "lib", "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.orc_md5.argtypes = [P, ctypes.c_size_t, P]
        L.orc_rolling_compute.argtypes = [P, ctypes.c_int32]
        L.orc_rolling_compute.restype = ctypes.c_int32
        L.orc_rolling_add.argtypes = [ctypes.c_int32, ctypes.c_uint8]
        L.orc_rolling_add.restype = ctypes.c_int32
        L.orc_rolling_subtract.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint8]
        L.orc_rolling_subtract.restype = ctypes.c_int32
        L.orc_block_length_for.argtypes = [ctypes.c_int64]
        L.orc_block_length_for.restype = ctypes.c_int32
        L.orc_digest_length.argtypes = [ctypes.c_int64, ctypes.c_int32]
        L.orc_digest_length.restype = ctypes.c_int32
        L.orc_header_make.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(Header)]
        L.orc_header_validate.argtypes = [ctypes.POINTER(Header)]
        L.orc_generator_sums.argtypes = [P, ctypes.c_int64, ctypes.POINTER(Header), P, P, P]
        L.orc_sender_scan.argtypes = [P, ctypes.c_int64, ctypes.POINTER(Header), P, P, P,
                                      ctypes.POINTER(ScanResult)]
        L.orc_scan_free.argtypes = [ctypes.POINTER(ScanResult)]
        L.orc_tokens.argtypes = [P, P, ctypes.c_int64, P, P]
        L.orc_tokens.restype = ctypes.c_int64
        L.orc_generator_bytes.argtypes = [ctypes.POINTER(Header), P, P, P]
        L.orc_generator_bytes.restype = ctypes.c_int64
        L.orc_receiver_combine.argtypes = [P, ctypes.c_int64, ctypes.POINTER(Header), P, ctypes.c_int64, ctypes.c_int,
                                           P, ctypes.c_int64, ctypes.POINTER(CombineResult)]
        L.orc_receiver_combine.restype = ctypes.c_int64
        L.orc_fill_splitmix.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64]
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u8(data):
    return np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data


def md5(data):
    a = _u8(data)
    out = np.zeros(16, np.uint8)
    lib().orc_md5(_ptr(a), a.size, _ptr(out))
    return out.tobytes()


def header(blen, dlen, n):
    h = Header()
    if lib().orc_header_make(blen, dlen, n, ctypes.byref(h)) != 0:
        raise OverflowError("ChunkOverflow")
    return h


def generator(basis, h, seed):
    a = _u8(basis)
    weak = np.zeros(max(h.chunk_count, 1), np.int32)
    strong = np.zeros(max(h.chunk_count * h.digest_length, 1), np.uint8)
    s = np.frombuffer(bytes(seed), np.uint8).copy()
    lib().orc_generator_sums(_ptr(a), a.size, ctypes.byref(h), _ptr(s), _ptr(weak), _ptr(strong))
    return weak[:h.chunk_count], strong[:h.chunk_count * h.digest_length]


def sender(src, h, weak, strong, seed):
    """Returns (events [(kind, off, len, idx)], file_md5 bytes, literal, matched, md5_windows)."""
    a = _u8(src)
    w = np.ascontiguousarray(weak, dtype=np.int32)
    st = np.ascontiguousarray(strong, dtype=np.uint8)
    s = np.frombuffer(bytes(seed), np.uint8).copy()
    r = ScanResult()
    rc = lib().orc_sender_scan(_ptr(a), a.size, ctypes.byref(h), _ptr(w) if w.size else None,
                               _ptr(st) if st.size else None, _ptr(s), ctypes.byref(r))
    if rc != 0:
        raise MemoryError("oracle scan failed")
    ev = [(r.ev[i].kind, r.ev[i].offset, r.ev[i].length, r.ev[i].index) for i in range(r.n_ev)]
    res = (ev, bytes(r.file_md5), r.literal, r.matched, r.md5_windows)
    lib().orc_scan_free(ctypes.byref(r))
    return res


def tokens(src, events, file_md5):
    a = _u8(src)
    n = len(events)
    evs = (Event * max(n, 1))()
    for i, (k, off, ln, idx) in enumerate(events):
        evs[i].kind, evs[i].offset, evs[i].length, evs[i].index = k, off, ln, idx
    fm = np.frombuffer(file_md5, np.uint8).copy()
    size = lib().orc_tokens(_ptr(a), evs, n, _ptr(fm), None)
    out = np.zeros(size, np.uint8)
    lib().orc_tokens(_ptr(a), evs, n, _ptr(fm), _ptr(out))
    return out.tobytes()


class CombineResult(ctypes.Structure):
    _fields_ = [("target_len", ctypes.c_int64), ("literal", ctypes.c_int64), ("matched", ctypes.c_int64),
                ("intact", ctypes.c_int32), ("md5", ctypes.c_uint8 * 16)]


def receiver_combine(tokens, h, replica, defer_write=False, target_cap=None):
    """Receiver.combineDataToFile: (rc, target bytes, literal, matched, intact, md5).  rc = tokens consumed
    (>= 4) or a negative error (-1 protocol, -2 truncated stream, -3 target too small, -4 replica short)."""
    t = _u8(tokens)
    rep = None if replica is None else _u8(replica)
    cap = target_cap if target_cap is not None else t.size + (t.size // 4) * max(h.block_length, 1) + 16
    tgt = np.zeros(max(cap, 1), np.uint8)
    r = CombineResult()
    rc = lib().orc_receiver_combine(_ptr(t), t.size, ctypes.byref(h), None if rep is None else _ptr(rep),
                                    0 if rep is None else rep.size, int(bool(defer_write)), _ptr(tgt), cap,
                                    ctypes.byref(r))
    return rc, tgt[:r.target_len].tobytes(), r.literal, r.matched, r.intact, bytes(r.md5)


def splitmix(n, key, offset=0):
    out = np.zeros(n, np.uint8)
    lib().orc_fill_splitmix(_ptr(out), n, key, offset)
    return out
