"""File ingest (rsh_block_sums_file / rsh_match_scan_file): the FileView reads of the two passes.

FileView (FileView.java:51-80, 187-278) reads exactly the size the FileInfo holds; a file that ends early
or fails to read is zero-filled from that point and the error surfaces at close() (FileViewException),
which the Sender turns into a corrupted file MD5 (Sender.java:1136-1143).  A missing file fails at open
(FileViewNotFound); an empty file is never opened.  Results are checked against the oracle over the
bytes FileView would have produced."""
import os

import numpy as np
import pytest

import oracle_ctypes as O
import rsync_hip as R

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])


@pytest.fixture(scope="module")
def ctx():
    R.build()
    c = R.Context(0)
    yield c
    c.close()


def _write(tmp_path, name, data):
    p = tmp_path / name
    p.write_bytes(data)
    return str(p)


@pytest.mark.parametrize("n,B", [(1, 512), (5 * 512 + 3, 512), ((3 << 20) + 77, 8192), ((200 << 20) + 5, 65536)])
def test_files_match_oracle(ctx, tmp_path, n, B):
    basis = O.splitmix(n, 0x5EED5EED00000031 ^ n).tobytes()
    src = bytearray(basis)
    src[n // 3:n // 3 + 10] = b"0123456789"[:len(src[n // 3:n // 3 + 10])]
    src = bytes(src[: n // 2]) + O.splitmix(777, 5).tobytes() + bytes(src[n // 2:])
    pb, ps = _write(tmp_path, "basis", basis), _write(tmp_path, "src", src)
    dl = max(2, R.digest_length_for(n, B))
    h = R.header_make(B, dl, n)
    w, s, err = ctx.block_sums_file(pb, n, h, SEED)
    ow, os_ = O.generator(basis, O.header(B, dl, n), SEED)
    assert not err and np.array_equal(w, ow) and np.array_equal(s, os_)
    ev, fm, lit, mat, _, err = ctx.match_scan_file(ps, len(src), h, ow, os_, SEED)
    oev, ofm, olit, omat, _ = O.sender(src, O.header(B, dl, n), ow, os_, SEED)
    assert not err and R.events_as_tuples(ev, B) == [tuple(e) for e in oev] and (fm, lit, mat) == (ofm, olit, omat)


def test_short_file_is_zero_filled_and_flagged(ctx, tmp_path):
    B = 1024
    data = O.splitmix(10 * B + 100, 7).tobytes()
    p = _write(tmp_path, "short", data)
    size = len(data) + 3 * B + 5  # the FileInfo says more than the file holds
    view = data + bytes(size - len(data))
    h = R.header_make(B, 3, size)
    w, s, err = ctx.block_sums_file(p, size, h, SEED)
    ow, os_ = O.generator(view, O.header(B, 3, size), SEED)
    assert err and np.array_equal(w, ow) and np.array_equal(s, os_)
    ev, fm, lit, mat, _, err = ctx.match_scan_file(p, size, h, ow, os_, SEED)
    oev, ofm, olit, omat, _ = O.sender(view, O.header(B, 3, size), ow, os_, SEED)
    assert err and R.events_as_tuples(ev, B) == [tuple(e) for e in oev] and fm == ofm
    # a FileInfo size below the file's: exactly that many bytes are read, no error
    h2 = R.header_make(B, 3, 5 * B)
    w2, s2, err = ctx.block_sums_file(p, 5 * B, h2, SEED)
    ow2, os2 = O.generator(data[:5 * B], O.header(B, 3, 5 * B), SEED)
    assert not err and np.array_equal(w2, ow2) and np.array_equal(s2, os2)


def test_open_errors(ctx, tmp_path):
    h = R.header_make(512, 2, 1000)
    missing = str(tmp_path / "missing")
    with pytest.raises(R.FileViewNotFound):
        ctx.block_sums_file(missing, 1000, h, SEED)
    with pytest.raises(R.FileViewNotFound):
        ctx.match_scan_file(missing, 1000, h, np.zeros(2, np.int32), np.zeros(4, np.uint8), SEED)
    # an empty file is never opened (FileView.java:62-72): no error even when the path is gone
    h0 = R.header_make(0, 0, 0)
    w, s, err = ctx.block_sums_file(missing, 0, h0, SEED)
    assert len(w) == 0 and not err
    ev, fm, lit, mat, _, err = ctx.match_scan_file(missing, 0, h0, np.zeros(0, np.int32), np.zeros(0, np.uint8), SEED)
    assert len(ev) == 0 and fm == O.md5(b"") and lit == mat == 0
    if os.geteuid() != 0:  # root reads anything
        p = _write(tmp_path, "locked", b"x" * 1000)
        os.chmod(p, 0)
        with pytest.raises(R.FileViewOpenFailed):
            ctx.block_sums_file(p, 1000, h, SEED)


@pytest.mark.parametrize("short", [False, True])
def test_file_scan_tiled(ctx, tmp_path, rsh_opt, short):
    """Files above file_tile_above (32 GiB by default; lowered here) are scanned with HBM holding one tile
    at a time (scan_tiled), read piece by piece from the file, the whole-file digest on its own pass: same
    events and digest as the oracle, FileView's zero fill and read_error included."""
    rsh_opt("file_tile_above", 1 << 20)
    rsh_opt("file_tile", 1 << 20)
    B = 4096
    n = (24 << 20) + 123
    basis = O.splitmix(n, 0x7711).tobytes()
    src = basis[:5 << 20] + O.splitmix(5000, 0x7712).tobytes() + basis[5 << 20:]
    size = len(src) + (3 * B + 7 if short else 0)  # the FileInfo size; a short file is zero-filled
    view = src + bytes(size - len(src))
    p = _write(tmp_path, "big", src)
    h = R.header_make(B, 3, n)
    ow, os_ = O.generator(basis, O.header(B, 3, n), SEED)
    ev, fm, lit, mat, st, err = ctx.match_scan_file(p, size, h, ow, os_, SEED)
    oev, ofm, olit, omat, _ = O.sender(view, O.header(B, 3, n), ow, os_, SEED)
    assert err == short
    assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev] and (fm, lit, mat) == (ofm, olit, omat)
    assert st["head_steps"] >= 20  # tile loads
