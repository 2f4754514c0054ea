"""CPU tests of librsynchip.so's host-side surface: it loads, exports every symbol include/rsync_hip.h
declares, and its pure-host functions (sizing rule, header validation, channel bytes) agree with the
oracle.  No compute calls that need a GPU."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

import oracle_ctypes as O
import rsync_hip as R
from conftest import ROOT, golden


@pytest.fixture(scope="module", autouse=True)
def built():
    R.build()


def test_header_declares_exports():
    text = open(os.path.join(ROOT, "include", "rsync_hip.h")).read()
    declared = set(re.findall(r"\b(rsh_[a-z0-9_]+)\s*\(", text))
    assert declared == set(R.EXPORTS)


def test_debug_header_declares_exports():
    text = open(os.path.join(ROOT, "include", "rsync_hip_debug.h")).read()
    declared = set(re.findall(r"\b(rsh_[a-z0-9_]+)\s*\(", text))
    assert declared == set(R.DEBUG_EXPORTS)


def test_library_exports_every_symbol():
    L = ctypes.CDLL(R.LIB_PATH)
    for name in R.EXPORTS + R.DEBUG_EXPORTS:
        assert hasattr(L, name), name
    assert R.lib().rsh_abi_version() == 5


def test_options_have_defaults_and_no_environment():
    """Tunables and diagnostic switches (include/rsync_hip_debug.h) change only through the debug ABI: an
    environment variable of the old A/B form is ignored, an unknown name is rejected, reset restores defaults."""
    assert R.get_option("k1_gather") == 1 and R.get_option("file_tile_above") == 32 << 30
    with R.option("k1_gather", 0):
        assert R.get_option("k1_gather") == 0
    assert R.get_option("k1_gather") == 1
    with pytest.raises(ValueError):
        R.set_option("no_such_option", 1)
    R.set_option("scan_samples", 17)
    R.reset_options()
    assert R.get_option("scan_samples") == 256
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import rsync_hip as R; print(R.get_option('k1_gather'))"
            % os.path.join(ROOT, "java-rsync_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, RSH_K1_GATHER="0"), capture_output=True,
                         text=True, check=True)
    assert out.stdout.strip() == "1"


def test_ab_switches_only_in_the_diagnostics_build():
    """options.h: the A/B switches (rejected alternatives, policy knobs) are compiled-in constants of the product
    library -- rsh_debug_set_option refuses them and their value is the default -- and settable only in the
    diagnostics build (make diag, lib/diag/librsynchip.so) that the A/B tools load."""
    if os.environ.get("RSH_LIB"):
        pytest.skip("a non-product library is loaded")
    for name, default in (("scan_spec_queue", 1), ("batch_spin_us", 200), ("scan_phase", 1), ("batch_spec", -1)):
        assert R.get_option(name) == default
        with pytest.raises(ValueError):
            R.set_option(name, 0)
        assert R.get_option(name) == default


def test_product_library_has_no_ab_scaffolding():
    """The kbench-only K1 variants (RSH_KBENCH) and the old getenv switches are not in librsynchip.so."""
    blob = open(R.LIB_PATH, "rb").read()
    for s in (b"RSH_K1_", b"RSH_SCAN_", b"RSH_BATCH_", b"RSH_FILE_", b"block_sums_quad_kernel", b"block_sums_dma_kernel",
              b"block_sums_pipe_k3_kernel"):
        assert s not in blob, s


def test_library_built_from_these_sources():
    """The build stamps librsynchip.so with its sources' sha256 (lib/librsynchip.srchash); rsync_hip.lib() refuses
    a library whose sources changed since, so no test or bench run measures a stale binary."""
    import os
    assert os.path.exists(os.path.join(os.path.dirname(R.LIB_PATH), "librsynchip.srchash"))
    assert R.stale_sources() == []


@pytest.mark.parametrize("n", [1, 511, 512, 557, 1000, 64 << 20, 128 << 20, 4 << 30, 16 << 30, 64 << 30, (1 << 40) + 3])
def test_sizing_matches_oracle(n):
    L = O.lib()
    b = R.block_length_for(n)
    assert b == L.orc_block_length_for(n)
    assert R.digest_length_for(n, b, 2) == max(2, L.orc_digest_length(n, b))
    assert R.digest_length_for(n, b, 16) == 16  # redo pass (Generator.java:371)


def test_header_make_and_validate():
    h = R.header_make(512, 2, 557)
    assert h.as_dict() == dict(chunk_count=2, block_length=512, digest_length=2, remainder=45)
    R.header_validate(h)
    with pytest.raises(OverflowError):
        R.header_make(1, 2, 1 << 40)
    for bad in [(1, (1 << 17) + 1, 2, 0), (1, 0, 2, 0), (2, 512, 2, 513), (-1, 512, 2, 0), (1, 512, -1, 0)]:
        with pytest.raises(R.ProtocolError):
            R.header_validate(R.Header(*bad))
    R.header_validate(R.Header(131072, 1 << 17, 4, 0))  # config 5 is accepted (check is '>')
    with pytest.raises(R.ProtocolError):                # config 3 (B = 2^18) is rejected
        R.header_validate(R.header_make(1 << 18, 5, 64 << 30))


def test_file_md5_host():
    for n in [0, 1, 55, 56, 63, 64, 65, 1000, 100000]:
        d = O.splitmix(n, 7).tobytes()
        assert R.file_md5(d) == hashlib.md5(d).digest()


@pytest.mark.parametrize("case", golden()[:12] + golden()[-8:], ids=lambda c: c["name"])
def test_tokens_match_oracle(case):
    ev = np.zeros(len(case["events"]), R.EVENT_DTYPE)
    for i, (k, off, ln, idx) in enumerate(case["events"]):
        ev[i] = (off, ln, k, idx, 1 if k == R.EV_MATCH else 0, 0)
    tok = R.tokens(case["src_bytes"], ev, bytes.fromhex(case["file_md5"]))
    assert hashlib.sha256(tok).hexdigest() == case["tokens_sha256"]


def test_tokens_match_runs():
    src = bytes(range(256)) * 100
    ev = np.zeros(3, R.EVENT_DTYPE)
    ev[0] = (0, 20000, R.EV_LITERAL, 0, 0, 0)
    ev[1] = (20000, 1536, R.EV_MATCH, 7, 3, 0)
    ev[2] = (21536, 5, R.EV_LITERAL, 0, 0, 0)
    tok = R.tokens(src, ev, bytes(16))
    oev = [(1, 0, 20000, 0), (2, 20000, 512, 7), (2, 20512, 512, 8), (2, 21024, 512, 9), (1, 21536, 5, 0)]
    assert tok == O.tokens(src, oev, bytes(16))
    assert R.events_as_tuples(ev, 512) == oev


def test_generator_bytes():
    g = {c["name"]: c for c in golden()}["systemtest_copy_twice_557"]
    h = R.Header(**g["header"])
    weak = np.array(g["weak"], np.int32)
    strong = np.frombuffer(bytes.fromhex(g["strong"]), np.uint8).copy()
    size = R.lib().rsh_generator_bytes(ctypes.byref(h), None, None, None, 0)
    out = np.zeros(size, np.uint8)
    assert R.lib().rsh_generator_bytes(ctypes.byref(h), weak.ctypes.data, strong.ctypes.data, out.ctypes.data,
                                       size) == size
    oh = O.Header(**g["header"])
    ref = np.zeros(size, np.uint8)
    O.lib().orc_generator_bytes(ctypes.byref(oh), weak.ctypes.data, strong.ctypes.data, ref.ctypes.data)
    assert out.tobytes() == ref.tobytes()


def test_no_device_fails_loudly():
    """Without a gfx950 GPU the product refuses to run: there is no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(R.DeviceError):
        R.Context(0)


def test_status_strings_and_last_error():
    L = R.lib()
    codes = [R.RSH_OK, R.RSH_E_INVAL, R.RSH_E_PROTOCOL, R.RSH_E_OVERFLOW, R.RSH_E_NOSPACE, R.RSH_E_DEVICE,
             R.RSH_E_NOMEM, R.RSH_E_BUSY]
    texts = [L.rsh_strerror(c).decode() for c in codes]
    assert len(set(texts)) == len(texts) and "unknown status" not in texts
    assert "another thread" in L.rsh_strerror(R.RSH_E_BUSY).decode()
    assert L.rsh_strerror(-99).decode() == "unknown status"
    assert isinstance(L.rsh_last_error(), bytes)  # "" until a HIP call of this thread fails
    with pytest.raises(R.ContextBusyError):
        R._check(R.RSH_E_BUSY)


@pytest.mark.parametrize("width", [0, 1, 8, 16])
def test_file_md5_batch_matches_hashlib(width):
    """rsh_file_md5_batch (md5_mb.cpp, the Sender's whole-file MD5s of a segment, Sender.java:1241,1326): every
    file's digest is hashlib's, whatever its length (every padding case around 55/56/64/119/120 bytes), its
    pieces (empty ones, blocks straddling pieces) and the lane it ran on.  width: the multi-buffer form (0 = the
    widest this CPU has, 1 scalar, 8 AVX2, 16 AVX-512; capped at what the CPU runs), several thread counts."""
    import random
    rng = random.Random(77 + width)
    sizes = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129, 1000, 4096, 70000]
    sizes += [rng.randrange(0, 300000) for _ in range(40)] + [1 << 20, 3 << 20]
    files = []
    for k, n in enumerate(sizes):
        a = O.splitmix(n, 0xABC + k) if n else np.zeros(0, np.uint8)
        cuts = sorted(rng.randrange(0, n + 1) for _ in range(rng.randrange(0, 5)))
        pieces, prev = [], 0
        for c in cuts + [n]:
            pieces.append(a[prev:c])
            prev = c
        files.append((a, pieces))
    with R.option("md5_width", width):
        for threads in (1, 3, 0):
            got = R.file_md5_batch([p for _, p in files], threads=threads)
            for (a, _), d in zip(files, got):
                assert d == hashlib.md5(a.tobytes()).digest(), (a.size, threads)
    assert R.file_md5_batch([]) == []


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_shard_files_matches_rank_rule(nparts):
    """rsh_shard_files (the split of rsh_*_batch_multi) is shard.py's LPT rule: longest first, equal sizes in file
    order, each file to the part with the fewest bytes so far, ties to the lower part."""
    import random

    import shard
    rng = random.Random(nparts)
    for sizes in ([128 << 20] * 1024, [rng.choice([0, 1, 5 << 20, 128 << 20, 3 << 30]) for _ in range(97)], [7], []):
        parts = R.shard_files(sizes, nparts)
        want = shard.shard_files(sizes, nparts)
        got = [sorted(int(i) for i in np.nonzero(parts == p)[0]) for p in range(nparts)]
        assert got == want


def _selftest(sizes, nparts, fail_part):
    import ctypes
    b = np.array(sizes, np.int64)
    part, order, status = (np.zeros(max(len(sizes), 1), np.int32) for _ in range(3))
    rc = R.lib().rsh_debug_multi_selftest(ctypes.c_void_p(b.ctypes.data), len(sizes), nparts, fail_part,
                                          ctypes.c_void_p(part.ctypes.data), ctypes.c_void_p(order.ctypes.data),
                                          ctypes.c_void_p(status.ctypes.data))
    n = len(sizes)
    return rc, part[:n], order[:n], status[:n]


def test_multi_merge_order():
    """The multi-context driver: every file lands on its rsh_shard_files part, a part sees its files in segment order,
    and each job's outputs come back to the caller's job of the same file (the stand-in member call records them)."""
    import random
    rng = random.Random(5)
    sizes = [rng.randrange(1, 1 << 30) for _ in range(200)]
    rc, part, order, status = _selftest(sizes, 8, -1)
    assert rc == R.RSH_OK and (status == R.RSH_OK).all()
    assert np.array_equal(part, R.shard_files(sizes, 8))
    for p in range(8):
        mine = np.nonzero(part == p)[0]
        assert list(order[mine]) == list(range(mine.size))  # file order within the part


def test_multi_failure_marks_one_member():
    """A member call that fails (after finishing its first file) marks only the files of its own part; the other
    parts' files are RSH_OK, and the call returns the first failing job's status in file order."""
    sizes = [100 << 20] * 16 + [1 << 20] * 16
    rc, part, order, status = _selftest(sizes, 4, 2)
    mine = np.nonzero(part == 2)[0]
    assert mine.size > 1
    failed = np.nonzero(status != R.RSH_OK)[0]
    assert list(failed) == list(mine[1:]) and (status[failed] == R.RSH_E_DEVICE).all()
    assert rc == R.RSH_E_DEVICE
    rc, _, _, status = _selftest(sizes, 4, -1)
    assert rc == R.RSH_OK and (status == R.RSH_OK).all()


def test_multi_entry_points_validate_contexts():
    """Null or repeated contexts are refused before any work (RSH_E_INVAL): a context serves one call at a time."""
    import ctypes
    L = R.lib()
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    fake = (ctypes.c_void_p * 2)(0x1000, 0x1000)
    nul = (ctypes.c_void_p * 2)(0x1000, None)
    for arr in (fake, nul):
        assert L.rsh_block_sums_batch_multi(arr, 2, None, 0, ctypes.c_void_p(seed.ctypes.data)) == R.RSH_E_INVAL
        assert L.rsh_match_scan_batch_multi(arr, 2, None, 0, ctypes.c_void_p(seed.ctypes.data), None) == R.RSH_E_INVAL
        assert L.rsh_receiver_combine_batch_multi(arr, 2, None, 0) == R.RSH_E_INVAL
    assert L.rsh_block_sums_batch_multi(fake, 0, None, 0, ctypes.c_void_p(seed.ctypes.data)) == R.RSH_E_INVAL
