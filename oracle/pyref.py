"""pyref.py -- TEST INFRASTRUCTURE ONLY.

An independent pure-Python restatement of java-rsync's checksum hot path, used (a) to cross-check
the C oracle (oracle/rsync_oracle.c) and (b) to generate the committed golden fixtures under
tests/golden/ (see tests/golden/make_golden.py).  MD5 comes from the stdlib (hashlib), i.e. an
implementation independent of the oracle's own RFC 1321 code.  Pure-Python loops: small inputs only.

Reference paths are relative to core/src/main/java/com/github/java/rsync/internal/.
"""
import hashlib
import math

CHUNK_SIZE = 8192            # Sender.java:230
DEFAULT_BLOCK_SIZE = 8192    # io/FileView.java:38
MAX_BLOCK_LENGTH = 1 << 17   # session/Checksum.java:151
LIT, MATCH = 1, 2


def _sb(b):
    """Java byte -> int (signed)."""
    return b - 256 if b >= 128 else b


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def weak(buf):
    """util/Rolling.java:31-46 (CHAR_OFFSET = 0): s1 = sum x, s2 = sum (L-i) x_i, packed s1 | s2 << 16."""
    s1 = 0
    s2 = 0
    for b in buf:
        s1 += _sb(b)
        s2 += s1
    return _i32((s1 & 0xFFFF) | ((s2 & 0xFFFF) << 16))


def rolling_add(cs, value):  # Rolling.java:25-29
    lo = (cs & 0xFFFF) + _sb(value)
    hi = ((cs & 0xFFFFFFFF) >> 16) + lo
    return _i32((lo & 0xFFFF) | ((hi & 0xFFFF) << 16))


def rolling_subtract(cs, block_length, value):  # Rolling.java:56-60
    lo = (cs & 0xFFFF) - _sb(value)
    hi = ((cs & 0xFFFFFFFF) >> 16) - block_length * _sb(value)
    return _i32((lo & 0xFFFF) | ((hi & 0xFFFF) << 16))


def block_length_for(n):  # Generator.java:198-206, 219-236
    if n == 0:
        return 0
    exp = n.bit_length() - 1
    return max(512, 1 << (exp // 2))


def digest_length(n, blen):  # Generator.java:208-212 with Util.log2 (Util.java:128-130)
    lf = int(math.log(n) / math.log(2))
    lb = int(math.log(blen) / math.log(2))
    r = int((10 + 2 * lf - lb) - 24)
    r = int(r / 8)  # Java truncating division
    return max(2, min(16, r))


def copy_of(digest, dl):  # Arrays.copyOf (Sender.java:1262): truncate, or zero-pad past 16 bytes
    return digest[:dl] + bytes(max(0, dl - len(digest)))


def header(blen, dlen, n):  # Checksum.java:94-113
    if blen == 0:
        return dict(chunk_count=0, block_length=0, digest_length=0, remainder=0)
    rem = n % blen
    return dict(chunk_count=n // blen + (1 if rem else 0), block_length=blen, digest_length=dlen, remainder=rem)


def generator(basis, hdr, seed):
    """Generator.java:886-895: per window (weak, MD5(window || seed)[:dl])."""
    B, dl = hdr["block_length"], hdr["digest_length"]
    out = []
    for i in range(hdr["chunk_count"]):
        blk = basis[i * B:(i + 1) * B]
        out.append((weak(blk), copy_of(hashlib.md5(blk + seed).digest(), dl)))
    return out


def sender(src, hdr, sums, seed):
    """Sender.sendMatchesAndData (Sender.java:1235-1327) / skipMatchSendData (:1386-1399).

    Returns (events, file_md5, literal, matched); events = [(LIT, off, len, 0) | (MATCH, off, len, idx)],
    zero-length literal calls omitted.
    """
    N = len(src)
    B = hdr["block_length"]
    ev = []

    def lit(off, ln):
        if ln:
            ev.append((LIT, off, ln, 0))

    if B == 0:
        for s in range(0, N, DEFAULT_BLOCK_SIZE):
            lit(s, min(DEFAULT_BLOCK_SIZE, N - s))
        return ev, hashlib.md5(src).digest(), N, 0
    if N == 0:
        return ev, hashlib.md5(b"").digest(), 0, 0

    dl = hdr["digest_length"]
    count = hdr["chunk_count"]
    rem = hdr["remainder"]
    buckets = {}
    for i, (w, s) in enumerate(sums):  # Multimap insertion order == chunk index order
        buckets.setdefault(w, []).append(i)

    def clen(i):  # Checksum.java:197-203
        return rem if (i == count - 1 and rem > 0) else B

    def candidates(key, length, pref):  # Checksum.java:206-276
        b = buckets.get(key)
        if not b:
            return
        # closeIndexOf: exact position, else the insertion point clamped to the last element
        lo, hi = 0, len(b)
        while lo < hi:
            m = (lo + hi) // 2
            if b[m] < pref:
                lo = m + 1
            else:
                hi = m
        init = lo if (lo < len(b) and b[lo] == pref) else min(lo, len(b) - 1)
        yield b[init]
        for j, c in enumerate(b):
            if j != init and clen(c) == length:
                yield c

    def W(s):
        return min(B, N - s)

    S = rem if rem > 0 else B
    fdig = hashlib.md5()
    start = mark = 0
    roll = weak(src[0:W(0)])
    pref = 0
    slit = smatch = 0
    md5c = None
    while W(start) >= S:
        w = W(start)
        for c in candidates(roll, w, pref):
            if md5c is None:
                md5c = copy_of(hashlib.md5(src[start:start + w] + seed).digest(), dl)
            if md5c == sums[c][1]:
                smatch += w
                first = min(start, mark)
                lit(mark, start - first)
                slit += start - first
                fdig.update(src[mark:start + w])
                ev.append((MATCH, start, w, c))
                pref = c + 1
                mark = start + w
                start += w - 1
                roll = weak(src[start:start + W(start)])
                md5c = None
                break
        w = W(start)
        roll = rolling_subtract(roll, w, src[start])
        first = min(start, mark)
        total = start + w - first
        if total == 10 * B:
            lit(first, total)
            slit += total
            fdig.update(src[first:start + w])
            mark = start + w
            start += w
        else:
            start += 1
        if W(start) == B:
            roll = rolling_add(roll, src[start + B - 1])
    first = min(start, mark)
    lit(first, N - first)
    slit += N - first
    fdig.update(src[first:N])
    return ev, fdig.digest(), slit, smatch


def tokens(src, events, file_md5):
    """Channel bytes written by the Sender for one file (LE ints, 8 KiB literal pieces)."""
    out = bytearray()
    for kind, off, ln, idx in events:
        if kind == LIT:
            cur, end = off, off + ln
            while cur < end:
                n = min(CHUNK_SIZE, end - cur)
                out += n.to_bytes(4, "little", signed=True)
                out += src[cur:cur + n]
                cur += n
        else:
            out += (-(idx + 1)).to_bytes(4, "little", signed=True)
    out += (0).to_bytes(4, "little")
    out += file_md5
    return bytes(out)


def splitmix_bytes(n, key, offset=0):
    """Counter-based splitmix64 stream (same definition as orc_fill_splitmix)."""
    M = (1 << 64) - 1
    out = bytearray(n)
    for i in range(n):
        pos = offset + i
        z = (key + (pos // 8 + 1) * 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out[i] = (z >> (8 * (pos % 8))) & 0xFF
    return bytes(out)
