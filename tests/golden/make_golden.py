"""Generate tests/golden/cases.json with the independent Python restatement (oracle/pyref.py).

Run from the repo root:  python tests/golden/make_golden.py
No JDK exists in this image, so the Java reference cannot produce these vectors itself; they are
restatement-derived (see DESIGN.md "Oracle").  The reference-pinned facts among them are the
SystemTest cases (rsync-app SystemTest.java:532-628) and the RFC 1321 MD5 vectors.
"""
import base64
import hashlib
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyref as P  # noqa: E402

SEED_A = bytes([1, 2, 3, 4])
KEY = 0x5EED5EED << 32


def rnd(n, k):
    return P.splitmix_bytes(n, KEY ^ k)


def enc(b):
    return base64.b64encode(zlib.compress(bytes(b), 9)).decode()


def weak_preserving_tweak(buf, start, end):
    """Add (+1, -2, +1) to three consecutive signed bytes inside [start, end): keeps Rolling.compute
    of the enclosing block unchanged (sum and position-weighted sum both preserved) but changes its MD5."""
    b = bytearray(buf)
    for i in range(start, end - 2):
        x0, x1, x2 = P._sb(b[i]), P._sb(b[i + 1]), P._sb(b[i + 2])
        if x0 <= 126 and x1 >= -126 and x2 <= 126:
            b[i] = (x0 + 1) & 0xFF
            b[i + 1] = (x1 - 2) & 0xFF
            b[i + 2] = (x2 + 1) & 0xFF
            return bytes(b)
    raise RuntimeError("no tweak site")


def cases():
    out = []

    def add(name, basis, src, blen=None, dlen=None, seed=SEED_A, note=""):
        out.append(dict(name=name, basis=basis, src=src, blen=blen, dlen=dlen, seed=seed, note=note))

    # -- reference-pinned: rsync-app SystemTest.java
    c557 = bytes([0x18]) * 557
    add("systemtest_copy_twice_557", c557, c557, seed=bytes(4),
        note="SystemTest.java:604-628: 2nd copy literal 0, matched 557")
    for n, v, line in [(257, 0xBC, 532), (2048, 0xF0, 550), (651, 0x19, 568), (512, 0xCD, 586)]:
        add(f"systemtest_new_file_{n}", None, bytes([v]) * n, seed=bytes(4),
            note=f"SystemTest.java:{line}: new file => literal {n}, matched 0")
    # -- edge sizes, identical basis (rule B = 512)
    for n in [1, 2, 3, 4, 5, 63, 64, 65, 511, 512, 513, 1023, 1024, 5 * 512 + 45, 40 * 512]:
        d = rnd(n, n)
        add(f"identical_{n}", d, d)
    # -- signed-byte extremes / low entropy
    add("all_0x80", bytes([0x80]) * 3000, bytes([0x80]) * 3000)
    add("all_0x7f", bytes([0x7F]) * 3000, bytes([0x7F]) * 2999)
    add("alt_80_7f", bytes([0x80, 0x7F]) * 1500, bytes([0x7F, 0x80]) * 1500)
    add("zeros_identical", bytes(20 * 512), bytes(20 * 512), note="one bucket holds every chunk")
    add("zeros_vs_shorter", bytes(20 * 512 + 100), bytes(9 * 512 + 7))
    rep = rnd(512, 77) * 6 + rnd(512, 78) + rnd(512, 77) * 5
    add("repeated_blocks", rep, rnd(512, 77) * 3 + rnd(300, 79) + rnd(512, 77) * 4 + rnd(512, 78),
        note="duplicate weak keys: preferred-index candidate order (Checksum.java:206-276)")
    # -- random, unrelated source (all literal, exercises flushes every 10*B)
    add("unrelated_24k", rnd(24000, 1), rnd(24000, 2))
    add("unrelated_small_table", rnd(3000, 3), rnd(30000, 4))
    # -- quirk B: a weak collision poisons the cached digest
    base = rnd(40 * 512, 5)
    add("poison_block5", base, weak_preserving_tweak(base, 5 * 512 + 10, 6 * 512),
        note="weak hit + MD5 miss at block 5 -> stale localChunkMd5sum, rest literal")
    base = rnd(30 * 512 + 77, 6)
    add("poison_last_partial", base, weak_preserving_tweak(base, 30 * 512, 30 * 512 + 77))
    # -- quirk A: >= 9*B modified run desyncs the rolling sum after the flush
    base = rnd(40 * 512, 7)
    add("edit_run_10B", base, base[:10 * 512] + rnd(10 * 512, 8) + base[20 * 512:])
    add("edit_run_8B", base, base[:10 * 512] + rnd(8 * 512, 9) + base[18 * 512:])
    add("edit_run_9B", base, base[:3 * 512] + rnd(9 * 512, 10) + base[12 * 512:])
    # -- every other block modified (config-5 shape at small scale)
    blocks = [rnd(512, 100 + i) if i % 2 else base[i * 512:(i + 1) * 512] for i in range(40)]
    add("half_modified", base, b"".join(blocks))
    add("half_modified_basis", b"".join(blocks), base)
    # -- insertions / deletions (shifted matches)
    base = rnd(30 * 512 + 200, 11)
    add("insert_100", base, base[:7000] + rnd(100, 12) + base[7000:])
    add("delete_100", base, base[:7000] + base[7100:])
    add("insert_1", base, base[:2048] + b"\x00" + base[2048:])
    # -- remainder chunk interplay (initial candidate is not length-filtered)
    base = rnd(1000, 13)
    add("remainder_identical", base, base)
    add("remainder_src_short", base, base[:600])
    add("remainder_src_tail_only", base, base[512:])
    add("remainder_src_longer", base, base + rnd(700, 14))
    # -- explicit block/digest overrides (BASELINE config shapes at small scale)
    base = rnd(32 * 1024, 15)
    add("gen_B512_dl3", base, base, blen=512, dlen=3)
    add("B700_nonpow2", base[:20000], base[:20000], blen=700, dlen=2)
    add("dl16_redo", base[:9000], base[:9000][::-1], blen=512, dlen=16)
    # -- empty inputs
    add("empty_source", rnd(2000, 16), b"")
    add("empty_basis_new_file", None, rnd(100, 17))
    return out


BLOBS = {}


def blob(b):
    """Store input bytes once (many cases share a base buffer); cases refer to them by sha256 prefix."""
    key = hashlib.sha256(b).hexdigest()[:16]
    BLOBS.setdefault(key, enc(b))
    return key


def run(c):
    basis, src = c["basis"], c["src"]
    if basis is None:
        hdr = P.header(0, 0, 0)  # ZERO_SUM: new file (Generator.java:507-509)
        sums = []
    else:
        nb = len(basis)
        blen = c["blen"] if c["blen"] is not None else P.block_length_for(nb)
        dlen = c["dlen"] if c["dlen"] is not None else (max(2, P.digest_length(nb, blen)) if nb > 0 else 0)
        hdr = P.header(blen, dlen, nb)
        sums = P.generator(basis, hdr, c["seed"])
    ev, fmd5, lit, mat = P.sender(src, hdr, sums, c["seed"])
    tok = P.tokens(src, ev, fmd5)
    return dict(
        name=c["name"], note=c["note"], seed=c["seed"].hex(),
        basis=None if basis is None else blob(basis), src=blob(src),
        basis_len=None if basis is None else len(basis), src_len=len(src),
        header=hdr,
        weak=[w for w, _ in sums], strong="".join(s.hex() for _, s in sums),
        events=[list(e) for e in ev], file_md5=fmd5.hex(), literal=lit, matched=mat,
        tokens_sha256=hashlib.sha256(tok).hexdigest(), tokens_len=len(tok),
    )


def main():
    res = [run(c) for c in cases()]
    path = os.path.join(HERE, "cases.json")
    with open(path, "w") as f:
        json.dump(dict(generator="oracle/pyref.py", blobs=BLOBS, cases=res), f, separators=(",", ":"))
    print(f"wrote {len(res)} cases to {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
