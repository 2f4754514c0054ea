"""TEST INFRASTRUCTURE: digests of full-size (GiB) Sender scans, so that a GPU run over BASELINE.json's sizes is
compared bit-exact against the oracle without shipping data ("Golden vectors").

tests/golden/make_fullsize.py runs the oracle (oracle/rsync_oracle.c: Generator.java:886-895 and
Sender.java:1235-1327 restated) over the inputs below in the build container and commits, per case:
  * events_sha256 -- SHA-256 of the event list at the oracle's granularity (one record per sendDataFrom call
    and one per matched chunk), each record packed little-endian as <i4 kind, <i4 index, <i8 offset, <i8 length>;
  * n_events, literal, matched, file_md5 (Sender.java:1241,1325-1326);
  * tokens_sha256 -- SHA-256 of the Sender's channel bytes for the file (Sender.java:794-809,1274,1316 and the
    16-byte digest of sendFiles :1148), computed here by a streaming restatement of sendDataFrom.
tests/test_gpu_fullsize.py rebuilds the same inputs on the device (rsh_fill_splitmix_device is the oracle's
splitmix64 stream) and compares its scan against these numbers.

Inputs are splitmix64 counter streams (orc_fill_splitmix); every case names its recipe, and both sides build it
with the same operations (slicing, concatenation, block replacement, reversal)."""
import hashlib

import numpy as np

KEY = 0x5EED5EED00000000
EV_LITERAL, EV_MATCH = 1, 2  # rsync_hip.h / rsync_oracle.h event kinds
REC = np.dtype([("kind", "<i4"), ("index", "<i4"), ("offset", "<i8"), ("length", "<i8")])

# name -> (n_basis, B, dl, recipe); recipes are applied by make_fullsize.py (host) and test_gpu_fullsize.py (device)
CASES = {
    # BASELINE config 2: 4 GiB, B = 65536 (the README rule), dl = 4
    "config2_identical": (4 << 30, 65536, 4, "identical"),
    # 1 GiB unchanged, 1000 inserted bytes, then a block reversed at 3 GiB + 500, a 33-byte tail
    "config2_insert": (4 << 30, 65536, 4, "insert1000_flip3g_tail33"),
    # BASELINE config 5: 16 GiB, B = 131072, dl = 4 (the bench's workload)
    "config5_identical": (16 << 30, 131072, 4, "identical"),
    "config5_half": (16 << 30, 131072, 4, "half"),
    # one byte inserted at offset 4096: a false weak hit in block 0 poisons the cached digest (quirk B), the
    # rest of the file is literal under the reference's semantics
    "config5_insert1": (16 << 30, 131072, 4, "insert1_at4096"),
    # one byte inserted at 155 * B + 4096, the first block >= 64 whose insert the scan rolls past without a
    # weak hit (make_fullsize.py --find-clean-insert): every later match is at phase kB + 1
    "config5_shift1": (16 << 30, 131072, 4, "insert1_at:20320256"),
}
BASIS_KEY = {"config2": KEY ^ 2, "config5": KEY ^ 5}


def records_from_oracle(events):
    """Oracle events [(kind, offset, length, index)] -> REC array."""
    a = np.zeros(len(events), REC)
    if events:
        e = np.array(events, dtype=np.int64)
        a["kind"], a["offset"], a["length"], a["index"] = e[:, 0], e[:, 1], e[:, 2], e[:, 3]
    return a


def records_from_runs(ev, block_length):
    """rsync_hip events (MATCH runs of `count` chunks) -> REC array at the oracle's granularity."""
    kind = ev["kind"].astype(np.int64)
    cnt = np.where(kind == EV_MATCH, ev["count"].astype(np.int64), 1)
    rep = np.repeat(np.arange(ev.size), cnt)
    j = np.arange(rep.size) - np.repeat(np.cumsum(cnt) - cnt, cnt)  # position inside the run
    out = np.zeros(rep.size, REC)
    k = kind[rep]
    out["kind"] = k
    out["index"] = np.where(k == EV_MATCH, ev["index"][rep].astype(np.int64) + j, 0)
    out["offset"] = ev["offset"][rep] + np.where(k == EV_MATCH, j * block_length, 0)
    last = j == cnt[rep] - 1  # every window of a run is a full block except possibly the run's last
    run_len = ev["length"][rep]
    out["length"] = np.where(k == EV_MATCH, np.where(last, run_len - j * block_length, block_length), run_len)
    return out


def events_sha(rec):
    return hashlib.sha256(np.ascontiguousarray(rec).tobytes()).hexdigest()


def tokens_sha_stream(src, rec, file_md5):
    """SHA-256 of the Sender's channel bytes, streamed: sendDataFrom (Sender.java:794-809) writes putInt(len) +
    bytes per <= 8192-byte piece of a literal; a match is putInt(-(index + 1)) (:1274); then putInt(0) (:1316)
    and the 16-byte file digest (sendFiles :1148).  Integers are little-endian (BufferedOutputChannel.java:50)."""
    h = hashlib.sha256()
    mv = memoryview(src)
    for kind, index, off, ln in zip(rec["kind"].tolist(), rec["index"].tolist(), rec["offset"].tolist(),
                                    rec["length"].tolist()):
        if kind == EV_LITERAL:
            cur, end = off, off + ln
            while cur < end:
                piece = min(8192, end - cur)
                h.update(piece.to_bytes(4, "little"))
                h.update(mv[cur:cur + piece])
                cur += piece
        else:
            h.update((-(index + 1) & 0xFFFFFFFF).to_bytes(4, "little"))
    h.update(bytes(4))
    h.update(file_md5)
    return h.hexdigest()
