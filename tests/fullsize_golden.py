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
    # BASELINE config 3: 64 GiB basis KEY ^ 3 scanned under the B = 131072 override (the rule's 2^18 is rejected
    # by the Sender, Checksum.java:81-82), dl = 5; the source is the basis with the block at 5 GiB reversed and
    # the block at 40 GiB rewritten from splitmix(B, KEY ^ 0x3E5) (test_gpu_fullsize.py::test_config3_64GiB).
    # Too large to hold twice in the build container: make_fullsize.py streams it through a file.
    "config3_edit": (64 << 30, 131072, 5, "rev5g_fill40g"),
}
BASIS_KEY = {"config2": KEY ^ 2, "config3": KEY ^ 3, "config5": KEY ^ 5}
CONFIG3_FILL_KEY = KEY ^ 0x3E5

# BASELINE config 4: a list of 128 MiB files (1024 over 8 GPUs), B = 8192 by the rule, dl = 3, each file its own
# splitmix stream (bench.py --workload files builds exactly these).  "half": every other block of each file's
# basis replaced from the stream KEY_EDIT ^ key(i); "identical": the basis is the source.
CONFIG4_FILES, CONFIG4_FILE_BYTES, CONFIG4_B, CONFIG4_DL = 1024, 128 << 20, 8192, 3
KEY_EDIT = KEY | 0xED17


def config4_key(i):
    """Source stream of file i of the config-4 list (bench.py main_files)."""
    return KEY ^ (i << 20) ^ 0x4F11E5


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
