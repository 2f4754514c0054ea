"""INTEGRATION.md's Sender segment diff (the read-ahead of transfer requests in Sender.sendFiles) against the
reference's per-file loop, as a model: both loops restated in Python, function for function, over random index
streams.  No JDK exists here, so the Java diff itself cannot run; the model pins its
ordering rule -- every queued answer is written before anything else -- by checking that the channel output of the
read-ahead loop equals the per-file loop's, write for write, with the same statistics and ioError bits.

The streams mix transfer requests (files that open, fail to open -- NO_SEND -- or hit a read error), non-transfer
indices, DONEs (segment deletion, phase transitions), file-list expansions and the EOF at the top of the loop, and
protocol errors (an invalid index, a transfer request in the wrong phase), delivered in random bursts
(numBytesAvailable() == 0 between bursts).  Reference lines: core/src/main/java/com/github/java/rsync/internal/
session/Sender.java:976-1170 (sendFiles), :1113-1148 (the per-file answer), :1120-1135 (NO_SEND)."""
import random

import pytest

TRANSFER, TEAR_DOWN_1, TEAR_DOWN_2, STOP = range(4)  # TransferPhase, next() in order
PARTIAL_FILE_LIST_SIZE = 8
VANISHED, GENERAL = 1, 2  # IoError bits


class ProtocolError(Exception):
    """RsyncProtocolException"""


class Channel:
    """The de-multiplexed input (messages with a burst number each) and the output (the writes, in order).  Liveness:
    the peer is assumed to send its next burst only once every transfer request it sent has been answered (the
    strictest peer), so reading past a burst's end with an answer still owed is a deadlock."""

    def __init__(self, msgs):
        self.msgs, self.at, self.out = msgs, 0, []
        self.owed = 0  # transfer requests read and not answered yet

    def num_bytes_available(self):  # AutoFlushableRsyncDuplexChannel.numBytesAvailable
        if self.at == 0 or self.at >= len(self.msgs):
            return 0
        return 1 if self.msgs[self.at][-1] == self.msgs[self.at - 1][-1] else 0

    def decode_index(self):
        if self.at >= len(self.msgs):
            raise AssertionError("the loop read past the peer's last message (it would block forever)")
        if self.owed and self.at > 0 and self.msgs[self.at][-1] != self.msgs[self.at - 1][-1]:
            raise AssertionError("deadlock: waiting for the peer's next burst with answers still owed")
        m = self.msgs[self.at]
        self.at += 1
        if m[0] == "XFER":
            self.owed += 1
        return m


class FileList:
    """The parts of Filelist the loop reads: segments still to expand (each with a file count) and live ones."""

    def __init__(self, live, to_expand):
        self.live = list(live)  # file counts of the expanded segments
        self.to_expand = list(to_expand)
        self.expanded = len(self.live)

    def is_expandable(self):
        return bool(self.to_expand)

    def expand_and_send(self, ch, lim):  # expandAndSendSegments: writes one segment
        n = self.to_expand.pop(0)
        self.live.append(n)
        self.expanded += 1
        ch.out.append(("SEGMENT", n, lim))
        return n


class Sender:
    """sendFiles with fileSelection == RECURSE; read_ahead = 0 is the reference's per-file loop."""

    def __init__(self, ch, flist, read_ahead):
        self.ch, self.fl, self.K = ch, flist, read_ahead
        self.pending = []
        self.stats = {"files": 0, "literal": 0, "matched": 0, "size": 0}
        self.transferred = set()

    # the condition of the two writes at the top of the loop (:982-1009)
    def expansion_due(self, in_transit, sent_eof):
        return (self.fl.is_expandable() and (self.fl.expanded == 1 or in_transit < PARTIAL_FILE_LIST_SIZE // 2)) or \
            (not self.fl.is_expandable() and not sent_eof)

    # what the reference writes for one transfer request (:1113-1148); the file's scan result is computed from
    # the request alone, so where it is computed does not matter -- only where it is written
    def answer(self, index, outcome, size):
        self.ch.owed -= 1
        if outcome == "openfail":  # :1120-1135
            self.ch.out.append(("NO_SEND", index))
            return GENERAL
        if outcome == "notfound":
            self.ch.out.append(("NO_SEND", index))
            return VANISHED
        ch = self.ch
        ch.out.append(("INDEX", index))  # sendIndexAndIflags
        ch.out.append(("HEADER", index))  # sendChecksumHeader
        ch.out.append(("TOKENS", index, size))  # sendMatchesAndData / skipMatchSendData, putInt(0)
        self.stats["literal"] += size // 3
        self.stats["matched"] += size - size // 3
        ch.out.append(("MD5", index, "bad" if outcome == "readerr" else "ok"))  # createIncorrectChecksum on a read error
        self.transferred.add(index)
        self.stats["files"] += 1
        self.stats["size"] += size
        return 0

    def read_ahead(self, index, outcome, size):  # readAhead: writes nothing
        return (index, outcome, size)

    def drain_pending(self):  # drainPending: every queued request, in arrival order
        io = 0
        for p in self.pending:
            io |= self.answer(*p)
        self.pending = []
        return io

    def send_files(self):
        ch, fl = self.ch, self.fl
        sent_eof = False
        phase = TRANSFER
        io_error = 0
        in_transit = sum(fl.live)
        try:
            while phase != STOP:
                if self.K and self.pending and (len(self.pending) >= self.K or ch.num_bytes_available() == 0 or
                                                self.expansion_due(in_transit, sent_eof)):
                    io_error |= self.drain_pending()
                if fl.is_expandable() and (fl.expanded == 1 or in_transit < PARTIAL_FILE_LIST_SIZE // 2):
                    lim = max(1, PARTIAL_FILE_LIST_SIZE - in_transit)
                    in_transit += fl.expand_and_send(ch, lim)
                if not fl.is_expandable() and not sent_eof:
                    ch.out.append(("EOF",))
                    sent_eof = True
                msg = ch.decode_index()
                kind = msg[0]
                if kind == "DONE":
                    if self.K:
                        io_error |= self.drain_pending()
                    if fl.live:  # recurse, !fileList.isEmpty()
                        removed = fl.live.pop(0)
                        if fl.live:
                            ch.out.append(("DONE",))
                        in_transit -= removed
                    if not fl.live:
                        phase += 1
                        if phase != STOP:
                            ch.out.append(("DONE",))
                elif kind in ("XFER", "NOXFER", "BAD"):
                    index = msg[1]
                    if kind == "BAD":  # no segment holds it
                        raise ProtocolError(f"invalid file index {index}")
                    if kind == "NOXFER":
                        if self.K:
                            io_error |= self.drain_pending()
                        in_transit -= 1
                        ch.out.append(("INDEX", index))
                    elif phase == TRANSFER:
                        _, _, outcome, size, _ = msg
                        if self.K:
                            self.pending.append(self.read_ahead(index, outcome, size))
                            continue
                        io_error |= self.answer(index, outcome, size)
                    else:
                        raise ProtocolError("received index in wrong phase")
                else:
                    raise ProtocolError(f"invalid index {msg}")
        except ProtocolError:
            if self.pending:
                self.drain_pending()
            raise
        assert not self.pending  # STOP is reached through a DONE, which drained
        return io_error


def random_stream(rng, errors):
    """Messages (kind, ..., burst) for a recursive transfer: live segments, later expansions, requests, DONEs."""
    live = [rng.randrange(1, 5) for _ in range(rng.randrange(1, 3))]
    to_expand = [rng.randrange(1, 5) for _ in range(rng.randrange(0, 4))]
    msgs, burst, idx = [], 0, 0
    nseg = len(live) + len(to_expand)
    for _ in range(nseg):
        for _ in range(rng.randrange(0, 9)):
            r = rng.random()
            idx += 1
            if r < 0.6:
                outcome = rng.choice(["ok"] * 6 + ["openfail", "notfound", "readerr"])
                msgs.append(["XFER", idx, outcome, rng.randrange(0, 1000)])
            else:
                msgs.append(["NOXFER", idx])
            if errors and rng.random() < 0.03:
                msgs.append(["BAD", 10 ** 6])
        msgs.append(["DONE"])
    msgs += [["DONE"], ["DONE"]]
    if errors and rng.random() < 0.3:  # a transfer request after the phase changed
        msgs.insert(len(msgs) - 1, ["XFER", 10 ** 6, "ok", 5])
    for m in msgs:
        if rng.random() < 0.35:
            burst += 1
        m.append(burst)
    return [tuple(m) for m in msgs], live, to_expand


def run(msgs, live, to_expand, K):
    ch = Channel(msgs)
    s = Sender(ch, FileList(live, to_expand), K)
    try:
        io, err = s.send_files(), None
    except ProtocolError as e:
        io, err = None, str(e)
    return ch.out, s.stats, sorted(s.transferred), io, err, ch.at


@pytest.mark.parametrize("K", [1, 2, 3, 5, 128])
def test_read_ahead_writes_what_the_per_file_loop_writes(K):
    rng = random.Random(K)
    queued_max = 0
    for trial in range(400):
        msgs, live, to_expand = random_stream(rng, errors=trial % 4 == 3)
        ref = run(msgs, live, to_expand, 0)
        got = run(msgs, live, to_expand, K)
        assert got == ref, (K, trial, msgs)
        queued_max = max(queued_max, sum(1 for m in msgs if m[0] == "XFER"))
    assert queued_max > K or K == 128  # the streams really exercise the bound


def test_read_ahead_batches_requests():
    """The model would pass trivially if it never queued: check that bursts of requests are answered together
    (the point of the diff), and that the read-ahead stops at a burst's end rather than blocking for more."""
    msgs = [("XFER", i, "ok", 10, 0) for i in range(1, 7)] + [("DONE", 1), ("DONE", 1), ("DONE", 1)]
    ch = Channel(msgs)
    s = Sender(ch, FileList([6], []), 128)
    batches = []
    orig = s.drain_pending

    def spy():
        batches.append(len(s.pending))
        return orig()
    s.drain_pending = spy
    s.send_files()
    assert batches[0] == 6 and ch.out == run(msgs, [6], [], 0)[0]
