/*
 * NativeChecksum.java -- the Java side of the JNI shim (java-rsync_amd/jni/rsync_hip_jni.c).
 *
 * A maintainer adds this class to core/src/main/java/com/github/java/rsync/internal/session/ (same
 * package as the package-private Checksum, Generator and Sender) and switches the two hot methods to
 * it when the system property "rsync.hip" is true (Environment-style switch, util/Environment.java:15-25).
 * Default off: the reference path is unchanged.  See INTEGRATION.md for the call-site diffs.
 *
 * Not compiled in this repository's CI (no JDK in the build image); it is the binding a maintainer
 * would add, kept next to the C shim so the two stay in sync.
 */
package com.github.java.rsync.internal.session;

import java.nio.ByteBuffer;
import java.util.concurrent.locks.ReentrantLock;

final class NativeChecksum implements AutoCloseable {
    static final boolean ENABLED = Boolean.getBoolean("rsync.hip");
    static final int EV_LITERAL = 1;
    static final int EV_MATCH = 2;

    static {
        if (ENABLED) {
            System.loadLibrary("rsynchip_jni"); // links librsynchip.so
        }
    }

    // One context per calling thread (Generator and Sender run on separate threads, RsyncClient.java:431).
    // Every context is registered so it is destroyed exactly once: by the owning task when it ends
    // (releaseForThread() in the finally of Generator.call / Sender.call, RsyncTask) or, for threads that
    // never release, by the shutdown hook.
    private static final java.util.Set<NativeChecksum> LIVE = java.util.concurrent.ConcurrentHashMap.newKeySet();
    private static final ThreadLocal<NativeChecksum> PER_THREAD = new ThreadLocal<>();

    // The hook destroys only contexts that no thread is using: a context whose owner is still inside a native
    // call (System.exit or SIGINT during a transfer) is left to the process exit, which reclaims its device
    // memory; destroying it under the running scan would free buffers and streams the scan still uses.
    static {
        if (ENABLED) {
            Runtime.getRuntime().addShutdownHook(new Thread(() -> {
                for (NativeChecksum c : LIVE) {
                    if (c.lock.tryLock()) {
                        try {
                            c.closeLocked();
                        } finally {
                            c.lock.unlock();
                        }
                    }
                }
            }, "rsync-hip-close"));
        }
    }

    /** The node's GPUs this process uses (system property rsync.hip.devices: devices 0 .. n-1). */
    static int devices() {
        return Math.max(1, Integer.getInteger("rsync.hip.devices", 1));
    }

    static NativeChecksum forThread() {
        NativeChecksum c = PER_THREAD.get();
        if (c == null) {
            int devices = devices();
            c = new NativeChecksum(Integer.getInteger("rsync.hip.device",
                    (int) (Thread.currentThread().getId() % devices)), devices);
            PER_THREAD.set(c);
            LIVE.add(c);
        }
        return c;
    }

    /**
     * More than one live NativeChecksum: each holds a context on every GPU of the device set, so the GPUs hold
     * several contexts each (trim() between segments, INTEGRATION.md).
     */
    static boolean sharesDevice() {
        return LIVE.size() > 1;
    }

    /** Destroys the calling thread's context, if it has one (idempotent). */
    static void releaseForThread() {
        NativeChecksum c = PER_THREAD.get();
        if (c != null) {
            PER_THREAD.remove();
            c.close();
        }
    }

    // The thread's home context (single-file calls; device = thread id mod rsync.hip.devices, or rsync.hip.device)
    // and its device set: one context per GPU of the set, created on the first segment call, over which the
    // segment calls split their files (rsh_*_batch_multi).  set[device] is ctx (set = {ctx} when the home device
    // lies outside the set, rsync.hip.device >= rsync.hip.devices).
    private long ctx;
    private final long[] set;
    // Held for every native call and by close(): a context is never destroyed under a running scan.  One
    // thread uses a context, so the lock is uncontended except against close() and the shutdown hook.
    private final ReentrantLock lock = new ReentrantLock();

    private NativeChecksum(int device, int devices) {
        ctx = ctxCreate(device);
        set = new long[device < devices ? devices : 1];
        set[device < devices ? device : 0] = ctx;
    }

    @Override
    public void close() {
        lock.lock();
        try {
            closeLocked();
        } finally {
            lock.unlock();
        }
    }

    private void closeLocked() {
        for (int d = 0; d < set.length; d++) {
            if (set[d] != 0 && set[d] != ctx) {
                ctxDestroy(set[d]);
            }
            set[d] = 0;
        }
        if (ctx != 0) {
            ctxDestroy(ctx);
            ctx = 0;
        }
        LIVE.remove(this);
    }

    /**
     * Releases the context's pass-sized buffers (rsh_ctx_trim: the segment and Receiver passes' HBM, the batched
     * scan's tables).  The segment loops call it after a segment when more than one context shares the GPU
     * (INTEGRATION.md "Per-context memory").
     */
    public void trim() {
        lock.lock();
        try {
            ctxTrim(handle());
            for (long c : set) {
                if (c != 0 && c != ctx) {
                    ctxTrim(c);
                }
            }
        } finally {
            lock.unlock();
        }
    }

    /** The live handle; the lock is held.  A closed context throws (the shim also rejects handle 0). */
    private long handle() {
        if (ctx == 0) {
            throw new IllegalStateException("NativeChecksum context is closed");
        }
        return ctx;
    }

    /** The device set's live handles, creating the contexts not made yet; the lock is held. */
    private long[] handles() {
        handle();
        for (int d = 0; d < set.length; d++) {
            if (set[d] == 0) {
                set[d] = ctxCreate(d);
            }
        }
        return set;
    }

    /** Generator.java:886-895: weak[i] and strong[i*dl .. i*dl+dl) for every chunk of the basis. */
    void blockSums(ByteBuffer basis, long size, Checksum.Header h, byte[] seed, int[] weak, byte[] strong) {
        lock.lock();
        try {
            blockSums(handle(), basis, size, toArray(h), seed, weak, strong);
        } finally {
            lock.unlock();
        }
    }

    /** As blockSums for a basis of any size held in several direct buffers (FileView.readPieces()). */
    void blockSums(ByteBuffer[] basis, long size, Checksum.Header h, byte[] seed, int[] weak, byte[] strong) {
        lock.lock();
        try {
            blockSumsBuffers(handle(), basis, size, toArray(h), seed, weak, strong);
        } finally {
            lock.unlock();
        }
    }

    /**
     * Sender.java:1235-1327: returns {kind, offset, length, index | count << 32} quadruples; the caller
     * replays them with sendDataFrom / putInt(-(index + j + 1)) and writes putInt(0) + fileMd5.
     */
    long[] matchScan(ByteBuffer source, long size, Checksum.Header h, int[] weak, byte[] strong, byte[] seed,
            byte[] fileMd5, long[] sizes) {
        lock.lock();
        try {
            return matchScan(handle(), source, size, toArray(h), weak, strong, seed, fileMd5, sizes);
        } finally {
            lock.unlock();
        }
    }

    /** As matchScan for a source of any size held in several direct buffers (FileView.readPieces()). */
    long[] matchScan(ByteBuffer[] source, long size, Checksum.Header h, int[] weak, byte[] strong, byte[] seed,
            byte[] fileMd5, long[] sizes) {
        lock.lock();
        try {
            return matchScanBuffers(handle(), source, size, toArray(h), weak, strong, seed, fileMd5, sizes);
        } finally {
            lock.unlock();
        }
    }

    /** As blockSums, reading the file natively (FileView semantics); true = read error (FileViewException). */
    boolean blockSumsFile(String path, long size, Checksum.Header h, byte[] seed, int[] weak, byte[] strong) {
        lock.lock();
        try {
            return blockSumsFile(handle(), path, size, toArray(h), seed, weak, strong);
        } finally {
            lock.unlock();
        }
    }

    /** As matchScan, reading the file natively; sizes = {sizeLiteral, sizeMatch, readError}. */
    long[] matchScanFile(String path, long size, Checksum.Header h, int[] weak, byte[] strong, byte[] seed,
            byte[] fileMd5, long[] sizes) {
        lock.lock();
        try {
            return matchScanFile(handle(), path, size, toArray(h), weak, strong, seed, fileMd5, sizes);
        } finally {
            lock.unlock();
        }
    }

    /**
     * A segment's Generator pass in one call (Generator.itemizeSegment, Generator.java:558-614): basis[f] holds
     * file f's bytes in one or more direct buffers, headers[f] its 3-arg Checksum.Header; weak[f] / strong[f]
     * receive its sums.  One device launch per GPU covers every file of the segment: with rsync.hip.devices > 1 the
     * files are split over the thread's contexts on every GPU (rsh_block_sums_batch_multi).
     */
    void blockSumsSegment(ByteBuffer[][] basis, long[] sizes, Checksum.Header[] headers, byte[] seed, int[][] weak,
            byte[][] strong) {
        Segment s = new Segment(basis, headers);
        lock.lock();
        try {
            if (set.length > 1) {
                blockSumsBatchMulti(handles(), s.buffers, s.filePieces, sizes, s.headers, seed, weak, strong);
            } else {
                blockSumsBatch(handle(), s.buffers, s.filePieces, sizes, s.headers, seed, weak, strong);
            }
        } finally {
            lock.unlock();
        }
    }

    /**
     * A segment's Sender pass in one call (Sender.sendFiles, Sender.java:1098-1148): returns, per file, its
     * events as {kind, offset, length, index | count << 32} quadruples (the caller replays each file's as
     * matchScan's, Sender.java:794-809 / 1274 / 1316); fileMd5[f] and sizes[f] = {sizeLiteral, sizeMatch}.
     * The files' MD5s run on the host's cores beside the device work.  With rsync.hip.devices > 1 the files are split
     * over the thread's contexts on every GPU (rsh_match_scan_batch_multi), results in file order.
     */
    long[][] matchScanSegment(ByteBuffer[][] source, long[] fileSizes, Checksum.Header[] headers, int[][] weak,
            byte[][] strong, byte[] seed, byte[][] fileMd5, long[][] sizes) {
        Segment s = new Segment(source, headers);
        int nf = headers.length;
        byte[] md5 = new byte[16 * nf];
        long[] per = new long[3 * nf];
        long[] flat;
        lock.lock();
        try {
            flat = set.length > 1
                    ? matchScanBatchMulti(handles(), s.buffers, s.filePieces, fileSizes, s.headers, weak, strong, seed,
                            md5, per)
                    : matchScanBatch(handle(), s.buffers, s.filePieces, fileSizes, s.headers, weak, strong, seed, md5,
                            per);
        } finally {
            lock.unlock();
        }
        long[][] events = new long[nf][];
        int at = 0;
        for (int f = 0; f < nf; f++) {
            int len = (int) (4 * per[3 * f]);
            events[f] = java.util.Arrays.copyOfRange(flat, at, at + len);
            at += len;
            System.arraycopy(md5, 16 * f, fileMd5[f], 0, 16);
            sizes[f][0] = per[3 * f + 1];
            sizes[f][1] = per[3 * f + 2];
        }
        return events;
    }

    /** One file's precomputed table (the Generator's segment hook, INTEGRATION.md). */
    static final class Sums {
        final Checksum.Header header;
        final int[] weak;
        final byte[] strong;

        Sums(Checksum.Header header, int[] weak, byte[] strong) {
            this.header = header;
            this.weak = weak;
            this.strong = strong;
        }
    }

    /** The flat argument form of a segment: every file's buffers in order, the count per file, 4 ints per header. */
    private static final class Segment {
        final ByteBuffer[] buffers;
        final int[] filePieces;
        final int[] headers;

        Segment(ByteBuffer[][] files, Checksum.Header[] hs) {
            int total = 0;
            for (ByteBuffer[] f : files) {
                total += f.length;
            }
            buffers = new ByteBuffer[total];
            filePieces = new int[files.length];
            headers = new int[4 * hs.length];
            int b = 0;
            for (int f = 0; f < files.length; f++) {
                filePieces[f] = files[f].length;
                for (ByteBuffer x : files[f]) {
                    buffers[b++] = x;
                }
                System.arraycopy(toArray(hs[f]), 0, headers, 4 * f, 4);
            }
        }
    }

    /**
     * Receiver.combineDataToFile (Receiver.java:459-555): result = {tokensUsed, targetLength, sizeLiteral,
     * sizeMatch}; returns true when the deferred write left the replica as the file.
     */
    boolean receiverCombine(ByteBuffer tokens, long tokensLen, Checksum.Header h, ByteBuffer replica, long replicaLen,
            boolean deferWrite, ByteBuffer target, long targetCap, long[] result, byte[] md5) {
        lock.lock();
        try {
            return receiverCombine(handle(), tokens, tokensLen, toArray(h), replica, replicaLen, deferWrite, target,
                    targetCap, result, md5);
        } finally {
            lock.unlock();
        }
    }

    private static int[] toArray(Checksum.Header h) {
        return new int[] { h.getChunkCount(), h.getBlockLength(), h.getDigestLength(), h.getRemainder() };
    }

    static native long ctxCreate(int device);

    static native void ctxDestroy(long ctx);

    static native void ctxTrim(long ctx);

    static native int blockLengthFor(long fileSize);

    static native int digestLengthFor(long fileSize, int blockLength, int minDigestLength);

    static native void blockSums(long ctx, ByteBuffer data, long n, int[] header, byte[] seed, int[] weakOut,
            byte[] strongOut);

    static native long[] matchScan(long ctx, ByteBuffer src, long n, int[] header, int[] weak, byte[] strong,
            byte[] seed, byte[] fileMd5Out, long[] sizesOut);

    static native void blockSumsBuffers(long ctx, ByteBuffer[] data, long n, int[] header, byte[] seed,
            int[] weakOut, byte[] strongOut);

    static native long[] matchScanBuffers(long ctx, ByteBuffer[] src, long n, int[] header, int[] weak,
            byte[] strong, byte[] seed, byte[] fileMd5Out, long[] sizesOut);

    static native boolean blockSumsFile(long ctx, String path, long size, int[] header, byte[] seed, int[] weakOut,
            byte[] strongOut);

    static native long[] matchScanFile(long ctx, String path, long size, int[] header, int[] weak, byte[] strong,
            byte[] seed, byte[] fileMd5Out, long[] sizesOut);

    static native void blockSumsBatch(long ctx, ByteBuffer[] data, int[] filePieces, long[] sizes, int[] headers,
            byte[] seed, int[][] weakOut, byte[][] strongOut);

    static native long[] matchScanBatch(long ctx, ByteBuffer[] src, int[] filePieces, long[] sizes, int[] headers,
            int[][] weak, byte[][] strong, byte[] seed, byte[] fileMd5Out, long[] perFileOut);

    static native void blockSumsBatchMulti(long[] ctxs, ByteBuffer[] data, int[] filePieces, long[] sizes, int[] headers,
            byte[] seed, int[][] weakOut, byte[][] strongOut);

    static native long[] matchScanBatchMulti(long[] ctxs, ByteBuffer[] src, int[] filePieces, long[] sizes,
            int[] headers, int[][] weak, byte[][] strong, byte[] seed, byte[] fileMd5Out, long[] perFileOut);

    static native boolean receiverCombine(long ctx, ByteBuffer tokens, long tokensLen, int[] header,
            ByteBuffer replica, long replicaLen, boolean deferWrite, ByteBuffer target, long targetCap,
            long[] resultOut, byte[] md5Out);
}
