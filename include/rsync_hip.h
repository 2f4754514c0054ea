/*
 * rsync_hip.h -- C-ABI of librsynchip.so: java-rsync's delta-transfer checksum path on MI355X (gfx950).
 *
 * The reference (alpapad/java-rsync, Java 8) has no native/FFI seam; the seam this library fills is
 * the two private hot methods and their helpers (paths relative to
 * core/src/main/java/com/github/java/rsync/internal/):
 *
 *   Generator.sendItemizeAndChecksums  session/Generator.java:866-909  -> rsh_block_sums[_device]
 *   Sender.sendMatchesAndData          session/Sender.java:1235-1327   -> rsh_match_scan[_device]
 *   Sender.skipMatchSendData           session/Sender.java:1386-1399   -> rsh_match_scan (block_length 0)
 *   Generator.getBlockLengthFor        session/Generator.java:198-206  -> rsh_block_length_for
 *   Generator.getDigestLength          session/Generator.java:208-212  -> rsh_digest_length_for
 *   Checksum.Header(int,int,long)      session/Checksum.java:94-113    -> rsh_header_make
 *   Checksum.Header(int,int,int,int)   session/Checksum.java:75-92     -> rsh_header_validate
 *   Sender.sendDataFrom + putInt(...)  session/Sender.java:794-809,1274,1316,1148 -> rsh_tokens_write
 *
 * A JNI shim (java-rsync_amd/jni/) binds these for the Java side; see INTEGRATION.md.
 * Plain pointers and sizes only; the caller owns every host buffer.  One rsh_ctx per calling thread
 * (the reference runs Generator and Sender on separate threads, RsyncClient.java:431); contexts are
 * independent and may target different devices (file-parallel sharding).
 */
#ifndef RSYNC_HIP_H
#define RSYNC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSH_ABI_VERSION 5

/* Status codes (the JNI shim maps them onto the reference's exception types). */
#define RSH_OK 0
#define RSH_E_INVAL (-1)    /* bad argument (IllegalArgumentException)                      */
#define RSH_E_PROTOCOL (-2) /* header fails Checksum.Header 4-arg validation (RsyncProtocolException,
                               Connection.java:28-38)                                        */
#define RSH_E_OVERFLOW (-3) /* chunk count > Integer.MAX_VALUE (Checksum.ChunkOverflow, :107-111) */
#define RSH_E_NOSPACE (-4)  /* event buffer too small; *n_ev holds the count needed          */
#define RSH_E_DEVICE (-5)   /* HIP runtime / kernel failure, or no gfx950 device present     */
#define RSH_E_NOMEM (-6)    /* host or device allocation failed                              */
#define RSH_E_BUSY (-7)     /* the context is serving a call on another thread               */
#define RSH_E_NOTFOUND (-8) /* the file does not exist (FileViewNotFound, FileView.java:74-75)    */
#define RSH_E_OPEN (-9)     /* the file cannot be opened (FileViewOpenFailed, FileView.java:76-78) */

/* Checksum.Header; wire order of Connection.sendChecksumHeader (Connection.java:40-45) is
 * chunk_count, block_length, digest_length, remainder (4 x little-endian int32). */
typedef struct {
    int32_t chunk_count;
    int32_t block_length;
    int32_t digest_length;
    int32_t remainder;
} rsh_header;

/* One Sender action.  RSH_EV_LITERAL = one sendDataFrom(buf, offset, length) call (length > 0; the
 * 8 KiB token split happens at replay, Sender.java:794-809).  RSH_EV_MATCH = `count` consecutive
 * putInt(-(i+1)) for chunks index .. index+count-1, matched at consecutive windows starting at file
 * offset `offset`; `length` = the bytes those windows add to sizeMatch (Sender.java:1269). */
enum { RSH_EV_LITERAL = 1, RSH_EV_MATCH = 2 };
typedef struct {
    int64_t offset;
    int64_t length;
    int32_t kind;
    int32_t index;
    int32_t count;
    int32_t reserved;
} rsh_event;

/* Per-scan counters (diagnostics; not part of the reference's output). */
typedef struct {
    int64_t chain_matches;   /* matches resolved by the aligned speculation fast path          */
    int64_t events;          /* candidate events the resolver evaluated                       */
    int64_t probe_launches;  /* range-probe kernel launches                                   */
    int64_t host_md5_windows;/* single-window digests computed on the host (resolver misses)  */
    int64_t flushes;         /* FileView.isFull flushes (Sender.java:1294-1302)                */
    double device_ms;        /* wall time of the bulk device phase (speculation kernels + copies) */
    double resolver_ms;      /* host resolver time (including its small device round trips)   */
    double table_ms;         /* host index of the received table (chained hash, built lazily)  */
    int64_t head_steps;      /* resolver steps taken before the aligned speculation landed    */
    int64_t speculation_aborted; /* 1: the scan ended first and the speculation launch was stopped;
                                    2: the scan ended in head mode before the speculation was launched;
                                    3: a tentative launch was stopped at once (the lead windows differ) */
    int64_t device_bytes;    /* source bytes the device work of this scan read: speculations that ran to
                                completion (a stopped one counts 0), probed ranges (+ B - 1 per interval),
                                weak-sum windows, gathered bytes and copied digest windows (ABI 2)  */
    int64_t phase_launches;  /* phase-shifted speculations launched (chains at kB + delta, ABI 2)   */
    int64_t phase_matches;   /* matches resolved from a phase-shifted speculation (ABI 2)           */
    double spec_kernel_ms;   /* the aligned speculation's K1 alone (HIP events on its stream), when it ran
                                to completion; 0 otherwise (ABI 2)                                   */
    double phase_kernel_ms;  /* the phase-shifted speculations' K1s that ran to completion, summed (ABI 2) */
    int64_t phase_guesses;   /* phase-shifted speculations started before the resolver, at the phase found
                                past a sampled run's end (ABI 2)                                     */
} rsh_scan_stats;

typedef struct rsh_ctx rsh_ctx;

int rsh_abi_version(void);
const char* rsh_strerror(int status);
/* Text of the calling thread's last HIP failure (error string and source line), "" if none. */
const char* rsh_last_error(void);
int rsh_device_count(int* count);
int rsh_ctx_create(int device, rsh_ctx** out);
void rsh_ctx_destroy(rsh_ctx* ctx);
/* hipStream_t the context launches on (opaque), for callers composing with their own streams. */
void* rsh_ctx_stream(rsh_ctx* ctx);

/* ---- sizing / header (pure host functions) ---- */
int32_t rsh_block_length_for(int64_t file_size);                                    /* Generator.java:198-206 */
int32_t rsh_digest_length_for(int64_t file_size, int32_t block_length, int32_t min_digest_length); /* :208-212,:873 */
int rsh_header_make(int32_t block_length, int32_t digest_length, int64_t file_size, rsh_header* out);
int rsh_header_validate(const rsh_header* h);

/* ---- Generator: per-chunk weak + MD5(chunk || seed)[0:digest_length] (Generator.java:886-895) ----
 * weak_out[chunk_count]; strong_out[chunk_count * digest_length].  Host buffers. */
int rsh_block_sums(rsh_ctx* ctx, const uint8_t* data, int64_t n, const rsh_header* h, const uint8_t seed[4],
                   int32_t* weak_out, uint8_t* strong_out);
/* Device-resident form: d_data, d_weak, d_strong are device pointers; runs on the context stream and
 * returns after the work is enqueued (rsh_ctx_sync waits). */
int rsh_block_sums_device(rsh_ctx* ctx, const void* d_data, int64_t n, const rsh_header* h, const uint8_t seed[4],
                          void* d_weak, void* d_strong);
int rsh_ctx_sync(rsh_ctx* ctx);
/* Releases the context's pass-sized buffers -- the segment passes' HBM (rsh_*_batch: up to 2 x the segment_bytes
 * budget, 16 GiB by default), the Receiver passes' and the host-input staging -- after waiting for the context's
 * streams.  The next call that needs them allocates them again.  The batched scan's state (chunk index, hit map,
 * descriptors, pinned event buffers: bounded by the largest segment's chunks and option chain_map_bytes) stays, so
 * that the next segment scan costs what the previous one did.  A JVM holding
 * several contexts on one GPU (a local transfer's Generator and Sender) calls it after each segment; see
 * INTEGRATION.md "Per-context memory".  Replaces nothing in the reference (its buffers are Java heap). */
int rsh_ctx_trim(rsh_ctx* ctx);

/* ---- Sender (Sender.java:1098-1148 per-file glue, :1235-1327 scan, :1386-1399 new file) ----
 * h: the header received from the Generator (validated here exactly as Connection.receiveChecksumHeader
 * does); weak[chunk_count], strong[chunk_count * digest_length]: the received table.
 * Events are written to ev[0..ev_cap); *n_ev receives the count (RSH_E_NOSPACE if ev_cap is short).
 * file_md5 = MD5 of the whole source (Sender.java:1241,1326); literal/matched = sizeLiteral/sizeMatch. */
int rsh_match_scan(rsh_ctx* ctx, const uint8_t* src, int64_t n, const rsh_header* h, const int32_t* weak,
                   const uint8_t* strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap, int64_t* n_ev,
                   uint8_t file_md5[16], int64_t* literal, int64_t* matched, rsh_scan_stats* stats);
/* Device-resident form: source and table already in HBM (d_src, d_weak, d_strong).  The serial
 * whole-file MD5 is not computed here (see rsh_file_md5); everything else is identical. */
int rsh_match_scan_device(rsh_ctx* ctx, const void* d_src, int64_t n, const rsh_header* h, const void* d_weak,
                          const void* d_strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap,
                          int64_t* n_ev, int64_t* literal, int64_t* matched, rsh_scan_stats* stats);

/* Tiled form for sources larger than the device (BASELINE config 3; FileView streams any file through a
 * 10*B window, FileView.java:235-278): the source stays in host memory and HBM holds one tile of tile_bytes
 * (rounded to a multiple of B, at least 16*B; 0 = 4 GiB) plus a 16*B halo at a time, paged in as the scan
 * advances; the aligned speculation runs tile by tile.  Events, literal and matched are those of
 * rsh_match_scan.  file_md5 may be NULL (the serial whole-file digest is then skipped). */
int rsh_match_scan_tiled(rsh_ctx* ctx, const uint8_t* src, int64_t n, const rsh_header* h, const int32_t* weak,
                         const uint8_t* strong, const uint8_t seed[4], int64_t tile_bytes, rsh_event* ev,
                         int64_t ev_cap, int64_t* n_ev, uint8_t file_md5[16], int64_t* literal, int64_t* matched,
                         rsh_scan_stats* stats);

/* After RSH_E_NOSPACE from rsh_match_scan[_device] the context keeps that scan's events: fetch them into
 * a buffer of at least *n_ev entries without recomputing (valid until the context's next scan). */
int rsh_fetch_events(rsh_ctx* ctx, rsh_event* ev, int64_t ev_cap, int64_t* n_ev);

/* Whole-file MD5 on the host (one serial chain; runs beside the device work). */
int rsh_file_md5(const uint8_t* data, int64_t n, uint8_t out[16]);

/* ---- channel bytes ----
 * Exact bytes Sender writes for one file: per literal event the 8 KiB-split putInt(len)+bytes tokens,
 * per matched chunk putInt(-(index+1)), then putInt(0) and the 16-byte file MD5. */
int64_t rsh_tokens_size(const rsh_event* ev, int64_t n_ev);
int rsh_tokens_write(const uint8_t* src, const rsh_event* ev, int64_t n_ev, const uint8_t file_md5[16],
                     uint8_t* out, int64_t cap);
/* Generator channel bytes: header + per chunk putInt(weak) + digest_length bytes. */
int64_t rsh_generator_bytes(const rsh_header* h, const int32_t* weak, const uint8_t* strong, uint8_t* out,
                            int64_t cap);

/* ---- batched files (one segment of the file list) ----
 * The reference handles a segment's files one after another: the Generator sends every file's header +
 * table (Generator.java:558-614, sendItemizeAndChecksums :866-909 per file) and the Sender answers each in
 * turn (Sender.sendFiles :1098-1148 -> sendMatchesAndData :1235-1327).  The batched forms take all the
 * files of a segment at once, so their kernels fill the device: one K1 launch for every file's block
 * sums, and one resolver per file whose device round trips are gathered into one launch per round.
 * Results are per file and identical to the single-file calls.  All pointers in a job are device
 * pointers except ev (host).  Returns RSH_OK, or the first failing job's status (every job's own status
 * is in its `status`). */
typedef struct {
    const void* d_data;  /* the basis file */
    int64_t n;
    rsh_header h;        /* as for rsh_block_sums (3-arg Checksum.Header semantics) */
    void* d_weak;        /* out: chunk_count weak sums */
    void* d_strong;      /* out: chunk_count * digest_length digest bytes */
} rsh_block_job;
int rsh_block_sums_batch_device(rsh_ctx* ctx, const rsh_block_job* jobs, int32_t njobs, const uint8_t seed[4]);

typedef struct {
    const void* d_src;     /* the source file */
    int64_t n;
    rsh_header h;          /* the received header (validated as by rsh_match_scan) */
    const void* d_weak;    /* the received table */
    const void* d_strong;
    rsh_event* ev;         /* host, caller-owned: ev_cap entries */
    int64_t ev_cap;
    int64_t n_ev;          /* out: event count (RSH_E_NOSPACE in status if > ev_cap; events then lost) */
    int64_t literal;       /* out */
    int64_t matched;       /* out */
    int32_t status;        /* out: RSH_OK or an error code for this file */
    int32_t reserved;
} rsh_scan_job;
/* stats (optional): summed over the files (device_ms / resolver_ms: wall time of the whole batch). */
int rsh_match_scan_batch_device(rsh_ctx* ctx, rsh_scan_job* jobs, int32_t njobs, const uint8_t seed[4],
                                rsh_scan_stats* stats);

/* ---- file ingest: the FileView reads of the two passes (FileView.java:51-80 open, :187-278 reads) ----
 * The file is read straight into pinned staging buffers by several threads (large preads), copied to the
 * device piece by piece while the next piece is read, and summed there.  `size` is the size the caller's
 * FileInfo holds (FileView reads exactly that many bytes): a file that ends early or fails to read is
 * zero-filled from that point, the result is computed over those bytes, and *read_error is set -- the
 * reference's deferred FileViewException at close() (the Sender then flips md5[0], Sender.java:1136-1143).
 * size == 0 opens nothing (FileView.java:62-72).
 * rsh_block_sums_file: the Generator pass; the device holds two pieces at a time, so the file may be
 * larger than HBM.  rsh_match_scan_file: the Sender pass; the source is assembled in HBM while a host
 * thread digests the pieces in order (the whole-file MD5 of Sender.java:1241,1326). */
int rsh_block_sums_file(rsh_ctx* ctx, const char* path, int64_t size, const rsh_header* h, const uint8_t seed[4],
                        int32_t* weak_out, uint8_t* strong_out, int32_t* read_error);
int rsh_match_scan_file(rsh_ctx* ctx, const char* path, int64_t size, const rsh_header* h, const int32_t* weak,
                        const uint8_t* strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap, int64_t* n_ev,
                        uint8_t file_md5[16], int64_t* literal, int64_t* matched, rsh_scan_stats* stats,
                        int32_t* read_error);

/* ---- a file handed over as a list of host buffers ----
 * A JVM cannot hold a file above 2^31 - 1 bytes in one direct ByteBuffer, while the reference streams any
 * file size through FileView (FileView.java:51-80,235-278).  These forms take the file as pieces (each a
 * caller-owned host buffer; the file is their concatenation, in order; a chunk or window may straddle
 * two pieces) and return exactly what rsh_block_sums / rsh_match_scan return for the concatenated bytes.
 * The Sender's literal events name file offsets; the binding replays each from the pieces
 * (INTEGRATION.md).  Sources above 32 GiB are paged through HBM a tile at a time. */
typedef struct {
    const uint8_t* data;
    int64_t len;
} rsh_piece;
int rsh_block_sums_pieces(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, const rsh_header* h,
                          const uint8_t seed[4], int32_t* weak_out, uint8_t* strong_out);
int rsh_match_scan_pieces(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, const rsh_header* h,
                          const int32_t* weak, const uint8_t* strong, const uint8_t seed[4], rsh_event* ev,
                          int64_t ev_cap, int64_t* n_ev, uint8_t file_md5[16], int64_t* literal, int64_t* matched,
                          rsh_scan_stats* stats);

/* ---- a segment's files from host memory (ABI 4) ----
 * What a Java Generator / Sender holding a file-list segment in JVM buffers calls: Generator.itemizeSegment
 * (Generator.java:558-614) sends every file's header + table (sendItemizeAndChecksums :866-909 per file), and
 * Sender.sendFiles (Sender.java:1098-1148) answers each file in turn with sendMatchesAndData (:1235-1327), whose
 * last 16 bytes are the whole-file MD5 (:1241,1326).  These forms take the whole segment in one call: each file
 * is a list of caller-owned host pieces (as rsh_*_pieces), the bytes are copied to HBM (up to a budget of about
 * 16 GiB per pass; a file larger than that goes through the tiled single-file path), every file's sums or scan
 * run in the batched device forms above, and -- for the Sender -- every file's MD5 runs on the host's cores
 * beside the copies and the scan, several files per core (rsh_file_md5_batch).  Per-file results equal the
 * single-file calls'.  Returns RSH_OK, or the first failing job's status; every job's own status is in it
 * (RSH_E_NOSPACE: ev_cap was short, n_ev holds the count needed and the file's events are not kept). */
typedef struct {
    const rsh_piece* pieces; /* the basis file: the concatenation of its pieces (npieces 0: an empty file) */
    int32_t npieces;
    int32_t status;          /* out */
    rsh_header h;            /* 3-arg Checksum.Header of the file (as for rsh_block_sums) */
    int32_t* weak_out;       /* host: chunk_count weak sums */
    uint8_t* strong_out;     /* host: chunk_count * digest_length digest bytes */
} rsh_block_batch_job;
int rsh_block_sums_batch(rsh_ctx* ctx, rsh_block_batch_job* jobs, int32_t njobs, const uint8_t seed[4]);

typedef struct {
    const rsh_piece* pieces; /* the source file */
    int32_t npieces;
    int32_t status;          /* out */
    rsh_header h;            /* the received header (validated as by rsh_match_scan) */
    const int32_t* weak;     /* host: the received table */
    const uint8_t* strong;
    rsh_event* ev;           /* host, caller-owned: ev_cap entries */
    int64_t ev_cap;
    int64_t n_ev;            /* out */
    int64_t literal;         /* out: sizeLiteral */
    int64_t matched;         /* out: sizeMatch */
    uint8_t file_md5[16];    /* out: MD5 of the whole source (Sender.java:1241,1326) */
} rsh_scan_batch_job;
/* stats (optional): summed over the files, as rsh_match_scan_batch_device's. */
int rsh_match_scan_batch(rsh_ctx* ctx, rsh_scan_batch_job* jobs, int32_t njobs, const uint8_t seed[4],
                         rsh_scan_stats* stats);

/* Whole-file MD5s of many files (pure host; no context): md5[16] of each job = MD5 of its pieces'
 * concatenation.  Independent files run side by side, up to 16 per core (AVX-512; 8 with AVX2), on `threads`
 * threads (0 = the process's cores, cgroup quota included). */
typedef struct {
    const rsh_piece* pieces;
    int32_t npieces;
    int32_t reserved;
    uint8_t md5[16];         /* out */
} rsh_md5_job;
int rsh_file_md5_batch(rsh_md5_job* jobs, int32_t njobs, int32_t threads);

/* ---- Receiver (Receiver.java:459-555 combineDataToFile, :557-578 copies, :204-209 blockSize) ----
 * Replays one file's de-multiplexed token stream -- putInt(len)+bytes, putInt(-(i+1)), putInt(0), exactly
 * what rsh_tokens_write produces -- against the replica (the basis the Generator summed; NULL when the
 * Receiver has none: matches are then skipped, :487-494).  The target receives the literal bytes and the
 * replica blocks in token order; with defer_write (and a replica) nothing is written while the matches
 * are 0, 1, 2, ... in order with no literal, and a stream that matched all chunk_count blocks that way
 * leaves the file intact (out->intact = 1, the replica is the result, :529-545).  out->md5 is the digest
 * the Receiver computes over the file content; compare it with the 16 bytes that follow the stream
 * (isRemoteAndLocalFileIdentical, :824-842).  Status: RSH_E_PROTOCOL for a block index out of range or a
 * match against block_length 0 (RsyncProtocolException, :480-485); RSH_E_INVAL for a truncated stream
 * or a replica shorter than a block it names (IllegalStateException, :1012-1017); RSH_E_NOSPACE when
 * target_cap < out->target_len (nothing written). */
typedef struct {
    int64_t tokens_used;  /* bytes consumed, including the terminating putInt(0) */
    int64_t target_len;   /* bytes of the rebuilt file written to the target (0 when intact) */
    int64_t literal;      /* sizeLiteral */
    int64_t matched;      /* sizeMatch */
    int32_t intact;       /* combineDataToFile's return value */
    int32_t reserved;
    uint8_t md5[16];
} rsh_combine_result;
/* Host buffers (the replica is uploaded, the target downloaded). */
int rsh_receiver_combine(rsh_ctx* ctx, const uint8_t* tokens, int64_t tokens_len, const rsh_header* h,
                         const uint8_t* replica, int64_t replica_len, int32_t defer_write, uint8_t* target,
                         int64_t target_cap, rsh_combine_result* out);
/* Device-resident replica and target (the tokens stay in host memory); the blocks are gathered by a
 * kernel, the literal bytes uploaded in one copy; the digest is computed on the host from the result. */
int rsh_receiver_combine_device(rsh_ctx* ctx, const uint8_t* tokens, int64_t tokens_len, const rsh_header* h,
                                const void* d_replica, int64_t replica_len, int32_t defer_write, void* d_target,
                                int64_t target_cap, rsh_combine_result* out);

/* ---- a segment's Receiver from host memory (Receiver.receiveFiles, Receiver.java:1145-1263: combineDataToFile
 * :459-556 and isRemoteAndLocalFileIdentical :824-842 for each file in turn) ----
 * One job per file: its de-multiplexed token stream, its replica as host pieces (nreplica 0: no replica), the
 * target buffer.  Each job gets rsh_receiver_combine's result and its own status (RSH_E_PROTOCOL / RSH_E_INVAL /
 * RSH_E_NOSPACE as there); a call that fails as a whole leaves every file it did not finish with its code.  The
 * rebuilt files are gathered on the device (the token streams and the replica ranges they name go up, every file's
 * blocks and literals are one gather launch, the targets come back) in passes of at most option segment_bytes,
 * overlapped; the verify digests -- one serial MD5 chain per file -- run on the host's cores beside the copies,
 * up to 16 files per core (md5_mb.cpp), over the replica ranges and literal bytes the tokens name, which are
 * exactly the rebuilt file's bytes.  A file is never split across passes: one whose token stream, replica ranges and
 * target together exceed segment_bytes gets a pass of its own of that size, and fails with RSH_E_NOMEM when the
 * device cannot hold it (the single-file rsh_receiver_combine's limit: its target and replica in HBM at once). */
typedef struct {
    const uint8_t* tokens;    /* host: the file's token stream, ending with putInt(0) */
    int64_t tokens_len;
    rsh_header h;             /* the file's checksum header (as sent by the Generator) */
    const rsh_piece* replica; /* host: the replica as pieces (their concatenation); NULL / 0 pieces: none */
    int32_t nreplica;
    int32_t defer_write;
    uint8_t* target;          /* host, caller-owned: target_cap bytes (nothing written when intact) */
    int64_t target_cap;
    int32_t status;           /* out */
    int32_t reserved;
    rsh_combine_result res;   /* out */
} rsh_combine_job;
int rsh_receiver_combine_batch(rsh_ctx* ctx, rsh_combine_job* jobs, int32_t njobs);

/* ---- a segment over several GPUs (ABI 5) ----
 * north_star: "files shard embarrassingly across the 8 GPUs of one node".  In the reference one thread walks every
 * file of a transfer: the Generator sums a segment's files in turn (Generator.java:558-614,806-860), one Sender thread
 * answers each (Sender.sendFiles, Sender.java:978-1170) and one Receiver thread rebuilds each (Receiver.java:1145-1263).
 * These forms take the calling thread's contexts ctxs[0 .. nctx) -- distinct contexts, typically one per GPU of the
 * node (several on one GPU also work: they run side by side there) -- split the segment's files over them by
 * rsh_shard_files, and run each context's share as the single-context call above (rsh_block_sums_batch,
 * rsh_match_scan_batch, rsh_receiver_combine_batch) on a host thread of its own, the process's cores shared evenly
 * among those threads.  No data moves between GPUs.  Every job's outputs and status are exactly what the
 * single-context call gives that file; a failure on one context marks only the files that context had not finished.
 * Returns RSH_OK, or the first failing job's status in file order (RSH_E_INVAL for a null or repeated context).
 * stats: summed over the contexts.  nctx == 1 is the single-context call. */
int rsh_block_sums_batch_multi(rsh_ctx* const* ctxs, int32_t nctx, rsh_block_batch_job* jobs, int32_t njobs,
                               const uint8_t seed[4]);
int rsh_match_scan_batch_multi(rsh_ctx* const* ctxs, int32_t nctx, rsh_scan_batch_job* jobs, int32_t njobs,
                               const uint8_t seed[4], rsh_scan_stats* stats);
/* (the Receiver's files are split by max(tokens_len, replica bytes): about the bytes each rebuilds) */
int rsh_receiver_combine_batch_multi(rsh_ctx* const* ctxs, int32_t nctx, rsh_combine_job* jobs, int32_t njobs);
/* The split (pure host): part_out[f] = the part (context) file f goes to.  Longest first by bytes (equal sizes in
 * file order), each file to the part with the fewest bytes so far (ties to the lower part): shard.py's rank rule. */
int rsh_shard_files(const int64_t* bytes, int32_t nfiles, int32_t nparts, int32_t* part_out);

/* ---- device buffers for the *_device entry points (callers without their own allocator, e.g. JNI) ---- */
int rsh_dev_alloc(rsh_ctx* ctx, int64_t bytes, void** out);
int rsh_dev_free(rsh_ctx* ctx, void* p);
int rsh_memcpy_h2d(rsh_ctx* ctx, void* dst, const void* src, int64_t bytes);  /* synchronous */
int rsh_memcpy_d2h(rsh_ctx* ctx, void* dst, const void* src, int64_t bytes);  /* synchronous */

/* ---- synthetic input for benchmarks: splitmix64 counter stream generated on the device ---- */
int rsh_fill_splitmix_device(rsh_ctx* ctx, void* d_out, int64_t n, uint64_t key, int64_t byte_offset);

#ifdef __cplusplus
}
#endif
#endif
