/*
 * rsync_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded CPU restatement of java-rsync's delta-transfer
 * checksum path (Generator block sums + Sender rolling/MD5 match scan).  It is
 * the parity oracle for the HIP path and the "port" CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * link or call it; the product library (java-rsync_amd/) never does.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * core/src/main/java/com/github/java/rsync/internal/).  Parity is pinned by:
 *   - RFC 1321 appendix A.5 MD5 vectors (MD5 is the JDK MessageDigest, not
 *     vendored in the reference);
 *   - rsync-app SystemTest.java:532-628 (new-file literal sizes; 557-byte
 *     second copy = literal 0 / matched 557);
 *   - an independent Python restatement (oracle/pyref.py, stdlib hashlib)
 *     that generated tests/golden/ (no JDK exists in this image, so the Java
 *     reference itself cannot be run -- see DESIGN.md "Oracle").
 */
#ifndef RSYNC_ORACLE_H
#define RSYNC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- MD5 (RFC 1321; reference: util/MD5.java:35-41 -> JDK MessageDigest) ---- */
typedef struct {
    uint32_t h[4];
    uint64_t nbytes;
    uint8_t buf[64];
    uint32_t nbuf;
} orc_md5_ctx;

void orc_md5_init(orc_md5_ctx* c);
void orc_md5_update(orc_md5_ctx* c, const uint8_t* p, size_t n);
void orc_md5_final(orc_md5_ctx* c, uint8_t out[16]); /* resets like MessageDigest.digest() */
void orc_md5(const uint8_t* p, size_t n, uint8_t out[16]);

/* ---- Rolling (util/Rolling.java:22-64), CHAR_OFFSET = 0, signed bytes ---- */
int32_t orc_rolling_compute(const uint8_t* buf, int32_t len);
int32_t orc_rolling_add(int32_t checksum, uint8_t value);
int32_t orc_rolling_subtract(int32_t checksum, int32_t block_length, uint8_t value);

/* ---- sizing (session/Generator.java:198-236, util/Util.java:128-130) ---- */
int32_t orc_block_length_for(int64_t file_size);
int32_t orc_digest_length(int64_t file_size, int32_t block_length);

/* ---- Checksum.Header (session/Checksum.java:66-143) ---- */
typedef struct {
    int32_t chunk_count;
    int32_t block_length;
    int32_t digest_length;
    int32_t remainder;
} orc_header;

/* 3-arg ctor (Checksum.java:94-113): 0 ok, -1 ChunkOverflow. */
int orc_header_make(int32_t block_length, int32_t digest_length, int64_t file_size, orc_header* out);
/* 4-arg ctor validation (Checksum.java:75-92): 0 ok, -1 IllegalArgumentException. */
int orc_header_validate(const orc_header* h);
int32_t orc_smallest_chunk_size(const orc_header* h); /* Checksum.java:131-137 */

/* ---- Generator.sendItemizeAndChecksums hot loop (Generator.java:866-909) ---- */
void orc_generator_sums(const uint8_t* basis, int64_t n, const orc_header* h, const uint8_t seed[4],
                        int32_t* weak_out, uint8_t* strong_out /* chunk_count * digest_length */);

/* ---- Sender.sendMatchesAndData / skipMatchSendData (Sender.java:1235-1327, 1386-1399) ----
 * Events: one ORC_LIT per non-empty sendDataFrom() call (Sender.java:794-809) and one ORC_MATCH per
 * putInt(-(idx+1)) (Sender.java:1274).  The terminating putInt(0) is implicit. */
enum { ORC_LIT = 1, ORC_MATCH = 2 };
typedef struct {
    int64_t offset; /* LIT: file offset of first byte; MATCH: file offset of the matched window */
    int64_t length; /* LIT: byte count; MATCH: window length (bytes added to sizeMatch) */
    int32_t kind;
    int32_t index; /* MATCH: chunk index */
} orc_event;

typedef struct {
    orc_event* ev;
    int64_t n_ev;
    int64_t cap;
    uint8_t file_md5[16];
    int64_t literal;
    int64_t matched;
    int64_t md5_windows; /* chunk-digest computations performed (for analysis only) */
} orc_scan_result;

/* weak/strong: the chunk table as received (Sender.java:758-767), header validated by caller.
 * header->block_length == 0 selects skipMatchSendData.  Returns 0, or -1 on allocation failure. */
int orc_sender_scan(const uint8_t* src, int64_t n, const orc_header* h, const int32_t* weak,
                    const uint8_t* strong, const uint8_t seed[4], orc_scan_result* res);
void orc_scan_free(orc_scan_result* res);

/* Serialise events into the exact channel bytes the Sender writes (little-endian putInt, raw
 * literal bytes split at CHUNK_SIZE = 8192, putInt(0), then the 16-byte file MD5).
 * Returns the byte count; writes only if out != NULL. */
int64_t orc_tokens(const uint8_t* src, const orc_event* ev, int64_t n_ev, const uint8_t file_md5[16],
                   uint8_t* out);

/* Generator channel bytes: header (Connection.java:40-45) + per chunk putInt(weak) + dl bytes. */
int64_t orc_generator_bytes(const orc_header* h, const int32_t* weak, const uint8_t* strong, uint8_t* out);

/* ---- synthetic input (bench / golden): splitmix64 counter stream ---- */
void orc_fill_splitmix(uint8_t* out, int64_t n, uint64_t key, int64_t byte_offset);

/* ---- Receiver.combineDataToFile (session/Receiver.java:459-555, 565-578, 204-209, 1006-1020) ----
 * Replays one file's de-multiplexed token stream (putInt(len)+bytes, putInt(-(i+1)), putInt(0)) against
 * the replica (NULL = the Receiver has none: matches are skipped, :487-494).  The target receives the
 * literal bytes and the replica blocks in token order, except when the write is deferred
 * (defer_write && replica, :465): then nothing is written while the matches are 0, 1, 2, ... in order and
 * no literal arrives, and if the stream ends with all chunk_count blocks matched that way the file is
 * intact (returns 1 in *intact; the target stays empty, the replica is the result).  md5 = the digest
 * the Receiver computes over the file content (:541-544, 565-578).
 * Returns bytes of `tokens` consumed (including the terminating 0), or -1 RsyncProtocolException
 * (block index out of range :480-482, a match against a header with block_length 0 :483-485), -2 a
 * truncated token stream, -3 target_cap too small, -4 replica shorter than a block it names. */
typedef struct {
    int64_t target_len; /* bytes written to target */
    int64_t literal;    /* sizeLiteral */
    int64_t matched;    /* sizeMatch */
    int32_t intact;     /* combineDataToFile's return value */
    uint8_t md5[16];
} orc_combine_result;
int64_t orc_receiver_combine(const uint8_t* tokens, int64_t tokens_len, const orc_header* h,
                             const uint8_t* replica, int64_t replica_len, int defer_write, uint8_t* target,
                             int64_t target_cap, orc_combine_result* out);

#ifdef __cplusplus
}
#endif
#endif
