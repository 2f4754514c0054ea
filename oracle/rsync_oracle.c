/*
 * rsync_oracle.c -- TEST INFRASTRUCTURE ONLY (see rsync_oracle.h).
 *
 * Plain C99 restatement of java-rsync's checksum hot path, written from the Java sources' behaviour
 * (paths below are relative to core/src/main/java/com/github/java/rsync/internal/).  Deliberately
 * simple and sequential: it is the thing the HIP path is checked against, never the thing shipped.
 */
#include "rsync_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------------
 * MD5, RFC 1321 (the JDK provider behind util/MD5.java:35-41).  Textbook byte-serial form.
 * ---------------------------------------------------------------------------------------------- */
static const uint32_t MD5_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const int MD5_R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

static void md5_block(uint32_t h[4], const uint8_t* blk) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) |
               ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) % 16;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) % 16;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) % 16;
        }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl32(a + f + MD5_K[i] + m[g], MD5_R[i]);
        a = t;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

void orc_md5_init(orc_md5_ctx* c) {
    c->h[0] = 0x67452301;
    c->h[1] = 0xefcdab89;
    c->h[2] = 0x98badcfe;
    c->h[3] = 0x10325476;
    c->nbytes = 0;
    c->nbuf = 0;
}

void orc_md5_update(orc_md5_ctx* c, const uint8_t* p, size_t n) {
    c->nbytes += n;
    while (n > 0) {
        size_t take = 64 - c->nbuf;
        if (take > n) take = n;
        memcpy(c->buf + c->nbuf, p, take);
        c->nbuf += (uint32_t)take;
        p += take;
        n -= take;
        if (c->nbuf == 64) {
            md5_block(c->h, c->buf);
            c->nbuf = 0;
        }
    }
}

void orc_md5_final(orc_md5_ctx* c, uint8_t out[16]) {
    uint64_t bits = c->nbytes * 8;
    uint8_t pad = 0x80;
    uint8_t zero = 0;
    uint64_t keep = c->nbytes;
    orc_md5_update(c, &pad, 1);
    while (c->nbuf != 56) orc_md5_update(c, &zero, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (8 * i));
    orc_md5_update(c, len, 8);
    (void)keep;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(c->h[i] >> (8 * j));
    orc_md5_init(c); /* MessageDigest.digest() resets the instance */
}

void orc_md5(const uint8_t* p, size_t n, uint8_t out[16]) {
    orc_md5_ctx c;
    orc_md5_init(&c);
    orc_md5_update(&c, p, n);
    orc_md5_final(&c, out);
}

/* ------------------------------------------------------------------------------------------------
 * Rolling (util/Rolling.java).  Java ints wrap mod 2^32; bytes are signed (CHAR_OFFSET = 0, :23).
 * ---------------------------------------------------------------------------------------------- */
static int32_t jbyte(uint8_t v) { return (int32_t)(int8_t)v; }
static int32_t to_int(uint32_t low16, uint32_t high16) { return (int32_t)((low16 & 0xFFFFu) | (high16 << 16)); }

/* Rolling.java:31-46 -- the 4-unrolled loop is algebraically the plain prefix-sum loop. */
int32_t orc_rolling_compute(const uint8_t* buf, int32_t len) {
    uint32_t low16 = 0, high16 = 0;
    int32_t idx;
    for (idx = 0; idx < len - 4; idx += 4) {
        high16 += 4u * ((uint32_t)jbyte(buf[idx]) + low16) + 3u * (uint32_t)jbyte(buf[idx + 1]) +
                  2u * (uint32_t)jbyte(buf[idx + 2]) + (uint32_t)jbyte(buf[idx + 3]);
        low16 += (uint32_t)jbyte(buf[idx]) + (uint32_t)jbyte(buf[idx + 1]) + (uint32_t)jbyte(buf[idx + 2]) +
                 (uint32_t)jbyte(buf[idx + 3]);
    }
    for (; idx < len; idx++) {
        low16 += (uint32_t)jbyte(buf[idx]);
        high16 += low16;
    }
    return to_int(low16, high16);
}

/* Rolling.java:25-29; low16()/high16() at :48-54 (high16 is checksum >>> 16). */
int32_t orc_rolling_add(int32_t checksum, uint8_t value) {
    uint32_t low16 = ((uint32_t)checksum & 0xFFFFu) + (uint32_t)jbyte(value);
    uint32_t high16 = ((uint32_t)checksum >> 16) + low16;
    return to_int(low16, high16);
}

/* Rolling.java:56-60 */
int32_t orc_rolling_subtract(int32_t checksum, int32_t block_length, uint8_t value) {
    uint32_t low16 = ((uint32_t)checksum & 0xFFFFu) - (uint32_t)jbyte(value);
    uint32_t high16 = ((uint32_t)checksum >> 16) - (uint32_t)block_length * (uint32_t)jbyte(value);
    return to_int(low16, high16);
}

/* ------------------------------------------------------------------------------------------------
 * Sizing (Generator.java:198-236, Util.java:128-130).
 * ---------------------------------------------------------------------------------------------- */
static int32_t pow2_square_root(int64_t num) { /* Generator.java:219-236 */
    if (num <= 0) return 0;
    int exponent = 63 - __builtin_clzll((unsigned long long)num); /* numberOfTrailingZeros(highestOneBit) */
    int sqrt_exponent = exponent / 2;
    return (int32_t)(1u << sqrt_exponent);
}

int32_t orc_block_length_for(int64_t file_size) { /* Generator.java:198-206, MIN_BLOCK_SIZE :186 */
    if (file_size == 0) return 0;
    int32_t bl = pow2_square_root(file_size);
    return bl > 512 ? bl : 512;
}

static double util_log2(double n) { return log(n) / log(2.0); } /* Util.java:128-130 */

int32_t orc_digest_length(int64_t file_size, int32_t block_length) { /* Generator.java:208-212 */
    int64_t lf = (int64_t)util_log2((double)file_size);
    int64_t lb = (int64_t)util_log2((double)block_length);
    int32_t result = ((int32_t)(10 + 2 * lf - lb) - 24) / 8; /* Java int division truncates like C */
    if (result > 16) result = 16;                            /* Checksum.MAX_DIGEST_LENGTH :153 */
    if (result < 2) result = 2;                              /* Checksum.MIN_DIGEST_LENGTH :154 */
    return result;
}

/* ------------------------------------------------------------------------------------------------
 * Checksum.Header (Checksum.java:66-143).
 * ---------------------------------------------------------------------------------------------- */
int orc_header_make(int32_t block_length, int32_t digest_length, int64_t file_size, orc_header* out) {
    if (block_length == 0) { /* :95-101 */
        out->block_length = 0;
        out->digest_length = 0;
        out->remainder = 0;
        out->chunk_count = 0;
        return 0;
    }
    out->block_length = block_length;
    out->digest_length = digest_length;
    out->remainder = (int32_t)(file_size % block_length);
    int64_t cc = file_size / block_length + (out->remainder > 0 ? 1 : 0);
    if (cc < 0 || cc > 2147483647LL) return -1; /* ChunkOverflow :107-111 */
    out->chunk_count = (int32_t)cc;
    return 0;
}

int orc_header_validate(const orc_header* h) { /* :75-92, MAX_CHECKSUM_BLOCK_LENGTH = 1 << 17 (:151) */
    if (h->chunk_count < 0) return -1;
    if (h->block_length == 0 && h->chunk_count > 0) return -1;
    if (h->block_length < 0 || h->block_length > (1 << 17)) return -1;
    if (h->remainder < 0 || h->remainder > h->block_length) return -1;
    if (h->digest_length < 0) return -1;
    return 0;
}

int32_t orc_smallest_chunk_size(const orc_header* h) { return h->remainder > 0 ? h->remainder : h->block_length; }

/* ------------------------------------------------------------------------------------------------
 * Generator hot loop (Generator.java:886-895): FileView(path, N, B, B) yields consecutive windows of
 * min(B, remaining) bytes; per window putInt(Rolling.compute) then MD5(window || seed)[0:dl].
 * ---------------------------------------------------------------------------------------------- */
void orc_generator_sums(const uint8_t* basis, int64_t n, const orc_header* h, const uint8_t seed[4],
                        int32_t* weak_out, uint8_t* strong_out) {
    int64_t B = h->block_length;
    int dl = h->digest_length;
    orc_md5_ctx md;
    orc_md5_init(&md);
    uint8_t dig[16];
    for (int64_t i = 0; i < h->chunk_count; i++) {
        int64_t off = i * B;
        int64_t len = n - off < B ? n - off : B;
        weak_out[i] = orc_rolling_compute(basis + off, (int32_t)len);
        orc_md5_update(&md, basis + off, (size_t)len);
        orc_md5_update(&md, seed, 4);
        orc_md5_final(&md, dig);
        /* the reference's rule never gives dl > 16 (and out.put(digest, 0, dl) would throw); a table
         * with dl > 16 is only built here for Sender tests, padded as the Sender pads (:1262) */
        memcpy(strong_out + i * dl, dig, (size_t)(dl < 16 ? dl : 16));
        if (dl > 16) memset(strong_out + i * dl + 16, 0, (size_t)(dl - 16));
    }
}

/* ------------------------------------------------------------------------------------------------
 * Checksum table: Multimap<Integer, Chunk> (util/Multimap.java) + candidate order
 * (Checksum.java:164-276).  Buckets hold chunks in insertion (= ascending index) order.
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    int32_t weak;
    int32_t idx;
} kv;

static int kv_cmp(const void* a, const void* b) {
    const kv* x = (const kv*)a;
    const kv* y = (const kv*)b;
    if (x->weak != y->weak) return x->weak < y->weak ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

typedef struct {
    kv* sorted;
    int32_t n;
    const orc_header* h;
    const uint8_t* strong;
} table;

static int32_t chunk_length_for(const orc_header* h, int32_t idx) { /* Checksum.java:197-203 */
    if (idx == h->chunk_count - 1 && h->remainder > 0) return h->remainder;
    return h->block_length;
}

/* bucket of `key`: [*lo, *hi) in t->sorted */
static void bucket_of(const table* t, int32_t key, int32_t* lo, int32_t* hi) {
    int32_t a = 0, b = t->n;
    while (a < b) {
        int32_t m = a + (b - a) / 2;
        if (t->sorted[m].weak < key) a = m + 1;
        else b = m;
    }
    int32_t e = a;
    while (e < t->n && t->sorted[e].weak == key) e++;
    *lo = a;
    *hi = e;
}

/* Checksum.java:175-195 binarySearch + :206-213 closeIndexOf, over bucket positions [0, size). */
static int32_t close_index_of(const kv* bucket, int32_t size, int32_t chunk_index) {
    int32_t l = 0, r = size - 1;
    while (l <= r) {
        int32_t m = l + (r - l) / 2;
        int32_t cm = bucket[m].idx;
        if (cm == chunk_index) return m;
        if (cm < chunk_index) l = m + 1;
        else r = m - 1;
    }
    int32_t ip = l;
    return ip < size - 1 ? ip : size - 1;
}

/* ------------------------------------------------------------------------------------------------
 * Event sink.
 * ---------------------------------------------------------------------------------------------- */
static int push_ev(orc_scan_result* r, int kind, int64_t off, int64_t len, int32_t idx) {
    if (kind == ORC_LIT && len == 0) return 0; /* sendDataFrom(…, 0) writes nothing (:802) */
    if (r->n_ev == r->cap) {
        int64_t nc = r->cap ? r->cap * 2 : 64;
        orc_event* ne = (orc_event*)realloc(r->ev, (size_t)nc * sizeof(orc_event));
        if (!ne) return -1;
        r->ev = ne;
        r->cap = nc;
    }
    orc_event* e = &r->ev[r->n_ev++];
    e->offset = off;
    e->length = len;
    e->kind = kind;
    e->index = idx;
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Sender.sendMatchesAndData (Sender.java:1235-1327) over FileView(src, N, B, 10*B) (:1104-1110).
 * File coordinates: `start` = FileView.startOffset, `mark` = markOffset, window = min(B, N - start)
 * (FileView.slide :243-274), firstOffset = min(start, mark) (:143-147), totalBytes = start + window -
 * first (:171-173), isFull <=> totalBytes == 10*B (:182-185).  The rolling sum is advanced with the
 * exact subtract/add calls of the Java loop, so the post-flush desync (quirk A) and the stale
 * localChunkMd5sum (quirk B, declared outside the loop at :1248) fall out naturally.
 * ---------------------------------------------------------------------------------------------- */
static int64_t wl(int64_t s, int64_t B, int64_t N) { return N - s < B ? N - s : B; }

static int sender_match(const uint8_t* x, int64_t N, const orc_header* h, const int32_t* weak,
                        const uint8_t* strong, const uint8_t seed[4], orc_scan_result* r) {
    const int64_t B = h->block_length;
    const int dl = h->digest_length;
    const int64_t bufsize = 10 * B; /* blockSize * blockFactor, :1105-1110 */
    table t;
    t.n = h->chunk_count;
    t.h = h;
    t.strong = strong;
    t.sorted = (kv*)malloc(sizeof(kv) * (size_t)(t.n > 0 ? t.n : 1));
    if (!t.sorted) return -1;
    for (int32_t i = 0; i < t.n; i++) { /* receiveChecksumsFor :758-767 -> addChunkInformation :164-173 */
        t.sorted[i].weak = weak[i];
        t.sorted[i].idx = i;
    }
    qsort(t.sorted, (size_t)t.n, sizeof(kv), kv_cmp);
    /* Lookup accelerator only (the Java HashMap lookup is O(1) as well): a filter of hashed keys; a clear bit proves the bucket empty, a set bit falls through to the exact binary search. */
    int fbits = 12; /* >= 64 filter bits per key, at most 2^24 */
    while (fbits < 24 && ((int64_t)1 << fbits) < 64 * (int64_t)t.n) fbits++;
    const int fshift = 32 - fbits;
    uint64_t* filt = (uint64_t*)calloc((size_t)1 << (fbits - 6), sizeof(uint64_t));
    if (!filt) {
        free(t.sorted);
        return -1;
    }
    for (int32_t i = 0; i < t.n; i++) {
        const uint32_t hk = ((uint32_t)weak[i] * 0x9E3779B1u) >> fshift;
        filt[hk >> 6] |= 1ull << (hk & 63);
    }

    orc_md5_ctx file_digest, chunk_digest;
    orc_md5_init(&file_digest);
    orc_md5_init(&chunk_digest);
    const int64_t S = orc_smallest_chunk_size(h); /* :1251 */
    int64_t start = 0, mark = 0;                  /* setMarkRelativeToStart(0) :1249 */
    int32_t rolling = orc_rolling_compute(x, (int32_t)wl(0, B, N)); /* :1244 */
    int32_t preferred = 0;
    int64_t size_literal = 0, size_match = 0;
    int md5c_valid = 0; /* localChunkMd5sum == null (:1248) */
    /* Arrays.copyOf(digest, md5.length) (:1262): dl bytes, zero past the 16 digest bytes */
    uint8_t* md5c = (uint8_t*)calloc((size_t)(dl > 0 ? dl : 1), 1);
    uint8_t dig[16];
    if (!md5c) {
        free(t.sorted);
        free(filt);
        return -1;
    }

    while (wl(start, B, N) >= S) {
        int64_t w = wl(start, B, N);
        int32_t lo = 0, hi = 0;
        const uint32_t hk = ((uint32_t)rolling * 0x9E3779B1u) >> fshift;
        if (filt[hk >> 6] >> (hk & 63) & 1) bucket_of(&t, rolling, &lo, &hi);
        int32_t size = hi - lo;
        if (size > 0) {
            const kv* bucket = t.sorted + lo;
            int32_t initial = close_index_of(bucket, size, preferred); /* :226 */
            int is_initial = 1;
            int32_t it = 0;
            for (;;) { /* for (Chunk chunk : getCandidateChunks(...)) -- iterator :232-273 */
                int32_t pos;
                if (is_initial) {
                    pos = initial;
                    is_initial = 0;
                } else {
                    int32_t i = it;
                    while (i < size && !(i != initial && chunk_length_for(h, bucket[i].idx) == w)) i++;
                    if (i >= size) break;
                    pos = i;
                    it = i + 1;
                }
                int32_t cidx = bucket[pos].idx;
                if (!md5c_valid) { /* :1259-1263 */
                    orc_md5_update(&chunk_digest, x + start, (size_t)w);
                    orc_md5_update(&chunk_digest, seed, 4);
                    orc_md5_final(&chunk_digest, dig);
                    memcpy(md5c, dig, (size_t)(dl < 16 ? dl : 16));
                    md5c_valid = 1;
                    r->md5_windows++;
                }
                if (memcmp(md5c, strong + (int64_t)cidx * dl, (size_t)dl) == 0) { /* :1265 */
                    size_match += w;
                    int64_t first = start < mark ? start : mark;
                    if (push_ev(r, ORC_LIT, mark, start - first, 0)) goto oom; /* :1270 */
                    size_literal += start - first;
                    int64_t total = start + w - first;
                    orc_md5_update(&file_digest, x + mark, (size_t)total); /* :1272 */
                    if (push_ev(r, ORC_MATCH, start, w, cidx)) goto oom;     /* :1274 */
                    preferred = cidx + 1;                                    /* :1275 */
                    mark = start + w;                                        /* :1279 */
                    start += w - 1;                                          /* :1282 */
                    rolling = orc_rolling_compute(x + start, (int32_t)wl(start, B, N)); /* :1286 */
                    md5c_valid = 0;                                                       /* :1287 */
                    break;
                }
            }
        }
        w = wl(start, B, N);
        rolling = orc_rolling_subtract(rolling, (int32_t)w, x[start]); /* :1292 */
        int64_t first = start < mark ? start : mark;
        int64_t total = start + w - first;
        if (total == bufsize) { /* isFull :1294-1302 */
            if (push_ev(r, ORC_LIT, first, total, 0)) goto oom;
            size_literal += total;
            orc_md5_update(&file_digest, x + first, (size_t)total);
            mark = start + w;
            start += w;
        } else {
            start += 1; /* :1304 */
        }
        if (wl(start, B, N) == B) rolling = orc_rolling_add(rolling, x[start + B - 1]); /* :1308-1310 */
    }
    {
        int64_t first = start < mark ? start : mark;
        int64_t total = N - first; /* window end is N once the loop exits */
        if (push_ev(r, ORC_LIT, first, total, 0)) goto oom; /* :1313 */
        size_literal += total;
        orc_md5_update(&file_digest, x + first, (size_t)total);
    }
    orc_md5_final(&file_digest, r->file_md5);
    r->literal = size_literal;
    r->matched = size_match;
    free(t.sorted);
    free(md5c);
    free(filt);
    return 0;
oom:
    free(t.sorted);
    free(md5c);
    free(filt);
    return -1;
}

/* Sender.skipMatchSendData (:1386-1399) over FileView(src, N, 8192, 8192). */
static int sender_skip(const uint8_t* x, int64_t N, orc_scan_result* r) {
    const int64_t W = 8192; /* FileView.DEFAULT_BLOCK_SIZE */
    for (int64_t s = 0; s < N; s += W) {
        int64_t w = N - s < W ? N - s : W;
        if (push_ev(r, ORC_LIT, s, w, 0)) return -1;
    }
    orc_md5(x, (size_t)N, r->file_md5);
    r->literal = N;
    r->matched = 0;
    return 0;
}

int orc_sender_scan(const uint8_t* src, int64_t n, const orc_header* h, const int32_t* weak,
                    const uint8_t* strong, const uint8_t seed[4], orc_scan_result* res) {
    memset(res, 0, sizeof(*res));
    if (h->block_length == 0) return sender_skip(src, n, res); /* isNew :1104, :1115-1116 */
    if (n == 0) {                                              /* empty source: loop never runs */
        orc_md5(src, 0, res->file_md5);
        return 0;
    }
    return sender_match(src, n, h, weak, strong, seed, res);
}

void orc_scan_free(orc_scan_result* res) {
    free(res->ev);
    res->ev = NULL;
    res->n_ev = res->cap = 0;
}

/* ------------------------------------------------------------------------------------------------
 * Channel bytes.  BufferedOutputChannel is little-endian (channels/BufferedOutputChannel.java:50).
 * ---------------------------------------------------------------------------------------------- */
static int64_t put_int(uint8_t* out, int64_t pos, int32_t v) {
    if (out)
        for (int i = 0; i < 4; i++) out[pos + i] = (uint8_t)((uint32_t)v >> (8 * i));
    return pos + 4;
}

int64_t orc_tokens(const uint8_t* src, const orc_event* ev, int64_t n_ev, const uint8_t file_md5[16],
                   uint8_t* out) {
    int64_t pos = 0;
    for (int64_t i = 0; i < n_ev; i++) {
        if (ev[i].kind == ORC_LIT) { /* sendDataFrom, Sender.java:794-809, CHUNK_SIZE 8192 (:230) */
            int64_t cur = ev[i].offset, end = ev[i].offset + ev[i].length;
            while (cur < end) {
                int64_t len = end - cur < 8192 ? end - cur : 8192;
                pos = put_int(out, pos, (int32_t)len);
                if (out) memcpy(out + pos, src + cur, (size_t)len);
                pos += len;
                cur += len;
            }
        } else {
            pos = put_int(out, pos, -(ev[i].index + 1)); /* :1274 */
        }
    }
    pos = put_int(out, pos, 0); /* :1316 / :1396 */
    if (out) memcpy(out + pos, file_md5, 16);
    return pos + 16; /* sendFiles :1148 */
}

int64_t orc_generator_bytes(const orc_header* h, const int32_t* weak, const uint8_t* strong, uint8_t* out) {
    int64_t pos = 0;
    pos = put_int(out, pos, h->chunk_count); /* Connection.java:40-45 */
    pos = put_int(out, pos, h->block_length);
    pos = put_int(out, pos, h->digest_length);
    pos = put_int(out, pos, h->remainder);
    for (int32_t i = 0; i < h->chunk_count; i++) { /* Generator.java:890-893 */
        pos = put_int(out, pos, weak[i]);
        if (out) memcpy(out + pos, strong + (int64_t)i * h->digest_length, (size_t)h->digest_length);
        pos += h->digest_length;
    }
    return pos;
}

/* ------------------------------------------------------------------------------------------------
 * splitmix64 counter stream: 8-byte word k of stream `key` = mix(key + (k + 1) * golden), LE bytes.
 * ---------------------------------------------------------------------------------------------- */
static uint64_t splitmix_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_fill_splitmix(uint8_t* out, int64_t n, uint64_t key, int64_t byte_offset) {
    for (int64_t i = 0; i < n; i++) {
        uint64_t pos = (uint64_t)(byte_offset + i);
        uint64_t wd = splitmix_mix(key + (pos / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        out[i] = (uint8_t)(wd >> (8 * (pos % 8)));
    }
}

/* ---- Receiver.combineDataToFile (Receiver.java:459-555) ---- */
static int32_t get_int(const uint8_t* p) { /* BufferedInputChannel little-endian getInt */
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

static int32_t block_size(int32_t index, const orc_header* h) { /* Receiver.java:204-209 */
    if (index == h->chunk_count - 1 && h->remainder != 0) return h->remainder;
    return h->block_length;
}

/* copyFromReplicaAndUpdateDigest (:570-578) with readFromReplica (:1006-1020) */
static int copy_block(const uint8_t* replica, int64_t replica_len, int32_t index, const orc_header* h,
                      uint8_t* target, int64_t cap, int64_t* tlen, orc_md5_ctx* md) {
    const int32_t len = block_size(index, h);
    const int64_t off = (int64_t)index * h->block_length;
    if (off + len > replica_len) return -4; /* truncated read from replica: IllegalStateException */
    if (*tlen + len > cap) return -3;
    memcpy(target + *tlen, replica + off, (size_t)len);
    *tlen += len;
    orc_md5_update(md, replica + off, (size_t)len);
    return 0;
}

int64_t orc_receiver_combine(const uint8_t* tokens, int64_t tokens_len, const orc_header* h,
                             const uint8_t* replica, int64_t replica_len, int defer_write, uint8_t* target,
                             int64_t target_cap, orc_combine_result* out) {
    orc_md5_ctx md;
    orc_md5_init(&md);
    int deferrable = defer_write && replica != NULL; /* :465 */
    int64_t pos = 0, tlen = 0, lit = 0, mat = 0;
    int32_t expected = 0;
    int rc;
    for (;;) {
        if (pos + 4 > tokens_len) return -2;
        const int32_t token = get_int(tokens + pos);
        pos += 4;
        if (token == 0) break; /* :471-473 */
        if (token < 0) {
            const int32_t index = -(token + 1);
            if (index > h->chunk_count - 1) return -1; /* :480-482 */
            if (h->block_length == 0) return -1;       /* :483-485 */
            if (replica == NULL) continue;             /* :487-494 */
            mat += block_size(index, h);               /* :496 */
            if (deferrable) {                          /* :498-510 */
                if (index == expected) {
                    expected++;
                    continue;
                }
                deferrable = 0;
                for (int32_t i = 0; i < expected; i++)
                    if ((rc = copy_block(replica, replica_len, i, h, target, target_cap, &tlen, &md)) != 0) return rc;
            }
            if ((rc = copy_block(replica, replica_len, index, h, target, target_cap, &tlen, &md)) != 0) return rc;
        } else { /* literal data (:512-525), copyFromPeerAndUpdateDigest (:557-568) */
            if (deferrable) {
                deferrable = 0;
                for (int32_t i = 0; i < expected; i++)
                    if ((rc = copy_block(replica, replica_len, i, h, target, target_cap, &tlen, &md)) != 0) return rc;
            }
            if (pos + token > tokens_len) return -2;
            if (tlen + token > target_cap) return -3;
            memcpy(target + tlen, tokens + pos, (size_t)token);
            orc_md5_update(&md, tokens + pos, (size_t)token);
            tlen += token;
            lit += token;
            pos += token;
        }
    }
    if (deferrable && expected != h->chunk_count) { /* :529-538: truncation of whole blocks */
        deferrable = 0;
        for (int32_t i = 0; i < expected; i++)
            if ((rc = copy_block(replica, replica_len, i, h, target, target_cap, &tlen, &md)) != 0) return rc;
    }
    if (deferrable) { /* :539-545: digest of the untouched replica */
        for (int32_t i = 0; i < expected; i++) {
            const int32_t len = block_size(i, h);
            const int64_t off = (int64_t)i * h->block_length;
            if (off + len > replica_len) return -4;
            orc_md5_update(&md, replica + off, (size_t)len);
        }
    }
    out->target_len = tlen;
    out->literal = lit;
    out->matched = mat;
    out->intact = deferrable;
    orc_md5_final(&md, out->md5);
    return pos;
}
