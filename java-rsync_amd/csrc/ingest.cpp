// ingest.cpp -- file ingest for the two passes: what FileView does for the Java code (FileView.java:51-80
// open, :187-278 reads with zero fill after an error), reorganised for a device: several threads pread
// large pieces of the file into pinned buffers, each piece goes to HBM while the next one is read, and
// the device sums it there.  The Generator needs only two pieces in HBM at a time (chunks never straddle
// a piece: pieces are multiples of B); the Sender assembles the whole source in HBM while a host thread
// digests the pieces in order (the whole-file MD5 chain, Sender.java:1241,1326), then scans.
#include <errno.h>
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "ctx.h"
#include "host_md5.h"
#include "options.h"

namespace rsh {
namespace {

constexpr int64_t kGenPiece = 128 << 20;   // Generator piece (rounded down to a multiple of B)
constexpr int64_t kScanPiece = 64 << 20;   // Sender piece
constexpr int kBuffers = 3;                // pinned staging buffers in the ring
constexpr int kReaders = 8;                // threads per piece read

// Reads [0, size) of a file into a ring of pinned buffers, piece after piece, on a background thread.
// Piece i lands in buffer i % nbuf; it is refilled with piece i + nbuf only after release(i).
// FileView semantics: exactly `size` bytes; after the first short read or error everything is zero.
class PieceReader {
  public:
    ~PieceReader() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
        if (fd_ >= 0) close(fd_);
    }
    int open_file(const char* path, int64_t size) {
        size_ = size;
        if (size == 0) return RSH_OK;  // FileView opens nothing for an empty file (:62-72)
        fd_ = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd_ < 0) return (errno == ENOENT || errno == ENOTDIR) ? RSH_E_NOTFOUND : RSH_E_OPEN;
        return RSH_OK;
    }
    void start(uint8_t* const* bufs, int nbuf, int64_t piece) {
        bufs_.assign(bufs, bufs + nbuf);
        piece_ = piece;
        npieces_ = (size_ + piece - 1) / piece;
        filled_.assign((size_t)npieces_, false);
        released_.assign((size_t)npieces_, false);
        th_ = std::thread([this] { run(); });
    }
    int64_t npieces() const { return npieces_; }
    int64_t piece_len(int64_t i) const { return std::min(piece_, size_ - i * piece_); }
    const uint8_t* wait_filled(int64_t i) {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return filled_[(size_t)i] || stop_; });
        return bufs_[(size_t)(i % (int64_t)bufs_.size())];
    }
    void release(int64_t i) {
        {
            std::lock_guard<std::mutex> l(mu_);
            released_[(size_t)i] = true;
        }
        cv_.notify_all();
    }
    bool read_error() const { return error_at_ < size_; }
    int fd() const { return fd_; }

  private:
    void run() {
        const int64_t nbuf = (int64_t)bufs_.size();
        for (int64_t i = 0; i < npieces_; ++i) {
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return i < nbuf || released_[(size_t)(i - nbuf)] || stop_; });
                if (stop_) return;
            }
            uint8_t* dst = bufs_[(size_t)(i % nbuf)];
            const int64_t off = i * piece_, len = piece_len(i);
            if (error_at_ > off) read_piece(dst, off, len);
            if (error_at_ < off + len) {  // zero from the first failure on (FileView.readZeroes)
                const int64_t z = std::max<int64_t>(error_at_, off) - off;
                memset(dst + z, 0, (size_t)(len - z));
            }
            {
                std::lock_guard<std::mutex> l(mu_);
                filled_[(size_t)i] = true;
            }
            cv_.notify_all();
        }
    }
    // kReaders threads, one contiguous sub-range each; error_at_ = the first offset not read
    void read_piece(uint8_t* dst, int64_t off, int64_t len) {
        const int64_t sub = (len + kReaders - 1) / kReaders;
        int64_t fail[kReaders];
        std::thread t[kReaders];
        for (int k = 0; k < kReaders; ++k) {
            fail[k] = INT64_MAX;
            const int64_t a = std::min(len, k * sub), b = std::min(len, a + sub);
            t[k] = std::thread([&, k, a, b] {
                int64_t p = a;
                while (p < b) {
                    const ssize_t r = pread(fd_, dst + p, (size_t)(b - p), (off_t)(off + p));
                    if (r < 0 && errno == EINTR) continue;
                    if (r <= 0) {  // EOF before `size` or an I/O error
                        fail[k] = off + p;
                        return;
                    }
                    p += r;
                }
            });
        }
        for (int k = 0; k < kReaders; ++k) t[k].join();
        for (int k = 0; k < kReaders; ++k) error_at_ = std::min(error_at_, fail[k]);
    }

    int fd_ = -1;
    int64_t size_ = 0, piece_ = 0, npieces_ = 0;
    int64_t error_at_ = INT64_MAX;
    std::vector<uint8_t*> bufs_;
    std::vector<bool> filled_, released_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    std::thread th_;
};

}  // namespace
}  // namespace rsh

using namespace rsh;

extern "C" {

int rsh_block_sums_file(rsh_ctx* ctx, const char* path, int64_t size, const rsh_header* h, const uint8_t seed[4],
                        int32_t* weak_out, uint8_t* strong_out, int32_t* read_error) {
    if (!ctx || !seed || !path) return RSH_E_INVAL;
    const int rc = check_generator_header(size, h);
    if (rc != RSH_OK) return rc;
    if (read_error) *read_error = 0;
    PieceReader rd;
    const int orc = rd.open_file(path, size);  // open before anything else, as new FileView does
    if (orc != RSH_OK) return orc;
    if (h->chunk_count == 0) return RSH_OK;
    if (!weak_out || (!strong_out && h->digest_length > 0)) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    const int64_t B = h->block_length, C = h->chunk_count, dl = h->digest_length;
    const int64_t piece = std::max<int64_t>(B, kGenPiece / B * B);
    RSH_HIP(ctx->h_stage.ensure((size_t)(kBuffers * piece)));
    RSH_HIP(ctx->data.ensure((size_t)(2 * piece)));  // device ring: two pieces
    RSH_HIP(ctx->weak.ensure((size_t)C * 4));
    RSH_HIP(ctx->strong.ensure((size_t)(C * dl + 1)));
    uint8_t* bufs[kBuffers];
    for (int k = 0; k < kBuffers; ++k) bufs[k] = ctx->h_stage.as<uint8_t>() + k * piece;
    hipEvent_t ev;
    RSH_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    rd.start(bufs, kBuffers, piece);
    hipError_t e = hipSuccess;
    for (int64_t i = 0; i < rd.npieces() && e == hipSuccess; ++i) {
        const uint8_t* hb = rd.wait_filled(i);
        const int64_t len = rd.piece_len(i);
        uint8_t* db = ctx->data.as<uint8_t>() + (i & 1) * piece;
        const int64_t c0 = i * piece / B;
        const int64_t nc = (len + B - 1) / B;
        e = hipMemcpyAsync(db, hb, (size_t)len, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipEventRecord(ev, ctx->stream);
        if (e == hipSuccess)
            e = launch_block_sums(db, len, (uint32_t)B, (uint32_t)nc, (uint32_t)dl, seed_word(seed),
                                  ctx->weak.as<int32_t>() + c0, ctx->strong.as<uint8_t>() + c0 * dl, ctx->stream);
        if (e == hipSuccess) e = hipEventSynchronize(ev);  // the staging buffer is free once copied
        rd.release(i);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(weak_out, ctx->weak.p, (size_t)C * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && dl > 0)
        e = hipMemcpyAsync(strong_out, ctx->strong.p, (size_t)(C * dl), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipEventDestroy(ev);
    if (e != hipSuccess) {
        note_error(e, __LINE__, "ingest.cpp");
        return RSH_E_DEVICE;
    }
    if (read_error) *read_error = rd.read_error() ? 1 : 0;
    return RSH_OK;
}

// Sources above file_tile_above (options.h: 32 GiB) are scanned tiled (scan_tiled): HBM then holds one tile of
// file_tile (4 GiB) at a time.

namespace rsh {
namespace {
// The tiled file scan: the tiles are read with pread into a pinned buffer and copied to HBM; the whole-file
// digest runs on its own thread over a second, sequential pass of the file (served by the page cache).  Both
// apply FileView's rule: exactly `size` bytes, zero from the first short read or error on (read_error).
int match_scan_file_tiled(rsh_ctx* ctx, int fd, const char* path, int64_t size, const rsh_header* h,
                          const int32_t* weak, const uint8_t* strong, const uint8_t seed[4], rsh::ResolveResult* r,
                          uint8_t file_md5[16], bool* read_error) {
    const int64_t C = h->chunk_count, dl = h->digest_length;
    std::atomic<int64_t> err_at{INT64_MAX};
    auto read_at = [&](int rfd, uint8_t* dst, int64_t off, int64_t len) {
        int64_t p = 0;
        while (p < len && off + p < err_at.load()) {
            const ssize_t k = pread(rfd, dst + p, (size_t)(len - p), (off_t)(off + p));
            if (k < 0 && errno == EINTR) continue;
            if (k <= 0) {
                int64_t cur = err_at.load();
                while (off + p < cur && !err_at.compare_exchange_weak(cur, off + p)) {
                }
                break;
            }
            p += k;
        }
        const int64_t z = std::max<int64_t>(0, std::min(len, err_at.load() - off));
        if (z < len) memset(dst + z, 0, (size_t)(len - z));
    };
    std::thread md5_thread([&] {
        const int mfd = ::open(path, O_RDONLY | O_CLOEXEC);
        std::vector<uint8_t> buf((size_t)std::min<int64_t>(size, kScanPiece));
        HostMd5 m;
        for (int64_t off = 0; off < size; off += kScanPiece) {
            const int64_t len = std::min<int64_t>(kScanPiece, size - off);
            if (mfd >= 0) read_at(mfd, buf.data(), off, len);
            else memset(buf.data(), 0, (size_t)len);
            m.update(buf.data(), (size_t)len);
        }
        m.final(file_md5);
        if (mfd >= 0) close(mfd);
    });
    int rc = RSH_OK;
    hipError_t e = ctx->h_stage.ensure((size_t)kScanPiece);
    if (e == hipSuccess) e = ctx->weak.ensure((size_t)C * 4 + 4);
    if (e == hipSuccess) e = ctx->strong.ensure((size_t)(C * dl + 1));
    if (e == hipSuccess && C > 0) e = hipMemcpyAsync(ctx->weak.p, weak, (size_t)C * 4, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && C > 0 && dl > 0)
        e = hipMemcpyAsync(ctx->strong.p, strong, (size_t)(C * dl), hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) {
        note_error(e, __LINE__, "ingest.cpp");
        rc = RSH_E_DEVICE;
    } else {
        auto fill = [&](uint8_t* dst, int64_t off, int64_t len) -> hipError_t {  // piece by piece, pinned
            for (int64_t p = 0; p < len; p += kScanPiece) {
                const int64_t l = std::min<int64_t>(kScanPiece, len - p);
                read_at(fd, ctx->h_stage.as<uint8_t>(), off + p, l);
                hipError_t e2 = hipMemcpyAsync(dst + p, ctx->h_stage.p, (size_t)l, hipMemcpyHostToDevice, ctx->stream);
                if (e2 == hipSuccess) e2 = hipStreamSynchronize(ctx->stream);
                if (e2 != hipSuccess) return e2;
            }
            return hipSuccess;
        };
        const int64_t tile = opt(OPT_FILE_TILE);
        rc = scan_tiled(ctx, fill, size, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(), weak, strong, seed,
                        tile, r);
    }
    md5_thread.join();
    *read_error = err_at.load() < size;
    return rc;
}
}  // namespace
}  // namespace rsh

int rsh_match_scan_file(rsh_ctx* ctx, const char* path, int64_t size, const rsh_header* h, const int32_t* weak,
                        const uint8_t* strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap, int64_t* n_ev,
                        uint8_t file_md5[16], int64_t* literal, int64_t* matched, rsh_scan_stats* stats,
                        int32_t* read_error) {
    if (!ctx || !h || !seed || !n_ev || !file_md5 || !path || size < 0) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    if (read_error) *read_error = 0;
    PieceReader rd;
    const int orc = rd.open_file(path, size);
    if (orc != RSH_OK) return orc;
    const int64_t C = h->chunk_count, dl = h->digest_length;
    if (h->block_length > 0 && C > 0 && (!weak || (!strong && dl > 0))) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    // test switches (options.h): file_tile_above and file_tile (bytes)
    const int64_t tile_above = opt(OPT_FILE_TILE_ABOVE);
    if (h->block_length > 0 && size > tile_above) {  // larger than we keep in HBM whole: tiled
        rsh::ResolveResult r;
        bool rerr = false;
        const int rc = rsh::match_scan_file_tiled(ctx, rd.fd(), path, size, h, weak, strong, seed, &r, file_md5, &rerr);
        if (rc != RSH_OK) return rc;
        if (read_error) *read_error = rerr ? 1 : 0;
        if (literal) *literal = r.literal;
        if (matched) *matched = r.matched;
        if (stats) *stats = r.stats;
        return emit_events(ctx, r, ev, ev_cap, n_ev);
    }
    const int64_t piece = kScanPiece;
    RSH_HIP(ctx->h_stage.ensure((size_t)(kBuffers * piece)));
    RSH_HIP(ctx->data.ensure((size_t)std::max<int64_t>(size, 1)));
    RSH_HIP(ctx->weak.ensure((size_t)C * 4 + 4));
    RSH_HIP(ctx->strong.ensure((size_t)(C * dl + 1)));
    if (C > 0) RSH_HIP(hipMemcpyAsync(ctx->weak.p, weak, (size_t)C * 4, hipMemcpyHostToDevice, ctx->stream));
    if (C > 0 && dl > 0)
        RSH_HIP(hipMemcpyAsync(ctx->strong.p, strong, (size_t)(C * dl), hipMemcpyHostToDevice, ctx->stream));
    uint8_t* bufs[kBuffers];
    for (int k = 0; k < kBuffers; ++k) bufs[k] = ctx->h_stage.as<uint8_t>() + k * piece;
    hipEvent_t evs[kBuffers];
    int nev = 0;
    hipError_t e = hipSuccess;
    for (; nev < kBuffers && e == hipSuccess; ++nev) e = hipEventCreateWithFlags(&evs[nev], hipEventDisableTiming);
    // the whole-file digest: a host thread consumes the pieces in order and releases each buffer once both
    // the digest and the piece's copy to HBM are done
    std::mutex mu;
    std::condition_variable cv;
    int64_t copied = 0;  // pieces whose copy has been enqueued
    rd.start(bufs, kBuffers, piece);
    std::thread md5_thread([&] {
        HostMd5 m;
        for (int64_t i = 0; i < rd.npieces(); ++i) {
            const uint8_t* hb = rd.wait_filled(i);
            m.update(hb, (size_t)rd.piece_len(i));
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return copied > i; });
            }
            if (nev == kBuffers) (void)hipEventSynchronize(evs[i % kBuffers]);
            rd.release(i);
        }
        m.final(file_md5);
    });
    for (int64_t i = 0; i < rd.npieces() && nev == kBuffers; ++i) {
        const uint8_t* hb = rd.wait_filled(i);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ctx->data.as<uint8_t>() + i * piece, hb, (size_t)rd.piece_len(i),
                               hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipEventRecord(evs[i % kBuffers], ctx->stream);
        {
            std::lock_guard<std::mutex> l(mu);
            copied = i + 1;
        }
        cv.notify_all();
    }
    if (nev < kBuffers) {  // no events: let the digest thread finish without copies
        std::lock_guard<std::mutex> l(mu);
        copied = rd.npieces();
    }
    cv.notify_all();
    // the scan starts as soon as the source is in HBM; the serial digest keeps running beside it
    rsh::ResolveResult r;
    int rc = RSH_OK;
    if (e != hipSuccess || nev < kBuffers) {
        rc = RSH_E_DEVICE;
    } else if (h->block_length == 0) {
        skip_events(size, &r);
    } else if (size > 0) {
        rc = scan_device(ctx, ctx->data.as<uint8_t>(), size, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(),
                         weak, strong, seed, &r);
    }
    md5_thread.join();
    for (int k = 0; k < nev; ++k) (void)hipEventDestroy(evs[k]);
    if (e != hipSuccess) note_error(e, __LINE__, "ingest.cpp");
    if (rc != RSH_OK) return rc;
    if (read_error) *read_error = rd.read_error() ? 1 : 0;
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

}  // extern "C"
