// receiver.cpp -- the Receiver's side of the delta: rebuild a file from the Sender's token stream and the
// replica (Receiver.combineDataToFile, Receiver.java:459-555), with the blocks gathered on the device.
//
// The token walk is sequential and cheap (one int per block or per <= 8 KiB literal), so it runs on the
// host and produces a list of byte ranges; the bytes themselves move on the device: literal bytes in one
// upload, replica blocks as device-to-device gathers (one launch for the whole file).  The digest the
// Receiver compares with the Sender's file MD5 (:824-842) is one serial MD5 chain over the rebuilt file;
// it runs on the host while the next piece of the file comes back over PCIe.
#include <condition_variable>
#include <mutex>
#include <thread>

#include "ctx.h"
#include "host_md5.h"
#include "md5_mb.h"
#include "options.h"

namespace rsh {
namespace {

constexpr int64_t kOpPiece = 1 << 20;   // gather ops are cut into pieces of at most this many bytes
constexpr int64_t kMd5Piece = 64 << 20; // D2H granularity of the digest pass

int32_t get_int(const uint8_t* p) {  // BufferedInputChannel.getInt: little-endian
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

int32_t block_size(int32_t index, const rsh_header& h) {  // Receiver.java:204-209
    if (index == h.chunk_count - 1 && h.remainder != 0) return h.remainder;
    return h.block_length;
}

// One range of the rebuilt file: a replica block run (src_off into the replica) or literal bytes
// (src_off into the token stream).
struct Piece {
    bool literal;
    int64_t src_off;
    int64_t len;
};

struct Plan {
    std::vector<Piece> pieces;  // in target order
    int64_t tokens_used = 0, target_len = 0, literal = 0, matched = 0, literal_bytes = 0;
    bool intact = false;
    int64_t intact_len = 0;  // replica bytes [0, intact_len) are the file when intact
};

// The token walk of combineDataToFile, recording what the Java code writes (and digests) instead of doing
// it.  Same control flow as the oracle's orc_receiver_combine.
int plan_combine(const uint8_t* tokens, int64_t tokens_len, const rsh_header& h, bool have_replica,
                 int64_t replica_len, bool defer_write, Plan* P) {
    bool deferrable = defer_write && have_replica;  // :465
    int32_t expected = 0;
    int64_t pos = 0;
    auto add_block = [&](int32_t index) -> int {  // copyFromReplicaAndUpdateDigest (:570-578)
        const int64_t len = block_size(index, h);
        const int64_t off = (int64_t)index * h.block_length;
        if (off + len > replica_len) return RSH_E_INVAL;  // truncated read from replica (:1015-1017)
        Piece* last = P->pieces.empty() ? nullptr : &P->pieces.back();
        if (last && !last->literal && last->src_off + last->len == off) last->len += len;  // runs merge
        else P->pieces.push_back(Piece{false, off, len});
        P->target_len += len;
        return RSH_OK;
    };
    auto flush_deferred = [&]() -> int {
        deferrable = false;
        for (int32_t i = 0; i < expected; ++i) {
            const int rc = add_block(i);
            if (rc != RSH_OK) return rc;
        }
        return RSH_OK;
    };
    for (;;) {
        if (pos + 4 > tokens_len) return RSH_E_INVAL;  // the stream ended without putInt(0)
        const int32_t token = get_int(tokens + pos);
        pos += 4;
        if (token == 0) break;  // :471-473
        if (token < 0) {
            const int32_t index = -(token + 1);
            if (index > h.chunk_count - 1) return RSH_E_PROTOCOL;  // :480-482
            if (h.block_length == 0) return RSH_E_PROTOCOL;        // :483-485
            if (!have_replica) continue;                           // :487-494
            P->matched += block_size(index, h);                    // :496
            if (deferrable) {                                      // :498-510
                if (index == expected) {
                    ++expected;
                    continue;
                }
                const int rc = flush_deferred();
                if (rc != RSH_OK) return rc;
            }
            const int rc = add_block(index);
            if (rc != RSH_OK) return rc;
        } else {  // literal data (:512-525)
            if (deferrable) {
                const int rc = flush_deferred();
                if (rc != RSH_OK) return rc;
            }
            if (pos + token > tokens_len) return RSH_E_INVAL;
            P->pieces.push_back(Piece{true, pos, token});
            P->target_len += token;
            P->literal += token;
            P->literal_bytes += token;
            pos += token;
        }
    }
    if (deferrable && expected != h.chunk_count) {  // :529-538
        const int rc = flush_deferred();
        if (rc != RSH_OK) return rc;
    }
    if (deferrable) {  // :539-545: the untouched replica is the file
        for (int32_t i = 0; i < expected; ++i) {
            const int64_t len = block_size(i, h);
            if ((int64_t)i * h.block_length + len > replica_len) return RSH_E_INVAL;
            P->intact_len = (int64_t)i * h.block_length + len;
        }
        P->intact = true;
    }
    P->tokens_used = pos;
    return RSH_OK;
}

// MD5 of device bytes [0, n): pieces come back into two pinned buffers, each digested while the next
// one is in flight.
int md5_device(rsh_ctx* c, const uint8_t* d, int64_t n, uint8_t out[16]) {
    HostMd5 m;
    if (n > 0) {
        const int64_t piece = std::min<int64_t>(kMd5Piece, n);
        RSH_HIP(c->h_win.ensure((size_t)(2 * piece)));
        uint8_t* buf[2] = {c->h_win.as<uint8_t>(), c->h_win.as<uint8_t>() + piece};
        hipEvent_t ev[2];
        RSH_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
        if (hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) {
            (void)hipEventDestroy(ev[0]);
            return RSH_E_DEVICE;
        }
        hipError_t e = hipSuccess;
        auto issue = [&](int64_t off, int k) {
            const int64_t len = std::min<int64_t>(piece, n - off);
            if (e == hipSuccess) e = hipMemcpyAsync(buf[k], d + off, (size_t)len, hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipEventRecord(ev[k], c->stream);
        };
        issue(0, 0);
        int k = 0;
        for (int64_t off = 0; off < n && e == hipSuccess; off += piece, k ^= 1) {
            if (off + piece < n) issue(off + piece, k ^ 1);
            if (e == hipSuccess) e = hipEventSynchronize(ev[k]);
            if (e == hipSuccess) m.update(buf[k], (size_t)std::min<int64_t>(piece, n - off));
        }
        (void)hipEventDestroy(ev[0]);
        (void)hipEventDestroy(ev[1]);
        if (e != hipSuccess) {
            note_error(e, __LINE__, "receiver.cpp");
            return RSH_E_DEVICE;
        }
    }
    m.final(out);
    return RSH_OK;
}

// The device gather for a plan: literal bytes to a device staging buffer in one upload, then every
// piece (cut to kOpPiece) as one gather op.
int gather_device(rsh_ctx* c, const Plan& P, const uint8_t* tokens, const uint8_t* d_replica, uint8_t* d_target) {
    RSH_HIP(c->out.ensure((size_t)P.literal_bytes + 16));
    RSH_HIP(c->h_out.ensure((size_t)P.literal_bytes + 16));
    uint8_t* h_lit = c->h_out.as<uint8_t>();
    uint8_t* d_lit = c->out.as<uint8_t>();
    std::vector<GatherOp> ops;
    int64_t t = 0, lo = 0;
    for (const Piece& p : P.pieces) {
        const uint8_t* src;
        if (p.literal) {
            memcpy(h_lit + lo, tokens + p.src_off, (size_t)p.len);
            src = d_lit + lo;
            lo += p.len;
        } else {
            src = d_replica + p.src_off;
        }
        for (int64_t o = 0; o < p.len; o += kOpPiece)
            ops.push_back(GatherOp{src + o, d_target + t + o, std::min<int64_t>(kOpPiece, p.len - o)});
        t += p.len;
    }
    if (ops.empty()) return RSH_OK;
    RSH_HIP(c->h_pos.ensure(ops.size() * sizeof(GatherOp)));  // read by the kernel from pinned memory
    memcpy(c->h_pos.p, ops.data(), ops.size() * sizeof(GatherOp));
    if (lo > 0) RSH_HIP(hipMemcpyAsync(d_lit, h_lit, (size_t)lo, hipMemcpyHostToDevice, c->stream));
    RSH_HIP(launch_gather_ops(c->h_pos.as<GatherOp>(), (uint32_t)ops.size(), c->stream));
    return RSH_OK;
}

void fill_result(const Plan& P, rsh_combine_result* out) {
    out->tokens_used = P.tokens_used;
    out->target_len = P.intact ? 0 : P.target_len;
    out->literal = P.literal;
    out->matched = P.matched;
    out->intact = P.intact ? 1 : 0;
    out->reserved = 0;
}


// ------------------------------------------------------------------------------------------------
// A segment's Receiver (rsh_receiver_combine_batch): every file planned on the host, the rebuilt bytes gathered on
// the device in passes, the verify digests on the host's cores from the bytes the plans name.
// ------------------------------------------------------------------------------------------------
constexpr int64_t kSpanGap = 1 << 20;  // replica ranges closer than this go up as one copy (fewer, larger copies)
constexpr int64_t kAlignR = 256;
int64_t alignr(int64_t v) { return (v + kAlignR - 1) / kAlignR * kAlignR; }

// A list of host pieces addressed by byte offset (the replica of one file).
struct PieceList {
    const rsh_piece* p = nullptr;
    int32_t n = 0;
    std::vector<int64_t> start;  // start[i] = offset of piece i; start[n] = total
    void init(const rsh_piece* pieces, int32_t count) {
        p = pieces;
        n = count;
        start.assign((size_t)count + 1, 0);
        for (int32_t i = 0; i < count; ++i) start[(size_t)i + 1] = start[(size_t)i] + pieces[i].len;
    }
    int64_t total() const { return start.empty() ? 0 : start.back(); }
    // bytes [off, off + len) as host pieces (appended to out)
    template <class F>
    void each(int64_t off, int64_t len, F&& f) const {
        int32_t k = (int32_t)(std::upper_bound(start.begin(), start.end(), off) - start.begin()) - 1;
        while (len > 0 && k < n) {
            const int64_t in = off - start[(size_t)k], take = std::min<int64_t>(len, p[k].len - in);
            if (take > 0) {
                f(p[k].data + in, take);
                off += take;
                len -= take;
            }
            ++k;
        }
    }
};

struct RFile {
    int32_t job = -1;
    Plan plan;
    PieceList rep;
    std::vector<std::pair<int64_t, int64_t>> spans;  // replica ranges the plan reads (merged), [off, end)
    std::vector<int64_t> span_at;                     // each span's offset in the pass's replica area
    int64_t rep_bytes = 0;                            // replica bytes uploaded
    int64_t tok_at = 0, rep_at = 0, tgt_at = 0;       // offsets in the pass buffer
    int64_t pass_bytes() const { return alignr(plan.tokens_used) + alignr(rep_bytes) + alignr(plan.target_len); }
};

void plan_spans(RFile& F) {
    std::vector<std::pair<int64_t, int64_t>> runs;
    for (const Piece& q : F.plan.pieces)
        if (!q.literal) runs.emplace_back(q.src_off, q.src_off + q.len);
    std::sort(runs.begin(), runs.end());
    for (const auto& r : runs) {
        if (!F.spans.empty() && r.first <= F.spans.back().second + kSpanGap)
            F.spans.back().second = std::max(F.spans.back().second, r.second);
        else
            F.spans.push_back(r);
    }
    F.span_at.resize(F.spans.size());
    int64_t at = 0;
    for (size_t i = 0; i < F.spans.size(); ++i) {
        F.span_at[i] = at;
        at += F.spans[i].second - F.spans[i].first;
    }
    F.rep_bytes = at;
}

// device address of replica byte `off` of file F in a pass whose replica area starts at base
const uint8_t* rep_addr(const RFile& F, const uint8_t* base, int64_t off) {
    const size_t i = (size_t)(std::upper_bound(F.spans.begin(), F.spans.end(), std::make_pair(off, INT64_MAX)) -
                              F.spans.begin()) - 1;
    return base + F.span_at[i] + (off - F.spans[i].first);
}


// The device passes of rsh_receiver_combine_batch over `files` (non-intact files with bytes to write).  A pass's
// buffer holds its files' token streams, the replica ranges they name and their targets; two buffers alternate, so
// a pass's uploads and gather (context stream) overlap the previous pass's downloads (aux stream, issued by a
// second host thread: downloads into pageable caller memory block the thread that issues them).  done[job] = 1
// once a file's target is on the host.
int combine_passes(rsh_ctx* c, rsh_combine_job* jobs, std::vector<RFile>& files, std::vector<char>& done) {
    RSH_CLAIM(c);
    RSH_HIP(hipSetDevice(c->device));
    int64_t total = 0;
    for (const RFile& F : files) total += F.pass_bytes();
    const int64_t budget = std::max<int64_t>(kAlignR, opt(OPT_SEGMENT_BYTES) / 2);  // per buffer
    const int64_t want = std::min(budget, std::max<int64_t>(total / 4, 256LL << 20));
    std::vector<std::pair<size_t, size_t>> passes;  // [first, last) of files
    {
        size_t a = 0;
        int64_t used = 0;
        for (size_t i = 0; i < files.size(); ++i) {
            const int64_t b = files[i].pass_bytes();
            if (i > a && used + b > want) {
                passes.emplace_back(a, i);
                a = i;
                used = 0;
            }
            used += b;
        }
        passes.emplace_back(a, files.size());
    }
    hipEvent_t ev_g[2] = {nullptr, nullptr};
    for (hipEvent_t& e : ev_g) RSH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct Events {
        hipEvent_t* e;
        ~Events() {
            for (int i = 0; i < 2; ++i)
                if (e[i]) (void)hipEventDestroy(e[i]);
        }
    } events_{ev_g};
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::pair<size_t, int>> queue;  // (pass, buffer) gathered, to download
    bool closing = false, busy[2] = {false, false};
    hipError_t derr = hipSuccess;
    std::thread down([&] {
        for (size_t qi = 0;; ++qi) {
            std::pair<size_t, int> d;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return queue.size() > qi || closing; });
                if (queue.size() <= qi) return;
                d = queue[qi];
            }
            const uint8_t* base = c->rcv[d.second].as<uint8_t>();
            hipError_t e = hipStreamWaitEvent(c->aux, ev_g[d.second], 0);
            for (size_t f = passes[d.first].first; f < passes[d.first].second && e == hipSuccess; ++f) {
                const RFile& F = files[f];
                e = hipMemcpyAsync(jobs[F.job].target, base + F.tgt_at, (size_t)F.plan.target_len,
                                   hipMemcpyDeviceToHost, c->aux);
            }
            if (e == hipSuccess) e = hipStreamSynchronize(c->aux);
            {
                std::lock_guard<std::mutex> lk(mu);
                if (e != hipSuccess && derr == hipSuccess) derr = e;
                if (e == hipSuccess)
                    for (size_t f = passes[d.first].first; f < passes[d.first].second; ++f) done[(size_t)files[f].job] = 1;
                busy[d.second] = false;
            }
            cv.notify_all();
        }
    });
    int rc = RSH_OK;
    hipError_t e = hipSuccess;
    std::vector<GatherOp> ops;
    for (size_t k = 0; k < passes.size() && rc == RSH_OK; ++k) {
        const int set = (int)(k & 1);
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return !busy[set] || derr != hipSuccess; });
            if (derr != hipSuccess) break;
            busy[set] = true;
        }
        int64_t off = 0;
        for (size_t f = passes[k].first; f < passes[k].second; ++f) {
            files[f].tok_at = off;
            off += alignr(files[f].plan.tokens_used);
        }
        for (size_t f = passes[k].first; f < passes[k].second; ++f) {
            files[f].rep_at = off;
            off += alignr(files[f].rep_bytes);
        }
        for (size_t f = passes[k].first; f < passes[k].second; ++f) {
            files[f].tgt_at = off;
            off += alignr(files[f].plan.target_len);
        }
        if (((opt(OPT_FAULT_INJECT) & 1) && fault_here()) || c->rcv[set].ensure((size_t)off + kAlignR) != hipSuccess) {
            snprintf(g_last_err, sizeof(g_last_err), "receiver pass of %lld bytes: device memory (receiver.cpp)",
                     (long long)off);
            rc = RSH_E_NOMEM;
            break;
        }
        uint8_t* base = c->rcv[set].as<uint8_t>();
        ops.clear();
        int64_t op_bytes = 0;
        for (size_t f = passes[k].first; f < passes[k].second; ++f) {
            const RFile& F = files[f];
            int64_t t = 0;
            for (const Piece& q : F.plan.pieces) {
                const uint8_t* src = q.literal ? base + F.tok_at + q.src_off : rep_addr(F, base + F.rep_at, q.src_off);
                for (int64_t o = 0; o < q.len; o += kOpPiece)
                    ops.push_back(GatherOp{src + o, base + F.tgt_at + t + o, std::min<int64_t>(kOpPiece, q.len - o)});
                t += q.len;
                op_bytes += q.len;
            }
        }
        if (c->rcv_ops[set].ensure(ops.size() * sizeof(GatherOp) + 16) != hipSuccess ||
            c->h_rcv_ops[set].ensure(ops.size() * sizeof(GatherOp) + 16) != hipSuccess) {
            rc = RSH_E_NOMEM;
            break;
        }
        memcpy(c->h_rcv_ops[set].p, ops.data(), ops.size() * sizeof(GatherOp));
        for (size_t f = passes[k].first; f < passes[k].second && e == hipSuccess; ++f) {
            const RFile& F = files[f];
            const rsh_combine_job& j = jobs[F.job];
            e = hipMemcpyAsync(base + F.tok_at, j.tokens, (size_t)F.plan.tokens_used, hipMemcpyHostToDevice, c->stream);
            for (size_t i = 0; i < F.spans.size() && e == hipSuccess; ++i) {
                uint8_t* dst = base + F.rep_at + F.span_at[i];
                F.rep.each(F.spans[i].first, F.spans[i].second - F.spans[i].first, [&](const uint8_t* d, int64_t n) {
                    if (e == hipSuccess) e = hipMemcpyAsync(dst, d, (size_t)n, hipMemcpyHostToDevice, c->stream);
                    dst += n;
                });
            }
        }
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->rcv_ops[set].p, c->h_rcv_ops[set].p, ops.size() * sizeof(GatherOp),
                               hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess)
            e = launch_gather_ops(c->rcv_ops[set].as<GatherOp>(), (uint32_t)ops.size(), c->stream,
                                  ops.empty() ? 0 : op_bytes / (int64_t)ops.size());
        if (e == hipSuccess) e = hipEventRecord(ev_g[set], c->stream);
        if (e != hipSuccess) {
            note_error(e, __LINE__, "receiver.cpp");
            rc = RSH_E_DEVICE;
            std::lock_guard<std::mutex> lk(mu);
            busy[set] = false;
            break;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            queue.emplace_back(k, set);
        }
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        closing = true;
    }
    cv.notify_all();
    down.join();
    (void)hipStreamSynchronize(c->stream);  // nothing of the caller's buffers is read after the call
    if (rc == RSH_OK && derr != hipSuccess) {
        note_error(derr, __LINE__, "receiver.cpp");
        rc = RSH_E_DEVICE;
    }
    return rc;
}

}  // namespace
}  // namespace rsh

using namespace rsh;

extern "C" {

int rsh_receiver_combine_device(rsh_ctx* ctx, const uint8_t* tokens, int64_t tokens_len, const rsh_header* h,
                                const void* d_replica, int64_t replica_len, int32_t defer_write, void* d_target,
                                int64_t target_cap, rsh_combine_result* out) {
    if (!ctx || !h || !out || !tokens || tokens_len < 0 || replica_len < 0 || target_cap < 0) return RSH_E_INVAL;
    Plan P;
    const int rc = plan_combine(tokens, tokens_len, *h, d_replica != nullptr, replica_len, defer_write != 0, &P);
    if (rc != RSH_OK) return rc;
    fill_result(P, out);
    if (!P.intact && P.target_len > target_cap) return RSH_E_NOSPACE;
    if (!P.intact && P.target_len > 0 && !d_target) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    const uint8_t* rep = static_cast<const uint8_t*>(d_replica);
    uint8_t* tgt = static_cast<uint8_t*>(d_target);
    if (!P.intact) {
        const int g = gather_device(ctx, P, tokens, rep, tgt);
        if (g != RSH_OK) return g;
    }
    return md5_device(ctx, P.intact ? rep : tgt, P.intact ? P.intact_len : P.target_len, out->md5);
}

int rsh_receiver_combine(rsh_ctx* ctx, const uint8_t* tokens, int64_t tokens_len, const rsh_header* h,
                         const uint8_t* replica, int64_t replica_len, int32_t defer_write, uint8_t* target,
                         int64_t target_cap, rsh_combine_result* out) {
    if (!ctx || !h || !out || !tokens || tokens_len < 0 || replica_len < 0 || target_cap < 0) return RSH_E_INVAL;
    Plan P;
    const int rc = plan_combine(tokens, tokens_len, *h, replica != nullptr, replica_len, defer_write != 0, &P);
    if (rc != RSH_OK) return rc;
    fill_result(P, out);
    if (!P.intact && P.target_len > target_cap) return RSH_E_NOSPACE;
    if (!P.intact && P.target_len > 0 && !target) return RSH_E_INVAL;
    HostMd5 m;
    if (P.intact) {  // nothing is written: the digest of the replica's blocks (:539-545)
        m.update(replica, (size_t)P.intact_len);
        m.final(out->md5);
        return RSH_OK;
    }
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    const bool any_block = std::any_of(P.pieces.begin(), P.pieces.end(), [](const Piece& p) { return !p.literal; });
    if (P.target_len > 0) {
        RSH_HIP(ctx->data.ensure((size_t)P.target_len));
        uint8_t* d_rep = nullptr;
        if (any_block) {
            RSH_HIP(ctx->strong.ensure((size_t)replica_len));
            d_rep = ctx->strong.as<uint8_t>();
            RSH_HIP(hipMemcpyAsync(d_rep, replica, (size_t)replica_len, hipMemcpyHostToDevice, ctx->stream));
        }
        const int g = gather_device(ctx, P, tokens, d_rep, ctx->data.as<uint8_t>());
        if (g != RSH_OK) return g;
        RSH_HIP(hipMemcpyAsync(target, ctx->data.p, (size_t)P.target_len, hipMemcpyDeviceToHost, ctx->stream));
        RSH_HIP(hipStreamSynchronize(ctx->stream));
        m.update(target, (size_t)P.target_len);
    }
    m.final(out->md5);
    return RSH_OK;
}

int rsh_receiver_combine_batch(rsh_ctx* ctx, rsh_combine_job* jobs, int32_t njobs) {
    if (!ctx || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    // (host) plan every file: the token walk of combineDataToFile, nothing written yet
    std::vector<RFile> files;
    std::vector<Md5File> md5_in;   // the digest of every planned file, from the host bytes its plan names
    std::vector<int32_t> md5_job;
    std::vector<std::vector<rsh_piece>> md5_pieces;
    for (int32_t i = 0; i < njobs; ++i) {
        rsh_combine_job& j = jobs[i];
        j.status = RSH_OK;
        j.res = rsh_combine_result{};
        if (!j.tokens || j.tokens_len < 0 || j.target_cap < 0 || j.nreplica < 0 || (j.nreplica > 0 && !j.replica)) {
            j.status = RSH_E_INVAL;
            continue;
        }
        RFile F;
        F.job = i;
        F.rep.init(j.replica, j.nreplica);
        bool bad = false;
        for (int32_t k = 0; k < j.nreplica; ++k) bad |= j.replica[k].len < 0 || (j.replica[k].len > 0 && !j.replica[k].data);
        if (bad) {
            j.status = RSH_E_INVAL;
            continue;
        }
        const int rc = plan_combine(j.tokens, j.tokens_len, j.h, j.nreplica > 0, F.rep.total(), j.defer_write != 0,
                                    &F.plan);
        if (rc != RSH_OK) {
            j.status = rc;
            continue;
        }
        fill_result(F.plan, &j.res);
        if (!F.plan.intact && F.plan.target_len > j.target_cap) {
            j.status = RSH_E_NOSPACE;
            continue;
        }
        if (!F.plan.intact && F.plan.target_len > 0 && !j.target) {
            j.status = RSH_E_INVAL;
            continue;
        }
        std::vector<rsh_piece> mp;  // the rebuilt file's bytes where they already are on the host
        if (F.plan.intact) {
            F.rep.each(0, F.plan.intact_len, [&](const uint8_t* d, int64_t n) { mp.push_back(rsh_piece{d, n}); });
        } else {
            for (const Piece& q : F.plan.pieces) {
                if (q.literal) mp.push_back(rsh_piece{j.tokens + q.src_off, q.len});
                else F.rep.each(q.src_off, q.len, [&](const uint8_t* d, int64_t n) { mp.push_back(rsh_piece{d, n}); });
            }
        }
        md5_pieces.push_back(std::move(mp));
        md5_job.push_back(i);
        if (!F.plan.intact && F.plan.target_len > 0) {
            plan_spans(F);
            files.push_back(std::move(F));
        }
    }
    for (size_t k = 0; k < md5_pieces.size(); ++k)
        md5_in.push_back(Md5File{md5_pieces[k].data(), (int32_t)md5_pieces[k].size()});
    std::vector<uint8_t> md5_out(md5_in.size() * 16 + 16);
    // (host) the digests on the cores beside the device passes: one serial chain per file, up to 16 per core
    const int md5_threads = std::max(1, call_cores() - (files.empty() ? 0 : 2));
    std::thread md5_thread([&] {
        md5_files(md5_in.data(), (int32_t)md5_in.size(), reinterpret_cast<uint8_t(*)[16]>(md5_out.data()), md5_threads,
                  (int)opt(OPT_MD5_WIDTH));
    });
    int rc = RSH_OK;
    std::vector<char> done((size_t)njobs, 0);
    if (!files.empty()) rc = combine_passes(ctx, jobs, files, done);
    md5_thread.join();
    for (size_t k = 0; k < md5_job.size(); ++k) memcpy(jobs[md5_job[k]].res.md5, md5_out.data() + 16 * k, 16);
    if (rc != RSH_OK) {
        for (const RFile& F : files)
            if (!done[(size_t)F.job] && jobs[F.job].status == RSH_OK) jobs[F.job].status = rc;
        return rc;
    }
    for (int32_t i = 0; i < njobs; ++i)
        if (jobs[i].status != RSH_OK) return jobs[i].status;
    return RSH_OK;
}

}  // extern "C"
