// receiver.cpp -- the Receiver's side of the delta: rebuild a file from the Sender's token stream and the
// replica (Receiver.combineDataToFile, Receiver.java:459-555), with the blocks gathered on the device.
//
// The token walk is sequential and cheap (one int per block or per <= 8 KiB literal), so it runs on the
// host and produces a list of byte ranges; the bytes themselves move on the device: literal bytes in one
// upload, replica blocks as device-to-device gathers (one launch for the whole file).  The digest the
// Receiver compares with the Sender's file MD5 (:824-842) is one serial MD5 chain over the rebuilt file;
// it runs on the host while the next piece of the file comes back over PCIe.
#include "ctx.h"
#include "host_md5.h"

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

}  // extern "C"
