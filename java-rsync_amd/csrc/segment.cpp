// segment.cpp -- a file-list segment from host memory: the entry points a Java Generator / Sender that holds a
// segment's files in JVM buffers calls once per segment instead of once per file.
//
//   Generator.itemizeSegment (Generator.java:558-614): every file's header + table, sendItemizeAndChecksums
//     (:866-909) per file                                            -> rsh_block_sums_batch
//   Sender.sendFiles (Sender.java:1098-1148): each file answered in turn by sendMatchesAndData (:1235-1327), the
//     whole-file MD5 last (:1241,1326)                                -> rsh_match_scan_batch
//
// A pass copies as many files as fit the segment budget (option segment_bytes, 16 GiB: a config-4 shard of
// 128 x 128 MiB is one pass) into HBM and runs the batched device forms over them (one K1 launch for every
// file's block sums; one resolver per file with the device round trips gathered per round, batch.cpp).  A file
// above the budget goes alone through the tiled single-file path (pieces.cpp).  The Sender's file MD5s -- one
// serial chain per file, the end-to-end bound of a single-file scan -- run on the host's cores while the files
// are copied and scanned, up to 16 files per core (md5_mb.cpp).
#include <thread>

#include "ctx.h"
#include "md5_mb.h"
#include "options.h"

namespace rsh {
int block_sums_pieces_claimed(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, int64_t n, const rsh_header* h,
                              const uint8_t seed[4], int32_t* weak_out, uint8_t* strong_out);
int scan_pieces_claimed(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, int64_t n, const rsh_header* h,
                        const int32_t* weak, const uint8_t* strong, const uint8_t seed[4], ResolveResult* r);
}  // namespace rsh

namespace {

constexpr int64_t kAlign = 256;  // file starts in a pass's HBM buffer (the K1's aligned path wants 128-B lines)

int64_t align_up(int64_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

// The pieces' total, or RSH_E_INVAL for a malformed list.
int64_t pieces_len(const rsh_piece* p, int32_t np) {
    if (np < 0 || (np > 0 && !p)) return RSH_E_INVAL;
    int64_t n = 0;
    for (int32_t i = 0; i < np; ++i) {
        if (p[i].len < 0 || (p[i].len > 0 && !p[i].data)) return RSH_E_INVAL;
        n += p[i].len;
    }
    return n;
}

hipError_t copy_pieces(const rsh_piece* p, int32_t np, uint8_t* dst, hipStream_t s) {
    for (int32_t i = 0; i < np; ++i) {
        if (p[i].len == 0) continue;
        const hipError_t e = hipMemcpyAsync(dst, p[i].data, (size_t)p[i].len, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        dst += p[i].len;
    }
    return hipSuccess;
}

int64_t budget() { return std::max<int64_t>(kAlign, rsh::opt(rsh::OPT_SEGMENT_BYTES)); }

// Fault injection (option fault_inject, tests only): the failure paths of a segment call must leave every
// unfinished file with a failing status.
bool fail_alloc() { return (rsh::opt(rsh::OPT_FAULT_INJECT) & 1) != 0 && rsh::fault_here(); }
hipError_t fail_copy(hipError_t e) {
    return e == hipSuccess && (rsh::opt(rsh::OPT_FAULT_INJECT) & 2) && rsh::fault_here() ? hipErrorInvalidValue : e;
}

// Passes over the files `idx` (in order): consecutive runs whose aligned sizes fit the budget; a file larger
// than the budget gets a pass of its own marked `alone`.
struct Pass {
    std::vector<int32_t> files;
    bool alone = false;
};
std::vector<Pass> plan_passes(const std::vector<int32_t>& idx, const std::vector<int64_t>& n) {
    std::vector<Pass> out;
    const int64_t cap = budget();
    int64_t used = 0;
    for (int32_t f : idx) {
        const int64_t sz = align_up(n[(size_t)f]);
        if (n[(size_t)f] > cap) {
            out.push_back(Pass{{f}, true});
            used = cap;  // the next file opens a new pass
            continue;
        }
        if (out.empty() || out.back().alone || used + sz > cap) {
            out.push_back(Pass{});
            used = 0;
        }
        out.back().files.push_back(f);
        used += sz;
    }
    return out;
}

}  // namespace

void rsh::add_scan_stats(rsh_scan_stats* to, const rsh_scan_stats& s) {
    to->chain_matches += s.chain_matches;
    to->events += s.events;
    to->probe_launches += s.probe_launches;
    to->host_md5_windows += s.host_md5_windows;
    to->flushes += s.flushes;
    to->device_ms += s.device_ms;
    to->resolver_ms += s.resolver_ms;
    to->table_ms += s.table_ms;
    to->head_steps += s.head_steps;
    to->speculation_aborted = std::max(to->speculation_aborted, s.speculation_aborted);
    to->device_bytes += s.device_bytes;
    to->phase_launches += s.phase_launches;
    to->phase_matches += s.phase_matches;
    to->spec_kernel_ms += s.spec_kernel_ms;
    to->phase_kernel_ms += s.phase_kernel_ms;
    to->phase_guesses += s.phase_guesses;
}

namespace {

// rsh_block_sums_batch's device work: the passes over `run` (validated files with chunks); done[f] once file f's
// sums are on the host.  Any early return is the call's status (the caller marks the unfinished files).
int block_sums_passes(rsh_ctx* ctx, rsh_block_batch_job* jobs, const std::vector<int32_t>& run,
                      const std::vector<int64_t>& n, const uint8_t seed[4], std::vector<char>& done) {
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    for (const Pass& pass : plan_passes(run, n)) {
        if (pass.alone) {  // larger than a pass: tile by tile (pieces.cpp)
            rsh_block_batch_job& j = jobs[pass.files[0]];
            j.status = rsh::block_sums_pieces_claimed(ctx, j.pieces, j.npieces, n[(size_t)pass.files[0]], &j.h, seed,
                                                      j.weak_out, j.strong_out);
            done[(size_t)pass.files[0]] = 1;
            if (j.status != RSH_OK) return j.status;
            continue;
        }
        int64_t data_bytes = 0, sum_bytes = 0;
        for (int32_t f : pass.files) {
            data_bytes += align_up(n[(size_t)f]);
            sum_bytes += align_up(4 * (int64_t)jobs[f].h.chunk_count) +
                         align_up((int64_t)jobs[f].h.chunk_count * jobs[f].h.digest_length);
        }
        if (fail_alloc() || ctx->seg_data.ensure((size_t)data_bytes + kAlign) != hipSuccess ||
            ctx->seg_tab.ensure((size_t)sum_bytes + kAlign) != hipSuccess) {
            snprintf(g_last_err, sizeof(g_last_err), "segment pass of %lld bytes: device memory (segment.cpp)",
                     (long long)(data_bytes + sum_bytes));
            return RSH_E_NOMEM;
        }
        std::vector<rsh_block_job> bj;
        int64_t doff = 0, soff = 0;
        for (int32_t f : pass.files) {
            const rsh_block_batch_job& j = jobs[f];
            uint8_t* d = ctx->seg_data.as<uint8_t>() + doff;
            uint8_t* w = ctx->seg_tab.as<uint8_t>() + soff;
            uint8_t* s = w + align_up(4 * (int64_t)j.h.chunk_count);
            RSH_HIP(fail_copy(copy_pieces(j.pieces, j.npieces, d, ctx->stream)));
            bj.push_back(rsh_block_job{d, n[(size_t)f], j.h, w, s});
            doff += align_up(n[(size_t)f]);
            soff += align_up(4 * (int64_t)j.h.chunk_count) + align_up((int64_t)j.h.chunk_count * j.h.digest_length);
        }
        const int rc = rsh::block_sums_batch_claimed(ctx, bj.data(), (int32_t)bj.size(), seed);
        if (rc != RSH_OK) return rc;
        for (size_t k = 0; k < bj.size(); ++k) {
            rsh_block_batch_job& j = jobs[pass.files[k]];
            const size_t C = (size_t)j.h.chunk_count, dl = (size_t)j.h.digest_length;
            RSH_HIP(hipMemcpyAsync(j.weak_out, bj[k].d_weak, C * 4, hipMemcpyDeviceToHost, ctx->stream));
            if (dl) RSH_HIP(hipMemcpyAsync(j.strong_out, bj[k].d_strong, C * dl, hipMemcpyDeviceToHost, ctx->stream));
        }
        RSH_HIP(hipStreamSynchronize(ctx->stream));
        for (int32_t f : pass.files) done[(size_t)f] = 1;
    }
    return RSH_OK;
}

}  // namespace

extern "C" {

int rsh_file_md5_batch(rsh_md5_job* jobs, int32_t njobs, int32_t threads) {
    if (njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    std::vector<rsh::Md5File> files((size_t)njobs);
    for (int32_t i = 0; i < njobs; ++i) {
        if (pieces_len(jobs[i].pieces, jobs[i].npieces) < 0) return RSH_E_INVAL;
        files[(size_t)i] = rsh::Md5File{jobs[i].pieces, jobs[i].npieces};
    }
    std::vector<uint8_t> out((size_t)njobs * 16 + 16);
    rsh::md5_files(files.data(), njobs, reinterpret_cast<uint8_t(*)[16]>(out.data()),
                   threads > 0 ? threads : rsh::host_cores(), (int)rsh::opt(rsh::OPT_MD5_WIDTH));
    for (int32_t i = 0; i < njobs; ++i) memcpy(jobs[i].md5, out.data() + 16 * (size_t)i, 16);
    return RSH_OK;
}

int rsh_block_sums_batch(rsh_ctx* ctx, rsh_block_batch_job* jobs, int32_t njobs, const uint8_t seed[4]) {
    if (!ctx || !seed || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    std::vector<int64_t> n((size_t)njobs, 0);
    std::vector<int32_t> run;  // files with chunks
    for (int32_t i = 0; i < njobs; ++i) {
        rsh_block_batch_job& j = jobs[i];
        j.status = RSH_OK;
        n[(size_t)i] = pieces_len(j.pieces, j.npieces);
        if (n[(size_t)i] < 0) {
            j.status = RSH_E_INVAL;
            continue;
        }
        j.status = check_generator_header(n[(size_t)i], &j.h);
        if (j.status != RSH_OK || j.h.chunk_count == 0) continue;
        if (!j.weak_out || (!j.strong_out && j.h.digest_length > 0)) {
            j.status = RSH_E_INVAL;
            continue;
        }
        run.push_back(i);
    }
    if (!run.empty()) {
        // every file of `run` is finished (its sums on the host) once its flag is set; a failure leaves the others
        // carrying the call's code, never RSH_OK with unwritten sums
        std::vector<char> done((size_t)njobs, 0);
        const int rc = block_sums_passes(ctx, jobs, run, n, seed, done);
        if (rc != RSH_OK) {
            (void)hipStreamSynchronize(ctx->stream);  // no copy from the caller's buffers outlives the call
            for (int32_t i : run)
                if (!done[(size_t)i] && jobs[i].status == RSH_OK) jobs[i].status = rc;
            return rc;
        }
    }
    for (int32_t i = 0; i < njobs; ++i)
        if (jobs[i].status != RSH_OK) return jobs[i].status;
    return RSH_OK;
}

int rsh_match_scan_batch(rsh_ctx* ctx, rsh_scan_batch_job* jobs, int32_t njobs, const uint8_t seed[4],
                         rsh_scan_stats* stats) {
    if (!ctx || !seed || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    if (stats) *stats = rsh_scan_stats{};
    std::vector<int64_t> n((size_t)njobs, 0);
    std::vector<int32_t> ok;        // every file with a valid job (its MD5 runs)
    std::vector<int32_t> dev, host; // ... scanned in passes / handed to the device batch without bytes
    for (int32_t i = 0; i < njobs; ++i) {
        rsh_scan_batch_job& j = jobs[i];
        j.status = RSH_OK;
        j.n_ev = j.literal = j.matched = 0;
        memset(j.file_md5, 0, 16);
        n[(size_t)i] = pieces_len(j.pieces, j.npieces);
        if (n[(size_t)i] < 0) {
            j.status = RSH_E_INVAL;
            continue;
        }
        const int v = rsh_header_validate(&j.h);
        if (v != RSH_OK) {
            j.status = v;
            continue;
        }
        const size_t C = (size_t)j.h.chunk_count, dl = (size_t)j.h.digest_length;
        if (j.h.block_length > 0 && n[(size_t)i] > 0 && C > 0 && (!j.weak || (!j.strong && dl > 0))) {
            j.status = RSH_E_INVAL;
            continue;
        }
        ok.push_back(i);
        (j.h.block_length > 0 && n[(size_t)i] > 0 ? dev : host).push_back(i);
    }
    if (ok.empty()) {
        for (int32_t i = 0; i < njobs; ++i)
            if (jobs[i].status != RSH_OK) return jobs[i].status;
        return RSH_OK;
    }
    // A failure leaves no file it did not finish at RSH_OK (zero counts must never read as a result):
    // every such file carries the call's code.
    std::vector<char> done((size_t)njobs, 0);
    auto fail_unfinished = [&](int code) {
        for (int32_t i : ok)
            if (!done[(size_t)i] && jobs[i].status == RSH_OK) jobs[i].status = code;
        return code;
    };
    CtxClaim claim_(ctx);
    if (!claim_.held) {
        snprintf(g_last_err, sizeof(g_last_err), "context in use by another thread");
        return fail_unfinished(RSH_E_BUSY);
    }
    if (const hipError_t e = hipSetDevice(ctx->device); e != hipSuccess) {
        note_error(e, __LINE__, "segment.cpp");
        return fail_unfinished(RSH_E_DEVICE);
    }
    // every file's MD5 beside the copies and the scans.  The cores are split: the MD5 pool takes all but
    // kScanCores, the batched scan's coordinator and resolver workers those (after the chain walks a segment
    // leaves a file or two to the host resolvers); together they stay within the process's cores.
    constexpr int kScanCores = 3;
    const int cores = rsh::call_cores();
    const int md5_threads = std::max(1, cores - kScanCores);
    rsh::WorkerCap cap(std::max(1, cores - md5_threads));
    std::vector<rsh::Md5File> mf;
    for (int32_t i : ok) mf.push_back(rsh::Md5File{jobs[i].pieces, jobs[i].npieces});
    std::vector<uint8_t> md5((size_t)ok.size() * 16 + 16);
    std::thread md5_thread([&] {
        rsh::md5_files(mf.data(), (int32_t)mf.size(), reinterpret_cast<uint8_t(*)[16]>(md5.data()), md5_threads,
                       (int)rsh::opt(rsh::OPT_MD5_WIDTH));
    });
    int rc = RSH_OK;
    // new files (skipMatchSendData) and empty sources: no bytes to copy
    if (!host.empty()) {
        std::vector<rsh_scan_job> sj;
        for (int32_t i : host) {
            const rsh_scan_batch_job& j = jobs[i];
            rsh_scan_job x{};
            x.n = n[(size_t)i];
            x.h = j.h;
            x.ev = j.ev;
            x.ev_cap = j.ev_cap;
            sj.push_back(x);
        }
        rc = rsh::match_scan_batch_claimed(ctx, sj.data(), (int32_t)sj.size(), seed, nullptr);
        for (size_t k = 0; k < sj.size(); ++k) {
            rsh_scan_batch_job& j = jobs[host[k]];
            j.status = sj[k].status;
            j.n_ev = sj[k].n_ev;
            j.literal = sj[k].literal;
            j.matched = sj[k].matched;
            if (rc == RSH_OK || rc == RSH_E_NOSPACE) done[(size_t)host[k]] = 1;
        }
        if (rc == RSH_E_NOSPACE) rc = RSH_OK;  // per file
    }
    for (const Pass& pass : plan_passes(dev, n)) {
        if (rc != RSH_OK && rc != RSH_E_NOSPACE) break;
        if (pass.alone) {  // larger than a pass: the tiled single-file scan
            rsh_scan_batch_job& j = jobs[pass.files[0]];
            rsh::ResolveResult r;
            j.status = rsh::scan_pieces_claimed(ctx, j.pieces, j.npieces, n[(size_t)pass.files[0]], &j.h, j.weak,
                                                j.strong, seed, &r);
            if (j.status == RSH_OK) {
                j.literal = r.literal;
                j.matched = r.matched;
                if (stats) rsh::add_scan_stats(stats, r.stats);
                j.status = emit_events(ctx, r, j.ev, j.ev_cap, &j.n_ev);
            }
            done[(size_t)pass.files[0]] = 1;
            if (j.status != RSH_OK && j.status != RSH_E_NOSPACE) rc = j.status;
            continue;
        }
        int64_t data_bytes = 0, tab_bytes = 0;
        for (int32_t f : pass.files) {
            data_bytes += align_up(n[(size_t)f]);
            tab_bytes += align_up(4 * (int64_t)jobs[f].h.chunk_count) +
                         align_up((int64_t)jobs[f].h.chunk_count * jobs[f].h.digest_length);
        }
        if (fail_alloc() || ctx->seg_data.ensure((size_t)data_bytes + kAlign) != hipSuccess ||
            ctx->seg_tab.ensure((size_t)tab_bytes + kAlign) != hipSuccess) {
            snprintf(g_last_err, sizeof(g_last_err), "segment pass of %lld bytes: device memory (segment.cpp)",
                     (long long)(data_bytes + tab_bytes));
            rc = RSH_E_NOMEM;
            break;
        }
        std::vector<rsh_scan_job> sj;
        int64_t doff = 0, toff = 0;
        hipError_t e = hipSuccess;
        for (int32_t f : pass.files) {
            const rsh_scan_batch_job& j = jobs[f];
            const size_t C = (size_t)j.h.chunk_count, dl = (size_t)j.h.digest_length;
            uint8_t* d = ctx->seg_data.as<uint8_t>() + doff;
            uint8_t* w = ctx->seg_tab.as<uint8_t>() + toff;
            uint8_t* s = w + align_up(4 * (int64_t)C);
            if (e == hipSuccess) e = fail_copy(copy_pieces(j.pieces, j.npieces, d, ctx->stream));
            if (e == hipSuccess && C) e = hipMemcpyAsync(w, j.weak, C * 4, hipMemcpyHostToDevice, ctx->stream);
            if (e == hipSuccess && C && dl) e = hipMemcpyAsync(s, j.strong, C * dl, hipMemcpyHostToDevice, ctx->stream);
            rsh_scan_job x{};
            x.d_src = d;
            x.n = n[(size_t)f];
            x.h = j.h;
            x.d_weak = w;
            x.d_strong = s;
            x.ev = j.ev;
            x.ev_cap = j.ev_cap;
            sj.push_back(x);
            doff += align_up(x.n);
            toff += align_up(4 * (int64_t)C) + align_up((int64_t)(C * dl));
        }
        if (e != hipSuccess) {
            note_error(e, __LINE__, "segment.cpp");
            rc = RSH_E_DEVICE;
            break;
        }
        rsh_scan_stats ps{};
        const int prc = rsh::match_scan_batch_claimed(ctx, sj.data(), (int32_t)sj.size(), seed, stats ? &ps : nullptr);
        for (size_t k = 0; k < sj.size(); ++k) {
            rsh_scan_batch_job& j = jobs[pass.files[k]];
            j.status = sj[k].status;
            j.n_ev = sj[k].n_ev;
            j.literal = sj[k].literal;
            j.matched = sj[k].matched;
            if (prc == RSH_OK || prc == RSH_E_NOSPACE) done[(size_t)pass.files[k]] = 1;
        }
        if (stats) rsh::add_scan_stats(stats, ps);
        if (prc != RSH_OK && prc != RSH_E_NOSPACE) rc = prc;
    }
    md5_thread.join();
    if (rc != RSH_OK) (void)hipStreamSynchronize(ctx->stream);  // no copy from the caller's buffers outlives the call
    for (size_t k = 0; k < ok.size(); ++k) memcpy(jobs[ok[k]].file_md5, md5.data() + 16 * k, 16);
    if (rc != RSH_OK) return fail_unfinished(rc);
    for (int32_t i = 0; i < njobs; ++i)
        if (jobs[i].status != RSH_OK) return jobs[i].status;
    return RSH_OK;
}

}  // extern "C"
