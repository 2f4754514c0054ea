// multi.cpp -- a file-list segment over several contexts: the GPUs of one node inside one transfer.
//
// north_star: "files shard embarrassingly across the 8 GPUs of one node".  In the reference one thread walks every
// file of a transfer: the Generator sums each file of a segment in turn (Generator.itemizeSegment,
// Generator.java:558-614 -> sendItemizeAndChecksums :866-909; the segment loop :806-860), one Sender thread answers
// each (Sender.sendFiles, Sender.java:978-1170 -> sendMatchesAndData :1235-1327) and one Receiver thread rebuilds each
// (Receiver.receiveFiles, Receiver.java:1145-1263).  A file's work depends only on that file, its table and the seed,
// so the segment forms here split the files over the calling thread's contexts (one per GPU, or several on one GPU)
// and run each context's share as the single-context segment call (segment.cpp, receiver.cpp) on a host thread of its
// own.  No data moves between the devices, and no collective is needed.
//
//   split    rsh_shard_files: longest first by bytes, each file to the context with the fewest bytes so far (ties to
//            the lower index); a context's files keep their segment order.  The same rule as shard.py's rank split.
//   run      one member call per context that got files, side by side; the process's cores are split evenly among
//            them (CoreShare, ctx.h), so the members' MD5 pools and resolver workers together stay within the cores.
//   merge    every job's outputs and status are copied back into the caller's job (file order is the jobs' order);
//            a member that fails marks only the files it had not finished, exactly as the single-context call does.
//            The call returns RSH_OK, or the first failing job's status in file order.
#include <thread>

#include "ctx.h"
#include "options.h"

namespace rsh {
namespace {

int64_t pieces_bytes(const rsh_piece* p, int32_t np) {
    if (np <= 0 || !p) return 0;
    int64_t n = 0;
    for (int32_t i = 0; i < np; ++i) n += p[i].len > 0 ? p[i].len : 0;
    return n;
}

// Whether the contexts can serve one multi call: at least one, none null, no context twice (a context serves one
// call at a time; the same context as two members would make one of them fail with RSH_E_BUSY).
bool ctxs_ok(rsh_ctx* const* ctxs, int32_t nctx) {
    if (nctx < 1 || !ctxs) return false;
    for (int32_t i = 0; i < nctx; ++i) {
        if (!ctxs[i]) return false;
        for (int32_t k = 0; k < i; ++k)
            if (ctxs[k] == ctxs[i]) return false;
    }
    return true;
}

}  // namespace

// The split, the member calls and the merge (see the top of the file).  member(p, sub, n) runs part p's jobs -- copies
// of the caller's, in file order -- and returns the member call's status; status_of reads a job's status.
template <class Job, class Member, class Status>
int run_members(int32_t nparts, Job* jobs, int32_t njobs, const std::vector<int64_t>& bytes, Member&& member,
                Status&& status_of) {
    std::vector<int32_t> part((size_t)njobs + 1, 0);
    if (njobs > 0) rsh_shard_files(bytes.data(), njobs, nparts, part.data());
    std::vector<std::vector<int32_t>> idx((size_t)nparts);
    for (int32_t f = 0; f < njobs; ++f) idx[(size_t)part[(size_t)f]].push_back(f);
    std::vector<int32_t> active;
    for (int32_t p = 0; p < nparts; ++p)
        if (!idx[(size_t)p].empty()) active.push_back(p);
    const int share = std::max(1, call_cores() / std::max<int>(1, (int)active.size()));
    std::vector<std::vector<Job>> sub((size_t)nparts);
    std::vector<int> rc((size_t)nparts, RSH_OK);
    for (int32_t p : active)
        for (int32_t f : idx[(size_t)p]) sub[(size_t)p].push_back(jobs[f]);
    auto run = [&](int32_t p) {
        CoreShare cs(share);
        rc[(size_t)p] = member(p, sub[(size_t)p].data(), (int32_t)sub[(size_t)p].size());
    };
    std::vector<std::thread> th;
    for (size_t k = 1; k < active.size(); ++k) th.emplace_back(run, active[k]);
    if (!active.empty()) run(active[0]);  // the calling thread serves the first member
    for (std::thread& t : th) t.join();
    for (int32_t p : active)
        for (size_t k = 0; k < idx[(size_t)p].size(); ++k) jobs[idx[(size_t)p][k]] = sub[(size_t)p][k];
    for (int32_t f = 0; f < njobs; ++f)
        if (status_of(jobs[f]) != RSH_OK) return status_of(jobs[f]);
    for (int32_t p : active)
        if (rc[(size_t)p] != RSH_OK) return rc[(size_t)p];
    return RSH_OK;
}

// Fault injection (option fault_inject bit 2, tests only): bits 0 / 1 apply only to member 1 of a multi call.
struct MemberFaults {
    static bool& here() {
        static thread_local bool v = false;
        return v;
    }
};
bool fault_here() { return !(opt(OPT_FAULT_INJECT) & 4) || MemberFaults::here(); }

namespace {
// Member p's call on its context, with member 1's fault scope set when fault_inject asks for it.
template <class Fn>
int member_call(int32_t p, Fn&& fn) {
    const bool saved = MemberFaults::here();
    MemberFaults::here() = p == 1;
    const int rc = fn();
    MemberFaults::here() = saved;
    return rc;
}
}  // namespace

}  // namespace rsh

using namespace rsh;

extern "C" {

int rsh_shard_files(const int64_t* bytes, int32_t nfiles, int32_t nparts, int32_t* part_out) {
    if (nfiles < 0 || nparts < 1 || (nfiles > 0 && (!bytes || !part_out))) return RSH_E_INVAL;
    std::vector<int32_t> order((size_t)nfiles);
    for (int32_t i = 0; i < nfiles; ++i) order[(size_t)i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return bytes[a] > bytes[b]; });
    std::vector<int64_t> load((size_t)nparts, 0);
    for (int32_t f : order) {
        int32_t best = 0;
        for (int32_t p = 1; p < nparts; ++p)
            if (load[(size_t)p] < load[(size_t)best]) best = p;
        part_out[f] = best;
        load[(size_t)best] += bytes[f];
    }
    return RSH_OK;
}

int rsh_block_sums_batch_multi(rsh_ctx* const* ctxs, int32_t nctx, rsh_block_batch_job* jobs, int32_t njobs,
                               const uint8_t seed[4]) {
    if (!ctxs_ok(ctxs, nctx) || !seed || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    if (nctx == 1) return rsh_block_sums_batch(ctxs[0], jobs, njobs, seed);
    std::vector<int64_t> bytes((size_t)njobs);
    for (int32_t f = 0; f < njobs; ++f) bytes[(size_t)f] = pieces_bytes(jobs[f].pieces, jobs[f].npieces);
    return run_members(
        nctx, jobs, njobs, bytes,
        [&](int32_t p, rsh_block_batch_job* sub, int32_t n) {
            return member_call(p, [&] { return rsh_block_sums_batch(ctxs[p], sub, n, seed); });
        },
        [](const rsh_block_batch_job& j) { return j.status; });
}

int rsh_match_scan_batch_multi(rsh_ctx* const* ctxs, int32_t nctx, rsh_scan_batch_job* jobs, int32_t njobs,
                               const uint8_t seed[4], rsh_scan_stats* stats) {
    if (!ctxs_ok(ctxs, nctx) || !seed || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    if (nctx == 1) return rsh_match_scan_batch(ctxs[0], jobs, njobs, seed, stats);
    if (stats) *stats = rsh_scan_stats{};
    std::vector<int64_t> bytes((size_t)njobs);
    for (int32_t f = 0; f < njobs; ++f) bytes[(size_t)f] = pieces_bytes(jobs[f].pieces, jobs[f].npieces);
    std::vector<rsh_scan_stats> ps((size_t)nctx);
    const int rc = run_members(
        nctx, jobs, njobs, bytes,
        [&](int32_t p, rsh_scan_batch_job* sub, int32_t n) {
            return member_call(p, [&] {
                return rsh_match_scan_batch(ctxs[p], sub, n, seed, stats ? &ps[(size_t)p] : nullptr);
            });
        },
        [](const rsh_scan_batch_job& j) { return j.status; });
    if (stats)
        for (const rsh_scan_stats& s : ps) add_scan_stats(stats, s);
    return rc;
}

int rsh_receiver_combine_batch_multi(rsh_ctx* const* ctxs, int32_t nctx, rsh_combine_job* jobs, int32_t njobs) {
    if (!ctxs_ok(ctxs, nctx) || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    if (nctx == 1) return rsh_receiver_combine_batch(ctxs[0], jobs, njobs);
    // a file's work is its rebuilt bytes: about its replica (mostly matched) or its token stream (mostly literal)
    std::vector<int64_t> bytes((size_t)njobs);
    for (int32_t f = 0; f < njobs; ++f)
        bytes[(size_t)f] = std::max<int64_t>(std::max<int64_t>(jobs[f].tokens_len, 0),
                                             pieces_bytes(jobs[f].replica, jobs[f].nreplica));
    return run_members(
        nctx, jobs, njobs, bytes,
        [&](int32_t p, rsh_combine_job* sub, int32_t n) {
            return member_call(p, [&] { return rsh_receiver_combine_batch(ctxs[p], sub, n); });
        },
        [](const rsh_combine_job& j) { return j.status; });
}

// The split / run / merge driver with a stand-in member call (no device): part p's call records, per job, the member
// and its position among the member's files (order_out) and -- for p == fail_part -- finishes its first file and fails
// the rest with RSH_E_DEVICE, as a member call that loses its device does.  status_out: every job's status after the
// merge; returns the driver's status.  CPU tests of the split, the merge order and a per-member failure.
int rsh_debug_multi_selftest(const int64_t* bytes, int32_t njobs, int32_t nparts, int32_t fail_part, int32_t* part_out,
                             int32_t* order_out, int32_t* status_out) {
    if (njobs < 0 || nparts < 1 || (njobs > 0 && (!bytes || !part_out || !order_out || !status_out))) return RSH_E_INVAL;
    struct FakeJob {
        int32_t file, part, order, status;
    };
    std::vector<FakeJob> jobs((size_t)njobs + 1);
    std::vector<int64_t> b(bytes, bytes + njobs);
    for (int32_t f = 0; f < njobs; ++f) jobs[(size_t)f] = FakeJob{f, -1, -1, RSH_E_INVAL};
    const int rc = run_members(
        nparts, jobs.data(), njobs, b,
        [&](int32_t p, FakeJob* sub, int32_t n) {
            for (int32_t k = 0; k < n; ++k) {
                sub[k].part = p;
                sub[k].order = k;
                sub[k].status = (p == fail_part && k > 0) ? RSH_E_DEVICE : RSH_OK;
            }
            return (p == fail_part && n > 1) ? RSH_E_DEVICE : RSH_OK;
        },
        [](const FakeJob& j) { return j.status; });
    for (int32_t f = 0; f < njobs; ++f) {
        if (jobs[(size_t)f].file != f) return RSH_E_INVAL;  // the merge put another file's job here
        part_out[f] = jobs[(size_t)f].part;
        order_out[f] = jobs[(size_t)f].order;
        status_out[f] = jobs[(size_t)f].status;
    }
    return rc;
}

}  // extern "C"
