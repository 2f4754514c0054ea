// device.h -- internal launchers for the gfx950 kernels in device.hip (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace rsh {

// Generator block sums (Generator.java:886-895): chunk c covers [c*B, min((c+1)*B, n)).
// Writes weak[c] and strong[c*dl .. c*dl+dl).  Also used by the Sender as aligned speculation.
// abort_flag (optional, host-pinned): the launch stops early, leaving its outputs undefined, once
// *abort_flag == abort_gen (the Sender's speculation when the resolver no longer needs it).
hipError_t launch_block_sums(const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks, uint32_t dl,
                             uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong, hipStream_t s,
                             const int* abort_flag = nullptr, int abort_gen = 0);

hipError_t launch_block_sums_variant(int variant, const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks,
                                     uint32_t dl, uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong,
                                     hipStream_t s, const int* abort_flag = nullptr, int abort_gen = 0);

// Chain flags for the Sender fast path: flag[k] = 1 iff source window k (aligned, from the source's
// own block sums) has the same weak key and the same dl-byte digest as basis chunk k.
hipError_t launch_chain_flags(const int32_t* d_wsrc, const uint8_t* d_ssrc, const int32_t* d_wbas,
                              const uint8_t* d_sbas, uint32_t count, uint32_t dl, uint8_t* d_flags,
                              hipStream_t s);

// Probe table: open-addressing hash of the distinct weak keys (key -> 1).  slots = power of two.
struct ProbeTable {
    const unsigned long long* slots;
    uint32_t mask;
};
hipError_t launch_table_clear(unsigned long long* d_slots, uint32_t nslots, hipStream_t s);
hipError_t launch_table_insert(unsigned long long* d_slots, uint32_t mask, const int32_t* d_keys, uint32_t nkeys,
                               hipStream_t s);

// Sender-side rolling key probe.  For each interval [a, b) the key is R(p) = T(p) + E(p), where T(p) is
// the true weak sum of window [p, p + min(B, n - p)) and E(p) = (e_lo, e_hi + e_lo * (min(p, n-B) -
// min(anchor, n-B))) mod 2^16 (the post-flush desync of Sender.java:1292-1310).  The work is cut into
// tiles of PROBE_TILE positions inside aligned blocks [kB, kB + B); aligned_weak[k] = T(kB) (the
// source's own block sums) anchors each block.  *first (uint64, preset to ~0 by the caller) receives
// the smallest hitting position over all tiles.
constexpr int PROBE_TILE = 4096;
struct ProbeIv {
    int64_t a, b, anchor;
    uint32_t e_lo, e_hi;
};
struct ProbeTile {
    int64_t q0;     // tile start (multiple of PROBE_TILE from its block start)
    int32_t iv;     // interval index
    int32_t pbase;  // index of its block's tile-0 partial sums in ProbeArgs::partials (unused for tile 0)
};
// Pass 1 of a probe: the four byte sums (x[j], (j - o) x[j] over the tile, and the same over the tile
// shifted by B) of every tile of a block that lies before a probed tile of that block, so that pass 2
// gets each tile's block prefix from at most 31 partials instead of re-reading up to B bytes per tile.
struct PartialTile {
    int64_t q0;
};
struct ProbeArgs {
    const uint8_t* data;
    int64_t n;
    uint32_t B;
    const int32_t* aligned_weak;
    ProbeTable table;
    const ProbeIv* ivs;
    const ProbeTile* tiles;
    const int4* partials;  // written by pass 1
    unsigned long long* first;
};
// Appends the tiles covering [a, b) for interval `iv` (host side).
void probe_tiles(int64_t a, int64_t b, int64_t B, int32_t iv, std::vector<ProbeTile>* out);
// Assigns ProbeTile::pbase and lists the partial tiles pass 1 computes (host side).
void probe_partials(std::vector<ProbeTile>* tiles, int64_t B, std::vector<PartialTile>* out);
// Both passes, back to back on stream s.
hipError_t launch_probe_first(const ProbeArgs& args, uint32_t ntiles, const PartialTile* d_ptiles, uint32_t nptiles,
                              int4* d_partials, hipStream_t s);
// After a probe: if *d_first holds a position p, the resolver's next questions answered in the same
// round trip, on stream s: the true weak sum T(p) into *h_weak, the window [p, p + min(B, n - p)) into
// pinned host memory h_win, and the bucket of the key R(p) = T(p) + E(p) (E from the interval holding
// p) in the received table d_table_weak[C]: *d_bucket = {count, key, idx[0 .. min(count, cap))}, in
// no particular order.
constexpr int HIT_BUCKET_CAP = 256;
hipError_t launch_hit_window(const uint8_t* d_data, int64_t n, uint32_t B, const unsigned long long* d_first,
                             const ProbeIv* ivs, int32_t niv, const int32_t* d_table_weak, int32_t C,
                             int32_t* d_bucket, int32_t* h_weak, uint8_t* h_win, hipStream_t s);

// n bytes of device memory into pinned host memory (h_dst 16-byte aligned), by a kernel.
hipError_t launch_copy_to_host(const uint8_t* d_src, int64_t n, uint8_t* h_dst, hipStream_t s);

// Bytes at arbitrary positions.
hipError_t launch_gather_bytes(const uint8_t* d_data, const int64_t* d_pos, uint32_t npos, uint8_t* d_out,
                               hipStream_t s);

// True weak sums at arbitrary positions: out[i] = Rolling.compute(data + pos[i], min(B, n - pos[i]))
// (by_block: written to out[pos[i] / B] instead, for aligned positions).
hipError_t launch_window_weak(const uint8_t* d_data, int64_t n, uint32_t B, const int64_t* d_pos, uint32_t npos,
                              int32_t* d_out, hipStream_t s, bool by_block = false);

// splitmix64 counter stream (bench input): byte i = byte (i % 8) of mix(key + (i / 8 + 1) * golden).
hipError_t launch_fill_splitmix(uint8_t* d_out, int64_t n, uint64_t key, int64_t byte_offset, hipStream_t s);

}  // namespace rsh
