/*
 * rsync_hip_debug.h -- testing and diagnostics ABI of librsynchip.so (not part of the drop-in boundary of
 * rsync_hip.h; a Java binding never calls it).
 *
 * The library's tunables and diagnostic switches (java-rsync_amd/csrc/options.h) have compiled-in defaults and
 * are never read from the environment.  The table is per process and applies to calls that start after a change.
 *  - settable in every build (tests force rare paths with them; a few are tunables): k1_gather, k1_shift,
 *    k1_unaligned, scan_trace, scan_segmented, scan_samples, batch_chain, batch_chain_prefix, host_cores,
 *    file_tile, file_tile_above, probe_long, segment_bytes, md5_width, chain_helpers, chain_map_bytes, time_gen, batch_warm,
 *    fault_inject;
 *  - A/B switches, settable only in the diagnostics build (make diag: lib/diag/librsynchip.so, loaded by the
 *    tools through RSH_LIB); the product library answers RSH_E_INVAL and runs their defaults: scan_diag,
 *    scan_phase, scan_phase_guess, scan_preprobe, scan_sample, scan_spec_order, scan_early, scan_wait,
 *    scan_defer_steps, scan_defer_us, scan_spec_queue, scan_flags_host, scan_prep_pieces, time_spec, batch_spec,
 *    batch_spin_us, batch_readahead, batch_prep_all, batch_chain_overlap, batch_skip_rest, chain_help_tiles.
 */
#ifndef RSYNC_HIP_DEBUG_H
#define RSYNC_HIP_DEBUG_H

#include <stdint.h>

#include "rsync_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RSH_OK, or RSH_E_INVAL for an unknown name or an A/B switch in the product build. */
int rsh_debug_set_option(const char* name, int64_t value);
int rsh_debug_get_option(const char* name, int64_t* value);
/* Every option back to its compiled-in default. */
void rsh_debug_reset_options(void);

/* The duration of a K1 from its own dispatch timestamps (HIP events recorded by the launch, hipExtLaunchKernelGGL):
 * which 0 = the last rsh_block_sums_device's K1 (the Generator), 1 = the last single-file scan's aligned speculation
 * when it ran to completion.  *ms = -1 when that launch was not timed (a shape whose kernel takes no events). */
int rsh_debug_kernel_ms(rsh_ctx* ctx, int32_t which, double* ms);

/* The context's launch generation (the abort and hit-map words' values): *gen its current value; set >= 0 (at most
 * the wrap point, 0x7FFFFF00) sets it first -- tests take a context across the wrap, where the device drains and every
 * abort and map word goes back to 0 (rsh_ctx::next_gen).  set = -1 only reads. */
int rsh_debug_generation(rsh_ctx* ctx, int32_t set, int32_t* gen);

/* Which of the context's streams still have work queued or running (hipStreamQuery): bit 0 the context stream,
 * bit 1 aux (the aligned speculation), bit 2 phase (the phase-shifted speculation).  After rsh_ctx_sync it is 0. */
int rsh_debug_streams_busy(rsh_ctx* ctx, int32_t* mask);

/* The clock the chip holds under the Generator's K1 (MI355X_MICROARCH.md, "DVFS give-back" item 6): reps launches of
 * a diagnostic instantiation of the production K1 body over the device bytes [d_data, d_data + n) (n a multiple of
 * 64 * block_length, block_length a multiple of 128) with each wave's s_memtime / s_memrealtime ticks stamped around
 * it; *clock_ghz = sum of shader ticks / sum of 100 MHz ticks x 0.1.  The production kernels never stamp.  bench.py
 * reports it beside the headline (k1_clock_ghz). */
int rsh_debug_k1_clock(rsh_ctx* ctx, const void* d_data, int64_t n, int32_t block_length, int32_t reps,
                       double* clock_ghz);

/* The multi-context segment driver (rsh_*_batch_multi: split, one member call per part, merge) with a stand-in member
 * call and no device: part p's call records per job its part (part_out) and its position among the part's files
 * (order_out); part fail_part (-1: none) finishes its first file and fails the rest with RSH_E_DEVICE.  status_out:
 * every job's status after the merge.  Returns the driver's status. */
int rsh_debug_multi_selftest(const int64_t* bytes, int32_t njobs, int32_t nparts, int32_t fail_part, int32_t* part_out,
                             int32_t* order_out, int32_t* status_out);

#ifdef __cplusplus
}
#endif
#endif
