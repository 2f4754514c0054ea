/*
 * rsync_hip_debug.h -- testing and diagnostics ABI of librsynchip.so (not part of the drop-in boundary of
 * rsync_hip.h; a Java binding never calls it).
 *
 * The library's tunables and diagnostic switches (java-rsync_amd/csrc/options.h) have compiled-in defaults and
 * are never read from the environment.  Tests set them to force paths the default policy takes only on rare
 * shapes; bench.py --opt NAME=VALUE and the tools use them for A/B runs.  The table is per process and
 * applies to calls that start after the change.  Names: k1_gather, k1_shift, k1_unaligned, scan_trace,
 * scan_diag, scan_phase, scan_phase_guess, scan_segmented, scan_preprobe, scan_samples, scan_sample,
 * scan_spec_order, scan_early, scan_wait, scan_defer_steps, scan_defer_us, batch_spec, batch_spin_us,
 * batch_readahead, batch_prep_all, batch_chain, batch_chain_prefix, batch_chain_overlap, host_cores, file_tile,
 * file_tile_above, probe_long.
 */
#ifndef RSYNC_HIP_DEBUG_H
#define RSYNC_HIP_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* RSH_OK, or RSH_E_INVAL for an unknown name. */
int rsh_debug_set_option(const char* name, int64_t value);
int rsh_debug_get_option(const char* name, int64_t* value);
/* Every option back to its compiled-in default. */
void rsh_debug_reset_options(void);

#ifdef __cplusplus
}
#endif
#endif
