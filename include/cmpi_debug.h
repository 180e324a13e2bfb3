/*
 * cmpi_debug.h — test hooks of libcmpi_aead.so (not part of the drop-in surface).
 * Used by tests/ to force every GCM work decomposition onto small inputs.
 */
#ifndef CMPI_DEBUG_H
#define CMPI_DEBUG_H

#include <stddef.h>
#include <stdint.h>

#include "cmpi_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Force GCM lanes-per-record (1, 2 or 4; anything else = automatic) and segments per record
 * (0 = automatic) for every subsequent launch in the process. */
void cmpi_debug_force_plan(int lanes_per_record, uint32_t segments);
/* Timing ablation of the GCM seal kernel (results become WRONG): 0 full, 1 no GHASH multiply,
 * 2 no AES, 3 neither, 4 coalesced stand-in addressing, 7 = 3 + 4, 8 = table staging only (first form,
 * gcm_batch_kernel); 16 no record loads/stores, 32 no AES, 48 both, 64 no GHASH, 80 AES only, 96 loads/stores only
 * (gcm_lane_kernel). */
void cmpi_debug_set_gcm_ablation(int mode);
/* CTR kernel occupancy experiment: dynamic LDS bytes requested (65536..163840; more than
 * 80 KiB forces one 1024-thread block per CU). */
void cmpi_debug_set_ctr_lds(int lds_bytes);
/* Wave priority in the main loops (default 7 | 16384): bit 0 GCM, bit 1 CTR, bit 2 OCB rotate it per
 * step; GCM lane kernel: bit 12 rotates per slot, bit 13 output-aligned windows, bit 14
 * progress-based priority (behind the workgroup average -> higher). */
void cmpi_debug_set_sched(int mode);
/* Chunk bytes of the pipelined host path (*_host calls; 0 = default 16 MiB). */
void cmpi_debug_set_host_chunk(size_t bytes);
/* GCM lane-group kernel: input prefetch depth in slots (2, 3, 4 or 6; anything else = 2). */
void cmpi_debug_set_gcm_prefetch(int slots);
/* GCM lane plan kernel: 0 = gcm_lane_kernel (default), 3 = gcm_lane_kernel with sector-aligned
 * windows where legal (writes 97 -> 81 MB per config-2 seal, ~10 % slower: off), 1 = the first
 * form gcm_batch_kernel (also selected by a prefetch depth other than 2, the cache-policy and
 * ablation knobs, sched bit 13).  Sched bit 15 keeps form 3's record-to-wave mapping without
 * its phases (A/B). */
void cmpi_debug_set_gcm_form(int form);
/* Diagnostics: when buf (device, >= 8 x grid u64) is non-null, every gcm_wide_kernel workgroup
   writes wall-clock (100 MHz) timestamps of its phases at buf[8*block + 0..6]: start, tables
   staged, own Horner done, all Horner done, weight tables staged, weights done, end. */
void cmpi_debug_set_wide_probe(void* buf);
/* Wide GCM decomposition (one wavefront per 64*steps-block chunk of a record, for few long
 * records): mode 0 automatic, 1 always when legal (host-keyed context, >= 64 data blocks),
 * -1 never; steps per chunk (0 = automatic). */
void cmpi_debug_force_wide(int mode, uint32_t steps);
/* Wide GCM plan, host-keyed contexts: 1 = barrier-free gcm_wide_kernel<FLOW> applying the chunk
   weights itself, the combine only XORs (default); 0 = phased kernel, weights in the combine kernel. */
void cmpi_debug_set_wide_chw(int on);
/* Kernel timing (bench.py): HIP events created with hipEventDisableSystemFence (no cache
   writeback/invalidate when recorded).  event_ms: elapsed ms between two recorded events after
   the stream has been synchronised, -1 on error. */
void* cmpi_debug_event_new(void);
int cmpi_debug_event_record(void* ev, void* stream);
float cmpi_debug_event_ms(void* a, void* b);
void cmpi_debug_event_free(void* ev);
/* FLOW wide GCM kernel (host-keyed, few long records): threads per workgroup 512 / 1024, or 0
 * for the round-1 gcm_wide_kernel; flags (default 1): bit 0 combine fused (last arriver), else a
 * separate gcm_xor_combine_kernel launch; bits 1-3 timing ablations that skip the lane tree (2),
 * the chunk-weight product (4), the AES (8) — outputs WRONG, for tools/ab_flow.py only; bit 4
 * the round-2 first form (byte-table Horner, radix-2 tree, gmul_wave4) instead of radix-4; bit 5
 * keeps `threads` even where the planner would pick 512-thread workgroups for few chunks. */
void cmpi_debug_set_flow(int threads, int fused);
/* FLOW kernel: a batch whose chunks all fit one workgroup finishes its tags in-kernel (1, default)
 * or through the XOR-combine launch (0, A/B). */
void cmpi_debug_set_flow_one_wg(int on);
/* Host-memory calls (cmpi_*_host) up to `bytes` of input + output records run the direct path
 * (kernel on page-locked host memory, no DMA); larger ones the 3-stream pipeline.  0 = never. */
void cmpi_debug_set_host_direct(size_t bytes);
/* GCM lane-group kernel: record data loaded (bit 0) / stored (bit 1) with the non-temporal policy. */
void cmpi_debug_set_gcm_mem(int mode);
/* Direct host path: wait for the kernel by polling the stream (1, default) or by a blocking
 * hipStreamSynchronize (0). */
void cmpi_debug_set_host_spin(int on);
/* The plan a GCM batch of nrec x len would use: out = {L, nseg, G, r0}; a wide plan reports
 * L = 64, nseg = chunks per record, G = X-blocks per chunk (64*steps). */
int cmpi_debug_gcm_plan(const cmpi_ctx *ctx, size_t len, size_t nrec, uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
