/*
 * cmpi_debug.h — test hooks of libcmpi_aead.so (not part of the drop-in surface).
 * Used by tests/ to force every GCM work decomposition onto small inputs, and by bench.py for
 * kernel timing.  Every hook picks among correct decompositions: none changes an output byte.
 * (Kernel phase probes exist only in the diagnostics build, tools/libcmpi_aead_tools.so.)
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
/* Chunk bytes of the pipelined host path (*_host calls; 0 = automatic: 8 MiB when records,
 * outputs and nonces are page-locked, else 16 MiB). */
void cmpi_debug_set_host_chunk(size_t bytes);
/* Staging slots (chunks in flight) of the pipelined host path: 2..4, anything else = default 3. */
void cmpi_debug_set_host_slots(int slots);
/* Wide GCM decomposition (gcm_flow_kernel: one wavefront per 64*steps-block chunk of a record,
 * for few long records): mode 0 automatic, 1 always when legal (>= 64 data blocks), -1 never;
 * steps per chunk (0 = automatic; rounded down to a power of two on device-keyed contexts). */
void cmpi_debug_force_wide(int mode, uint32_t steps);
/* Kernel timing (bench.py): HIP events created with hipEventDisableSystemFence (no cache
   writeback/invalidate when recorded).  event_ms: elapsed ms between two recorded events after
   the stream has been synchronised, -1 on error. */
void* cmpi_debug_event_new(void);
/* Streaming device-to-device copy of n bytes (n % 16 == 0, 16-byte aligned), asynchronous on
   `stream`: bench.py's measured HBM peak (16 B per lane, grid-stride over 4 workgroups per CU:
   the fastest of the forms measured, ctr_kernels.hpp copy16_kernel). */
int cmpi_debug_copy(void* dst, const void* src, size_t n, void* stream);
int cmpi_debug_event_record(void* ev, void* stream);
float cmpi_debug_event_ms(void* a, void* b);
void cmpi_debug_event_free(void* ev);
/* Kernel timing (bench.py's roofline): the kernels the calling thread launches through the library
 * from now on go through hipExtLaunchKernel, the first with start_ev and each with stop_ev, so the
 * pair times the next call's kernels themselves (first start to last end; rocprofv3's view), not
 * the stream between two records.  (NULL, NULL) ends it. */
void cmpi_debug_time_next_launch(void* start_ev, void* stop_ev);
/* gcm_flow_kernel threads per workgroup: 0 automatic (always 512 since round 4: the 1024-thread
 * form spills), 512 or 1024 forced (the chunk plan then assumes that many waves per CU). */
void cmpi_debug_set_flow_threads(int threads);
/* ctr_kernel workgroups per CU (1 or 2; default 2 = every VGPR of the CU): 1 leaves room for a
 * co-resident kernel (tools/probe/hybrid_ctr_probe.hip). */
void cmpi_debug_set_ctr_wg_per_cu(int n);
/* gcm_lane_kernel (L = 4) record stores grouped by 128-byte output line (each line stored whole in
 * the step that completes it), on batches of at least one group per thread of the grid: 2 =
 * predicated selects (default), 1 = branches, 0 = a store per step; 3 / 4 = the select / branch
 * form on every batch (tests). */
void cmpi_debug_set_lane_pair(int on);
/* resident service: smallest chunk length exponent (chunks of 64·2^ls blocks, 0..3; 0 default),
 * taken at the service's next launch. */
void cmpi_debug_set_svc_ls_min(int ls);
/* Test hook: service shutdowns (cmpi_service_stop, re-key, cmpi_ctx_free) treat the stop as failed
 * and the generation as still resident, so the service object is leaked, never freed while a stream
 * slot may still name it (1 on, 0 off). */
void cmpi_debug_set_svc_fake_stuck(int on);
/* FLOW kernel: a batch whose chunks all fit one workgroup finishes its tags in-kernel (1, default)
 * or through the XOR-combine launch (0). */
void cmpi_debug_set_flow_one_wg(int on);
/* Host-memory calls (cmpi_*_host) up to `bytes` of input + output records run the direct path
 * (kernel on page-locked host memory, no DMA); larger ones the 3-stream pipeline.  0 = never. */
void cmpi_debug_set_host_direct(size_t bytes);
/* Host pipeline (cmpi_gcm/ocb_*_host, batches above the direct threshold), how chunks move:
 * 0 = hipMemcpyAsync both ways; 1 = the kernel writes page-locked dense outputs (and open's
 * statuses) over PCIe itself; 4 = hipMemcpyAsync H2D, D2H on an SDMA engine through HSA;
 * 5 (default) = both directions on SDMA through HSA, the calling thread launching each chunk's
 * kernel when its input landed (page-locked records, outputs and nonces, more than one chunk;
 * otherwise mode 4's D2H where the outputs allow, otherwise mode 0).  Anything else = 5.
 * Process-wide. */
void cmpi_debug_set_host_out_direct(int mode);
/* Direct host path: how the host waits for a call's kernels — 0 blocking hipStreamSynchronize,
 * 1 spin on a host word written by hipStreamWriteValue32, 2 the same word written by a one-wave
 * kernel, 3 polling hipStreamQuery. */
void cmpi_debug_set_host_spin(int mode);
/* Framed host-memory requests (602 / 700 / 702 *_host calls) whose input + output spans total at
 * most `bytes` run direct: the kernels access the page-locked spans over PCIe, no DMA copies
 * (default 16 MiB; 0 = always DMA). */
void cmpi_debug_set_span_direct(size_t bytes);
/* How the library creates its own streams from now on (host pipeline, async request pool,
 * message service): 0 non-blocking (default), 1 non-blocking at the greatest priority,
 * 2 CU-masked over every CU (a hardware queue of its own). */
void cmpi_debug_set_stream_mode(int mode);
/* The plan a GCM batch of nrec x len would use: out = {L, nseg, G, r0}; a wide plan reports
 * L = 64, nseg = chunks per record, G = X-blocks per chunk (64*steps). */
int cmpi_debug_gcm_plan(const cmpi_ctx *ctx, size_t len, size_t nrec, uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
