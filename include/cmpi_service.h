/*
 * cmpi_service.h — resident message service (opt-in, per context).
 *
 * CryptMPI seals and opens most point-to-point messages one at a time through the EVP API
 * (MPI_SEC_Multi_Thread_Send_OpenMP: EVP_AEAD_CTX_seal per message, MV/src/mpi/pt2pt/send.c:294-315;
 * the receiver's EVP_AEAD_CTX_open, recv.c:322).  On the device every such message otherwise costs
 * a kernel launch, the staging of the tables and the host's completion wait.  With the service
 * started, single GCM messages from host memory — cmpi_gcm_seal_host / cmpi_gcm_open_host with
 * nrec = 1 and len <= 512 KiB, and therefore the EVP drop-in's per-message calls — are handed to a
 * kernel that stays resident on 8 CUs with its tables in LDS, polls a page-locked request ring and
 * writes one page-locked completion slot per workgroup that served the message (its share of the
 * tag); the host combines the slots into the tag, writes a seal's and checks an open's.  Outputs,
 * statuses and errors are those of the calls it serves (bit-exact; forged messages zero-filled,
 * CMPI_EAUTH).
 *
 * The kernel returns its CUs after `idle_us` microseconds without a message (0 = 2000) and at
 * least every 100 ms; the next message relaunches it.  While it runs it occupies 8 CUs: large
 * batches launched meanwhile on other streams share the remaining CUs.  The kernel also holds
 * the hardware queue of its stream: HIP maps streams of one priority onto at most
 * GPU_MAX_HW_QUEUES hardware queues, and work on a stream that shares a resident kernel's queue
 * waits until it exits.  The services of a device therefore run on 4 shared stream slots of the
 * greatest priority (normal-priority streams — the caller's, torch's, the library's others —
 * never share them), at most one resident generation per slot: a service that needs a slot held
 * by another context's kicks that generation, which leaves after the message it is serving, and
 * queues behind it (6 contexts round-robin: p99 31 µs per message instead of 20 ms).  Other
 * greatest-priority streams of the process may still share a slot's queue.
 * hipDeviceSynchronize / torch.cuda.synchronize() wait for the kernels to exit: call
 * cmpi_service_stop first, or keep idle_us short.
 * On an AES-128-CTR context the service serves CryptMPI's counter-mode small messages instead
 * (cmpi_ctrmode.h, cmpi_ring.h: the 702 ring XOR, send.c:1273-1465; the receiver's premask and
 * mask XOR, recv.c:954-1023, :1107-1220; the 700 / 702 direct CTR of messages up to 64 KiB;
 * cmpi_ctr_xor_host, the EVP shim's EVP_EncryptUpdate, on host buffers):
 * each such op of at most 64 KiB is posted to the kernel instead of launched, and is complete
 * when the call returns.  It runs outside stream order, so the call first waits for the work
 * already queued on its `stream` (and for the ring's last fill); bytes, headers and ring state
 * are those of the launched form.
 * On an AES-128-ECB context it serves cmpi_ecb_encrypt_host of up to 64 KiB (the 602 sub-key
 * derivation, send.c:583).
 * Host-keyed AES-128-GCM, -CTR and -ECB contexts only (CMPI_EINVAL otherwise).  cmpi_ctx_rekey and
 * cmpi_ctx_rekey_subkey stop a running service (the next message restarts it with the new key;
 * a device-keyed context ends the service).  cmpi_ctx_free stops it.
 */
#ifndef CMPI_SERVICE_H
#define CMPI_SERVICE_H

#include <stdint.h>

#include "cmpi_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

int cmpi_service_start(cmpi_ctx *ctx, uint32_t idle_us);
int cmpi_service_stop(cmpi_ctx *ctx);
/* 1 while a service kernel of this context is resident, else 0. */
int cmpi_service_running(const cmpi_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
