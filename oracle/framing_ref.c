/*
 * framing_ref.c — CryptMPI wire-framing helpers (nonce / header byte layouts).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * orc_nonce602: MV/src/mpi/pt2pt/send.c:651-670 (flag '4' path: local_nonce[0..7] = '0',
 *   [8..11] = BE32 segment) and :781-804 (pipeline path: [7] = '1' on the last segment);
 *   receiver rebuilds it from the 5-byte segment prefix, recv.c:594-607, :749-762.
 * orc_header600: MV/src/mpi/pt2pt/send.c:241-266 (MSG_HEADER_SIZE = 25).
 */
#include "oracle.h"

#include <string.h>

void orc_nonce602(uint8_t nonce[12], uint8_t flag, uint32_t seg) {
  memset(nonce, '0', 7);
  nonce[7] = flag;
  nonce[8] = (uint8_t)(seg >> 24);
  nonce[9] = (uint8_t)(seg >> 16);
  nonce[10] = (uint8_t)(seg >> 8);
  nonce[11] = (uint8_t)seg;
}

void orc_header600(uint8_t hdr[25], uint32_t total, uint8_t kind, uint32_t chunk) {
  hdr[0] = (uint8_t)(total >> 24);
  hdr[1] = (uint8_t)(total >> 16);
  hdr[2] = (uint8_t)(total >> 8);
  hdr[3] = (uint8_t)total;
  hdr[20] = kind;
  hdr[21] = (uint8_t)(chunk >> 24);
  hdr[22] = (uint8_t)(chunk >> 16);
  hdr[23] = (uint8_t)(chunk >> 8);
  hdr[24] = (uint8_t)chunk;
}
