/*
 * aes_ref.c — AES-128 block cipher, byte-oriented restatement of FIPS-197.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  The reference reaches this primitive through
 * BoringSSL's EVP_aes_128_ecb (sub-key derivation, MV/src/mpi/pt2pt/send.c:583,
 * MV/src/mpi/init/init.c:842-849) and inside every AEAD/CTR call.
 *
 * Deliberately naive: S-box derived from the GF(2^8) inverse + affine map (FIPS-197 §5.1.1),
 * no T-tables, so it shares no structure with the GPU kernels it checks.
 */
#include "oracle.h"

#include <string.h>

static uint8_t SBOX[256];
static uint8_t INV_SBOX[256];
/* MUL[k][x] = x * {2,3,9,11,13,14}[k] in GF(2^8): precomputed from gf8_mul for speed only */
static uint8_t MUL[6][256];
enum { M2, M3, M9, M11, M13, M14 };

static uint8_t gf8_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  while (b) {
    if (b & 1) p ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0x00));
    b >>= 1;
  }
  return p;
}

static uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }

__attribute__((constructor)) static void orc_aes_init(void) {
  for (int x = 0; x < 256; ++x) {
    /* multiplicative inverse: x^254 (0 maps to 0) */
    uint8_t inv = 0;
    if (x) {
      uint8_t r = 1, base = (uint8_t)x;
      int e = 254;
      while (e) {
        if (e & 1) r = gf8_mul(r, base);
        base = gf8_mul(base, base);
        e >>= 1;
      }
      inv = r;
    }
    uint8_t s = (uint8_t)(inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63);
    SBOX[x] = s;
    INV_SBOX[s] = (uint8_t)x;
    static const uint8_t k[6] = {2, 3, 9, 11, 13, 14};
    for (int j = 0; j < 6; ++j) MUL[j][x] = gf8_mul((uint8_t)x, k[j]);
  }
}

void orc_aes128_expand(const uint8_t key[16], uint8_t rk[176]) {
  memcpy(rk, key, 16);
  uint8_t rcon = 0x01;
  for (int i = 4; i < 44; ++i) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % 4 == 0) {
      uint8_t t0 = t[0];
      t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
      t[1] = SBOX[t[2]];
      t[2] = SBOX[t[3]];
      t[3] = SBOX[t0];
      rcon = gf8_mul(rcon, 2);
    }
    for (int k = 0; k < 4; ++k) rk[4 * i + k] = (uint8_t)(rk[4 * (i - 4) + k] ^ t[k]);
  }
}

/* state s[r + 4c] = byte of row r, column c (input byte order, FIPS-197 §3.4) */
static void add_round_key(uint8_t s[16], const uint8_t *k) {
  for (int i = 0; i < 16; ++i) s[i] ^= k[i];
}

void orc_aes128_encrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16], t[16];
  memcpy(s, in, 16);
  add_round_key(s, rk);
  for (int round = 1; round <= 10; ++round) {
    for (int i = 0; i < 16; ++i) s[i] = SBOX[s[i]];                      /* SubBytes  */
    for (int c = 0; c < 4; ++c)                                           /* ShiftRows */
      for (int r = 0; r < 4; ++r) t[r + 4 * c] = s[r + 4 * ((c + r) % 4)];
    if (round != 10) {                                                    /* MixColumns */
      for (int c = 0; c < 4; ++c) {
        const uint8_t *a = t + 4 * c;
        s[4 * c + 0] = (uint8_t)(MUL[M2][a[0]] ^ MUL[M3][a[1]] ^ a[2] ^ a[3]);
        s[4 * c + 1] = (uint8_t)(a[0] ^ MUL[M2][a[1]] ^ MUL[M3][a[2]] ^ a[3]);
        s[4 * c + 2] = (uint8_t)(a[0] ^ a[1] ^ MUL[M2][a[2]] ^ MUL[M3][a[3]]);
        s[4 * c + 3] = (uint8_t)(MUL[M3][a[0]] ^ a[1] ^ a[2] ^ MUL[M2][a[3]]);
      }
    } else {
      memcpy(s, t, 16);
    }
    add_round_key(s, rk + 16 * round);
  }
  memcpy(out, s, 16);
}

void orc_aes128_decrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16], t[16];
  memcpy(s, in, 16);
  add_round_key(s, rk + 160);
  for (int round = 9; round >= 0; --round) {
    for (int c = 0; c < 4; ++c)                                           /* InvShiftRows */
      for (int r = 0; r < 4; ++r) t[r + 4 * ((c + r) % 4)] = s[r + 4 * c];
    for (int i = 0; i < 16; ++i) t[i] = INV_SBOX[t[i]];                   /* InvSubBytes  */
    add_round_key(t, rk + 16 * round);
    if (round != 0) {                                                     /* InvMixColumns */
      for (int c = 0; c < 4; ++c) {
        const uint8_t *a = t + 4 * c;
        s[4 * c + 0] = (uint8_t)(MUL[M14][a[0]] ^ MUL[M11][a[1]] ^ MUL[M13][a[2]] ^ MUL[M9][a[3]]);
        s[4 * c + 1] = (uint8_t)(MUL[M9][a[0]] ^ MUL[M14][a[1]] ^ MUL[M11][a[2]] ^ MUL[M13][a[3]]);
        s[4 * c + 2] = (uint8_t)(MUL[M13][a[0]] ^ MUL[M9][a[1]] ^ MUL[M14][a[2]] ^ MUL[M11][a[3]]);
        s[4 * c + 3] = (uint8_t)(MUL[M11][a[0]] ^ MUL[M13][a[1]] ^ MUL[M9][a[2]] ^ MUL[M14][a[3]]);
      }
    } else {
      memcpy(s, t, 16);
    }
  }
  memcpy(out, s, 16);
}

void orc_aes128_ecb(const uint8_t key[16], const uint8_t *in, uint8_t *out, size_t nblocks) {
  uint8_t rk[176];
  orc_aes128_expand(key, rk);
  for (size_t i = 0; i < nblocks; ++i) orc_aes128_encrypt(rk, in + 16 * i, out + 16 * i);
}
