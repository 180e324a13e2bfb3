// aes_tables.hpp — AES-128 constant tables generated at compile time (constexpr) from the
// GF(2^8) definitions of FIPS-197 §4, §5.1.1; no table literals.
//
// Word convention used everywhere in this library: a 16-byte block is 4 little-endian 32-bit
// words w[c] = bytes 4c..4c+3, i.e. AES state column c with row r at bits 8r..8r+7.  With
// that convention
//   Te0[x] = { 2·S[x], S[x], S[x], 3·S[x] }  (bytes 0..3),  Te_r[x] = rotl32(Te0[x], 8r)
//   Td0[x] = { 14·Si[x], 9·Si[x], 13·Si[x], 11·Si[x] },     Td_r[x] = rotl32(Td0[x], 8r)
// and S[x] = (Te0[x] >> 8) & 0xff, so the last encryption round needs no extra table.
#pragma once
#include <stdint.h>

namespace cmpi {

struct AesTables {
  uint8_t sbox[256];
  uint8_t inv_sbox[256];
  uint32_t te0[256];
  uint32_t td0[256];
};

constexpr uint8_t gf8_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) p ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return p;
}

constexpr AesTables make_aes_tables() {
  AesTables t{};
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x) {
      uint8_t r = 1, base = (uint8_t)x;
      for (int e = 254; e; e >>= 1) {
        if (e & 1) r = gf8_mul(r, base);
        base = gf8_mul(base, base);
      }
      inv = r;
    }
    uint8_t s = inv;
    for (int k = 1; k <= 4; ++k) s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    s ^= 0x63;
    t.sbox[x] = s;
    t.inv_sbox[s] = (uint8_t)x;
  }
  for (int x = 0; x < 256; ++x) {
    uint8_t s = t.sbox[x], si = t.inv_sbox[x];
    t.te0[x] = (uint32_t)gf8_mul(s, 2) | ((uint32_t)s << 8) | ((uint32_t)s << 16) |
               ((uint32_t)gf8_mul(s, 3) << 24);
    t.td0[x] = (uint32_t)gf8_mul(si, 14) | ((uint32_t)gf8_mul(si, 9) << 8) |
               ((uint32_t)gf8_mul(si, 13) << 16) | ((uint32_t)gf8_mul(si, 11) << 24);
  }
  return t;
}

inline constexpr AesTables kAes = make_aes_tables();

// FIPS-197 §5.2 key expansion; rk[i] = LE word of key-schedule bytes 4i..4i+3.
inline void aes128_expand_words(const uint8_t key[16], uint32_t rk[44]) {
  uint8_t w[176];
  for (int i = 0; i < 16; ++i) w[i] = key[i];
  uint8_t rcon = 1;
  for (int i = 4; i < 44; ++i) {
    uint8_t t0 = w[4 * i - 4], t1 = w[4 * i - 3], t2 = w[4 * i - 2], t3 = w[4 * i - 1];
    if (i % 4 == 0) {
      uint8_t a = t0;
      t0 = (uint8_t)(kAes.sbox[t1] ^ rcon);
      t1 = kAes.sbox[t2];
      t2 = kAes.sbox[t3];
      t3 = kAes.sbox[a];
      rcon = gf8_mul(rcon, 2);
    }
    w[4 * i + 0] = (uint8_t)(w[4 * i - 16] ^ t0);
    w[4 * i + 1] = (uint8_t)(w[4 * i - 15] ^ t1);
    w[4 * i + 2] = (uint8_t)(w[4 * i - 14] ^ t2);
    w[4 * i + 3] = (uint8_t)(w[4 * i - 13] ^ t3);
  }
  for (int i = 0; i < 44; ++i)
    rk[i] = (uint32_t)w[4 * i] | ((uint32_t)w[4 * i + 1] << 8) | ((uint32_t)w[4 * i + 2] << 16) |
            ((uint32_t)w[4 * i + 3] << 24);
}

// Equivalent inverse cipher round keys (FIPS-197 §5.3.5): drk[0..3] = rk[40..43],
// drk[4r..4r+3] = InvMixColumns(rk[40-4r..]) for r = 1..9, drk[40..43] = rk[0..3].
inline void aes128_dec_words(const uint32_t rk[44], uint32_t drk[44]) {
  for (int r = 0; r <= 10; ++r) {
    for (int c = 0; c < 4; ++c) {
      uint32_t w = rk[4 * (10 - r) + c];
      if (r == 0 || r == 10) {
        drk[4 * r + c] = w;
        continue;
      }
      uint8_t a[4] = {(uint8_t)w, (uint8_t)(w >> 8), (uint8_t)(w >> 16), (uint8_t)(w >> 24)};
      uint8_t o[4];
      o[0] = gf8_mul(a[0], 14) ^ gf8_mul(a[1], 11) ^ gf8_mul(a[2], 13) ^ gf8_mul(a[3], 9);
      o[1] = gf8_mul(a[0], 9) ^ gf8_mul(a[1], 14) ^ gf8_mul(a[2], 11) ^ gf8_mul(a[3], 13);
      o[2] = gf8_mul(a[0], 13) ^ gf8_mul(a[1], 9) ^ gf8_mul(a[2], 14) ^ gf8_mul(a[3], 11);
      o[3] = gf8_mul(a[0], 11) ^ gf8_mul(a[1], 13) ^ gf8_mul(a[2], 9) ^ gf8_mul(a[3], 14);
      drk[4 * r + c] = (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16) | ((uint32_t)o[3] << 24);
    }
  }
}

// Host scalar AES-128 encryption with the same word convention (ctx setup only: H = E_K(0)).
inline void aes128_encrypt_words_host(const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]) {
  uint32_t s[4], t[4];
  for (int c = 0; c < 4; ++c) s[c] = in[c] ^ rk[c];
  auto rotl = [](uint32_t x, int n) { return (x << n) | (x >> (32 - n)); };
  for (int r = 1; r < 10; ++r) {
    for (int c = 0; c < 4; ++c)
      t[c] = kAes.te0[s[c] & 0xff] ^ rotl(kAes.te0[(s[(c + 1) & 3] >> 8) & 0xff], 8) ^
             rotl(kAes.te0[(s[(c + 2) & 3] >> 16) & 0xff], 16) ^ rotl(kAes.te0[s[(c + 3) & 3] >> 24], 24) ^
             rk[4 * r + c];
    for (int c = 0; c < 4; ++c) s[c] = t[c];
  }
  for (int c = 0; c < 4; ++c)
    out[c] = ((uint32_t)kAes.sbox[s[c] & 0xff] | ((uint32_t)kAes.sbox[(s[(c + 1) & 3] >> 8) & 0xff] << 8) |
              ((uint32_t)kAes.sbox[(s[(c + 2) & 3] >> 16) & 0xff] << 16) |
              ((uint32_t)kAes.sbox[s[(c + 3) & 3] >> 24] << 24)) ^
             rk[40 + c];
}

}  // namespace cmpi
