// gf128_host.hpp — host-side GF(2^128) arithmetic in GCM's bit order (SP 800-38D §6.3) and the
// builders of the per-key GHASH lookup tables the HIP kernels stage into LDS.
//
// A field element is kept as its 16 memory bytes (byte 0 bit 7 = coefficient of x^0).  The
// kernels XOR tables in that same memory order, so no bit reflection is ever performed on
// the device.  All of this runs once per key (ctx setup), mirroring BoringSSL's
// CRYPTO_ghash_init / gcm_init_* precomputation that EVP_AEAD_CTX_new triggers.
#pragma once
#include <stdint.h>
#include <string.h>

namespace cmpi {

struct Blk {
  uint8_t b[16];
};

inline uint64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}
inline void put_be64(uint8_t* p, uint64_t v) {
  for (int i = 7; i >= 0; --i) {
    p[i] = (uint8_t)v;
    v >>= 8;
  }
}

inline Blk gf_mul(const Blk& x, const Blk& y) {
  uint64_t zh = 0, zl = 0, vh = be64(y.b), vl = be64(y.b + 8);
  for (int i = 0; i < 128; ++i) {
    if ((x.b[i >> 3] >> (7 - (i & 7))) & 1) {
      zh ^= vh;
      zl ^= vl;
    }
    uint64_t lsb = vl & 1;
    vl = (vl >> 1) | (vh << 63);
    vh = (vh >> 1) ^ (lsb ? 0xE100000000000000ULL : 0);
  }
  Blk z;
  put_be64(z.b, zh);
  put_be64(z.b + 8, zl);
  return z;
}

inline Blk gf_one() {
  Blk o{};
  o.b[0] = 0x80;
  return o;
}

inline Blk gf_pow(const Blk& h, uint64_t e) {
  Blk r = gf_one(), b = h;
  while (e) {
    if (e & 1) r = gf_mul(r, b);
    b = gf_mul(b, b);
    e >>= 1;
  }
  return r;
}

// Byte-position table for multiplication by P, value-major: tab[v*16 + p] = (block with
// byte p = v) · P.  16 × 256 × 16 B = 64 KiB.  X·P = XOR_p tab[X[p]*16 + p].  (Value-major so a
// wave's lanes, each visiting a different position p at a given step, hit distinct LDS slots.)
inline void build_byte_table(const Blk& P, Blk* tab) {
  for (int p = 0; p < 16; ++p) {
    Blk basis[8];
    for (int k = 0; k < 8; ++k) {
      Blk e{};
      e.b[p] = (uint8_t)(1u << k);
      basis[k] = gf_mul(e, P);
    }
    for (int v = 0; v < 256; ++v) {
      Blk acc{};
      for (int k = 0; k < 8; ++k)
        if (v & (1 << k))
          for (int i = 0; i < 16; ++i) acc.b[i] ^= basis[k].b[i];
      tab[v * 16 + p] = acc;
    }
  }
}

// Columns of the linear maps X -> X^(2^i), i = 1..31: mat[(i-1)*128 + k] = (x^k)^(2^i), where
// x^k is the element with only GCM-order bit k set (byte k/8, bit 7 - k%8).  31 x 2 KiB.
inline void build_sq_columns(Blk* mat) {
  for (int k = 0; k < 128; ++k) {
    Blk v{};
    v.b[k >> 3] = (uint8_t)(0x80u >> (k & 7));
    for (int i = 1; i <= 31; ++i) {
      v = gf_mul(v, v);
      mat[(i - 1) * 128 + k] = v;
    }
  }
}

// Nibble-position table: tab[(2p)*16 + v] = (byte p = v<<4)·P, tab[(2p+1)*16 + v] = (byte p = v)·P.
// 32 × 16 × 16 B = 8 KiB.
inline void build_nibble_table(const Blk& P, Blk* tab) {
  for (int p = 0; p < 16; ++p) {
    for (int half = 0; half < 2; ++half) {
      for (int v = 0; v < 16; ++v) {
        Blk e{};
        e.b[p] = (uint8_t)(half == 0 ? (v << 4) : v);
        tab[(2 * p + half) * 16 + v] = gf_mul(e, P);
      }
    }
  }
}

}  // namespace cmpi
