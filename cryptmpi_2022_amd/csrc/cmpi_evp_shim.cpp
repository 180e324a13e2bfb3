// cmpi_evp_shim.cpp — libcmpi_evp.so: BoringSSL-ABI drop-in (include/cmpi_evp.h) forwarding
// CryptMPI's EVP calls to the MI355X engine (include/cmpi_aead.h).  Each EVP call becomes a
// batch of one record through the synchronous *_host entry points; the batched ABI is the fast
// path, this layer is the literal boundary CryptMPI's libmpi links against.
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "../../include/cmpi_aead.h"
#include "../../include/cmpi_evp.h"

struct evp_aead_st {
  int id;
};
struct evp_cipher_st {
  int alg;
};
struct evp_aead_ctx_st {
  cmpi_ctx* c;
};
struct evp_cipher_ctx_st {
  int alg = 0;             // CMPI_AES_128_CTR / _ECB, 0 = unset
  cmpi_ctx* c = nullptr;
  uint8_t iv[16] = {0};    // counter block at the start of the current stream
  uint64_t pos = 0;        // CTR bytes consumed since the last IV (EVP keeps `num` state)
  uint8_t partial[16];     // ECB: buffered bytes of an incomplete block
  int npartial = 0;
};

namespace {
const evp_aead_st kGcm{1};
const evp_cipher_st kCtr{CMPI_AES_128_CTR};
const evp_cipher_st kEcb{CMPI_AES_128_ECB};

int pick_device() {
  const char* vars[] = {"CMPI_DEVICE", "MV2_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK",
                        "LOCAL_RANK"};
  int n = cmpi_device_count();
  if (n <= 0) return 0;
  for (const char* v : vars) {
    const char* s = getenv(v);
    if (s && *s) return atoi(s) % n;
  }
  return 0;
}

void add128(uint8_t cb[16], uint64_t k) {
  unsigned carry = 0;
  for (int i = 15; i >= 0; --i) {
    unsigned s = (unsigned)cb[i] + (unsigned)(k & 0xff) + carry;
    cb[i] = (uint8_t)s;
    carry = s >> 8;
    k >>= 8;
  }
}

int cipher_init(EVP_CIPHER_CTX* ctx, const EVP_CIPHER* cipher, const uint8_t* key, const uint8_t* iv) {
  if (!ctx) return 0;
  if (cipher) {
    if (ctx->c && ctx->alg != cipher->alg) {
      cmpi_ctx_free(ctx->c);
      ctx->c = nullptr;
    }
    ctx->alg = cipher->alg;
  }
  if (!ctx->alg) return 0;
  if (key) {
    if (ctx->c) cmpi_ctx_free(ctx->c);
    ctx->c = cmpi_ctx_new(ctx->alg, key, 16, 0, pick_device());
    if (!ctx->c) return 0;
  }
  if (iv) memcpy(ctx->iv, iv, 16);
  if (iv || key) {
    ctx->pos = 0;
    ctx->npartial = 0;
  }
  return 1;
}

int cipher_update(EVP_CIPHER_CTX* ctx, uint8_t* out, int* out_len, const uint8_t* in, int in_len) {
  if (!ctx || !ctx->c || in_len < 0 || !out_len) return 0;
  *out_len = 0;
  if (in_len == 0) return 1;
  if (ctx->alg == CMPI_AES_128_CTR) {
    uint8_t cb[16];
    memcpy(cb, ctx->iv, 16);
    add128(cb, ctx->pos / 16);
    if (cmpi_ctr_xor_host(ctx->c, out, in, (size_t)in_len, cb, (unsigned)(ctx->pos % 16)) != CMPI_OK) return 0;
    ctx->pos += (uint64_t)in_len;
    *out_len = in_len;
    return 1;
  }
  // ECB, no padding on Update: emit whole blocks, keep the remainder
  int total = ctx->npartial + in_len;
  int full = total / 16 * 16;
  if (full == 0) {
    memcpy(ctx->partial + ctx->npartial, in, (size_t)in_len);
    ctx->npartial = total;
    return 1;
  }
  uint8_t* buf = (uint8_t*)malloc((size_t)full);
  if (!buf) return 0;
  memcpy(buf, ctx->partial, (size_t)ctx->npartial);
  memcpy(buf + ctx->npartial, in, (size_t)(full - ctx->npartial));
  int rest = total - full;
  uint8_t tail[16];
  memcpy(tail, in + (in_len - rest), (size_t)rest);
  int rc = cmpi_ecb_encrypt_host(ctx->c, out, buf, (size_t)full / 16);
  free(buf);
  if (rc != CMPI_OK) return 0;
  memcpy(ctx->partial, tail, (size_t)rest);
  ctx->npartial = rest;
  *out_len = full;
  return 1;
}
}  // namespace

extern "C" {

const EVP_AEAD* EVP_aead_aes_128_gcm(void) { return &kGcm; }
size_t EVP_AEAD_nonce_length(const EVP_AEAD*) { return 12; }
size_t EVP_AEAD_max_overhead(const EVP_AEAD*) { return 16; }

EVP_AEAD_CTX* EVP_AEAD_CTX_new(const EVP_AEAD* aead, const uint8_t* key, size_t key_len, size_t tag_len) {
  if (aead != &kGcm || key_len != 16 || !(tag_len == 0 || tag_len == 16)) return nullptr;
  cmpi_ctx* c = cmpi_ctx_new(CMPI_AES_128_GCM, key, key_len, tag_len, pick_device());
  if (!c) return nullptr;
  auto* ctx = new evp_aead_ctx_st;
  ctx->c = c;
  return ctx;
}

void EVP_AEAD_CTX_free(EVP_AEAD_CTX* ctx) {
  if (!ctx) return;
  cmpi_ctx_free(ctx->c);
  delete ctx;
}

int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX* ctx, uint8_t* out, size_t* out_len, size_t max_out_len,
                      const uint8_t* nonce, size_t nonce_len, const uint8_t* in, size_t in_len,
                      const uint8_t* ad, size_t ad_len) {
  (void)ad;
  if (ctx && out && out_len && nonce && nonce_len == 12 && ad_len == 0 && max_out_len >= in_len + 16 &&
      (in || in_len == 0) &&
      cmpi_gcm_seal_host(ctx->c, out, 0, in ? in : out, 0, nonce, 12, in_len, 1) == CMPI_OK) {
    *out_len = in_len + 16;
    return 1;
  }
  if (out) memset(out, 0, max_out_len);  // aead.h:251-253
  if (out_len) *out_len = 0;
  return 0;
}

int EVP_AEAD_CTX_open(const EVP_AEAD_CTX* ctx, uint8_t* out, size_t* out_len, size_t max_out_len,
                      const uint8_t* nonce, size_t nonce_len, const uint8_t* in, size_t in_len,
                      const uint8_t* ad, size_t ad_len) {
  (void)ad;
  if (ctx && out && out_len && nonce && in && nonce_len == 12 && ad_len == 0 && in_len >= 16 &&
      max_out_len >= in_len - 16) {
    int32_t st = 0;
    int rc = cmpi_gcm_open_host(ctx->c, out, 0, in, 0, nonce, 12, in_len - 16, 1, &st);
    if (rc == CMPI_OK && st == 1) {
      *out_len = in_len - 16;
      return 1;
    }
  }
  if (out) memset(out, 0, max_out_len);  // aead.h:276-278
  if (out_len) *out_len = 0;
  return 0;
}

const EVP_CIPHER* EVP_aes_128_ecb(void) { return &kEcb; }
const EVP_CIPHER* EVP_aes_128_ctr(void) { return &kCtr; }

EVP_CIPHER_CTX* EVP_CIPHER_CTX_new(void) { return new evp_cipher_ctx_st; }

void EVP_CIPHER_CTX_free(EVP_CIPHER_CTX* ctx) {
  if (!ctx) return;
  if (ctx->c) cmpi_ctx_free(ctx->c);
  delete ctx;
}

int EVP_EncryptInit_ex(EVP_CIPHER_CTX* ctx, const EVP_CIPHER* cipher, ENGINE*, const uint8_t* key,
                       const uint8_t* iv) {
  return cipher_init(ctx, cipher, key, iv);
}

int EVP_DecryptInit_ex(EVP_CIPHER_CTX* ctx, const EVP_CIPHER* cipher, ENGINE*, const uint8_t* key,
                       const uint8_t* iv) {
  if (ctx && ((cipher && cipher->alg == CMPI_AES_128_ECB) || (!cipher && ctx->alg == CMPI_AES_128_ECB)))
    return 0;  // ECB decryption is never used by CryptMPI and not provided by the engine
  return cipher_init(ctx, cipher, key, iv);
}

int EVP_EncryptUpdate(EVP_CIPHER_CTX* ctx, uint8_t* out, int* out_len, const uint8_t* in, int in_len) {
  return cipher_update(ctx, out, out_len, in, in_len);
}

int EVP_DecryptUpdate(EVP_CIPHER_CTX* ctx, uint8_t* out, int* out_len, const uint8_t* in, int in_len) {
  if (ctx && ctx->alg != CMPI_AES_128_CTR) return 0;
  return cipher_update(ctx, out, out_len, in, in_len);
}

}  // extern "C"
