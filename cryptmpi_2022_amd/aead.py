"""Python mirror of the reference's crypto interface for the hot path, over libcmpi_aead.so.

CryptMPI calls BoringSSL's EVP_AEAD_CTX_* (MV/boringssl-master/include/openssl/aead.h:208-285)
and EVP_EncryptInit_ex/EVP_EncryptUpdate for CTR/ECB (cipher.h:158-191) once per message.  This
module exposes the same operations, plus the batched forms the GPU engine is built for:

  AeadCtx(key, "aes-128-gcm"|"aes-128-ocb")  ~ EVP_AEAD_CTX_new(EVP_aead_aes_128_gcm(), key, 16, 0)
  ctx.seal(nonce, pt) -> ct||tag               ~ EVP_AEAD_CTX_seal (host bytes, one record)
  ctx.open(nonce, ct_tag) -> pt | None         ~ EVP_AEAD_CTX_open (None = the 0 return)
  ctx.seal_batch / open_batch                  device-resident uniform batches (torch tensors)
  CipherCtx(key, "aes-128-ctr"|"aes-128-ecb")  ~ EVP_CIPHER_CTX + EVP_EncryptInit_ex
  iv_count(iv, cter)                           ~ IV_Count (MV/src/mpi/pt2pt/send.c:1019-1030)

Device tensors are torch uint8 CUDA(HIP) tensors; the engine receives their raw device
pointers and the current torch stream.  Nothing here computes crypto on the host.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N

_ALGS = {"aes-128-gcm": N.CMPI_AES_128_GCM, "aes-128-ocb": N.CMPI_AES_128_OCB,
         "aes-128-ctr": N.CMPI_AES_128_CTR, "aes-128-ecb": N.CMPI_AES_128_ECB}

TAG_LEN = 16
NONCE_LEN = 12


def _stream_ptr(stream) -> int | None:
    import torch

    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def _dptr(t) -> int:
    if t is None:
        return None
    assert t.is_cuda, "device tensor expected"
    return t.data_ptr()


class _Ctx:
    def __init__(self, key: bytes, alg: str, device: int = 0, _handle=None):
        self.alg = alg
        if _handle is not None:
            self._h = _handle
        else:
            key = bytes(key)
            kb = (ctypes.c_uint8 * len(key)).from_buffer_copy(key)
            self._h = N.lib().cmpi_ctx_new(_ALGS[alg], kb, len(key), 0, device)
        if not self._h:
            raise N.CmpiError(N.CMPI_EINVAL, N.last_error())
        self.device = N.lib().cmpi_ctx_device(self._h)

    def close(self):
        if getattr(self, "_h", None) and N is not None and N.lib is not None:  # N is None at interpreter exit
            N.lib().cmpi_ctx_free(self._h)
        self._h = None

    __del__ = close

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ resident message service
    def service_start(self, idle_us: int = 0) -> None:
        """Serve this context's single host messages (GCM: seal_host/open_host with nrec = 1,
        <= 512 KiB; CTR: the 700 / 702 ops of messages <= 64 KiB, synchronously) from a resident
        kernel (include/cmpi_service.h); it returns its CUs after `idle_us` (0 = 2000) without a
        message and restarts on the next."""
        N.check(N.lib().cmpi_service_start(self._h, idle_us))

    def service_stop(self) -> None:
        N.check(N.lib().cmpi_service_stop(self._h))

    def service_running(self) -> bool:
        return bool(N.lib().cmpi_service_running(self._h))


class AeadCtx(_Ctx):
    """AES-128-GCM (default) or AES-128-OCB AEAD context: 12-byte nonce, 16-byte tag, no AAD."""

    def __init__(self, key: bytes, alg: str = "aes-128-gcm", device: int = 0, _handle=None):
        if alg not in ("aes-128-gcm", "aes-128-ocb"):
            raise ValueError(alg)
        super().__init__(key, alg, device, _handle)
        self._gcm = alg == "aes-128-gcm"

    @classmethod
    def subkey602(cls, base: "_Ctx", v: bytes) -> "AeadCtx":
        """GCM context for K' = AES-ECB_K(V) (send.c:572-600), K' derived on the GPU."""
        vb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(v))
        h = N.lib().cmpi_ctx_new_subkey(base.handle, vb)
        if not h:
            raise N.CmpiError(N.CMPI_EINVAL, N.last_error())
        return cls(b"", "aes-128-gcm", _handle=h)

    @classmethod
    def derive_subkey(cls, base: "_Ctx", v: bytes, stream=None) -> "AeadCtx":
        """Stream-ordered 602 sub-key context: K' = AES_K(V), its schedule and GHASH tables are
        built by one device kernel on `stream` (K' never reaches the host)."""
        vb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(v))
        h = N.lib().cmpi_ctx_derive_subkey(base.handle, vb, _stream_ptr(stream))
        if not h:
            raise N.CmpiError(N.CMPI_EINVAL, N.last_error())
        return cls(b"", "aes-128-gcm", _handle=h)

    def rekey(self, key: bytes, stream=None) -> None:
        """Re-key this context in place to the host key `key` (cmpi_ctx_rekey: tables rebuilt on
        the device, on `stream`; the drop-in's EVP_AEAD_CTX_new path)."""
        kb = (ctypes.c_uint8 * len(key)).from_buffer_copy(bytes(key))
        N.check(N.lib().cmpi_ctx_rekey(self._h, kb, len(key), _stream_ptr(stream)))

    def rekey_subkey(self, base: "_Ctx", v: bytes, stream=None) -> None:
        """Re-key this GCM context in place to K' = AES_K(V) on `stream` (no allocation)."""
        vb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(v))
        N.check(N.lib().cmpi_ctx_rekey_subkey(self._h, base.handle, vb, _stream_ptr(stream)))

    # ------------------------------------------------------------ device-resident batches
    def seal_batch(self, out, inp, nonces, length: int, nrec: int, *, in_stride=None, out_stride=None,
                   nonce_stride=NONCE_LEN, workspace=None, stream=None) -> None:
        """out[i] = ct||tag of inp[i] (uniform records; byte strides; torch uint8 device tensors)."""
        in_stride = length if in_stride is None else in_stride
        out_stride = length + TAG_LEN if out_stride is None else out_stride
        fn = N.lib().cmpi_gcm_seal_batch if self._gcm else N.lib().cmpi_ocb_seal_batch
        N.check(fn(self._h, _dptr(out), out_stride, _dptr(inp), in_stride, _dptr(nonces), nonce_stride,
                   length, nrec, _dptr(workspace), _stream_ptr(stream)))

    def open_batch(self, out, inp, nonces, length: int, nrec: int, *, status=None, in_stride=None,
                   out_stride=None, nonce_stride=NONCE_LEN, workspace=None, stream=None) -> None:
        """out[i] = pt of ct||tag inp[i]; status[i] (int32 device tensor) = 1 ok / 0 forged."""
        in_stride = length + TAG_LEN if in_stride is None else in_stride
        out_stride = length if out_stride is None else out_stride
        fn = N.lib().cmpi_gcm_open_batch if self._gcm else N.lib().cmpi_ocb_open_batch
        N.check(fn(self._h, _dptr(out), out_stride, _dptr(inp), in_stride, _dptr(nonces), nonce_stride,
                   length, nrec, _dptr(status), _dptr(workspace), _stream_ptr(stream)))

    def workspace_size(self, length: int, nrec: int) -> int:
        fn = N.lib().cmpi_gcm_workspace_size if self._gcm else N.lib().cmpi_ocb_workspace_size
        return fn(self._h, length, nrec)

    # ------------------------------------------------------------ host (EVP_AEAD_CTX_seal/open)
    def seal_host_batch(self, nonces: np.ndarray, pt: np.ndarray) -> np.ndarray:
        """(N,12) nonces, (N,n) plaintexts (host) -> (N, n+16) ct||tag through the pipelined host
        path (chunked H2D / kernel / D2H on three streams)."""
        nrec, n = pt.shape
        out = np.empty((nrec, n + TAG_LEN), np.uint8)
        pt = np.ascontiguousarray(pt)
        nonces = np.ascontiguousarray(nonces)
        fn = N.lib().cmpi_gcm_seal_host if self._gcm else N.lib().cmpi_ocb_seal_host
        N.check(fn(self._h, out.ctypes.data, out.strides[0], pt.ctypes.data, max(pt.strides[0], 1),
                   nonces.ctypes.data, 12, n, nrec))
        return out

    def open_host_batch(self, nonces: np.ndarray, ct_tag: np.ndarray):
        """-> (plaintexts, status): status[i] 1 ok / 0 forged (that record zero-filled)."""
        nrec, m = ct_tag.shape
        n = m - TAG_LEN
        out = np.empty((nrec, n), np.uint8)
        status = np.zeros(nrec, np.int32)
        ct_tag = np.ascontiguousarray(ct_tag)
        nonces = np.ascontiguousarray(nonces)
        fn = N.lib().cmpi_gcm_open_host if self._gcm else N.lib().cmpi_ocb_open_host
        rc = fn(self._h, out.ctypes.data, max(out.strides[0], 1), ct_tag.ctypes.data, ct_tag.strides[0],
                nonces.ctypes.data, 12, n, nrec, status.ctypes.data)
        if rc not in (N.CMPI_OK, N.CMPI_EAUTH):
            N.check(rc)
        return out, status

    # ------------------------------------------------------------ asynchronous host batches
    def seal_host_begin(self, nonces: np.ndarray, pt: np.ndarray, out: np.ndarray) -> "Request":
        """MPI_Isend-style: enqueue the seal of (N, n) host plaintexts into out (N, n+16) and
        return a Request (include/cmpi_async.h); out must stay alive until it completes."""
        nrec, n = pt.shape
        pt, nonces = np.ascontiguousarray(pt), np.ascontiguousarray(nonces)
        fn = N.lib().cmpi_gcm_seal_host_begin if self._gcm else N.lib().cmpi_ocb_seal_host_begin
        r = ctypes.c_void_p()
        N.check(fn(self._h, out.ctypes.data, out.strides[0], pt.ctypes.data, max(pt.strides[0], 1),
                   nonces.ctypes.data, 12, n, nrec, ctypes.byref(r)))
        return Request(r, keep=(out,))

    def open_host_begin(self, nonces: np.ndarray, ct_tag: np.ndarray, out: np.ndarray, status: np.ndarray) -> "Request":
        nrec, m = ct_tag.shape
        ct_tag, nonces = np.ascontiguousarray(ct_tag), np.ascontiguousarray(nonces)
        fn = N.lib().cmpi_gcm_open_host_begin if self._gcm else N.lib().cmpi_ocb_open_host_begin
        r = ctypes.c_void_p()
        N.check(fn(self._h, out.ctypes.data, max(out.strides[0], 1), ct_tag.ctypes.data, ct_tag.strides[0],
                   nonces.ctypes.data, 12, m - TAG_LEN, nrec, status.ctypes.data, ctypes.byref(r)))
        return Request(r, keep=(out, status))

    def seal(self, nonce: bytes, pt: bytes) -> bytes:
        """EVP_AEAD_CTX_seal for one message (host memory)."""
        if len(nonce) != NONCE_LEN:
            raise ValueError("nonce must be 12 bytes")
        return self.seal_host_batch(np.frombuffer(nonce, np.uint8)[None, :],
                                    np.frombuffer(pt, np.uint8)[None, :] if pt else np.zeros((1, 0), np.uint8))[0].tobytes()

    def open(self, nonce: bytes, ct_tag: bytes):
        """EVP_AEAD_CTX_open for one message: plaintext, or None when authentication fails."""
        if len(nonce) != NONCE_LEN or len(ct_tag) < TAG_LEN:
            return None
        out, st = self.open_host_batch(np.frombuffer(nonce, np.uint8)[None, :], np.frombuffer(ct_tag, np.uint8)[None, :])
        return out[0].tobytes() if st[0] == 1 else None


class Request:
    """An outstanding asynchronous host batch (cmpi_req): test() ~ MPI_Test, wait() ~ MPI_Wait.
    wait() returns CMPI_OK or CMPI_EAUTH (open: some record failed) and raises on errors."""

    def __init__(self, handle, keep=()):
        self._r = handle
        self._keep = keep

    def test(self) -> bool:
        if self._r is None:
            return True
        done = ctypes.c_int(0)
        rc = N.lib().cmpi_test(self._r, ctypes.byref(done))
        if done.value:
            self._r = None
            self._keep = ()
            if rc not in (N.CMPI_OK, N.CMPI_EAUTH):
                N.check(rc)
        return bool(done.value)

    def wait(self) -> int:
        if self._r is None:
            return N.CMPI_OK
        rc = N.lib().cmpi_wait(self._r)
        self._r = None
        self._keep = ()
        if rc not in (N.CMPI_OK, N.CMPI_EAUTH):
            N.check(rc)
        return rc


class CipherCtx(_Ctx):
    """AES-128-CTR / AES-128-ECB context (EVP_CIPHER_CTX with EVP_aes_128_ctr/ecb)."""

    def __init__(self, key: bytes, alg: str = "aes-128-ctr", device: int = 0):
        if alg not in ("aes-128-ctr", "aes-128-ecb"):
            raise ValueError(alg)
        super().__init__(key, alg, device)

    def ctr_xor(self, out, inp, nbytes: int, ctr_block: bytes, stream=None) -> None:
        cb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(ctr_block))
        N.check(N.lib().cmpi_ctr_xor(self._h, _dptr(out), _dptr(inp), nbytes, cb, _stream_ptr(stream)))

    def keystream(self, out, nblocks: int, ctr_block: bytes, stream=None) -> None:
        cb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(ctr_block))
        N.check(N.lib().cmpi_ctr_keystream(self._h, _dptr(out), nblocks, cb, _stream_ptr(stream)))

    def ecb_encrypt(self, out, inp, nblocks: int, stream=None) -> None:
        N.check(N.lib().cmpi_ecb_encrypt(self._h, _dptr(out), _dptr(inp), nblocks, _stream_ptr(stream)))


def iv_count(iv: bytes, cter: int) -> bytes:
    """IV_Count (send.c:1019-1030) through the engine's host helper."""
    b = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(iv))
    N.lib().cmpi_iv_count(b, cter & 0xFFFFFFFFFFFFFFFF)
    return bytes(b)


def force_plan(lanes_per_record: int = 0, segments: int = 0) -> None:
    """Test hook: force the GCM work decomposition (0 = automatic)."""
    N.lib().cmpi_debug_force_plan(lanes_per_record, segments)


def force_wide(mode: int = 0, steps: int = 0) -> None:
    """Test hook: wide GCM decomposition 0 automatic / 1 always (when legal) / -1 never;
    steps per chunk (0 = automatic)."""
    N.lib().cmpi_debug_force_wide(mode, steps)


def set_flow_threads(threads: int = 0) -> None:
    """Test hook (cmpi_debug_set_flow_threads): FLOW kernel workgroup size, 0 = automatic (512 for
    batches of at most 8 waves per CU, else 1024), 512 or 1024 forced."""
    N.lib().cmpi_debug_set_flow_threads(threads)


def set_flow_one_wg(on: bool = True) -> None:
    """Test hook (cmpi_debug_set_flow_one_wg): a FLOW batch whose chunks fit one workgroup
    finishes its tags in-kernel (True, default) or through the XOR-combine launch (False)."""
    N.lib().cmpi_debug_set_flow_one_wg(1 if on else 0)


def gcm_plan(ctx: AeadCtx, length: int, nrec: int):
    out = (ctypes.c_uint32 * 4)()
    N.check(N.lib().cmpi_debug_gcm_plan(ctx.handle, length, nrec, out))
    return tuple(out)
