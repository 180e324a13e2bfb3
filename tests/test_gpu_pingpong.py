"""CryptMPI's per-message 600 exchange between two processes in C through the BoringSSL-ABI drop-in
(tools/evp_pingpong.c: send.c:221-337 / recv.c:219-341 framing over a shared-memory transport,
static large_send/recv_buffer, malloc'd user buffers), with the shim's defaults — each context's
resident message service, static message buffers page-locked on first use — and with a kernel
launch per call.  Every message is checked by the receiving process; the last wire record rank 1
received (nonce || ct || tag, as CryptMPI's large_recv_buffer holds it) is checked against the
oracle under the key the program uses."""
import json
import os
import subprocess

import pytest

import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "evp_pingpong")
KEY = bytes(0x30 + i for i in range(16))  # evp_pingpong.c run_side


@pytest.fixture(scope="module", autouse=True)
def _built():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools"), "evp_pingpong"])


@pytest.mark.parametrize("n", [1, 1000, 4096, 65536, 300001])
@pytest.mark.parametrize("service_us", ["2000", "0"])
def test_c_pingpong_600(tmp_path, n, service_us):
    dump = tmp_path / "wire.bin"
    env = dict(os.environ, CMPI_EVP_SERVICE_US=service_us, CMPI_EVP_DEBUG="1", PINGPONG_DUMP=str(dump))
    r = subprocess.run([EXE, "secure", str(n), "50", "0.05"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["verified"] and line["provider"] == "libcmpi_evp.so"
    if n >= 4096:  # messages of >= 4 KiB page-lock the static buffers they touch (the program's .bss)
        assert "page-locked: yes" in r.stderr, r.stderr[-2000:]
    b = dump.read_bytes()
    assert len(b) == (n + 28) + n
    wire, pt = b[: n + 28], b[n + 28:]
    assert wire[12:] == oracle.gcm_seal(KEY, wire[:12], pt)
