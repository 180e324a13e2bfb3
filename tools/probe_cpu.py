import ctypes, os, time, numpy as np, sys
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"):
    try: print(f, open(f).read().strip())
    except Exception as e: print(f, e)
print("OMP_NUM_THREADS", os.environ.get("OMP_NUM_THREADS"))
L = ctypes.CDLL("tools/libcpu_baseline.so")
P,S,I=ctypes.c_void_p,ctypes.c_size_t,ctypes.c_int
L.cb_aead_batch.argtypes=[I,I,P,P,P,S,P,S,I,ctypes.c_long,I]
n=1024; N=65536
pt=np.random.randint(0,256,(N,n),dtype=np.uint8); nn=np.random.randint(0,256,(N,12),dtype=np.uint8); ct=np.empty((N,n+16),np.uint8)
key=bytes(range(16))
for T in (1,2,4,8,16,32):
    ts=[]
    for r in range(5):
        t0=time.perf_counter(); L.cb_aead_batch(1,0,key,nn.ctypes.data,pt.ctypes.data,n,ct.ctypes.data,n+16,n,N if T>1 else 8192,T); ts.append(time.perf_counter()-t0)
    recs = N if T>1 else 8192
    print("threads",T,"seal GiB/s", round(recs*n/np.median(ts)/2**30,3), flush=True)
