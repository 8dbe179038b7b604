import torch, ctypes, numpy as np, time, os
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe.so"))
print("device", torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
A = np.arange(64, dtype=np.float64).reshape(16, 4) + 1.0
B = (np.arange(64, dtype=np.float64).reshape(4, 16) * 3.0 + 7.0) % 11.0 + 1
C = np.zeros(256)
rc = lib.probe_layout(A.ctypes.data_as(ctypes.c_void_p), B.ctypes.data_as(ctypes.c_void_p), C.ctypes.data_as(ctypes.c_void_p))
ref = A @ B
C = C.reshape(64, 4)
ok1 = all(abs(C[l, r] - ref[(l >> 4) + 4 * r, l & 15]) < 1e-9 for l in range(64) for r in range(4))
ok2 = all(abs(C[l, r] - ref[(l >> 4) * 4 + r, l & 15]) < 1e-9 for l in range(64) for r in range(4))
print("layout rc", rc, "row=(l>>4)+4r:", ok1, " row=(l>>4)*4+r:", ok2)
lib.probe_rate.restype = ctypes.c_double
lib.probe_vfma.restype = ctypes.c_double
cyc = ctypes.c_longlong(0)
for nacc in (1, 2, 4, 8):
    for blocks, threads in ((256, 256), (1024, 256), (256, 512)):
        tf = lib.probe_rate(nacc, blocks, threads, 20000, ctypes.byref(cyc))
        print(f"mfma_f64 nacc={nacc} blocks={blocks} thr={threads}: {tf:.1f} TF  cycles/iter/wave={cyc.value/20000/nacc:.1f} per-mfma")
print("vfma f64:", lib.probe_vfma(2048, 256, 20000), "TF")
# torch reference dgemm (rocBLAS/hipBLASLt)
for n in (512, 1024, 4096, 8192):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda"); b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    for _ in range(3): c = a @ b
    torch.cuda.synchronize(); t = time.perf_counter(); it = max(3, int(2e10 / n**3))
    for _ in range(it): c = a @ b
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / it
    print(f"torch dgemm n={n}: {2*n**3/dt/1e12:.1f} TF ({dt*1e6:.0f} us)")
# torch cholesky reference
for n in (16384,):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda"); a = a @ a.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
    torch.linalg.cholesky(a); torch.cuda.synchronize()
    t = time.perf_counter(); L = torch.linalg.cholesky(a); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"torch cholesky (rocSOLVER) n={n}: {n**3/3/dt/1e9:.0f} GFLOP/s ({dt*1e3:.1f} ms)")
