import sys, numpy as np
sys.path.insert(0, "/root/repo")
import parsec_amd as pa
M = N = 512; nb = 256
ctx = pa.init(3)
A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, M, N)
T = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, M, N)
S = np.random.default_rng(0).standard_normal((M, N))
for m in range(A.mt):
    for n in range(A.nt):
        A.tile(m, n)[:, :] = S[m*nb:(m+1)*nb, n*nb:(n+1)*nb]
tp = pa.dgeqrf_new(A, T, 32)
ctx.add_taskpool(tp); ctx.start(); ctx.wait()
R = np.zeros((M, N))
for m in range(A.mt):
    for n in range(A.nt):
        R[m*nb:(m+1)*nb, n*nb:(n+1)*nb] = A.tile(m, n)
R = np.triu(R)
print("qr small err", np.linalg.norm(R.T @ R - S.T @ S) / np.linalg.norm(S.T @ S), flush=True)
ctx.fini()
