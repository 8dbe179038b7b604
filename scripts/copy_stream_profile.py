"""Copy-stream load of the GPU engine on HOST-resident tiles (round 6, VERDICT
item 7): DPOTRF (the ptgpp-compiled dpotrf_L.jdf) with every tile staged in
through the GPU's one shared copy stream -- stage-in (H2D), write-back /
W2R (D2H), prefetch and, with device_hip_replicas 2, device-to-device stage-in
all queue on it (csrc/device/hip_device.cpp gpu_copy_stream). Prints the span,
the engine's transfer counters and the summed time tasks waited for their
stage-in copies; run under `rocprofv3 --memory-copy-trace --kernel-trace
--stats` for the copy engine's busy time (occupancy = copy time / span).

usage: python scripts/copy_stream_profile.py N nb cache_fraction [replicas]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N, nb, frac = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    import torch

    torch.cuda.set_device(0)
    import parsec_amd as pa

    pa.require_native()
    pa.mca_set("device_hip_memory_max", str(int(frac * N * N * 8)))
    # the engine times every copy it issues on the copy stream when profiling is
    # on (GPU_MOVEIN / MOVEOUT / PREFETCH spans): busy time and window below
    trace = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"copyprof{os.getpid()}")
    pa.mca_set("profile_filename", trace)
    if reps > 1:
        pa.mca_set("device_hip_replicas", str(reps))
    ctx = pa.init(4)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)  # host storage
    rng = np.random.default_rng(4)
    S = rng.random((N, N)) - 0.5
    S = (S + S.T) * 0.5 + N * np.eye(N)
    NT = N // nb
    for m in range(NT):
        for n in range(NT):
            A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
    tp, info = pa.dpotrf_jdf_new(A)
    ctx.add_taskpool(tp)
    t0 = time.perf_counter()
    ctx.start()
    ctx.wait()
    dt = time.perf_counter() - t0
    gpus = [d for d in pa.devices() if d["type"] == pa.DEV_HIP]
    L = np.zeros((N, N))
    for m in range(NT):
        for n in range(m + 1):
            L[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = A.tile(m, n)
    ctx.fini()
    X = rng.random((N, 4)) - 0.5
    res = np.linalg.norm(S @ X - np.tril(L) @ (np.tril(L).T @ X)) / (np.linalg.norm(S) * np.linalg.norm(X))
    tot = {k: sum(g[k] for g in gpus) for k in ("executed_tasks", "bytes_in", "bytes_out", "bytes_d2d", "data_faults", "w2r_tasks", "staged_tasks", "ms_stage_wait",
                                                 "copies_timed", "ms_copy_busy")}
    window = max(g["ms_copy_window"] for g in gpus)
    print(f"copy-stream N={N} nb={nb} cache={frac:.2f} devices={len(gpus)} info={pa.read_int(info)} residual={res:.2e} span_ms={dt * 1e3:.1f} "
          f"GF={N ** 3 / 3 / dt / 1e9:.0f} tasks={tot['executed_tasks']} in_MiB={tot['bytes_in'] >> 20} out_MiB={tot['bytes_out'] >> 20} "
          f"d2d_MiB={tot['bytes_d2d'] >> 20} faults={tot['data_faults']} w2r={tot['w2r_tasks']} staged_tasks={tot['staged_tasks']} "
          f"stage_wait_ms_sum={tot['ms_stage_wait']:.1f} stage_wait_ms_per_task={tot['ms_stage_wait'] / max(1, tot['staged_tasks']):.3f} "
          f"copies_timed={tot['copies_timed']} copy_busy_ms={tot['ms_copy_busy']:.1f} copy_window_ms={window:.1f} "
          f"copy_occupancy={tot['ms_copy_busy'] / max(window, 1e-9) / max(1, len(gpus)):.2f} copy_GBps={(tot['bytes_in'] + tot['bytes_out'] + tot['bytes_d2d']) / max(tot['ms_copy_busy'], 1e-9) / 1e6:.1f}", flush=True)
    for f in os.listdir(os.path.dirname(trace)):
        if f.startswith(os.path.basename(trace)):
            os.unlink(os.path.join(os.path.dirname(trace), f))
    sys.exit(0 if pa.read_int(info) == 0 and res < 1e-12 else 1)


if __name__ == "__main__":
    main()
