"""Multi-process launcher for native parsec-amd programs (the role mpiexec
plays for the reference's `:mp` tests, tests/CMakeLists.txt:26-59).

    python -m parsec_amd.launch -n 4 ./program args...

Starts N copies with PARSEC_COMM_RANK / PARSEC_COMM_SIZE / PARSEC_COMM_JOB set
(parsec_init joins the shared-memory communication engine from them) and
returns the first non-zero exit code. PARSEC_COMM_GPU=<ordinal> per rank is
set when --gpus is given (rank r -> GPU r % gpus).
"""
import argparse
import os
import subprocess
import sys
import time


def launch(nprocs, cmd, gpus=0, timeout=None, env=None, capture=False):
    job = f"launch{os.getpid()}_{int(time.time() * 1000) % 100000000}"
    procs = []
    for r in range(nprocs):
        e = dict(os.environ)
        if env:
            e.update(env)
        e.update({"PARSEC_COMM_RANK": str(r), "PARSEC_COMM_SIZE": str(nprocs), "PARSEC_COMM_JOB": job})
        if gpus:
            e["PARSEC_COMM_GPU"] = str(r % gpus)
        kw = dict(stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) if capture else {}
        procs.append(subprocess.Popen(cmd, env=e, **kw))
    # drain every rank's pipes concurrently: a rank blocked on a full pipe
    # would otherwise stall the ranks waiting for it (collective deadlock)
    results = [None] * len(procs)

    def _wait(i, p):
        try:
            results[i] = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            results[i] = "timeout"

    import threading

    th = [threading.Thread(target=_wait, args=(i, p), daemon=True) for i, p in enumerate(procs)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if any(r == "timeout" for r in results):
        for q in procs:
            if q.poll() is None:
                q.kill()
        for q in procs:
            try:
                q.communicate(timeout=10)
            except Exception:
                pass
        raise subprocess.TimeoutExpired(cmd, timeout)
    outs = [r if r is not None else (None, None) for r in results]
    rc = 0
    for p in procs:
        if p.returncode and not rc:
            rc = p.returncode
    return (rc, outs) if capture else rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nprocs", type=int, default=2)
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    sys.exit(launch(a.nprocs, a.cmd, a.gpus, a.timeout))


if __name__ == "__main__":
    main()
