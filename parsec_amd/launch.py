"""Multi-process launcher for native parsec-amd programs (the role mpiexec
plays for the reference's `:mp` tests, tests/CMakeLists.txt:26-59).

    python -m parsec_amd.launch -n 4 ./program args...

Starts N copies with PARSEC_COMM_RANK / PARSEC_COMM_SIZE / PARSEC_COMM_JOB set
(parsec_init joins the shared-memory communication engine from them) and
returns the first non-zero exit code; when a rank fails the others are killed
(mpiexec semantics), and --timeout bounds the whole job. PARSEC_COMM_GPU=<ordinal> per rank is
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
    import threading

    results = [None] * len(procs)

    def _drain(i, p):
        results[i] = p.communicate()

    th = [threading.Thread(target=_drain, args=(i, p), daemon=True) for i, p in enumerate(procs)]
    for t in th:
        t.start()
    # like mpiexec: the first rank that fails (or the time limit) ends the job,
    # so survivors blocked on that rank in a collective cannot hang forever
    t0 = time.monotonic()
    failed = timed_out = False
    while any(p.poll() is None for p in procs):
        if any(p.returncode not in (None, 0) for p in procs):
            failed = True
            break
        if timeout is not None and time.monotonic() - t0 > timeout:
            timed_out = True
            break
        time.sleep(0.05)
    if failed or timed_out:
        for q in procs:
            if q.poll() is None:
                q.kill()
    for t in th:
        t.join(timeout=30)
    if timed_out:
        raise subprocess.TimeoutExpired(cmd, timeout)
    outs = [r if r is not None else (None, None) for r in results]
    rc = 0
    for p in procs:  # first failing rank in rank order; killed survivors report -9
        if p.returncode and p.returncode != -9 and not rc:
            rc = p.returncode
    if not rc:
        rc = next((p.returncode for p in procs if p.returncode), 0)
    return (rc, outs) if capture else rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nprocs", type=int, default=2)
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=3600.0, help="seconds before every rank is killed (0 = none)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    sys.exit(launch(a.nprocs, a.cmd, a.gpus, a.timeout or None))


if __name__ == "__main__":
    main()
