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
    deadline = time.time() + timeout if timeout else None
    outs = []
    rc = 0
    for p in procs:
        left = max(1.0, deadline - time.time()) if deadline else None
        try:
            o, er = p.communicate(timeout=left)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((o, er))
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
