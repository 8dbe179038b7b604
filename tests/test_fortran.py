"""Fortran 2008 bindings (csrc/fortran/parsecf.F90, parsec_profilef.F90; reference
parsec/fortran/parsecf.F90, parsec_profilef.F90) compiled with ROCm's flang: a
Fortran program builds a DTD task graph with Fortran task bodies, uses the
taskpool callbacks and writes a profiling trace that the offline reader opens."""
import os
import subprocess

import pytest

from parsec_amd import _build

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "parsec_amd", "lib")
MODS = os.path.join(ROOT, "parsec_amd", "include", "fortran")

pytestmark = pytest.mark.skipif(not os.path.exists(_build.FLANG), reason="flang not available")


def test_fortran_dtd_program(tmp_path, pa):
    if not os.path.exists(os.path.join(LIB, "libparsec_amd_f08.a")):
        _build.build()
    exe = tmp_path / "dtd_fortran"
    cmd = [_build.FLANG, f"-I{MODS}", "-module-dir", str(tmp_path), os.path.join(HERE, "fortran", "dtd_fortran.F90"), "-o", str(exe),
           f"-L{LIB}", "-lparsec_amd_f08", "-lparsec_amd", f"-Wl,-rpath,{LIB}", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, cwd=tmp_path,
                       env=dict(os.environ, PARSEC_MCA_device_hip_enabled="0"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fortran dtd sum 85344 expect 85344 completed 1 enqueued 1" in r.stdout
    assert "fortran ok" in r.stdout
    trace = tmp_path / "fortran_trace-0.prof"  # <base>-<rank>.prof (reference parsec_profiling_dbp_start)
    assert trace.exists()
    from parsec_amd import profiling

    t = profiling.read_trace(str(trace))
    names = {d["name"] for d in t.dictionary}
    # the user events recorded by the Fortran program are in the trace
    assert sum(len(s["events"]) for s in t.streams) >= 128
    assert "fortran_event" in names
