"""Host-side sanitizer builds of the runtime (reference CMake PARSEC_DEBUG_MEM_ADDR,
PARSEC_DEBUG_MEM_LEAK, PARSEC_DEBUG_MEM_RACE, CMakeLists.txt:195-200,320-360):
`python -m parsec_amd._build --sanitize KIND` rebuilds the host code with
-fsanitize=KIND into build-KIND/, and these tests run the lock-free container
test and the C99 DTD program (1..4 processes over the shared-memory engine)
under ThreadSanitizer and AddressSanitizer + LeakSanitizer. Races these runs
found and that are fixed: unlocked emptiness checks of the dequeue / sorted
queue / max-heap / VP queues (now atomic counts), termination detection set
up after the taskpool was published to the comm thread, remote DTD shadows
published before their tile edges were complete; leaks: termdet callbacks,
comm / manager execution streams, DTD remote shadows' insertion reference, and
(round 4, 3+ ranks) an edge between two shadows of OTHER ranks that was never
released."""
import os
import subprocess

import pytest

from parsec_amd import _build, launch

pytestmark = pytest.mark.skipif(subprocess.run(["which", "ninja"], capture_output=True).returncode != 0, reason="ninja missing")


@pytest.fixture(scope="module", params=["thread", "address"])
def sanitized(request, pa):
    return request.param, _build.build_sanitized(request.param)


def _env(kind):
    e = dict(os.environ)
    e["TSAN_OPTIONS"] = "halt_on_error=1 exitcode=66"
    e["ASAN_OPTIONS"] = "detect_leaks=1 exitcode=67"
    return e


def test_containers_sanitized(sanitized):
    kind, out = sanitized
    r = subprocess.run([os.path.join(out, "test_containers")], capture_output=True, text=True, timeout=600, env=_env(kind))
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "Sanitizer" not in r.stderr
    assert "all container tests passed" in r.stdout


@pytest.mark.parametrize("nranks", [1, 2, 4])
def test_dtd_program_sanitized(sanitized, nranks):
    kind, out = sanitized
    old = dict(os.environ)
    os.environ.update(_env(kind))
    try:
        rc, outs = launch.launch(nranks, [os.path.join(out, "dtd_capi")], timeout=300, capture=True)
    finally:
        os.environ.clear()
        os.environ.update(old)
    errs = "\n".join(e for _, e in outs)
    first = errs.find("WARNING: ")  # the report's own head: the two racing accesses
    assert rc == 0, errs[first:first + 6000] if first >= 0 else errs[-4000:]
    assert "Sanitizer" not in errs
    assert sum("ok" in o for o, _ in outs) == nranks
