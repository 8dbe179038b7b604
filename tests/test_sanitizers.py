"""Host-side sanitizer builds of the runtime (reference CMake PARSEC_DEBUG_MEM_ADDR,
PARSEC_DEBUG_MEM_LEAK, PARSEC_DEBUG_MEM_RACE, CMakeLists.txt:195-200,320-360):
`python -m parsec_amd._build --sanitize KIND` rebuilds the host code with
-fsanitize=KIND into build-KIND/, and these tests run the lock-free container
test and the C99 DTD program (1..4 processes over the shared-memory engine)
under ThreadSanitizer and AddressSanitizer + LeakSanitizer, plus (round 5)
the distributed PTG Cholesky with CPU bodies on 1 / 2 / 4 ranks, the
reference's dtd_test_multiple_handle_wait.c and its reshape family. Races these runs
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

from parsec_amd import _build, launch, ptgpp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

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


@pytest.mark.parametrize("nranks", [1, 2, 4])
def test_dpotrf_program_sanitized(sanitized, nranks):
    """The distributed PTG Cholesky (ptgpp-compiled dpotrf_L.jdf through
    parsec_dpotrf_New, CPU bodies) on 1 / 2 / 4 ranks: the PTG engine, the
    remote-dependency send / receive / deliver path and the priority fetch
    queue, instrumented."""
    kind, out = sanitized
    old = dict(os.environ)
    os.environ.update(_env(kind))
    os.environ["PARSEC_MCA_device_hip_enabled"] = "0"
    try:
        rc, outs = launch.launch(nranks, [os.path.join(out, "dpotrf_capi"), "512", "64"], timeout=600, capture=True)
    finally:
        os.environ.clear()
        os.environ.update(old)
    errs = "\n".join(e for _, e in outs)
    first = errs.find("WARNING: ")
    assert rc == 0, errs[first:first + 6000] if first >= 0 else errs[-4000:]
    assert "Sanitizer" not in errs
    assert sum(" ok" in o for o, _ in outs) == nranks, [o for o, _ in outs]


def _run_sanitized(kind, exe, args=(), timeout=300, leaks=True):
    env = _env(kind)
    env["PARSEC_MCA_device_hip_enabled"] = "0"
    if not leaks:
        env["ASAN_OPTIONS"] = "detect_leaks=0 exitcode=67"
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout, env=env)
    first = r.stderr.find("WARNING: ")
    assert r.returncode == 0, r.stdout[-2000:] + (r.stderr[first:first + 6000] if first >= 0 else r.stderr[-4000:])
    assert "Sanitizer" not in r.stderr
    return r


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
@pytest.mark.parametrize("prog,runs,args", [("multiple_handle_wait", 3, []), ("tp_enqueue_dequeue", 2, ["4"]), ("new_tile", 2, [])])
def test_reference_dtd_programs_sanitized(sanitized, tmp_path, prog, runs, args):
    """Reference DTD programs (tests/dsl/dtd/dtd_test_<prog>.c, unmodified):
    multiple_handle_wait found round 4's two use-after-frees under a manual ASan
    run; tp_enqueue_dequeue frees taskpools from bodies (deferred deletion) and
    completes an ASYNC task from another taskpool's completion callback;
    new_tile sizes tiles at their first insertion and flushes them home."""
    kind, _ = sanitized
    cc, libs = ptgpp.compile_flags(False, kind)
    exe = str(tmp_path / prog)
    r = subprocess.run(cc + list(ptgpp.C_BODIES) + [f"-I{REF}/tests", f"-I{REF}", f"-I{REF}/tests/dsl/dtd", "-x", "c++",
                                                    os.path.join(REF, f"tests/dsl/dtd/dtd_test_{prog}.c"),
                                                    os.path.join(REF, "tests/tests_data.c"), "-o", exe] + libs, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    for _ in range(runs):
        _run_sanitized(kind, exe, args)


_RS = "tests/collections/reshape/"
RESHAPE = [
    ("avoidable_reshape.jdf", ["testing_avoidable_reshape.c", "common.c"], 1),
    ("input_dep_single_copy_reshape.jdf", ["testing_input_dep_reshape_single_copy.c", "common.c"], 1),
    ("remote_multiple_outs_same_pred_flow.jdf", ["remote_multiple_outs_same_pred_flow_multiple_deps.jdf", "testing_remote_multiple_outs_same_pred_flow.c", "common.c"], 2),
    ("local_no_reshape.jdf", [j + ".jdf" for j in ("local_read_reshape", "local_output_reshape", "local_input_reshape", "local_input_LU_LL",
                                                   "remote_read_reshape", "remote_no_re_reshape")] + ["testing_reshape.c", "common.c"], 7),
]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
@pytest.mark.parametrize("jdf,srcs,npass", RESHAPE, ids=[r[0] for r in RESHAPE])
def test_reference_reshape_sanitized(sanitized, tmp_path, jdf, srcs, npass):
    """The reference's reshape family (JDFs + drivers unmodified, as in
    tests/test_ptgpp.py) against the instrumented runtime: reshape futures,
    shared reshaped copies, typed write-backs."""
    kind, _ = sanitized
    if kind == "thread" and jdf == "input_dep_single_copy_reshape.jdf":
        # its BODY spins on a plain global (`do {} while (set == 0)`,
        # input_dep_single_copy_reshape.jdf:64-73): a race in the program itself
        pytest.skip("the reference program's body races on its own global by design")
    if kind == "thread" and jdf == "local_no_reshape.jdf":
        # this driver also runs remote_no_re_reshape.jdf, whose TASK_A(m, k)
        # writes descA(m, k) from READ_A(k, m)'s data while READ_A(m, k) may
        # still read descA(m, k): the DAG orders neither (lines 30-48), a race in
        # the test program that ThreadSanitizer reports in the runtime's copy
        # code (an early-termination probe over 30 runs found the runtime's
        # taskpool boundaries intact); AddressSanitizer runs it
        pytest.skip("remote_no_re_reshape.jdf leaves a read and a write of one tile unordered")
    d = os.path.join(REF, _RS)
    extra = [ptgpp.compile_jdf(os.path.join(d, x), str(tmp_path), None)[0] if x.endswith(".jdf") else os.path.join(d, x) for x in srcs]
    exe = ptgpp.build_program(os.path.join(d, jdf), str(tmp_path), extra_sources=extra, sanitize=kind,
                              cxxflags=ptgpp.C_BODIES + (f"-I{d}", f"-I{REF}/tests", f"-I{REF}"))
    r = _run_sanitized(kind, exe)
    out = r.stdout + r.stderr
    assert out.count(" PASSED") == npass and "FAILED" not in out, out[-2000:]


def test_hash_table_sanitized(sanitized, tmp_path):
    """The public hash table under 8 racing threads (tests/capi/hash_table_capi.c):
    bucket handles held across find-then-insert, growth while other threads
    hold no bucket, for_all with removal."""
    kind, _ = sanitized
    cc, libs = ptgpp.compile_flags(False, kind)
    exe = str(tmp_path / "ht")
    cmd = ["gcc", "-std=c99", "-O1", "-g", "-pthread", f"-fsanitize={kind}", f"-I{ROOT}/include", os.path.join(ROOT, "tests/capi/hash_table_capi.c"), "-o", exe] + libs
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _run_sanitized(kind, exe)
    assert "hash table ok" in r.stdout


@pytest.mark.skipif(not os.path.isdir(REF + "/tests/class"), reason="reference tree not present")
@pytest.mark.parametrize("prog,args", [("hash", ["-#", "16384", "-r", "2", "-n", "-c", "4"]), ("lifo", ["-c", "4"]), ("list", ["-c", "4"]),
                                       ("future", ["-c", "4"]), ("future_datacopy", [])])
def test_reference_class_programs_sanitized(sanitized, tmp_path, prog, args):
    """The reference's tests/class hash / lifo / list (unmodified) against the
    instrumented library: bucket locking and growth, the tagged-head LIFO, the
    locked list, from 4 threads."""
    kind, _ = sanitized
    cc, libs = ptgpp.compile_flags(False, kind)
    exe = str(tmp_path / prog)
    r = subprocess.run(cc + ["-x", "c++", "-fpermissive", "-w", f"-I{REF}", os.path.join(REF, "tests/class", prog + ".c"), "-o", exe] + libs,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # the programs keep some of their own buffers to the end (lifo.c:259): leak
    # checking would report the test, not the containers
    r = _run_sanitized(kind, exe, args, timeout=600, leaks=False)
    assert "Error in implementation" not in r.stdout + r.stderr


HAAR = os.path.join(REF, "tests/apps/haar_tree")
SUM_VALUE = 0xbdae8a4ea45fc32e  # reference tests/apps/haar_tree/main.c:23


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
@pytest.mark.parametrize("dyn", [False, True], ids=["project", "project_dyn"])
def test_reference_haar_tree_sanitized(sanitized, tmp_path, dyn):
    """The reference's haar-tree application (project(_dyn).jdf + walk.jdf over
    tree_dist.c, unmodified) under TSan / ASan: generated per-class task views,
    a user startup_fn building the root task by hand, make_key / hash_struct /
    find_deps / alloc_deps hooks on a 2^32-wide space, the concurrent hash table
    and a body ending the taskpool (set_nb_tasks from a body)."""
    kind, _ = sanitized
    proj = "project_dyn" if dyn else "project"
    srcs = [ptgpp.compile_jdf(os.path.join(HAAR, j + ".jdf"), str(tmp_path))[0] for j in (proj, "walk")]
    cc, libs = ptgpp.compile_flags(False, kind)
    exe = str(tmp_path / proj)
    drv = os.path.join(ROOT, "tests", "capi", "haar_tree_driver.cpp")
    r = subprocess.run(cc + list(ptgpp.C_BODIES) + (["-DHAAR_DYN"] if dyn else []) +
                       [f"-I{HAAR}", f"-I{tmp_path}", f"-I{REF}", "-x", "c++", drv, os.path.join(HAAR, "tree_dist.c"), "-x", "none"] + srcs +
                       ["-o", exe] + libs + ["-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _run_sanitized(kind, exe, ["--"], leaks=False)
    line = [l.split() for l in r.stdout.splitlines() if l.startswith("haar rank")]
    assert len(line) == 1, r.stdout[-2000:]
    if not dyn:
        assert int(line[0][line[0].index("cksum") + 1], 16) == SUM_VALUE, r.stdout[-2000:]
