"""C API (include/parsec.h) tests: a C99 DTD program and a compiled JDF,
single process and multi-process through parsec_amd.launch (the `:mp`
variants of the reference's tests, tests/dsl/dtd/Testings.cmake:15-28)."""
import os
import subprocess

import pytest

from parsec_amd import launch, ptgpp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def dtd_capi(tmp_path_factory, pa):
    out = tmp_path_factory.mktemp("capi") / "dtd_capi"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "dtd_capi.c"), "-o", str(out),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return str(out)


def test_checkpoint_user_storage_after_init(tmp_path, pa):
    """data_write / data_read with dc.mat assigned after init (lazy pickup)."""
    exe = tmp_path / "ckpt"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "checkpoint_capi.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe), str(tmp_path / "A.ckpt")], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PARSEC_MCA_device_hip_enabled="0"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


def test_datatypes_c_program(tmp_path, pa):
    """Derived datatypes: vector / hvector / indexed / struct / resized / lower (reference datatype.h)."""
    exe = tmp_path / "dtt"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "datatype_capi.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "datatype ok" in r.stdout


def test_dtd_c_program(dtd_capi):
    r = subprocess.run([dtd_capi], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


@pytest.mark.parametrize("nranks", [2, 3])
def test_dtd_c_program_multiprocess(dtd_capi, nranks):
    rc, outs = launch.launch(nranks, [dtd_capi], timeout=120, capture=True)
    assert rc == 0, outs
    assert sum("ok" in o for o, _ in outs) == nranks


@pytest.fixture(scope="module")
def bcast_gather(tmp_path_factory, pa):
    return ptgpp.build_program(os.path.join(HERE, "jdf", "bcast_gather.jdf"), str(tmp_path_factory.mktemp("jdfmp")))


@pytest.mark.parametrize("nranks", [2, 4])
def test_jdf_multiprocess(bcast_gather, nranks):
    """PTG broadcast of a NEW buffer to remote LEAF tasks and a remote CTL gather."""
    rc, outs = launch.launch(nranks, [bcast_gather], timeout=120, capture=True)
    assert rc == 0, outs
    sinks = sum(int(o.split("sink")[1].split()[0]) for o, _ in outs)
    leaves = sum(int(o.split("leaves")[1].split()[0]) for o, _ in outs)
    assert sinks == 1 and leaves == 37


@pytest.fixture(scope="module")
def apps(tmp_path_factory, pa):
    out = str(tmp_path_factory.mktemp("jdfapps"))
    return {n: ptgpp.build_program(os.path.join(HERE, "jdf", n + ".jdf"), out) for n in ("tree_reduce", "pingpong", "all2all")}


@pytest.mark.parametrize("nranks", [2, 3])
def test_tree_reduce_multiprocess(apps, nranks):
    """Binary reduction tree of NEW buffers whose interior edges cross ranks
    (reference tests/apps/haar_tree, generalized_reduction)."""
    rc, outs = launch.launch(nranks, [apps["tree_reduce"], "6"], timeout=120, capture=True)
    assert rc == 0, outs
    assert "root 2080" in outs[0][0]
    assert sum(int(o.split("nodes")[1].split()[0]) for o, _ in outs) == 63


def test_pingpong_two_ranks(apps):
    """Round trips of a 256 KiB tile between two ranks, payload checked at every hop
    (reference tests/apps/pingpong rtt.jdf / bandwidth.jdf)."""
    rc, outs = launch.launch(2, [apps["pingpong"], "20", "32768"], timeout=120, capture=True)
    assert rc == 0, outs
    assert "rtt_us" in outs[0][0]
    hops = sum(int(o.split("hops")[1].split()[0]) for o, _ in outs)
    assert hops == 41


@pytest.mark.parametrize("nranks", [2, 4])
def test_all2all_multiprocess(apps, nranks):
    """Every rank sends a distinct NEW buffer to every rank; each DONE gathers
    one CTL per sender (reference tests/apps/all2all)."""
    rc, outs = launch.launch(nranks, [apps["all2all"]], timeout=120, capture=True)
    assert rc == 0, outs
    assert sum(int(o.split("recv")[1].split()[0]) for o, _ in outs) == nranks * nranks
    assert all("bad 0" in o for o, _ in outs)


def test_dynamic_termdet_multiprocess(tmp_path):
    """ptgpp --dynamic-termdet across 3 ranks: remote first activations count the
    tasks they create; termination still waits for the last remote NODE."""
    exe = ptgpp.build_program(os.path.join(HERE, "jdf", "tree_reduce.jdf"), str(tmp_path), flags=["--dynamic-termdet"])
    rc, outs = launch.launch(3, [exe, "6"], timeout=120, capture=True)
    assert rc == 0, outs
    assert "root 2080" in outs[0][0]
    assert sum(int(o.split("nodes")[1].split()[0]) for o, _ in outs) == 63


def _build_ce(tmp_path, gpu=False):
    exe = tmp_path / ("ce_capi_gpu" if gpu else "ce_capi")
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "ce_capi.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    if gpu:
        cmd[1:1] = ["-DCE_WITH_HIP", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
    else:
        cmd.insert(1, "-Werror")
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return str(exe)


def test_comm_engine_c_program(tmp_path, pa):
    """The communication-engine vtable from C (port of the reference's
    tests/dsl/dtd/dtd_test_ce.c): active messages both ways, a GET and a PUT on
    registered host memory with AM completion notices, pack / unpack, and five
    messages on a tag rank 0 registers only after they arrived (kept in order
    by the engine's unexpected-message queue, not dropped)."""
    exe = _build_ce(tmp_path)
    rc, outs = launch.launch(2, [exe], timeout=120, capture=True)
    assert rc == 0, outs
    text = "".join(o for o, _ in outs)
    assert text.count("ce ok") == 2 and "[1] GET ok" in text and "[1] PUT ok" in text, text


def test_runtime_extras_c_program(tmp_path, pa):
    """at_fini, taskpool ids, device registry, data advice and info registries
    from C (reference runtime.h:221,255,448-495, device.c:79,987, class/info.h)."""
    exe = tmp_path / "runtime_capi"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "runtime_capi.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, env=dict(os.environ, PARSEC_MCA_device_hip_enabled="0"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime capi ok" in r.stdout


@pytest.mark.parametrize("nranks", [1, 3])
def test_matrix_operators_c_program(tmp_path, pa, nranks):
    """parsec_apply / map_operator / reduce_col / redistribute (PTG) from C
    (reference data_dist/matrix/matrix.h:143-290), 1 and 3 ranks."""
    exe = tmp_path / "matrix_ops_capi"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "matrix_ops_capi.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rc, outs = launch.launch(nranks, [str(exe)], timeout=90, capture=True, env={"PARSEC_MCA_device_hip_enabled": "0"})
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert text.count("bad 0") == nranks


@pytest.mark.parametrize("nranks", [1, 3])
def test_collections_c_program(tmp_path, pa, nranks):
    """parsec_matrix_sym_block_cyclic_init, parsec_matrix_tabular_init (+ random
    table), parsec_vector_two_dim_cyclic_init, parsec_hash_datadist_create and
    parsec_broadcast_New from C, 1 and 3 ranks (reference
    sym_two_dim_rectangle_cyclic.c:228, two_dim_tabular.c:126,
    vector_two_dim_cyclic.c:40, hash_datadist.c:27, broadcast.jdf:160)."""
    exe = tmp_path / "collections_capi"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "collections_capi.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rc, outs = launch.launch(nranks, [str(exe)], timeout=90, capture=True, env={"PARSEC_MCA_device_hip_enabled": "0"})
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert text.count("collections capi rank") == nranks and text.count(f"/{nranks} bad 0") == nranks, text
    if nranks > 1:
        assert text.count("broadcast rank") == nranks


@pytest.fixture(scope="module")
def dtd_more(tmp_path_factory, pa):
    exe = tmp_path_factory.mktemp("dtdmore") / "dtd_more"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", "-D_DEFAULT_SOURCE", f"-I{ROOT}/include", os.path.join(HERE, "capi", "dtd_more_capi.c"),
           "-o", str(exe), f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64",
           "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return str(exe)


@pytest.mark.parametrize("args,nranks", [
    (["interface"], 1),
    (["hierarchy"], 1), (["hierarchy"], 3),
    (["template_counter"], 1), (["template_counter"], 4),
    (["global_id"], 3),
    (["explicit"], 1), (["explicit"], 2),
    (["interleave", ""], 2), (["interleave", "a"], 3), (["interleave", "if"], 4), (["interleave", "afiw"], 2),
])
def test_dtd_reference_programs(dtd_more, args, nranks):
    """dtd_test_insert_task_interface / explicit_task_creation / hierarchy (a task that runs its own DTD
    taskpool) / template_counter / global_id_for_dc_assumed / interleave_actions
    (ranks > 0 lag before add / insert / flush / wait), reference tests/dsl/dtd."""
    rc, outs = launch.launch(nranks, [dtd_more, *args], timeout=90, capture=True, env={"PARSEC_MCA_device_hip_enabled": "0"})
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert text.count(f"dtd_more {args[0]} rank") == nranks and "FAILED" not in text
    if args[0] == "global_id":
        ids = {line.split("ids ")[1] for line in text.splitlines() if "ids " in line}
        assert len(ids) == 1, ids  # the same ids on every rank


@pytest.mark.parametrize("nranks", [1, 3, 4])
def test_redistribute_random_c_program(tmp_path, pa, nranks):
    """Port of the reference's testing_redistribute_random.c: a window between
    two tabular collections with random tile -> rank tables (seeds 2873 /
    3872) and different tile sizes, PTG and DTD redistribution, checked in the
    target and after the round trip back into a zeroed source."""
    exe = tmp_path / "redistribute_random"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{ROOT}/include", os.path.join(HERE, "capi", "redistribute_random.c"), "-o", str(exe),
           f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rc, outs = launch.launch(nranks, [str(exe)], timeout=120, capture=True, env={"PARSEC_MCA_device_hip_enabled": "0"})
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert "Redistribute Result is CORRECT" in text and text.count("bad 0, round trip bad 0") == 2 * nranks, text


_LINK = [f"-L{ROOT}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
HAAR = "/root/reference/tests/apps/haar_tree"


def test_hash_table_c_program(tmp_path, pa):
    """Public parsec_hash_table (include/parsec/class/parsec_hash_table.h):
    8 threads racing find-then-insert under bucket handles, growth from 16
    buckets, for_all with removal, user key functions (reference
    tests/class/hash.c)."""
    exe = tmp_path / "hash_table"
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", "-pthread", f"-I{ROOT}/include", os.path.join(HERE, "capi", "hash_table_capi.c"),
           "-o", str(exe), *_LINK]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hash table ok" in r.stdout and "40000 items" in r.stdout


@pytest.mark.skipif(not os.path.exists(os.path.join(HAAR, "tree_dist.c")), reason="reference tree not present")
def test_reference_tree_dist_collection(tmp_path, pa):
    """The reference's haar-tree collection (tests/apps/haar_tree/tree_dist.c),
    compiled unmodified with -Werror against include/ (hash table, vpmap,
    device module, register_memory / key_to_string hooks) and driven by
    tests/capi/tree_dist_driver.c."""
    exe = tmp_path / "tree_dist"
    cmd = ["gcc", "-std=gnu99", "-Wall", "-Wextra", "-Werror", "-O1", "-pthread", f"-I{ROOT}/include", f"-I{HAAR}",
           os.path.join(HERE, "capi", "tree_dist_driver.c"), os.path.join(HAAR, "tree_dist.c"), "-o", str(exe), *_LINK]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    dot = tmp_path / "tree.dot"
    r = subprocess.run([str(exe), str(dot)], capture_output=True, text=True, timeout=60, env=dict(os.environ, PARSEC_MCA_device_hip_enabled="0"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tree_dist ok" in r.stdout
    text = dot.read_text()
    assert text.startswith("digraph G {") and text.count("->") == 62


@pytest.mark.skipif(not os.path.isdir("/root/reference/tests/class"), reason="reference tree not present")
@pytest.mark.parametrize("prog,args,check", [
    ("hash", ["-#", "65536", "-r", "4", "-n"], "threads"),
    ("hash", ["-#", "65536", "-r", "4", "-n", "-H"], "threads"),
    ("atomics", ["-c", "4"], "No error in integer operation on 64 bits"),
    ("rwlock", ["-c", "4"], None),
    ("lifo", ["-c", "4"], "all tests passed"),
    ("list", ["-c", "4"], "all tests passed"),
    ("future", ["-c", "4"], "countable future successfully triggered"),
    ("future_datacopy", [], "Nested parsec_datacopy_future validated"),
], ids=["hash", "hash-handles", "atomics", "rwlock", "lifo", "list", "future", "future_datacopy"])
def test_reference_class_programs(tmp_path, pa, prog, args, check):
    """The reference's tests/class programs (Testings.cmake: hash -# 65536 -r 4 -n,
    atomics / rwlock / lifo / list -c 4), compiled unmodified against include/:
    the public hash table under concurrent find-then-insert / remove with and
    without bucket handles (every inconsistency is printed as 'Error in
    implementation'), the C atomics, the reader / writer lock, the object
    system (PARSEC_OBJ_CONSTRUCT) with the lock-free LIFO (tagged head, aligned
    items) and the locked list (sort by priority offset), base / countable /
    datacopy futures with nested futures (future / future_datacopy), with the barrier /
    bindthread / timing / hwloc / MCA-index helpers they use."""
    ref = "/root/reference"
    exe = tmp_path / prog
    cmd = ["g++", "-x", "c++", "-std=c++20", "-fpermissive", "-w", "-O1", "-pthread", f"-I{ROOT}/include", f"-I{ref}",
           os.path.join(ref, "tests/class", prog + ".c"), "-o", str(exe), *_LINK]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "Error in implementation" not in r.stdout + r.stderr
    if check:
        assert check in r.stdout + r.stderr, r.stdout[-2000:]
