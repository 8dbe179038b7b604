"""The reference's GPU test programs, rewritten for HIP:

    reference                                   here
    tests/dsl/ptg/cuda/stress.jdf               tests/jdf/stress_hip.jdf
    tests/dsl/ptg/cuda/get_best_device_check    tests/jdf/get_best_device_check_hip.jdf
    tests/dsl/ptg/cuda/nvlink.jdf               tests/jdf/nvlink_hip.jdf
    contrib/build_with_parsec/write_check       contrib/build_with_parsec/ (CMake package)
    tests/dsl/dtd/dtd_test_new_tile.c           tests/capi/dtd_gpu_capi.c (new_tile)
    tests/dsl/dtd/dtd_test_cuda_task_insert.c   tests/capi/dtd_gpu_capi.c (memset / read / write,
                                                multiple devices) + per-stream handle DGEMM

Every program also runs without a GPU (the CPU chores / simulated devices of
the reference's own fallbacks); the `gpu`-marked variants require the HIP path
(no CPU chore may run where a GPU one was asked for)."""
import os
import shutil
import subprocess

import pytest

from parsec_amd import launch, ptgpp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
JDF = os.path.join(HERE, "jdf")
CONTRIB = os.path.join(ROOT, "contrib", "build_with_parsec")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
NOGPU = {"PARSEC_MCA_device_hip_enabled": "0"}


def _run(cmd, env=None, timeout=100):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)


@pytest.fixture(scope="module")
def progs(tmp_path_factory, pa):
    """Lazily built programs, shared by the CPU and GPU variants of a test."""
    out = tmp_path_factory.mktemp("gpuprogs")
    built = {}

    def get(name):
        if name not in built:
            if name == "write_check":
                built[name] = ptgpp.build_program(os.path.join(CONTRIB, "write_check.jdf"), str(out),
                                                  extra_sources=[os.path.join(CONTRIB, "write_check_kernels.hip")])
            elif name == "dtd_gpu_capi":
                exe = out / "dtd_gpu_capi"
                obj_c, obj_k = out / "dgc.o", out / "dgk.o"
                cc = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", "-D__HIP_PLATFORM_AMD__", f"-I{ROOT}/include", f"-I{ROCM}/include",
                      "-c", os.path.join(HERE, "capi", "dtd_gpu_capi.c"), "-o", str(obj_c)]
                kc = [f"{ROCM}/bin/hipcc", f"--offload-arch={ptgpp.ARCH}", "-O2", "-c", os.path.join(HERE, "capi", "dtd_gpu_kernels.hip"), "-o", str(obj_k)]
                ln = [f"{ROCM}/bin/hipcc", f"--offload-arch={ptgpp.ARCH}", str(obj_c), str(obj_k), "-o", str(exe), f"-L{ROOT}/parsec_amd/lib",
                      "-lparsec_amd", f"-Wl,-rpath,{ROOT}/parsec_amd/lib"]
                for cmd in (cc, kc, ln):
                    r = subprocess.run(cmd, capture_output=True, text=True)
                    assert r.returncode == 0, " ".join(cmd) + "\n" + r.stderr
                built[name] = str(exe)
            else:
                built[name] = ptgpp.build_program(os.path.join(JDF, name + ".jdf"), str(out))
        return built[name]

    return get


# ------------------------------------------------------------------ stress
def test_stress_simulated_gpus(progs):
    """stress.jdf without GPUs: 4 pseudo devices, every GEMM on the CPU body."""
    r = _run([progs("stress_hip"), "6", "64"], env=NOGPU)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpus 4 simulated 1 gemms 24/24 gpu 0 cpu 24 misplaced 0 discards 4 bad_c 0" in r.stdout


def test_stress_simulated_two_ranks(progs):
    exe = progs("stress_hip")
    rc, outs = launch.launch(2, [exe, "4", "32"], timeout=100, capture=True, env=NOGPU)
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert text.count("gemms 16/16") == 2 and text.count("bad_c 0") == 2


@pytest.mark.gpu
def test_stress_gpu(progs):
    """Every GEMM on the GPU its C was pinned to, C intact (alpha 0, beta 1)."""
    r = _run([progs("stress_hip"), "16", "512"])
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("stress ")][-1]
    assert "simulated 0" in line and " cpu 0 " in line and "misplaced 0" in line and "bad_c 0" in line, line


# ------------------------------------------------------- get_best_device
def test_best_device_cpu(progs):
    r = _run([progs("get_best_device_check_hip"), "512", "64"], env=NOGPU)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpus 0 tasks 36 checked 36 gpu 0 cpu 36 wrong_device 0 bad_values 0" in r.stdout


@pytest.mark.gpu
def test_best_device_gpu(progs):
    """PREFERRED_DEVICE advice on a READ tile steers the reader; B (NEW, filled
    on the GPU) comes back to the host intact. Task weights are per-task
    expressions (weight=m+n+1)."""
    r = _run([progs("get_best_device_check_hip"), "2048", "128"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tasks 136 checked 136 gpu 136 cpu 0 wrong_device 0 bad_values 0" in r.stdout, r.stdout


# ------------------------------------------------------------------ nvlink
def test_nvlink_needs_a_gpu(progs):
    r = _run([progs("nvlink_hip")], env=NOGPU)
    assert r.returncode == 0 and "skipped" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_nvlink_user_device_copies(progs):
    """GEMM1 chains move A between GPUs; GEMM2 runs in place on the
    application's own hipMalloc'ed copy of userM(g) (parsec_data_copy_new +
    transfer_ownership), with a per-stream handle from the info registry."""
    r = _run([progs("nvlink_hip"), "8", "256"])
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("nvlink ")][-1]
    n = int(line.split("gpus ")[1].split()[0])
    assert f"gemm1 {8 * n}/{8 * n} gemm2 {8 * n}/{8 * n} user_ptr {8 * n} misplaced 0 cpu 0 bad_c 0 bad_user 0 bad_handle 0" in line, line


def _d2d_bytes(stderr):
    """Summed d2d bytes of device_show_statistics lines, and the HIP device names."""
    tot, names = 0, []
    for line in stderr.splitlines():
        if line.startswith("[parsec] device ") and " d2d=" in line:
            names.append(line.split()[3])
            tot += int(line.split(" d2d=")[1].split()[0])
    return tot, names


TWO_LOGICAL = {"PARSEC_MCA_device_hip_replicas": "2", "PARSEC_MCA_device_show_statistics": "1"}


@pytest.mark.gpu
def test_nvlink_two_logical_devices(progs):
    """The GPU registered twice (device_hip_replicas 2): nvlink's GEMM1 chains
    move A from one device to the next, so the device-to-device stage-in
    (hipMemcpyPeerAsync between two devices of the process) really runs --
    the route two distinct GPUs of one process take, here on one GPU."""
    r = _run([progs("nvlink_hip"), "8", "256"], env=TWO_LOGICAL)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("nvlink ")][-1]
    assert "gpus 2 " in line, line
    assert "gemm1 16/16 gemm2 16/16 user_ptr 16 misplaced 0 cpu 0 bad_c 0 bad_user 0 bad_handle 0" in line, line
    d2d, names = _d2d_bytes(r.stderr)
    assert "hip0.0" in names and "hip0.1" in names, r.stderr[-2000:]
    assert d2d > 0, r.stderr[-2000:]


@pytest.mark.gpu
def test_dtd_gpu_chores_two_logical_devices(progs):
    """The DTD GPU-chore programs over two devices of one process (the
    reference's dtd_test_cuda_task_insert multi-device cases)."""
    r = _run([progs("dtd_gpu_capi")], env=TWO_LOGICAL)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("new_tile", "memset (GPU)", "memset (alternating)", "memset_read (GPU)", "write_read (GPU)", "gemm_handle"):
        assert f"{name}: ok" in r.stdout, r.stdout
    _, names = _d2d_bytes(r.stderr)
    assert [n for n in names if n.startswith("hip")] == ["hip0.0", "hip0.1"], r.stderr[-2000:]


# ------------------------------------------------------------- write_check
@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not available")
def test_write_check_out_of_tree_cmake(tmp_path, pa):
    """An application outside the tree (contrib/build_with_parsec) finds the
    framework with find_package(ParsecAmd), compiles its JDF (HIP bodies) and a
    separate HIP kernel file, and runs (reference contrib/build_with_parsec)."""
    b = tmp_path / "wc"
    r = subprocess.run(["cmake", "-S", CONTRIB, "-B", str(b), "-G", "Ninja", f"-DCMAKE_HIP_COMPILER={ROCM}/lib/llvm/bin/clang++"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(["cmake", "--build", str(b)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    r = _run([str(b / "write_check"), "-n=2000", "-b=50"], env=NOGPU)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "elements 2000 gpu_bodies 0 errors 0" in r.stdout


def test_write_check_two_ranks(progs):
    exe = progs("write_check")
    rc, outs = launch.launch(2, [exe, "-n=1000", "-b=10"], timeout=100, capture=True, env=NOGPU)
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert text.count("errors 0") == 2


@pytest.mark.gpu
def test_write_check_gpu(progs):
    r = _run([progs("write_check"), "-n=100000", "-b=1000"])
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("write_check ")][-1]
    assert "errors 0" in line and "gpu_bodies 200" in line, line


# ------------------------------------------------------------ DTD GPU chores
def test_dtd_gpu_chores_cpu_fallback(progs):
    r = _run([progs("dtd_gpu_capi")], env=NOGPU)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "errors 0" in r.stdout


def test_dtd_gpu_chores_two_ranks_cpu(progs):
    rc, outs = launch.launch(2, [progs("dtd_gpu_capi")], timeout=100, capture=True, env=NOGPU)
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert "FAILED" not in text and text.count("errors 0") == 2
    assert text.count("superseded: ok") == 2, text


@pytest.mark.gpu
def test_dtd_gpu_chores_two_ranks_gpu(progs):
    """The same program on 2 ranks sharing the GPU: GPU chores, remote tiles
    over the IPC device plane. `superseded`: a remote GPU writer's version of a
    tile lands in device memory, a slow local CPU reader reads it, and the
    writer's NEXT version lands before that reader ran -- the reader still sees
    the first version (pulled to the host from its own, superseded copy)."""
    rc, outs = launch.launch(2, [progs("dtd_gpu_capi")], timeout=120, capture=True, env={"PARSEC_COMM_GPU": "0"})
    text = "".join(o for o, _ in outs)
    assert rc == 0, text + "".join(e for _, e in outs)
    assert "FAILED" not in text and text.count("errors 0") == 2, text
    assert text.count("superseded: ok") == 2, text


@pytest.mark.gpu
def test_dtd_gpu_chores(progs):
    """new_tile / memset / read / write / per-stream handle DGEMM with GPU chores
    chosen at insertion (parsec_dtd_insert_task_with_task_class device_type)."""
    r = _run([progs("dtd_gpu_capi")])
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    for name in ("new_tile", "memset (GPU)", "memset (alternating)", "memset_read (GPU)", "write_read (GPU)", "gemm_handle"):
        assert f"{name}: ok" in out, out
    gpu = int(out.split("chores gpu ")[1].split()[0])
    assert gpu >= 80, out
