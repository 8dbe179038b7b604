"""Native build driver: generates build/build.ninja and runs ninja.

Outputs (in-tree so they travel with the repo snapshot to the GPU box):
  parsec_amd/lib/libparsec_amd.so   runtime + gfx950 HIP kernels
  parsec_amd/_C.<abi>.so            pybind11 bindings
  parsec_amd/bin/parsec-ptgpp       .jdf -> C++ compiler
  build/tests/*                     native unit tests

Usage: python -m parsec_amd._build [--clean] [-j N] [--sanitize address|thread|leak]

--sanitize KIND (reference CMake PARSEC_DEBUG_MEM_ADDR / _LEAK / _RACE,
CMakeLists.txt:195-200): host code of the runtime rebuilt with -fsanitize=KIND
into build-KIND/ (libparsec_amd.so, the container test and the C DTD program);
the gfx950 kernel objects of the main build are linked in uninstrumented.
"""
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "parsec_amd")
BUILD = os.path.join(ROOT, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

CORE_SOURCES = [
    "csrc/core/mca.cpp",
    "csrc/core/context.cpp",
    "csrc/core/scheduling.cpp",
    "csrc/core/recursive.cpp",
    "csrc/sched/schedulers.cpp",
    "csrc/termdet/termdet.cpp",
    "csrc/data/data.cpp",
    "csrc/data/collections.cpp",
    "csrc/device/device.cpp",
    "csrc/device/hip_device.cpp",
    "csrc/prof/profiling.cpp",
    "csrc/prof/ptg_to_dtd.cpp",
    "csrc/comm/remote_dep.cpp",
    "csrc/comm/shm_engine.cpp",
    "csrc/comm/shm_onesided.cpp",
    "csrc/comm/fourcounter.cpp",
    "csrc/ptg/ptg.cpp",
    "csrc/dtd/dtd.cpp",
    "csrc/algos/dpotrf.cpp",
    "csrc/algos/dgeqrf.cpp",
    "csrc/algos/dgeqrf_hqr.cpp",
    "csrc/algos/stencil3d.cpp",
    "csrc/algos/collection_ops.cpp",
    "csrc/algos/host_gemm.cpp",
    "csrc/algos/dtd_builtins.cpp",
    "csrc/capi/capi.cpp",
    "csrc/capi/hash_table.cpp", "csrc/capi/object.cpp", "csrc/capi/future_c.cpp", "csrc/capi/mpi_shim.cpp", "csrc/capi/redistribute_core.cpp",
    "csrc/algos/dpotrf_jdf.cpp",
    "csrc/algos/dgeqrf_jdf.cpp",
    "csrc/algos/redistribute_ptg.cpp",
]
HIP_SOURCES = [
    "csrc/kernels/tile_kernels.hip",
    "csrc/kernels/qr_kernels.hip",
    "csrc/kernels/stencil_kernels.hip",
]
PY_SOURCES = ["csrc/python/bindings.cpp"]
PTGPP_SOURCES = ["tools/ptgpp/ptgpp.cpp"]
# Taskpools written in the JDF language: compiled by parsec-ptgpp into build/gen
# and linked into the runtime library (reference: DPLASMA ships its *.jdf the same way)
JDF_SOURCES = [
    "csrc/algos/jdf/dpotrf_L.jdf",
    "csrc/algos/jdf/dgeqrf.jdf",
    "csrc/algos/jdf/redistribute.jdf",
    "csrc/algos/jdf/redistribute_reshuffle.jdf",
    "csrc/algos/jdf/diag_band_to_rect.jdf",
]
# runtime sources that include generated JDF headers
JDF_USERS = ["csrc/algos/dpotrf_jdf.cpp", "csrc/algos/dgeqrf_jdf.cpp", "csrc/algos/redistribute_ptg.cpp"]
FORTRAN_SOURCES = ["csrc/fortran/parsecf.F90", "csrc/fortran/parsec_profilef.F90"]
FLANG = os.path.join(ROCM, "lib", "llvm", "bin", "flang")
TEST_SOURCES = ["tests/native/test_containers.cpp", "tests/native/test_futures.cpp", "tests/native/test_fetch_queue.cpp"]


def _exists(paths):
    return [p for p in paths if os.path.exists(os.path.join(ROOT, p))]


def _pybind_include():
    import pybind11

    return pybind11.get_include()


def generate():
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.join(PKG, "lib"), exist_ok=True)
    os.makedirs(os.path.join(PKG, "bin"), exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    common = f"-std=c++20 -O3 -g -fPIC -Wall -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I{ROCM}/include -I{ROOT}/csrc -I{ROOT}/include"
    hipflags = f"-std=c++20 -O3 -fPIC --offload-arch={ARCH} -D__HIP_PLATFORM_AMD__ -I{ROOT}/csrc -Wno-unused-result"
    lines = [
        f"rocm = {ROCM}",
        f"cxxflags = {common}",
        f"hipflags = {hipflags}",
        "rule cxx",
        "  command = g++ $cxxflags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $out",
        "rule hipcc",
        f"  command = {ROCM}/bin/hipcc $hipflags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $out",
        "rule solink",
        "  command = g++ -shared -o $out $in $libs",
        "  description = LINK $out",
        "rule exelink",
        "  command = g++ -o $out $in $libs",
        "  description = LINK $out",
        "rule pycxx",
        f"  command = g++ $cxxflags -I{py_inc} -I{_pybind_include()} -fvisibility=hidden -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = PYCXX $out",
    ]
    lines += [
        "rule ptgpp",
        f"  command = {PKG}/bin/parsec-ptgpp -i $in -o $base -f $fname",
        "  description = PTGPP $in",
    ]
    ptgpp_exe = os.path.join(PKG, "bin", "parsec-ptgpp")
    gen = os.path.join(BUILD, "gen")
    gen_headers, objs = [], []
    for src in _exists(JDF_SOURCES):
        name = os.path.splitext(os.path.basename(src))[0]
        base = os.path.join(gen, name)
        lines.append(f"build {base}.cpp {base}.h: ptgpp {os.path.join(ROOT, src)} | {ptgpp_exe}")
        lines.append(f"  base = {base}")
        lines.append(f"  fname = {name}")
        obj = os.path.join("obj", "gen_" + name + ".o")
        lines.append(f"build {obj}: cxx {base}.cpp")
        lines.append(f"  cxxflags = {common} -I{gen} -Wno-unused-variable -Wno-unused-but-set-variable")
        objs.append(obj)
        gen_headers.append(base + ".h")
    for src in _exists(CORE_SOURCES):
        obj = os.path.join("obj", src.replace("/", "_") + ".o")
        if src in JDF_USERS:
            lines.append(f"build {obj}: cxx {os.path.join(ROOT, src)} || {' '.join(gen_headers)}")
            lines.append(f"  cxxflags = {common} -I{gen}")
        else:
            lines.append(f"build {obj}: cxx {os.path.join(ROOT, src)}")
        objs.append(obj)
    for src in _exists(HIP_SOURCES):
        obj = os.path.join("obj", src.replace("/", "_") + ".o")
        lines.append(f"build {obj}: hipcc {os.path.join(ROOT, src)}")
        objs.append(obj)
    lib = os.path.join(PKG, "lib", "libparsec_amd.so")
    libs = f"-L{ROCM}/lib -lamdhip64 -lrocprofiler-sdk-roctx -latomic -lpthread -lrt -ldl -Wl,-rpath,{ROCM}/lib"
    lines.append(f"build {lib}: solink {' '.join(objs)}")
    lines.append(f"  libs = {libs}")
    pyobjs = []
    for src in _exists(PY_SOURCES):
        obj = os.path.join("obj", src.replace("/", "_") + ".o")
        lines.append(f"build {obj}: pycxx {os.path.join(ROOT, src)}")
        pyobjs.append(obj)
    if pyobjs:
        mod = os.path.join(PKG, "_C" + ext)
        lines.append(f"build {mod}: solink {' '.join(pyobjs)} | {lib}")
        lines.append(f"  libs = -L{PKG}/lib -lparsec_amd '-Wl,-rpath,$$ORIGIN/lib' {libs}")
    ptg_objs = []
    for src in _exists(PTGPP_SOURCES):
        obj = os.path.join("obj", src.replace("/", "_") + ".o")
        lines.append(f"build {obj}: cxx {os.path.join(ROOT, src)}")
        ptg_objs.append(obj)
    if ptg_objs:
        lines.append(f"build {os.path.join(PKG, 'bin', 'parsec-ptgpp')}: exelink {' '.join(ptg_objs)}")
        lines.append("  libs = ")
    # GPU bandwidth shmoo (host code only, links the HIP runtime)
    bw = "tools/bandwidth/bandwidth.cpp"
    if os.path.exists(os.path.join(ROOT, bw)):
        lines.append(f"build obj/tools_bandwidth.o: cxx {os.path.join(ROOT, bw)}")
        lines.append(f"build {os.path.join(PKG, 'bin', 'parsec-bandwidth')}: exelink obj/tools_bandwidth.o")
        lines.append(f"  libs = -L{ROCM}/lib -lamdhip64 -Wl,-rpath,{ROCM}/lib")
    # Fortran 2008 modules (parsec_f08, parsec_profile_f08) with ROCm's flang:
    # objects in parsec_amd/lib, .mod files in parsec_amd/include/fortran
    if os.path.exists(FLANG) and _exists(FORTRAN_SOURCES):
        moddir = os.path.join(PKG, "include", "fortran")
        os.makedirs(moddir, exist_ok=True)
        lines.append("rule fc")
        lines.append(f"  command = {FLANG} -O2 -fPIC -module-dir {moddir} -c $in -o $out")
        lines.append("  description = FC $out")
        fobjs = []
        for src in _exists(FORTRAN_SOURCES):
            fo = os.path.join(PKG, "lib", os.path.splitext(os.path.basename(src))[0] + ".o")
            lines.append(f"build {fo}: fc {os.path.join(ROOT, src)}")
            fobjs.append(fo)
        lines.append("rule ar")
        lines.append("  command = rm -f $out && ar rcs $out $in")
        lines.append("  description = AR $out")
        lines.append(f"build {os.path.join(PKG, 'lib', 'libparsec_amd_f08.a')}: ar {' '.join(fobjs)}")
    for src in _exists(TEST_SOURCES):
        obj = os.path.join("obj", src.replace("/", "_") + ".o")
        exe = os.path.join(BUILD, "tests", os.path.splitext(os.path.basename(src))[0])
        lines.append(f"build {obj}: cxx {os.path.join(ROOT, src)}")
        lines.append(f"build {exe}: exelink {obj} | {lib}")
        lines.append(f"  libs = -L{PKG}/lib -lparsec_amd -Wl,-rpath,{PKG}/lib {libs}")
    with open(os.path.join(BUILD, "build.ninja"), "w") as f:
        f.write("\n".join(lines) + "\n")


SANITIZERS = ("address", "thread", "leak")


def sanitize_dir(kind):
    return os.path.join(ROOT, "build-" + kind)


def generate_sanitized(kind):
    """build-KIND/build.ninja: instrumented host runtime + test executables."""
    if kind not in SANITIZERS:
        raise ValueError(f"unknown sanitizer {kind!r}")
    out = sanitize_dir(kind)
    os.makedirs(os.path.join(out, "obj"), exist_ok=True)
    flags = (f"-std=c++20 -O1 -g -fno-omit-frame-pointer -fPIC -fsanitize={kind} -D__HIP_PLATFORM_AMD__ "
             f"-I{ROCM}/include -I{ROOT}/csrc -I{ROOT}/include -Wno-unused-result")
    libs = f"-fsanitize={kind} -L{ROCM}/lib -lamdhip64 -lrocprofiler-sdk-roctx -latomic -lpthread -lrt -Wl,-rpath,{ROCM}/lib"
    lines = [
        "rule cxx",
        f"  command = g++ {flags} $flags_extra -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX[" + kind + "] $out",
        "rule cc",
        f"  command = gcc -std=c99 -D_DEFAULT_SOURCE -O1 -g -fno-omit-frame-pointer -fsanitize={kind} -I{ROOT}/include -c $in -o $out",
        "  description = CC[" + kind + "] $out",
        "rule solink",
        "  command = g++ -shared -o $out $in $libs",
        "  description = LINK $out",
        "rule exelink",
        "  command = g++ -o $out $in $libs",
        "  description = LINK $out",
    ]
    objs = []
    gen = os.path.join(BUILD, "gen")  # generated by the main build (run it first)
    for src in _exists(JDF_SOURCES):
        name = os.path.splitext(os.path.basename(src))[0]
        obj = os.path.join(out, "obj", "gen_" + name + ".o")
        lines.append(f"build {obj}: cxx {os.path.join(gen, name + '.cpp')}")
        lines.append(f"  flags_extra = -I{gen}")
        objs.append(obj)
    for src in _exists(CORE_SOURCES):
        obj = os.path.join(out, "obj", src.replace("/", "_") + ".o")
        lines.append(f"build {obj}: cxx {os.path.join(ROOT, src)}")
        if src in JDF_USERS:
            lines.append(f"  flags_extra = -I{gen}")
        objs.append(obj)
    # device kernels: the main build's objects (host stubs only, not instrumented)
    for src in _exists(HIP_SOURCES):
        objs.append(os.path.join(BUILD, "obj", src.replace("/", "_") + ".o"))
    lib = os.path.join(out, "libparsec_amd.so")
    lines.append(f"build {lib}: solink {' '.join(objs)}")
    lines.append(f"  libs = {libs}")
    for src in _exists(TEST_SOURCES):
        obj = os.path.join(out, "obj", src.replace("/", "_") + ".o")
        exe = os.path.join(out, os.path.splitext(os.path.basename(src))[0])
        lines.append(f"build {obj}: cxx {os.path.join(ROOT, src)}")
        lines.append(f"build {exe}: exelink {obj} | {lib}")
        lines.append(f"  libs = -L{out} -lparsec_amd -Wl,-rpath,{out} {libs}")
    # C API programs run instrumented: the DTD program and the distributed PTG
    # Cholesky (ptgpp-compiled dpotrf_L.jdf, CPU bodies on 1..4 ranks)
    for capi in ("tests/capi/dtd_capi.c", "tests/capi/dpotrf_capi.c"):
        if not os.path.exists(os.path.join(ROOT, capi)):
            continue
        name = os.path.splitext(os.path.basename(capi))[0]
        lines.append(f"build {os.path.join(out, 'obj', name + '.o')}: cc {os.path.join(ROOT, capi)}")
        lines.append(f"build {os.path.join(out, name)}: exelink {os.path.join(out, 'obj', name + '.o')} | {lib}")
        lines.append(f"  libs = -L{out} -lparsec_amd -Wl,-rpath,{out} {libs} -lm")
    with open(os.path.join(out, "build.ninja"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return out


def _headers_fingerprint():
    import hashlib

    h = hashlib.sha1()
    for top in ("csrc", "include"):
        for root, _, files in sorted(os.walk(os.path.join(ROOT, top))):
            for f in sorted(files):
                if f.endswith((".h", ".hpp")):
                    st = os.stat(os.path.join(root, f))
                    h.update(f"{root}/{f}:{st.st_mtime_ns}:{st.st_size};".encode())
    return h.hexdigest()


def build_sanitized(kind, jobs=None):
    """Build the instrumented runtime (needs the main build's kernel objects)."""
    need = [os.path.join(BUILD, "obj", s.replace("/", "_") + ".o") for s in _exists(HIP_SOURCES)]
    need += [os.path.join(BUILD, "gen", os.path.splitext(os.path.basename(s))[0] + ".cpp") for s in _exists(JDF_SOURCES)]
    if not all(os.path.exists(p) for p in need):
        build(jobs)
    # one builder at a time per tree: parallel test workers (pytest -n) that
    # ran ninja in the same directory together corrupted its log and linked a
    # half-written library
    import fcntl
    os.makedirs(sanitize_dir(kind), exist_ok=True)
    with open(os.path.join(sanitize_dir(kind), ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        out = generate_sanitized(kind)
        # ninja's header dependencies live in its deps log; a log cut short (an
        # interrupted build) forgets them and left objects compiled against an
        # older runtime.hpp linked into the instrumented library. A changed
        # header set rebuilds everything.
        stamp = os.path.join(out, ".headers")
        fp = _headers_fingerprint()
        if not os.path.exists(stamp) or open(stamp).read() != fp:
            import shutil
            shutil.rmtree(os.path.join(out, "obj"), ignore_errors=True)
            for f in (".ninja_deps", ".ninja_log"):
                if os.path.exists(os.path.join(out, f)):
                    os.remove(os.path.join(out, f))
        r = subprocess.run(["ninja", "-C", out, f"-j{jobs or min(8, os.cpu_count() or 4)}"])
        if r.returncode == 0:
            with open(stamp, "w") as f:
                f.write(fp)
    if r.returncode != 0:
        raise RuntimeError(f"sanitized ({kind}) build failed")
    return out


def build(jobs=None, verbose=False):
    generate()
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmd = ["ninja", "-C", BUILD, f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd)
    if r.returncode != 0:
        raise RuntimeError("native build failed")


if __name__ == "__main__":
    if "--clean" in sys.argv:
        subprocess.run(["rm", "-rf", BUILD])
    j = None
    if "-j" in sys.argv:
        j = int(sys.argv[sys.argv.index("-j") + 1])
    if "--sanitize" in sys.argv:
        build_sanitized(sys.argv[sys.argv.index("--sanitize") + 1], j)
    else:
        build(j, verbose="-v" in sys.argv)
