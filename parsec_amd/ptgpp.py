"""Driver for the PTG compiler: .jdf -> C++ (parsec-ptgpp) -> program / library.

    from parsec_amd import ptgpp
    exe = ptgpp.build_program("chain.jdf", "/tmp/out")     # main() in the JDF epilogue
    ptgpp.compile_jdf("chain.jdf", "/tmp/out")              # just the generated .cpp/.h

CPU-only JDFs are compiled with g++; JDFs with BODY [type=HIP] (or hip=True)
with hipcc for gfx950. Mirrors the reference's CMake helper
target_ptg_sources (cmake_modules/ParsecCompilePTG.cmake:142-150).
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "parsec_amd")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
PTGPP = os.path.join(PKG, "bin", "parsec-ptgpp")


class CompileError(RuntimeError):
    pass


def run_ptgpp(jdf, out_base=None, function_base=None, check_only=False, flags=()):
    """Run parsec-ptgpp; returns CompletedProcess (stdout/stderr captured).
    ``flags``: extra compiler options (--dynamic-termdet, --dep-management X, --noline, -W...)."""
    if not os.path.exists(PTGPP):
        raise CompileError("parsec-ptgpp is not built (python -m parsec_amd._build)")
    cmd = [PTGPP, "-i", jdf]
    if out_base:
        cmd += ["-o", out_base]
    if function_base:
        cmd += ["-f", function_base]
    if check_only:
        cmd.append("-E")
    cmd += list(flags)
    return subprocess.run(cmd, capture_output=True, text=True)


def compile_jdf(jdf, outdir, name=None, flags=()):
    os.makedirs(outdir, exist_ok=True)
    name = name or os.path.splitext(os.path.basename(jdf))[0]
    base = os.path.join(outdir, name)
    r = run_ptgpp(jdf, base, name, flags=flags)
    if r.returncode != 0:
        raise CompileError(r.stderr)
    return base + ".cpp", base + ".h"


def _has_hip_body(jdf):
    with open(jdf) as f:
        src = f.read()
    return "type=HIP" in src.replace(" ", "")


def compile_flags(hip=False, sanitize=None):
    """sanitize: "thread" / "address": instrumented host code linked against the
    sanitized runtime of build-<kind>/ (parsec_amd._build.build_sanitized)."""
    inc = [f"-I{ROOT}/include", f"-I{ROOT}/csrc", f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__"]
    lib = os.path.join(ROOT, "build-" + sanitize) if sanitize else os.path.join(PKG, "lib")
    libs = [f"-L{lib}", "-lparsec_amd", f"-Wl,-rpath,{lib}", f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib", "-lpthread"]
    if sanitize:
        if hip:
            raise CompileError("sanitized builds are host-only (no HIP bodies)")
        return ["g++", "-std=c++20", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"] + inc, [f"-fsanitize={sanitize}"] + libs
    if hip:
        return [f"{ROCM}/bin/hipcc", "-std=c++20", "-O2", f"--offload-arch={ARCH}"] + inc, libs
    return ["g++", "-std=c++20", "-O2"] + inc, libs


# JDF bodies written in C (the reference's): compiled as C++ with C's lenient rules
C_BODIES = ("-fpermissive", "-Drestrict=__restrict__", "-w")


def build_program(jdf, outdir, extra_sources=(), hip=None, name=None, flags=(), cxxflags=(), sanitize=None):
    """cxxflags: extra compiler flags, e.g. C_BODIES for JDFs whose C code
    relies on C rules (implicit void * conversions, `restrict`); sanitize: see
    compile_flags."""
    cpp, _ = compile_jdf(jdf, outdir, name, flags=flags)
    hip = (_has_hip_body(jdf) if hip is None else hip) and not sanitize
    cc, libs = compile_flags(hip, sanitize)
    exe = os.path.splitext(cpp)[0]
    cmd = cc + list(cxxflags) + [f"-I{outdir}", f"-I{os.path.dirname(os.path.abspath(jdf))}", cpp] + list(extra_sources) + ["-o", exe] + libs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise CompileError(" ".join(cmd) + "\n" + r.stderr[-6000:])
    return exe
