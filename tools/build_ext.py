"""Build the mipipe HIP extension for gfx950 in-tree (no hipify, no JIT cache).

    python tools/build_ext.py [--force] [-j N]
    python tools/build_ext.py --asan-host     # host runtime under ASan/UBSan, built and run


Each ``csrc/kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` into an
object (plain HIP, no torch headers: seconds per file); ``csrc/bindings.cpp`` is the only
translation unit that includes torch.  Everything links into
``distributed-training-with-pipeline-parallelism_amd/_C.so`` against the libtorch /
HIP runtime that ships with the installed PyTorch, so the built file travels with the
repo snapshot to a GPU box.  Objects are rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-training-with-pipeline-parallelism_amd")
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("MIPIPE_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


# per-file compile flags.  attention.hip: no SLP packing -- -O3 pairs the softmax's independent
# f32 adds / multiplies into v_pk_*_f32, which beside MFMAs cost more issue cycles than the
# scalar ops they replace (MI355X_MICROARCH.md, 'price of one filler beside MFMAs')
FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"]}


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    tdir = os.path.dirname(torch.__file__)
    return ce.include_paths(device_type="cuda"), os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1]}")
    return r.stderr


def build(force: bool = False, jobs: int = 8, verbose: bool = False, variant: str = "", defines=()) -> str:
    """``variant`` + ``defines``: an A/B build (``_C_<variant>.so``, its own object dir) of the
    same sources with extra ``-D`` flags, loaded with MIPIPE_EXT_VARIANT=<variant>."""
    OBJ = os.path.join(ROOT, "build", "obj" + (f"_{variant}" if variant else ""))
    OUT = os.path.join(PKG, f"_C_{variant}.so" if variant else "_C.so")
    os.makedirs(OBJ, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "include", "*.h"))
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    base = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(CSRC, "include"),
            "-Wno-unused-result", "-Wno-unused-variable"] + [f"-D{d}" for d in defines]
    jobs_list = []
    objs = []
    for k in kernels:
        o = os.path.join(OBJ, os.path.basename(k) + ".o")
        objs.append(o)
        if force or _newer([k] + headers, o):
            jobs_list.append(base + FILE_FLAGS.get(os.path.basename(k), []) + ["-c", k, "-o", o])
    incs, tlib, abi = _torch_paths()
    # translation units that include torch: the pybind module, the native RCCL engine, the stage runner
    host_hdrs = glob.glob(os.path.join(CSRC, "comm", "*.h"))
    for bsrc in (os.path.join(CSRC, "bindings.cpp"), os.path.join(CSRC, "comm", "rccl_engine.cpp"),
                 os.path.join(CSRC, "runtime", "stage_runner.cpp")):
        bobj = os.path.join(OBJ, os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if force or _newer([bsrc] + host_hdrs, bobj):
            cmd = base + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
                          "-DTORCH_EXTENSION_NAME=_C", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                          "-isystem", "/opt/rocm/include"]
            for i in incs:
                cmd += ["-isystem", i]
            cmd += ["-isystem", sysconfig.get_paths()["include"], "-c", bsrc, "-o", bobj]
            jobs_list.append(cmd)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for msg in ex.map(_run, jobs_list):
            if verbose and msg:
                sys.stderr.write(msg)
    if force or jobs_list or not os.path.exists(OUT) or _newer(objs, OUT):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs + [
            "-L", tlib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
            "-ldl", f"-Wl,-rpath,{tlib}"]
        _run(link)
        # every symbol resolves (a kernel template whose host stub the compiler dropped links
        # fine and only fails at import -- or, worse, on the GPU box)
        import ctypes
        try:
            ctypes.CDLL(OUT, mode=os.RTLD_NOW | os.RTLD_LOCAL)
        except OSError as e:
            raise RuntimeError(f"{OUT} does not load: {e}") from None
    return OUT


def asan_host(run: bool = True) -> int:
    """The native runtime (csrc/runtime/stage_runner.cpp + csrc/comm/rccl_engine.h) built with
    g++ for the host under AddressSanitizer + UndefinedBehaviorSanitizer against the stand-in
    HIP / RCCL / torch headers of csrc/tests/host_stubs, and csrc/tests/host_asan_test.cpp run:
    two ranks replay tapes through an in-process fabric.  GPU sanitizers are not available on
    the MI355X pool, so this is where heap misuse, leaks and UB in the runtime are caught.
    Returns the test's exit status (0: clean)."""
    src = os.path.join(CSRC, "tests", "host_asan_test.cpp")
    exe = os.path.join(ROOT, "build", "host_asan_test")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    deps = [src] + glob.glob(os.path.join(CSRC, "tests", "host_stubs", "**", "*.h"), recursive=True) + [
        os.path.join(CSRC, "runtime", "stage_runner.cpp")] + glob.glob(os.path.join(CSRC, "comm", "*.h"))
    if _newer(deps, exe):
        _run([os.environ.get("CXX", "g++"), "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined",
              "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-Wall", "-Wno-unused-variable",
              "-I", os.path.join(CSRC, "tests", "host_stubs"), src, "-o", exe, "-lpthread", "-ldl"])
    if not run:
        return 0
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=600)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    return r.returncode


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--variant", default="", help="A/B build name: writes _C_<variant>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra define for a --variant build")
    ap.add_argument("--asan-host", action="store_true",
                    help="build + run the host runtime test under ASan/UBSan (no GPU, no hipcc)")
    a = ap.parse_args()
    if a.asan_host:
        sys.exit(asan_host())
    if a.defines and not a.variant:
        ap.error("-D needs --variant (the default _C.so is always the plain build)")
    print(build(a.force, a.j, a.v, a.variant, a.defines))
