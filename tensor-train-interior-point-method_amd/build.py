"""Build libttk.so for gfx950 (hipcc cross-compiles here; the .so travels to the GPU box).

Each translation unit compiles to its own object in parallel (build/obj/), then one link."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libttk.so")
SOURCES = ["ttk_runtime.hip", "ttk_contract.hip", "ttk_einsum.hip", "ttk_linalg.hip", "ttk_lgmres.hip", "ttk_dense.hip",
           "ttk_host.hip"]
HEADERS = ["ttk_common.h", "ttk_internal.h", os.path.join("..", "..", "include", "ttk.h")]
FLAGS = ["-O3", "-fPIC", "--offload-arch=gfx950", "-std=c++17", "-Wno-unused-variable",
         "-Wno-unused-but-set-variable", "-I" + os.path.join(HERE, "..", "include")]


def _present(names):
    return [os.path.join(CSRC, s) for s in names if os.path.exists(os.path.join(CSRC, s))]


def _stale(out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in _present(SOURCES + HEADERS))


def build(force=False, verbose=False, out=OUT, defines=()):
    if not force and not _stale(out):
        return out
    tag = os.path.splitext(os.path.basename(out))[0]
    objdir = os.path.join(HERE, "build", "obj", tag)
    os.makedirs(objdir, exist_ok=True)
    extra = [f"-D{d}" for d in defines]

    def cc(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = ["hipcc", "-c"] + FLAGS + extra + ["-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd, cwd=CSRC)
        return obj

    srcs = _present(SOURCES)
    with ThreadPoolExecutor(max_workers=min(len(srcs), 6)) as ex:
        objs = list(ex.map(cc, srcs))
    cmd = ["hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", out] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    return out


BIND_SRC = os.path.join(CSRC, "ttk_host_bind.cpp")
BIND_DEPS = [BIND_SRC, os.path.join(CSRC, "ttk_host_eig.inc")]
BIND_OUT = os.path.join(HERE, "_ttkbind" + __import__("sysconfig").get_config_var("EXT_SUFFIX"))


def build_bind(force=False, verbose=False):
    """Host-side argument packer (`csrc/ttk_host_bind.cpp`): a torch C++ extension compiled with
    g++ (no device code), loaded next to libttk.so by dev.py."""
    if not force and os.path.exists(BIND_OUT) and \
            all(os.path.getmtime(BIND_OUT) >= os.path.getmtime(d) for d in BIND_DEPS):
        return BIND_OUT
    import sysconfig
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths() + [sysconfig.get_paths()["include"]]
    libdir = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    # -ffp-contract=off: the restated host arithmetic (NumPy's polar Gaussian, the pruning sums)
    # must round like NumPy's own, never through fused multiply-adds
    cmd = (["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-w", "-ffp-contract=off", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
            "-DTORCH_EXTENSION_NAME=_ttkbind", "-DTORCH_API_INCLUDE_EXTENSION_H"] + [f"-I{i}" for i in inc] +
           [BIND_SRC, "-o", BIND_OUT, f"-L{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            f"-Wl,-rpath,{libdir}"])
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    return BIND_OUT


CTEST_SRC = os.path.join(HERE, "..", "tests", "c", "test_abi.cpp")
CTEST_OUT = os.path.join(HERE, "..", "tests", "c", "test_abi")


def build_ctest(force=False, verbose=False):
    """The C-ABI test program (tests/c/test_abi.cpp): host code only, linked against libttk.so and
    the HIP runtime, rpath'd to the in-tree library."""
    if not os.path.exists(CTEST_SRC):
        return None
    deps = [CTEST_SRC, OUT, os.path.join(HERE, "..", "include", "ttk.h")]
    if not force and os.path.exists(CTEST_OUT) and all(os.path.getmtime(CTEST_OUT) >= os.path.getmtime(d) for d in deps):
        return CTEST_OUT
    cmd = ["hipcc", "-O2", "-std=c++17", "-o", CTEST_OUT, CTEST_SRC, "-L" + HERE, "-lttk", "-lpthread",
           "-Wl,-rpath,$ORIGIN/../../tensor-train-interior-point-method_amd"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=HERE)
    return CTEST_OUT


if __name__ == "__main__":
    defs = [a[2:] for a in sys.argv[1:] if a.startswith("-D")]
    outs = [a[6:] for a in sys.argv[1:] if a.startswith("--out=")]
    print(build(force="--force" in sys.argv, verbose=True, out=outs[0] if outs else OUT, defines=defs))
    print(build_bind(force="--force" in sys.argv, verbose=True))
    print(build_ctest(force="--force" in sys.argv, verbose=True))
