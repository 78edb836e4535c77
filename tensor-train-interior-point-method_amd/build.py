"""Build libttk.so for gfx950 (hipcc cross-compiles here; the .so travels to the GPU box)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libttk.so")
SOURCES = ["ttk_runtime.hip", "ttk_contract.hip", "ttk_einsum.hip", "ttk_linalg.hip", "ttk_lgmres.hip"]
HEADERS = ["ttk_common.h", os.path.join("..", "..", "include", "ttk.h")]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS if os.path.exists(os.path.join(CSRC, s))]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    cmd = ["hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950", "-std=c++17",
           "-Wno-unused-variable", "-Wno-unused-but-set-variable", "-o", OUT] + srcs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
