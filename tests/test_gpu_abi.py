"""The C ABI driven from C++ alone (tests/c/test_abi.cpp): one local KKT solve (Schur operator
handle + whole-solve PETSc LGMRES) on two library contexts with two streams from two host threads
concurrently; both solutions bit-identical and equal to the oracle's to 1e-8 with the same
iteration count.  Fixture: tests/golden/make_abi_fixture.py."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "test_abi")
FIX = os.path.join(ROOT, "tests", "golden", "abi_lgmres.bin")


def test_c_abi_local_kkt_solve_on_two_contexts():
    assert os.path.exists(BIN), "tests/c/test_abi not built (run __graft_entry__.build())"
    p = subprocess.run([BIN, FIX], capture_output=True, text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0 and "PASS" in p.stdout, p.stdout + p.stderr
