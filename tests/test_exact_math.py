"""The SPA kernel's tanh/atanh (qkd_ldpc_v_amd/csrc/exact_math.h) must be
bit-identical to the C library the reference calls (src/qkd_ldpc_algorithm.cpp:
60,68).  Host build of the same source, compared against live glibc."""
import os
import subprocess

from conftest import ROOT


def test_exact_math_matches_libc_bitwise(tmp_path):
    exe = tmp_path / "emc"
    subprocess.run(["g++", "-std=c++20", "-O2", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tools", "exact_math_check.cpp"), "-lpthread"], check=True)
    r = subprocess.run([str(exe), "1500000", "20251015"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tanh mismatches: 0" in r.stdout and "atanh mismatches: 0" in r.stdout
    assert "boundary mismatches: 0" in r.stdout
