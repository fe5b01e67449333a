"""The C ABI library: it loads without a GPU, exports every symbol the header
declares, and its host-only paths behave (no compute calls here)."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_fixture
import qkd_ldpc_v_amd as Q
from qkd_ldpc_v_amd import HMatrix, QLDPCError


def _declared():
    hdr = open(os.path.join(ROOT, "include", "qkd_ldpc_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return set(re.findall(r"\b(qldpc_\w+)\s*\(", hdr))


def test_header_symbols_exported():
    so = Q._lib.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (qldpc_\w+)", out))
    declared = _declared()
    assert declared, "no declarations parsed"
    assert declared <= exported, declared - exported
    assert declared == set(Q.exported_symbols())
    Q.lib()  # every signature resolves


def test_version_and_log_p():
    assert "gfx950" in Q.version()
    for q in (0.0215, 0.015, 0.2, 0.013, 1e-3):
        assert Q.log_p(q) == math.log((1.0 - q) / q)


def test_graph_rejects_inconsistent_bit_nodes():
    """bit_nodes must list every edge of check_nodes (any order: the reference's
    occurrence pairing, tests/test_unsorted.py); a column that names a check
    twice instead of its two checks is refused."""
    H = HMatrix.from_check_nodes(4, [[0, 1, 2], [1, 2, 3]])
    ri = H.row_idx.copy()
    cp = H.col_ptr
    ri[cp[1]:cp[2]] = [1, 1]  # bit 1 lists check 1 twice
    bad = HMatrix(H.n, H.m, H.row_ptr, H.col_idx, cp, ri)
    with pytest.raises(QLDPCError, match="EUNSUP"):
        Q.Graph(bad)


def test_graph_rejects_inconsistent_edges():
    H = HMatrix.from_check_nodes(4, [[0, 1, 2], [1, 2, 3]])
    bad = HMatrix(H.n, H.m, H.row_ptr, H.col_idx, H.col_ptr.copy(), H.row_idx.copy())
    bad.col_ptr[-1] -= 1
    with pytest.raises(QLDPCError):
        Q.Graph(bad)


def test_atomic_optimizer_workaround_on_every_product_compile():
    """The split-frame miscompile workaround (Makefile comment)
    must reach every hipcc line of the product library."""
    mk = open(os.path.join(ROOT, "Makefile")).read()
    hipflags = re.search(r"^HIPFLAGS := (.*?)(?<!\\)\n", mk, flags=re.S | re.M).group(1)
    assert "-amdgpu-atomic-optimizer-strategy=None" in hipflags
    for line in mk.splitlines():
        if line.strip().startswith("$(HIPCC)") and " -c " in line:
            assert "$(HIPFLAGS)" in line, line


def test_bank_relabelling_host_plan():
    """The planner's bank-aware bit labels (relabel.cpp), host only: a
    permutation, deterministic, and on the random 10k codes it drives every
    slot group's busiest LDS bank down (C2: 3.5 -> about 2 addresses per half)."""
    from conftest import load_fixture

    for name in ("c2_n10240_m2201.alist", "c3_n10240_m1801.alist"):
        H = load_fixture(name)
        lab, st = Q.Graph(H, host_only=True).labels()
        assert np.array_equal(np.sort(lab), np.arange(H.n))
        assert st["cycles_after"] < 0.7 * st["cycles_before"], st
        assert st["excess_after"] < st["excess_before"]
        lab2, _ = Q.Graph(H, host_only=True).labels()
        assert np.array_equal(lab, lab2)


def test_relabelling_only_on_one_workgroup_register_shapes():
    from conftest import load_fixture

    H = load_fixture("c4s_n102400_m32001.alist")  # split frames: reference ids
    lab, st = Q.Graph(H, host_only=True).labels()
    assert np.array_equal(lab, np.arange(H.n)) and st["cycles_before"] == 0
    old = os.environ.get("QLDPC_RELABEL")
    os.environ["QLDPC_RELABEL"] = "0"
    try:
        lab, _ = Q.Graph(load_fixture("c2_n10240_m2201.alist"), host_only=True).labels()
        assert np.array_equal(lab, np.arange(lab.size))
    finally:
        if old is None:
            os.environ.pop("QLDPC_RELABEL")
        else:
            os.environ["QLDPC_RELABEL"] = old


def test_split_part_size_by_frames_per_xcd():
    """plan_v2_split (host planner, no GPU): parts of 16 waves (one per CU) or
    of 8 (two per CU, half the LDS), whichever runs more frames at once on an
    XCD's 32 CUs (ties: 8 waves).  C4 stand-in (307,200 edges): 8 x 16 waves
    or 15 x 8, 4 frames per XCD either way -> 8-wave parts.  C4 (ii) (409,600 edges): 11 x 16 waves
    leave 10 CUs of an XCD waiting (2 frames), 21 x 8 waves run 3 -> 8-wave
    parts within 80 KiB of LDS each."""
    from conftest import load_fixture

    p4 = Q.Graph(load_fixture("c4s_n102400_m32001.alist"), host_only=True).plan(0, Q.SPA)
    assert p4["variant"] == "v2_split" and p4["lanes"] == 15 * 512, p4
    g = Q.Graph(Q.regular_code(102400, 22001, 4, 777), host_only=True)
    for alg in (Q.SPA, Q.OMSA):
        p = g.plan(0, alg)
        assert p["variant"] == "v2_split" and p["lanes"] == 21 * 512 and p["lds_bytes"] <= 80 * 1024, p
    old = os.environ.get("QLDPC_SPLIT_WP")
    os.environ["QLDPC_SPLIT_WP"] = "16"
    try:
        p16 = Q.Graph(Q.regular_code(102400, 22001, 4, 777), host_only=True).plan(0, Q.SPA)
        assert p16["lanes"] == 11 * 1024, p16
        p4 = Q.Graph(load_fixture("c4s_n102400_m32001.alist"), host_only=True).plan(0, Q.SPA)
        assert p4["lanes"] == 8 * 1024, p4
    finally:
        if old is None:
            os.environ.pop("QLDPC_SPLIT_WP")
        else:
            os.environ["QLDPC_SPLIT_WP"] = old


def test_device_entries_refuse_non_row_major_buffers():
    """The C ABI reads [frame][bit] rows: a transposed (column-major) tensor is
    refused before any call, and the host syndrome helper is row-major (numpy's
    last-axis fancy indexing returns Fortran order, which torch.from_numpy keeps)."""
    import torch

    from qkd_ldpc_v_amd.graph import _dp

    t = torch.zeros((4, 3), dtype=torch.uint8)
    assert _dp(t) == t.data_ptr() and _dp(None) is None
    with pytest.raises(ValueError, match="C-contiguous"):
        _dp(t.t())
    H = load_fixture("c1_n1024_m220.alist")
    a, _, _ = Q.bsc_frames(H.n, 0.03, 4, seed=1)
    assert H.syndrome(a).flags["C_CONTIGUOUS"]
