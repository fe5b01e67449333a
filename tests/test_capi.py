"""The C ABI library: it loads without a GPU, exports every symbol the header
declares, and its host-only paths behave (no compute calls here)."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
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


def test_graph_rejects_unsorted_bit_nodes():
    H = HMatrix.from_check_nodes(4, [[0, 1, 2], [1, 2, 3]])
    ri = H.row_idx.copy()
    cp = H.col_ptr
    ri[cp[1]:cp[2]] = ri[cp[1]:cp[2]][::-1]  # bit 1 lists checks [1, 0]
    bad = HMatrix(H.n, H.m, H.row_ptr, H.col_idx, cp, ri)
    with pytest.raises(QLDPCError, match="EUNSUP"):
        Q.Graph(bad)


def test_graph_rejects_inconsistent_edges():
    H = HMatrix.from_check_nodes(4, [[0, 1, 2], [1, 2, 3]])
    bad = HMatrix(H.n, H.m, H.row_ptr, H.col_idx, H.col_ptr.copy(), H.row_idx.copy())
    bad.col_ptr[-1] -= 1
    with pytest.raises(QLDPCError):
        Q.Graph(bad)
