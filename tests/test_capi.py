"""The C ABI library: it loads without a GPU, exports every symbol the header
declares, and its host-only paths behave (no compute calls here)."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, diag_env, load_fixture
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
    with diag_env(QLDPC_RELABEL="0"):
        lab, _ = Q.Graph(load_fixture("c2_n10240_m2201.alist"), host_only=True).labels()
        assert np.array_equal(lab, np.arange(lab.size))


def test_split_part_size_by_frames_per_xcd():
    """plan_v2_split (host planner, no GPU): four families — parts of 8 waves
    (two per CU) or 16 (one per CU), with or without 12 scratch message slots
    per lane — each at its smallest part count K.  Per slot budget the most
    frames per XCD (64 / K or 32 / K) wins (ties: 8 waves without scratch
    slots, 16 with them); the scratch-slot plan is taken at >= 4/3 the frames
    of the plan without.  C4 stand-in (307,200 edges): 8/0 K = 15 (4 frames)
    vs 16/12 K = 6 (5) -> 8/0.  C4 (ii) (409,600 edges): 8/0 K = 21 (3) vs
    16/12 K = 8 (4) -> 16/12."""
    from conftest import load_fixture

    c4s = load_fixture("c4s_n102400_m32001.alist")
    g = Q.Graph(c4s, host_only=True)
    p4 = g.plan(0, Q.SPA)
    assert p4["variant"] == "v2_split" and p4["lanes"] == 15 * 512 and p4["edges_per_lane"] <= 40, p4
    assert g.split_plan() == {"parts": 15, "part_lanes": 512, "scratch_slots": 0}
    g = Q.Graph(Q.regular_code(102400, 22001, 4, 777), host_only=True)
    for alg in (Q.SPA, Q.OMSA):
        p = g.plan(0, alg)
        assert p["variant"] == "v2_split" and p["lanes"] == 8 * 1024 and p["lds_bytes"] <= 160 * 1024, p
    assert g.split_plan() == {"parts": 8, "part_lanes": 1024, "scratch_slots": 12}
    expect = {  # (WP, SCRATCH) -> (parts, part lanes) for the stand-in / C4 (ii)
        ("8", "0"): ((15, 512), (21, 512)), ("8", "1"): ((12, 512), (16, 512)),
        ("16", "0"): ((8, 1024), (11, 1024)), ("16", "1"): ((6, 1024), (8, 1024)),
    }
    for (wp, sc), want in expect.items():
        with diag_env(QLDPC_SPLIT_WP=wp, QLDPC_SPLIT_SCRATCH=sc):
            for H, (k, pl) in zip((c4s, Q.regular_code(102400, 22001, 4, 777)), want):
                sp = Q.Graph(H, host_only=True).split_plan()
                assert (sp["parts"], sp["part_lanes"], sp["scratch_slots"]) == (k, pl, 12 if sc == "1" else 0), (wp, sc)
    with diag_env(QLDPC_SPLIT_SCRATCH="0"):  # without scratch slots: 8-wave parts (ties: 8 waves)
        assert Q.Graph(c4s, host_only=True).split_plan()["parts"] == 15
    with diag_env(QLDPC_SPLIT_SCRATCH="1"):  # with them: 16-wave parts (ties: 16 waves)
        assert Q.Graph(c4s, host_only=True).split_plan() == {"parts": 6, "part_lanes": 1024, "scratch_slots": 12}
    with diag_env(QLDPC_SPLIT_WP="16"):  # 16-wave family: the stand-in 8 x 16 (5/4 < 4/3), C4 (ii) 8 x 16 + scratch
        assert Q.Graph(c4s, host_only=True).split_plan() == {"parts": 8, "part_lanes": 1024, "scratch_slots": 0}
        assert Q.Graph(Q.regular_code(102400, 22001, 4, 777), host_only=True).split_plan()["scratch_slots"] == 12
    with diag_env(QLDPC_SPLIT_K="10"):  # the K = 10 layout the GPU parity suite decodes
        p10 = Q.Graph(c4s, host_only=True).plan(0, Q.SPA)
        assert p10["lanes"] == 10 * 1024, p10
    # one-workgroup frames answer one part
    assert Q.Graph(load_fixture("c2_n10240_m2201.alist"), host_only=True).split_plan()["parts"] == 1


# Every QLDPC_* A/B knob the library or its loader reads (capi.hip env_int /
# qldpc_diag_env, trials.hip, _lib.py); none may act without QLDPC_DIAG=1.
TUNING_KNOBS = {
    "QLDPC_VARIANT": "v1", "QLDPC_V2_WAVES": "12", "QLDPC_ROWS_LDS": "0", "QLDPC_RGLB_SHARE": "40",
    "QLDPC_SPLIT": "0", "QLDPC_SPLIT_X": "0", "QLDPC_SPLIT_K": "10", "QLDPC_SPLIT_WP": "16",
    "QLDPC_RELABEL": "0", "QLDPC_RELABEL_ITERS": "1", "QLDPC_HD_TABLES": "1", "QLDPC_VNG_DEAL": "0",
    "QLDPC_SPLIT_XORDER": "0", "QLDPC_DEBUG_PLAN": "1", "QLDPC_SPLIT_WGS": "64", "QLDPC_ROWS_COPY": "0",
    "QLDPC_VNG": "0", "QLDPC_ORDER": "0", "QLDPC_TRIAL_CHUNK": "3", "QLDPC_TRIAL_SERIAL": "1",
    "QLDPC_SPLIT_SCRATCH": "0",
}


def _plans():
    from conftest import load_fixture

    out = {}
    for name in ("c2_n10240_m2201.alist", "c3_n10240_m1801.alist", "c5_n10240_m2048.sp2", "c5c_n10240_m5120.sp2",
                 "c4s_n102400_m32001.alist"):
        g = Q.Graph(load_fixture(name), host_only=True)
        lab, _ = g.labels()
        out[name] = ([g.plan(0, a) for a in range(6)], lab)
    return out


def test_tuning_variables_ignored_without_diag_switch(monkeypatch):
    """With no diagnostic switch the product ignores every QLDPC_* tuning
    variable: the plans (variant, lanes, EPL, LDS) and bit labels of C2, C3,
    C5 (R = 0.8 and 0.5) and the C4 stand-in are unchanged with all of them
    set; under QLDPC_DIAG=1 they act (the A/B builds and tests use that)."""
    monkeypatch.delenv("QLDPC_DIAG", raising=False)
    for k in TUNING_KNOBS:
        monkeypatch.delenv(k, raising=False)
    clean = _plans()
    for k, v in TUNING_KNOBS.items():
        monkeypatch.setenv(k, v)
    stray = _plans()
    for name in clean:
        assert stray[name][0] == clean[name][0], name
        assert np.array_equal(stray[name][1], clean[name][1]), name
    monkeypatch.setenv("QLDPC_DIAG", "1")
    diag = _plans()
    assert diag["c4s_n102400_m32001.alist"][0] != clean["c4s_n102400_m32001.alist"][0]
    assert diag["c2_n10240_m2201.alist"][0][0]["variant"] != "v2"  # QLDPC_VARIANT=v1 acts


def test_loader_ignores_build_selectors_without_diag_switch():
    """QLDPC_AB_BUILD / QLDPC_DIAG_STAMPS / QLDPC_ASAN pick another in-tree
    library only under QLDPC_DIAG=1; otherwise the product library loads."""
    import subprocess
    import sys

    code = "import qkd_ldpc_v_amd._lib as L; print(L.LIB_PATH)"
    base = {k: v for k, v in os.environ.items() if not k.startswith("QLDPC_")}
    for sel in ({"QLDPC_AB_BUILD": "x"}, {"QLDPC_DIAG_STAMPS": "1"}, {"QLDPC_ASAN": "1"}):
        r = subprocess.run([sys.executable, "-c", code], env=dict(base, **sel), capture_output=True, text=True,
                           cwd=ROOT, timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout.strip() == os.path.join(ROOT, "qkd_ldpc_v_amd", "libqkdldpc_hip.so"), (sel, r.stdout)
        r = subprocess.run([sys.executable, "-c", code], env=dict(base, QLDPC_DIAG="1", **sel), capture_output=True,
                           text=True, cwd=ROOT, timeout=120)
        assert r.stdout.strip() != os.path.join(ROOT, "qkd_ldpc_v_amd", "libqkdldpc_hip.so"), sel


def test_library_reads_environment_only_through_the_diag_gate():
    """Static check of the product sources: the only getenv calls are the
    diagnostic gate itself (capi.hip qldpc_diag_env) — every knob goes through
    it — and the drop-in's device selection (QKD_LDPC_HIP_DEVICES, not a
    tuning knob: which GPUs the reference's driver runs on)."""
    import glob
    import re

    hits = []
    for f in sorted(glob.glob(os.path.join(ROOT, "qkd_ldpc_v_amd", "csrc", "*")) +
                    glob.glob(os.path.join(ROOT, "qkd_ldpc_v_amd", "host", "**", "*.?pp"), recursive=True)):
        if not f.endswith((".hip", ".cpp", ".hpp", ".h")):
            continue
        for i, line in enumerate(open(f), 1):
            if re.search(r"\bgetenv\s*\(", line):
                hits.append((os.path.basename(f), line.strip()))
    allowed = {'const char *d = std::getenv("QLDPC_DIAG");', "return std::getenv(name);"}
    rest = [h for h in hits if h[1] not in allowed and "QKD_LDPC_HIP_DEVICES" not in h[1]]
    assert not rest, rest
    assert sum(1 for h in hits if h[1] in allowed) == 2


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
