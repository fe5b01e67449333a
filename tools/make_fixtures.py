#!/usr/bin/env python3
"""Regenerate tests/golden/matrices/ from the reference checkout (this container only).

The GPU box has no /root/reference, so the parity tests and bench.py read gzip
copies of the reference's matrix DATA files (parity-check matrices are inputs,
not source).  Each copy is recorded in MANIFEST.json with the reference path it
came from and the sha256 of the original bytes; tests/test_fixtures.py checks
that decompressing gives those bytes back.
"""
import gzip
import hashlib
import json
import os
import sys

REF = "/root/reference/sparse_matrices"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "matrices")

_M2K = [(1024, "0.9"), (1536, "0.85"), (2560, "0.75"), (3072, "0.7"), (4096, "0.6"), (4608, "0.55")]

# fixture name -> (reference path relative to sparse_matrices/, format id, role)
FIXTURES = {
    "c1_n1024_m220.alist": ("matrices_alist_1k_all/(N=1024,M=220,R=0.79,CW=5,SEED=444).mtrx", 1,
                            "C1: 1k R~0.8 (configs_all/config 1k.json)"),
    "c2_n10240_m2201.alist": ("matrices_alist_10k_all/(N=10240,M=2201,R=0.79,CW=4,SEED=777).mtrx", 1,
                              "C2: 10k R~0.8 SPA headline"),
    "c3_n10240_m1801.alist": ("matrices_alist_10k_all/(N=10240,M=1801,R=0.82,CW=4,SEED=777).mtrx", 1,
                              "C3: 10k R=0.82 OMSA"),
    "c4s_n102400_m32001.alist": ("matrices_alist_100k_all/(N=102400,M=32001,R=0.69,CW=3,SEED=777).mtrx", 1,
                                 "C4 stand-in: 100k R=0.69 (the R=0.79 file is absent upstream)"),
    "c5_n10240_m2048.sp2": ("matrices_2/(N=10240,M=2048,R=0.8).mtrx", 3, "C5: format-3 irregular R=0.8"),
    "c5_n10240_m2048.untp": ("matrices_2/(N=10240,M=2048,R=0.8).untp", -1, "C5 untainted puncturing cache"),
    "c5b_n10240_m3584.sp2": ("matrices_2/(N=10240,M=3584,R=0.65).mtrx", 3, "C5 sweep: format-3 irregular R=0.65"),
    "c5b_n10240_m3584.untp": ("matrices_2/(N=10240,M=3584,R=0.65).untp", -1, "C5 sweep: R=0.65 untainted list"),
    "c5c_n10240_m5120.sp2": ("matrices_2/(N=10240,M=5120,R=0.5).mtrx", 3, "C5 sweep: format-3 irregular R=0.5"),
    "c5c_n10240_m5120.untp": ("matrices_2/(N=10240,M=5120,R=0.5).untp", -1, "C5 sweep: R=0.5 untainted list"),
    # matrices_2_10k_all: the other format-3 codes with the reference's untainted lists
    # (the R=0.8 / 0.65 / 0.5 files there are byte-identical to matrices_2's)
    **{f"m2k_n10240_m{m}.sp2": (f"matrices_2_10k_all/(N=10240,M={m},R={r}).mtrx", 3,
                                f"format-3 irregular R={r} (matrices_2_10k_all)") for m, r in _M2K},
    **{f"m2k_n10240_m{m}.untp": (f"matrices_2_10k_all/(N=10240,M={m},R={r}).untp", -1,
                                 f"R={r} untainted list (matrices_2_10k_all)") for m, r in _M2K},
    "kat_n6_m4.dense": ("matrices_uncompressed/(N=6,K=2,M=4,R=0.34).mtrx", 0, "Johnson Ex. 2.5 KAT matrix"),
    "u_n7_m3.dense": ("matrices_uncompressed/(N=7,K=4,M=3,R=0.57).mtrx", 0, "small uncompressed"),
    "u_n10_m5.dense": ("matrices_uncompressed/(N=10,K=5,M=5,R=0.5).mtrx", 0, "small uncompressed"),
    "s1_n10_m5.sp1": ("matrices_1/(N=10,M=5,R=0.5).mtrx", 2, "format-2 (sparse_1) sample"),
}


def main() -> int:
    if not os.path.isdir(REF):
        print("reference checkout not present; nothing to do", file=sys.stderr)
        return 1
    os.makedirs(OUT, exist_ok=True)
    manifest = {}
    for name, (rel, fmt, role) in FIXTURES.items():
        data = open(os.path.join(REF, rel), "rb").read()
        with open(os.path.join(OUT, name + ".gz"), "wb") as f:
            f.write(gzip.compress(data, compresslevel=9, mtime=0))
        manifest[name] = {"reference_path": "sparse_matrices/" + rel, "format": fmt, "role": role,
                          "sha256": hashlib.sha256(data).hexdigest(), "bytes": len(data)}
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(f"wrote {len(manifest)} fixtures to {os.path.normpath(OUT)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
