#!/usr/bin/env python3
"""Disassemble the gfx950 code object embedded in a hipcc object file and count
instructions per kernel / per region.  Diagnostic only.

usage: tools/isa_dump.py <file.o> <out.dis> [kernel_substring]
Extracts .hip_fatbin (an uncompressed clang offload bundle), writes the gfx950
code object next to <out.dis>, disassembles it with llvm-objdump and, when a
kernel substring is given, prints that kernel's instruction histogram."""
import collections
import os
import re
import struct
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"


def extract(obj, co_path):
    fat = co_path + ".fatbin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    assert data.startswith(magic), "compressed or unknown bundle format"
    (nb,) = struct.unpack_from("<Q", data, len(magic))
    pos = len(magic) + 8
    for _ in range(nb):
        off, size, tl = struct.unpack_from("<QQQ", data, pos)
        pos += 24
        triple = data[pos:pos + tl].decode()
        pos += tl
        if "gfx950" in triple:
            open(co_path, "wb").write(data[off:off + size])
            return
    raise SystemExit("no gfx950 bundle")


def main():
    obj, out = sys.argv[1], sys.argv[2]
    co = out + ".co"
    extract(obj, co)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                         check=True).stdout
    open(out, "w").write(dis)
    if len(sys.argv) > 3:
        pat = sys.argv[3]
        cur, hist = None, collections.Counter()
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
            if m:
                cur = m.group(1)
                continue
            if cur and pat in cur:
                t = line.strip().split()
                if t and re.match(r"^[a-z_0-9]+$", t[0]):
                    hist[t[0]] += 1
        v = sum(c for k, c in hist.items() if k.startswith("v_"))
        print(f"VALU {v}  SALU {sum(c for k, c in hist.items() if k.startswith('s_'))}  "
              f"LDS {sum(c for k, c in hist.items() if k.startswith('ds_'))}")
        for k, c in hist.most_common(40):
            print(f"{c:7d} {k}")


if __name__ == "__main__":
    main()
