#!/usr/bin/env python3
"""Fetch-boundary report for the hash kernels' hot loops.

For every loop longer than 1,500 bytes in the device code of an object built
by vortex_amd/csrc/Makefile, print its head offset mod 8, its instruction
count and how many instructions straddle a 32-byte boundary.  On gfx950 each
straddle in an issue-bound single-wave loop cost about one issue slot.

usage: python tools/straddle_report.py [vortex_amd/csrc/sha1_kernels.o]
(needs objcopy and the ROCm LLVM tools; CPU only)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "dev.co")
        # an explicit output file: with only an input, objcopy rewrites it in place
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", obj, os.path.join(d, "scratch.o")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True,
                              text=True).stdout


def report(text: str) -> list[str]:
    out, kern, base, insts = [], None, 0, []

    def flush():
        if not kern:
            return
        for a, n, op, line in insts:
            m = re.search(r"s_cbranch_\w+ .*<.*\+0x([0-9a-f]+)>", line)
            if not m:
                continue
            tgt = base + int(m.group(1), 16)
            if tgt >= a or a - tgt < 1500:
                continue
            body = [x for x in insts if tgt <= x[0] <= a]
            s32 = sum(1 for x in body if x[0] // 32 != (x[0] + x[1] - 1) // 32)
            out.append(f"{kern[:70]:70s} loop@+{tgt - base:#7x} mod8={tgt % 8} insts={len(body):5d} "
                       f"straddle32={s32}")

    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            flush()
            kern, base, insts = m.group(2), int(m.group(1), 16), []
            continue
        m = re.search(r"//\s*([0-9A-F]+):\s*((?:[0-9A-F]{8}\s*)+)", line)
        if m and kern:
            insts.append((int(m.group(1), 16), 4 * len(m.group(2).split()), line.strip().split()[0], line))
    flush()
    return out


if __name__ == "__main__":
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "vortex_amd", "csrc",
                                                            "sha1_kernels.o")
    print("\n".join(report(disassemble(obj))))
